#!/bin/bash
# Snapshot a git revision (default HEAD) as a runnable tree with its library
# built, at ab_tree/ (git-ignored; travels to the GPU box), for A/B runs of
# the whole stack: bash tools/ab_bench.sh DIR=ab_tree AB_X=1
set -e
rev=${1:-HEAD}
root=$(cd "$(dirname "$0")/.." && pwd)
rm -rf "$root/ab_tree" && mkdir -p "$root/ab_tree"
files="s-cgib_amd include bench.py oracle __graft_entry__.py"
git -C "$root" cat-file -e "$rev:finetune_bench.py" 2>/dev/null && files="$files finetune_bench.py"
git -C "$root" archive "$rev" $files | tar -x -C "$root/ab_tree"
# the fine-tune bench reads the checkpoint fixture
mkdir -p "$root/ab_tree/tests/golden" && cp "$root/tests/golden/ckpt_pre_training_v1_GIN_64_5_1.npz" "$root/ab_tree/tests/golden/"
make -s -j8 -C "$root/ab_tree/s-cgib_amd/csrc" >/dev/null
echo "ab_tree <- $rev"

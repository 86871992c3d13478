#!/bin/bash
# Snapshot a git revision (default HEAD) as a runnable tree with its library
# built, at ab_tree/ (git-ignored; travels to the GPU box), for A/B runs of
# the whole stack: bash tools/ab_bench.sh DIR=ab_tree AB_X=1
set -e
rev=${1:-HEAD}
root=$(cd "$(dirname "$0")/.." && pwd)
rm -rf "$root/ab_tree" && mkdir -p "$root/ab_tree"
git -C "$root" archive "$rev" s-cgib_amd include bench.py oracle __graft_entry__.py | tar -x -C "$root/ab_tree"
make -s -j8 -C "$root/ab_tree/s-cgib_amd/csrc" >/dev/null
echo "ab_tree <- $rev"

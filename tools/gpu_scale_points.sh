#!/bin/bash
# Per-rank step time at the batch sizes of the 8-GPU prediction (DESIGN.md
# §6): QM9-like B = 128 / 512 / 1024 molecules on one GPU (one bench line each)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r03_scale}; mkdir -p $O
A="--steps 200 --warmup 20 --no-cpu-baseline --no-superbatch --no-kernel-timer"
for b in 128 512 1024; do
  timeout -k 10 300 python bench.py --batch $b $A > $O/qm9_b$b.log 2>&1 || { echo "B=$b failed"; tail -3 $O/qm9_b$b.log; exit 1; }
  tail -1 $O/qm9_b$b.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('B=$b', d['ms_per_step'], d['value'], d['config']['nodes_per_batch'])"
done

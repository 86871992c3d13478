#!/bin/bash
# The driver's bench command (20 steps, 5 warm-up) against the A/B protocol
# (300 steps, 20 warm-up), alternating on one box: how much of the short run's
# per-step time is the timed region's edges (first replay, clocks).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-short_long}; mkdir -p $O
X="--no-cpu-baseline --no-superbatch --no-kernel-timer"
for i in 1 2; do
  for v in "--steps 20 --warmup 5" "--steps 20 --warmup 60" "--steps 100 --warmup 5" "--steps 300 --warmup 20"; do
    timeout -k 10 200 python bench.py $v $X > $O/b.log 2>&1 || { echo bench failed; tail -5 $O/b.log; exit 1; }
    tail -1 $O/b.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'])" | tee -a $O/res.txt
  done
done

#!/bin/bash
# Timeline of the replayed pretrain step with the hand-offs on: device
# wall-clock stamps (ops.stamp, SCGIB_STAMPS=1 coarse / 2 per layer) of the
# last replay, plus the unstamped step time for reference.
set -o pipefail
TAG=${1:-stamps}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
for lvl in ${LEVELS:-0 1 2}; do
  SCGIB_STAMPS=$([ $lvl -gt 0 ] && echo $lvl) timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline \
    --no-superbatch --no-kernel-timer --no-finetune ${EXTRA:-} > $O/stamps_$lvl.log 2>&1 || { echo "level $lvl failed"; tail -5 $O/stamps_$lvl.log; exit 1; }
  echo "== level $lvl: $(grep 'timed:' $O/stamps_$lvl.log | sed 's/.*timed: //')"
  grep "stamp " $O/stamps_$lvl.log | sed 's/.*\] stamp/stamp/'
done

#!/bin/bash
# Fine-tune step timeline with the hand-offs on (ops.stamp, SCGIB_STAMPS=1 / 2)
set -o pipefail
TAG=${1:-ft_stamps}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
for lvl in ${LEVELS:-0 1 2}; do
  SCGIB_STAMPS=$([ $lvl -gt 0 ] && echo $lvl) timeout -k 10 200 python bench.py --finetune molhiv --steps 100 --warmup 10 \
    --no-cpu-baseline --no-kernel-timer > $O/stamps_$lvl.log 2>&1 || { echo "level $lvl failed"; tail -5 $O/stamps_$lvl.log; exit 1; }
  echo "== level $lvl: $(tail -1 $O/stamps_$lvl.log | python -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  grep "stamp " $O/stamps_$lvl.log | sed 's/.*\] stamp/stamp/'
done

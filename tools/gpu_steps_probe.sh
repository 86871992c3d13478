#!/bin/bash
# Per-step event times of the timed loop (SCGIB_STEP_PROBE=1) at the driver's
# K=20/W=5 and with longer warm-ups, same box.
set -o pipefail
TAG=${1:-probe}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
python -c "import __graft_entry__ as g; g.build()" > /dev/null 2>&1 || exit 3
for cfg in ${CFGS:-"20 5" "20 5" "20 100" "300 20" "20 5"}; do
  set -- $cfg
  SCGIB_STEP_PROBE=1 timeout -k 10 200 python bench.py --steps $1 --warmup $2 --no-cpu-baseline --no-superbatch \
    --no-kernel-timer --no-finetune > $O/run.log 2>&1 || { echo "run $cfg failed"; tail -5 $O/run.log; exit 1; }
  echo "== K=$1 W=$2: $(tail -1 $O/run.log | python -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  grep "step probe" $O/run.log | sed 's/.*step probe (ms): //' | tr ' ' '\n' | awk '{a[NR]=$1} END {printf "first10:"; for(i=1;i<=10&&i<=NR;i++) printf " %s", a[i]; printf "\nlast5:"; for(i=NR-4;i<=NR;i++) if(i>0) printf " %s", a[i]; print ""}'
  grep "host replay" $O/run.log | sed 's/.*host replay (us): //' | cut -d' ' -f1-10 | sed 's/^/host us first10: /'
  grep "timed:" $O/run.log
done

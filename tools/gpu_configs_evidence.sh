#!/bin/bash
# configs[2] and configs[3] on one GPU with rocprof evidence (VERDICT r05
# item 6): for molpcba B1024 k1 and PCQM4Mv2 B2048 k2, the FETCH_SIZE /
# WRITE_SIZE PMC passes and a kernel trace of the replayed step (traffic and
# replay files for the bench line), then the line itself (100 replayed steps,
# the kernel-timer roofline; CPU legs off: a CPU step there is 3-5 s, BASELINE.md
# §2 has those).  Usage: bash tools/gpu_configs_evidence.sh TAG
set -o pipefail
TAG=${1:-configs}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
for C in "molpcba 1024 1" "pcqm4mv2 2048 2"; do
  set -- $C; W=$1; B=$2; K=$3
  A="--workload $W --batch $B --k $K"; mkdir -p $O/$W
  for P in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d "$O/$W/pmc/$P" -o pmc \
      -- python bench.py $A --steps 5 --warmup 2 --no-cpu-baseline --no-superbatch --no-kernel-timer --no-finetune \
      > "$O/$W/pmc_$P.log" 2>&1 || { echo "$W pmc $P failed"; exit 1; }
  done
  python tools/pmc_summary.py "$O/$W/pmc" $W,$B,$K > "$O/$W/traffic.json" && echo "$W traffic ok"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$W/kt -o kt \
    -- python bench.py $A --steps 20 --warmup 5 --no-cpu-baseline --no-superbatch --no-finetune > $O/$W/kt_bench.log 2>&1 || { echo "$W trace failed"; exit 1; }
  python tools/kernel_instances.py $O/$W/kt --split adam_step_k --json $O/$W/replay.json --config $W,$B,$K > $O/$W/kernel_instances.txt 2>&1 && echo "$W replay ok"
  SCGIB_TRAFFIC_FILE=$O/$W/traffic.json SCGIB_REPLAY_FILE=$O/$W/replay.json timeout -k 10 600 \
    python bench.py $A --steps 100 --warmup 10 --no-cpu-baseline --no-superbatch --no-finetune > $O/$W/bench.log 2>&1 || { echo "$W bench failed"; exit 1; }
  tail -1 $O/$W/bench.log | python -c "
import sys,json; l=json.loads(sys.stdin.read()); r=l['roofline']
print('$W', l['ms_per_step'], l['value'], r['kernel'], r['frac'], r.get('replay_avg_us'), r.get('traffic_over_algorithmic'))"
done
echo done

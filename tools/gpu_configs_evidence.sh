#!/bin/bash
# configs[2] and configs[3] on one GPU with rocprof evidence (VERDICT r05
# item 6): for molpcba B1024 k1 and PCQM4Mv2 B2048 k2, the FETCH_SIZE /
# WRITE_SIZE PMC passes and a kernel trace of the replayed step (traffic and
# replay files for the bench line), then the line itself (100 replayed steps,
# the kernel-timer roofline; CPU legs off: a CPU step there is 3-5 s, BASELINE.md
# §2 has those).  Usage: bash tools/gpu_configs_evidence.sh TAG ["W B K" ...]
# (default: "molpcba 1024 1" "pcqm4mv2 2048 2"; the per-rank points of the
# strong-scaling prediction: "molpcba 128 1" "pcqm4mv2 256 2" ...)
set -o pipefail
TAG=${1:-configs}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
shift $(( $# > 0 ? 1 : 0 ))
CONFIGS=("$@"); [ ${#CONFIGS[@]} -eq 0 ] && CONFIGS=("molpcba 1024 1" "pcqm4mv2 2048 2")
for C in "${CONFIGS[@]}"; do
  set -- $C; W=$1; B=$2; K=$3
  A="--workload $W --batch $B --k $K"
  D=$O/${W}_B$B; mkdir -p $D
  for P in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d "$D/pmc/$P" -o pmc \
      -- python bench.py $A --steps 5 --warmup 2 --no-cpu-baseline --no-superbatch --no-kernel-timer --no-finetune \
      > "$D/pmc_$P.log" 2>&1 || { echo "$W pmc $P failed"; exit 1; }
  done
  python tools/pmc_summary.py "$D/pmc" $W,$B,$K > "$D/traffic.json" && echo "$W traffic ok"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt -o kt \
    -- python bench.py $A --steps 20 --warmup 5 --no-cpu-baseline --no-superbatch --no-finetune > $D/kt_bench.log 2>&1 || { echo "$W trace failed"; exit 1; }
  python tools/kernel_instances.py $D/kt --split adam_step_k,adam_reduce_k --json $D/replay.json --config $W,$B,$K > $D/kernel_instances.txt 2>&1 && echo "$W replay ok"
  SCGIB_TRAFFIC_FILE=$D/traffic.json SCGIB_REPLAY_FILE=$D/replay.json timeout -k 10 600 \
    python bench.py $A --steps 100 --warmup 10 --no-cpu-baseline --no-superbatch --no-finetune > $D/bench.log 2>&1 || { echo "$W bench failed"; exit 1; }
  tail -1 $D/bench.log | python -c "
import sys,json; l=json.loads(sys.stdin.read()); r=l['roofline']
print('$W', l['ms_per_step'], l['value'], r['kernel'], r['frac'], r.get('replay_avg_us'), r.get('traffic_over_algorithmic'))"
done
echo done

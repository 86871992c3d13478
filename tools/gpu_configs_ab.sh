#!/bin/bash
# configs[2] / configs[3] on one GPU and the agg-free
# threshold A/B: molpcba B1024 k1 and PCQM4Mv2 B2048 k2 steps (100 replayed
# after 10), each with every encoder agg-free and with none; the QM9 per-rank
# points of strong scaling (B = 128, 256).  Usage: bash tools/gpu_configs_ab.sh TAG
set -o pipefail
TAG=${1:-configs_ab}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
ARGS="--steps 100 --warmup 10 --no-cpu-baseline --no-superbatch --no-finetune --no-kernel-timer"
for C in "molpcba --batch 1024" "pcqm4mv2 --batch 2048 --k 2"; do
  W=${C%% *}
  for T in 0 1000000000; do
    timeout -k 10 300 python bench.py $ARGS --workload $C --agg-free-min-rows $T > $O/${W}_$T.log 2>&1 || { echo "$W $T failed"; tail -5 $O/${W}_$T.log; exit 1; }
    echo "$W min_rows=$T $(tail -1 $O/${W}_$T.log | python -c 'import sys,json; l=json.loads(sys.stdin.read()); print(l["ms_per_step"], l["value"], l["config"]["nodes_per_batch"])')"
  done
done
for B in 128 256; do
  timeout -k 10 300 python bench.py $ARGS --batch $B > $O/qm9_$B.log 2>&1 || { echo "qm9 $B failed"; exit 1; }
  echo "qm9 B=$B $(tail -1 $O/qm9_$B.log | python -c 'import sys,json; l=json.loads(sys.stdin.read()); print(l["ms_per_step"], l["value"])')"
done
echo done

#!/bin/bash
# Latency-floor A/B: the persistent encoder pair vs the
# per-layer path at small per-rank batches.  Usage: bash tools/gpu_pair_small.sh TAG [B...]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-pair_small}; mkdir -p $O; shift
BS=${@:-64 128 512}
A="--steps 300 --warmup 20 --no-cpu-baseline --no-superbatch --no-kernel-timer"
for i in 1 2; do
  for b in $BS; do
    for m in off on; do
      timeout -k 10 200 python tools/pair_ab.py $m $A --batch $b > $O/ab_${m}_b${b}_$i.log 2>&1 || { echo "ab $m b$b failed"; tail -5 $O/ab_${m}_b${b}_$i.log; exit 1; }
      tail -1 $O/ab_${m}_b${b}_$i.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('B=$b $m', d['ms_per_step'], d['value'])" | tee -a $O/summary.txt
    done
  done
done

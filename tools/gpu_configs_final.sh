#!/bin/bash
# configs[2] / configs[3] (molpcba B1024 k1, PCQM4Mv2 B2048 k2) with the
# round's final step (noise one step ahead, last reduce + Adam fused) against
# the step without the two (--no-noise-prefetch --no-fuse-adam), 2 interleaved
# rounds x 300 steps.  Usage: bash tools/gpu_configs_final.sh [TAG]
set -o pipefail
O=gpurun_out/${1:-configs_final}; mkdir -p $O
ARGS="--steps 300 --warmup 20 --no-cpu-baseline --no-superbatch --no-finetune --no-kernel-timer"
for r in 1 2; do
  for C in "molpcba --batch 1024" "pcqm4mv2 --batch 2048 --k 2"; do
    W=${C%% *}
    for V in "" "--no-noise-prefetch --no-fuse-adam"; do
      timeout -k 10 300 python bench.py $ARGS --workload $C $V > $O/run.log 2>&1 || { echo "$W failed"; tail -5 $O/run.log; exit 1; }
      echo "$W ${V:-final} $(tail -1 $O/run.log | python -c 'import sys,json; l=json.loads(sys.stdin.read()); print(l["ms_per_step"], l["value"])')" | tee -a $O/lines.txt
    done
  done
done

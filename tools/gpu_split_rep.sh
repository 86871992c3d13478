#!/bin/bash
# Repeated A/B of the two-lane replay at one batch size: lanes / whole
# alternated R times, K steps each.  Usage: bash tools/gpu_split_rep.sh TAG B K R
set -o pipefail
TAG=${1:-split_rep}; B=${2:-512}; K=${3:-300}; R=${4:-3}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
X="--no-cpu-baseline --no-superbatch --no-finetune --no-kernel-timer"
for r in $(seq 1 $R); do
  for S in "" "--no-split"; do
    T=$([ -z "$S" ] && echo lanes || echo whole)
    timeout -k 10 200 python bench.py --batch $B --steps $K --warmup 10 $X $S > $O/${T}_$r.log 2>&1 || { echo "$T $r failed"; exit 1; }
    echo "$T $r $(grep -h 'timed:' $O/${T}_$r.log)"
  done
done

#!/bin/bash
# CU-mask A/B: the probe, then the QM9 B512 step (300
# replayed after 20) with the encoder pair's side stream on all CUs vs on the
# last 192 / 128 CUs, three times each, and a kernel trace of the masked step.
# Usage: bash tools/gpu_cumask_ab.sh TAG
set -o pipefail
TAG=${1:-cumask}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 60 ./tools/cumask_probe.bin > $O/probe.txt 2>&1 || { echo probe failed; exit 1; }
cat $O/probe.txt
ARGS="--steps 300 --warmup 20 --no-cpu-baseline --no-superbatch --no-finetune --no-kernel-timer"
for i in 1 2 3; do
  for K in 0 192 128; do
    timeout -k 10 200 python bench.py $ARGS --side-cu-mask $K > $O/step_${K}_$i.log 2>&1 || { echo "step $K failed"; tail -5 $O/step_${K}_$i.log; exit 1; }
    echo "mask=$K run $i $(tail -1 $O/step_${K}_$i.log | python -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
echo done

#!/bin/bash
# Kernel traces of the QM9 B512 replayed step with and without ops.AGG_FREE
# (per-kernel replayed durations, tools/kernel_instances.py).  Usage: bash tools/gpu_aggfree_trace.sh TAG
set -o pipefail
TAG=${1:-aggfree_kt}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
for V in "" "--no-agg-free"; do
  N=$([ -z "$V" ] && echo free || echo agg)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$N -o kt \
    -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-superbatch --no-finetune --no-kernel-timer $V > $O/b_$N.log 2>&1 || { echo "trace $N failed"; exit 1; }
  python tools/kernel_instances.py $O/kt_$N --split adam_step_k,adam_reduce_k > $O/ki_$N.txt 2>&1
  echo "== $N"; sed -n 1,22p $O/ki_$N.txt
done

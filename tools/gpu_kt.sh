#!/bin/bash
# Isolated layer-kernel timing (bench.py's HIP-event KernelTimer) per library:
# bash tools/gpu_kt.sh [LIB ...]  (default: the in-tree libscgib.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in "${@:-$PWD/s-cgib_amd/libscgib.so}"; do
  SCGIB_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-superbatch \
    > gpurun_out/kt_$(basename $lib .so).log 2>&1 || { echo "bench failed: $lib"; tail -3 gpurun_out/kt_$(basename $lib .so).log; exit 1; }
  tail -1 gpurun_out/kt_$(basename $lib .so).log | python -c "
import sys, json; d = json.loads(sys.stdin.read()); r = d['roofline']; f = d['roofline_gin_fwd']
print('$(basename $lib)', 'bwd', r['avg_launch_us'], 'us', r['frac'], '| fwd', f['avg_launch_us'], 'us', f['frac'], '| step', d['ms_per_step'])"
done

#!/bin/bash
# Persistent encoder-pair kernels on / off: bench lines with the kernel timer
# (per-kernel per-step times) and a rocprofv3 kernel trace of each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-pair2}; mkdir -p $O
for m in on off; do
  timeout -k 10 300 python tools/pair_ab.py $m --steps 100 --warmup 10 --no-cpu-baseline --no-superbatch > $O/bench_$m.log 2>&1 || { echo "bench $m failed"; tail -5 $O/bench_$m.log; exit 1; }
  tail -1 $O/bench_$m.log | python -c "
import sys, json
d = json.loads(sys.stdin.read())
print('$m', d['ms_per_step'])
for k, r in (d.get('roofline_kernels') or {}).items():
    print('  ', k, r['per_step_us'], r['avg_launch_us'], r['launches_per_step'], r['mfma_frac'], r['hbm_frac'])"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt_$m -o kt \
    -- python tools/pair_ab.py $m --steps 20 --warmup 5 --no-cpu-baseline --no-superbatch --no-kernel-timer > $O/prof_$m.log 2>&1 || { echo "rocprof $m failed"; exit 1; }
  python tools/kernel_instances.py $O/kt_$m > $O/kernel_instances_$m.txt 2>&1
  head -25 $O/kernel_instances_$m.txt
done

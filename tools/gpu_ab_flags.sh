#!/bin/bash
# One call: the GPU suite, a same-box A/B of bench.py flag sets (ROUNDS x 300
# steps each, interleaved), and the superbatch section for each flag set.
# The library is built here beforehand (the in-tree .so travels).  Each GPU
# step has its own limit; the first failure ends the script.
# Usage: bash tools/gpu_ab_flags.sh TAG "FLAGS_A" "FLAGS_B" ...   ("" = defaults)
set -o pipefail
TAG=${1:-abf}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
for i in $(seq ${ROUNDS:-3}); do
  for cfg in "$@"; do
    timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-superbatch \
      --no-kernel-timer $cfg > $O/ab_last.log 2>&1 || { echo "bench [$cfg] failed"; tail -5 $O/ab_last.log; exit 1; }
    tail -1 $O/ab_last.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('[$cfg]', d['ms_per_step'], d['value'])" | tee -a $O/ab.txt
  done
done
if [ -z "$NO_SB" ]; then
  for cfg in "$@"; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $cfg > $O/sb.log 2>&1 || { echo "sb [$cfg] failed"; tail -5 $O/sb.log; exit 1; }
    tail -1 $O/sb.log > "$O/sb_line_$(echo "$cfg" | tr -c 'a-z0-9' '_').json"
    tail -1 $O/sb.log | python -c "
import sys,json; d=json.loads(sys.stdin.read()); sb=d['roofline_superbatch']; rk=d['roofline_kernels'] or {}
print('[$cfg] sb', {k: {kk: sb[k].get(kk) for kk in ('us','frac','frac_inclusive','mfma_frac')} for k in ('gin_fwd_k','gin_bwd_stats_k','gin_bwd5_k')})
print('[$cfg] B512', {k: (v['avg_launch_us'], v['frac']) for k, v in rk.items()})" | tee -a $O/sb.txt
  done
fi
echo done

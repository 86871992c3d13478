#!/bin/bash
# Persistent pair kernels: GPU tests, then the phase trace (tools/pair_trace.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-trace1}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pair.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/pair_trace.py > $O/trace.txt 2>&1; rc=$?
cat $O/trace.txt; [ $rc -eq 0 ] || exit $rc
for m in on off; do
  timeout -k 10 200 python tools/pair_ab.py $m --steps 300 --warmup 20 --no-cpu-baseline --no-superbatch --no-kernel-timer > $O/ab_$m.log 2>&1 || { echo "ab $m failed"; tail -5 $O/ab_$m.log; exit 1; }
  tail -1 $O/ab_$m.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$m', d['ms_per_step'])"
done

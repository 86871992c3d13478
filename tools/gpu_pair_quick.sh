#!/bin/bash
# Persistent encoder-pair kernels: their GPU tests, then an A/B of the bench
# step with them on / off (3 rounds).  Output under gpurun_out/pair1.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/pair1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pair.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -30 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
A="--steps 300 --warmup 20 --no-cpu-baseline --no-superbatch --no-kernel-timer"
for i in 1 2 3; do
  for m in off on; do
    timeout -k 10 200 python tools/pair_ab.py $m $A > $O/ab_$m$i.log 2>&1 || { echo "ab $m failed"; tail -5 $O/ab_$m$i.log; exit 1; }
    tail -1 $O/ab_$m$i.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$m', d['ms_per_step'], d['value'])"
  done
done

#!/bin/bash
# Ego prefetch for k >= 2: capacity-mode GPU tests, then the PCQM4Mv2-like
# B2048 k = 2 step with / without the prefetch (3 rounds each, same box).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-pf_k2}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_capacity.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -6 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
A="--workload pcqm4mv2 --batch 2048 --k 2 --steps 100 --warmup 10 --no-cpu-baseline --no-superbatch --no-kernel-timer"
for i in 1 2 3; do
  for v in "" "--no-ego-prefetch"; do
    timeout -k 10 200 python bench.py $A $v > $O/b.log 2>&1 || { echo bench failed; tail -5 $O/b.log; exit 1; }
    tail -1 $O/b.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('pcqm k2 ${v:-prefetch}', d['ms_per_step'], d['value'])" | tee -a $O/ab.txt
  done
done

#!/bin/bash
# interaction kernels on NW waves per graph: parity tests, then pretrain and fine-tune A/B vs ab_tree
set -o pipefail
TAG=${1:-r05_intnw}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$TAG
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "interaction or golden or config or finetune or capacity or noise" > gpurun_out/$TAG/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/$TAG/pytest.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=3 timeout -k 10 600 bash tools/ab_bench.sh --no-finetune "DIR=ab_tree" > gpurun_out/$TAG/ab.txt 2>&1; rc=$?
cat gpurun_out/$TAG/ab.txt; [ $rc -eq 0 ] || exit $rc
NO_TESTS=1 NO_FULL=1 ROUNDS=3 bash tools/gpu_ft_ab.sh $TAG "" "DIR=ab_tree"

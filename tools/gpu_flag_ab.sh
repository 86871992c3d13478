#!/bin/bash
# Selected GPU tests (-k EXPR), then the pretrain and fine-tune step A/B of the
# default against one bench flag, ROUNDS x 300 steps interleaved on one box.
# Usage: bash tools/gpu_flag_ab.sh TAG "--flag" "pytest -k expression"
set -o pipefail
TAG=${1:-flagab}; FLAG=$2; KEXPR=$3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
if [ -n "$KEXPR" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread -k "$KEXPR" > $O/pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
ROUNDS=${ROUNDS:-3} timeout -k 10 600 bash tools/ab_bench.sh --no-finetune "--no-finetune $FLAG" > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; [ $rc -eq 0 ] || exit $rc
NO_TESTS=1 NO_FULL=1 ROUNDS=${ROUNDS:-3} timeout -k 10 600 bash tools/gpu_ft_ab.sh $TAG "" "$FLAG"

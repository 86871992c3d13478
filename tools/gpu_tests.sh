#!/bin/bash
# GPU test pass (+ optional short bench): bash tools/gpu_tests.sh TAG [pytest-args...]
set -o pipefail
TAG=${1:-tests}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu "${@:-tests}" > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" $O/pytest_gpu.log | tail -3
exit $rc

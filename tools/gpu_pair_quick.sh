#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pair1
timeout -k 10 300 python -u -m pytest tests/test_gpu_pair.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pair1/pytest.log 2>&1; rc=$?
tail -30 gpurun_out/pair1/pytest.log
exit $rc

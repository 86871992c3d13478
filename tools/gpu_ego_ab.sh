#!/bin/bash
# ego-builder change: its GPU tests, the phase trace, then the step A/B vs ab_tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ego_ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "ego or k1 or bitmap" > gpurun_out/ego_ab/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/ego_ab/pytest.log; [ $rc -eq 0 ] || exit $rc
SCGIB_LIB=$PWD/s-cgib_amd/libscgib_trace.so timeout -k 10 200 python tools/phase_trace.py > gpurun_out/ego_ab/trace.txt 2>&1 || { echo trace failed; tail -5 gpurun_out/ego_ab/trace.txt; exit 1; }
head -6 gpurun_out/ego_ab/trace.txt
ROUNDS=3 timeout -k 10 800 bash tools/ab_bench.sh AB_NONE=1 DIR=ab_tree

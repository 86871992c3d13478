#!/bin/bash
# Kernel iteration on the box: GPU tests, the phase trace (trace build made on
# the box), then an A/B bench of the working tree against s-cgib_amd/libscgib_ab.so
# (tools/build_ab_lib.sh).  Every GPU step has its own limit; the first failure
# ends the script.  Usage: bash tools/gpu_iter.sh TAG [extra A/B configs]
set -o pipefail
TAG=${1:-iter}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
if [ -z "$NO_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
make -s -j16 -C s-cgib_amd/csrc trace > $O/mk_trace.log 2>&1 || { echo trace build failed; exit 3; }
SCGIB_LIB=$PWD/s-cgib_amd/libscgib_trace.so timeout -k 10 300 python tools/phase_trace.py > $O/phase.txt 2>&1 || { echo phase trace failed; tail -5 $O/phase.txt; exit 1; }
ROUNDS=${ROUNDS:-3} timeout -k 10 900 bash tools/ab_bench.sh SCGIB_LIB=$PWD/s-cgib_amd/libscgib_ab.so AB_NONE=1 "$@" > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; exit $rc

#!/bin/bash
# XCD-aware tile mapping A/B (SCGIB_XCD_TILES build of s-cgib_amd/libscgib_xcd.so,
# tools/build_ab_lib.sh): GIN parity tests on the variant library, the
# superbatch layer timings of both libraries, and the step A/B (3 rounds)
# against ab_tree: bash tools/gpu_xcd.sh TAG
set -o pipefail
TAG=${1:-xcd}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
XLIB=$PWD/s-cgib_amd/libscgib_xcd.so
SCGIB_LIB=$XLIB timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "layer or encoder" > $O/pytest_xcd.log 2>&1; rc=$?
echo "pytest (xcd lib) rc=$rc"; tail -1 $O/pytest_xcd.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_sb.sh $TAG/sb_default || exit 1
SCGIB_LIB=$XLIB bash tools/gpu_sb.sh $TAG/sb_xcd || exit 1
ROUNDS=3 bash tools/ab_bench.sh DIR=ab_tree AB_NEW=1 SCGIB_LIB=$XLIB > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; exit $rc

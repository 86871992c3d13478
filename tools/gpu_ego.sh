#!/bin/bash
# Ego-builder iteration: the ego-net GPU tests, tools/ego_bench.py on the working
# tree and on s-cgib_amd/libscgib_ab.so, then the A/B step bench.  Every GPU step
# has its own limit; the first failure ends the script.  Usage: bash tools/gpu_ego.sh TAG
set -o pipefail
TAG=${1:-ego}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_new -o kt -- python tools/ego_bench.py > $O/ego_new.txt 2>&1 || { echo ego bench failed; tail -5 $O/ego_new.txt; exit 1; }
SCGIB_LIB=$PWD/s-cgib_amd/libscgib_ab.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_old -o kt -- python tools/ego_bench.py > $O/ego_old.txt 2>&1 || { echo ego bench ab failed; exit 1; }
for d in new old; do echo $d; find $O/kt_$d -name "*kernel_stats.csv" -exec grep -h egonet {} \; | cut -c1-160; done
ROUNDS=${ROUNDS:-3} timeout -k 10 900 bash tools/ab_bench.sh SCGIB_LIB=$PWD/s-cgib_amd/libscgib_ab.so SCGIB_LIB=$PWD/s-cgib_amd/libscgib_ab1.so AB_NONE=1 "$@" > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; exit $rc

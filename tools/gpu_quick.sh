#!/bin/bash
# Iteration check: GPU tests, the phase trace of one eager step (trace build,
# made on the box) and a short bench line.  Each GPU step has its own limit;
# the first failure ends the script.  Usage: bash tools/gpu_quick.sh TAG [bench args]
set -o pipefail
TAG=${1:-quick}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
if [ -z "$NO_TRACE" ]; then
make -s -j16 -C s-cgib_amd/csrc trace > $O/mk_trace.log 2>&1 || { echo trace build failed; exit 3; }
SCGIB_LIB=$PWD/s-cgib_amd/libscgib_trace.so timeout -k 10 300 python tools/phase_trace.py > $O/phase.txt 2>&1 || { echo phase trace failed; tail -5 $O/phase.txt; exit 1; }
fi
timeout -k 10 300 python bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-superbatch --no-kernel-timer "$@" > $O/bench.log 2>&1 || { echo bench failed; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], 'ms', d['value'], d['unit'])"

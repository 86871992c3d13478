#!/bin/bash
# round-end rehearsal: the GPU suite, smoke, then `python bench.py` exactly as
# the driver runs it (defaults), timed
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-final}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
s=$(date +%s); timeout -k 10 900 python bench.py > $O/bench_default.log 2>&1 || { echo bench failed; tail -5 $O/bench_default.log; exit 1; }
echo "bench wall $(( $(date +%s) - s )) s"; tail -1 $O/bench_default.log | cut -c1-300

#!/bin/bash
# Build, GPU parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/timeout ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo build failed; tail gpurun_out/build.log; exit 3; }
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log
ok $rc || exit $rc
fi
timeout -k 10 600 python bench.py --steps ${STEPS:-30} --warmup 10 --cpu-seconds ${CPUSEC:-15} ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-600
ok $rc || exit $rc
if [ -z "$SKIP_PROF" ]; then
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_kt -o kt \
  -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1; rc=$?
echo "rocprof rc=$rc"
fi
exit $rc

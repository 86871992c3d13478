#!/bin/bash
# rocprofv3 kernel-trace summary of the bench (no CPU baseline / superbatch legs).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_kt -o kt \
  -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline ${EXTRA:-} > gpurun_out/prof_bench.log 2>&1; rc=$?
echo "rocprof rc=$rc"; tail -2 gpurun_out/prof_bench.log
find gpurun_out/prof_kt -name "*stats*" | head
exit $rc

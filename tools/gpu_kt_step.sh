#!/bin/bash
# rocprofv3 kernel trace of the default bench's replayed steps only, and one
# step's timeline (tools/prof_step.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-kt_step}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o kt \
  -- python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-superbatch --no-kernel-timer ${2:-} > $O/prof_bench.log 2>&1 || { echo rocprof failed; tail -5 $O/prof_bench.log; exit 1; }
python tools/prof_step.py $O/prof_kt/kt_kernel_trace.csv 20 > $O/step_timeline.txt
head -20 $O/step_timeline.txt; tail -1 $O/step_timeline.txt

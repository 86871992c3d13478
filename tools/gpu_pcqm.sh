#!/bin/bash
# PCQM4Mv2-like B2048 k = 2 (BASELINE configs): one bench line with its
# roofline, then the rocprofv3 kernel-trace summary of the same command (the
# k = 2 ego builder's share of the step).  Usage: bash tools/gpu_pcqm.sh TAG
set -o pipefail
TAG=${1:-r03_pcqm}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
A="--workload pcqm4mv2 --batch 2048 --k 2 --no-cpu-baseline --no-superbatch"
timeout -k 10 400 python bench.py $A --steps 50 --warmup 5 > $O/bench.log 2>&1 || { echo bench failed; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_kt -o kt \
  -- python bench.py $A --steps 20 --warmup 5 --no-kernel-timer > $O/prof_bench.log 2>&1 || { echo rocprof failed; exit 1; }
python tools/kernel_instances.py $O/prof_kt > $O/kernel_instances.txt 2>&1
head -30 $O/kernel_instances.txt

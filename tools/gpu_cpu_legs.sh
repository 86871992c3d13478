#!/bin/bash
# the bench's CPU-baseline legs alone (on the GPU box's host)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cpu_legs
timeout -k 10 600 python -c "
import sys, json
sys.argv = ['bench.py']
import bench
r = bench.cpu_baselines(1, 5, 'qm9', 512, 20.0)
print(json.dumps(r))
" > gpurun_out/cpu_legs/legs.log 2>&1; rc=$?
tail -3 gpurun_out/cpu_legs/legs.log | cut -c1-1500; exit $rc

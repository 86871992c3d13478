#!/bin/bash
# The compression noise drawn one step ahead (ops.NoisePrefetch, the bench
# default) vs at the head of the forward core chain (--no-noise-prefetch):
# the replay tests, then 3 interleaved rounds x 300 steps at B = 512 and B = 32.
# Usage: bash tools/gpu_noise_ab.sh [TAG]
set -o pipefail
O=gpurun_out/${1:-noise}; mkdir -p $O
python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 || { echo build failed; exit 3; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_graph_split.py \
  "tests/test_gpu_trajectory.py::test_pretrain_trajectory_replayed" tests/test_gpu_capacity.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
ROUNDS=3 bash tools/ab_bench.sh "AB_X=1" "--no-noise-prefetch" > $O/b512.txt 2>&1 || { cat $O/b512.txt; exit 1; }
cat $O/b512.txt
ROUNDS=3 bash tools/ab_bench.sh "--batch=32" "--batch=32 --no-noise-prefetch" > $O/b32.txt 2>&1 || { cat $O/b32.txt; exit 1; }
cat $O/b32.txt

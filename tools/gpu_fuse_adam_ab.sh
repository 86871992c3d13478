#!/bin/bash
# The ego chain's final weight-gradient reduce and Adam in one launch
# (scgib_adam_step_reduce, the bench default) vs two (--no-fuse-adam): the
# optimizer / replay / trajectory tests, then 3 interleaved rounds x 300
# steps at B = 512 and B = 32.  Usage: bash tools/gpu_fuse_adam_ab.sh [TAG]
set -o pipefail
O=gpurun_out/${1:-fuseadam}; mkdir -p $O
python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 || { echo build failed; exit 3; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_optim.py \
  tests/test_gpu_graph_split.py tests/test_gpu_trajectory.py tests/test_gpu_capacity.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
ROUNDS=3 bash tools/ab_bench.sh "AB_X=1" "--no-fuse-adam" > $O/b512.txt 2>&1 || { cat $O/b512.txt; exit 1; }
cat $O/b512.txt
ROUNDS=3 bash tools/ab_bench.sh "--batch=32" "--batch=32 --no-fuse-adam" > $O/b32.txt 2>&1 || { cat $O/b32.txt; exit 1; }
cat $O/b32.txt

#!/bin/bash
# Adam elements per thread in the fused reduce + Adam launch (SCGIB_FUSE_EPT
# 4, default, vs 1: libscgib_ept1.so, tools/build_ab_lib.sh) at B = 512, and at
# B = 32 with the slab gate off (ab_tree: ops.FUSE_FINAL_MIN_SLABS = 0) against
# the gated (unfused) default; 3 interleaved rounds x 300 steps.
set -o pipefail
O=gpurun_out/fuseept; mkdir -p $O
L=$GRAFT_REPO_ROOT/s-cgib_amd/libscgib_ept1.so
ROUNDS=3 bash tools/ab_bench.sh "AB_X=1" "SCGIB_LIB=$L" > $O/b512.txt 2>&1 || { cat $O/b512.txt; exit 1; }
ROUNDS=3 bash tools/ab_bench.sh "--batch=32" "DIR=ab_tree --batch=32" "DIR=ab_tree SCGIB_LIB=$L --batch=32" > $O/b32.txt 2>&1 || { cat $O/b32.txt; exit 1; }
sed "s#SCGIB_LIB=[^ ]*/##" $O/b512.txt $O/b32.txt

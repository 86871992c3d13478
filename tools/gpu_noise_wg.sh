#!/bin/bash
# noise_uniform_k's workgroup cap (SCGIB_NOISE_WG: 64 default, 256, 1024;
# tools/build_ab_lib.sh builds) with the noise drawn one step ahead (default)
# and at the head of the forward (--no-noise-prefetch), B = 512 and B = 32.
set -o pipefail
O=gpurun_out/noisewg; mkdir -p $O
L=$PWD/s-cgib_amd
ROUNDS=3 bash tools/ab_bench.sh "AB_X=1" "SCGIB_LIB=$L/libscgib_nw256.so" "SCGIB_LIB=$L/libscgib_nw1024.so" \
  "SCGIB_LIB=$L/libscgib_nw1024.so --no-noise-prefetch" > $O/b512.txt 2>&1 || { cat $O/b512.txt; exit 1; }
cat $O/b512.txt
ROUNDS=3 bash tools/ab_bench.sh "--batch=32" "SCGIB_LIB=$L/libscgib_nw256.so --batch=32" "SCGIB_LIB=$L/libscgib_nw1024.so --batch=32" \
  "SCGIB_LIB=$L/libscgib_nw1024.so --batch=32 --no-noise-prefetch" > $O/b32.txt 2>&1 || { cat $O/b32.txt; exit 1; }
cat $O/b32.txt

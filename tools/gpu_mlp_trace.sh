#!/bin/bash
# Dense MLP phase stamps (trace build of the library, built here)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/mlp
make -s -j16 -C s-cgib_amd/csrc trace > gpurun_out/mlp/build.log 2>&1 || { echo "trace build failed"; exit 3; }
SCGIB_LIB=$PWD/s-cgib_amd/libscgib_trace.so timeout -k 10 300 python tools/mlp_trace.py > gpurun_out/mlp/trace.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/mlp/trace.txt | head -60; exit $rc

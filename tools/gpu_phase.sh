#!/bin/bash
# phase trace of the GIN / ego-build kernels (trace build of the library)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/phase
make -s -j16 -C s-cgib_amd/csrc trace > gpurun_out/phase/build.log 2>&1 || { echo "trace build failed"; exit 3; }
SCGIB_LIB=$PWD/s-cgib_amd/libscgib_trace.so timeout -k 10 300 python tools/phase_trace.py > gpurun_out/phase/trace.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/phase/trace.txt | head -60; exit $rc

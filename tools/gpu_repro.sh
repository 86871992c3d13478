#!/bin/bash
# HIP-only nested-fork capture reproduction (tools/nested_capture_repro.hip),
# each mode in its own process with a time limit.  Usage: bash tools/gpu_repro.sh OUTDIR
O=${1:-gpurun_out/repro}; mkdir -p $O build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 tools/nested_capture_repro.hip -o build/nested_repro > $O/build.log 2>&1 || { echo repro build failed; exit 3; }
for m in flat sibling nested flat_destroy sibling_destroy nested_destroy nested_autofree nested_destroy_autofree; do
  timeout -k 5 60 build/nested_repro $m > $O/$m.log 2>&1; echo "$m rc=$?" >> $O/summary.txt
done
cat $O/summary.txt

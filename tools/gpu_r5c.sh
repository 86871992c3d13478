#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05_cslots
ROUNDS=3 timeout -k 10 900 bash tools/ab_bench.sh --no-finetune "SCGIB_LIB=$PWD/s-cgib_amd/libscgib_c128.so --no-finetune" "SCGIB_LIB=$PWD/s-cgib_amd/libscgib_c96.so --no-finetune" > gpurun_out/r05_cslots/ab.txt 2>&1; rc=$?
cat gpurun_out/r05_cslots/ab.txt; exit $rc

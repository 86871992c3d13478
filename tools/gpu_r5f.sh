#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05_s2sdefer
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "finetune or set2set or domain" > gpurun_out/r05_s2sdefer/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r05_s2sdefer/pytest.log; [ $rc -eq 0 ] || exit $rc
NO_TESTS=1 NO_FULL=1 ROUNDS=3 bash tools/gpu_ft_ab.sh r05_s2sdefer "" "DIR=ab_tree"

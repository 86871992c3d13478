#!/bin/bash
# One call: the whole GPU suite, the step A/B against ab_tree (3 x 300 steps),
# and the fine-tune check (tools/gpu_ft.sh).  Usage: bash tools/gpu_check_all.sh TAG
set -o pipefail
TAG=${1:-all}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
bash tools/gpu_tests.sh $TAG || exit 1
ROUNDS=3 bash tools/ab_bench.sh DIR=ab_tree AB_NEW=1 > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ft.sh $TAG/ft

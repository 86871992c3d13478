#!/bin/bash
# One step timeline of the replayed pretrain step (tools/gpu_kt_step.sh) and a
# same-box A/B of this tree against ab_tree/ (tools/make_ab_tree.sh REV).
# Usage: bash tools/gpu_step_check.sh TAG
set -o pipefail
TAG=${1:-stepchk}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$TAG
bash tools/gpu_kt_step.sh $TAG "--no-finetune" || exit 1
ROUNDS=${ROUNDS:-3} timeout -k 10 900 bash tools/ab_bench.sh --no-finetune DIR=ab_tree > gpurun_out/$TAG/ab.txt 2>&1; rc=$?
cat gpurun_out/$TAG/ab.txt; exit $rc

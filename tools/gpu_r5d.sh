#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_round.sh r05_final2 || exit 1
bash tools/gpu_phase.sh

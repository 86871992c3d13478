#!/bin/bash
# few-tile Gram path of the recon finish: its parity tests, the B = 32 phase
# trace (fin:gram), then small-batch pretrain A/B against ab_tree (previous commit)
set -o pipefail
TAG=${1:-r05_gram}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "recon" -x -v --timeout 120 \
  --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
PT_BATCH=32 SCGIB_LIB=$PWD/s-cgib_amd/libscgib_trace.so timeout -k 10 200 python -u tools/phase_trace.py \
  > $O/pt32.txt 2>&1 || { tail -5 $O/pt32.txt; exit 1; }
grep -A10 "recon_contrastive_fwd" $O/pt32.txt
ROUNDS=3 timeout -k 10 900 bash tools/ab_bench.sh "--batch=32" "DIR=ab_tree --batch=32" \
  "--batch=128" "DIR=ab_tree --batch=128" > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; exit $rc

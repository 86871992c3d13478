#!/bin/bash
# A/B of an alternative build of libscgib.so (tools/build_ab_lib.sh OUT=NAME):
# superbatch section and the pretrain step, ROUNDS x interleaved on one box.
# Usage: bash tools/gpu_lib_ab.sh TAG libscgib_xxx.so
set -o pipefail
TAG=${1:-libab}; ALT=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
for i in $(seq ${ROUNDS:-2}); do
  for lib in libscgib.so $ALT; do
    SCGIB_LIB=$PWD/s-cgib_amd/$lib timeout -k 10 300 python bench.py --superbatch-only > $O/sb_last.log 2>&1 || { echo "sb $lib failed"; tail -5 $O/sb_last.log; exit 1; }
    tail -1 $O/sb_last.log | python -c "
import sys,json; sb=json.loads(sys.stdin.read())['roofline_superbatch']
print('sb [$lib]', {k: (sb.get(k) or {}).get('us') for k in ('gin_fwd_k','gin_bwd_stats_k','gin_bwd5_k','gin_aggregate_k')})" | tee -a $O/sb_ab.txt
  done
done
ROUNDS=${ROUNDS:-3} timeout -k 10 600 bash tools/ab_bench.sh --no-finetune "SCGIB_LIB=$PWD/s-cgib_amd/$ALT --no-finetune" > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; exit $rc

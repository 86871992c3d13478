#!/bin/bash
# Superbatch evidence: a rocprofv3 kernel trace and the
# FETCH_SIZE / WRITE_SIZE PMC passes of `bench.py --superbatch-only` (the
# program directly after --), summarised by tools/sb_evidence.py, then the
# superbatch section again with the evidence file (its fields beside the
# event times).  Each GPU step has its own limit; the first failure ends it.
# Usage: bash tools/gpu_sb_evidence.sh TAG
set -o pipefail
TAG=${1:-sbev}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt \
  -- python bench.py --superbatch-only > $O/kt_bench.log 2>&1 || { echo "trace failed"; tail -5 $O/kt_bench.log; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$O/pmc/$C" -o pmc \
    -- python bench.py --superbatch-only > "$O/pmc_$C.log" 2>&1 || { echo "pmc $C failed"; tail -5 "$O/pmc_$C.log"; exit 1; }
done
python tools/sb_evidence.py $O/kt $O/pmc $O/sb_evidence.json > $O/sb_evidence.txt && echo evidence ok
SCGIB_SB_EVIDENCE_FILE=$O/sb_evidence.json timeout -k 10 300 python bench.py --superbatch-only > $O/sb_line.log 2>&1 || { echo "sb line failed"; exit 1; }
tail -1 $O/sb_line.log | python -c "
import sys,json; sb=json.loads(sys.stdin.read())['roofline_superbatch']
for k in ('gin_fwd_k','gin_fwd_k_agg_free','gin_bwd_stats_k','gin_bwd_statsz_k','gin_bwd5_k','gin_bwd5z_k','gin_aggregate_k'):
    e=sb.get(k) or {}; print(k, {kk: e.get(kk) for kk in ('us','trace_avg_us','trace_vs_event','frac','bytes','traffic','traffic_over_algorithmic','hbm_frac_measured')})"
echo done

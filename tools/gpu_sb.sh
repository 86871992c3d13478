#!/bin/bash
# Superbatch roofline: bench's roofline_superbatch section (+ the phase trace).
# Usage: bash tools/gpu_sb.sh TAG [trace]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-sb}; mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timer > $O/bench_sb.log 2>&1 || { echo bench failed; tail -5 $O/bench_sb.log; exit 1; }
tail -1 $O/bench_sb.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('ms/step', d['ms_per_step']); sb=d['roofline_superbatch']; [print(k, {kk: sb[k].get(kk) for kk in ('us','frac','frac_inclusive','mfma_frac')}) for k in ('gin_fwd_k','gin_bwd_stats_k','gin_bwd5_k','gin_aggregate_k')]"
if [ "$2" = trace ]; then
  SCGIB_LIB=$PWD/s-cgib_amd/libscgib_trace.so timeout -k 10 200 python tools/superbatch_trace.py > $O/sb_trace.txt 2>&1 || { echo trace failed; exit 1; }
  grep -E "layer|tail" $O/sb_trace.txt
fi

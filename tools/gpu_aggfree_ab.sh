#!/bin/bash
# ops.AGG_FREE A/B: the superbatch kernels both ways, then
# the QM9 B512 step (300 replayed steps after 20) alternating agg-free and
# --no-agg-free three times each.  Usage: bash tools/gpu_aggfree_ab.sh TAG
set -o pipefail
TAG=${1:-aggfree_ab}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
for V in "" "--no-agg-free"; do
  N=$([ -z "$V" ] && echo free || echo agg)
  timeout -k 10 300 python bench.py --superbatch-only $V > $O/sb_$N.log 2>&1 || { echo "sb $N failed"; tail -5 $O/sb_$N.log; exit 1; }
  tail -1 $O/sb_$N.log | python -c "
import sys,json; sb=json.loads(sys.stdin.read())['roofline_superbatch']
for k in ('gin_fwd_k','gin_fwd_k_agg_free','gin_bwd_stats_k','gin_bwd_statsz_k','gin_bwd5_k','gin_bwd5z_k'):
    e=sb.get(k)
    if e: print('$N', k, e['us'], e['frac'], e.get('launches'), e.get('mfma_frac'))
print('$N agg_free_layer_bwd_us', sb.get('agg_free_layer_bwd_us'))"
done
ARGS="--steps 300 --warmup 20 --no-cpu-baseline --no-superbatch --no-finetune --no-kernel-timer"
for i in 1 2 3; do
  for V in "" "--no-agg-free"; do
    N=$([ -z "$V" ] && echo free || echo agg)
    timeout -k 10 200 python bench.py $ARGS $V > $O/step_${N}_$i.log 2>&1 || { echo "step $N failed"; tail -5 $O/step_${N}_$i.log; exit 1; }
    echo "$N $i $(tail -1 $O/step_${N}_$i.log | python -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
echo done

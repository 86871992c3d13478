#!/bin/bash
# Two-lane replay A/B: the pretrain step at B = 32, 128
# and 512 and the molhiv fine-tune step, each with the split (default) and
# --no-split, at the driver's K = 20 / W = 5 and at 300 steps; one line per
# run with ms/step and host enqueue.  Each run has its own limit; the first
# failure ends the script.  Usage: bash tools/gpu_split_ab.sh TAG
set -o pipefail
TAG=${1:-split_ab}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
X="--no-cpu-baseline --no-superbatch --no-finetune --no-kernel-timer"
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 200 python bench.py "$@" > $O/$n.log 2>&1 || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }
  tail -1 $O/$n.log | python -c "
import sys, json; l = json.loads(sys.stdin.read()); l = l.get('finetune', l) if '--finetune' in '$*' else l
c = l['config']; print('%-22s %8.4f ms/step  host %s ms  nodes %s' % ('$n', l['ms_per_step'], c.get('host_enqueue_ms'), c.get('graph_nodes')))"
}
for B in 32 128 512; do
  for S in "" "--no-split"; do
    T=$([ -z "$S" ] && echo lanes || echo whole)
    run pre_B${B}_${T}_k20 --batch $B --steps 20 --warmup 5 $X $S
    run pre_B${B}_${T}_k300 --batch $B --steps 300 --warmup 10 $X $S
  done
done
for S in "" "--no-split"; do
  T=$([ -z "$S" ] && echo lanes || echo whole)
  run ft_${T}_k20 --finetune molhiv --steps 20 --warmup 5 --no-cpu-baseline $S
  run ft_${T}_k300 --finetune molhiv --steps 300 --warmup 10 --no-cpu-baseline $S
done
echo done

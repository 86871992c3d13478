#!/bin/bash
# Single-GPU throughput on the BASELINE.json configurations beside the
# headline one (QM9 B512 k1): ogbg-molpcba-like B1024 k1, PCQM4Mv2-like
# B2048 k2 (capacity mode + graph replay).  One bench line each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/configs
A="--steps ${STEPS:-100} --warmup 10 --no-cpu-baseline --no-superbatch --no-kernel-timer"
for cfg in "qm9 512 1" "molpcba 1024 1" "pcqm4mv2 2048 2"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --workload $1 --batch $2 --k $3 $A > gpurun_out/configs/$1.log 2>&1 || { echo "$1 failed"; tail -5 gpurun_out/configs/$1.log; exit 1; }
  tail -1 gpurun_out/configs/$1.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$1', d['config']['workload'], d['ms_per_step'], d['value'], d['config']['nodes_per_batch'])"
done

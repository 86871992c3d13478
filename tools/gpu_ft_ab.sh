#!/bin/bash
# GPU suite, then the fine-tune step A/B of bench flag sets (ROUNDS x 300
# steps, interleaved), then one full default bench line (pretrain + its
# fine-tune leg).  Each GPU step has its own limit; the first failure ends it.
# Usage: bash tools/gpu_ft_ab.sh TAG "FLAGS_A" "FLAGS_B" ...
set -o pipefail
TAG=${1:-ftab}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
for i in $(seq ${ROUNDS:-3}); do
  for cfg in "$@"; do
    dir=.; args="$cfg"
    if [[ "$cfg" == DIR=* ]]; then dir=${cfg#DIR=}; args=""; fi  # another revision (tools/make_ab_tree.sh)
    (cd $dir && timeout -k 10 200 python bench.py --finetune molhiv --steps 300 --warmup 20 --no-cpu-baseline \
      --no-kernel-timer $args) > $O/ft_last.log 2>&1 || { echo "ft [$cfg] failed"; tail -5 $O/ft_last.log; exit 1; }
    tail -1 $O/ft_last.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('[$cfg]', d['ms_per_step'], d['value'])" | tee -a $O/ft_ab.txt
  done
done
if [ -z "$NO_FULL" ]; then
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_full.log 2>&1 || { echo "full bench failed"; tail -5 $O/bench_full.log; exit 1; }
  tail -1 $O/bench_full.log | python -c "
import sys,json; d=json.loads(sys.stdin.read()); f=d.get('finetune') or {}
print('pretrain', d['ms_per_step'], d['value'], 'finetune', f.get('ms_per_step'), f.get('value'), (f.get('roofline') or {}).get('kernel'), (f.get('cpu_baseline') or {}).get('value'))"
fi
echo done

#!/bin/bash
# gin_bwd5_k grid A/B: step time with the default grid vs 128 / 64 slots
# (libraries from tools/build_ab_lib.sh), then the PMC traffic of the 64-slot build
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/bwd5_ab; mkdir -p $O
A="--steps 300 --warmup 20 --no-cpu-baseline --no-superbatch --no-kernel-timer"
for i in 1 2 3; do
  for v in default s128 s64; do
    if [ $v = default ]; then L=""; else L="$PWD/s-cgib_amd/libscgib_$v.so"; fi
    SCGIB_LIB=$L timeout -k 10 200 python bench.py $A > $O/ab_$v$i.log 2>&1 || { echo "ab $v failed"; tail -3 $O/ab_$v$i.log; exit 1; }
    tail -1 $O/ab_$v$i.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'])"
  done
done
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-superbatch --no-kernel-timer"
for C in FETCH_SIZE WRITE_SIZE; do
  SCGIB_LIB=$PWD/s-cgib_amd/libscgib_s64.so timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$O/pmc/$C" -o pmc \
    -- python bench.py $ARGS > "$O/pmc_$C.log" 2>&1 || { echo "pmc $C failed"; exit 1; }
done
python tools/pmc_summary.py "$O/pmc" > "$O/traffic_s64.json" && grep -A4 '"gin_bwd5_k' $O/traffic_s64.json

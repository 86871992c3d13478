#!/bin/bash
# The first timed steps after the contract's warm-up (DESIGN §5 "Round 6",
# "The driver's K = 20 vs 300 steps"): per-step HIP events of K = 20 after
#   W=5 | W=100 | W=100 then 300 ms idle | W=5 after 20000 one-element launches
#   | W=5 after 1000 ms of matrix products, each twice.
# (SCGIB_PRELOAD_MS / SCGIB_PRELAUNCH / SCGIB_IDLE_MS: bench.py diagnostics hooks)
set -o pipefail
mkdir -p gpurun_out/ramp
X="--steps 20 --no-cpu-baseline --no-superbatch --no-kernel-timer --no-finetune"
for rep in 1 2; do
for cfg in "W5" "W100" "W100_IDLE300" "W5_LAUNCH20000" "W5_PRELOAD1000"; do
  case $cfg in
    W5) E="AB_X=1"; W=5;;
    W100) E="AB_X=1"; W=100;;
    W100_IDLE300) E="SCGIB_IDLE_MS=300"; W=100;;
    W5_LAUNCH20000) E="SCGIB_PRELAUNCH=20000"; W=5;;
    W5_PRELOAD1000) E="SCGIB_PRELOAD_MS=1000"; W=5;;
  esac
  env $E SCGIB_STEP_PROBE=1 timeout -k 10 200 python bench.py $X --warmup $W > gpurun_out/ramp/r.log 2>&1 || { tail -5 gpurun_out/ramp/r.log; exit 1; }
  echo "== $cfg: $(grep 'timed:' gpurun_out/ramp/r.log | sed 's/.*timed: //')"
  grep "step probe" gpurun_out/ramp/r.log | sed 's/.*step probe (ms): //'
done
done

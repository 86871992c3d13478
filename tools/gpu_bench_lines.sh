#!/bin/bash
# The round's two bench lines (300 steps, and the driver's K = 20 / W = 5)
# against the evidence files of profiles/TAG (PMC traffic, replay traces,
# fine-tune stamps) — for a re-run of the lines without the profiling passes.
# Usage: bash tools/gpu_bench_lines.sh TAG
set -o pipefail
P=profiles/$1; O=gpurun_out/$1_lines; mkdir -p $O
export SCGIB_TRAFFIC_FILE=$P/traffic.json SCGIB_REPLAY_FILE=$P/replay.json \
  SCGIB_FT_TRAFFIC_FILE=$P/traffic_finetune.json SCGIB_FT_REPLAY_FILE=$P/replay_finetune.json \
  SCGIB_FT_STAMPS_FILE=$P/ft_stamps.json
timeout -k 10 600 python bench.py --steps 300 --warmup 20 --cpu-seconds 20 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { tail -5 $O/bench_driver.log; exit 1; }
tail -1 $O/bench_driver.log | cut -c1-300

#!/bin/bash
# A/B of the forward layer's early neighbour-row loads (bench.py --early-tiles,
# scgib_set_fwd_early_tiles): the bitwise test, then the pretrain step at
# B = 512 and B = 32 and the molhiv fine-tune, 3 interleaved rounds each.
# Usage: bash tools/gpu_early_ab.sh [TAG]
set -o pipefail
O=gpurun_out/${1:-early}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fwd_early.py > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
tail -1 $O/t.log
ROUNDS=3 bash tools/ab_bench.sh "AB_X=1" "--early-tiles=160" "--early-tiles=1000" > $O/ab512.txt 2>&1 || { cat $O/ab512.txt; exit 1; }
cat $O/ab512.txt
ROUNDS=3 bash tools/ab_bench.sh "--batch=32" "--batch=32 --early-tiles=1000" > $O/ab32.txt 2>&1 || { cat $O/ab32.txt; exit 1; }
cat $O/ab32.txt
ROUNDS=3 STEPS=200 bash tools/ab_bench.sh "--finetune=molhiv" "--finetune=molhiv --early-tiles=1000" > $O/abft.txt 2>&1 || { cat $O/abft.txt; exit 1; }
cat $O/abft.txt

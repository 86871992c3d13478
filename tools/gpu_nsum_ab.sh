#!/bin/bash
# A/B of the current tree against ab_tree/ (tools/make_ab_tree.sh REV) at the
# QM9 B = 512 and B = 32 pretrain steps, 3 interleaved rounds of 300 steps
# each (used for the recon backward's saved neighbour sums, round 6).
# Usage: bash tools/gpu_nsum_ab.sh [TAG]
set -o pipefail
O=gpurun_out/${1:-nsum}; mkdir -p $O
[ -n "$SKIP512" ] || { ROUNDS=3 bash tools/ab_bench.sh "AB_X=1" "DIR=ab_tree" > $O/ab512.txt 2>&1 || { cat $O/ab512.txt; exit 1; }; }
cat $O/ab512.txt
ROUNDS=3 bash tools/ab_bench.sh "AB_X=1 --batch=32" "DIR=ab_tree --batch=32" > $O/ab32.txt 2>&1 || { cat $O/ab32.txt; exit 1; }
cat $O/ab32.txt

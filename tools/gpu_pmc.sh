#!/bin/bash
# HBM traffic of the bench's kernels from rocprofv3 PMC counters, one counter
# per pass (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), then a
# per-kernel summary (tools/pmc_summary.py).  Usage: bash tools/gpu_pmc.sh OUTDIR
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/pmc}
mkdir -p "$OUT"
python -c "import __graft_entry__ as g; g.build()" > "$OUT/build.log" 2>&1 || { echo build failed; exit 3; }
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-superbatch --no-kernel-timer"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d "$OUT/$C" -o pmc \
    -- python bench.py $ARGS > "$OUT/$C.log" 2>&1 || { echo "pmc $C failed rc=$?"; tail -5 "$OUT/$C.log"; exit 1; }
done
python tools/pmc_summary.py "$OUT" > "$OUT/traffic.json" && cat "$OUT/traffic.json"

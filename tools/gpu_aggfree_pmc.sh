#!/bin/bash
# PMC traffic of the QM9 B512 step with the agg-free layers forced on
# (--agg-free-min-rows 0) and with the stored aggregate (--no-agg-free):
# FETCH_SIZE / WRITE_SIZE passes, summarised per kernel by tools/pmc_summary.py
# (gin_fwd_k<64> write per launch).  Usage: bash tools/gpu_aggfree_pmc.sh TAG
set -o pipefail
TAG=${1:-aggfree_pmc}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
for V in "--agg-free-min-rows 0" "--no-agg-free"; do
  N=$([ "$V" = "--no-agg-free" ] && echo stored || echo free)
  for P in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d "$O/$N/$P" -o pmc \
      -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-superbatch --no-kernel-timer --no-finetune $V \
      > "$O/${N}_$P.log" 2>&1 || { echo "$N pmc $P failed"; exit 1; }
  done
  python tools/pmc_summary.py "$O/$N" qm9,512,1 > "$O/traffic_$N.json" && echo "$N ok"
done
python - "$O" <<'PY'
import json, sys
for n in ("free", "stored"):
    t = json.load(open(f"{sys.argv[1]}/traffic_{n}.json"))
    for k, v in t.items():
        if k.startswith("gin_fwd_k<64") or k.startswith("gin_bwd_stats") or k.startswith("gin_bwd5"):
            print(n, k, v["dispatches"], "write MB %.2f" % (v["write_bytes"] / 1e6), "traffic MB %.2f" % (v["traffic_bytes"] / 1e6))
PY

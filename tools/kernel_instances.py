"""Per-instance kernel durations from a rocprofv3 kernel trace (csv):
python tools/kernel_instances.py gpurun_out/TAG/prof_kt [max_grid]

Groups dispatches by full kernel name (template arguments kept) and grid
size, so the bench's roofline kernel (e.g. gin_fwd_k<64, true, true, ...>
at the step's grid) can be checked against rocprof's own durations; rows
with a grid above max_grid (the ZINC-scale superbatch) are listed apart."""
import collections
import csv
import glob
import os
import sys

path = sys.argv[1]
files = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True) if os.path.isdir(path) else [path]
per = collections.defaultdict(list)
for fn in files:
    for r in csv.DictReader(open(fn)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("scgib::", "").replace("pair::", "").strip()
        per[(name, int(r["Grid_Size_X"]))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
print(f"{'kernel':60s} {'grid':>9s} {'calls':>6s} {'avg_us':>9s} {'min_us':>8s}")
for (name, grid), ds in sorted(per.items(), key=lambda kv: -sum(kv[1])):
    if len(ds) < 2 and sum(ds) < 50_000:
        continue
    print(f"{name[:60]:60s} {grid:9d} {len(ds):6d} {sum(ds) / len(ds) / 1e3:9.2f} {min(ds) / 1e3:8.2f}")

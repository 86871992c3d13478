"""Per-instance kernel durations from a rocprofv3 kernel trace (csv):
python tools/kernel_instances.py gpurun_out/TAG/prof_kt [--split KERNEL]

--split KERNEL: two tables, the dispatches up to the last KERNEL dispatch
(the bench's replayed steps, which end in adam_step_k or adam_reduce_k) and those after it
(the bench's kernel-timer pass: forward + backward, unforked, no optimizer
step) — the second is the set of launches the bench's HIP-event timer
averages.

Groups dispatches by full kernel name (template arguments kept) and grid
size, so the bench's roofline kernel (e.g. gin_fwd_k<64, true, true, ...>
at the step's grid) can be checked against rocprof's own durations; rows
with a grid above max_grid (the ZINC-scale superbatch) are listed apart.

--json OUT --config WORKLOAD,BATCH,K: also write the replayed steps' per-kernel
(full template name) dispatch count and average duration to OUT, tagged with
the bench configuration — bench.py reads it (SCGIB_REPLAY_FILE, default
profiles/replay_current.json) to report each roofline kernel's replay-derived
launch time beside its isolated kernel-timer time."""
import collections
import csv
import glob
import os
import sys

args = sys.argv[1:]
json_out = config = None
for flag in ("--json", "--config"):
    if flag in args:
        i = args.index(flag)
        if flag == "--json":
            json_out = args[i + 1]
        else:
            w, b, k = args[i + 1].split(",")
            config = {"workload": w, "batch": int(b), "k": int(k)}
        del args[i:i + 2]
split = None
if "--split" in args:
    i = args.index("--split")
    split = args[i + 1]
    del args[i:i + 2]
path = args[0]
files = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True) if os.path.isdir(path) else [path]
rows = []
for fn in files:
    for r in csv.DictReader(open(fn)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("scgib::", "").replace("pair::", "").strip()
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, int(r["Grid_Size_X"])))
rows.sort()
parts = [("all dispatches", rows)]
if split:
    # (comma-separated: the last dispatch of any, e.g. adam_step_k,adam_reduce_k —
    # the replayed pretraining step ends in the fused reduce + Adam launch)
    last = max((i for i, r in enumerate(rows) if r[2].startswith(tuple(split.split(",")))),
               default=-1)
    parts = [(f"up to the last {split} (replayed steps)", rows[:last + 1]),
             (f"after it (kernel-timer pass)", rows[last + 1:])]
for title, part in parts:
    per = collections.defaultdict(list)
    for t0, t1, name, grid in part:
        per[(name, grid)].append(t1 - t0)
    print(f"== {title}")
    print(f"{'kernel':60s} {'grid':>9s} {'calls':>6s} {'avg_us':>9s} {'min_us':>8s}")
    for (name, grid), ds in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        if len(ds) < 2 and sum(ds) < 50_000:
            continue
        print(f"{name[:60]:60s} {grid:9d} {len(ds):6d} {sum(ds) / len(ds) / 1e3:9.2f} {min(ds) / 1e3:8.2f}")

if json_out:
    import json
    replayed = parts[0][1]
    per = collections.defaultdict(list)
    for t0, t1, name, grid in replayed:
        per[name].append(t1 - t0)
    with open(json_out, "w") as fh:
        json.dump({"_config": config, "_source": os.path.abspath(path),
                   "kernels": {name: {"dispatches": len(ds), "avg_us": round(sum(ds) / len(ds) / 1e3, 3)}
                               for name, ds in per.items()}}, fh, indent=1, sort_keys=True)

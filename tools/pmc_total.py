"""Whole-run HBM traffic from one rocprofv3 PMC pass directory:
python tools/pmc_total.py DIR COUNTER [n_steps] -> total bytes (x2 for
FETCH_SIZE, the gfx950 correction of tools/pmc_summary.py) and per step."""
import csv
import glob
import os
import sys

path, counter = sys.argv[1], sys.argv[2]
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
tot = 0.0
n = 0
for fn in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(fn)):
        if row.get("Counter_Name") == counter:
            tot += float(row["Counter_Value"]) * 1024.0
            n += 1
scale = 2.0 if counter == "FETCH_SIZE" else 1.0
print(f"{counter}: dispatches={n} total_MB={scale * tot / 1e6:.1f} per_step_MB={scale * tot / 1e6 / steps:.2f}")

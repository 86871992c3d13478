"""Per-kernel HBM traffic from the rocprofv3 PMC passes of tools/gpu_pmc.sh.

traffic = 2 x FETCH_SIZE + WRITE_SIZE per dispatch (MI355X_MICROARCH.md,
"HBM [CDNA4]": on gfx950 FETCH_SIZE reports half the bytes of 16-B-per-lane
coalesced reads; WRITE_SIZE is exact for 16-B stores).  rocprofv3 reports both
in KB.  Prints JSON {kernel: {dispatches, fetch_bytes, write_bytes,
traffic_bytes}} averaged over dispatches."""
import collections
import csv
import glob
import json
import os
import sys


def load(path, counter):
    files = glob.glob(os.path.join(path, counter, "**", "*counter_collection.csv"), recursive=True)
    per = collections.defaultdict(list)
    for fn in files:
        for row in csv.DictReader(open(fn)):
            if row.get("Counter_Name") != counter:
                continue
            # keep template arguments: gin_bwd_k<64, true> (GIN) vs <128, false> (MLP)
            name = row["Kernel_Name"].split("(")[0]
            name = name.replace("void ", "").replace("scgib::", "").replace("pair::", "").strip()
            per[name].append(float(row["Counter_Value"]) * 1024.0)  # KB -> bytes
    return per


def main(out, config=None):
    fetch, write = load(out, "FETCH_SIZE"), load(out, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        f = sum(fetch.get(k, [0])) / max(len(fetch.get(k, [])), 1)
        w = sum(write.get(k, [0])) / max(len(write.get(k, [])), 1)
        res[k] = {"dispatches": max(len(fetch.get(k, [])), len(write.get(k, []))),
                  "fetch_bytes": round(2 * f), "write_bytes": round(w),
                  "traffic_bytes": round(2 * f + w)}
    if config:  # the bench configuration the passes ran ("qm9,512,1")
        wl, b, k = config.split(",")
        res["_config"] = {"workload": wl, "batch": int(b), "k": int(k)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)

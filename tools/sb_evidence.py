"""rocprofv3 evidence for the bench's superbatch section.

python tools/sb_evidence.py KT_DIR PMC_DIR OUT.json

KT_DIR: a `rocprofv3 --kernel-trace --stats` run of `bench.py --superbatch-only`;
PMC_DIR: FETCH_SIZE/ and WRITE_SIZE/ subdirectories, one `rocprofv3 --pmc` run
each of the same program.  Writes, per superbatch kernel the bench reports
(the same launches its HIP-event timer brackets), the traced average duration
and the HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md
gfx950 correction, as tools/pmc_summary.py).  bench.py reads the file
(SCGIB_SB_EVIDENCE_FILE, default profiles/sb_evidence_current.json) and puts
`trace_avg_us`, `traffic` and `traffic_over_algorithmic` beside each
superbatch entry's event time and algorithmic bytes.
"""
import collections
import csv
import glob
import json
import os
import sys

# bench.superbatch_roofline's kernels -> the trace-name prefixes of the launches
# it times (gin_bwd_stats_k: the gathering instance only, as the bench keeps
# the launches with e > 0)
# (a launch may count for two keys: gin_fwd_k averages all five d = 64
# layers, gin_fwd_k_agg_free the four XFORM ones, which are agg-free)
KERNELS = {
    "gin_fwd_k": ("gin_fwd_k<64,",),
    "gin_fwd_k_agg_free": ("gin_fwd_k<64, true,",),
    "gin_bwd_stats_k": ("gin_bwd_stats_k<true,",),
    "gin_bwd_statsz_k": ("gin_bwd_statsz_k<true>",),
    "gin_bwd5_k": ("gin_bwd5_k<64", "gin_bwd5r_k<64"),
    "gin_bwd5z_k": ("gin_bwd5z_k<true>",),
    "gin_aggregate_k": ("gin_aggregate_k<",),
}


def _name(raw):
    return raw.split("(")[0].replace("void ", "").replace("scgib::", "").strip()


def _kernels_of(name):
    return [key for key, prefixes in KERNELS.items() if name.startswith(prefixes)]


def trace(path):
    per = collections.defaultdict(list)
    for fn in glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            for k in _kernels_of(_name(r["Kernel_Name"])):
                per[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return per


def pmc(path, counter):
    per = collections.defaultdict(list)
    for fn in glob.glob(os.path.join(path, counter, "**", "*counter_collection.csv"),
                        recursive=True):
        for r in csv.DictReader(open(fn)):
            if r.get("Counter_Name") != counter:
                continue
            for k in _kernels_of(_name(r["Kernel_Name"])):
                per[k].append(float(r["Counter_Value"]) * 1024.0)  # KB -> bytes
    return per


def main(kt, pm, out):
    t, f, w = trace(kt), pmc(pm, "FETCH_SIZE"), pmc(pm, "WRITE_SIZE")
    res = {}
    for k in KERNELS:
        e = {}
        if t.get(k):
            e["trace_dispatches"] = len(t[k])
            e["trace_avg_us"] = round(sum(t[k]) / len(t[k]), 3)
        if f.get(k) and w.get(k):
            fb, wb = sum(f[k]) / len(f[k]), sum(w[k]) / len(w[k])
            e["pmc_dispatches"] = min(len(f[k]), len(w[k]))
            e["fetch_bytes"], e["write_bytes"] = round(2 * fb), round(wb)
            e["traffic_bytes"] = round(2 * fb + wb)
        if e:
            res[k] = e
    line = None
    for fn in glob.glob(os.path.join(kt, "..", "*.log")):
        for ln in open(fn):
            if ln.startswith("{") and "roofline_superbatch" in ln:
                line = json.loads(ln)["roofline_superbatch"]
    if line:
        res["_nodes"] = line.get("nodes")
    res["_note"] = ("rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of "
                    "bench.py --superbatch-only; traffic = 2 x FETCH_SIZE + WRITE_SIZE per launch")
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])

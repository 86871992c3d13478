"""S-CGIB pretrain-step throughput on MI355X (BASELINE.json metric).

One step = on-device ego-net build (k-hop in-subgraphs of every node) +
forward (transfer_d, GIN-64x5 x 2 encoders, fused compression/attention,
MLP, KL + contrastive + reconstruction losses) + backward + gradient
all-reduce (N > 1) + Adam(lr 1e-4, wd 5e-5) — exp_pretraining.py:290-333 with
the Mainmodel_continue wrapper it trains (:109-113).

Workload (config.workload): QM9-like synthetic molecules, B = 512 per GPU,
k = 1, F = 11 (BASELINE.json configs[1]); weak scaling across GPUs.
Inputs are resident in HBM before the timed region: a pool of distinct
collated batches, cycled so consecutive steps see different molecules.

Prints ONE JSON line on rank 0 (see README/DESIGN.md for the fields).
"""
from __future__ import annotations

import argparse
import contextlib
import importlib
import json
import os
import statistics
import sys
import time
from types import SimpleNamespace

import numpy as np
import torch
import torch.distributed as dist
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("s-cgib_amd")

HBM_PEAK_GBS = 8000.0       # MI355X spec (MI355X_MICROARCH.md:36)
HBM_MEASURED_GBS = 6290.0   # float4 copy, same file
F32_MFMA_PEAK_TFLOPS = 157.3  # dense fp32 MFMA (MI355X_MICROARCH.md)
# HBM bytes per launch of each kernel from the rocprofv3 PMC passes of
# tools/gpu_pmc.sh (2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md "HBM
# [CDNA4]"), committed under profiles/ by the round measurement of the CURRENT
# code (tools/gpu_round.sh) — the bench itself runs unprofiled.  A timed kernel
# without an entry there is reported with traffic null and a traffic_note.
TRAFFIC_FILE = os.environ.get("SCGIB_TRAFFIC_FILE",
                              os.path.join(ROOT, "profiles", "traffic_current.json"))
# the same passes over the fine-tune step (bench.py --finetune molhiv)
FT_TRAFFIC_FILE = os.environ.get("SCGIB_FT_TRAFFIC_FILE",
                                 os.path.join(ROOT, "profiles", "traffic_finetune_current.json"))


def _load_json(path):
    try:
        with open(path) as fh:
            return json.load(fh)
    except (OSError, ValueError):
        return {}


TRAFFIC_SETS = [(TRAFFIC_FILE, _load_json(TRAFFIC_FILE)),
                (FT_TRAFFIC_FILE, _load_json(FT_TRAFFIC_FILE))]
RUN_CONFIG = None  # {"workload", "batch", "k"} of this run (main)
# Replay-derived launch times: the same bench command traced by rocprofv3
# (tools/gpu_round.sh: kernel_instances.py --json over the replayed steps of
# its traced run), per kernel template instance — the timer pass below times
# each kernel isolated and cache-warm, the replayed step runs it beside the
# other encoder chain.
REPLAY_FILE = os.environ.get("SCGIB_REPLAY_FILE",
                             os.path.join(ROOT, "profiles", "replay_current.json"))
FT_REPLAY_FILE = os.environ.get("SCGIB_FT_REPLAY_FILE",
                                os.path.join(ROOT, "profiles", "replay_finetune_current.json"))
REPLAY_SETS = [(REPLAY_FILE, _load_json(REPLAY_FILE)),
               (FT_REPLAY_FILE, _load_json(FT_REPLAY_FILE))]


def _for_run(sets):
    """(path, data) of the evidence file measured on this run's
    configuration; the first file (for its note) when none is."""
    for path, data in sets:
        if data.get("_config") == RUN_CONFIG:
            return path, data
    return sets[0]


SB_FILE = os.environ.get("SCGIB_SB_EVIDENCE_FILE") or os.path.join(
    ROOT, "profiles", "sb_evidence_current.json")


def _sb_evidence():
    """rocprofv3 evidence of the superbatch launches (tools/sb_evidence.py):
    per kernel the traced average duration and the PMC HBM bytes per launch."""
    try:
        with open(SB_FILE) as fh:
            return json.load(fh)
    except (OSError, ValueError):
        return {}


def replay_of(variants):
    """(dispatches, dispatch-weighted mean duration in us) of the replayed
    launches whose kernel names start with one of ``variants``; None when the
    file is of another configuration or holds none."""
    _, rep = _for_run(REPLAY_SETS)
    if rep.get("_config") != RUN_CONFIG:
        return None
    got = [v for k, v in rep.get("kernels", {}).items() if any(k.startswith(p) for p in variants)]
    n = sum(g["dispatches"] for g in got)
    if not n:
        return None
    return n, sum(g["avg_us"] * g["dispatches"] for g in got) / n


def traffic_of(variants):
    """Dispatch-weighted mean HBM bytes per launch over the template
    instantiations whose names start with one of ``variants`` (e.g. the GIN
    variants of gin_bwd_k, not the MLP one); None when none is in the file."""
    _, tr = _for_run(TRAFFIC_SETS)
    cfg = tr.get("_config")
    if cfg is not None and cfg != RUN_CONFIG:
        return None  # measured on another configuration
    got = [t for k, t in tr.items()
           if not k.startswith("_") and any(k.startswith(v) for v in variants)]
    n = sum(g["dispatches"] for g in got)
    if not n:
        return None
    return round(sum(g["traffic_bytes"] * g["dispatches"] for g in got) / n)


def agg_bytes(n, e, d):
    """Algorithmic bytes of one GIN aggregation: neighbour +
    self rows read, output written, col + rowptr read."""
    return 4 * d * (e + n) + 4 * d * n + 4 * e + 4 * (n + 1)


def make_model(F_in, k, gin_layers, dev):
    args = SimpleNamespace(recons_type="adj", useAtt=1, readout_f="sum", d_transfer=32,
                           batch_size=512, gin_layers=gin_layers, task="graph_classification")
    inner = pkg.models.Mainmodel(args, F_in, 64, 4, 4, k, "GIN")
    model = pkg.models.Mainmodel_continue(args, F_in, 64, 4, 4, k, 1, inner, "GIN")
    return model.to(dev).train()


def agg_fwd_bytes(n, e, d_in):
    """Algorithmic bytes of one gin_fwd_k launch = SURVEY.md §8(d)'s
    aggregation figure for the layer (neighbour + self rows read, output
    written, col + rowptr read).  The kernel's own saved-activation writes
    (agg, r, z2) and the weights are NOT counted: they are this design's
    choice, not bytes the algorithm needs (`layer_fwd_bytes_inclusive`)."""
    return agg_bytes(n, e, d_in)


def layer_fwd_bytes_inclusive(n, e, d_in, store_r=False, store_agg=True):
    """Everything one gin_fwd_k launch moves: the gather (neighbour + self
    rows, col + rowptr), W1/b1/W2/b2, the z2 writes (+ r's when the forward
    stores it, ops.STORE_R; + agg's unless the layer is agg-free, ops.AGG_FREE)
    and the per-tile BN statistics (reported beside the §8(d) figure as
    frac_inclusive)."""
    return (4 * d_in * (e + n) + 4 * e + 4 * (n + 1)
            + 4 * (64 * d_in + 64 + 64 * 64 + 64)
            + 4 * n * ((d_in if store_agg else 0) + 64 + (64 if store_r else 0))
            + 512 * ((n + 63) // 64))


def layer_fwd_flops(n, e, d_in):
    return 2 * n * 64 * (d_in + 64)


def layer_bwd_bytes(n, e, d_in, store_r=False, wg=True):
    """Algorithmic bytes of one GIN layer backward launch (gin_bwd5r_k /
    gin_bwd5_k): the dy, z2 and agg rows read (+ r's when the
    forward stored it), W1/b1/W2 + BN coefficients, d(agg) written.  The
    per-workgroup dW slabs are NOT counted: they are partials of a 33 KB
    gradient, not bytes the layer needs (their cost shows in `traffic`).
    wg False (a frozen layer, need_w = 0): the agg rows are not read."""
    return (4 * n * ((3 if store_r else 2) * 64 + (d_in if wg else 0))
            + 4 * (64 * d_in + 64 * 64 + 7 * 64) + 4 * n * d_in)


def bwdz_bytes(n, e, d_in, wg=True):
    """Algorithmic bytes of one gin_bwd5z_k launch (the agg-free layer
    backward, ops.AGG_FREE): the dy, z2 and r rows read, W2 + BN coefficients,
    dz1 written (slabs not counted, as layer_bwd_bytes)."""
    return 4 * n * 3 * 64 + 4 * (64 * 64 + 7 * 64) + 4 * n * 64


def bwdz_flops(n, e, d_in, wg=True):
    return (4 if wg else 2) * n * 64 * 64  # dW2 and dr (frozen: dr)


def statsz_bytes(n, e, d, wg=True):
    """Algorithmic bytes of one gin_bwd_statsz_k launch: gin_bwd_stats_k's
    (the transposed gather of dz1, z2 read, dy written) + W1 (its dW1
    partials not counted, as the layer kernels' slabs)."""
    return stats_bytes(n, e, d) + 4 * 64 * 64


def statsz_flops(n, e, d, wg=True):
    return (4 if wg else 2) * n * 64 * 64  # dh = g W1 and dW1 += g^T h (frozen: dh)


def stats_bytes(n, e, d):
    """Algorithmic bytes of one gin_bwd_stats_k launch: the transposed
    aggregation of d(agg) (§8(d)'s figure when it gathers, e > 0; the plain
    dh read otherwise) + z2 read and dy written."""
    gather = agg_bytes(n, e, d) - 4 * d * n if e > 0 else 4 * d * n
    return gather + 4 * 64 * n * 2


def no_flops(n, e, d):
    return 0


def layer_bwd_flops(n, e, d_in, wg=True):
    return (4 if wg else 2) * n * 64 * (64 + d_in)  # dW2, dr, dW1, d(agg) (frozen: dr, d(agg))


def _call_meta(fn, m):
    """bytes / flops of one launch from its meta (n, e, d_in[, r stored])."""
    if fn is layer_fwd_bytes_inclusive:
        return fn(m["n"], m["e"], m["d_in"], m.get("r", False), m.get("agg", True))
    if fn in (bwdz_bytes, bwdz_flops, statsz_bytes, statsz_flops):
        return fn(m["n"], m["e"], m["d_in"], m.get("wg", True))
    if fn is layer_bwd_bytes:
        return fn(m["n"], m["e"], m["d_in"], m.get("r", False), m.get("wg", True))
    if fn is layer_bwd_flops:
        return fn(m["n"], m["e"], m["d_in"], m.get("wg", True))
    return fn(m["n"], m["e"], m["d_in"])


# The step's kernels timed by KernelTimer, by kernel (the C-ABI entries that
# launch it, a filter on the launch sizes, §8(d) bytes, flops, and the PMC
# name prefixes of its template instances in the traffic file)
KERNELS = {
    "gin_fwd_k": dict(entries=("scgib_gin_layer0_fwd", "scgib_gin_layer_fwd_bn"),
                      keep=lambda m: True, bytes=agg_fwd_bytes, flops=layer_fwd_flops,
                      pmc=["gin_fwd_k<32, false, true, true,", "gin_fwd_k<64, true, true,",
                           "gin_fwd_k<64, false, true,"],
                      desc="fused GIN layer forward: gather (+ previous BN + ReLU on load) + "
                           "2 f32-MFMA GEMMs + BN tile statistics"),
    "gin_bwd5_k": dict(entries=("scgib_gin_layer_bwd",), keep=lambda m: m["d_in"] == 64,
                       bytes=layer_bwd_bytes, flops=layer_bwd_flops,
                       # (the instance with weight products: <64, true>; <64, false>
                       # is the frozen-layer fine-tune kernel)
                       pmc=["gin_bwd5r_k<64>", "gin_bwd5_k<64, true>", "gin_bwd5_k<64>"],
                       desc="fused GIN layer backward (d_in = 64): BN-backward apply + 4 "
                            "f32-MFMA GEMMs on 32-row sub-tiles (gin_bwd5r_k: + the hidden "
                            "activation r recomputed, not read; flops count the 4 GEMMs)"),
    "gin_bwd_stats_k": dict(entries=("scgib_gin_bwd_stats_bn_fold", "scgib_gin_bwd_stats_seg_bn",
                                     "scgib_gin_bwd_stats_bn"),
                            keep=lambda m: True, bytes=stats_bytes, flops=no_flops,
                            pmc=["gin_bwd_stats_k<"],
                            desc="GIN backward statistics: transposed gather of d(agg) + ReLU "
                                 "mask + BN-backward sums"),
    "gin_bwd5z_k": dict(entries=("scgib_gin_layer_bwd_z",), keep=lambda m: m.get("wg", True),
                        bytes=bwdz_bytes, flops=bwdz_flops, pmc=["gin_bwd5z_k<true>"],
                        desc="agg-free GIN layer backward (layers 1..4, ops.AGG_FREE): BN-backward "
                             "apply + dW2 and dr on f32 MFMA, dz1 written (dW1 moves to "
                             "gin_bwd_statsz_k)"),
    "gin_bwd_statsz_k": dict(entries=("scgib_gin_bwd_stats_z",), keep=lambda m: m.get("wg", True),
                             bytes=statsz_bytes, flops=statsz_flops,
                             pmc=["gin_bwd_statsz_k<true>"],
                             desc="GIN backward statistics below an agg-free layer: transposed "
                                  "gather of dz1, dh = g W1 and dW1 += g^T h on f32 MFMA, ReLU "
                                  "mask + BN-backward sums"),
    "gin_bwd_k": dict(entries=("scgib_gin_layer0_bwd",), keep=lambda m: True,
                      bytes=layer_bwd_bytes, flops=layer_bwd_flops,
                      pmc=["gin_bwd_k<32, true, true,"],
                      desc="layer-0 backward with transfer_d folded (d_in = 32)"),
}


class KernelTimer:
    """HIP-event timing of every launch of the given C-ABI entry points
    (routed through ops._launch) on the stream they are launched on (torch's
    current stream).  A ~170 us spin kernel is queued ahead of each bracketed
    launch so the GPU is still busy while the host submits [start event,
    kernel, end event]: the events bracket the kernel, not the host's launch
    latency."""

    REPEAT = 10  # back-to-back launches per bracket (the kernels are idempotent)

    def __init__(self, *names):
        self.names = set(names)
        self.records = {n: [] for n in names}  # name -> [(start, end, meta)]

    def __enter__(self):
        def observe(name, meta, launch):
            if name not in self.names:
                return launch()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(400_000)
            s.record()
            # the timed kernels read only their inputs and overwrite their
            # outputs (the fused forward also re-applies its BN running-stat
            # update, harmless here: this pass runs after the timed steps);
            # REPEAT launches per bracket amortise the event/dispatch latency
            for _ in range(self.REPEAT):
                rc = launch()
            e.record()
            self.records[name].append((s, e, meta))
            return rc

        pkg.ops.OBSERVER = observe
        return self

    def __exit__(self, *exc):
        pkg.ops.OBSERVER = None

    def kernel_summary(self, spec, steps):
        """Launch-averaged time, §8(d) bytes and flops of one KERNELS entry,
        and its summed time per step over ``steps`` timed steps."""
        torch.cuda.synchronize()
        rec = [r for name in spec["entries"] for r in self.records.get(name, ())
               if spec["keep"](r[2])]
        if not rec:
            return None
        ms = [s.elapsed_time(e) / self.REPEAT for s, e, _ in rec]
        byts = [_call_meta(spec["bytes"], m) for _, _, m in rec]
        fl = [_call_meta(spec["flops"], m) for _, _, m in rec]
        k = len(ms)
        avg_ms = sum(ms) / k
        avg_b, avg_f = sum(byts) / k, sum(fl) / k
        gbs = avg_b / (avg_ms * 1e-3) / 1e9
        tfs = avg_f / (avg_ms * 1e-3) / 1e12
        return {"avg_bytes": avg_b, "avg_flops": avg_f, "avg_ms": avg_ms, "launches": k,
                "per_step_us": sum(ms) / steps * 1e3, "launches_per_step": k / steps,
                "gbs": gbs, "tflops": tfs, "hbm_frac": gbs / HBM_PEAK_GBS,
                "mfma_frac": tfs / F32_MFMA_PEAK_TFLOPS}


def roofline_entry(kernel, desc, r, variants):
    """`roofline` object: bound = the resource this kernel is closer to
    saturating (both fractions are reported); traffic = PMC HBM bytes per
    launch of the same kernel from TRAFFIC_FILE (null + a note if absent)."""
    if r["mfma_frac"] > r["hbm_frac"]:
        bound, ach, peak, unit = "mfma", r["tflops"], F32_MFMA_PEAK_TFLOPS, "TFLOP/s"
    else:
        bound, ach, peak, unit = "hbm", r["gbs"], HBM_PEAK_GBS, "GB/s"
    traffic = traffic_of(variants)
    t_path, t_data = _for_run(TRAFFIC_SETS)
    r_path, _ = _for_run(REPLAY_SETS)
    out = {"bound": bound, "kernel": kernel, "kernel_desc": desc, "achieved": round(ach, 2),
           "peak": peak, "unit": unit, "frac": round(ach / peak, 4), "traffic": traffic,
           "traffic_file": os.path.relpath(t_path, ROOT),
           "hbm_gbs": round(r["gbs"], 1), "hbm_frac": round(r["hbm_frac"], 4),
           "hbm_frac_vs_measured_copy": round(r["gbs"] / HBM_MEASURED_GBS, 4),
           "mfma_f32_tflops": round(r["tflops"], 2), "mfma_frac": round(r["mfma_frac"], 4),
           "avg_launch_us": round(r["avg_ms"] * 1e3, 3),
           "per_step_us": round(r["per_step_us"], 2),
           "launches_per_step": round(r["launches_per_step"], 2),
           "avg_bytes_per_launch": int(r["avg_bytes"]),
           "avg_flops_per_launch": int(r["avg_flops"]), "launches_timed": r["launches"]}
    rep = replay_of(variants)
    out["replay_file"] = os.path.relpath(r_path, ROOT)
    if rep is None:
        out["replay_avg_us"] = out["replay_frac"] = None
        out["replay_note"] = (f"no replayed-step trace of {RUN_CONFIG} for {variants} in "
                              f"{out['replay_file']}: run tools/gpu_round.sh on this code")
    else:
        d, us = rep
        rate = (r["avg_flops"] / (us * 1e-6) / 1e12 if bound == "mfma" else
                r["avg_bytes"] / (us * 1e-6) / 1e9)
        out["replay_avg_us"] = round(us, 3)
        out["replay_dispatches"] = d
        out["replay_frac"] = round(rate / peak, 4)  # same bytes / flops, replayed launch time
    if traffic is None:
        cfg = t_data.get("_config")
        out["traffic_note"] = (
            f"{out['traffic_file']} holds PMC passes of {cfg}, not of this configuration "
            f"{RUN_CONFIG}" if cfg is not None and cfg != RUN_CONFIG else
            f"no PMC entry for {variants} in {out['traffic_file']}: run tools/gpu_round.sh on "
            "this code")
    else:
        out["traffic_over_algorithmic"] = round(traffic / r["avg_bytes"], 3)
    return out


def superbatch_roofline(dev, n_target=1_200_000, reps=20):
    """GIN gather-scatter on a ZINC-scale superbatch whose [N,64] fp32 features
    (1.2 M nodes: 307 MB) exceed the 256 MiB Infinity Cache, so the rows come
    from HBM (north_star's >= 40 % target).  Measured on the kernels the
    pretrain step runs (models.py:69 GINConv gspmm is fused into them):
    gin_fwd_k (gather + BN/ReLU of the previous layer on load + 2 GEMMs + BN
    tile statistics, d = 64 layers) and gin_bwd_stats_k (the transposed
    gather of d(agg) + mask + BN-backward sums) — one eager forward+backward
    of a GIN-64x5 encoder on the superbatch, every launch HIP-event timed.
    gin_aggregate_k (the plain aggregation, not in the replayed step) is
    kept as a labelled reference kernel."""
    mols = pkg.synth.molecules(int(n_target / 23.2) + 1, "zinc", seed=123)
    g, _ = pkg.graph.collate_pyg(mols)
    g = g.to(dev)
    n, e = g.num_nodes(), g.num_edges()
    h = torch.randn(n, 64, device=dev)
    out = torch.empty_like(h)
    for _ in range(3):
        out = pkg.ops._aggregate(h, g.rowptr, g.col, 1.0)
    torch.cuda.synchronize()
    s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        out = pkg.ops._aggregate(h, g.rowptr, g.col, 1.0)
    t.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(t) / reps
    del out
    res = {"nodes": n, "edges": e, "feature_mb": round(n * 64 * 4 / 1e6, 1),
           "gin_aggregate_k": _frac_entry(agg_bytes(n, e, 64), ms)}
    # the on-path kernels: a GIN-64x5 encoder forward + backward, events per launch
    gin = pkg.models.GIN(64, 64, 5).to(dev).train()
    x = h.requires_grad_(True)
    torch.cuda.synchronize()
    # the statistics kernel alone: the previous layer's slab reduce is not
    # folded into its launches here (stats_bytes counts the gather only)
    fold = pkg.ops.FOLD_SLABS
    pkg.ops.FOLD_SLABS = False
    try:
        with KernelTimer("scgib_gin_layer_fwd_bn", "scgib_gin_bwd_stats_bn",
                         "scgib_gin_bwd_stats_bn_fold", "scgib_gin_layer_bwd",
                         "scgib_gin_layer_bwd_z", "scgib_gin_bwd_stats_z") as timer:
            y = gin(g, x)
            y.sum().backward()
    finally:
        pkg.ops.FOLD_SLABS = fold
    fwd = timer.records["scgib_gin_layer_fwd_bn"]
    st = [rec for name in ("scgib_gin_bwd_stats_bn", "scgib_gin_bwd_stats_bn_fold")
          for rec in timer.records[name] if rec[2]["e"] > 0]
    stz = timer.records["scgib_gin_bwd_stats_z"]
    torch.cuda.synchronize()
    # gin_fwd_k over its d = 64 layers: frac on §8(d)'s aggregation bytes;
    # frac_inclusive counts everything the launch moves (its own saved
    # z2 (+ r if stored, + agg unless agg-free) writes and the weights too);
    # mfma_frac on its two GEMMs.  This GIN runs on a given h0, so its layer 0
    # is a d_in = 64 layer that stores agg (the step's layer 0 is the
    # transfer_d fold, d_in = 32): gin_fwd_k averages all five, and
    # gin_fwd_k_agg_free the four agg-free ones — the step's d = 64 layers
    fwd = [rec for rec in fwd if rec[2]["d_in"] == 64]
    fwd_free = [rec for rec in fwd if not rec[2].get("agg", True)]
    for key, recs, fn in (("gin_fwd_k", fwd, agg_fwd_bytes),
                          ("gin_fwd_k_agg_free", fwd_free, agg_fwd_bytes),
                          ("gin_bwd_stats_k", st, stats_bytes),
                          ("gin_bwd_statsz_k", stz, statsz_bytes)):
        if recs:
            ms_k = statistics.mean(a.elapsed_time(b) / KernelTimer.REPEAT for a, b, _ in recs)
            m = recs[0][2]
            res[key] = _frac_entry(fn(m["n"], m["e"], m["d_in"]), ms_k)
            res[key]["launches"] = len(recs)
            if key.startswith("gin_fwd_k"):
                inc = statistics.mean(layer_fwd_bytes_inclusive(
                    r[2]["n"], r[2]["e"], r[2]["d_in"], r[2].get("r", False), r[2].get("agg", True))
                    for r in recs)
                res[key]["stores_r"] = bool(m.get("r", False))
                res[key]["stores_agg"] = sum(bool(r[2].get("agg", True)) for r in recs)
                res[key]["bytes_inclusive"] = int(inc)
                res[key]["frac_inclusive"] = round(inc / (ms_k * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                fl = layer_fwd_flops(m["n"], m["e"], m["d_in"])
                res[key]["mfma_frac"] = round(fl / (ms_k * 1e-3) / 1e12 / F32_MFMA_PEAK_TFLOPS, 4)
            if key == "gin_bwd_statsz_k":
                fl = statsz_flops(m["n"], m["e"], m["d_in"])
                res[key]["mfma_frac"] = round(fl / (ms_k * 1e-3) / 1e12 / F32_MFMA_PEAK_TFLOPS, 4)
    # the step's dominant kernel (gin_bwd5_k, d_in = 64 layers) at this scale:
    # ~37 k sub-tiles, ~146 per workgroup, so its start-of-kernel chain is
    # amortised — the steady-state rate of the sub-tile loop
    bw = [rec for rec in timer.records["scgib_gin_layer_bwd"] if rec[2]["d_in"] == 64]
    if bw:
        ms_k = statistics.mean(a.elapsed_time(b) / KernelTimer.REPEAT for a, b, _ in bw)
        m = bw[0][2]
        fl = layer_bwd_flops(m["n"], m["e"], m["d_in"])
        ent = _frac_entry(layer_bwd_bytes(m["n"], m["e"], m["d_in"], m.get("r", False)), ms_k)
        ent["recomputes_r"] = not m.get("r", False)
        ent["tflops"] = round(fl / (ms_k * 1e-3) / 1e12, 2)
        ent["mfma_frac"] = round(fl / (ms_k * 1e-3) / 1e12 / F32_MFMA_PEAK_TFLOPS, 4)
        ent["launches"] = len(bw)
        res["gin_bwd5_k"] = ent
    bz = timer.records["scgib_gin_layer_bwd_z"]
    if bz:
        ms_k = statistics.mean(a.elapsed_time(b) / KernelTimer.REPEAT for a, b, _ in bz)
        m = bz[0][2]
        fl = bwdz_flops(m["n"], m["e"], m["d_in"])
        ent = _frac_entry(bwdz_bytes(m["n"], m["e"], m["d_in"]), ms_k)
        ent["tflops"] = round(fl / (ms_k * 1e-3) / 1e12, 2)
        ent["mfma_frac"] = round(fl / (ms_k * 1e-3) / 1e12 / F32_MFMA_PEAK_TFLOPS, 4)
        ent["launches"] = len(bz)
        res["gin_bwd5z_k"] = ent
    if "gin_bwd5z_k" in res and "gin_bwd_statsz_k" in res:
        # an agg-free layer's whole backward (the statistics launch below it
        # and its own): against gin_bwd_stats_k + gin_bwd5_k of a stored-agg layer
        res["agg_free_layer_bwd_us"] = round(res["gin_bwd5z_k"]["us"]
                                             + res["gin_bwd_statsz_k"]["us"], 2)
    del y, x, h, gin
    # rocprofv3 evidence of these launches (same program, separate runs):
    # the traced average duration beside the event time, and the PMC HBM
    # bytes per launch beside the algorithmic bytes
    ev = _sb_evidence()
    for key in ("gin_fwd_k", "gin_fwd_k_agg_free", "gin_bwd_stats_k", "gin_bwd_statsz_k",
                "gin_bwd5_k", "gin_bwd5z_k", "gin_aggregate_k"):
        e = ev.get(key)
        if key not in res or not e:
            continue
        r = res[key]
        r["trace_avg_us"] = e.get("trace_avg_us")
        if e.get("trace_avg_us"):
            r["trace_vs_event"] = round(e["trace_avg_us"] / r["us"], 4)
        r["traffic"] = e.get("traffic_bytes")
        r["traffic_fetch"] = e.get("fetch_bytes")
        r["traffic_write"] = e.get("write_bytes")
        if e.get("traffic_bytes"):
            r["traffic_over_algorithmic"] = round(e["traffic_bytes"] / r["bytes"], 4)
            r["hbm_frac_measured"] = round(e["traffic_bytes"] / (r["us"] * 1e-6) / 1e9
                                           / HBM_PEAK_GBS, 4)
    if ev:
        res["evidence_file"] = os.path.relpath(SB_FILE, ROOT)
        res["evidence_nodes"] = ev.get("_nodes")
    return res


def _frac_entry(byts, ms):
    gbs = byts / (ms * 1e-3) / 1e9
    return {"bytes": int(byts), "us": round(ms * 1e3, 2), "achieved_gbs": round(gbs, 1),
            "frac": round(gbs / HBM_PEAK_GBS, 4),
            "frac_vs_measured_copy": round(gbs / HBM_MEASURED_GBS, 4)}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def progress(msg):
    """A progress line on stderr (long phases: the driver and gpurun treat a
    silent process as hung)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


# CPU legs run in child processes (a fresh OpenMP pool per thread count, and
# a leg that cannot finish — e.g. hundreds of threads on a small CPU share —
# is stopped at its time limit and reported as such)
LEG_TIMEOUT = {"all_affinity": 150.0, "share": 120.0, "one_core": 150.0}
# BASELINE.md §2's protocol: 3 warm-up steps, then the median of >= 10
CPU_WARMUP, CPU_MIN_STEPS = 3, 10


def _run_leg(name, spec):
    import subprocess
    progress(f"cpu baseline leg {name}: {spec['threads']} threads")
    # (passive OpenMP waits: a thread count far above the CPU share must not
    # spin the share away)
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="",
               OMP_NUM_THREADS=str(spec["threads"]), OMP_WAIT_POLICY="PASSIVE")
    p = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-leg", json.dumps(spec)],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
    t0 = time.perf_counter()
    while True:
        try:
            out, err = p.communicate(timeout=20)
            break
        except subprocess.TimeoutExpired:
            if time.perf_counter() - t0 > LEG_TIMEOUT[name]:
                p.kill()
                p.communicate()
                progress(f"cpu baseline leg {name}: stopped at {LEG_TIMEOUT[name]:.0f} s")
                return None
            progress(f"cpu baseline leg {name}: running ({time.perf_counter() - t0:.0f} s)")
    if p.returncode != 0:
        progress(f"cpu baseline leg {name} failed: {err.strip()[-300:]}")
        return None
    return json.loads(out.strip().splitlines()[-1])


def cpu_baselines(k, gin_layers, workload, batch, seconds=20.0):
    """the CPU path at all the CPUs this process may run on
    (len(os.sched_getaffinity(0)) torch threads: `value`), at the box's CPU
    share (torch's default thread count, OMP_NUM_THREADS) and at 1 core, with
    the CPU model, nproc and the thread counts.  Each leg is a bounded sample
    of ~seconds/2 of CPU work in its own process."""
    threads = torch.get_num_threads()
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or threads
    leg = max(seconds / 2, 5.0)
    legs = {}
    for name, nt in (("all_affinity", affinity), ("share", threads), ("one_core", 1)):
        legs[name] = _run_leg(name, {"threads": nt, "k": k, "gin_layers": gin_layers,
                                     "workload": workload, "batch": batch, "seconds": leg,
                                     "warmup": CPU_WARMUP, "min_steps": CPU_MIN_STEPS})
    done = {k: v for k, v in legs.items() if v is not None}
    if not done:
        return None
    # value: the fastest leg (the CPU path at its best thread count on this
    # host's CPU share); every leg is reported beside it
    best = max(done, key=lambda k: done[k]["value"])
    base = done[best]
    out = dict(base)
    out.update({"cores": base["cores"], "value_leg": best,
                "cpu_model": cpu_model(), "nproc": os.cpu_count(),
                "sched_affinity_cpus": affinity, "torch_default_threads": threads})
    for name, tag in (("all_affinity", "all_affinity"), ("share", "share_threads"),
                      ("one_core", "1core")):
        r = legs[name]
        out[f"value_{tag}"] = r["value"] if r else None
        out[f"ms_per_step_{tag}"] = r["ms_per_step"] if r else None
        out[f"steps_{tag}"] = r["steps"] if r else None
    if legs["all_affinity"] is None:
        out["note"] = (f"the {affinity}-thread leg did not finish within "
                       f"{LEG_TIMEOUT['all_affinity']:.0f} s (threads far above this process's CPU "
                       "share)")
    out["sample"] = base["sample"] + (f"; legs in child processes: {affinity} threads (all "
                                      f"affinity CPUs), {threads} threads (CPU share), 1 thread; "
                                      f"value = the fastest leg ({best})")
    return out


def _cpu_leg_main(spec_json):
    """Child of _run_leg: one CPU leg, its result as a JSON line."""
    spec = json.loads(spec_json)
    torch.set_num_threads(spec["threads"])
    pool = [pkg.graph.collate_pyg(pkg.synth.molecules(spec["batch"], spec["workload"], seed=i))[0]
            for i in range(2)]
    F_in = pkg.synth.WORKLOADS[spec["workload"]][2]
    r = cpu_baseline(pool, spec["k"], spec["gin_layers"], F_in, spec["workload"], spec["seconds"],
                     warmup=spec["warmup"], min_steps=spec["min_steps"])
    print(json.dumps(r), flush=True)


def cpu_baseline(pool_host, k, gin_layers, F_in, workload, seconds=20.0, warmup=CPU_WARMUP,
                 min_steps=CPU_MIN_STEPS):
    """The oracle (literal restatement of the reference's CPU path: per-graph
    loops, dense N x N recon) timed on this host's cores, bounded sample."""
    from oracle import egonet
    from oracle import scgib_ref as R

    torch.manual_seed(0)
    model = make_model(F_in, k, gin_layers, "cpu")
    params = {kk: v.detach().clone().requires_grad_(v.is_floating_point() and "running" not in kk
                                                    and not kk.endswith(".eps"))
              for kk, v in R.strip_continue(
                  {kk: v for kk, v in model.state_dict().items()
                   if kk.startswith(("transfer_d.", "MLP.", "model.Encoder", "model.compressor.",
                                     "model.attn_layer."))}).items()}
    buffers = {kk: v for kk, v in params.items() if "running" in kk or "num_batches" in kk}
    opt = torch.optim.Adam([v for v in params.values() if v.requires_grad], lr=1e-4,
                           weight_decay=5e-5)
    times, ego_times = [], []
    t_end = time.perf_counter() + seconds
    i = 0
    while time.perf_counter() < t_end or i < warmup + min_steps:
        gh = pool_host[i % len(pool_host)]
        t0 = time.perf_counter()
        sizes, ecount, nodes, esrc, edst = egonet.egonets(gh.rowptr.numpy(), gh.col.numpy(), k)
        t1 = time.perf_counter()
        off = np.repeat(np.concatenate([[0], np.cumsum(sizes)[:-1]]), ecount)
        counts = torch.from_numpy(gh.batch_num_nodes_host())
        src, dst = gh.edges()
        batch = {"src": src, "dst": dst, "counts": counts}
        ego = {"src": torch.from_numpy(esrc + off), "dst": torch.from_numpy(edst + off),
               "counts": torch.from_numpy(sizes)}
        x = F.normalize(gh.ndata["x"].float())
        xs = x[torch.from_numpy(nodes)]
        t2 = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        out = R.pretrain_forward(params, batch, ego, x, xs, torch.rand(len(x)),
                                 torch.rand(len(x), 64), 512, buffers)
        out["loss_total"].backward()
        opt.step()
        t3 = time.perf_counter()
        if i >= warmup:
            times.append(t3 - t2)
            ego_times.append(t1 - t0)
        i += 1
        if t3 - t0 > 5.0:
            progress(f"  cpu step {i}: {t3 - t2:.1f} s")
    B = gh.batch_size
    step = statistics.median(times)
    return {"value": round(B / step, 2), "unit": "graphs/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": (f"oracle/scgib_ref.py pretrain step (fwd+bwd+Adam, dense NxN recon, "
                       f"per-graph loops) on {B}-molecule {workload}-like batches, k={k}, median of "
                       f"{len(times)} steps after {warmup} warm-up, torch CPU threads="
                       f"{torch.get_num_threads()}, os.cpu_count={os.cpu_count()}; ego-nets "
                       f"pre-extracted as in the reference (oracle/egonet_ref.c, "
                       f"{statistics.median(ego_times) * 1e3:.1f} ms/batch, not in value)"),
            "ms_per_step": round(step * 1e3, 2), "steps": len(times)}


WORKLOAD_DESC = {"qm9": "QM9-like", "molpcba": "ogbg-molpcba-like", "pcqm4mv2": "PCQM4Mv2-like",
                 "zinc": "ZINC-like", "mutagenicity": "Mutagenicity-like",
                 "molhiv": "ogbg-molhiv-like"}


def finetune_leg(a, dev):
    """BASELINE.json configs[4] in the same run (finetune_bench.run: the molhiv
    fine-tune step from the shipped checkpoint's weights, B = 32, captured and
    replayed, a.steps timed after a.warmup), its dominant kernel's roofline and
    its oracle CPU baseline (half the pretrain leg's CPU budget)."""
    import finetune_bench
    global RUN_CONFIG
    keep = RUN_CONFIG
    ns = SimpleNamespace(batch=32, pool=a.pool, steps=a.steps, warmup=a.warmup,
                         no_kernel_timer=a.no_kernel_timer, no_cpu_baseline=a.no_cpu_baseline,
                         cpu_seconds=a.cpu_seconds, no_ego_prefetch=a.no_ego_prefetch,
                         no_split=a.no_split)
    try:
        line = finetune_bench.run(sys.modules[__name__], ns, dev)
    finally:
        RUN_CONFIG = keep
    return {k: line[k] for k in ("metric", "value", "unit", "ms_per_step", "steps", "warmup",
                                 "dtype", "data", "config", "roofline", "critical_path_us",
                                 "cpu_baseline")}


def build_replay_step(model, opt, pool_host, k, batch, dev, prefetch=True, noise=None,
                      collective=False, reducer=None, warm=3, split=True, noise_prefetch=True,
                      fuse_adam=True):
    """The bench's pretrain step (exp_pretraining.py:290-333) as ONE captured
    HIP graph in capacity mode: the pool's next resident batch (and the ego-nets
    the previous step built for it) loaded inside the graph, forward, backward,
    [the RCCL all-reduce of the gradient bucket,] Adam.  ``warm`` eager steps
    on a side stream first (allocator, Adam state, RCCL communicator).
    ``noise`` = (u_gate [n_cap], u_feat [n_cap, 64]) static device buffers the
    step reads instead of drawing its own (tests/test_gpu_trajectory.py fills
    them before each replay); None = the device Philox draws of every replay,
    with ``noise_prefetch`` one step ahead (ops.NoisePrefetch: each step's
    backward draws the next step's noise at the end of its core chain, off
    the forward's critical path; the same draws in the same order).
    ``split``: replay the captured graph as two linear lanes (ops.SplitGraph:
    ~6 us of host enqueue per lane instead of ~3 us per node) where the
    hand-off rule allows and the graph is one launch.
    Returns step(i), the static losses (kl, rec, con), the static batch, the
    device pool and its prefetch, the all-reduce mode, the node count of the
    captured graph, the split (None: the captured graph is replayed) and the
    noise prefetch (None: drawn in the forward, or passed in).  ``fuse_adam``
    (no collective): the ego chain's final weight-gradient reduce and Adam
    as one launch (ops.fuse_final_into_step; the same bits)."""
    n_cap, e_cap, mgn, ego_caps = pkg.graph.StaticBatch.capacities(pool_host, k, slack=1.02)
    F_in = pool_host[0].ndata["x"].shape[1]
    static = pkg.graph.StaticBatch(batch, n_cap, e_cap, F_in, mgn, ego_caps, dev, k=k)
    padded = []
    for gh in pool_host:
        gx = pkg.graph.GraphBatch.from_edges(*[t.numpy() for t in gh.edges()], gh.num_nodes(),
                                             True, gh.batch_num_nodes_host())
        dict.__setitem__(gx.ndata, "x", F.normalize(gh.ndata["x"].float()))
        padded.append(static.pad(gx))

    pool_dev = static.pool(padded)
    one = torch.ones((), dtype=torch.float32, device=dev)
    # each step builds the NEXT batch's ego-nets (on the encoder
    # pair's queue during the loss section) and its batch load moves them
    # in with the batch: the build leaves the head of the critical path
    pf = None
    if prefetch:
        pf = pkg.graph.EgoPrefetch(static, pool_dev)
        pf.prime()  # the first batch's, before the first load
    nf = None
    if noise is None and noise_prefetch:  # the device noise one step ahead (ops.NoisePrefetch)
        nf = pkg.ops.NoisePrefetch(static.graph, dev)
        nf.prime()

    def body():
        # the pool's next batch (and its prefetched ego-nets) into the static inputs
        pkg.ops.stamp("step_start")
        static.load_next(pool_dev, pf)
        pkg.ops.stamp("loaded")
        _, kl, con, rec = model(static.graph, static.x, None, None, None, 1, None, k, dev,
                                batch, noise=noise)
        # loss = KL + contrastive + recon (exp_pretraining.py:321): d loss / d part = 1,
        # so the parts are backpropagated directly with a resident ones scalar (no sum
        # kernels, no ones fill in the replayed step); the total is formed after timing
        torch.autograd.backward((kl, rec, con), (one, one, one))
        if pf is not None:
            pf.join()  # (no-op: the encoder pair's backward joined it)
        # detached aliases (the replays refresh their storage): the step's
        # autograd graph is not kept alive past the capture
        return (kl.detach(), rec.detach(), con.detach())

    def bucket():
        reducer.pack()
        reducer.reduce(force=True)
        reducer.unpack()

    def fused():  # (a collective reads the gradients between the backward and the step)
        return (pkg.ops.fuse_final_into_step() if fuse_adam and not collective
                else contextlib.nullcontext())

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # warm-up (allocator, Adam state, RCCL comm) off the capture
        for i in range(warm):
            opt.zero_grad(set_to_none=True)
            with fused():
                body()
                if collective:
                    bucket()
                opt.step()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph2 = None
    if os.environ.get("SCGIB_STAMPS"):  # diagnostics: wall-clock stamps in the captured step
        pkg.ops.stamps_enable(dev, int(os.environ["SCGIB_STAMPS"]))
    # keep_graph: the captured graph stays queryable for its node count
    # (graph_node_counts) and is instantiated explicitly below
    graph = torch.cuda.CUDAGraph(keep_graph=True)
    opt.zero_grad(set_to_none=True)
    # N > 1: the RCCL all-reduce captured inside the replayed step graph
    # (falls back to the all-reduce between two replays if the capture raises)
    capture_ok = dist.is_initialized() and dist.get_backend() == "nccl"
    allreduce_mode = None
    if collective and capture_ok:  # (gloo's all-reduce is a host round trip: not capturable)
        # the whole step incl. the RCCL all-reduce of the bucket in ONE graph:
        # no host enqueue between the backward and the optimizer step
        try:
            # thread_local: the process group's watchdog thread queries the
            # warm-up all-reduce's event while this thread captures; under
            # the default global mode that query invalidates the capture
            with torch.cuda.graph(graph, capture_error_mode="thread_local"):
                static_loss = body()
                bucket()
                opt.step()
            allreduce_mode = "captured in the step graph"
        except Exception as exc:  # RCCL without graph-capture support: two graphs
            print(f"bench: all-reduce capture failed ({exc!r}); two-graph fallback",
                  file=sys.stderr, flush=True)
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph(keep_graph=True)
            opt.zero_grad(set_to_none=True)
            graph2 = "fallback"
    if not collective:
        with torch.cuda.graph(graph), fused():
            static_loss = body()
            opt.step()
    elif graph2 is not None or not capture_ok:
        with torch.cuda.graph(graph):  # gradients -> the flat bucket, one launch
            static_loss = body()
            reducer.pack()
        graph2 = torch.cuda.CUDAGraph()  # 1/world unpack + Adam, after the all-reduce
        with torch.cuda.graph(graph2):
            reducer.unpack()
            opt.step()
        allreduce_mode = "between two graph replays"
    nodes = graph_node_counts(graph)
    # (one process per GPU with the RCCL all-reduce in the graph keeps the whole
    # graph: its collective nodes are not exercised by the split's tests here)
    lanes = split_graph(graph, dev) if (split and not collective) else None
    if lanes is None:
        graph.instantiate()

    def step(i):
        if lanes is not None:
            lanes.replay()
            return static_loss
        graph.replay()
        if graph2 is not None:  # RCCL all-reduce of the bucket between the two replays
            reducer.reduce(force=True)
            graph2.replay()
        return static_loss

    # `one` is read by the captured backward through its device pointer only:
    # the namespace holds it, or the allocator would hand its block to the next
    # allocation and the replays would seed the backward with whatever lands there
    return SimpleNamespace(step=step, loss=static_loss, static=static, pool=pool_dev,
                           padded=padded, prefetch=pf, allreduce_mode=allreduce_mode,
                           graph=graph, graph_nodes=nodes, split=lanes, one=one,
                           noise_prefetch=nf)


def split_graph(graph, dev):
    """ops.SplitGraph of a captured step (two linear lanes), or None where the
    hand-offs are off (serialised dispatch: a kernel trace, PMC) or the graph
    does not split (a non-kernel node, e.g. a captured RCCL all-reduce)."""
    if not pkg.ops.xq_enabled():
        return None
    try:
        lanes = pkg.ops.SplitGraph(graph, dev)
    except pkg.ops.SplitUnsupported as exc:
        progress(f"graph replayed whole: {exc}")
        return None
    progress(f"graph split into two lanes: {lanes.info}")
    return lanes


def set_side_cu_mask(dev, k):
    """The encoder pair's side stream (models._side_stream) as a HIP stream
    restricted to the device's last k CUs (hipExtStreamCreateWithCUMask;
    tools/cumask_probe.hip: a captured node keeps its stream's mask when the
    graph is replayed on another stream, as torch replays it)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    words = (ncu + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for i in range(ncu - k, ncu):
        mask[i // 32] |= 1 << (i % 32)
    s = ctypes.c_void_p()
    if hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), words, mask) != 0:
        raise SystemExit("hipExtStreamCreateWithCUMask failed")
    ext = torch.cuda.ExternalStream(s.value, device=dev)
    pkg.models._SIDE_STREAMS[dev.index] = pkg.ops.register_fork_stream(ext)
    progress(f"side stream on CUs [{ncu - k}, {ncu})")


def graph_node_counts(graph):
    """{kernel, memcpy, memset, other, total} nodes of a captured torch
    CUDAGraph (hipGraphGetNodes + hipGraphNodeGetType through ops), or None
    where the runtime does not expose the graph."""
    try:
        return pkg.ops.graph_node_counts(graph)
    except Exception as exc:  # noqa: BLE001 (diagnostic field only)
        progress(f"graph node count unavailable: {exc!r}")
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="qm9")
    ap.add_argument("--batch", type=int, default=512,
                    help="molecules per GPU (weak scaling: per-GPU work fixed as N grows)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="strong scaling: this many molecules per step in total, "
                         "split evenly over the ranks (BASELINE.md §3: 1024 = 128/rank at 8)")
    ap.add_argument("--force-allreduce", action="store_true",
                    help="run the gradient all-reduce (and its graph capture) even at N=1 "
                         "(a 1-rank process group; exercises the collective path on one GPU)")
    ap.add_argument("--k", type=int, default=1)
    ap.add_argument("--gin-layers", type=int, default=5)
    ap.add_argument("--pool", type=int, default=8)
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-superbatch", action="store_true")
    ap.add_argument("--superbatch-only", action="store_true",
                    help="only the superbatch pass (a program for rocprofv3 kernel-trace / PMC "
                         "passes over exactly those launches: tools/sb_evidence.py)")
    ap.add_argument("--no-kernel-timer", action="store_true",
                    help="skip the event-timed kernel pass (PMC runs: only real step launches)")
    ap.add_argument("--eager", action="store_true",
                    help="launch every kernel from Python (no HIP-graph capture)")
    ap.add_argument("--no-fuse-adam", action="store_true",
                    help="launch the ego chain's final weight-gradient reduce and Adam "
                         "separately (ops.fuse_final_into_step; A/B)")
    ap.add_argument("--no-noise-prefetch", action="store_true",
                    help="pretrain: draw each step's compression noise at the head of its forward "
                         "core chain instead of in the step before's backward (ops.NoisePrefetch; "
                         "A/B; the fine-tune step draws it in its forward)")
    ap.add_argument("--no-split", action="store_true",
                    help="replay the captured step graph whole instead of as two linear lanes "
                         "(ops.SplitGraph; A/B of the host enqueue)")
    ap.add_argument("--no-ego-prefetch", action="store_true",
                    help="build each step's ego-nets at the head of the step instead of one "
                         "batch ahead (graph.EgoPrefetch; A/B)")
    ap.add_argument("--torch-adam", action="store_true",
                    help="torch's fused Adam instead of the one-launch scgib Adam")
    ap.add_argument("--recompute-r", action="store_true",
                    help="the GIN forward does not store r, the backward recomputes it "
                         "(ops.STORE_R = False; A/B, same bits: profiles/r05_recompute)")
    ap.add_argument("--no-agg-free", action="store_true",
                    help="every GIN layer stores agg and runs the stored-agg backward "
                         "(ops.AGG_FREE = False; A/B)")
    ap.add_argument("--agg-free-min-rows", type=int, default=None,
                    help="encoders of at least this many rows run agg-free "
                         "(ops.AGG_FREE_MIN_ROWS; 0: every encoder; A/B)")
    ap.add_argument("--side-cu-mask", type=int, default=0,
                    help="probe (VERDICT r05 item 4): the encoder pair's side stream made with "
                         "hipExtStreamCreateWithCUMask on the last K CUs (0: an ordinary stream)")
    ap.add_argument("--finetune", choices=["molhiv"], default=None,
                    help="time the fine-tune step of BASELINE.json configs[4] instead "
                         "(finetune_bench.py; --batch defaults to 32 there)")
    ap.add_argument("--no-handoffs", action="store_true",
                    help="the encoder pair joins its streams with ordinary stream edges instead "
                         "of signal / wait kernels (ops.XQ_FLAGS = False; A/B)")
    ap.add_argument("--torch-head", action="store_true",
                    help="fine-tune: torch's predict head / sigmoid / BCE instead of csrc/head.hip "
                         "(models.FUSE_HEAD; A/B)")
    ap.add_argument("--no-finetune", action="store_true",
                    help="skip the fine-tune leg (configs[4]) the N = 1 line carries in 'finetune'")
    a = ap.parse_args()
    pkg.ops.STORE_R = not a.recompute_r
    pkg.ops.AGG_FREE = not a.no_agg_free
    if a.agg_free_min_rows is not None:
        pkg.ops.AGG_FREE_MIN_ROWS = a.agg_free_min_rows
    if a.superbatch_only:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        print(json.dumps({"roofline_superbatch": superbatch_roofline(dev)}), flush=True)
        return
    pkg.models.FUSE_HEAD = not a.torch_head
    if a.finetune:
        import finetune_bench
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        finetune_bench.main_line(sys.modules[__name__], a, dev)
        return

    rank, world, local = pkg.dist.init_from_env()
    if a.force_allreduce and world == 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        torch.cuda.set_device(local)
        dist.init_process_group(os.environ.get("SCGIB_DIST_BACKEND") or "nccl",
                                rank=0, world_size=1)
    collective = world > 1 or a.force_allreduce
    if a.global_batch:
        if a.global_batch % world:
            raise SystemExit(f"--global-batch {a.global_batch} is not a multiple of {world} ranks")
        a.batch = a.global_batch // world
    # (more ranks than devices only in local gloo rehearsals: ranks share GPUs)
    dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)
    # the encoder pair's signal / wait hand-offs need one process's two
    # queues to run concurrently (ops.handoff_rule: e.g. ranks sharing a GPU
    # are time-sliced processes); where the rule refuses, ordinary stream edges
    xq_env = dict(os.environ)
    xq_env.setdefault("LOCAL_WORLD_SIZE", str(world))
    xq_ok, xq_why = pkg.ops.handoff_rule(torch.cuda.device_count(), xq_env)
    pkg.ops.XQ_FLAGS, pkg.ops.XQ_REASON = xq_ok, xq_why
    if xq_ok and a.no_handoffs:
        pkg.ops.XQ_FLAGS, pkg.ops.XQ_REASON = False, "--no-handoffs"
    if a.side_cu_mask:
        set_side_cu_mask(dev, a.side_cu_mask)
    torch.manual_seed(1234 + rank)
    global RUN_CONFIG
    RUN_CONFIG = {"workload": a.workload, "batch": a.batch, "k": a.k}
    F_in = pkg.synth.WORKLOADS[a.workload][2]

    # per-rank pool of distinct batches, resident in HBM
    pool_host, pool = [], []
    for i in range(a.pool):
        mols = pkg.synth.molecules(a.batch, a.workload, seed=100_000 * rank + i)
        gh, _ = pkg.graph.collate_pyg(mols)
        pool_host.append(gh)
        g = gh.to(dev)
        dict.__setitem__(g.ndata, "x", F.normalize(g.ndata["x"].float()))  # exp_pretraining.py:312
        pool.append(g)

    model = make_model(F_in, a.k, a.gin_layers, dev)
    # rank 0's initial weights everywhere (each rank's seed still drives its
    # own Gumbel / noise draws): replicas from the first step on
    pkg.dist.broadcast_replicas(model)
    # gradients + the BN running statistics, averaged in one bucket per step
    reducer = pkg.dist.GradAllReducer(model.parameters(), buffers=pkg.dist.bn_buffers(model))

    graph_nodes = None
    noise_draw = "in the step's forward, head of the core chain"
    if a.eager:
        opt = (torch.optim.Adam(model.parameters(), lr=1e-4, weight_decay=5e-5, fused=True)
               if a.torch_adam else pkg.optim.Adam(model.parameters(), lr=1e-4, weight_decay=5e-5))

        def step(i):
            g = pool[i % len(pool)]
            opt.zero_grad(set_to_none=True)
            _, kl, con, rec = model(g, g.ndata["x"], None, None, None, 1, None, a.k, dev, a.batch)
            loss = kl + rec + con
            loss.backward()
            if collective:
                reducer.pack()
                reducer.reduce(force=True)
                reducer.unpack()
            opt.step()
            return loss
    else:
        if a.torch_adam:
            opt = torch.optim.Adam(model.parameters(), lr=1e-4, weight_decay=5e-5,
                                   capturable=True, fused=True)
        else:  # one-launch device Adam, same arithmetic (tests/test_gpu_optim.py)
            opt = pkg.optim.Adam(model.parameters(), lr=1e-4, weight_decay=5e-5)
        rs = build_replay_step(model, opt, pool_host, a.k, a.batch, dev,
                               prefetch=not a.no_ego_prefetch, collective=collective,
                               reducer=reducer, split=not a.no_split,
                               noise_prefetch=not a.no_noise_prefetch,
                               fuse_adam=not a.no_fuse_adam)
        step, allreduce_mode, graph_nodes = rs.step, rs.allreduce_mode, rs.graph_nodes
        if rs.noise_prefetch is not None:
            noise_draw = "in the step before's backward, core chain end (ops.NoisePrefetch)"
        if graph_nodes is not None:  # the replayed lanes (ops.SplitGraph), or the whole graph
            graph_nodes = dict(graph_nodes, replay=(
                {k: rs.split.info[k] for k in ("lane0_nodes", "lane1_nodes", "handoffs")}
                if rs.split is not None else "whole graph"))

    if os.environ.get("SCGIB_PRELOAD_MS"):  # diagnostics only (DESIGN §5 "Round 6"): busy
        # the GPU for that long before the warm-up, to tell a clock ramp from
        # a per-launch effect in the first timed steps; never set by the driver
        t_end = time.perf_counter() + float(os.environ["SCGIB_PRELOAD_MS"]) / 1e3
        m = torch.randn(2048, 2048, device=dev)
        while time.perf_counter() < t_end:
            for _ in range(8):
                m = torch.tanh(m @ m * 1e-3)
            torch.cuda.synchronize()
    if os.environ.get("SCGIB_PRELAUNCH"):  # diagnostics only: that many one-element
        # kernel launches before the warm-up (a per-launch effect, not a clock one)
        t = torch.zeros(1, device=dev)
        for _ in range(int(os.environ["SCGIB_PRELAUNCH"])):
            t.add_(1.0)
        torch.cuda.synchronize()
    for i in range(a.warmup):
        step(i)
    progress(f"warm-up done ({a.warmup} steps); timing {a.steps} steps")
    if os.environ.get("SCGIB_IDLE_MS"):  # diagnostics only: the GPU idle that long
        torch.cuda.synchronize()  # between the warm-up and the timed steps
        time.sleep(float(os.environ["SCGIB_IDLE_MS"]) / 1e3)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    if os.environ.get("SCGIB_STAMPS_FIRST"):  # diagnostics: the stamps of one step from idle
        step(a.warmup)
        barrier()
        for lab, us in pkg.ops.stamps_read():
            progress(f"first-step stamp {us:9.2f} us  {lab}")
        barrier()
    # SCGIB_STEP_PROBE=1 (diagnostics only, tools/gpu_steps_probe.sh): HIP events
    # around every timed step
    probe = [] if os.environ.get("SCGIB_STEP_PROBE") == "1" else None
    host_us = [] if probe is not None else None
    t0 = time.perf_counter()
    for i in range(a.steps):
        if probe is not None:
            probe.append(torch.cuda.Event(enable_timing=True))
            probe[-1].record()
            th = time.perf_counter()
        loss = step(a.warmup + i)
        if probe is not None:
            host_us.append((time.perf_counter() - th) * 1e6)
    if probe is not None:
        probe.append(torch.cuda.Event(enable_timing=True))
        probe[-1].record()
    t_enq = time.perf_counter() - t0  # host time to enqueue the K steps
    barrier()
    elapsed = time.perf_counter() - t0
    if os.environ.get("SCGIB_STAMPS"):
        for lab, us in pkg.ops.stamps_read():
            progress(f"stamp {us:9.2f} us  {lab}")
    if probe is not None:
        progress("step probe (ms): " + " ".join(
            f"{probe[i].elapsed_time(probe[i + 1]):.4f}" for i in range(len(probe) - 1)))
        progress("host replay (us): " + " ".join(f"{u:.0f}" for u in host_us))
    progress(f"timed: {elapsed / a.steps * 1e3:.4f} ms/step, host enqueue "
             f"{t_enq / a.steps * 1e3:.4f} ms/step")
    xq_to = pkg.ops.xq_timeouts(dev)
    if xq_to:  # a hand-off wait gave up: its queue ran ahead of the data
        raise SystemExit(f"bench: {xq_to} cross-queue hand-off waits timed out (ops.XQ_FLAGS)")
    pkg.ops.check_handoff(dev)
    replica_diff = None
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # replica mode's invariant after the timed steps: every rank holds the
        # same parameters and BatchNorm statistics (the averaged bucket is
        # applied identically) — the largest difference to rank 0's, any rank
        flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()] +
                         [b.reshape(-1) for b in pkg.dist.bn_buffers(model)])
        ref = flat.clone()
        dist.broadcast(ref, 0)
        d = (flat - ref).abs().max().reshape(1).double()
        dist.all_reduce(d, op=dist.ReduceOp.MAX)
        replica_diff = float(d.item())
    final_loss = float(sum(loss).item()) if isinstance(loss, tuple) else float(loss.item())

    # instrumented eager pass over the same batches: HIP events around every
    # launch of the measured kernel (forward+backward of the same model)
    # (one stream: the encoder branches are not forked here, so no other
    # kernel runs inside a bracket)
    kernels = {}
    fork_losses = pkg.models.FORK_LOSSES
    if not a.no_kernel_timer:
        entries = [e for spec in KERNELS.values() for e in spec["entries"]]
        timed_steps = min(a.steps, 10)
        pkg.models.FORK_ENCODERS = pkg.models.FORK_LOSSES = False
        try:
            with KernelTimer(*entries) as timer:
                for i in range(timed_steps):
                    g = pool[i % len(pool)]
                    model.zero_grad(set_to_none=True)
                    _, kl, con, rec = model(g, g.ndata["x"], None, None, None, 1, None, a.k, dev,
                                            a.batch)
                    (kl + rec + con).backward()
        finally:
            pkg.models.FORK_ENCODERS = True
            pkg.models.FORK_LOSSES = fork_losses
        for name, spec in KERNELS.items():
            r = timer.kernel_summary(spec, timed_steps)
            if r is not None:
                kernels[name] = roofline_entry(name, spec["desc"], r, spec["pmc"])
    progress("timed steps and kernel timer done")
    # the dominant kernel = the largest summed time per step (kernel-timer pass)
    dominant = max(kernels, key=lambda k: kernels[k]["per_step_us"]) if kernels else None

    sb = None if a.no_superbatch or rank != 0 else superbatch_roofline(dev)
    if sb is not None:
        progress("superbatch roofline done")
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baselines(a.k, a.gin_layers, a.workload, a.batch, a.cpu_seconds)
    ft = None
    if rank == 0 and world == 1 and not a.no_finetune:
        ft = finetune_leg(a, dev)
        progress("fine-tune leg done")

    if rank == 0:
        total_graphs = world * a.batch * a.steps
        n_nodes = statistics.mean(g.num_nodes() for g in pool)
        line = {
            "metric": f"graphs/sec (pretrain step, GIN-64×{a.gin_layers}, k={a.k}) at "
                      f"1/2/4/8 MI355X; % HBM roofline",
            "value": round(total_graphs / elapsed, 1),
            "unit": "graphs/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if a.global_batch else "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": f"synthetic (seeded {WORKLOAD_DESC.get(a.workload, a.workload)} molecules, "
                    f"SURVEY.md §8(d)); random-init weights",
            "config": {"workload": f"{a.workload} pretrain step GIN-64x{a.gin_layers} "
                                   f"k={a.k}, batch {a.batch}/GPU, Mainmodel_continue + Adam",
                       "launch": "eager" if a.eager else (
                           "hip-graph replay (capacity mode)" + (
                               ", two linear lanes" if isinstance((graph_nodes or {}).get("replay"), dict)
                               else "")),
                       "ego_build": ("in the step, for the batch the next step loads "
                                     "(graph.EgoPrefetch)" if not a.eager
                                     and not a.no_ego_prefetch else "at the head of the step"),
                       "noise_draw": noise_draw,
                       "adam": ("one launch with the ego chain's final weight-gradient reduce "
                                "(scgib_adam_step_reduce)" if not (a.eager or collective
                                                                  or a.no_fuse_adam)
                                else "its own launch"),
                       "allreduce": None if not collective else
                       ("eager" if a.eager else allreduce_mode),
                       "handoffs": ("signal / wait kernels" if pkg.ops.xq_enabled() else
                                    f"stream edges ({pkg.ops.XQ_REASON})"),
                       "global_batch": world * a.batch, "nodes_per_batch": round(n_nodes, 1),
                       # the replayed step graph's nodes by kind (each is host
                       # enqueue work) and the host's enqueue time per timed step
                       "graph_nodes": graph_nodes,
                       "host_enqueue_ms": round(t_enq / a.steps * 1e3, 4),
                       "parallelism": f"dp{world}", "final_loss": round(final_loss, 4),
                       "replica_max_abs_diff": replica_diff,
                       "bn_semantics": ("single rank: BatchNorm statistics over the whole batch"
                                        if world == 1 else
                                        "replica mode (DESIGN.md §6): each rank's BatchNorm, "
                                        "contrastive, recon and last-graph KL over its own "
                                        f"{a.batch}-molecule sub-batch (= the reference at batch "
                                        f"{a.batch}); gradients and BN running statistics "
                                        "averaged over ranks by the one all-reduce")},
            # the kernel with the largest summed time per step in the kernel-timer
            # pass; every timed kernel's entry is in roofline_kernels
            "roofline": kernels.get(dominant),
            "roofline_kernels": kernels or None,
            "roofline_superbatch": None if sb is None else dict(
                sb, bound="hbm", peak=HBM_PEAK_GBS, unit="GB/s",
                note="ZINC-like superbatch, [N,64] fp32 > 256 MiB Infinity Cache; frac = "
                     "algorithmic bytes / launch time / 8.0 TB/s (north_star target >= 0.40 on "
                     "the on-path gather kernels; gin_aggregate_k is a reference kernel, not in "
                     "the step).  At this size layers 1-4 run agg-free "
                     "(ops.AGG_FREE_MIN_ROWS): gin_fwd_k_agg_free = those four forward launches "
                     "(no aggregate store, the step's d = 64 layers), gin_fwd_k = all five "
                     "(this GIN's layer 0 is a d_in = 64 layer that stores its aggregate); "
                     "the backward pair is gin_bwd_statsz_k (gather of dz1, dh = g W1, "
                     "dW1 = g^T h, BN-backward sums) + gin_bwd5z_k (dz1, dW2, db2, db1); "
                     "gin_bwd_stats_k / gin_bwd5_k appear when the stored-agg path runs "
                     "(--no-agg-free).  gin_fwd_k frac on §8(d) aggregation bytes, "
                     "frac_inclusive on everything the launch moves (its saved-activation "
                     "writes too); mfma_frac = flops / time / 157.3 TF/s"),
            "cpu_baseline": cpu,
            # BASELINE.json configs[4] (molhiv fine-tune from the shipped
            # checkpoint, B = 32, 1 GPU): its own timed replay after this leg
            "finetune": ft,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    if len(sys.argv) == 3 and sys.argv[1] == "--cpu-leg":
        _cpu_leg_main(sys.argv[2])
    else:
        main()

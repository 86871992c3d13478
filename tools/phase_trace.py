"""Per-workgroup phase timeline of the fused GIN layer kernels (debug build).

    make -C s-cgib_amd/csrc trace
    SCGIB_LIB=$PWD/s-cgib_amd/libscgib_trace.so python tools/phase_trace.py
    (PT_BATCH=32: the same step at the fine-tune batch size)

Runs one eager pretrain step of the bench workload on one stream; every
launch routed through ops._launch is synchronised and its [grid][8] wall-clock
stamps (100 MHz, common.h SCGIB_MARK; [grid][32]: wall clock, then shader
clock) are summarised: kernel span, spread of
workgroup start times, and per-phase durations (median / p90 / max, us).
"""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("s-cgib_amd")
import bench  # noqa: E402

PHASES = {
    "scgib_egonet_k1_build_onepass": ["window", "count", "lookback", "fill"],
    "scgib_gin_layer_fwd_bn": ["gather", "gemm1", "gemm2+st", "tilestat", "bn_hier"],
    "scgib_gin_layer0_fwd": ["gather", "gemm1", "gemm2+st", "tilestat", "bn_hier"],
    # gin_bwd5_k: marks of the first sub-tile, then the remaining sub-tiles
    "scgib_gin_layer_bwd": ["prologue", "dz2", "pairA", "pairB", "rest", "slab"],
    # gin_bwdf_k: + layer l-1's statistics (gather from the LDS d(agg) image)
    "scgib_gin_layer_bwd_fused": ["prologue", "dz2", "pairA", "pairB", "rest", "stats", "bn_hier"],
    "scgib_gin_layer0_bwd": ["ld+dz2", "dW2,dr", "dW1,dagg", "slab"],
    "scgib_gin_bwd_stats_bn": ["gather+dy", "bn_hier"],
    # the agg-free pair (ops.AGG_FREE): the statistics walk's first tile, then
    # its dW1 slab + BN arrivals; the layer backward as gin_bwd5_k (no pair B)
    "scgib_gin_bwd_stats_z": ["gather+img", "gemms+stage", "stats", "slab+hier"],
    "scgib_gin_layer_bwd_z": ["prologue", "dz2", "pairA", "-", "rest", "slab"],
    "scgib_gin_bwd_stats_bn_fold": ["gather+dy", "bn_hier"],
    # head MLP (+ recon) tiles mark 1..3, the contrastive workgroups 5
    # (+ the fused loss finish: published, waited + acquire, then recon_fin.h's
    # edge gather, Gram chunks, arrival / last-arrival loss)
    "scgib_mlp2_recon_contrastive_fwd": ["load", "gemm1", "-", "-", "contrast", "gemm2+pub",
                                         "wait+acq", "fin:edges", "fin:gram", "fin:arrive"],
    "scgib_mlp2_recon_contrastive_bwd": ["dz2(recon)", "dW2,dr,dz1", "dW1,dx", "-", "contrast"],
    # one wave per graph (padding blocks carry no marks)
    "scgib_interaction_fwd": ["gptr", "passA+red", "stats", "passB", "end"],
    "scgib_interaction_bwd": ["ld stats", "attention", "compress", "bn bwd"],
}
MAXB = 4096


def main():
    assert os.environ.get("SCGIB_LIB", "").endswith("libscgib_trace.so"), "use the trace build"
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    lib = pkg._lib.load()
    buf = torch.zeros(MAXB * 32, dtype=torch.int64, device=dev)
    lib.scgib_trace_set.argtypes = [ctypes.c_void_p]
    assert lib.scgib_trace_set(ctypes.c_void_p(buf.data_ptr())) == 0
    F_in = pkg.synth.WORKLOADS["qm9"][2]
    B = int(os.environ.get("PT_BATCH", "512"))  # e.g. 32: the fine-tune batch size
    mols = pkg.synth.molecules(B, "qm9", seed=0)
    gh, _ = pkg.graph.collate_pyg(mols)
    g = gh.to(dev)
    dict.__setitem__(g.ndata, "x", F.normalize(g.ndata["x"].float()))
    model = bench.make_model(F_in, 1, 5, dev)
    pkg.models.FORK_ENCODERS = False
    recs = []

    def observe(name, meta, launch):
        if name not in PHASES:
            return launch()
        torch.cuda.synchronize()
        buf.zero_()
        out = launch()
        torch.cuda.synchronize()
        recs.append((name, meta, buf.view(MAXB, 32).cpu().numpy().copy()))
        return out

    for it in range(2):  # second iteration: warm caches / allocator
        recs.clear()
        pkg.ops.OBSERVER = observe if it == 1 else None
        _, kl, con, rec = model(g, g.ndata["x"], None, None, None, 1, None, 1, dev, B)
        (kl + con + rec).backward()
        torch.cuda.synchronize()
    pkg.ops.OBSERVER = None
    for name, meta, t in recs:
        nb = int((t[:, 0] != 0).sum())
        if nb == 0:
            print(f"{name}: no stamps")
            continue
        t = t[:nb]
        ph = PHASES[name]
        start = t[:, 0]
        t0 = start.min()
        ends = np.where(t[:, 1:1 + len(ph)] != 0, t[:, 1:1 + len(ph)], 0)
        last = ends.max()
        hw = t[:, 15]
        xcc = (hw >> 32) & 0xF
        cu = (hw >> 8) & 0xF
        se = (hw >> 13) & 0x7
        sh = (hw >> 12) & 1
        ncu = len(set(zip(xcc.tolist(), se.tolist(), sh.tolist(), cu.tolist())))
        print(f"{name} n={meta.get('n')} d_in={meta.get('d_in')} blocks={nb} distinct_CUs={ncu} "
              f"span={(last - t0) / 100:.2f}us start_spread(p50/p90/max)="
              f"{np.percentile(start - t0, 50) / 100:.2f}/{np.percentile(start - t0, 90) / 100:.2f}/"
              f"{(start - t0).max() / 100:.2f}us")
        prev = start
        prevc = t[:, 16]
        for k, pname in enumerate(ph):
            col = t[:, 1 + k]
            ok = col != 0
            if not ok.any():
                continue
            d = (col[ok] - prev[ok]) / 100.0
            cyc = t[:, 17 + k][ok] - prevc[ok]
            ghz = np.where(d > 0, cyc / np.maximum(d, 1e-9) / 1e3, 0)
            print(f"    {pname:10s} n={ok.sum():4d} p50={np.percentile(d, 50):6.2f} "
                  f"p90={np.percentile(d, 90):6.2f} max={d.max():6.2f} us  "
                  f"clock p50={np.percentile(ghz, 50):.2f} GHz  cycles p50={np.percentile(cyc, 50):.0f}")
            prev = np.where(ok, col, prev)
            prevc = np.where(ok, t[:, 17 + k], prevc)
        if name == "scgib_gin_layer_fwd_bn" and (t[:, 6] != 0).any():
            d = (t[:, 6] - start) / 100.0
            print(f"    (finish prev BN: start->mark6 p50={np.percentile(d, 50):.2f} "
                  f"p90={np.percentile(d, 90):.2f} max={d.max():.2f} us)")
            if os.environ.get("FIN_MARKS"):  # debug build with marks 4/5 around the combine
                for a_, b_, lab in ((0, 8, "start->fin"), (8, 9, "fin compute"), (9, 6, "barrier")):
                    d = (t[:, b_] - t[:, a_]) / 100.0
                    print(f"      {lab}: p50={np.percentile(d, 50):.2f} p90={np.percentile(d, 90):.2f}")
        if name == "scgib_gin_layer_bwd" and os.environ.get("BWD2_MARKS"):  # gin_bwd2_k sub-marks
            for a_, b_, lab in ((1, 6, "GEMM1 MFMA"), (6, 2, "db2+dz1"), (2, 7, "db1+GEMM2 MFMA"),
                                (7, 3, "dagg stores")):
                d = (t[:, b_] - t[:, a_]) / 100.0
                cyc = t[:, 16 + b_] - t[:, 16 + a_]
                print(f"      {lab:16s}: p50={np.percentile(d, 50):.2f} us  "
                      f"cycles p50={np.percentile(cyc, 50):.0f}")
        per_cu = {}
        for i in range(nb):
            per_cu.setdefault((xcc[i], se[i], sh[i], cu[i]), []).append(i)
        occ = np.bincount([len(v) for v in per_cu.values()])
        print(f"    blocks/CU histogram: {occ.tolist()}")


if __name__ == "__main__":
    main()

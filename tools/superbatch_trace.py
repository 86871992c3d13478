"""Per-workgroup phase timeline of the GIN forward layer on the ZINC-scale
superbatch (bench.py roofline_superbatch's workload), trace build only:

    make -C s-cgib_amd/csrc trace
    SCGIB_LIB=$PWD/s-cgib_amd/libscgib_trace.so python tools/superbatch_trace.py

One eager GIN-64x5 forward (train); every scgib_gin_layer_fwd_bn launch is
synchronised and its per-workgroup wall-clock stamps (common.h SCGIB_MARK,
100 MHz) summarised: kernel span, phase durations, the serial tail after the
last tile's statistics (the BatchNorm finish of the last arriver), the number
of resident workgroups over time and the tile completion rate.
"""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("s-cgib_amd")

PH = ["gather", "gemm1", "gemm2+st", "tilestat", "bn_hier"]


def main():
    assert os.environ.get("SCGIB_LIB", "").endswith("libscgib_trace.so"), "use the trace build"
    dev = torch.device("cuda", 0)
    n_target = int(os.environ.get("N_TARGET", "1200000"))
    mols = pkg.synth.molecules(int(n_target / 23.2) + 1, "zinc", seed=123)
    g, _ = pkg.graph.collate_pyg(mols)
    g = g.to(dev)
    n = g.num_nodes()
    tiles = (n + 63) // 64
    lib = pkg._lib.load()
    buf = torch.zeros(tiles * 32 + 64, dtype=torch.int64, device=dev)
    lib.scgib_trace_set.argtypes = [ctypes.c_void_p]
    assert lib.scgib_trace_set(ctypes.c_void_p(buf.data_ptr())) == 0
    gin = pkg.models.GIN(64, 64, 5).to(dev).train()
    h = torch.randn(n, 64, device=dev)
    recs = []

    def observe(name, meta, launch):
        if name != os.environ.get("TRACE_ENTRY", "scgib_gin_layer_fwd_bn"):
            return launch()
        torch.cuda.synchronize()
        buf.zero_()
        out = launch()
        torch.cuda.synchronize()
        recs.append((meta, buf[: tiles * 32].view(tiles, 32).cpu().numpy().copy()))
        return out

    with torch.no_grad():
        for it in range(2):
            recs.clear()
            pkg.ops.OBSERVER = observe if it == 1 else None
            gin(g, h)
            torch.cuda.synchronize()
    pkg.ops.OBSERVER = None
    print(f"superbatch n={n} e={g.num_edges()} tiles={tiles}")
    for li, (meta, t) in enumerate(recs):
        nb = int((t[:, 0] != 0).sum())
        t = t[t[:, 0] != 0]
        start = t[:, 0]
        t0 = start.min()
        marks = t[:, 1:6]
        end = np.where(marks != 0, marks, 0).max(axis=1)
        last = end.max()
        print(f"layer {li} d_in={meta.get('d_in')} blocks={nb} span={(last - t0) / 100:.1f}us "
              f"last tile start={(start.max() - t0) / 100:.1f}us")
        prev = start
        for k, p in enumerate(PH):
            col = marks[:, k]
            ok = col != 0
            if not ok.any():
                continue
            d = (col[ok] - prev[ok]) / 100.0
            print(f"    {p:9s} p50={np.percentile(d, 50):6.2f} p90={np.percentile(d, 90):6.2f} "
                  f"max={d.max():7.2f} us")
            prev = np.where(ok, col, prev)
        m4 = marks[:, 3]
        print(f"    tail: last tilestat -> kernel end {(last - m4.max()) / 100:.2f} us; "
              f"tile total p50={np.percentile((end - start) / 100, 50):.2f} us")
        # resident workgroups and completion rate in 10 us windows
        edges = np.arange(t0, last + 1000, 1000)
        res = [int(((start <= x) & (end > x)).sum()) for x in edges[:-1]]
        done = np.histogram(end, bins=edges)[0]
        print("    resident per 10us:", res[:: max(1, len(res) // 24)])
        print("    tiles done per 10us:", done[:: max(1, len(done) // 24)].tolist())


if __name__ == "__main__":
    main()

"""Folded layer-0 forward (BN fused) vs transfer_d + plain fused layer."""
import ctypes
import importlib
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
pkg = importlib.import_module("s-cgib_amd")
L = pkg._lib
P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731


def rel(a, b):
    return float((a.double() - b.double()).norm() / max(b.double().norm(), 1e-30))


def main():
    dev = torch.device("cuda", 0)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for nm in (50, 200, 1000):
        gh, _ = pkg.graph.collate_pyg(pkg.synth.molecules(nm, "qm9", seed=7))
        g = gh.to(dev)
        n = g.num_nodes()
        torch.manual_seed(1)
        x = F.normalize(torch.rand(n, 11)).to(dev)
        wt = torch.randn(32, 11, device=dev) * 0.3
        w1, b1 = torch.randn(64, 32, device=dev) * 0.2, torch.randn(64, device=dev) * 0.1
        w2, b2 = torch.randn(64, 64, device=dev) * 0.2, torch.randn(64, device=dev) * 0.1
        gamma, beta = torch.rand(64, device=dev) + 0.5, torch.randn(64, device=dev) * 0.1
        outs = []
        for fold in (True, False):
            agg = torch.empty(n, 32, device=dev)
            r = torch.empty(n, 64, device=dev)
            z2 = torch.empty(n, 64, device=dev)
            stat = torch.empty(4, 64, device=dev)
            ws = torch.empty(int(L.query("scgib_gin_bn_ws_floats", n)), device=dev)
            cnt = torch.zeros(int(L.query("scgib_gin_counters", n)), dtype=torch.int32, device=dev)
            rm, rv = torch.zeros(64, device=dev), torch.ones(64, device=dev)
            aggx = torch.zeros(n, 16, device=dev)
            if fold:
                L.call("scgib_gin_layer0_fwd", P(x), 11, None, P(wt), P(g.rowptr), P(g.col), n,
                       1.0, P(w1), P(b1), P(w2), P(b2), P(agg), P(aggx), P(r), P(z2), P(gamma),
                       P(beta), 1e-5, 0.1, P(rm), P(rv), None, P(stat), P(ws), P(cnt), None, st)
            else:
                h0 = (x @ wt.t()).contiguous()
                L.call("scgib_gin_layer_fwd_bn", P(h0), 32, None, P(g.rowptr), P(g.col), n, 1.0,
                       P(w1), P(b1), P(w2), P(b2), P(agg), P(r), P(z2), P(gamma), P(beta), 1e-5,
                       0.1, P(rm), P(rv), None, P(stat), P(ws), P(cnt), None, st)
            torch.cuda.synchronize()
            outs.append((agg, r, z2, stat, aggx, rm, rv, cnt))
        a, b = outs
        src, dst = gh.edges()
        ax = x.cpu().double().clone().index_add(0, dst, x.cpu().double()[src])
        print(f"mols={nm} n={n} tiles={(n+63)//64} agg={rel(a[0], b[0]):.2e} r={rel(a[1], b[1]):.2e} "
              f"z2={rel(a[2], b[2]):.2e} stat={rel(a[3], b[3]):.2e} rm={rel(a[5], b[5]):.2e} "
              f"aggx={rel(a[4][:, :11].cpu(), ax):.2e} cnt={int(a[7].abs().sum())},{int(b[7].abs().sum())}")


main()

"""Diagnostic: one fused GIN layer's backward (dy, dgamma/dbeta, dW, d(agg),
transposed gather) vs fp64 autograd."""
import ctypes
import importlib
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from conftest import load_golden, rel_l2  # noqa: E402

pkg = importlib.import_module("s-cgib_amd")
L_ = pkg._lib
dev = torch.device("cuda", 0)
P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731


def run(gh, d_in, gather, label):
    torch.manual_seed(0)
    n = gh.num_nodes()
    g = gh.to(dev)
    W1, b1 = torch.randn(64, d_in) * 0.3, torch.randn(64) * 0.1
    W2, b2 = torch.randn(64, 64) * 0.2, torch.randn(64) * 0.1
    gam, bet = 1 + 0.3 * torch.randn(64), 0.3 * torch.randn(64)
    h = torch.randn(n, d_in).abs()
    src, dst = gh.edges()
    # fp64 reference of the layer: out = relu(BN(MLP(agg)))
    dd = lambda t: t.double().clone().requires_grad_(True)  # noqa: E731
    W1d, b1d, W2d, b2d, gd_, bd_ = map(dd, (W1, b1, W2, b2, gam, bet))
    agg = h.double() + torch.zeros(n, d_in, dtype=torch.float64).index_add(0, dst, h.double()[src])
    z1 = agg @ W1d.t() + b1d
    r = F.relu(z1)
    z2 = r @ W2d.t() + b2d
    y = F.batch_norm(z2, None, None, gd_, bd_, True, 0.1, 1e-5)
    out = F.relu(y)
    G = torch.randn(n, 64, dtype=torch.float64)  # upstream gradient
    if gather:  # dh = (A^T + I) G  (as if G were the next layer's d(agg))
        dh_ref = G + torch.zeros_like(G).index_add(0, src, G[dst])
    else:
        dh_ref = G
    aggd = agg.detach().requires_grad_(True)
    z1b = aggd @ W1d.t() + b1d
    outb = F.relu(F.batch_norm(F.relu(z1b) @ W2d.t() + b2d, None, None, gd_, bd_, True, 0.1, 1e-5))
    (dh_ref * outb).sum().backward()
    # HIP layer
    f32 = lambda t: t.float().contiguous().to(dev)  # noqa: E731
    hD, W1D, b1D, W2D, b2D, gD, bD = map(f32, (h, W1, b1, W2, b2, gam, bet))
    nt = int(L_.query("scgib_gin_tiles", n))
    ts = torch.empty(nt, 128, device=dev)
    aggD = torch.empty(n, d_in, device=dev); rD = torch.empty(n, 64, device=dev); z2D = torch.empty(n, 64, device=dev)
    L_.call("scgib_gin_layer_fwd", P(hD), d_in, None, P(g.rowptr), P(g.col), n, 1.0, P(W1D), P(b1D), P(W2D), P(b2D), P(aggD), P(rD), P(z2D), P(ts), st())
    stat = torch.empty(4, 64, device=dev)
    L_.call("scgib_bn_finalize", P(ts), n, P(gD), P(bD), 1e-5, 0.1, 1, None, None, None, P(stat), st())
    print(f"[{label}] fwd: agg {rel_l2(aggD.cpu(), agg):.1e} r {rel_l2(rD.cpu(), r.detach()):.1e} z2 {rel_l2(z2D.cpu(), z2.detach()):.1e}")
    Gd = f32(G)
    dy = torch.empty(n, 64, device=dev)
    if gather:
        L_.call("scgib_gin_bwd_stats", P(Gd), P(g.rowptr_t), P(g.col_t), 1.0, P(z2D), P(stat), n, P(dy), P(ts), st())
    else:
        L_.call("scgib_gin_bwd_stats", P(Gd), None, None, 1.0, P(z2D), P(stat), n, P(dy), P(ts), st())
    dy_ref = dh_ref * (y > 0).double()
    bn_g = torch.empty(2, 64, device=dev); coef = torch.empty(2, 64, device=dev)
    L_.call("scgib_bn_bwd_finalize", P(ts), n, 1, P(bn_g[0]), P(bn_g[1]), P(coef), st())
    dagg = torch.empty(n, d_in, device=dev)
    slab = torch.empty(int(L_.query("scgib_gin_slab_floats", n, d_in)), device=dev)
    wg = torch.empty(4096 + 64 * d_in + 128, device=dev)
    L_.call("scgib_gin_layer_bwd", P(dy), P(z2D), P(rD), P(aggD), d_in, P(stat), P(coef), P(W1D), P(W2D), n, P(dagg), P(slab), P(wg), st())
    torch.cuda.synchronize()
    o = 4096
    print(f"[{label}] dy {rel_l2(dy.cpu(), dy_ref):.1e} dgamma {rel_l2(bn_g[0].cpu(), gd_.grad):.1e} dbeta {rel_l2(bn_g[1].cpu(), bd_.grad):.1e} "
          f"dW2 {rel_l2(wg[:o].view(64,64).cpu(), W2d.grad):.1e} dW1 {rel_l2(wg[o:o+64*d_in].view(64,d_in).cpu(), W1d.grad):.1e} "
          f"db2 {rel_l2(wg[o+64*d_in:o+64*d_in+64].cpu(), b2d.grad):.1e} db1 {rel_l2(wg[o+64*d_in+64:].cpu(), b1d.grad):.1e} "
          f"dagg {rel_l2(dagg.cpu(), aggd.grad):.1e}")


gold = load_golden("pretrain_L5_k1_qm9_continue")
ego = pkg.graph.GraphBatch.from_edges(gold["ego_src"], gold["ego_dst"], int(gold["ego_batch_num_nodes"].sum()), True, gold["ego_batch_num_nodes"])
rnd, _ = pkg.graph.collate_pyg(pkg.synth.molecules(13, "qm9", seed=2))
for gh, lab in ((ego, "ego"), (rnd, "rand")):
    for d_in in (32, 64):
        for gather in (False, True):
            run(gh, d_in, gather, f"{lab} d{d_in} gather={gather} n={gh.num_nodes()}")

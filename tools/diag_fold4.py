"""Real fold run (L=1, 200 molecules, train): re-run the layer-0 backward on
the saved forward tensors, PRE kernel vs plain kernel + host dWt."""
import ctypes
import importlib
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
pkg = importlib.import_module("s-cgib_amd")
L = pkg._lib
P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731


def main():
    dev = torch.device("cuda", 0)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    torch.manual_seed(7)
    gh, _ = pkg.graph.collate_pyg(pkg.synth.molecules(200, "qm9", seed=7))
    g = gh.to(dev)
    n = g.num_nodes()
    x = F.normalize(torch.rand(n, 11)).to(dev)
    lin = torch.nn.Linear(11, 32, bias=False).to(dev)
    gin = pkg.models.GIN(32, 64, 1).to(dev).train()
    h = pkg.ops.gin_encoder_x(x, g, gin, lin)
    saved = h.grad_fn.saved_tensors
    agg, r, z2, stat = saved[0:4]
    aggx = saved[-1]
    w1, w2 = saved[4], saved[6]
    gout = torch.randn_like(h)
    # BN-backward stats for layer 0 (as ops does)
    dy = torch.empty(n, 64, device=dev)
    bn_g = torch.empty(2, 64, device=dev)
    coef = torch.empty(2, 64, device=dev)
    ws = torch.empty(int(L.query("scgib_gin_bn_ws_floats", n)), device=dev)
    cnt = torch.zeros(int(L.query("scgib_gin_counters", n)), dtype=torch.int32, device=dev)
    L.call("scgib_gin_bwd_stats_bn", P(gout), None, None, 1.0, P(z2), P(stat), n, 1, P(dy),
           P(bn_g[0]), P(bn_g[1]), P(coef), P(ws), P(cnt), None, st)
    nslab = int(L.query("scgib_gin_bwd_slabs", n))
    wa = 64 * 64 + 64 * 32 + 128
    slab_a = torch.empty(nslab * wa, device=dev)
    dagg = torch.empty(n, 32, device=dev)
    L.call("scgib_gin_layer_bwd", P(dy), P(z2), P(r), P(agg), 32, P(stat), P(coef), P(w1),
           P(w2), n, P(dagg), P(slab_a), None, None, st)
    wb = int(L.query("scgib_gin_layer0_slab_width"))
    slab_b = torch.empty(nslab * wb, device=dev)
    L.call("scgib_gin_layer0_bwd", P(dy), P(z2), P(r), P(agg), P(aggx), P(stat), P(coef),
           P(w1), P(w2), n, P(slab_b), None, st)
    gb = torch.empty(wb, device=dev)
    L.call("scgib_slab_reduce", P(slab_b), nslab, wb, P(gb), st)
    torch.cuda.synchronize()
    dwt_k = gb[wa:].view(32, 16)[:, :11].double().cpu()
    dwt_host = (dagg.double().t() @ aggx.double()).cpu()[:, :11]
    # unfused: dWt = dh0^T x, dh0 = transposed aggregation of dagg
    src, dst = gh.edges()
    dagg64 = dagg.double().cpu()
    dh0 = dagg64.clone().index_add(0, src, dagg64[dst])
    dwt_unf = dh0.t() @ x.double().cpu()
    src_, dst_ = src, dst
    ax = x.double().cpu().clone().index_add(0, dst_, x.double().cpu()[src_])
    rel = lambda a, b: float((a - b).norm() / b.norm())  # noqa: E731
    print(f"n={n} kernel-vs-host(saved aggx)={rel(dwt_k, dwt_host):.2e} "
          f"host(saved aggx)-vs-unfused={rel(dwt_host, dwt_unf):.2e} "
          f"saved aggx vs host aggregate={rel(aggx.double().cpu()[:, :11], ax):.2e} "
          f"dagg rows nan={int(torch.isnan(dagg).sum())}")
    # which rows of aggx differ?
    d = (aggx.double().cpu()[:, :11] - ax).abs().max(dim=1).values
    bad = torch.nonzero(d > 1e-5).flatten().tolist()
    print("aggx rows off:", len(bad), bad[:20])


main()

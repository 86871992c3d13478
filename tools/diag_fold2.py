"""PRE layer-0 backward kernel vs the plain DIN=32 kernel on identical inputs."""
import ctypes
import importlib
import sys

import torch

sys.path.insert(0, ".")
pkg = importlib.import_module("s-cgib_amd")
L = pkg._lib
P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731


def main():
    dev = torch.device("cuda", 0)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for n in (931, 3583, 20000):
        torch.manual_seed(n)
        dy = torch.randn(n, 64, device=dev)
        z2 = torch.randn(n, 64, device=dev)
        r = torch.relu(torch.randn(n, 64, device=dev))
        agg = torch.randn(n, 32, device=dev)
        aggx = torch.randn(n, 16, device=dev)
        aggx[:, 11:] = 0
        stat = torch.randn(4, 64, device=dev)
        coef = torch.randn(2, 64, device=dev) * 0.1
        w1 = torch.randn(64, 32, device=dev)
        w2 = torch.randn(64, 64, device=dev)
        nslab = int(L.query("scgib_gin_bwd_slabs", n))
        wa = 64 * 64 + 64 * 32 + 128
        slab_a = torch.empty(nslab * wa, device=dev)
        dagg = torch.empty(n, 32, device=dev)
        L.call("scgib_gin_layer_bwd", P(dy), P(z2), P(r), P(agg), 32, P(stat), P(coef), P(w1),
               P(w2), n, P(dagg), P(slab_a), None, None, st)
        ga = torch.empty(wa, device=dev)
        L.call("scgib_slab_reduce", P(slab_a), nslab, wa, P(ga), st)
        wb = int(L.query("scgib_gin_layer0_slab_width"))
        slab_b = torch.empty(nslab * wb, device=dev)
        L.call("scgib_gin_layer0_bwd", P(dy), P(z2), P(r), P(agg), P(aggx), 11, P(stat), P(coef),
               P(w1), P(w2), n, P(slab_b), None, st)
        gb = torch.empty(wb, device=dev)
        L.call("scgib_slab_reduce", P(slab_b), nslab, wb, P(gb), st)
        torch.cuda.synchronize()
        same = torch.equal(ga, gb[:wa])
        dwt = gb[wa:].view(32, 16).double().cpu()
        want = (dagg.double().t() @ aggx.double()).cpu()
        e = (dwt - want).norm() / want.norm()
        # per-slab check: which slabs are off?
        sb = slab_b.view(nslab, wb)[:, wa:].view(nslab, 32, 16).double().cpu()
        bad = []
        for t in range(nslab):
            rows = slice(64 * t, min(64 * t + 64, n))
            wt_t = dagg[rows].double().t().cpu() @ aggx[rows].double().cpu()
            et = (sb[t] - wt_t).norm() / max(wt_t.norm(), 1e-30)
            if et > 1e-4:
                bad.append((t, round(float(et), 4)))
        print(f"n={n} slabs={nslab} common grads identical={same} dWt rel={e:.2e} "
              f"bad slabs={bad[:10]} (#{len(bad)})")


main()

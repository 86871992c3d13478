"""Phase stamps of the dense two-layer MLP kernels (debug build) at the molhiv
fine-tune shape: scgib_mlp2_fwd / scgib_mlp2_bwd, Linear(128, 64) - ReLU -
Linear(64, 64) over ~790 rows (Mainmodel_finetuning's MLP, models.py:512).

    make -C s-cgib_amd/csrc trace
    SCGIB_LIB=$PWD/s-cgib_amd/libscgib_trace.so python tools/mlp_trace.py
"""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("s-cgib_amd")
ops, _lib = pkg.ops, pkg._lib

FWD = ["-", "load", "gemm1", "gemm2+st"]
BWD = ["-", "dz2", "dW2,dr,dz1", "dW1,dx", "slab"]


def summary(buf, nblk, marks, names):
    t = buf[:nblk * 32].reshape(nblk, 32)[:, :16].astype(np.float64) / 100.0  # us (100 MHz)
    ok = t[:, marks[0]] != 0
    t = t[ok]
    t0 = t[:, marks[0]].min()
    print(f"  workgroups {len(t)}: start spread {t[:, marks[0]].max() - t0:.2f} us, "
          f"end {max(t[:, m].max() for m in marks) - t0:.2f} us after the first start")
    for a, b, name in zip(marks[:-1], marks[1:], names[1:]):
        d = t[:, b] - t[:, a]
        d = d[t[:, b] != 0]
        if len(d):
            print(f"    {name:12s} p50 {np.median(d):7.2f}  max {d.max():7.2f} us")


def main():
    lib = _lib.load()
    lib.scgib_trace_set.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    n, d_in, H = 790, 128, 64
    f = dict(device=dev, dtype=torch.float32)
    x = torch.randn(n, d_in, **f)
    w1, b1 = torch.randn(H, d_in, **f) * 0.1, torch.randn(H, **f)
    w2, b2 = torch.randn(H, H, **f) * 0.1, torch.randn(H, **f)
    r, out, g = torch.empty(n, H, **f), torch.empty(n, H, **f), torch.randn(n, H, **f)
    dx = torch.empty(n, d_in, **f)
    slab = torch.empty(int(_lib.query("scgib_mlp2_slab_floats", n, d_in)), **f)
    wg = torch.empty(H * H + H * d_in + 2 * H, **f)
    buf = torch.zeros(4096 * 32, dtype=torch.int64, device=dev)
    assert lib.scgib_trace_set(ctypes.c_void_p(buf.data_ptr())) == 0
    p = ops._p

    def fwd():
        _lib.call("scgib_mlp2_fwd", p(x), d_in, n, p(w1), p(b1), p(w2), p(b2), p(r), p(out),
                  None, ops._stream())

    def bwd():
        _lib.call("scgib_mlp2_bwd", p(g), p(x), p(r), d_in, p(w1), p(w2), n, p(dx), p(slab),
                  None, None, ops._stream())
    for _ in range(3):
        fwd()
        bwd()
    torch.cuda.synchronize()
    nt = (n + 63) // 64
    for it in range(3):
        buf.zero_()
        fwd()
        torch.cuda.synchronize()
        print(f"forward (iteration {it})")
        summary(buf.cpu().numpy(), nt, [0, 1, 2, 3], FWD)
        buf.zero_()
        bwd()
        torch.cuda.synchronize()
        print(f"backward (iteration {it})")
        summary(buf.cpu().numpy(), 256, [0, 1, 2, 3, 4], BWD)  # (2 per tile when split)


if __name__ == "__main__":
    main()

"""Phase stamps of the fine-tune head kernels (debug build): scgib_head_fwd /
scgib_head_bwd at the molhiv fine-tune shape (B = 32 graphs, K = 128 Set2Set
outputs, one sigmoid class).

    make -C s-cgib_amd/csrc trace
    SCGIB_LIB=$PWD/s-cgib_amd/libscgib_trace.so python tools/head_trace.py
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

FWD = ["-", "load+stage", "hidden", "out"]
BWD = ["-", "weights", "chunk stage", "dW2+dh", "dh store", "dW1+db1", "dx", "writes"]


def summary(buf, nblk, marks, names):
    t = buf[:nblk * 32].reshape(nblk, 32)[:, :16].astype(np.float64) / 100.0  # us (100 MHz)
    t0 = t[:, marks[0]].min()
    print(f"  workgroups {nblk}: start spread {t[:, marks[0]].max() - t0:.2f} us, "
          f"end {t[:, marks[-1]].max() - t0:.2f} us after the first start")
    for a, b, name in zip(marks[:-1], marks[1:], names[1:]):
        d = t[:, b] - t[:, a]
        print(f"    {name:12s} p50 {np.median(d):7.2f}  max {d.max():7.2f} us")


def main():
    lib = _lib.load()
    lib.scgib_trace_set.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    B, K, C, H = 32, 128, 1, 64
    f = dict(device=dev, dtype=torch.float32)
    x, w1, b1 = torch.randn(B, K, **f), torch.randn(H, K, **f) * 0.1, torch.randn(H, **f)
    w2, b2 = torch.randn(C, H, **f) * 0.1, torch.randn(C, **f)
    hid, out = torch.empty(B, H, **f), torch.empty(B, C, **f)
    d_out = torch.randn(B, C, **f)
    dx, dw1, db1 = torch.empty(B, K, **f), torch.empty(H, K, **f), torch.empty(H, **f)
    dw2, db2 = torch.empty(C, H, **f), torch.empty(C, **f)
    buf = torch.zeros(4096 * 32, dtype=torch.int64, device=dev)
    assert lib.scgib_trace_set(ctypes.c_void_p(buf.data_ptr())) == 0
    p = ops._p

    def fwd():
        _lib.call("scgib_head_fwd", p(x), B, K, p(w1), p(b1), p(w2), p(b2), C, 1, p(hid), p(out),
                  None, ops._stream())

    def bwd():
        _lib.call("scgib_head_bwd", p(x), p(hid), p(out), p(d_out), B, K, p(w1), p(w2), C, 1,
                  p(dx), p(dw1), p(db1), p(dw2), p(db2), ops._stream())
    for _ in range(3):
        fwd()
        bwd()
    torch.cuda.synchronize()
    for it in range(3):
        buf.zero_()
        fwd()
        torch.cuda.synchronize()
        print(f"forward (iteration {it})")
        summary(buf.cpu().numpy(), (B + 15) // 16, [0, 1, 2, 3], FWD)
        buf.zero_()
        bwd()
        torch.cuda.synchronize()
        print(f"backward (iteration {it})")
        summary(buf.cpu().numpy(), 4, [0, 1, 2, 3, 4, 5, 6, 7], BWD)


if __name__ == "__main__":
    main()

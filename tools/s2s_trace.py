"""Phase stamps of the Set2Set kernels (debug build): one forward + backward
of models.Set2Set(64, 2, 1) over a molhiv-like batch of 32 molecules.

    make -C s-cgib_amd/csrc trace
    SCGIB_LIB=$PWD/s-cgib_amd/libscgib_trace.so python tools/s2s_trace.py
"""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("s-cgib_amd")

FWD = ["prologue", "stage+bias", "r0 gates", "r0 cell", "r0 attention", "r1 + out"]
BWD = ["-", "stage", "r1 h", "r1 attention", "r1 cell", "r1 products", "r1 comb + r0 h",
       "r0 attention", "r0 cell", "r0 dG out", "dx out"]
# (round 0 leaves the loop before its products: mark 10 is never written)
BWD_MARKS = [0, 1, 2, 3, 4, 5, 7, 8, 9, 12, 13]


def summary(buf, nblk, marks, names):
    t = buf[:nblk * 32].reshape(nblk, 32)[:, :16].astype(np.float64) / 100.0  # us (100 MHz)
    t0 = t[:, marks[0]].min()
    print(f"  workgroups {nblk}: start spread {t[:, marks[0]].max() - t0:.2f} us, "
          f"end {t[:, marks[-1]].max() - t0:.2f} us after the first start")
    for a, b, name in zip(marks[:-1], marks[1:], names[1:]):
        d = t[:, b] - t[:, a]
        print(f"    {name:14s} p50 {np.median(d):7.2f}  max {d.max():7.2f} us")


def main():
    lib = pkg._lib.load()
    lib.scgib_trace_set.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    gh, _ = pkg.graph.collate_pyg(pkg.synth.molecules(32, "molhiv", seed=3))
    g = gh.to(dev)
    torch.manual_seed(0)
    s2s = pkg.models.Set2Set(64, 2, 1).to(dev)
    feat = torch.randn(g.num_nodes(), 64, device=dev, requires_grad=True)
    buf = torch.zeros(4096 * 32, dtype=torch.int64, device=dev)
    assert lib.scgib_trace_set(ctypes.c_void_p(buf.data_ptr())) == 0
    for _ in range(3):  # warm
        out = s2s(g, feat)
        out.sum().backward()
    torch.cuda.synchronize()
    for it in range(3):
        buf.zero_()
        out = s2s(g, feat)
        torch.cuda.synchronize()
        print(f"forward (iteration {it})")
        summary(buf.cpu().numpy(), 32, [0, 1, 2, 3, 4, 5], ["-"] + FWD[1:])
        buf.zero_()
        out.sum().backward()
        torch.cuda.synchronize()
        print(f"backward (iteration {it})")
        summary(buf.cpu().numpy(), 32, BWD_MARKS, BWD)


if __name__ == "__main__":
    main()

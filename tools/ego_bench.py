"""Time the ego-net builders (k = 1: two-launch window builder vs the general
three-launch bitmap builder) on a bench batch: python tools/ego_bench.py"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("s-cgib_amd")

dev = torch.device("cuda", 0)
for wl, b in (("qm9", 512), ("molpcba", 1024)):
    gh, _ = pkg.graph.collate_pyg(pkg.synth.molecules(b, wl, seed=0))
    g = gh.to(dev)
    for fast in (True, False):
        pkg.graph.EGO_K1_FAST = fast
        for _ in range(3):
            pkg.graph.egonet_batch(g, 1)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(100):
            pkg.graph.egonet_batch(g, 1)
        e.record()
        torch.cuda.synchronize()
        print(wl, "k1" if fast else "bitmap", f"{s.elapsed_time(e) * 10:.1f} us/build")

"""Diagnostic (GPU): exact mode vs capacity-mode graph replay of the pretrain
step (test_gpu_capacity's replay test body), per-tensor gradient rel-L2, with
ops.AGG_FREE on and off.  Usage: python tools/aggfree_probe.py"""
import copy
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import test_gpu_capacity as T  # noqa: E402
from conftest import rel_l2  # noqa: E402
import importlib  # noqa: E402

pkg = importlib.import_module("s-cgib_amd")
dev = torch.device("cuda", 0)
k = 1
for free in (True, False):
    pkg.ops.AGG_FREE = free
    hosts = T._batches(pkg, (4, 5, 6, 7))
    n_cap, e_cap, mgn, caps = pkg.graph.StaticBatch.capacities(hosts, k, slack=1.02)
    static = pkg.graph.StaticBatch(T.B, n_cap, e_cap, T.F_IN, mgn, caps, dev, k=k)
    padded = [static.pad(gh) for gh in hosts]
    exact_m = T._model(pkg, dev, k=k)
    cap_m = copy.deepcopy(exact_m)
    for i in (0, 1):
        gh = hosts[i]
        n = gh.num_nodes()
        ug, uf = T._noise(n_cap, dev, 200 + i)
        g = gh.to(dev)
        le = T._step(exact_m, g, g.ndata["x"], (ug[:n], uf[:n]), dev, k)
        static.load(padded[i])
        lc = T._step(cap_m, static.graph, static.x, (ug, uf), dev, k)
        torch.cuda.synchronize()
        ge = {kk: p.grad for kk, p in exact_m.named_parameters() if p.grad is not None}
        gc = {kk: p.grad for kk, p in cap_m.named_parameters() if p.grad is not None}
        errs = sorted(((rel_l2(gc[kk].cpu(), ge[kk].cpu()), kk) for kk in ge), reverse=True)
        print(f"AGG_FREE={free} batch {i}: losses {le.tolist()} vs {lc.tolist()}")
        for e, kk in errs[:6]:
            print(f"   {e:.3e} {kk}")

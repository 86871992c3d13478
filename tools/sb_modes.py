"""bench.py's superbatch roofline with the forward layer's walking form off
(0), at its default threshold (1) and forced (2): python tools/sb_modes.py [modes]"""
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("s-cgib_amd")
import bench  # noqa: E402

dev = torch.device("cuda", 0)
lib = pkg._lib.load()
for mode in [int(m) for m in (sys.argv[1:] or ["0", "1"])]:
    lib.scgib_set_fwd_walk(mode)
    sb = bench.superbatch_roofline(dev)
    print(f"walk={mode}", {k: {kk: sb[k].get(kk) for kk in ("us", "frac", "frac_inclusive")}
                           for k in ("gin_fwd_k", "gin_bwd_stats_k", "gin_bwd5_k")}, flush=True)

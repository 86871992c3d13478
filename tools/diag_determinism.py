"""Run the same pretrain step twice (deep copies, same noise) and report which
parameter gradients differ bitwise: python tools/diag_determinism.py"""
import copy
import importlib
import os
import sys
from types import SimpleNamespace

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("s-cgib_amd")

dev = torch.device("cuda", 0)
mols = pkg.synth.molecules(64, "qm9", seed=9)
gh, _ = pkg.graph.collate_pyg(mols)
g = gh.to(dev)
x = F.normalize(g.ndata["x"].float())
args = SimpleNamespace(recons_type="adj", useAtt=1, readout_f="sum", d_transfer=32,
                       batch_size=64, gin_layers=5)
torch.manual_seed(3)
base = pkg.models.Mainmodel(args, 11, 64, 4, 4, 1, "GIN").to(dev).train()
n = g.num_nodes()
noise = (torch.rand(n, device=dev), torch.rand(n, 64, device=dev))
for mode in sys.argv[1:] or ["default"]:
    res = []
    for rep in range(3):
        m = copy.deepcopy(base)
        _, kl, con, rec = m(g, x, None, None, None, 1, None, 1, dev, 64,
                            noise=(noise[0].clone(), noise[1].clone()))
        (kl + con + rec).backward()
        torch.cuda.synchronize()
        res.append({k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None})
    for k in res[0]:
        d = max(float((res[0][k] - r[k]).abs().max()) for r in res[1:])
        if d:
            print(mode, k, d)
    print(mode, "done")

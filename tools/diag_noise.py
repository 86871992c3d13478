"""Device noise vs the same draws replayed explicitly: which gradients differ.
python tools/diag_noise.py"""
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
gh, _ = pkg.graph.collate_pyg(pkg.synth.molecules(64, "qm9", seed=9))
g = gh.to(dev)
x = F.normalize(g.ndata["x"].float())
args = SimpleNamespace(recons_type="adj", useAtt=1, readout_f="sum", d_transfer=32,
                       batch_size=64, gin_layers=5)
torch.manual_seed(3)
base = pkg.models.Mainmodel(args, 11, 64, 4, 4, 1, "GIN").to(dev).train()


def run(noise):
    m = copy.deepcopy(base)
    if noise is None:
        pkg.ops.seed_noise(dev, 1234)
    _, kl, con, rec = m(g, x, None, None, None, 1, None, 1, dev, 64, noise=noise)
    (kl + con + rec).backward()
    torch.cuda.synchronize()
    return m, {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}


m1, g1 = run(None)
ug, uf = m1._last_noise
m1b, g1b = run(None)
print("device twice, noise equal:", torch.equal(m1b._last_noise[1], uf))
for k in g1:
    d = float((g1[k] - g1b[k]).abs().max())
    if d:
        print("device-vs-device", k, d)
m2, g2 = run((ug.clone(), uf.clone()))
for k in g1:
    d = float((g1[k] - g2[k]).abs().max())
    if d:
        print("device-vs-explicit", k, d, float(g1[k].abs().max()))
print("done")

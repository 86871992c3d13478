"""Seed sweep: fold and unfused dWt error vs fp64 (train, L=1/5, 200 mols)
plus the number of output-ReLU sign flips of each fp32 path vs fp64."""
import copy
import importlib
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
pkg = importlib.import_module("s-cgib_amd")
from oracle import scgib_ref as R  # noqa: E402


def one(seed, L):
    dev = torch.device("cuda", 0)
    torch.manual_seed(seed)
    gh, _ = pkg.graph.collate_pyg(pkg.synth.molecules(200, "qm9", seed=seed))
    g = gh.to(dev)
    x = F.normalize(torch.rand(g.num_nodes(), 11)).to(dev)
    lin = torch.nn.Linear(11, 32, bias=False).to(dev)
    gin = pkg.models.GIN(32, 64, L).to(dev).train()
    gin_b, lin_b = copy.deepcopy(gin), copy.deepcopy(lin)
    p64 = {("E." + k): (v.detach().cpu().double() if v.is_floating_point() else v.detach().cpu())
           for k, v in gin.state_dict().items()}
    wt64 = lin.weight.detach().cpu().double().clone().requires_grad_(True)
    src, dst = gh.edges()
    h64 = R.gin_encoder(p64, "E", src, dst, x.cpu().double() @ wt64.t(),
                        {k: v.clone() for k, v in p64.items()}, L)
    h = pkg.ops.gin_encoder_x(x, g, gin, lin)
    hb = gin_b(g, lin_b(x))
    w = torch.randn_like(h)
    (h * w).sum().backward()
    (hb * w).sum().backward()
    (h64 * w.cpu().double()).sum().backward()
    rel = lambda a: float((a.cpu().double() - wt64.grad).norm() / wt64.grad.norm())  # noqa: E731
    fl_a = int(((h.detach().cpu() > 0) != (h64.detach() > 0)).sum())
    fl_b = int(((hb.detach().cpu() > 0) != (h64.detach() > 0)).sum())
    print(f"seed={seed} L={L} fold={rel(lin.weight.grad):.2e} (out flips {fl_a})  "
          f"unfused={rel(lin_b.weight.grad):.2e} (out flips {fl_b})")


for L in (1, 5):
    for seed in range(1, 9):
        one(seed, L)

"""Localise the transfer_d-fold dWt error: fold vs fp64 over layers / sizes."""
import copy
import importlib
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
pkg = importlib.import_module("s-cgib_amd")
from oracle import scgib_ref as R  # noqa: E402


def run(n_mols, L, training, seed=7):
    dev = torch.device("cuda", 0)
    torch.manual_seed(seed)
    gh, _ = pkg.graph.collate_pyg(pkg.synth.molecules(n_mols, "qm9", seed=seed))
    g = gh.to(dev)
    x = F.normalize(torch.rand(g.num_nodes(), 11)).to(dev)
    lin = torch.nn.Linear(11, 32, bias=False).to(dev)
    gin = pkg.models.GIN(32, 64, L).to(dev).train(training)
    p64 = {("E." + k): (v.detach().cpu().double() if v.is_floating_point() else v.detach().cpu())
           for k, v in gin.state_dict().items()}
    wt64 = lin.weight.detach().cpu().double().clone().requires_grad_(True)
    src, dst = gh.edges()
    h0 = x.cpu().double() @ wt64.t()
    if training:
        h64 = R.gin_encoder(p64, "E", src, dst, h0, {k: v.clone() for k, v in p64.items()}, L)
    else:
        orig = R._batchnorm_train
        R._batchnorm_train = lambda xx, pp, name, buf: F.batch_norm(
            xx, pp[name + ".running_mean"], pp[name + ".running_var"], pp[name + ".weight"],
            pp[name + ".bias"], False, 0.1, 1e-5)
        h64 = R.gin_encoder(p64, "E", src, dst, h0, None, L)
        R._batchnorm_train = orig
    h = pkg.ops.gin_encoder_x(x, g, gin, lin)
    w = torch.randn_like(h)
    (h * w).sum().backward()
    (h64 * w.cpu().double()).sum().backward()
    e = (lin.weight.grad.cpu().double() - wt64.grad).norm() / wt64.grad.norm()
    col = ((lin.weight.grad.cpu().double() - wt64.grad).norm(dim=0) / wt64.grad.norm(dim=0))
    torch.cuda.synchronize()
    pool = pkg.ops._COUNTERS.get(0)
    nz = [] if pool is None else torch.nonzero(pool).flatten().tolist()
    ranges = {k: v for k, v in pkg.ops._COUNTER_RANGES.items()}
    bad = [(k[1][0], off, size) for k, (off, size) in ranges.items()
           if any(off <= i < off + size for i in nz)]
    print(f"mols={n_mols:4d} N={g.num_nodes():6d} tiles={(g.num_nodes()+63)//64:4d} L={L} "
          f"train={int(training)} dWt rel={e:.2e}  worst col={col.max():.2e} "
          f"nonzero counters={len(nz)} in {bad[:4]}")


for L in (1, 2):
    for training in (True, False):
        for n in (3, 4, 8, 16, 50, 200):
            run(n, L, training)

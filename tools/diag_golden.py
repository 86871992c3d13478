"""Diagnostic: GPU gradients (fused and layer-by-layer GIN) vs an fp64 oracle
evaluation of a golden pretrain step."""
import importlib
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from conftest import CANCELLED, load_golden, rel_l2  # noqa: E402
from oracle import scgib_ref as R  # noqa: E402
from test_gpu_parity import build_model_from_golden  # noqa: E402
from test_oracle_golden import golden_inputs  # noqa: E402

pkg = importlib.import_module("s-cgib_amd")
dev = torch.device("cuda", 0)
name = sys.argv[1] if len(sys.argv) > 1 else "pretrain_L5_k1_qm9_continue"
g = load_golden(name)
batch, ego, x, xs = golden_inputs(g)
raw = {k[6:]: v for k, v in g.items() if k.startswith("param_")}
p = {}
for k, v in R.strip_continue(raw).items():
    t = torch.tensor(v)
    if t.is_floating_point():
        t = t.double()
        if "running" not in k and not k.endswith(".eps"):
            t.requires_grad_(True)
    p[k] = t
bufs = {k: v.clone() for k, v in p.items() if "running" in k or "num_batches" in k}
out = R.pretrain_forward(p, batch, ego, x.double(), xs.double(), torch.tensor(g["u_gate"]).double(),
                         torch.tensor(g["u_feat"]).double(), int(g["chunk"]), bufs)
out["loss_total"].backward()
truth = {k: v.grad.numpy() for k, v in p.items() if v.grad is not None}

for fused in (True, False):
    model = build_model_from_golden(pkg, g, dev)
    for m in model.modules():
        if isinstance(m, pkg.models.GIN):
            m.fused = fused
    bg = pkg.graph.GraphBatch.from_edges(g["src"], g["dst"], len(g["x_raw"]), True,
                                         g["batch_num_nodes"]).to(dev)
    xd = F.normalize(torch.tensor(g["x_raw"]).float()).to(dev)
    noise = (torch.tensor(g["u_gate"], device=dev), torch.tensor(g["u_feat"], device=dev))
    _, kl, con, rec = model.forward(bg, xd, None, None, None, 1, None, 2, dev, int(g["chunk"]), noise=noise)
    (kl + con + rec).backward()
    print(f"fused={fused} losses vs fp64: kl {abs(kl.item()-out['loss_kl'].item())/out['loss_kl'].item():.2e} "
          f"con {abs(con.item()-out['loss_contrastive'].item())/out['loss_contrastive'].item():.2e} "
          f"rec {abs(rec.item()-out['loss_recon'].item())/out['loss_recon'].item():.2e}")
    errs = []
    for n_, prm in model.named_parameters():
        if prm.grad is None:
            continue
        k = R.strip_continue({n_: 0}).popitem()[0]
        if k not in truth or k.endswith(CANCELLED) or k.endswith("attn_layer.weight"):
            continue
        gk = "grad_" + n_
        e_gpu = rel_l2(prm.grad.cpu().numpy(), truth[k])
        e_gold = rel_l2(g[gk], truth[k]) if gk in g else float("nan")
        errs.append((e_gpu, e_gold, k))
    errs.sort(reverse=True)
    for e in errs[:8]:
        print(f"   gpu {e[0]:.2e}  golden {e[1]:.2e}  {e[2]}")

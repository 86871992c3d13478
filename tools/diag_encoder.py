"""Diagnostic: fused GIN encoder on a golden's Encoder2 input vs fp64."""
import importlib
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from conftest import load_golden, rel_l2  # noqa: E402
from oracle import scgib_ref as R  # noqa: E402

pkg = importlib.import_module("s-cgib_amd")
dev = torch.device("cuda", 0)
g = load_golden(sys.argv[1] if len(sys.argv) > 1 else "pretrain_L5_k1_qm9_continue")
enc = sys.argv[2] if len(sys.argv) > 2 else "Encoder2"
raw = R.strip_continue({k[6:]: v for k, v in g.items() if k.startswith("param_")})
L = int(g["L"])
x_raw = torch.tensor(g["x_raw"]).float()
if enc == "Encoder2":
    xs = F.normalize(x_raw[torch.tensor(g["ego_nodes_global"])])
    src, dst, counts = g["ego_src"], g["ego_dst"], g["ego_batch_num_nodes"]
else:
    xs = F.normalize(x_raw)
    src, dst, counts = g["src"], g["dst"], g["batch_num_nodes"]
h0 = xs @ torch.tensor(raw["transfer_d.weight"]).t()
n = h0.shape[0]
gh = pkg.graph.GraphBatch.from_edges(src, dst, n, True, counts)
gd = gh.to(dev)
gin = pkg.models.GIN(32, 64, L)
sd = {k[len(enc) + 1:]: torch.tensor(v) for k, v in raw.items() if k.startswith(enc + ".")}
print(gin.load_state_dict(sd, strict=False))
p64 = {enc + "." + k: (v.double() if v.is_floating_point() else v).clone().requires_grad_(
    v.is_floating_point() and "running" not in k and not k.endswith(".eps")) for k, v in sd.items()}
bufs = {k: v for k, v in p64.items() if "running" in k or "num_batches" in k}
h64 = h0.double().requires_grad_(True)
ref = R.gin_encoder(p64, enc, torch.tensor(src), torch.tensor(dst), h64, bufs, L)
torch.manual_seed(0)
w = torch.randn(n, 64, dtype=torch.float64)
(w * ref).sum().backward()
for fused in (True, False):
    m = pkg.models.GIN(32, 64, L)
    m.load_state_dict(sd, strict=False)
    m = m.to(dev).train()
    m.fused = fused
    hd = h0.to(dev).requires_grad_(True)
    out = m(gd, hd)
    (w.float().to(dev) * out).sum().backward()
    print(f"fused={fused}: out err {rel_l2(out.detach().cpu(), ref.detach()):.2e} "
          f"dh0 err {rel_l2(hd.grad.cpu(), h64.grad):.2e}")
    for nme, prm in m.named_parameters():
        e = rel_l2(prm.grad.cpu(), p64[enc + "." + nme].grad)
        if e > 1e-4 and not nme.endswith("mlp.2.bias"):
            print(f"    {nme}: {e:.2e}")

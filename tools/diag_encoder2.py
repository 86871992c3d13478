"""Which factor breaks the fused multi-layer backward: graph, input, params?"""
import importlib
import itertools
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from conftest import load_golden, rel_l2  # noqa: E402
from oracle import scgib_ref as R  # noqa: E402

pkg = importlib.import_module("s-cgib_amd")
dev = torch.device("cuda", 0)
g = load_golden("pretrain_L5_k1_qm9_continue")
raw = R.strip_continue({k[6:]: v for k, v in g.items() if k.startswith("param_")})
enc = "Encoder2"
sd_gold = {k[len(enc) + 1:]: torch.tensor(v) for k, v in raw.items() if k.startswith(enc + ".")}
x_raw = torch.tensor(g["x_raw"]).float()
h0_gold = F.normalize(x_raw[torch.tensor(g["ego_nodes_global"])]) @ torch.tensor(raw["transfer_d.weight"]).t()
ego = pkg.graph.GraphBatch.from_edges(g["ego_src"], g["ego_dst"], len(h0_gold), True, g["ego_batch_num_nodes"])
rnd, _ = pkg.graph.collate_pyg(pkg.synth.molecules(13, "qm9", seed=2))
torch.manual_seed(5)
sd_rand = pkg.models.GIN(32, 64, 5).state_dict()
for gname, hname, pname in itertools.product(("ego", "rand"), ("gold", "randn"), ("gold", "rand")):
    gh = ego if gname == "ego" else rnd
    n = gh.num_nodes()
    if hname == "gold":
        h0 = h0_gold[:n] if n <= len(h0_gold) else torch.cat([h0_gold, h0_gold])[:n]
    else:
        h0 = torch.randn(n, 32)
    sd = sd_gold if pname == "gold" else sd_rand
    for L in (2, 5):
        sdl = {k: v for k, v in sd.items() if not any(f"s.{i}." in k for i in range(L, 5))}
        p64 = {enc + "." + k: (v.double() if v.is_floating_point() else v).clone().requires_grad_(
            v.is_floating_point() and "running" not in k and not k.endswith(".eps")) for k, v in sdl.items()}
        bufs = {k: v for k, v in p64.items() if "running" in k or "num_batches" in k}
        h64 = h0.double().requires_grad_(True)
        src, dst = gh.edges()
        ref = R.gin_encoder(p64, enc, src, dst, h64, bufs, L)
        w = torch.randn(n, 64, dtype=torch.float64)
        (w * ref).sum().backward()
        m = pkg.models.GIN(32, 64, L)
        m.load_state_dict(sdl)
        m = m.to(dev).train()
        hd = h0.to(dev).requires_grad_(True)
        out = m(gh.to(dev), hd)
        (w.float().to(dev) * out).sum().backward()
        worst = max((rel_l2(prm.grad.cpu(), p64[enc + "." + nme].grad), nme) for nme, prm in m.named_parameters()
                    if not nme.endswith("mlp.2.bias"))
        print(f"graph={gname:4s} h0={hname:5s} params={pname:4s} L={L}: out {rel_l2(out.detach().cpu(), ref.detach()):.1e} "
              f"dh0 {rel_l2(hd.grad.cpu(), h64.grad):.1e} worst {worst[0]:.1e} {worst[1]}", flush=True)

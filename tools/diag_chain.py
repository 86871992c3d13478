"""2-layer fused chain, every intermediate vs fp64 (golden ego case)."""
import ctypes
import importlib
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from conftest import load_golden, rel_l2  # noqa: E402
from oracle import scgib_ref as R  # noqa: E402

pkg = importlib.import_module("s-cgib_amd")
L_ = pkg._lib
dev = torch.device("cuda", 0)
P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
g = load_golden("pretrain_L5_k1_qm9_continue")
raw = R.strip_continue({k[6:]: v for k, v in g.items() if k.startswith("param_")})
T = lambda k: torch.tensor(raw["Encoder2." + k])  # noqa: E731
x_raw = torch.tensor(g["x_raw"]).float()
h0 = F.normalize(x_raw[torch.tensor(g["ego_nodes_global"])]) @ torch.tensor(raw["transfer_d.weight"]).t()
gh = pkg.graph.GraphBatch.from_edges(g["ego_src"], g["ego_dst"], len(h0), True, g["ego_batch_num_nodes"])
gd = gh.to(dev)
n = len(h0)
src, dst = gh.edges()
lay = []
for l in range(2):
    pre = f"ginlayers.{l}.apply_func.mlp."
    lay.append([T(pre + "0.weight"), T(pre + "0.bias"), T(pre + "2.weight"), T(pre + "2.bias"),
                T(f"batch_norms.{l}.weight"), T(f"batch_norms.{l}.bias")])
# fp64 chain with retained intermediates
h = h0.double().requires_grad_(True)
ref = {}
x = h
for l in range(2):
    W1, b1, W2, b2, ga, be = (t.double() for t in lay[l])
    agg = x + torch.zeros_like(x).index_add(0, dst, x[src])
    agg.retain_grad()
    z1 = agg @ W1.t() + b1
    r = F.relu(z1)
    z2 = r @ W2.t() + b2
    z2.retain_grad()
    y = F.batch_norm(z2, None, None, ga, be, True, 0.1, 1e-5)
    x = F.relu(y)
    ref[l] = dict(agg=agg, z1=z1, r=r, z2=z2, y=y)
torch.manual_seed(0)
w = torch.randn(n, 64, dtype=torch.float64)
(w * x).sum().backward()
# fused chain
f32 = lambda t: t.float().contiguous().to(dev)  # noqa: E731
nt = int(L_.query("scgib_gin_tiles", n))
ts = torch.empty(nt, 128, device=dev)
hin, stat_prev, sv = f32(h0), None, []
for l in range(2):
    W1, b1, W2, b2, ga, be = map(f32, lay[l])
    d_in = hin.shape[1]
    agg = torch.empty(n, d_in, device=dev); r = torch.empty(n, 64, device=dev); z2 = torch.empty(n, 64, device=dev)
    L_.call("scgib_gin_layer_fwd", P(hin), d_in, P(stat_prev), P(gd.rowptr), P(gd.col), n, 1.0, P(W1), P(b1), P(W2), P(b2), P(agg), P(r), P(z2), P(ts), st())
    stat = torch.empty(4, 64, device=dev)
    L_.call("scgib_bn_finalize", P(ts), n, P(ga), P(be), 1e-5, 0.1, 1, None, None, None, P(stat), st())
    sv.append((agg, r, z2, stat))
    rr = ref[l]
    y32 = stat[2].cpu() * z2.cpu() + stat[3].cpu()
    print(f"L{l} fwd: agg {rel_l2(agg.cpu(), rr['agg'].detach()):.1e} r {rel_l2(r.cpu(), rr['r'].detach()):.1e} "
          f"z2 {rel_l2(z2.cpu(), rr['z2'].detach()):.1e} mean {rel_l2(stat[0].cpu(), rr['z2'].detach().mean(0)):.1e} "
          f"r-mask flips {int(((r.cpu() > 0) != (rr['r'] > 0)).sum())} y-mask flips {int(((y32 > 0) != (rr['y'] > 0)).sum())} "
          f"|y|<1e-5: {int((rr['y'].abs() < 1e-5).sum())} |z1|<1e-5: {int((rr['z1'].abs() < 1e-5).sum())}")
    hin, stat_prev = z2, stat
print("min |y| per layer:", [float(ref[l]['y'].abs().min()) for l in range(2)],
      "min |z1|:", [float(ref[l]['z1'].abs().min()) for l in range(2)])

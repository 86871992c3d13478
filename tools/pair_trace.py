"""Phase timeline of the persistent encoder-pair kernels (gin_pair.hip) on
one bench batch: every workgroup's wall-clock stamps (100 MHz) through
ops.PAIR_TRACE, summarised per layer.  python tools/pair_trace.py [workload batch k]

forward stamps per layer l (slot 8 l + i): 0 start, 1 aggregation done,
2 GEMM1 + r stored, 3 z2 stored (exchange entered), 4 group arrival counted,
5 group partial stored (group's last chunk), 6 every group partial seen,
7 (scale, shift) in LDS.  backward: 0 start, 1 sums stored, 2 group arrival,
3 group partial, 4 every group seen, 5 coefficients in LDS, 6 dW2 / dz1 done.  56 start, 57 chunk loaded, 58 layer-0 gather, 60 exit."""
import importlib
import os
import statistics
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("s-cgib_amd")
import bench  # noqa: E402

wl, B, k = (sys.argv[1], int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else ("qm9", 512, 1)
dev = torch.device("cuda", 0)
torch.manual_seed(0)
F_in = pkg.synth.WORKLOADS[wl][2]
gh, _ = pkg.graph.collate_pyg(pkg.synth.molecules(B, wl, seed=0))
g = gh.to(dev)
dict.__setitem__(g.ndata, "x", F.normalize(g.ndata["x"].float()))
model = bench.make_model(F_in, k, 5, dev)
pkg.ops.PAIR_PERSISTENT = True
pkg.models.FORK_ENCODERS = False


def step():
    model.zero_grad(set_to_none=True)
    _, kl, con, rec = model(g, g.ndata["x"], None, None, None, 1, None, k, dev, B)
    (kl + rec + con).backward()


for _ in range(3):
    step()
torch.cuda.synchronize()
tr = [torch.zeros(1024 * 64, dtype=torch.int64, device=dev) for _ in range(2)]
pkg.ops.PAIR_TRACE = tr
step()
torch.cuda.synchronize()
pkg.ops.PAIR_TRACE = None
assert pkg.ops.pair_sync_error(dev) == 0


def summary(name, t, names, layers):
    t = t.view(1024, 64).cpu()
    live = t[:, 56] > 0
    t = t[live].double()
    t0 = t[:, 56].min()
    us = lambda x: (x - t0) / 100.0  # noqa: E731  (wall clock: 10 ns ticks)
    print(f"{name}: {int(live.sum())} workgroups, start spread {float(us(t[:, 56]).max()):.2f} us, "
          f"exit median {float(us(t[:, 60]).median()):.2f} max {float(us(t[:, 60]).max()):.2f} us")
    for l in layers:
        row = []
        for i, nm in enumerate(names):
            col = t[:, 8 * l + i]
            col = col[col > 0]
            if len(col):
                v = us(col)
                row.append(f"{nm} {float(v.median()):7.2f}/{float(v.max()):7.2f}")
        print(f"  layer {l}: " + " | ".join(row))


def slowest(t, l, i0, i1, k=8):
    t = t.view(1024, 64).cpu()
    t = t[t[:, 56] > 0]
    d = (t[:, 8 * l + i1] - t[:, 8 * l + i0]).double() / 100.0
    order = torch.argsort(d, descending=True)[:k]
    info = t[:, 61]
    print(f"  slowest phase {i0}->{i1} of layer {l}: " + ", ".join(
        f"{float(d[j]):.1f}us(enc{int(info[j]) >> 31 & 1} nr{int(info[j]) & 255} "
        f"ne{int(info[j]) >> 8 & 0x3fffff} lds{int(info[j]) >> 30 & 1})" for j in order))
    print(f"  phase {i0}->{i1} median {float(d.median()):.2f} p90 {float(d.quantile(0.9)):.2f} us")


summary("forward", tr[0], ["start", "agg", "gemm1", "ready", "arrive", "group", "seen", "go"], range(5))
summary("backward", tr[1], ["start", "sums", "arrive", "group", "seen", "go", "dz1"], range(4, -1, -1))
def prologue(name, t, stamps):
    t = t.view(1024, 64).cpu()
    t = t[t[:, 56] > 0].double()
    parts = []
    for a, b in zip(stamps[:-1], stamps[1:]):
        d = (t[:, b] - t[:, a]) / 100.0
        parts.append(f"{a}->{b} {float(d.median()):.2f}/{float(d.max()):.2f}")
    print(f"  {name} prologue: " + " | ".join(parts))


prologue("forward", tr[0], [56, 57, 58, 0])
prologue("backward", tr[1], [56, 57, 8 * 4])
slowest(tr[0], 1, 0, 1)
slowest(tr[0], 1, 1, 2)
slowest(tr[0], 1, 2, 3)

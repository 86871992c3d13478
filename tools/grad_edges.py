"""List the parameters whose gradient autograd sums from several contributions
(an AccumulateGrad node reached by more than one edge, or a tensor whose
grad_fn feeds several consumers) in one eager pretrain step of the bench
workload: python tools/grad_edges.py  (GPU)"""
import importlib
import os
import sys
from collections import Counter

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("s-cgib_amd")
import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    F_in = pkg.synth.WORKLOADS["qm9"][2]
    gh, _ = pkg.graph.collate_pyg(pkg.synth.molecules(512, "qm9", seed=0))
    g = gh.to(dev)
    dict.__setitem__(g.ndata, "x", F.normalize(g.ndata["x"].float()))
    model = bench.make_model(F_in, 1, 5, dev)
    names = {id(p): n for n, p in model.named_parameters()}
    _, kl, con, rec = model(g, g.ndata["x"], None, None, None, 1, None, 1, dev, 512)
    indeg = Counter()
    seen, stack = set(), [t.grad_fn for t in (kl, con, rec) if t.grad_fn is not None]
    while stack:
        fn = stack.pop()
        if fn in seen:
            continue
        seen.add(fn)
        for nxt, _ in fn.next_functions:
            if nxt is None:
                continue
            indeg[nxt] += 1
            stack.append(nxt)
    for fn, k in indeg.items():
        if k > 1:
            var = getattr(fn, "variable", None)
            label = names.get(id(var), "?") if var is not None else type(fn).__name__
            shape = tuple(var.shape) if var is not None else ""
            print(f"{k} contributions -> {label} {shape}")
    (kl + con + rec).backward()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()

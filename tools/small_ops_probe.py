"""Where the pretrain step's small torch kernels come from: runs the bench's
capacity-mode step body (batch load, ego prefetch, forward, backward, Adam)
eagerly and prints, for every kernel-launching aten op the step runs (a TorchDispatchMode: also the ops the autograd
engine runs, e.g. gradient accumulation) the package frames of its Python
stack.  The replayed graph holds the same
launches (profiles/*/kernel_instances.txt: __amd_rocclr_copyBuffer,
FillFunctor).

    python tools/small_ops_probe.py            (on the GPU box)
"""
import collections
import importlib
import os
import sys

import torch
import torch.nn.functional as F
import traceback
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

pkg = importlib.import_module("s-cgib_amd")
# no kernel (allocation, views, metadata)
QUIET = {"empty", "empty_like", "empty_strided", "view", "_unsafe_view", "reshape", "t",
         "transpose", "detach", "alias", "as_strided", "select", "slice", "unsqueeze",
         "squeeze", "expand", "permute", "lift_fresh", "_to_copy_meta", "is_same_size",
         "sym_size", "sym_stride", "sym_numel", "sym_storage_offset", "_local_scalar_dense",
         "set_", "resize_", "new_empty", "new_empty_strided"}


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(1234)
    batch, k, workload = 512, 1, "qm9"
    F_in = pkg.synth.WORKLOADS[workload][2]
    pool_host = []
    for i in range(4):
        gh, _ = pkg.graph.collate_pyg(pkg.synth.molecules(batch, workload, seed=i))
        pool_host.append(gh)
    model = bench.make_model(F_in, k, 5, dev)
    opt = pkg.optim.Adam(model.parameters(), lr=1e-4, weight_decay=5e-5)
    n_cap, e_cap, mgn, ego_caps = pkg.graph.StaticBatch.capacities(pool_host, k, slack=1.02)
    static = pkg.graph.StaticBatch(batch, n_cap, e_cap, F_in, mgn, ego_caps, dev, k=k)
    padded = []
    for gh in pool_host:
        gx = pkg.graph.GraphBatch.from_edges(*[t.numpy() for t in gh.edges()], gh.num_nodes(),
                                             True, gh.batch_num_nodes_host())
        dict.__setitem__(gx.ndata, "x", F.normalize(gh.ndata["x"].float()))
        padded.append(static.pad(gx))
    pool_dev = static.pool(padded)
    one = torch.ones((), dtype=torch.float32, device=dev)
    prefetch = pkg.graph.EgoPrefetch(static, pool_dev)
    prefetch.prime()

    def step():
        static.load_next(pool_dev, prefetch)
        _, kl, con, rec = model(static.graph, static.x, None, None, None, 1, None, k, dev, batch)
        torch.autograd.backward((kl, rec, con), (one, one, one))
        prefetch.join()
        opt.step()

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            opt.zero_grad(set_to_none=True)
            step()
        torch.cuda.synchronize()
        opt.zero_grad(set_to_none=True)  # as before the capture
        log = []

        class Mode(TorchDispatchMode):
            def __torch_dispatch__(self, func, types, args=(), kwargs=None):
                name = str(func.overloadpacket.__name__)
                if name not in QUIET:
                    st = [f"{os.path.basename(fr.filename)}:{fr.lineno} {fr.name}"
                          for fr in traceback.extract_stack()
                          if "s-cgib_amd" in fr.filename or "small_ops" in fr.filename]
                    log.append((name, tuple(st[-3:])))
                return func(*args, **(kwargs or {}))
        with Mode():
            step()
        torch.cuda.synchronize()
    counts = collections.Counter(log)
    print(f"{len(log)} aten ops (views / empty / metadata excluded) in one eager step:")
    for (name, st), c in sorted(counts.items(), key=lambda kv: kv[0][1]):
        print(f"{c:3d} x aten.{name}")
        for f in st:
            print(f"        {f}")


if __name__ == "__main__":
    main()

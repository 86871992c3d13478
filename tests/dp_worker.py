"""One rank of the data-parallel parity run (tests/test_gpu_dp.py), launched by
``python -m torch.distributed.run --nproc-per-node 2 tests/dp_worker.py OUT``
with SCGIB_DIST_BACKEND=gloo (two ranks on one GPU; the 8-GPU runs use RCCL).

Each rank runs the product step exactly as bench.py's N > 1 path does —
capacity mode, one captured graph of (forward, backward, bucket pack), the
all-reduce of the bucket between replays, a second captured graph of
(1/world unpack, Adam) — on its own shard of the molecules
(exp_pretraining.py:290-333 on a sub-batch, then the gradient average of
exp_pretraining.py:321-323's optimizer step), with explicit noise.  It writes
its shard's raw gradients and BatchNorm statistics (before the average) and
every parameter and buffer after the step, for the test to compare."""
import copy
import importlib
import os
import sys
from types import SimpleNamespace

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

B_TOTAL = 128
WORKLOAD = "qm9"
K = 1


def make_model(pkg, F_in, B):
    """Mainmodel_continue (exp_pretraining.py:109-113), GIN-64x5, seeded so
    every rank and the test process build the same weights."""
    args = SimpleNamespace(recons_type="adj", useAtt=1, readout_f="sum", d_transfer=32,
                           batch_size=B, gin_layers=5, task="graph_classification")
    torch.manual_seed(2024)
    inner = pkg.models.Mainmodel(args, F_in, 64, 4, 4, K, "GIN")
    model = pkg.models.Mainmodel_continue(args, F_in, 64, 4, 4, K, 1, inner, "GIN")
    with torch.no_grad():
        for n, p in model.named_parameters():
            if "batch_norms" in n or "compressor.1" in n:
                p.add_(0.2 * torch.randn_like(p))
    return model


def shard_and_noise(pkg, rank, world):
    """This rank's molecules (dist.shard of one seeded set) and its noise."""
    mols = pkg.synth.molecules(B_TOTAL, WORKLOAD, seed=41)
    mine = pkg.dist.shard(mols, rank, world)
    gh, _ = pkg.graph.collate_pyg(mine)
    gen = torch.Generator().manual_seed(500 + rank)
    n = gh.num_nodes()
    return gh, torch.rand(n, generator=gen), torch.rand(n, 64, generator=gen)


def main(out_dir):
    pkg = importlib.import_module("s-cgib_amd")
    rank, world, local = pkg.dist.init_from_env()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    # both ranks share one GPU (time-sliced processes): the hand-off rule
    # refuses the signal / wait kernels (as in bench.py)
    ok, why = pkg.ops.handoff_rule(torch.cuda.device_count())
    assert not ok, why
    pkg.ops.XQ_FLAGS = False
    F_in = pkg.synth.WORKLOADS[WORKLOAD][2]
    B = B_TOTAL // world
    gh, u_gate, u_feat = shard_and_noise(pkg, rank, world)
    model = make_model(pkg, F_in, B).to(dev).train()
    reducer = pkg.dist.GradAllReducer(model.parameters(), buffers=pkg.dist.bn_buffers(model))
    opt = pkg.optim.Adam(model.parameters(), lr=1e-3, weight_decay=5e-5)

    n_cap, e_cap, mgn, caps = pkg.graph.StaticBatch.capacities([gh], K, slack=1.02)
    static = pkg.graph.StaticBatch(B, n_cap, e_cap, F_in, mgn, caps, dev, k=K)
    gx = pkg.graph.GraphBatch.from_edges(*[t.numpy() for t in gh.edges()], gh.num_nodes(), True,
                                         gh.batch_num_nodes_host())
    dict.__setitem__(gx.ndata, "x", F.normalize(gh.ndata["x"].float()))
    static.load(static.pad(gx))
    s_ug = torch.zeros(n_cap, device=dev)
    s_uf = torch.zeros(n_cap, 64, device=dev)
    n = gh.num_nodes()
    s_ug[:n].copy_(u_gate)
    s_uf[:n].copy_(u_feat)

    def body():
        _, kl, con, rec = model(static.graph, static.x, None, None, None, 1, None, K, dev, B,
                                noise=(s_ug, s_uf))
        (kl + con + rec).backward()
        return torch.stack([kl, con, rec]).detach()

    snap = copy.deepcopy(model.state_dict())
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # warm-up: allocator, Adam state, the flat bucket
        opt.zero_grad(set_to_none=True)
        body()
        reducer.pack()
        reducer.reduce(force=True)
        reducer.unpack()
        opt.step()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    model.load_state_dict(snap)  # undo the warm-up step (same storages)
    for st in opt.state.values():
        for v in st.values():
            v.zero_()
    opt.zero_grad(set_to_none=True)
    g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1):
        losses = body()
        reducer.pack()
    with torch.cuda.graph(g2):
        reducer.unpack()
        opt.step()
    g1.replay()
    torch.cuda.synchronize()
    names = [k for k, p in model.named_parameters() if p.grad is not None]
    params = dict(model.named_parameters())
    raw = {"grads": {k: params[k].grad.detach().cpu().clone() for k in names},
           "buffers": {k: v.detach().cpu().clone() for k, v in model.named_buffers()},
           "losses": losses.cpu()}
    reducer.reduce(force=True)  # gloo all-reduce (SUM) of the bucket between the replays
    g2.replay()
    torch.cuda.synchronize()
    after = {"params": {k: p.detach().cpu().clone() for k, p in model.named_parameters()},
             "buffers": {k: v.detach().cpu().clone() for k, v in model.named_buffers()},
             "xq_timeouts": pkg.ops.xq_timeouts(dev)}
    torch.save({"raw": raw, "after": after, "init": {k: v.cpu() for k, v in snap.items()}},
               os.path.join(out_dir, f"rank{rank}.pt"))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])

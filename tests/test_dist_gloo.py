"""Data-parallel path on CPU with gloo, world_size 2.

Replica mode: each rank runs the pretrain step on its own shard of the
molecules; the averaged gradient must equal the mean of the per-shard
gradients computed in one process.  The per-shard step here is the oracle
(CPU) so the test runs without a GPU; the reducer is the product's."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F

from conftest import CANCELLED

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_grads(molecules, seed, buffers=None):
    """Oracle pretrain-step gradients for one shard of molecules."""
    import importlib
    sys.path.insert(0, ROOT)
    from oracle import egonet
    from oracle import scgib_ref as R
    pkg = importlib.import_module("s-cgib_amd")
    torch.manual_seed(seed)
    g, _ = pkg.graph.collate_pyg(molecules)
    sizes, ecount, nodes, esrc, edst = egonet.egonets(g.rowptr.numpy(), g.col.numpy(), 1)
    off = np.repeat(np.concatenate([[0], np.cumsum(sizes)[:-1]]), ecount)
    src, dst = g.edges()
    batch = {"src": src, "dst": dst, "counts": torch.from_numpy(g.batch_num_nodes_host())}
    ego = {"src": torch.from_numpy(esrc + off), "dst": torch.from_numpy(edst + off),
           "counts": torch.from_numpy(sizes)}
    x = F.normalize(g.ndata["x"].float())
    torch.manual_seed(0)  # identical init on every rank
    from types import SimpleNamespace
    args = SimpleNamespace(recons_type="adj", useAtt=1, readout_f="sum", d_transfer=32,
                           gin_layers=2)
    model = pkg.models.Mainmodel(args, 11, 64, 4, 4, 1, "GIN")
    params = {k: v.detach().clone().requires_grad_(v.is_floating_point() and "running" not in k
                                                   and not k.endswith(".eps"))
              for k, v in model.state_dict().items()}
    gen = torch.Generator().manual_seed(seed)
    if buffers is not None:  # BN running statistics, updated by this step
        buffers.update({k: v.detach().clone() for k, v in params.items()
                        if "running" in k or "num_batches" in k})
    out = R.pretrain_forward(params, batch, ego, x, x[torch.from_numpy(nodes)],
                             torch.rand(len(x), generator=gen), torch.rand(len(x), 64, generator=gen),
                             64, buffers)
    out["loss_total"].backward()
    return {k: v.grad.clone() for k, v in params.items() if v.grad is not None}, params


def _worker(rank, world, port, molecules, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    import importlib
    pkg = importlib.import_module("s-cgib_amd")
    r, w, _ = pkg.dist.init_from_env(backend="gloo")
    shard = pkg.dist.shard(molecules, r, w)
    grads, params = _shard_grads(shard, seed=100 + r)
    holder = [p for p in params.values() if p.requires_grad]
    reducer = pkg.dist.GradAllReducer(holder)
    reducer()
    if r == 0:
        # numpy (pickled by value): torch tensors would travel as shared fds that
        # race with this process's exit
        q.put({k: params[k].grad.numpy().copy() for k in grads})
    dist.barrier()
    dist.destroy_process_group()


# world sizes of the driver's runs (2, 4, 8 ranks) and an odd one; 13
# molecules divide evenly by none of them, so the shards are uneven (at 8
# ranks: 2,2,2,2,2,1,1,1) — replica mode still weights every rank's
# per-shard mean by 1/world, not by its shard size
WORLDS = [2, 3, 4, 8]
N_MOLS = 13


@pytest.mark.timeout(400)
@pytest.mark.parametrize("world", WORLDS)
def test_grad_allreduce_matches_mean_of_shards(pkg, world):
    mols = pkg.synth.molecules(N_MOLS, "qm9", seed=21)
    assert N_MOLS % world != 0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mols, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=360)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = {}
    for r in range(world):
        gr, _ = _shard_grads(pkg.dist.shard(mols, r, world), seed=100 + r)
        for k, v in gr.items():
            expect[k] = expect.get(k, 0) + v / world
    assert set(got) == set(expect)
    # per-tensor tolerance (an uneven-shard weighting error on a small-gradient
    # tensor must not hide under the largest tensor's scale); only the tensors
    # whose true gradient is exactly zero — a GIN MLP's last bias feeds a
    # BatchNorm, which removes it — hold fp32 summation-order noise on both
    # sides (CPU threads differ between the workers and this process): those
    # are bounded absolutely, by name, against their weight's gradient scale
    for k in expect:
        exp = expect[k]
        if k.endswith(CANCELLED):
            floor = 1e-5 * float(expect[k.rsplit(".", 1)[0] + ".weight"].abs().max())
            assert float((torch.from_numpy(got[k]) - exp).abs().max()) <= floor, k
            continue
        assert torch.allclose(torch.from_numpy(got[k]), exp, rtol=1e-5,
                              atol=1e-5 * float(exp.abs().max())), k


def test_shard_covers_everything_once(pkg):
    items = list(range(103))
    parts = [pkg.dist.shard(items, r, 8) for r in range(8)]
    assert sum(parts, []) == items
    assert max(map(len, parts)) - min(map(len, parts)) <= 1


def _buffer_worker(rank, world, port, molecules, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    import importlib
    pkg = importlib.import_module("s-cgib_amd")
    r, w, _ = pkg.dist.init_from_env(backend="gloo")
    bufs = {}
    _, params = _shard_grads(pkg.dist.shard(molecules, r, w), seed=100 + r, buffers=bufs)
    holder = [p for p in params.values() if p.requires_grad]
    running = [v for k, v in sorted(bufs.items()) if "running" in k]
    pkg.dist.GradAllReducer(holder, buffers=running)()
    out = {k: v.numpy().copy() for k, v in bufs.items() if "running" in k}
    q.put((r, out))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(400)
@pytest.mark.parametrize("world", WORLDS)
def test_bn_buffers_identical_across_ranks(pkg, world):
    """With the BN running statistics in the gradient bucket (GradAllReducer
    buffers=), every rank holds the same statistics after each step — their
    mean over the ranks' (uneven) shards, 1/world each."""
    mols = pkg.synth.molecules(N_MOLS, "qm9", seed=22)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_buffer_worker, args=(r, world, port, mols, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=360) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(got) == world and len(got[0]) > 0
    assert all(set(got[r]) == set(got[0]) for r in range(world))
    expect = {}
    for r in range(world):
        bufs = {}
        _shard_grads(pkg.dist.shard(mols, r, world), seed=100 + r, buffers=bufs)
        for k, v in bufs.items():
            if "running" in k:
                expect[k] = expect.get(k, 0) + v / world
    for k in got[0]:
        for r in range(1, world):  # every replica bitwise rank 0's
            np.testing.assert_array_equal(got[0][k], got[r][k], err_msg=f"{k} rank {r}")
        assert torch.allclose(torch.from_numpy(got[0][k]), expect[k], rtol=1e-6, atol=1e-7), k


def _bcast_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    import importlib
    from types import SimpleNamespace
    pkg = importlib.import_module("s-cgib_amd")
    pkg.dist.init_from_env(backend="gloo")
    torch.manual_seed(1234 + rank)  # the bench's per-rank seed: different initial weights
    args = SimpleNamespace(recons_type="adj", useAtt=1, readout_f="sum", d_transfer=32,
                           gin_layers=2)
    model = pkg.models.Mainmodel(args, 11, 64, 4, 4, 1, "GIN")
    with torch.no_grad():  # a rank-dependent buffer too
        next(iter(b for n, b in model.named_buffers() if n.endswith("running_mean"))).fill_(rank)
    before = {k: v.numpy().copy() for k, v in model.state_dict().items()}
    pkg.dist.broadcast_replicas(model)
    q.put((rank, before, {k: v.numpy().copy() for k, v in model.state_dict().items()}))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_broadcast_replicas_makes_ranks_identical(pkg):
    """bench.py's replica sync: differently seeded ranks hold rank 0's
    parameters and buffers, bitwise, after broadcast_replicas."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bcast_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (b, a)) for r, b, a in (q.get(timeout=240) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (b0, a0), (b1, a1) = got[0], got[1]
    assert any(not np.array_equal(b0[k], b1[k]) for k in b0)  # they did differ
    for k in a0:
        np.testing.assert_array_equal(a0[k], b0[k], err_msg=k)  # rank 0 kept its own
        np.testing.assert_array_equal(a1[k], a0[k], err_msg=k)

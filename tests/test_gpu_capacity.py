"""Capacity mode and whole-step HIP-graph replay.

A ``graph.StaticBatch`` holds capacity-sized buffers; every kernel reads the
batch's actual node / edge counts from the device (``dims``), so one captured
step serves every batch that fits.  The bar: the same pretrain step (ego-net
build, both GIN encoders, interaction, losses, backward) on the same batch and
noise gives the exact-mode losses, gradients and BN running statistics —
eager on the static buffers, and replayed from a captured graph over several
different batches.  Exact mode itself is pinned to the reference goldens by
test_gpu_parity.py; the two modes differ only in grid sizes, hence in fp32
reduction grouping, and fp32 ReLU-kink flips are tolerated as there.
"""
import copy
from types import SimpleNamespace

import pytest
import torch
import torch.nn.functional as F

from conftest import CANCELLED, check_grads_model, rel_err, rel_l2

pytestmark = pytest.mark.gpu

B = 48
F_IN = 11
LOSS_TOL = 2e-5


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    return torch.device("cuda", 0)


def _model(pkg, dev, layers=5, k=1):
    args = SimpleNamespace(recons_type="adj", useAtt=1, readout_f="sum", d_transfer=32,
                           batch_size=B, gin_layers=layers)
    torch.manual_seed(11)
    m = pkg.models.Mainmodel(args, F_IN, 64, 4, 4, k, "GIN").to(dev).train()
    with torch.no_grad():  # non-trivial BN affine so the BN paths are exercised
        for enc in (m.Encoder1, m.Encoder2):
            for bn in enc.batch_norms:
                bn.weight.add_(0.2 * torch.randn(64, device=dev))
                bn.bias.add_(0.2 * torch.randn(64, device=dev))
    return m


def _batches(pkg, seeds):
    out = []
    for s in seeds:
        gh, _ = pkg.graph.collate_pyg(pkg.synth.molecules(B, "qm9", seed=s))
        dict.__setitem__(gh.ndata, "x", F.normalize(gh.ndata["x"].float()))
        out.append(gh)
    return out


def _step(model, g, x, noise, dev, k=1):
    model.zero_grad(set_to_none=True)
    _, kl, con, rec = model(g, x, None, None, None, 1, None, k, dev, B, noise=noise)
    loss = kl + rec + con
    loss.backward()
    return torch.stack([kl, con, rec, loss]).detach()


def _compare(exact_model, cap_model, exact_losses, cap_losses):
    for a, b in zip(exact_losses.tolist(), cap_losses.tolist()):
        assert rel_err(b, a) < LOSS_TOL, (a, b)
    ref = {k: p.grad.detach().double().cpu() for k, p in exact_model.named_parameters()
           if p.grad is not None}
    mine = dict(cap_model.named_parameters())
    check_grads_model(ref, lambda n: mine[n].grad, tol=1e-3)
    bufs = dict(cap_model.named_buffers())
    for k, v in exact_model.named_buffers():
        if "running" in k:
            assert rel_err(bufs[k].cpu(), v.cpu()) < 1e-5, k
        elif "num_batches" in k:
            assert int(bufs[k]) == int(v), k


def _noise(n_cap, dev, seed):
    gen = torch.Generator(device=dev).manual_seed(seed)
    return (torch.rand(n_cap, device=dev, generator=gen),
            torch.rand(n_cap, 64, device=dev, generator=gen))


def test_capacity_mode_eager_matches_exact(pkg, dev):
    hosts = _batches(pkg, (1, 2, 3))
    n_cap, e_cap, mgn, caps = pkg.graph.StaticBatch.capacities(hosts, 1, slack=1.05)
    static = pkg.graph.StaticBatch(B, n_cap, e_cap, F_IN, mgn, caps, dev)
    exact_m = _model(pkg, dev)
    cap_m = copy.deepcopy(exact_m)
    for i, gh in enumerate(hosts):
        n = gh.num_nodes()
        ug, uf = _noise(n_cap, dev, 100 + i)
        g = gh.to(dev)
        le = _step(exact_m, g, g.ndata["x"], (ug[:n], uf[:n]), dev)
        static.load(static.pad(gh))
        lc = _step(cap_m, static.graph, static.x, (ug, uf), dev)
        torch.cuda.synchronize()
        _compare(exact_m, cap_m, le, lc)


@pytest.mark.parametrize("k,fork_losses", [(1, False), (2, False), (1, True)])
def test_graph_replay_matches_exact_over_batches(pkg, dev, k, fork_losses, monkeypatch):
    """Graph replay over several batches == exact mode; fork_losses: the
    contrastive loss on the side stream (SCGIB_FORK_LOSSES=1) together with
    the forked encoder pair — flat forks only, captured and replayed."""
    monkeypatch.setattr(pkg.models, "FORK_LOSSES", fork_losses)
    hosts = _batches(pkg, (4, 5, 6, 7))
    n_cap, e_cap, mgn, caps = pkg.graph.StaticBatch.capacities(hosts, k, slack=1.02)
    static = pkg.graph.StaticBatch(B, n_cap, e_cap, F_IN, mgn, caps, dev, k=k)
    padded = [static.pad(gh) for gh in hosts]
    exact_m = _model(pkg, dev, k=k)
    cap_m = copy.deepcopy(exact_m)
    s_ug = torch.zeros(n_cap, device=dev)
    s_uf = torch.zeros(n_cap, 64, device=dev)

    # warm-up on a side stream (allocator), then capture one step
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    snap = copy.deepcopy(cap_m.state_dict())
    with torch.cuda.stream(side):
        static.load(padded[0])
        _step(cap_m, static.graph, static.x, (s_ug, s_uf), dev, k)
    torch.cuda.current_stream().wait_stream(side)
    cap_m.load_state_dict(snap)  # undo the warm-up's BN running updates
    cap_m.zero_grad(set_to_none=True)
    arenas = len(pkg.ops._SCAN_ARENAS[dev.index or 0])
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        _, kl, con, rec = cap_m(static.graph, static.x, None, None, None, 1, None, k, dev, B,
                                noise=(s_ug, s_uf))
        loss = kl + rec + con
        loss.backward()
        static_losses = torch.stack([kl, con, rec, loss]).detach()
    # the capture's stream is new to every scan-state call site: their words
    # came from the pre-zeroed arena, no zero-fill was captured into the step
    assert len(pkg.ops._SCAN_ARENAS[dev.index or 0]) == arenas

    t0 = pkg.ops.xq_timeouts(dev)
    for i in (0, 1, 2, 3, 1):  # includes a batch seen before (replay is stateless)
        gh = hosts[i]
        n = gh.num_nodes()
        ug, uf = _noise(n_cap, dev, 200 + i)
        g = gh.to(dev)
        le = _step(exact_m, g, g.ndata["x"], (ug[:n], uf[:n]), dev, k)
        s_ug.copy_(ug)
        s_uf.copy_(uf)
        static.load(padded[i])
        graph.replay()
        torch.cuda.synchronize()
        _compare(exact_m, cap_m, le, static_losses.clone())
    # the encoder pair's signal / wait hand-offs (ops.XQ_FLAGS): every wait saw
    # its signal in the replayed graph (the kernels landed on different queues)
    assert pkg.ops.xq_timeouts(dev) == t0


def test_capacity_step_r_recompute_bitwise(pkg, dev, monkeypatch):
    """The whole pretrain step in capacity mode (padded rows, device dims:
    the recompute kernels' zero-padding and clamped-row paths) with the
    hidden activation r recomputed in the backward vs stored by the forward
    (ops.STORE_R): losses, every gradient and BN buffer bitwise equal.  (Both
    on the stored-agg backward, ops.AGG_FREE off: the recompute reads agg.)"""
    monkeypatch.setattr(pkg.ops, "AGG_FREE", False)
    hosts = _batches(pkg, (21, 22))
    n_cap, e_cap, mgn, caps = pkg.graph.StaticBatch.capacities(hosts, 1, slack=1.05)
    static = pkg.graph.StaticBatch(B, n_cap, e_cap, F_IN, mgn, caps, dev)
    base = _model(pkg, dev)
    res = []
    for store in (True, False):
        monkeypatch.setattr(pkg.ops, "STORE_R", store)
        m = copy.deepcopy(base)
        losses = []
        for i, gh in enumerate(hosts):
            static.load(static.pad(gh))
            losses.append(_step(m, static.graph, static.x, _noise(n_cap, dev, 300 + i), dev))
        torch.cuda.synchronize()
        res.append((torch.stack(losses), {k: p.grad.clone() for k, p in m.named_parameters()
                                          if p.grad is not None},
                    {k: b.clone() for k, b in m.named_buffers()}))
    (la, ga, ba), (lb, gb, bb) = res
    assert torch.equal(la, lb)
    assert ga.keys() == gb.keys()
    for k in ga:
        assert torch.equal(ga[k], gb[k]), k
    for k in ba:
        assert torch.equal(ba[k], bb[k]), k


def test_capacity_step_agg_free_matches_stored_agg(pkg, dev, monkeypatch):
    """the agg-free layers (ops.AGG_FREE: no agg stored,
    dz1 out of the layer backward, dW1 = g^T h and d h = g W1 in the layer
    below's statistics launch) against the stored-agg backward, on the whole
    pretrain step in capacity mode over two batches: the forward is the same
    kernels minus a store, so losses and every BatchNorm buffer are bitwise
    equal; the gradients associate the same sums differently — every tensor
    within 2e-5 relative L2 (the rounding-only bound; a wrong product or
    index is O(1))."""
    monkeypatch.setattr(pkg.ops, "AGG_FREE_MIN_ROWS", 0)  # (every encoder, whatever its size)
    hosts = _batches(pkg, (23, 24))
    n_cap, e_cap, mgn, caps = pkg.graph.StaticBatch.capacities(hosts, 1, slack=1.05)
    static = pkg.graph.StaticBatch(B, n_cap, e_cap, F_IN, mgn, caps, dev)
    base = _model(pkg, dev)
    res = []
    for free in (True, False):
        monkeypatch.setattr(pkg.ops, "AGG_FREE", free)
        m = copy.deepcopy(base)
        losses = []
        for i, gh in enumerate(hosts):
            static.load(static.pad(gh))
            losses.append(_step(m, static.graph, static.x, _noise(n_cap, dev, 400 + i), dev))
        torch.cuda.synchronize()
        res.append((torch.stack(losses), {k: p.grad.clone() for k, p in m.named_parameters()
                                          if p.grad is not None},
                    {k: b.clone() for k, b in m.named_buffers()}))
    (la, ga, ba), (lb, gb, bb) = res
    assert torch.equal(la, lb)
    assert ga.keys() == gb.keys()
    worst = 0.0
    for k in ga:
        if k.endswith(CANCELLED):  # rounding noise on both sides
            continue
        e = rel_l2(ga[k].cpu(), gb[k].cpu())
        worst = max(worst, e)
        assert e < 2e-5, (k, e)
    print(f"agg-free vs stored agg: worst gradient rel-L2 {worst:.2e}")
    for k in ba:
        assert torch.equal(ba[k], bb[k]), k


def test_static_batch_rejects_oversized(pkg, dev):
    small, big = _batches(pkg, (8,)), None
    n_cap, e_cap, mgn, caps = pkg.graph.StaticBatch.capacities(small, 1)
    static = pkg.graph.StaticBatch(B, n_cap, e_cap, F_IN, mgn, caps, dev)
    for seed in range(9, 40):
        cand = _batches(pkg, (seed,))[0]
        if cand.num_nodes() > n_cap or cand.num_edges() > e_cap:
            big = cand
            break
    assert big is not None
    with pytest.raises(pkg._lib.ScgibError):
        static.pad(big)


def test_nested_fork_refused_while_capturing(pkg, dev, monkeypatch):
    """ops.check_fork: a fork taken from one of the library's forked streams
    while a HIP graph is being captured raises (torch-ROCm's capture_end
    crashes on nested forks); from any other stream, or outside
    a capture, it is allowed.  The capture state is simulated: a real nested
    capture would end in the crash this guard exists to prevent."""
    side = pkg.models._side_stream(dev)
    other = torch.cuda.Stream(dev)
    pkg.ops.check_fork(side)  # not capturing: fine
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: True)
    pkg.ops.check_fork(other)
    pkg.ops.check_fork(torch.cuda.current_stream(dev))
    with pytest.raises(RuntimeError, match="nested forks"):
        pkg.ops.check_fork(side)
    _, aux = pkg.ops._aux_stream(dev)
    with pytest.raises(RuntimeError, match="nested forks"):
        pkg.ops.check_fork(aux)


def test_deferred_loss_reduces_bitwise(pkg, dev, monkeypatch):
    """SlabScope: the interaction's and compressor[0]'s weight-gradient slabs
    summed by Encoder1's final multi-job reduce give the same gradients, bit
    for bit, as their own reduce launches (same fixed order per job); the
    head MLP's, reduced by the fold workgroups of Encoder1's first backward
    launch (4 partitions per column, fp64 final sum),
    agree to fp32 summation order; and the deferral is actually taken (3
    jobs per step)."""
    gh = _batches(pkg, (9,))[0]
    g = gh.to(dev)
    n = g.num_nodes()
    ug, uf = _noise(n, dev, 300)
    m_inline = _model(pkg, dev)
    m_defer = copy.deepcopy(m_inline)
    added = []
    orig_add = pkg.ops.SlabScope.add

    def counting_add(self, *a):
        added.append(a[2])
        return orig_add(self, *a)

    monkeypatch.setattr(pkg.ops.SlabScope, "add", counting_add)
    monkeypatch.setattr(pkg.ops, "DEFER_LOSS_REDUCE", False)
    l_inline = _step(m_inline, g, g.ndata["x"], (ug, uf), dev)
    assert added == []
    monkeypatch.setattr(pkg.ops, "DEFER_LOSS_REDUCE", True)
    l_defer = _step(m_defer, g, g.ndata["x"], (ug, uf), dev)
    torch.cuda.synchronize()
    assert len(added) == 3, added  # head MLP, interaction, compressor[0]
    assert torch.equal(l_inline, l_defer)
    inline = dict(m_inline.named_parameters())
    for k, p in m_defer.named_parameters():
        if p.grad is None:
            continue
        if k.startswith("MLP."):
            ref = inline[k].grad
            assert (p.grad - ref).norm() <= 1e-6 * ref.norm() + 1e-12, k
        else:
            assert torch.equal(p.grad, inline[k].grad), k
    # a .grad already present (accumulation): the reduces stay inline
    added.clear()
    _, kl, con, rec = m_defer(g, g.ndata["x"], None, None, None, 1, None, 1, dev, B,
                              noise=(ug, uf))
    (kl + rec + con).backward()
    torch.cuda.synchronize()
    assert added == []


@pytest.mark.parametrize("mode", ["grad", "inputs", "double"])
def test_deferred_loss_reduce_partial_and_cast_backward(pkg, dev, mode, monkeypatch):
    """SlabScope safety (ops.py): a backward that never reaches the encoder
    pair — autograd.grad over the head MLP's parameters only, or
    backward(inputs=[...]) — still reduces the deferred slabs (an engine
    callback at the end of the graph task), and a model whose parameters are
    not fp32 is never deferred (autograd casts the returned gradient at once).
    Each case equals the same run with the deferral off."""
    gh = _batches(pkg, (9,))[0]
    g = gh.to(dev)
    n = g.num_nodes()
    ug, uf = _noise(n, dev, 301)
    base = _model(pkg, dev)
    got = {}
    for defer in (False, True):
        monkeypatch.setattr(pkg.ops, "DEFER_LOSS_REDUCE", defer)
        m = copy.deepcopy(base)
        if mode == "double":
            m = m.double()
        m.zero_grad(set_to_none=True)
        _, kl, con, rec = m(g, g.ndata["x"], None, None, None, 1, None, 1, dev, B,
                            noise=(ug, uf))
        loss = kl + rec + con
        head = list(m.MLP.parameters()) + list(m.attn_layer.parameters())
        if mode == "grad":
            grads = torch.autograd.grad(loss, head)
        elif mode == "inputs":
            loss.backward(inputs=head)
            grads = [p.grad for p in head]
        else:
            loss.backward()
            grads = [p.grad for p in m.parameters() if p.grad is not None]
        torch.cuda.synchronize()
        got[defer] = [t.detach().clone() for t in grads]
    assert len(got[True]) == len(got[False]) > 0
    for a, b in zip(got[False], got[True]):
        assert torch.isfinite(b).all()
        assert (a - b).norm() <= 1e-6 * a.norm() + 1e-12


def test_pool_load_next_walks_the_pool(pkg, dev):
    """StaticBatch.load_next (scgib_pool_copy, bench.py's in-graph batch load):
    eager and captured in a HIP graph, each call / replay copies the pool's
    next batch in, in order, byte for byte; the cursor's arrival word stays 0."""
    hosts = _batches(pkg, (4, 5, 6))
    n_cap, e_cap, mgn, caps = pkg.graph.StaticBatch.capacities(hosts, 1, slack=1.02)
    static = pkg.graph.StaticBatch(B, n_cap, e_cap, F_IN, mgn, caps, dev)
    padded = [static.pad(gh) for gh in hosts]
    pool = static.pool(padded)
    for i in range(4):
        static.load_next(pool)
        torch.cuda.synchronize()
        assert torch.equal(static.blob, padded[i % 3]["blob"])
    graph = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        with torch.cuda.graph(graph):
            static.load_next(pool)
    torch.cuda.synchronize()
    for i in range(4, 9):
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(static.blob, padded[i % 3]["blob"])
    assert pool["cursor"].tolist() == [9, 0]


@pytest.mark.parametrize("k", [1, 2])
def test_ego_prefetch_replay_bitwise(pkg, dev, k):
    """graph.EgoPrefetch (bench.py's step): each replayed step builds the ego-nets
    of the batch the next step loads (pool-indirect one-pass builder, on the
    encoder pair's side stream) and the next load_next moves them in.  Against
    the same step building its own ego-nets at its head: the same losses,
    gradients and BN running statistics bit for bit over the pool, and the
    moved-in ego buffers equal an eager egonet_batch of the loaded batch."""
    hosts = _batches(pkg, (4, 5, 6, 7))
    n_cap, e_cap, mgn, caps = pkg.graph.StaticBatch.capacities(hosts, k, slack=1.02)
    ug, uf = _noise(n_cap, dev, 300)
    runs = {}
    for mode in (False, True):
        static = pkg.graph.StaticBatch(B, n_cap, e_cap, F_IN, mgn, caps, dev, k=k)
        padded = [static.pad(gh) for gh in hosts]
        pool = static.pool(padded)
        pf = pkg.graph.EgoPrefetch(static, pool) if mode else None
        if pf is not None:
            assert pf.onepass == (k == 1)
        model = _model(pkg, dev, k=k)

        def body():
            static.load_next(pool, pf)
            _, kl, con, rec = model(static.graph, static.x, None, None, None, 1, None, k, dev,
                                    B, noise=(ug, uf))
            (kl + rec + con).backward()
            if pf is not None:
                pf.join()
            return torch.stack([kl, con, rec]).detach()

        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            if pf is not None:
                pf.prime()
            for _ in range(2):  # eager steps (allocator warm-up), batches 0, 1
                model.zero_grad(set_to_none=False)
                body()
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        model.zero_grad(set_to_none=False)
        with torch.cuda.graph(graph):
            out = body()
        got = []
        for i in range(6):  # batches 2, 3, 0, 1, 2, 3
            for p in model.parameters():
                if p.grad is not None:
                    p.grad.zero_()
            graph.replay()
            torch.cuda.synchronize()
            grads = [p.grad.clone() for p in model.parameters() if p.grad is not None]
            bufs = [b.clone() for n, b in model.named_buffers() if "running" in n]
            got.append((out.clone(), grads, bufs))
            if pf is not None:
                ref = pkg.graph.egonet_batch(static.graph, k)
                torch.cuda.synchronize()
                n_s = int(ref.dims[0])
                e_s = int(ref.dims[1])
                assert torch.equal(pf.ego.dims, ref.dims)
                assert torch.equal(pf.ego.graph_ptr, ref.graph_ptr)
                assert torch.equal(pf.ego.ndata["_ID"][:n_s], ref.ndata["_ID"][:n_s])
                assert torch.equal(pf.ego.rowptr[: n_s + 1], ref.rowptr[: n_s + 1])
                assert torch.equal(pf.ego.col[:e_s], ref.col[:e_s])
        assert pkg.ops.xq_timeouts(dev) == 0
        if pf is not None:
            assert pf.error() == 0
        runs[mode] = got
    for (la, ga, ba), (lb, gb, bb) in zip(runs[False], runs[True]):
        assert torch.isfinite(la).all()
        assert torch.equal(la, lb)
        assert len(ga) == len(gb) > 0
        assert all(torch.equal(x, y) for x, y in zip(ga, gb))
        assert all(torch.equal(x, y) for x, y in zip(ba, bb))


def test_ego_prefetch_forward_only_joins(pkg, dev):
    """EgoPrefetch without a backward (no_grad forwards): the prefetch left on
    the side stream is joined by the next load_next before it copies the
    staging blob, so every loaded batch still carries its own ego-nets."""
    hosts = _batches(pkg, (4, 5, 6))
    n_cap, e_cap, mgn, caps = pkg.graph.StaticBatch.capacities(hosts, 1, slack=1.02)
    static = pkg.graph.StaticBatch(B, n_cap, e_cap, F_IN, mgn, caps, dev)
    pool = static.pool([static.pad(gh) for gh in hosts])
    pf = pkg.graph.EgoPrefetch(static, pool)
    model = _model(pkg, dev).eval()
    ug, uf = _noise(n_cap, dev, 302)
    pf.prime()
    with torch.no_grad():
        for _ in range(5):
            static.load_next(pool, pf)
            model(static.graph, static.x, None, None, None, 1, None, 1, dev, B, noise=(ug, uf))
            ref = pkg.graph.egonet_batch(static.graph, 1)
            torch.cuda.synchronize()
            n_s, e_s = (int(v) for v in ref.dims.tolist())
            assert torch.equal(pf.ego.ndata["_ID"][:n_s], ref.ndata["_ID"][:n_s])
            assert torch.equal(pf.ego.col[:e_s], ref.col[:e_s])
    pf.join()
    assert pf.error() == 0


def test_handoff_timeout_poisons_loss(pkg, dev):
    """A cross-queue hand-off wait that gives up (here: a wait with no signal
    at all) sets the device's sticky fault word, and from then on the
    pretraining step reports a NaN recon loss — not finite losses computed
    from data that may not have been written — until the caller clears it."""
    ops = pkg.ops
    ops.clear_handoff_fault(dev)
    gh = _batches(pkg, (21,))[0]
    g = gh.to(dev)
    m = _model(pkg, dev)
    ug, uf = _noise(g.num_nodes(), dev, 7)
    ok = _step(m, g, g.ndata["x"], (ug, uf), dev)
    assert torch.isfinite(ok).all()
    w = ops._xq_words(dev, "test_orphan_wait")
    ops._lib.call("scgib_stream_wait", ops._p(w), ops._p(ops.handoff_fault_word(dev)),
                  ops._p(ops._host_fault_word(dev)), ops._stream())
    torch.cuda.synchronize()
    assert int(w[2].item()) == 1 and ops.handoff_fault(dev)
    # loud: the pinned host word is set too, so the next
    # model forward / optimizer step raises, naming the hand-off
    assert int(ops._host_fault_word(dev)[0]) == 1
    with pytest.raises(ops._lib.ScgibError, match="hand-off"):
        _step(m, g, g.ndata["x"], (ug, uf), dev)
    opt = pkg.optim.Adam(m.parameters(), lr=1e-4)
    with pytest.raises(ops._lib.ScgibError, match="hand-off"):
        opt.step()
    # the device word alone (a caller that bypasses the host check): the
    # step's recon loss, and so the total, is NaN
    ops._host_fault_word(dev).zero_()
    bad = _step(m, g, g.ndata["x"], (ug, uf), dev)
    assert torch.isnan(bad[2]) and torch.isnan(bad[3])
    ops.clear_handoff_fault(dev)
    again = _step(m, g, g.ndata["x"], (ug, uf), dev)
    assert torch.isfinite(again).all()


def test_handoff_fault_raises_in_finetune(pkg, dev):
    """the fine-tune head ends in torch's BCE (NaN scores would
    trip its device-side range assert), so a hand-off fault reaches it as the
    host check: with the pinned host word set, the next fine-tune forward
    raises a ScgibError naming the hand-off; cleared, the step is finite."""
    import finetune_bench
    ops = pkg.ops
    ops.clear_handoff_fault(dev)
    ft, _ = finetune_bench.make_finetune_model(pkg, 9, 8, dev)
    gh, _ = pkg.graph.collate_pyg(pkg.synth.molecules(8, "molhiv", seed=3))
    g = gh.to(dev)
    x = F.normalize(g.ndata["x"].float())
    tgt = torch.randint(0, 2, (8, 1), device=dev).float()
    scores, *_ = ft(g, x, None, None, 1, None, 2, dev, 8)
    assert torch.isfinite(ft.loss(scores, tgt))
    ops._host_fault_word(dev).fill_(1)  # as a wait that gave up sets it
    with pytest.raises(ops._lib.ScgibError, match="hand-off"):
        ft(g, x, None, None, 1, None, 2, dev, 8)
    ops.clear_handoff_fault(dev)
    scores, *_ = ft(g, x, None, None, 1, None, 2, dev, 8)
    assert torch.isfinite(ft.loss(scores, tgt))

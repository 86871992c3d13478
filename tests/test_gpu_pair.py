"""The persistent encoder-pair forward (scgib_gin_pair_fwd, gin_pair.hip)
against the per-layer kernels it replaces (ops.PAIR_PERSISTENT off) and the
fp64 oracle: one launch must give the same losses, gradients, saved
activations and BatchNorm running statistics, in exact mode and in capacity
mode under HIP-graph replay, and never time out."""
import copy

import pytest
import torch

from conftest import check_grads_model, rel_err
from test_gpu_capacity import B, _batches, _model, _noise

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    return torch.device("cuda", 0)


def _run(pkg, model, g, x, noise, dev, persistent, monkeypatch):
    monkeypatch.setattr(pkg.ops, "PAIR_PERSISTENT", persistent)
    model.zero_grad(set_to_none=True)
    _, kl, con, rec = model(g, x, None, None, None, 1, None, 1, dev, B, noise=noise)
    (kl + rec + con).backward()
    torch.cuda.synchronize()
    return torch.stack([kl, con, rec]).detach()


@pytest.mark.parametrize("layers", [5, 4, 1])
def test_pair_forward_matches_per_layer(pkg, dev, layers, monkeypatch):
    gh = _batches(pkg, (21,))[0]
    g = gh.to(dev)
    n = g.num_nodes()
    noise = _noise(n, dev, 77)
    base = _model(pkg, dev, layers=layers)
    m_ref, m_new = copy.deepcopy(base), copy.deepcopy(base)
    calls = []
    orig = pkg.ops._pair_forward_persistent

    def counting(*a, **k):
        calls.append(1)
        return orig(*a, **k)

    monkeypatch.setattr(pkg.ops, "_pair_forward_persistent", counting)
    l_ref = _run(pkg, m_ref, g, g.ndata["x"], noise, dev, False, monkeypatch)
    assert not calls
    l_new = _run(pkg, m_new, g, g.ndata["x"], noise, dev, True, monkeypatch)
    assert calls, "the persistent path was not taken"
    assert pkg.ops.pair_sync_error(dev) == 0
    for a, b in zip(l_ref.tolist(), l_new.tolist()):
        assert rel_err(b, a) < 2e-5, (a, b)
    ref = {k: p.grad.detach().double().cpu() for k, p in m_ref.named_parameters()
           if p.grad is not None}
    mine = dict(m_new.named_parameters())
    assert set(ref) == {k for k, p in mine.items() if p.grad is not None}
    check_grads_model(ref, lambda k: mine[k].grad, tol=1e-3)
    bufs = dict(m_new.named_buffers())
    for k, v in m_ref.named_buffers():
        if "running" in k:
            assert rel_err(bufs[k].cpu(), v.cpu()) < 1e-5, k
        elif "num_batches" in k:
            assert int(bufs[k]) == int(v), k
    # the encoders' outputs themselves
    for attr in ("graph_features", "subgraphs_features"):
        a, b = getattr(m_ref, attr), getattr(m_new, attr)
        assert rel_err(b.detach().cpu(), a.detach().cpu()) < 1e-5, attr


def test_pair_forward_graph_replay(pkg, dev, monkeypatch):
    """Capacity mode + one captured step replayed over several batches: the
    persistent launch re-arms its counters itself (no memset node), the
    padded rows stay zero, and every replay equals the eager per-layer step."""
    hosts = _batches(pkg, (31, 32, 33))
    n_cap, e_cap, mgn, caps = pkg.graph.StaticBatch.capacities(hosts, 1, slack=1.05)
    static = pkg.graph.StaticBatch(B, n_cap, e_cap, 11, mgn, caps, dev)
    base = _model(pkg, dev)
    m_ref, m_cap = copy.deepcopy(base), copy.deepcopy(base)
    ug = torch.empty(n_cap, device=dev)
    uf = torch.empty(n_cap, 64, device=dev)
    monkeypatch.setattr(pkg.ops, "PAIR_PERSISTENT", True)
    calls = []
    orig = pkg.ops._pair_forward_persistent

    def counting(*a, **k):
        calls.append(1)
        return orig(*a, **k)

    monkeypatch.setattr(pkg.ops, "_pair_forward_persistent", counting)
    # warm-up off the capture
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        static.load(static.pad(hosts[0]))
        m_warm = copy.deepcopy(base)
        m_warm(static.graph, static.x, None, None, None, 1, None, 1, dev, B, noise=(ug, uf))
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    m_cap.zero_grad(set_to_none=True)
    with torch.cuda.graph(graph):
        _, kl, con, rec = m_cap(static.graph, static.x, None, None, None, 1, None, 1, dev, B,
                                noise=(ug, uf))
        (kl + rec + con).backward()
    assert len(calls) == 2, "the persistent path was not captured"
    for i, gh in enumerate(hosts):
        n = gh.num_nodes()
        nz = _noise(n_cap, dev, 500 + i)
        ug.copy_(nz[0])
        uf.copy_(nz[1])
        static.load(static.pad(gh))
        graph.replay()
        torch.cuda.synchronize()
        assert pkg.ops.pair_sync_error(dev) == 0
        g = gh.to(dev)
        l_ref = _run(pkg, m_ref, g, g.ndata["x"], (nz[0][:n], nz[1][:n]), dev, False, monkeypatch)
        for a, b in zip(l_ref.tolist(), [kl.item(), con.item(), rec.item()]):
            assert rel_err(b, a) < 2e-5, (i, a, b)
        ref = {k: p.grad.detach().double().cpu() for k, p in m_ref.named_parameters()
               if p.grad is not None}
        mine = dict(m_cap.named_parameters())
        check_grads_model(ref, lambda k: mine[k].grad, tol=1e-3)
        # the padded rows of Encoder1's output are zero
        assert torch.count_nonzero(m_cap.graph_features[n:]).item() == 0
        monkeypatch.setattr(pkg.ops, "PAIR_PERSISTENT", True)

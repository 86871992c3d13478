"""The fine-tune step at the BASELINE.json fine-tune configurations vs the
oracle.

The reference-golden fine-tune tests (test_gpu_parity.py) run B = 8 batches of
~9-atom molecules.  Here the step the fine-tune bench times runs at config
size, B = 32:

  * ogbg-molhiv (configs[4]): molhiv-like molecules (25.5 +- 8 atoms, F = 9),
    BCE on sigmoid scores (models.py:522-523, train_molhiv.py:107-152);
  * Mutagenicity (configs[0]'s shape): 30 +- 8 atoms, F = 14 one-hot, two
    classes, CE on sigmoid scores (models.py:527-530, train_tudataset.py:109-158)

with the shipped checkpoint's weights (the weights-only fixture) and the
reference's freezing quirk (models.py:424-434), in exact mode and as the
captured capacity-mode replay finetune_bench.py times, each against
oracle/scgib_ref.finetune_forward in float64 on the same explicit noise.

Bars (written here): scores and loss within 1e-4 relative; every trainable
gradient within 2e-3 per-tensor relative L2 (check_grads_model each_tol, plus
its concatenated 1e-3 and cosine 0.999); every BatchNorm running statistic the
step updates within 1e-4 relative; frozen parameters receive no gradient.
"""
import copy

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import check_grads_model, rel_err

pytestmark = pytest.mark.gpu

B = 32
TOL = 1e-4
EACH_TOL = 2e-3
CONFIGS = {  # id -> (workload, dataset, num_classes, loss)
    "molhiv_B32_bce": ("molhiv", "ogbg-molhiv", 1, "bce"),
    "mutag_B32_ce": ("mutagenicity", "Mutagenicity", 2, "ce"),
}


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    return torch.device("cuda", 0)


def _loss(kind, scores, targets):
    if kind == "bce":  # models.py:522-523
        return F.binary_cross_entropy(scores, targets)
    return F.cross_entropy(scores, targets.squeeze(-1))  # models.py:527-530


def _oracle(ft, gh, k, u_gate, u_feat, dataset, kind, targets):
    """float64 oracle step: scores, loss, the trainable gradients, the BN
    running statistics after the step (ego-nets from oracle/egonet_ref.c)."""
    from oracle import egonet
    from oracle import scgib_ref as R
    trainable = {n for n, p in ft.named_parameters() if p.requires_grad}
    p = {}
    for kk, v in ft.state_dict().items():
        t = v.detach().cpu().clone()
        if t.is_floating_point():
            t = t.double()
            if kk in trainable:
                t.requires_grad_(True)
        p[kk] = t
    buffers = {kk: v for kk, v in p.items() if "running" in kk or "num_batches" in kk}
    sizes, ecount, nodes, esrc, edst = egonet.egonets(gh.rowptr.numpy(), gh.col.numpy(), k)
    off = np.repeat(np.concatenate([[0], np.cumsum(sizes)[:-1]]), ecount)
    src, dst = gh.edges()
    batch = {"src": src, "dst": dst, "counts": torch.from_numpy(gh.batch_num_nodes_host())}
    ego = {"src": torch.from_numpy(esrc + off), "dst": torch.from_numpy(edst + off),
           "counts": torch.from_numpy(sizes)}
    x = F.normalize(gh.ndata["x"].double())
    scores = R.finetune_forward(p, batch, ego, x, x[torch.from_numpy(nodes)], u_gate.double(),
                                u_feat.double(), dataset, buffers)
    loss = _loss(kind, scores, targets.double() if kind == "bce" else targets)
    loss.backward()
    # (the head's own Encoder1 / Encoder2 / compressor exist for state_dict
    # parity only and get no gradient, in the reference as here)
    grads = {kk: p[kk].grad.numpy() for kk in trainable if p[kk].grad is not None}
    return {"scores": scores.detach(), "loss": loss.item(), "grads": grads,
            "buffers": {kk: v.clone() for kk, v in buffers.items()}}


@pytest.fixture(scope="module", params=list(CONFIGS))
def case(request, pkg, dev):
    import finetune_bench
    workload, dataset, ncls, kind = CONFIGS[request.param]
    F_in = pkg.synth.WORKLOADS[workload][2]
    ft, k = finetune_bench.make_finetune_model(pkg, F_in, B, dev, seed=5, dataset=dataset,
                                               num_classes=ncls)
    gh, _ = pkg.graph.collate_pyg(pkg.synth.molecules(B, workload, seed=41))
    other, _ = pkg.graph.collate_pyg(pkg.synth.molecules(B, workload, seed=42))
    n = gh.num_nodes()
    gen = torch.Generator().manual_seed(88)
    u_gate, u_feat = torch.rand(n, generator=gen), torch.rand(n, 64, generator=gen)
    if kind == "bce":
        targets = torch.randint(0, 2, (B, 1), generator=gen).float()
    else:
        targets = torch.randint(0, ncls, (B, 1), generator=gen)
    ref = _oracle(copy.deepcopy(ft).cpu(), gh, k, u_gate, u_feat, dataset, kind, targets)
    return dict(name=request.param, kind=kind, k=k, F_in=F_in, ft=ft, gh=gh, other=other,
                u_gate=u_gate, u_feat=u_feat, targets=targets, ref=ref)


def _check(c, ft, scores, loss):
    ref = c["ref"]
    assert rel_err(scores.detach().cpu(), ref["scores"]) < TOL, c["name"]
    assert rel_err(loss, ref["loss"]) < TOL, (c["name"], loss, ref["loss"])
    params = dict(ft.named_parameters())
    errs = check_grads_model(ref["grads"], lambda n: params[n].grad, each_tol=EACH_TOL)
    worst = max(errs.items(), key=lambda kv: kv[1])
    print(f"{c['name']}: {len(errs)} trainable tensors, worst grad rel-L2 {worst[0]} "
          f"{worst[1]:.2e}")
    assert all(p.grad is None for n, p in params.items() if n not in ref["grads"])
    bufs = dict(ft.named_buffers())
    moved = 0
    for kk, v in ref["buffers"].items():
        if "num_batches" in kk:
            assert int(bufs[kk]) == int(v), kk
        else:
            assert rel_err(bufs[kk].cpu(), v) < TOL, (kk, rel_err(bufs[kk].cpu(), v))
            moved += 1
    assert moved > 0


def test_finetune_config_exact_mode(pkg, dev, case):
    c = case
    ft = copy.deepcopy(c["ft"])
    g = c["gh"].to(dev)
    x = F.normalize(g.ndata["x"].float())
    ft.zero_grad(set_to_none=True)
    scores, *_ = ft(g, x, None, None, 1, None, 2, dev, B,
                    noise=(c["u_gate"].to(dev), c["u_feat"].to(dev)))
    loss = _loss(c["kind"], scores, c["targets"].to(dev))
    loss.backward()
    torch.cuda.synchronize()
    _check(c, ft, scores, loss.item())


def test_finetune_config_graph_replay(pkg, dev, case):
    """The bench's launch path (finetune_bench.py): capacity-sized static
    buffers over this batch and another one, the batch loaded from a resident
    pool inside the graph, forward + loss + backward captured once and
    replayed on this batch."""
    c = case
    ft = copy.deepcopy(c["ft"])
    k, F_in = c["k"], c["F_in"]
    hosts = [c["other"], c["gh"]]
    n_cap, e_cap, mgn, caps = pkg.graph.StaticBatch.capacities(hosts, k, slack=1.02)
    static = pkg.graph.StaticBatch(B, n_cap, e_cap, F_in, mgn, caps, dev, k=k)
    padded = []
    for gh in hosts:
        gx = pkg.graph.GraphBatch.from_edges(*[t.numpy() for t in gh.edges()], gh.num_nodes(),
                                             True, gh.batch_num_nodes_host())
        dict.__setitem__(gx.ndata, "x", F.normalize(gh.ndata["x"].float()))
        padded.append(static.pad(gx))
    pool = static.pool(padded)
    s_ug = torch.zeros(n_cap, device=dev)
    s_uf = torch.zeros(n_cap, 64, device=dev)
    tg = c["targets"].to(dev)

    def body():
        static.load_next(pool)
        scores, *_ = ft(static.graph, static.x, None, None, 1, None, 2, dev, B,
                        noise=(s_ug, s_uf))
        loss = _loss(c["kind"], scores, tg)
        loss.backward()
        return scores.detach(), loss.detach()

    snap = copy.deepcopy(ft.state_dict())
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # warm-up on pool[0] (allocator)
        body()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    ft.load_state_dict(snap)  # undo the warm-up's running-stat updates
    ft.zero_grad(set_to_none=True)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        scores, loss = body()
    n = c["gh"].num_nodes()
    s_ug[:n].copy_(c["u_gate"])
    s_uf[:n].copy_(c["u_feat"])
    graph.replay()  # loads pool[1] = this batch (the warm-up took pool[0])
    torch.cuda.synchronize()
    assert pool["cursor"].tolist()[0] == 2
    _check(c, ft, scores, loss.item())


@pytest.mark.parametrize("agg_free", [False, True])
def test_frozen_layers_skip_weight_grads_bitwise(pkg, dev, case, agg_free, monkeypatch):
    """The frozen GIN layers' backward skips the weight products
    (scgib_gin_layer_bwd / _layer0_bwd need_w = 0): the
    trainable gradients (transfer_d through layer 0, ginlayers.2, the head)
    are bitwise those of the same step with every parameter trainable, and
    the frozen ones still get none.  agg_free: the agg-free layers forced on
    at this size (ops.AGG_FREE_MIN_ROWS = 0): a frozen layer runs
    scgib_gin_layer_bwd_z / scgib_gin_bwd_stats_z with need_w = 0."""
    if agg_free:
        monkeypatch.setattr(pkg.ops, "AGG_FREE_MIN_ROWS", 0)
    c = case
    g = c["gh"].to(dev)
    x = F.normalize(g.ndata["x"].float())
    noise = (c["u_gate"].to(dev), c["u_feat"].to(dev))
    out = []
    for unfreeze in (False, True):
        ft = copy.deepcopy(c["ft"])
        trainable = {n for n, p in ft.named_parameters() if p.requires_grad}
        if unfreeze:
            for p in ft.parameters():
                p.requires_grad_(True)
        scores, *_ = ft(g, x, None, None, 1, None, 2, dev, B, noise=noise)
        _loss(c["kind"], scores, c["targets"].to(dev)).backward()
        torch.cuda.synchronize()
        out.append((scores.detach(), {n: p.grad for n, p in ft.named_parameters()}, trainable))
    (sa, ga, tr), (sb, gb, _) = out
    assert torch.equal(sa, sb)
    assert {n for n, v in ga.items() if v is not None} <= tr
    checked = 0
    for n in tr:
        # a trainable tensor the all-trainable step gives a gradient must get
        # one with the freezing too (a dropped need_w slice would lose it)
        assert (ga[n] is None) == (gb[n] is None), n
        if gb[n] is not None:
            assert torch.equal(ga[n], gb[n]), n
            checked += 1
    assert checked > 0


@pytest.mark.parametrize("n,k,c,sig", [(32, 128, 1, True), (32, 128, 2, True), (1, 128, 1, True),
                                       (33, 64, 3, False), (100, 128, 1, True), (7, 12, 16, False),
                                       (5, 36, 2, True)])
def test_predict_head_and_bce_vs_torch(pkg, dev, n, k, c, sig):
    """csrc/head.hip against torch in float64: the head's output (and its
    sigmoid), every gradient, and the BCE loss and its gradient (the tail of
    Mainmodel_finetuning, models.py:510-523).  n = 100: backward row chunks
    of 32 with a partial last one; k = 12 / 36 / 64: dx column slices of the
    four backward workgroups that are empty / uneven / half width."""
    import torch.nn as nn
    gen = torch.Generator().manual_seed(n * 1000 + k + c)
    seq = nn.Sequential(nn.Linear(k, 64), nn.ReLU(), nn.Linear(64, c))
    x = torch.randn(n, k, generator=gen)
    up = torch.rand(n, c, generator=gen)
    tg = torch.randint(0, 2, (n, c), generator=gen).float()
    seq64 = copy.deepcopy(seq).double()
    x64 = x.double().requires_grad_(True)
    ref = seq64(x64)
    ref = torch.sigmoid(ref) if sig else ref
    (ref * up.double()).sum().backward()
    seqd = copy.deepcopy(seq).to(dev)
    xd = x.to(dev).requires_grad_(True)
    assert pkg.ops.predict_head_ok(xd, seqd)
    out = pkg.ops.predict_head(xd, seqd, sig)
    (out * up.to(dev)).sum().backward()
    assert rel_err(out.detach().cpu(), ref.detach()) < 1e-5
    assert rel_err(xd.grad.cpu(), x64.grad) < 1e-5
    for (na, pa), (_, pb) in zip(seqd.named_parameters(), seq64.named_parameters()):
        assert rel_err(pa.grad.cpu(), pb.grad) < 1e-5, na
    if sig:  # BCE on the scores
        s = out.detach().clamp(1e-6, 1 - 1e-6).requires_grad_(True)
        s64 = s.detach().cpu().double().requires_grad_(True)
        lr = F.binary_cross_entropy(s64, tg.double())
        lr.backward()
        l = pkg.ops.bce_mean(s, tg.to(dev))
        l.backward()
        assert rel_err(l.item(), lr.item()) < 1e-5
        assert rel_err(s.grad.cpu(), s64.grad) < 1e-4


def test_predict_head_empty_batch(pkg, dev):
    """an empty batch through the fused head — the forward
    returns [0, C], the backward zero weight gradients (as torch's head)."""
    import torch.nn as nn
    seq = nn.Sequential(nn.Linear(128, 64), nn.ReLU(), nn.Linear(64, 1)).to(dev)
    x = torch.zeros(0, 128, device=dev, requires_grad=True)
    out = pkg.ops.predict_head(x, seq, True)
    assert out.shape == (0, 1)
    out.sum().backward()
    torch.cuda.synchronize()
    assert x.grad.shape == (0, 128)
    for p in seq.parameters():
        assert p.grad is not None and float(p.grad.abs().max()) == 0.0


def test_predict_head_refuses_k_not_multiple_of_4(pkg, dev):
    """The head kernels stage float4 runs: K % 4 != 0 is not the fused head
    (predict_head_ok False: the model keeps torch's head) and the C-ABI
    refuses it loudly."""
    import torch.nn as nn
    seq = nn.Sequential(nn.Linear(9, 64), nn.ReLU(), nn.Linear(64, 1)).to(dev)
    x = torch.randn(4, 9, device=dev)
    assert not pkg.ops.predict_head_ok(x, seq)
    with pytest.raises(pkg._lib.ScgibError):
        pkg.ops.predict_head(x, seq, True)

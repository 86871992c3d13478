"""Two-lane replay of a captured step graph (ops.SplitGraph,
csrc/graph_split.hip; DESIGN.md §3 "Host enqueue").

The split must be invisible in the results: the same kernels with the same
launch parameters, one lane per captured chain, the cross-chain edges as
signal / wait kernels.  Checked three ways:
  * a toy two-stream graph of torch elementwise ops with two fork / join
    sections and a read of the main chain's data on the side chain, replayed
    50 times back to back (no host sync: cross-replay ordering included)
    against the closed-form values;
  * the bench's pretrain step (bench.build_replay_step) and the fine-tune
    step (finetune_bench.build_finetune_step), split and whole, from the same
    initial state and the same explicit noise: losses, every parameter, the
    Adam moments and the BatchNorm buffers bitwise equal after K replays
    (every reduction of the step is in a fixed order, so a whole replay and a
    split one are bit-for-bit the same computation).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    return torch.device("cuda", 0)


def test_split_toy_two_stream_graph(pkg, dev):
    if not pkg.ops.xq_enabled():
        pytest.skip(f"hand-offs off here: {pkg.ops.XQ_REASON}")
    n = 1 << 16
    a, b, c, d, e, f = (torch.zeros(n, device=dev) for _ in range(6))
    main = torch.cuda.Stream(dev)
    side = torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.stream(main):
        with torch.cuda.graph(g, stream=main):
            a.add_(1.0)                         # main
            side.wait_stream(main)              # fork 1
            with torch.cuda.stream(side):
                b.mul_(2.0).add_(a)             # side reads main's a
            torch.mul(a, 3.0, out=d)            # main, beside it
            main.wait_stream(side)              # join 1
            torch.add(b, d, out=c)
            side.wait_stream(main)              # fork 2
            with torch.cuda.stream(side):
                e.add_(c)
            f.add_(1.0)
            main.wait_stream(side)              # join 2
            c.add_(e)
    lanes = pkg.ops.SplitGraph(g, dev)
    info = lanes.info
    assert info["serialised"] == 0 and info["lane0_kernels"] and info["lane1_kernels"], info
    assert info["lane0_kernels"] + info["lane1_kernels"] == info["captured"], info
    assert info["handoffs"] >= 4, info  # two forks, two joins
    K = 50
    for _ in range(K):  # back to back: the next replay's lanes queue behind this one's
        lanes.replay()
    torch.cuda.synchronize()
    ea = eb = ec = ed = ee = ef = 0.0
    for _ in range(K):
        ea += 1.0
        eb = 2.0 * eb + ea
        ed = 3.0 * ea
        ec = eb + ed
        ee += ec
        ef += 1.0
        ec += ee
    # b doubles each replay: compare in relative terms (fp32 of exact integers
    # up to 2^24, then rounded the same way on both sides within 1 ulp chains)
    for t, v in ((a, ea), (d, ed), (f, ef)):
        assert torch.all(t == v), (t[0].item(), v)
    for t, v in ((b, eb), (c, ec), (e, ee)):
        assert torch.allclose(t, torch.full_like(t, v), rtol=1e-5), (t[0].item(), v)
    assert lanes.timeouts() == 0
    lanes.close()


def _state(model, opt):
    out = {n: p.detach().clone() for n, p in model.named_parameters()}
    out.update({"buf." + n: b.detach().clone() for n, b in model.named_buffers()})
    for n, p in model.named_parameters():
        st = opt.state.get(p)
        if st:
            for k, v in st.items():
                if torch.is_tensor(v):
                    out[f"opt.{n}.{k}"] = v.detach().clone()
    return out


def _assert_bitwise(sa, sb):
    assert sa.keys() == sb.keys()
    bad = [k for k in sa if not torch.equal(sa[k], sb[k])]
    assert not bad, bad[:10]


def test_split_pretrain_step_matches_whole_replay(pkg, dev):
    import bench
    from test_gpu_trajectory import _pretrain_model
    if not pkg.ops.xq_enabled():
        pytest.skip(f"hand-offs off here: {pkg.ops.XQ_REASON}")
    k, B, K, POOL = 1, 128, 6, 3
    F_in = pkg.synth.WORKLOADS["qm9"][2]
    hosts = [pkg.graph.collate_pyg(pkg.synth.molecules(B, "qm9", seed=30 + i))[0]
             for i in range(POOL)]
    n_cap = pkg.graph.StaticBatch.capacities(hosts, k, slack=1.02)[0]
    gen = torch.Generator().manual_seed(77)
    noise = [(torch.rand(n_cap, generator=gen), torch.rand(n_cap, 64, generator=gen))
             for _ in range(K)]
    runs = []
    for split in (False, True):
        model = _pretrain_model(pkg, F_in, k, B, dev)
        opt = pkg.optim.Adam(model.parameters(), lr=1e-4, weight_decay=5e-5)
        s_ug = torch.zeros(n_cap, device=dev)
        s_uf = torch.zeros(n_cap, 64, device=dev)
        rs = bench.build_replay_step(model, opt, hosts, k, B, dev, prefetch=True,
                                     noise=(s_ug, s_uf), split=split)
        assert (rs.split is not None) == split
        if split:
            assert rs.split.info["serialised"] == 0, rs.split.info
        losses = []
        for j in range(K):
            s_ug.copy_(noise[j][0])
            s_uf.copy_(noise[j][1])
            kl, rec, con = rs.step(j)
            losses.append(torch.stack([kl, rec, con]).clone())
        torch.cuda.synchronize()
        assert pkg.ops.xq_timeouts(dev) == 0
        runs.append((torch.stack(losses), _state(model, opt)))
        if rs.split is not None:
            rs.split.close()
    assert torch.equal(runs[0][0], runs[1][0]), (runs[0][0], runs[1][0])
    _assert_bitwise(runs[0][1], runs[1][1])


def test_noise_prefetch_matches_inline_draw(pkg, dev):
    """ops.NoisePrefetch: the bench's replayed step with its compression
    noise drawn one step ahead (by the step before's backward, at the end of
    the core chain) computes bitwise what the step drawing it at the head of
    its forward computes — the same Philox draws in the same order."""
    import bench
    from test_gpu_trajectory import _pretrain_model
    k, B, K, POOL = 1, 128, 6, 3
    F_in = pkg.synth.WORKLOADS["qm9"][2]
    hosts = [pkg.graph.collate_pyg(pkg.synth.molecules(B, "qm9", seed=40 + i))[0]
             for i in range(POOL)]
    runs = []
    for ahead in (False, True):
        model = _pretrain_model(pkg, F_in, k, B, dev)
        opt = pkg.optim.Adam(model.parameters(), lr=1e-4, weight_decay=5e-5)
        pkg.ops.seed_noise(dev, 2024)
        rs = bench.build_replay_step(model, opt, hosts, k, B, dev, prefetch=True,
                                     noise_prefetch=ahead)
        assert (rs.noise_prefetch is not None) == ahead
        losses = []
        for j in range(K):
            kl, rec, con = rs.step(j)
            losses.append(torch.stack([kl, rec, con]).clone())
        torch.cuda.synchronize()
        assert pkg.ops.xq_timeouts(dev) == 0
        runs.append((torch.stack(losses), _state(model, opt)))
        if rs.split is not None:
            rs.split.close()
    assert torch.isfinite(runs[0][0]).all()
    assert torch.equal(runs[0][0], runs[1][0]), (runs[0][0], runs[1][0])
    _assert_bitwise(runs[0][1], runs[1][1])


def test_split_finetune_step_matches_whole_replay(pkg, dev):
    import finetune_bench
    if not pkg.ops.xq_enabled():
        pytest.skip(f"hand-offs off here: {pkg.ops.XQ_REASON}")
    B, K, POOL = 32, 6, 3
    F_in = pkg.synth.WORKLOADS["molhiv"][2]
    hosts = [pkg.graph.collate_pyg(pkg.synth.molecules(B, "molhiv", seed=60 + i))[0]
             for i in range(POOL)]
    gen = torch.Generator().manual_seed(5)
    targets = [torch.randint(0, 2, (B, 1), generator=gen).float() for _ in range(POOL)]
    runs = []
    for split in (False, True):
        ft, k = finetune_bench.make_finetune_model(pkg, F_in, B, dev, seed=11)
        n_cap = pkg.graph.StaticBatch.capacities(hosts, k, slack=1.02)[0]
        if not runs:
            ng = torch.Generator().manual_seed(8)
            noise = [(torch.rand(n_cap, generator=ng), torch.rand(n_cap, 64, generator=ng))
                     for _ in range(K)]
        opt = pkg.optim.Adam(ft.parameters(), lr=1e-3, weight_decay=1e-5)
        s_ug = torch.zeros(n_cap, device=dev)
        s_uf = torch.zeros(n_cap, 64, device=dev)
        fs = finetune_bench.build_finetune_step(pkg, ft, opt, hosts, targets, k, B, dev,
                                                prefetch=True, noise=(s_ug, s_uf), split=split)
        assert (fs.split is not None) == split
        losses = []
        for j in range(K):
            s_ug.copy_(noise[j][0])
            s_uf.copy_(noise[j][1])
            fs.replay()
            losses.append(torch.cat([fs.loss.reshape(1), fs.scores.reshape(-1)]).clone())
        torch.cuda.synchronize()
        assert pkg.ops.xq_timeouts(dev) == 0
        runs.append((torch.stack(losses), _state(ft, opt)))
        if fs.split is not None:
            fs.split.close()
    assert torch.equal(runs[0][0], runs[1][0])
    _assert_bitwise(runs[0][1], runs[1][1])


def test_finetune_noise_prefetch_matches_inline_draw(pkg, dev):
    """The fine-tune step (frozen lower GIN layers, as finetune_bench builds
    it) with ops.NoisePrefetch computes bitwise what the inline draw gives."""
    import finetune_bench
    B, K, POOL = 32, 6, 3
    F_in = pkg.synth.WORKLOADS["molhiv"][2]
    hosts = [pkg.graph.collate_pyg(pkg.synth.molecules(B, "molhiv", seed=70 + i))[0]
             for i in range(POOL)]
    gen = torch.Generator().manual_seed(6)
    targets = [torch.randint(0, 2, (B, 1), generator=gen).float() for _ in range(POOL)]
    runs = []
    for ahead in (False, True):
        ft, k = finetune_bench.make_finetune_model(pkg, F_in, B, dev, seed=12)
        opt = pkg.optim.Adam(ft.parameters(), lr=1e-3, weight_decay=1e-5)
        pkg.ops.seed_noise(dev, 77)
        fs = finetune_bench.build_finetune_step(pkg, ft, opt, hosts, targets, k, B, dev,
                                                prefetch=True, noise_prefetch=ahead)
        assert (fs.noise_prefetch is not None) == ahead
        losses = []
        for _ in range(K):
            fs.replay()
            losses.append(torch.cat([fs.loss.reshape(1), fs.scores.reshape(-1)]).clone())
        torch.cuda.synchronize()
        assert pkg.ops.xq_timeouts(dev) == 0
        runs.append((torch.stack(losses), _state(ft, opt)))
        if fs.split is not None:
            fs.split.close()
    assert torch.isfinite(runs[0][0]).all()
    assert torch.equal(runs[0][0], runs[1][0]), (runs[0][0], runs[1][0])
    _assert_bitwise(runs[0][1], runs[1][1])


def test_fused_final_reduce_adam_matches_separate(pkg, dev, monkeypatch):
    """scgib_adam_step_reduce (ops.fuse_final_into_step): the bench's replayed
    step with the ego chain's final weight-gradient reduce and Adam in one
    launch computes bitwise what the two launches compute — losses, every
    parameter, Adam's moments and steps — over 6 replays."""
    import bench
    from test_gpu_trajectory import _pretrain_model
    k, B, K, POOL = 1, 128, 6, 3
    monkeypatch.setattr(pkg.ops, "FUSE_FINAL_MIN_SLABS", 0)  # (whatever the default gate)
    F_in = pkg.synth.WORKLOADS["qm9"][2]
    hosts = [pkg.graph.collate_pyg(pkg.synth.molecules(B, "qm9", seed=80 + i))[0]
             for i in range(POOL)]
    runs = []
    for fuse in (False, True):
        model = _pretrain_model(pkg, F_in, k, B, dev)
        opt = pkg.optim.Adam(model.parameters(), lr=1e-4, weight_decay=5e-5)
        pkg.ops.seed_noise(dev, 99)
        rs = bench.build_replay_step(model, opt, hosts, k, B, dev, prefetch=True, fuse_adam=fuse)
        assert not pkg.ops._FINAL_PENDING and not pkg.ops._FINAL_ARMED[0]
        losses = []
        for j in range(K):
            kl, rec, con = rs.step(j)
            losses.append(torch.stack([kl, rec, con]).clone())
        torch.cuda.synchronize()
        assert pkg.ops.xq_timeouts(dev) == 0
        runs.append((torch.stack(losses), _state(model, opt)))
        if rs.split is not None:
            rs.split.close()
    assert torch.isfinite(runs[0][0]).all()
    assert torch.equal(runs[0][0], runs[1][0]), (runs[0][0], runs[1][0])
    _assert_bitwise(runs[0][1], runs[1][1])

"""Multi-step trajectory parity of the replayed steps the benches time
(VERDICT r05 item 2).

Every other whole-step test compares ONE forward + backward (+ one Adam
update) with the oracle.  What compounds over steps — the resident pool's
cursor and the ego-nets prefetched one batch ahead, the BatchNorm running
statistics and ``num_batches_tracked``, Adam's moments, step count and bias
correction under capture — is checked here by running K replays of the
benches' own captured steps beside the float64 oracle (``oracle/scgib_ref.py``
+ ``torch.optim.Adam`` in float64) on the same batches and the same explicit
noise, fed through the steps' static noise buffers:

  * pretrain: ``bench.build_replay_step`` (exp_pretraining.py:290-333, the
    bench's configs[1] step: QM9 B512 k1, pool load + ego prefetch + forward
    + backward + Adam(1e-4, wd 5e-5) in ONE graph), K = 8 replays over a pool
    of 3 batches (the cursor wraps twice); and K = 4 replays of configs[2] /
    configs[3]'s per-GPU steps (molpcba B1024 k1, PCQM4Mv2 B2048 k2), whose
    ego layers take the agg-free backward and, at k = 2, the bitmap builder;
  * fine-tune: ``finetune_bench.build_finetune_step`` (train_molhiv.py:107-152,
    configs[4]: molhiv B32 from the shipped checkpoint, BCE, Adam(1e-3, wd
    1e-5)), K = 20 replays over a pool of 4 batches, then
    ``evaluate_network``'s eval-mode pass (train_molhiv.py:161-208: BatchNorm
    on the running estimates, noise still drawn) over a held-out labelled set
    of 8 batches, scored with ``metrics.eval_rocauc`` (metrics.py:18-37).

Lock-step (teacher-forced): before each replay the oracle takes the HIP
step's whole state — parameters, BatchNorm buffers, Adam moments and step
count — and runs the same step on the batch the pool cursor loads, with the
noise of that replay; after the replay every output and every piece of the
new state is compared.  Every comparison is thus one step from identical
state, so the single-step bars hold at step 20 as at step 1, and any
misalignment that builds up over replays (cursor, prefetched ego-nets, a
running statistic, Adam's state under capture) shows at the step it happens.
The eval pass runs both sides on the HIP model's state after the K steps.

Free-running: a second oracle steps on its own from the first state.  fp32
and fp64 trajectories separate — Adam gives a parameter whose gradient is a
few rows' ReLU-tie contributions (a nearly dead unit) a whole +-lr step either
way, and the fine-tune's lr 1e-3 on 32-molecule batches grows that drift
~1.6x per step (measured: scores 1e-7 at steps 1-2, 1e-4 at step 5, 3e-2 at
step 20) — so its per-step distance is printed as the measured drift; the
pretrain run (lr 1e-4, 8 steps) is held to the 1e-4 loss bar free-running too.

Bars (written here): losses and scores within 1e-4 relative (north star);
parameters within 2e-3 per-tensor relative L2; the step's update (theta_new -
theta_old) of the well-conditioned elements within 2e-2 (COND below); the
gradient each Adam took (from its first moment) within 1e-2 per tensor of >=
4096 elements, cosine 0.999 on every tensor and 3e-3 over all tensors
together (ReLU-tie bars: GRAD_TOL's note); the second moment within 2e-3 per
tensor of >= 4096 elements, 5e-3 per smaller one; both moments within 1e-3
over all tensors together; every BatchNorm running statistic within 1e-4
relative; num_batches_tracked and Adam's step exact; the eval ROC-AUC within
1e-6 of the oracle's, widened only by the pairs whose oracle scores lie within
the score tolerance of each other (a swap there is a tie of two correct fp32
evaluations, counted and printed).  The gradients whose true value is zero
(conftest.CANCELLED: biases feeding a train-mode BatchNorm and the attention
logit's bias; the z-bar half of its weight) hold only rounding noise on both
sides, which Adam normalises to +-lr steps: their parameters and moments are
not compared, only that they stay finite.
"""
from types import SimpleNamespace

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import CANCELLED, rel_err, rel_l2

pytestmark = pytest.mark.gpu

LOSS_TOL = 1e-4
SCORE_TOL = 1e-4
PARAM_TOL = 2e-3
# the gradient each side's Adam took in the step, g = (m_new - beta1 m_old) /
# (1 - beta1) from the moments (m_old: the shared state before the step): per
# tensor within 2e-3 relative L2 — the config-size single-step bar
# (test_gpu_config_parity EACH_TOL).  The first moment itself moves by
# (1 - beta1) g, measured against an m that is ~10x smaller than g where the
# gradient's sign alternates between batches (measured 3.2e-3 on a 4096-element
# fine-tune weight whose gradient matched to 3e-4), so the moments are held
# per tensor only where they are the better-conditioned quantity (exp_avg_sq,
# MOMENT_TOL) and together (MOMENT_TOL_ALL, every tensor concatenated)
# The gradient each Adam took is held to bars for ReLU-tie noise, not for
# rounding: a hidden unit whose pre-activation sits within rounding of 0 for a
# row decides differently in two correct fp32 evaluations, moving that
# layer's weight gradients by one row's contribution — at the fine-tune's 32
# molecules, where only ginlayers.2 trains, by up to 6.1e-3 per tensor and
# 1.8e-3 over all tensors in one step (measured, step 1; the pretrain step at
# B512: 1.4e-3 over all tensors).  The single-step config tests hold fixed
# seeds to 2e-3; here 28 steps of fresh parameters sample many more ties.
# A structural error (a misaligned batch, a stale BatchNorm record, a wrong
# Adam state) moves a gradient by O(1) and its cosine far below 0.999.
GRAD_TOL = 1e-2
GRAD_TOL_SMALL = None  # (under BIG elements: the cosine and the concatenation only)
GRAD_TOL_ALL = 3e-3
COS_MIN = 0.999
MOMENT_TOL = 2e-3
# a tensor under BIG elements (the 64-element biases, BatchNorm affines): one
# row's ReLU-tie decision moves its gradient by a few 1e-3 at the fine-tune's
# 32 molecules (measured 2.96e-3, step 1, Encoder1.ginlayers.2 mlp.0.bias)
BIG = 4096
MOMENT_TOL_SMALL = 5e-3
MOMENT_TOL_ALL = 1e-3
# rel-L2 of one step's update over the well-conditioned elements (Adam's
# sqrt(v) >= COND of the tensor's largest): Adam gives every element a ~lr
# step whatever its gradient's size, so an element whose gradient is a
# handful of rows' ReLU-tie contributions has an update two correct fp32
# evaluations may set apart by its whole size
UPD_TOL = 2e-2
COND = 1e-2
BUF_TOL = 1e-4
AUC_TOL = 1e-6
HOT = ("transfer_d.", "MLP.", "model.Encoder", "model.compressor.", "model.attn_layer.")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    return torch.device("cuda", 0)


def _ego_inputs(gh, k):
    """Oracle batch / ego dicts of a host batch (ego-nets from oracle/egonet_ref.c)."""
    from oracle import egonet
    sizes, ecount, nodes, esrc, edst = egonet.egonets(gh.rowptr.numpy(), gh.col.numpy(), k)
    off = np.repeat(np.concatenate([[0], np.cumsum(sizes)[:-1]]), ecount)
    src, dst = gh.edges()
    batch = {"src": src, "dst": dst, "counts": torch.from_numpy(gh.batch_num_nodes_host())}
    ego = {"src": torch.from_numpy(esrc + off), "dst": torch.from_numpy(edst + off),
           "counts": torch.from_numpy(sizes)}
    x = F.normalize(gh.ndata["x"].double())
    return batch, ego, x, x[torch.from_numpy(nodes)]


def _snapshot(model, opt):
    """CPU copies of the HIP step's state: state_dict, and per parameter name
    Adam's (step, exp_avg, exp_avg_sq)."""
    torch.cuda.synchronize()
    sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    adam = {}
    for n, p in model.named_parameters():
        st = opt.state.get(p)
        if st:
            adam[n] = (float(st["step"]), st["exp_avg"].detach().cpu().clone(),
                       st["exp_avg_sq"].detach().cpu().clone())
    return sd, adam


class Oracle:
    """float64 leaves of the HIP optimizer's parameters (``names``; key_of
    maps a HIP name to the oracle's key), the BatchNorm buffers, and a float64
    torch Adam holding the HIP optimizer's state."""

    def __init__(self, snap, names, key_of, lr, wd, prefixes):
        sd, adam = snap
        self.names, self.key_of = names, key_of
        p = {}
        for kk, v in sd.items():
            if not kk.startswith(prefixes):
                continue
            t = v.clone()
            p[key_of(kk)] = t.double() if t.is_floating_point() else t
        leaves = []
        for n in names:
            p[key_of(n)].requires_grad_(True)
            leaves.append(p[key_of(n)])
        self.opt = torch.optim.Adam(leaves, lr=lr, weight_decay=wd)
        for n, t in zip(names, leaves):
            s, m, v = adam[n]
            self.opt.state[t] = {"step": torch.tensor(s, dtype=torch.float32),
                                 "exp_avg": m.double().clone(), "exp_avg_sq": v.double().clone()}
        self.p = p
        self.buffers = {kk: v for kk, v in p.items() if "running" in kk or "num_batches" in kk}


def _check_state(tag, snap0, snap1, orc, worst, prefixes):
    """The HIP state after a step (snap1) against the oracle's after the same
    step from the same state (snap0): parameters, the update, Adam's moments
    and step, the BatchNorm buffers.  Returns the failures, tracks the worst."""
    sd0, adam0 = snap0
    sd1, adam1 = snap1
    b1 = orc.opt.param_groups[0]["betas"][0]
    fails, tot = [], {}
    for n in orc.names:
        key = orc.key_of(n)
        mine, ref = sd1[n].double(), orc.p[key].detach()
        s_mine, m_mine, v_mine = adam1[n]
        rst = orc.opt.state[orc.p[key]]
        if int(s_mine) != int(float(rst["step"])):
            fails.append((n, "step", s_mine, float(rst["step"])))
        if not torch.isfinite(mine).all():
            fails.append((n, "finite"))
        if n.endswith(CANCELLED):
            continue  # rounding-noise gradients on both sides (module docstring)
        m_mine, v_mine = m_mine.double(), v_mine.double()
        m_ref, v_ref = rst["exp_avg"], rst["exp_avg_sq"]
        m_old = adam0[n][1].double()
        g_mine, g_ref = (m_mine - b1 * m_old) / (1 - b1), (m_ref - b1 * m_old) / (1 - b1)
        d_mine, d_ref = mine - sd0[n].double(), ref - sd0[n].double()
        if n.endswith("attn_layer.weight"):  # the z-bar half's gradient is ~0
            mine, ref, d_mine, d_ref = mine[:, 64:], ref[:, 64:], d_mine[:, 64:], d_ref[:, 64:]
            m_mine, v_mine, m_ref, v_ref = m_mine[:, 64:], v_mine[:, 64:], m_ref[:, 64:], v_ref[:, 64:]
            g_mine, g_ref = g_mine[:, 64:], g_ref[:, 64:]
        sv = v_ref.sqrt()
        cond = sv >= COND * sv.max()
        e = {"param": rel_l2(mine, ref), "update": rel_l2(d_mine[cond], d_ref[cond]),
             "grad": rel_l2(g_mine, g_ref), "exp_avg": rel_l2(m_mine, m_ref),
             "exp_avg_sq": rel_l2(v_mine, v_ref)}
        big = m_ref.numel() >= BIG
        mtol = MOMENT_TOL if big else MOMENT_TOL_SMALL
        for kk, bar in (("param", PARAM_TOL), ("update", UPD_TOL),
                        ("grad", GRAD_TOL if big else GRAD_TOL_SMALL), ("exp_avg", None),
                        ("exp_avg_sq", mtol)):
            worst[kk] = max(worst.get(kk, (0.0, "")), (e[kk], f"{n} @ {tag}"))
            if bar is not None and not e[kk] < bar:
                fails.append((n, kk, e[kk]))
        cos = float((g_mine * g_ref).sum() / max(float(g_mine.norm() * g_ref.norm()), 1e-300))
        worst["grad_cos_min"] = min(worst.get("grad_cos_min", (1.0, "")), (cos, f"{n} @ {tag}"))
        if cos < COS_MIN:
            fails.append((n, "grad cosine", cos))
        for kk, a, b in (("exp_avg", m_mine, m_ref), ("exp_avg_sq", v_mine, v_ref),
                         ("grad", g_mine, g_ref)):
            num, den = tot.get(kk, (0.0, 0.0))
            tot[kk] = (num + float(((a - b) ** 2).sum()), den + float((b ** 2).sum()))
    for kk, (num, den) in tot.items():
        e = (num / max(den, 1e-300)) ** 0.5
        worst[kk + "_all"] = max(worst.get(kk + "_all", (0.0, "")), (e, tag))
        if not e < (GRAD_TOL_ALL if kk == "grad" else MOMENT_TOL_ALL):
            fails.append(("all tensors", kk, e))
    nb = 0
    for kk, v in sd1.items():
        if not kk.startswith(prefixes) or not ("running" in kk or "num_batches" in kk):
            continue
        ref = orc.p[orc.key_of(kk)]
        if "num_batches" in kk:
            if int(v) != int(ref):
                fails.append((kk, "num_batches_tracked", int(v), int(ref)))
        else:
            err = rel_err(v, ref)
            worst["bn_buffer"] = max(worst.get("bn_buffer", (0.0, "")), (err, f"{kk} @ {tag}"))
            if not err < BUF_TOL:
                fails.append((kk, "running", err))
        nb += 1
    assert nb > 0
    return fails


def _lockstep(name, model, opt, replay, oracle_step, plan, names, key_of, lr, wd, prefixes):
    """Replay the captured step len(plan) times; before each replay an Oracle
    takes the HIP state and runs the same step (teacher-forced lock-step);
    returns the per-step HIP outputs, the first and the last state."""
    worst, fails, outs = {}, [], []
    snap = first = _snapshot(model, opt)
    for j, item in enumerate(plan):
        orc = Oracle(snap, names, key_of, lr, wd, prefixes)
        mine = replay(j, item)
        nxt = _snapshot(model, opt)
        ref = oracle_step(orc, item)
        checks = [("losses", mine["losses"], ref["losses"], LOSS_TOL)]
        if "scores" in mine:
            checks.append(("scores", mine["scores"], ref["scores"], SCORE_TOL))
        for kind, a, b, tol in checks:
            err = rel_err(a, b)
            worst[kind] = max(worst.get(kind, (0.0, "")), (err, f"step {j}"))
            if not err < tol:
                fails.append((j, kind, err))
        fails += [(j,) + f for f in _check_state(f"step {j}", snap, nxt, orc, worst, prefixes)]
        outs.append(mine)
        snap = nxt
    print(f"{name} lock-step over {len(plan)} replays, worst: " +
          ", ".join(f"{k} {v:.2e} ({t})" for k, (v, t) in sorted(worst.items())))
    assert not fails, (name, fails[:20])
    return outs, first, snap


# ---------------------------------------------------------------------------
# pretrain (configs[1])
# ---------------------------------------------------------------------------
K_PRE, POOL_PRE = 8, 3


def _pretrain_model(pkg, F_in, k, B, dev):
    """Mainmodel_continue (exp_pretraining.py:109-113), GIN-64x5, random init
    with non-trivial BN affine parameters."""
    args = SimpleNamespace(recons_type="adj", useAtt=1, readout_f="sum", d_transfer=32,
                           batch_size=B, gin_layers=5, task="graph_classification")
    torch.manual_seed(2025)
    inner = pkg.models.Mainmodel(args, F_in, 64, 4, 4, k, "GIN")
    model = pkg.models.Mainmodel_continue(args, F_in, 64, 4, 4, k, 1, inner, "GIN")
    with torch.no_grad():
        for n, p in model.named_parameters():
            if "batch_norms" in n or "compressor.1" in n:
                p.add_(0.2 * torch.randn_like(p))
    return model.to(dev).train()


@pytest.mark.parametrize("B_PRE,split,seed,wl,k,n_steps",
                         [(512, True, 70, "qm9", 1, K_PRE), (512, False, 70, "qm9", 1, K_PRE),
                          (128, True, 70, "qm9", 1, K_PRE), (128, False, 70, "qm9", 1, K_PRE),
                          (128, True, 30, "qm9", 1, K_PRE), (128, False, 30, "qm9", 1, K_PRE),
                          (1024, True, 50, "molpcba", 1, 4), (2048, True, 60, "pcqm4mv2", 2, 4)],
                         ids=["B512-lanes", "B512-whole", "B128-lanes", "B128-whole",
                              "B128-lanes-s30", "B128-whole-s30", "molpcba-B1024-aggfree",
                              "pcqm-B2048-k2-aggfree"])
def test_pretrain_trajectory_replayed(pkg, dev, B_PRE, split, seed, wl, k, n_steps):
    """(molpcba B1024 k1 and PCQM4Mv2 B2048 k2 = configs[2] / configs[3]'s
    per-GPU steps: their ego layers run above ops.AGG_FREE_MIN_ROWS, so the
    agg-free backward is on the replayed path, and k = 2 takes the bitmap
    ego builder)"""
    import bench
    from oracle import scgib_ref as R
    F_in = pkg.synth.WORKLOADS[wl][2]
    hosts = [pkg.graph.collate_pyg(pkg.synth.molecules(B_PRE, wl, seed=seed + i))[0]
             for i in range(POOL_PRE)]
    model = _pretrain_model(pkg, F_in, k, B_PRE, dev)
    opt = pkg.optim.Adam(model.parameters(), lr=1e-4, weight_decay=5e-5)
    n_cap = pkg.graph.StaticBatch.capacities(hosts, k, slack=1.02)[0]
    s_ug = torch.zeros(n_cap, device=dev)
    s_uf = torch.zeros(n_cap, 64, device=dev)
    rs = bench.build_replay_step(model, opt, hosts, k, B_PRE, dev, prefetch=True,
                                 noise=(s_ug, s_uf), split=split)
    assert (rs.split is not None) == (split and pkg.ops.xq_enabled())
    c0 = int(rs.pool["cursor"][0])
    assert c0 == 3  # the builder's three eager warm-up steps loaded pool[0..2]
    gen = torch.Generator().manual_seed(4242)
    plan = []
    if wl != "qm9":  # the agg-free layers are on this step's path
        n_ego = pkg.graph.StaticBatch.capacities(hosts, k, slack=1.02)[3][0]
        assert pkg.ops.AGG_FREE and n_ego >= pkg.ops.AGG_FREE_MIN_ROWS, n_ego
    for j in range(n_steps):
        b = (c0 + j) % POOL_PRE
        n = hosts[b].num_nodes()
        plan.append((b, torch.rand(n, generator=gen), torch.rand(n, 64, generator=gen)))
    inputs = {b: _ego_inputs(hosts[b], k) for b in range(POOL_PRE)}

    def replay(j, item):
        b, ug, uf = item
        n = len(ug)
        s_ug[:n].copy_(ug)
        s_uf[:n].copy_(uf)
        kl, rec, con = rs.step(j)
        return {"losses": [kl.item(), con.item(), rec.item()]}

    def oracle_step(orc, item):
        b, ug, uf = item
        batch, ego, x, xs = inputs[b]
        orc.opt.zero_grad(set_to_none=True)
        out = R.pretrain_forward(orc.p, batch, ego, x, xs, ug.double(), uf.double(), B_PRE,
                                 orc.buffers, dense_recon=False)
        out["loss_total"].backward()
        orc.opt.step()
        return {"losses": [out["loss_kl"].item(), out["loss_contrastive"].item(),
                           out["loss_recon"].item()]}

    # the HIP optimizer's parameters (those with Adam state) must all be oracle parameters
    names = [n for n, p in model.named_parameters() if p in opt.state]
    assert names and all(n.startswith(HOT) for n in names), names
    key_of = lambda kk: R.strip_continue({kk: 0}).popitem()[0]  # noqa: E731
    # (the wrapper's own Encoder1 / Encoder2 / compressor exist for state_dict
    # parity and stay untouched: only the HOT modules are the oracle's)
    outs, first, _ = _lockstep("pretrain", model, opt, replay, oracle_step, plan, names, key_of,
                               1e-4, 5e-5, HOT)
    assert int(rs.pool["cursor"][0]) == c0 + n_steps
    assert rs.prefetch.error() == 0 and rs.static.ego_error() == 0
    pkg.ops.check_handoff(dev)
    # free-running: the fp64 oracle's own trajectory from the first state
    orc = Oracle(first, names, key_of, 1e-4, 5e-5, HOT)
    drift = []
    for j, item in enumerate(plan):
        ref = oracle_step(orc, item)["losses"]
        drift.append(max(rel_err(a, r) for a, r in zip(outs[j]["losses"], ref)))
    print("pretrain free-running loss drift per step:", [f"{d:.1e}" for d in drift])
    assert max(drift) < LOSS_TOL, drift


# ---------------------------------------------------------------------------
# fine-tune (configs[4]) + evaluate_network
# ---------------------------------------------------------------------------
K_FT, POOL_FT, B_FT, EVAL_BATCHES = 20, 4, 32, 8


def test_finetune_trajectory_and_eval_rocauc(pkg, dev):
    import finetune_bench
    from oracle import scgib_ref as R
    F_in = pkg.synth.WORKLOADS["molhiv"][2]
    ft, k = finetune_bench.make_finetune_model(pkg, F_in, B_FT, dev, seed=9)
    hosts = [pkg.graph.collate_pyg(pkg.synth.molecules(B_FT, "molhiv", seed=900 + i))[0]
             for i in range(POOL_FT)]
    gen = torch.Generator().manual_seed(515)
    targets = [torch.randint(0, 2, (B_FT, 1), generator=gen).float() for _ in range(POOL_FT)]
    opt = pkg.optim.Adam(ft.parameters(), lr=1e-3, weight_decay=1e-5)
    n_cap = pkg.graph.StaticBatch.capacities(hosts, k, slack=1.02)[0]
    s_ug = torch.zeros(n_cap, device=dev)
    s_uf = torch.zeros(n_cap, 64, device=dev)
    fs = finetune_bench.build_finetune_step(pkg, ft, opt, hosts, targets, k, B_FT, dev,
                                            prefetch=True, noise=(s_ug, s_uf))
    c0 = int(fs.pool["cursor"][0])
    assert c0 == 3 and int(fs.targets[2][0]) == 3  # batch and target cursors in step
    plan = []
    for j in range(K_FT):
        b = (c0 + j) % POOL_FT
        n = hosts[b].num_nodes()
        plan.append((b, torch.rand(n, generator=gen), torch.rand(n, 64, generator=gen)))
    inputs = {b: _ego_inputs(hosts[b], k) for b in range(POOL_FT)}

    def replay(j, item):
        b, ug, uf = item
        n = len(ug)
        s_ug[:n].copy_(ug)
        s_uf[:n].copy_(uf)
        fs.replay()
        return {"losses": [fs.loss.item()], "scores": fs.scores.cpu().double()}

    def oracle_step(orc, item):
        b, ug, uf = item
        batch, ego, x, xs = inputs[b]
        orc.opt.zero_grad(set_to_none=True)
        scores = R.finetune_forward(orc.p, batch, ego, x, xs, ug.double(), uf.double(),
                                    "ogbg-molhiv", orc.buffers)
        loss = F.binary_cross_entropy(scores, targets[b].double())  # models.py:522-523
        loss.backward()
        orc.opt.step()
        return {"losses": [loss.item()], "scores": scores.detach()}

    names = [n for n, p in ft.named_parameters() if p in opt.state]
    trainable = {n for n, p in ft.named_parameters() if p.requires_grad}
    assert names and set(names) <= trainable, sorted(set(names) - trainable)
    key_of = lambda kk: kk  # noqa: E731 (the oracle takes the fine-tune model's own keys)
    outs, first, last = _lockstep("finetune", ft, opt, replay, oracle_step, plan, names, key_of,
                                  1e-3, 1e-5, ("",))
    assert int(fs.pool["cursor"][0]) == c0 + K_FT and int(fs.targets[2][0]) == c0 + K_FT
    assert fs.prefetch.error() == 0 and fs.static.ego_error() == 0
    pkg.ops.check_handoff(dev)
    orc = Oracle(first, names, key_of, 1e-3, 1e-5, ("",))
    drift = []
    for j, item in enumerate(plan):
        ref = oracle_step(orc, item)
        drift.append((rel_err(outs[j]["scores"], ref["scores"]),
                      rel_err(outs[j]["losses"], ref["losses"])))
    print("fine-tune free-running drift per step (scores, BCE):",
          [(f"{a:.1e}", f"{b:.1e}") for a, b in drift])

    # evaluate_network (train_molhiv.py:161-208): eval mode, no grad, a held-out
    # set; the oracle on the HIP model's state after the K steps
    orc = Oracle(last, names, key_of, 1e-3, 1e-5, ("",))
    ft.eval()
    ev_scores, ref_scores, labels = [], [], []
    egen = torch.Generator().manual_seed(616)
    with torch.no_grad():
        for i in range(EVAL_BATCHES):
            gh = pkg.graph.collate_pyg(pkg.synth.molecules(B_FT, "molhiv", seed=5000 + i))[0]
            n = gh.num_nodes()
            ug, uf = torch.rand(n, generator=egen), torch.rand(n, 64, generator=egen)
            y = torch.randint(0, 2, (B_FT, 1), generator=egen).float()
            g = gh.to(dev)
            x = F.normalize(g.ndata["x"].float())
            sc, *_ = ft(g, x, None, None, 1, None, 2, dev, B_FT, noise=(ug.to(dev), uf.to(dev)))
            batch, ego, xd, xs = _ego_inputs(gh, k)
            rs = R.finetune_forward(orc.p, batch, ego, xd, xs, ug.double(), uf.double(),
                                    "ogbg-molhiv", orc.buffers, training=False)
            ev_scores.append(sc.cpu().double())
            ref_scores.append(rs.detach())
            labels.append(y)
    pkg.ops.check_handoff(dev)
    mine, ref, y = torch.cat(ev_scores), torch.cat(ref_scores), torch.cat(labels)
    assert rel_err(mine, ref) < SCORE_TOL, rel_err(mine, ref)
    auc_mine = pkg.metrics.eval_rocauc(y, mine)["rocauc"]
    auc_ref = pkg.metrics.eval_rocauc(y, ref)["rocauc"]
    # positive / negative pairs whose oracle scores are within the score
    # tolerance: the only pairs two correct fp32 evaluations may order differently
    r, yy = ref[:, 0].numpy(), y[:, 0].numpy()
    pos, neg = r[yy == 1], r[yy == 0]
    close = int((np.abs(pos[:, None] - neg[None, :]) < SCORE_TOL * np.abs(r).max()).sum())
    bound = AUC_TOL + close / (len(pos) * len(neg))
    print(f"eval ROC-AUC: HIP {auc_mine:.9f} oracle {auc_ref:.9f} (|d| "
          f"{abs(auc_mine - auc_ref):.2e}, {close} near-tied pairs, bound {bound:.2e}); "
          f"score rel err {rel_err(mine, ref):.2e}")
    assert abs(auc_mine - auc_ref) <= bound
    # the eval pass leaves every BatchNorm running statistic as the training left it
    sd_now = {kk: v.detach().cpu() for kk, v in ft.state_dict().items()}
    for kk, v in last[0].items():
        if "running" in kk or "num_batches" in kk:
            assert torch.equal(sd_now[kk], v), kk

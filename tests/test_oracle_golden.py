"""The oracle (CPU restatement) against the goldens produced by the reference's
own models.py (oracle/gen_golden.py).  Pins the restatement before it is used
as the checker of the HIP path."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import FINETUNE_GOLDENS, MODEL_GOLDENS, check_grads, golden_logms, load_golden, rel_err, rel_l2
from oracle import scgib_ref as R


def golden_inputs(g):
    counts = torch.tensor(g["batch_num_nodes"])
    batch = {"src": torch.tensor(g["src"]), "dst": torch.tensor(g["dst"]), "counts": counts}
    ego = {"src": torch.tensor(g["ego_src"]), "dst": torch.tensor(g["ego_dst"]),
           "counts": torch.tensor(g["ego_batch_num_nodes"])}
    x_raw = torch.tensor(g["x_raw"]).float()
    x = F.normalize(x_raw)
    x_subs = F.normalize(x_raw[torch.tensor(g["ego_nodes_global"])])
    return batch, ego, x, x_subs


def golden_params(g):
    raw = {k[6:]: v for k, v in g.items() if k.startswith("param_")}
    return R.make_params(R.strip_continue(raw)), raw


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)


@pytest.mark.parametrize("name", MODEL_GOLDENS)
def test_oracle_matches_reference_golden(name):
    g = load_golden(name)
    batch, ego, x, x_subs = golden_inputs(g)
    params, raw = golden_params(g)
    buffers = {k: v.clone() for k, v in params.items() if "running" in k or "num_batches" in k}
    logms = golden_logms(g)
    out = R.pretrain_forward(params, batch, ego, x, x_subs, torch.tensor(g["u_gate"]),
                             torch.tensor(g["u_feat"]), int(g["chunk"]), buffers,
                             logms=None if logms is None else [torch.tensor(m) for m in logms],
                             kstep=int(g["k"]))
    for key in ("loss_kl", "loss_contrastive", "loss_recon", "loss_total"):
        assert rel(out[key].item(), g[key]) < 1e-5, key
    for key in ("graph_features", "subgraph_features", "noisy", "kl_tensor",
                "interaction_map", "graph_readout", "im_mlp"):
        assert rel(out[key].detach(), g["act_" + key]) < 1e-5, key
    out["loss_total"].backward()
    check_grads({k[5:]: v for k, v in g.items() if k.startswith("grad_")},
                lambda n: params[R.strip_continue({n: 0}).popitem()[0]].grad)
    for k, v in g.items():
        if k.startswith("after_"):
            assert np.allclose(buffers[R.strip_continue({k[6:]: 0}).popitem()[0]].numpy(), v,
                               rtol=1e-5, atol=1e-6), k


# ---------------------------------------------------------------------------
# Fine-tune head: oracle restatement vs the reference's Mainmodel_finetuning
# ---------------------------------------------------------------------------


def finetune_inputs(g):
    counts = torch.tensor(g["batch_num_nodes"])
    batch = {"src": torch.tensor(g["src"]), "dst": torch.tensor(g["dst"]), "counts": counts}
    ego = {"src": torch.tensor(g["ego_src"]), "dst": torch.tensor(g["ego_dst"]),
           "counts": torch.tensor(g["ego_batch_num_nodes"])}
    x = F.normalize(torch.tensor(g["x_raw"]).float())
    x_subs = x[torch.tensor(g["ego_nodes_global"])]
    return batch, ego, x, x_subs


@pytest.mark.parametrize("name", FINETUNE_GOLDENS)
def test_oracle_finetune_matches_reference(name):
    g = load_golden(name)
    batch, ego, x, x_subs = finetune_inputs(g)
    p = R.make_params({k[6:]: v for k, v in g.items() if k.startswith("param_")})
    buffers = {k: v.clone() for k, v in p.items() if "running" in k or "num_batches" in k}
    scores = R.finetune_forward(p, batch, ego, x, x_subs, torch.tensor(g["u_gate"]),
                                torch.tensor(g["u_feat"]), str(g["dataset"]), buffers)
    assert rel_err(scores.detach(), g["scores"]) < 1e-5
    t = torch.tensor(g["targets"])
    loss = (F.cross_entropy(scores, t.squeeze(-1)) if str(g["loss_kind"]) == "ce"
            else F.binary_cross_entropy(scores, t.float()))
    assert rel_err(loss.item(), g["loss"]) < 1e-5
    loss.backward()
    trainable = set(str(s) for s in g["trainable"])
    golden_grads = {k[5:]: v for k, v in g.items() if k.startswith("grad_")}
    assert set(golden_grads) <= trainable
    # frozen by the quirk: pretrained parameters outside "layers.2"
    assert not any(k.startswith("model.") and "layers.2" not in k for k in golden_grads)
    check_grads(golden_grads, lambda n_: p[n_].grad, tol=1e-4, metric="l2")


def test_oracle_domainadapt_matches_reference():
    """Mainmodel_domainadapt (models.py:107-355): X loss and every gradient."""
    g = load_golden("domainadapt_molhiv")
    batch, ego, x, x_subs = finetune_inputs(g)
    p = R.make_params({k[6:]: v for k, v in g.items() if k.startswith("param_")})
    buffers = {k: v.clone() for k, v in p.items() if "running" in k or "num_batches" in k}
    loss = R.domainadapt_forward(p, batch, ego, x, x_subs, torch.tensor(g["u_gate"]),
                                 torch.tensor(g["u_feat"]), buffers)
    assert rel_err(loss.item(), g["loss"]) < 1e-5
    loss.backward()
    golden_grads = {k[5:]: v for k, v in g.items() if k.startswith("grad_")}
    assert any(k.startswith("model.") for k in golden_grads)  # the pretrained model trains too
    assert any(k.startswith("s2s_rev.") for k in golden_grads)
    check_grads(golden_grads, lambda n_: p[n_].grad, tol=1e-4, metric="l2")


def test_oracle_finetune_after_domainadapt_matches_reference():
    """Fine-tuning on the adapted model runs the DA model's OWN extract_features
    (models.py:283, its freshly built encoders) — the reference's quirk."""
    g = load_golden("finetune_after_da_molhiv")
    batch, ego, x, x_subs = finetune_inputs(g)
    p = R.make_params({k[6:]: v for k, v in g.items() if k.startswith("param_")})
    buffers = {k: v.clone() for k, v in p.items() if "running" in k or "num_batches" in k}
    scores = R.finetune_forward(p, batch, ego, x, x_subs, torch.tensor(g["u_gate"]),
                                torch.tensor(g["u_feat"]), "ogbg-molhiv", buffers)
    assert rel_err(scores.detach(), g["scores"]) < 1e-5
    loss = F.binary_cross_entropy(scores, torch.tensor(g["targets"]).float())
    assert rel_err(loss.item(), g["loss"]) < 1e-5
    loss.backward()
    golden_grads = {k[5:]: v for k, v in g.items() if k.startswith("grad_")}
    check_grads(golden_grads, lambda n_: p[n_].grad, tol=1e-4, metric="l2")


def test_trans_logM_matches_reference_targets(pkg):
    """graph.trans_logM (restated util.getM_logM) == the reference's targets, bit-exact."""
    g = load_golden("pretrain_L4_k2_logm")
    k = int(g["k"])
    src, dst, counts = g["src"], g["dst"], g["batch_num_nodes"]
    gptr = np.concatenate([[0], np.cumsum(counts)])
    for i, want in enumerate(golden_logms(g)):
        m = (src >= gptr[i]) & (src < gptr[i + 1])
        gi = pkg.graph.GraphBatch.from_edges(src[m] - gptr[i], dst[m] - gptr[i], int(counts[i]),
                                             True)
        got = pkg.graph.trans_logM(gi, k).numpy()
        np.testing.assert_array_equal(got, want)


def test_oracle_recon_gram_form_equals_dense():
    """The Gram form of loss_recon_adj that the config-size oracle runs use
    above B = 512 (scgib_ref.pretrain_forward(dense_recon=False):
    (||IM^T IM||^2 - 2 sum_{(u,v) in E} <im_u, im_v> + |E|) / N) against the
    dense N x N restatement of models.py:762-768, in float64: loss and its
    gradient w.r.t. IM, on a 3000-node graph with directed edges (A != A^T)
    and self-loops — the restatement the large parity tests rely on."""
    import torch
    from oracle import scgib_ref as R
    gen = torch.Generator().manual_seed(3)
    n = 3000
    src = torch.randint(0, n, (9000,), generator=gen)
    dst = torch.randint(0, n, (9000,), generator=gen)
    pairs = sorted(set(zip(src.tolist(), dst.tolist())) | {(i, i) for i in range(0, n, 97)})
    src = torch.tensor([p[0] for p in pairs])
    dst = torch.tensor([p[1] for p in pairs])
    im = (0.2 * torch.randn(n, 64, generator=gen, dtype=torch.float64)).requires_grad_(True)
    dense = R.recon_adj_dense(im, src, dst)
    (gd,) = torch.autograd.grad(dense, im)
    g = im.t() @ im
    e = (im[src] * im[dst]).sum()
    gram = (torch.sum(g * g) - 2 * e + len(src)) / n
    (gg,) = torch.autograd.grad(gram, im)
    assert abs(gram.item() - dense.item()) <= 1e-10 * abs(dense.item())
    assert float((gg - gd).abs().max()) <= 1e-10 * float(gd.abs().max())

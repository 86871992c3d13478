"""CPU restatement of the S-CGIB pretrain hot path (torch fp32, literal semantics).

TEST INFRASTRUCTURE ONLY: imported by ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg, never by the product path.

It restates, in its own code, what ``/root/reference/models.py`` computes, and
keeps the reference's *structure* (per-graph Python loops, dense N x N
reconstruction) so it doubles as the "reference CPU path" baseline:

  GIN / GINConv / MLP ............ models.py:38-72  (+ DGL GINConv, eps buffer)
  transfer_d on x and x_subs ...... models.py:668-669, 1164-1165
  sum_nodes readouts .............. models.py:714-716, 724-726
  compress / compression .......... models.py:595-604, 631-660
  attention interaction ........... models.py:729-749
  MLP on the interaction map ...... models.py:676, 1174
  KL mean ......................... models.py:679
  batched_semi_loss / sim ......... models.py:606-629
  loss_recon_adj .................. models.py:762-768
  forward (A13) / continue (A14) .. models.py:662-700, 1158-1195

Quirks kept on purpose: per-graph compressor BatchNorm (one
running-stat update per graph), uniform noise, only the last graph's KL,
z-bar term of the attention logit included (it cancels in the softmax).

Randomness is explicit: ``u_gate`` [N] and ``u_feat`` [N, 64] replace the
reference's ``torch.rand(n_i, 1)`` / ``torch.rand_like`` draws per graph, in
the same order (models.py:599, 650).

Parameters are a dict keyed like ``Mainmodel.state_dict()`` (``model.``
prefixes of the ``Mainmodel_continue`` wrapper stripped by
``strip_continue``).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

BN_EPS = 1e-5
BN_MOMENTUM = 0.1
KL_EPS = 1e-7


def strip_continue(params):
    """Map Mainmodel_continue keys onto Mainmodel keys (A14 == A13 math)."""
    return {(k[6:] if k.startswith("model.") else k): v for k, v in params.items()}


def _linear(x, p, name, bias=True):
    w = p[name + ".weight"]
    b = p.get(name + ".bias") if bias else None
    return F.linear(x, w, b)


def _batchnorm_train(x, p, name, buffers, training=True):
    """nn.BatchNorm1d in train mode (torch's own batch_norm kernel, as the
    reference): batch stats for the output, unbiased var into the running
    estimate, momentum 0.1, eps 1e-5.  training False: eval mode (the running
    estimates normalise, nothing is updated), as evaluate_network's
    model.eval() (train_molhiv.py:161-162) runs every BatchNorm."""
    if not training:
        return F.batch_norm(x, buffers[name + ".running_mean"], buffers[name + ".running_var"],
                            p[name + ".weight"], p[name + ".bias"], False, BN_MOMENTUM, BN_EPS)
    if x.shape[0] <= 1:
        raise ValueError("Expected more than 1 value per channel when training")
    if buffers is not None:
        rm, rv = buffers[name + ".running_mean"], buffers[name + ".running_var"]
        buffers[name + ".num_batches_tracked"] += 1
    else:
        rm = rv = None
    return F.batch_norm(x, rm, rv, p[name + ".weight"], p[name + ".bias"], True,
                        BN_MOMENTUM, BN_EPS)


def _relu(x, mask, tie):
    """ReLU; with `mask` (the implementation under test's own decisions), the
    elements within `tie` of 0 — where an fp32 implementation may decide
    either way — follow the mask (x passes, or 0), all others the sign."""
    if mask is None:
        return F.relu(x)
    amb = x.abs() < tie
    return torch.where(amb, x * mask.to(x.dtype), F.relu(x))


def gin_encoder(p, prefix, src, dst, h, buffers, num_layers, relu_masks=None, tie=1e-5,
                training=True):
    """GIN.forward with DGL GINConv semantics (sum aggregation, (1+eps)*h).
    relu_masks (test use): per layer (hidden ReLU mask, output ReLU mask) of
    the fp32 implementation under test, applied only at pre-activations
    within `tie` of 0 (_relu), so that a gradient comparison is not decided
    by which way a rounding-level pre-activation fell."""
    for i in range(num_layers):
        lp = f"{prefix}.ginlayers.{i}"
        neigh = torch.zeros_like(h).index_add(0, dst, h[src])
        eps = p.get(lp + ".eps", torch.zeros(1))
        rst = (1 + eps) * h + neigh
        m1, m2 = relu_masks[i] if relu_masks is not None else (None, None)
        z = _relu(_linear(rst, p, lp + ".apply_func.mlp.0"), m1, tie)
        z = _linear(z, p, lp + ".apply_func.mlp.2")
        z = _batchnorm_train(z, p, f"{prefix}.batch_norms.{i}", buffers, training)
        h = _relu(z, m2, tie)
    return h


def num_gin_layers(p, prefix="Encoder1"):
    i = 0
    while f"{prefix}.ginlayers.{i}.apply_func.mlp.0.weight" in p:
        i += 1
    return i


def sum_nodes(x, counts):
    seg = torch.repeat_interleave(torch.arange(len(counts)), counts)
    return torch.zeros(len(counts), x.shape[1], dtype=x.dtype).index_add(0, seg, x)


def compression(p, graph_features, counts, u_gate, u_feat, buffers, training=True):
    """Per-graph loop of models.py:631-660 with explicit noise."""
    noisy_all, p_all, kl_all = [], [], None
    off = 0
    for n_i in counts.tolist():
        feats = graph_features[off:off + n_i]
        # compress(): compressor = Linear-BN-ReLU-Linear (models.py:589-596)
        t = _linear(feats, p, "compressor.0")
        t = _batchnorm_train(t, p, "compressor.1", buffers, training)
        pv = _linear(F.relu(t), p, "compressor.3")
        bias = 0.0 + 0.0001
        eps = (bias - (1 - bias)) * u_gate[off:off + n_i].reshape(-1, 1) + (1 - bias)
        gate = torch.log(eps) - torch.log(1 - eps)
        lam = torch.sigmoid((gate + pv) / 1.0).squeeze().reshape(-1, 1)
        lam_neg = 1 - lam
        static = feats.clone().detach()
        std, mean = torch.std_mean(static, dim=0)
        noisy_mean = lam * feats + lam_neg * mean
        noisy_std = lam_neg * std
        noisy = noisy_mean + u_feat[off:off + n_i] * noisy_std
        noisy_all.append(noisy)
        p_all.append(pv)
        kl = 0.5 * ((noisy_std ** 2) / (std + KL_EPS) ** 2) + torch.sum(
            ((noisy_mean - mean) / (std + KL_EPS)) ** 2, dim=0)
        kl_all = torch.cat((kl, kl), 0)  # only the last graph survives (models.py:659)
        off += n_i
    return torch.cat(noisy_all, 0), torch.cat(p_all, 0), kl_all


def attention(p, noisy, sub_readout, counts):
    """models.py:729-749 (readout == 'sum', useAtt == 1)."""
    zbar = sum_nodes(noisy, counts)
    outs, off = [], 0
    for i, n_i in enumerate(counts.tolist()):
        s_i = sub_readout[off:off + n_i]
        inter = torch.cat((zbar[i].repeat(n_i, 1), s_i), -1)
        logits = _linear(inter, p, "attn_layer")
        alpha = F.softmax(logits, dim=0)
        outs.append(s_i * alpha)
        off += n_i
    return torch.cat((noisy, torch.cat(outs, 0)), -1)


def semi_loss(z1, z2, chunk):
    """batched_semi_loss with tau = 1 (models.py:606-629)."""
    n = z1.shape[0]
    nb = (n - 1) // chunk + 1
    z1n, z2n = F.normalize(z1), F.normalize(z2)
    losses = []
    for i in range(nb):
        a, b = i * chunk, min((i + 1) * chunk, n)
        refl = torch.exp(z1n[a:b] @ z1n.t())
        betw = torch.exp(z1n[a:b] @ z2n.t())
        losses.append(-torch.log(betw[:, a:b].diag() /
                                 (refl.sum(1) + betw.sum(1) - refl[:, a:b].diag())))
    return torch.cat(losses).mean()


def recon_adj_dense(im, src, dst):
    """Dense N x N restatement of loss_recon_adj (models.py:762-768)."""
    n = im.shape[0]
    adj = torch.zeros(n, n).index_put_((src, dst), torch.ones(len(src)), accumulate=True)
    return torch.sum((im @ im.t() - adj) ** 2) / n


def recon_logm(im, logms, counts, kstep):
    """loss_recon (models.py:770-782), literally: per molecule h = X X^T and
    sum over the k targets of sum((h - logM_i)^2) / (n^2), then / k."""
    loss = 0
    for X, L in zip(torch.split(im, tuple(int(c) for c in counts)), logms):
        h = X @ X.t()
        n = h.shape[0]
        for i in range(kstep):
            loss = loss + torch.sum((h - L[i]) ** 2) / (n * n)
    return loss / kstep


def extract_features(p, batch, ego, h0, hs0, u_gate, u_feat, buffers, training=True):
    L = num_gin_layers(p)
    gf = gin_encoder(p, "Encoder1", batch["src"], batch["dst"], h0, buffers, L, training=training)
    sf = gin_encoder(p, "Encoder2", ego["src"], ego["dst"], hs0, buffers, L, training=training)
    readout = sum_nodes(gf, batch["counts"])
    noisy, _, kl_tensor = compression(p, gf, batch["counts"], u_gate, u_feat, buffers, training)
    sub_readout = sum_nodes(sf, ego["counts"])
    im = attention(p, noisy, sub_readout, batch["counts"])
    return {"graph_features": gf, "subgraph_features": sf, "graph_readout": readout,
            "noisy": noisy, "kl_tensor": kl_tensor, "interaction_map": im}


def pretrain_forward(p, batch, ego, x, x_subs, u_gate, u_feat, chunk, buffers=None,
                     dense_recon=True, logms=None, kstep=None):
    """Mainmodel.forward (A13) == Mainmodel_continue.forward (A14).

    ``x`` / ``x_subs`` are the already-normalised features, as the training loop
    passes them (exp_pretraining.py:312-314).  Returns a dict with the three
    losses, their sum and the intermediate activations.
    """
    h0 = _linear(x, p, "transfer_d", bias=False)
    hs0 = _linear(x_subs, p, "transfer_d", bias=False)
    acts = extract_features(p, batch, ego, h0, hs0, u_gate, u_feat, buffers)
    im = _linear(F.relu(_linear(acts["interaction_map"], p, "MLP.0")), p, "MLP.2")
    kl = torch.mean(acts["kl_tensor"])
    z1 = sum_nodes(acts["noisy"], batch["counts"])
    con = semi_loss(z1, acts["graph_readout"], chunk)
    if logms is not None:  # recons_type == 'logM'
        rec = recon_logm(im, logms, batch["counts"], kstep)
    elif dense_recon:
        rec = recon_adj_dense(im, batch["src"], batch["dst"])
    else:  # Gram form (exact restatement, used for large oracle runs)
        g = im.t() @ im
        e = (im[batch["src"]] * im[batch["dst"]]).sum()
        rec = (torch.sum(g * g) - 2 * e + len(batch["src"])) / im.shape[0]
    acts.update(im_mlp=im, loss_kl=kl, loss_contrastive=con, loss_recon=rec,
                loss_total=kl + rec + con)
    return acts


def make_params(arrays, requires_grad=True):
    """Tensors (fp32 leaf params, int buffers) from a fixture's ``param_*``."""
    out = {}
    for k, v in arrays.items():
        t = torch.tensor(v)
        if t.is_floating_point() and "running" not in k and not k.endswith(".eps"):
            t.requires_grad_(requires_grad)
        out[k] = t
    return out


# ---------------------------------------------------------------------------
# Fine-tune head: Mainmodel_finetuning, models.py:358-543
# ---------------------------------------------------------------------------
FINETUNE_TASKS = ("ZINC", "Peptides-struct", "FreeSolv", "ESOL")  # models.py:384


def set2set(p, prefix, feat, counts, n_iters=2):
    """DGL Set2Set(d, n_iters, 1) (models.py:565 / :362): LSTM(2d -> d) on
    q_star, per-graph softmax attention, readout = sum(alpha * feat);
    q_star = [q || readout].  Functional single-layer LSTM, PyTorch gate order
    (i, f, g, o)."""
    B, d = len(counts), feat.shape[1]
    seg = torch.repeat_interleave(torch.arange(B), counts)
    w_ih, w_hh = p[prefix + ".lstm.weight_ih_l0"], p[prefix + ".lstm.weight_hh_l0"]
    b = p[prefix + ".lstm.bias_ih_l0"] + p[prefix + ".lstm.bias_hh_l0"]
    hx = feat.new_zeros(B, d)
    cx = feat.new_zeros(B, d)
    q_star = feat.new_zeros(B, 2 * d)
    for _ in range(n_iters):
        gates = q_star @ w_ih.t() + hx @ w_hh.t() + b
        i, f, g, o = gates.chunk(4, dim=1)
        cx = torch.sigmoid(f) * cx + torch.sigmoid(i) * torch.tanh(g)
        hx = torch.sigmoid(o) * torch.tanh(cx)
        q = hx
        e = (feat * q[seg]).sum(dim=-1)
        emax = torch.stack([e[seg == k].max() for k in range(B)])
        a = torch.exp(e - emax[seg])
        den = torch.zeros(B, dtype=feat.dtype).index_add(0, seg, a)
        alpha = (a / den[seg]).unsqueeze(-1)
        readout = sum_nodes(feat * alpha, counts)
        q_star = torch.cat([q, readout], dim=-1)
    return q_star


def domainadapt_forward(p, batch, ego, x, x_subs, u_gate, u_feat, buffers=None):
    """Mainmodel_domainadapt.forward (models.py:256-275): own transfer_d -> the
    pretrained model's extract_features ("model." prefix: a Mainmodel_continue
    runs its wrapper-level encoders) -> own MLP -> Set2Set -> r_transfer_d,
    against s2s_rev(raw normalised features); loss_X = sum of squared
    differences (models.py:277-282)."""
    h0 = _linear(x, p, "transfer_d", bias=False)
    hs0 = _linear(x_subs, p, "transfer_d", bias=False)
    pre = {k[6:]: v for k, v in p.items() if k.startswith("model.")}
    bufs = None if buffers is None else {k[6:]: v for k, v in buffers.items()
                                         if k.startswith("model.")}
    acts = extract_features(pre, batch, ego, h0, hs0, u_gate, u_feat, bufs)
    im = _linear(F.relu(_linear(acts["interaction_map"], p, "MLP.0")), p, "MLP.2")
    g = set2set(p, "s2s", im, batch["counts"])
    rec = _linear(F.relu(_linear(g, p, "r_transfer_d.0")), p, "r_transfer_d.2")
    org = set2set(p, "s2s_rev", x, batch["counts"])
    return torch.sum((rec - org) ** 2)


def finetune_forward(p, batch, ego, x, x_subs, u_gate, u_feat, dataset, buffers=None,
                     training=True):
    """Mainmodel_finetuning.forward: own transfer_d -> the pretrained model's
    extract_features (its wrapper-level encoders, "model." prefix) -> own MLP
    -> Set2Set -> predict -> sigmoid (unless a regression dataset).  training
    False: evaluate_network's eval mode (train_molhiv.py:161-193) — every
    BatchNorm on its running estimates; the compression noise is still drawn
    (models.py:650 does not look at self.training)."""
    h0 = _linear(x, p, "transfer_d", bias=False)
    hs0 = _linear(x_subs, p, "transfer_d", bias=False)
    pre = {k[6:]: v for k, v in p.items() if k.startswith("model.")}
    bufs = None if buffers is None else {k[6:]: v for k, v in buffers.items()
                                         if k.startswith("model.")}
    acts = extract_features(pre, batch, ego, h0, hs0, u_gate, u_feat, bufs, training)
    im = _linear(F.relu(_linear(acts["interaction_map"], p, "MLP.0")), p, "MLP.2")
    g = set2set(p, "s2s", im, batch["counts"])
    scores = _linear(F.relu(_linear(g, p, "predict.0")), p, "predict.2")
    if dataset not in FINETUNE_TASKS:
        scores = torch.sigmoid(scores)
    return scores

"""Generate the golden fixtures under tests/golden/ from the REFERENCE's own code.

TEST INFRASTRUCTURE ONLY.  Runs in the build container only (it needs
``/root/reference``); the fixtures it writes are plain ``.npz`` data (inputs,
explicit noise, parameters, activations, losses, gradients, index arrays) —
no reference source or bytecode is copied.

What runs from the reference (imported behind ``oracle/refshim.py``):
  * ``util.load_dgl_fromPyG``                       util.py:277-325
  * ``models.Mainmodel``  forward/backward          models.py:546-782
  * ``models.Mainmodel_continue`` forward/backward  models.py:1010-1276
  * ``models.Mainmodel_finetuning`` forward + loss  models.py:358-543
The DGL primitives underneath are the restatements in
``oracle/dgl_semantics.py`` (DGL itself is absent: parity at the DGL boundary
is unpinned).

Usage:  python -m oracle.gen_golden        (from the repo root)
"""
from __future__ import annotations

import importlib
import os
import sys
from itertools import chain
from types import SimpleNamespace

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)

from oracle import refshim  # noqa: E402
from oracle import dgl_semantics as D  # noqa: E402

synth = importlib.import_module("s-cgib_amd.synth")


# ---------------------------------------------------------------------------
def _edge_cases():
    """Hand-made PyG-style molecules for the ingest + ego-net fixtures."""
    cases = []
    # 0: ring of 6 with a tail (benzene + substituent)
    ring = [(i, (i + 1) % 6) for i in range(6)] + [(0, 6), (6, 7)]
    cases.append(ring)
    # 1: one-directional + duplicate bonds (to_bidirected must fix)
    cases.append([(0, 1), (1, 2), (1, 2), (2, 3), (3, 1)])
    # 2: self loop kept once
    cases.append([(0, 1), (1, 1), (1, 2)])
    # 3: star (high degree centre)
    cases.append([(0, i) for i in range(1, 9)])
    # 4: two atoms
    cases.append([(0, 1), (1, 0)])
    # 5: trailing isolated atom -> skipped by the reference (x has 4 rows)
    cases.append(("skip", [(0, 1), (1, 2)], 4))
    # 6: no bonds at all -> skipped
    cases.append(("skip", [], 1))
    # 7: leading isolated atom (id 0 unused) -> kept, node 0 isolated
    cases.append([(1, 2), (2, 3)])
    return cases


def gen_ingest_and_ego(util_mod):
    """A1 (load_dgl_fromPyG + skip rule) and A2 (khop_in_subgraph) fixtures."""
    rng = np.random.default_rng(7)
    mols = []
    for c in _edge_cases():
        if isinstance(c, tuple):
            _, bonds, n = c
        else:
            bonds, n = c, (max(max(a, b) for a, b in c) + 1)
        ei = np.array(bonds, dtype=np.int64).T.reshape(2, -1)
        mols.append((ei, rng.random((n, 3), dtype=np.float32)))
    mols += synth.molecules(6, "qm9", seed=11, F=3)
    out = {"num_mols": np.array(len(mols))}
    for i, (ei, x) in enumerate(mols):
        out[f"m{i}_edge_index"] = ei
        out[f"m{i}_x"] = x
        data = SimpleNamespace(edge_index=torch.from_numpy(ei), x=torch.from_numpy(x))
        try:
            g = util_mod.load_dgl_fromPyG(data)  # the reference's own function
            kept = True
        except Exception:  # the reference's bare except (exp_pretraining.py:276)
            kept = False
        out[f"m{i}_kept"] = np.array(kept)
        if not kept:
            continue
        s, d = g.edges()
        out[f"m{i}_src"] = s.numpy()
        out[f"m{i}_dst"] = d.numpy()
        out[f"m{i}_n"] = np.array(g.num_nodes())
        for k in (1, 2, 3):
            sizes, nodes, es, ed, ecount = [], [], [], [], []
            for v in g.nodes():  # exp_pretraining.py:269-272
                sg = D.khop_in_subgraph(g, v, k=k)[0]
                ids = sg.ndata["_ID"].numpy()
                sizes.append(len(ids))
                nodes.append(ids)
                a, b = sg.edges()
                es.append(a.numpy())
                ed.append(b.numpy())
                ecount.append(len(a))
            out[f"m{i}_k{k}_sizes"] = np.array(sizes, dtype=np.int64)
            out[f"m{i}_k{k}_nodes"] = np.concatenate(nodes).astype(np.int64)
            out[f"m{i}_k{k}_ecount"] = np.array(ecount, dtype=np.int64)
            out[f"m{i}_k{k}_esrc"] = np.concatenate(es).astype(np.int64)
            out[f"m{i}_k{k}_edst"] = np.concatenate(ed).astype(np.int64)
    np.savez_compressed(os.path.join(OUT, "ingest_egonet.npz"), **out)
    print("wrote ingest_egonet.npz", len(mols), "molecules")


# ---------------------------------------------------------------------------
class _NoiseRecorder:
    """Records every torch.rand / torch.rand_like draw made inside forward."""

    def __init__(self):
        self.draws = []

    def __enter__(self):
        self._rand, self._rand_like = torch.rand, torch.rand_like

        def rand(*a, **k):
            t = self._rand(*a, **k)
            self.draws.append(t.detach().clone())
            return t

        def rand_like(x, *a, **k):
            t = self._rand_like(x, *a, **k)
            self.draws.append(t.detach().clone())
            return t

        torch.rand, torch.rand_like = rand, rand_like
        return self

    def __exit__(self, *exc):
        torch.rand, torch.rand_like = self._rand, self._rand_like


def _grow_gin(models, gin, layers):
    """The checkpoint/paper GIN has 5 GINConv layers; shipped code builds 4
    (models.py:57-58).  Append layers with the reference's own classes."""
    while len(gin.ginlayers) < layers:
        gin.ginlayers.append(models.GINConv(models.MLP(64, 64, 64), learn_eps=False))
        gin.batch_norms.append(torch.nn.BatchNorm1d(64))


def gen_model_golden(models, util_mod, name, *, workload, F, B, L, k, continue_wrapper,
                     chunk, seed, recons_type="adj"):
    torch.manual_seed(seed)
    mols = synth.molecules(B - 1, workload, seed=seed, mu=12.0, sigma=4.0, F=F)
    # always include the smallest legal molecule (2 atoms) in the middle
    x2 = np.random.default_rng(seed).random((2, F), dtype=np.float32)
    mols.insert(B // 2, (np.array([[0, 1], [1, 0]], dtype=np.int64), x2))

    graphs, subgraphs = [], []
    for ei, x in mols:
        g = util_mod.load_dgl_fromPyG(SimpleNamespace(edge_index=torch.from_numpy(ei),
                                                      x=torch.from_numpy(x)))
        graphs.append(g)
        subgraphs.append([D.khop_in_subgraph(g, v, k=k)[0] for v in g.nodes()])
    batch_g = D.batch(graphs)                                          # molecules.py:359
    ego_g = D.batch(list(chain.from_iterable(subgraphs)))             # exp_pretraining.py:308-309
    batch_x = F_normalize(batch_g.ndata["x"].float())                  # exp_pretraining.py:312
    x_subs = F_normalize(ego_g.ndata["x"].float())                     # exp_pretraining.py:314

    args = SimpleNamespace(recons_type=recons_type, useAtt=1, readout_f="sum", d_transfer=32,
                           device="cpu", batch_size=chunk, task="graph_classification",
                           dataset="pre-train")
    batch_logMs = None
    if recons_type == "logM":
        # util.getM_logM (util.py:74-91) per molecule, as exp_tudataset.py:430-433 does
        batch_logMs = [torch.from_numpy(np.array(util_mod.getM_logM(g, kstep=k)[1])).float()
                       for g in graphs]
    inner = models.Mainmodel(args, F, hidden_dim=64, num_layers=4, num_heads=4,
                             k_transition=k, encoder="GIN")
    _grow_gin(models, inner.Encoder1, L)
    _grow_gin(models, inner.Encoder2, L)
    if continue_wrapper:
        real_load = models.torch.load
        models.torch.load = lambda *a, **kw: inner  # in-memory: nothing is unpickled
        try:
            model = models.Mainmodel_continue(args, F, hidden_dim=64, num_layers=4, num_heads=4,
                                              k_transition=k, num_classes=1, cp_filename="<mem>",
                                              encoder="GIN")
        finally:
            models.torch.load = real_load
    else:
        model = inner
    model.train()
    # perturb BN affine params so gamma/beta are exercised (defaults are 1/0)
    with torch.no_grad():
        for n_, p_ in model.named_parameters():
            if "batch_norms" in n_ or "compressor.1" in n_:
                p_.add_(0.1 * torch.randn_like(p_))

    acts = {}
    hooks = [inner.Encoder1.register_forward_hook(lambda m, i, o: acts.__setitem__("graph_features", o)),
             inner.Encoder2.register_forward_hook(lambda m, i, o: acts.__setitem__("subgraph_features", o)),
             model.MLP.register_forward_hook(lambda m, i, o: acts.__setitem__("im_mlp", o))]
    real_extract = inner.extract_features

    def extract(*a, **kw):
        r = real_extract(*a, **kw)
        acts["interaction_map"], acts["kl_tensor"], acts["noisy"], acts["graph_readout"] = r
        return r

    inner.extract_features = extract
    state0 = {kk: v.detach().clone() for kk, v in model.state_dict().items()}

    torch.manual_seed(seed + 1000)
    with _NoiseRecorder() as rec:
        _, kl, con, rec_loss = model.forward(batch_g, batch_x, ego_g, batch_logMs, x_subs, 1,
                                             batch_g.edges(), 2, "cpu", chunk)
    for h in hooks:
        h.remove()
    loss = kl + rec_loss + con
    loss.backward()

    draws = rec.draws
    assert len(draws) == 2 * B, len(draws)
    u_gate = torch.cat([draws[2 * i].reshape(-1) for i in range(B)])
    u_feat = torch.cat([draws[2 * i + 1] for i in range(B)])

    out = {
        "B": np.array(B), "L": np.array(L), "k": np.array(k), "F": np.array(F),
        "chunk": np.array(chunk), "continue_wrapper": np.array(continue_wrapper),
        "batch_num_nodes": batch_g.batch_num_nodes().numpy(),
        "src": batch_g.src.numpy(), "dst": batch_g.dst.numpy(),
        "x_raw": batch_g.ndata["x"].numpy(),
        "ego_batch_num_nodes": ego_g.batch_num_nodes().numpy(),
        "ego_nodes": ego_g.ndata["_ID"].numpy() if "_ID" in ego_g.ndata else np.zeros(0),
        "ego_src": ego_g.src.numpy(), "ego_dst": ego_g.dst.numpy(),
        "u_gate": u_gate.numpy(), "u_feat": u_feat.numpy(),
        "loss_kl": kl.detach().numpy(), "loss_contrastive": con.detach().numpy(),
        "loss_recon": rec_loss.detach().numpy(), "loss_total": loss.detach().numpy(),
        "recons_type": np.array(recons_type),
    }
    if batch_logMs is not None:  # ragged [k, n_i, n_i] per molecule, flattened
        out["logm_flat"] = np.concatenate([m.numpy().reshape(-1) for m in batch_logMs])
    # ego node ids in the batched ego graph are local to each molecule: make
    # them global (ego j belongs to molecule graph_of(j))
    gptr = np.concatenate([[0], np.cumsum(out["batch_num_nodes"])])
    node_graph = np.repeat(np.arange(B), out["batch_num_nodes"])
    ego_owner = np.repeat(np.arange(len(out["ego_batch_num_nodes"])), out["ego_batch_num_nodes"])
    out["ego_nodes_global"] = out["ego_nodes"] + gptr[node_graph[ego_owner]]
    for kk, v in acts.items():
        out["act_" + kk] = v.detach().numpy()
    inner_pfx = "model." if continue_wrapper else ""
    used = ("transfer_d.", "MLP.") + tuple(inner_pfx + m for m in
                                           ("Encoder1.", "Encoder2.", "compressor.", "attn_layer."))
    for kk, v in state0.items():
        if kk.startswith(used):
            out["param_" + kk] = v.numpy()
    for kk, v in model.state_dict().items():
        if kk.startswith(used) and ("running" in kk or "num_batches" in kk):
            out["after_" + kk] = v.numpy()
    for kk, p in model.named_parameters():
        if p.grad is not None:
            assert kk.startswith(used), kk
            out["grad_" + kk] = p.grad.numpy()
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **out)
    print(f"wrote {name}.npz  N={len(out['x_raw'])} N_s={len(out['ego_nodes'])} "
          f"losses kl={kl.item():.6g} con={con.item():.6g} rec={rec_loss.item():.6g}")


def gen_finetune_golden(models, util_mod, name, *, workload, F, B, k, dataset, num_classes,
                        loss_kind, seed, L=4):
    """Mainmodel_finetuning (models.py:358-543) on a pretrained
    Mainmodel_continue: scores, loss, trainable-parameter gradients (the
    freezing quirk decides which), with recorded noise."""
    torch.manual_seed(seed)
    mols = synth.molecules(B, workload, seed=seed, mu=12.0, sigma=4.0, F=F)
    graphs, subgraphs = [], []
    for ei, x in mols:
        g = util_mod.load_dgl_fromPyG(SimpleNamespace(edge_index=torch.from_numpy(ei),
                                                      x=torch.from_numpy(x)))
        graphs.append(g)
        subgraphs.append([D.khop_in_subgraph(g, v, k=k)[0] for v in g.nodes()])
    batch_g = D.batch(graphs)
    ego_g = D.batch(list(chain.from_iterable(subgraphs)))
    batch_x = F_normalize(batch_g.ndata["x"].float())                 # train_tudataset.py:139
    x_subs = F_normalize(ego_g.ndata["x"].float())                    # :140
    args = SimpleNamespace(recons_type="adj", useAtt=1, readout_f="sum", d_transfer=32,
                           device="cpu", batch_size=B, task="graph_classification",
                           dataset=dataset)
    inner = models.Mainmodel(args, F, hidden_dim=64, num_layers=4, num_heads=4,
                             k_transition=k, encoder="GIN")
    real_load = models.torch.load
    try:
        models.torch.load = lambda *a, **kw: inner  # in-memory: nothing is unpickled
        pre = models.Mainmodel_continue(args, F, hidden_dim=64, num_layers=4, num_heads=4,
                                        k_transition=k, num_classes=num_classes,
                                        cp_filename="<mem>", encoder="GIN")
        # the shipped checkpoint's (and the paper's) 5-GINConv encoders: grown
        # before the fine-tune model is built, so its freezing loop sees them
        for enc in (inner.Encoder1, inner.Encoder2, pre.Encoder1, pre.Encoder2):
            _grow_gin(models, enc, L)
        models.torch.load = lambda *a, **kw: pre
        model = models.Mainmodel_finetuning(args, F, hidden_dim=64, num_layers=4, num_heads=4,
                                            k_transition=k, num_classes=num_classes,
                                            cp_filename="<mem>", encoder="GIN")
    finally:
        models.torch.load = real_load
    # the fine-tune model's own (unused) encoders, as deep as the checkpoint's
    for enc in (model.Encoder1, model.Encoder2):
        _grow_gin(models, enc, L)
    model.train()
    with torch.no_grad():
        for n_, p_ in model.named_parameters():
            if "batch_norms" in n_ or "compressor.1" in n_:
                p_.add_(0.1 * torch.randn_like(p_))
    state0 = {kk: v.detach().clone() for kk, v in model.state_dict().items()}
    trainable = [kk for kk, p in model.named_parameters() if p.requires_grad]
    targets = torch.randint(0, 2, (B,)) if loss_kind == "ce" else \
        torch.randint(0, 2, (B, 1)).float()
    torch.manual_seed(seed + 1000)
    with _NoiseRecorder() as rec:
        scores, *_ = model.forward(batch_g, batch_x, ego_g, x_subs, 1, batch_g.edges(), 2, "cpu",
                                   B)
    loss = model.loss_CrossEntropy(scores, targets) if loss_kind == "ce" else \
        model.loss(scores, targets)
    loss.backward()
    draws = rec.draws
    assert len(draws) == 2 * B, len(draws)
    u_gate = torch.cat([draws[2 * i].reshape(-1) for i in range(B)])
    u_feat = torch.cat([draws[2 * i + 1] for i in range(B)])
    out = {
        "B": np.array(B), "k": np.array(k), "F": np.array(F), "L": np.array(L),
        "num_classes": np.array(num_classes), "dataset": np.array(dataset),
        "loss_kind": np.array(loss_kind),
        "batch_num_nodes": batch_g.batch_num_nodes().numpy(),
        "src": batch_g.src.numpy(), "dst": batch_g.dst.numpy(),
        "x_raw": batch_g.ndata["x"].numpy(),
        "ego_batch_num_nodes": ego_g.batch_num_nodes().numpy(),
        "ego_src": ego_g.src.numpy(), "ego_dst": ego_g.dst.numpy(),
        "u_gate": u_gate.numpy(), "u_feat": u_feat.numpy(),
        "targets": targets.numpy(), "scores": scores.detach().numpy(),
        "loss": loss.detach().numpy(),
        "trainable": np.array(trainable),
    }
    gptr = np.concatenate([[0], np.cumsum(out["batch_num_nodes"])])
    node_graph = np.repeat(np.arange(B), out["batch_num_nodes"])
    ego_owner = np.repeat(np.arange(len(out["ego_batch_num_nodes"])), out["ego_batch_num_nodes"])
    out["ego_nodes_global"] = ego_g.ndata["_ID"].numpy() + gptr[node_graph[ego_owner]]
    for kk, v in state0.items():
        out["param_" + kk] = v.numpy()
    for kk, p in model.named_parameters():
        if p.grad is not None:
            out["grad_" + kk] = p.grad.numpy()
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **out)
    print(f"wrote {name}.npz  N={len(out['x_raw'])} loss={loss.item():.6g} "
          f"trainable={len(trainable)}")


CKPT = "/root/reference/outputs/pre_training_v1_GIN_64_5_1.pt"
CKPT_FIXTURE = "ckpt_pre_training_v1_GIN_64_5_1"


def gen_checkpoint_fixture():
    """The shipped checkpoint's 544 tensors and its wrapper chain, read
    weights-only through inert stand-in classes (s-cgib_amd/refckpt.py — the
    product's reader: this fixture pins it, tests/test_host_cpu.py re-reads
    the file and compares), written as plain npz data for the GPU box."""
    refckpt = importlib.import_module("s-cgib_amd.refckpt")
    levels, cfg, sd = refckpt.read(CKPT)
    out = {"sd/" + k: v.numpy() for k, v in sd.items()}
    out["levels"] = np.array([f"{k}:{f}" for k, f in levels])
    for k in ("hidden_dim", "k_transition", "gin_layers", "num_classes", "d_transfer",
              "batch_size", "useAtt"):
        out["cfg_" + k] = np.array(cfg[k])
    for k in ("recons_type", "readout_f"):
        out["cfg_" + k] = np.array(cfg[k])
    np.savez_compressed(os.path.join(OUT, f"{CKPT_FIXTURE}.npz"), **out)
    print(f"wrote {CKPT_FIXTURE}.npz  tensors={len(sd)} levels={levels}")
    return levels, cfg, sd


def gen_checkpoint_finetune_golden(models, util_mod, name, *, B, seed):
    """BASELINE configs[4]: Mainmodel_finetuning (models.py:358-543) built on
    the shipped pre_training_v1_GIN_64_5_1.pt — the reference's own classes
    rebuilt in memory level by level (Mainmodel_continue x 3 around a
    Mainmodel, each with its own transfer_d width, 5-GINConv encoders) and
    loaded with the checkpoint's tensors (strict), then one ogbg-molhiv-like
    fine-tune step (BCE) in train mode and a forward in eval mode (the
    checkpoint's BatchNorm running statistics), with recorded noise."""
    levels, cfg, sd = gen_checkpoint_fixture()
    k, L, F = cfg["k_transition"], cfg["gin_layers"], levels[0][1]
    torch.manual_seed(seed)
    mols = synth.molecules(B, "molhiv", seed=seed, mu=12.0, sigma=4.0, F=F)
    graphs, subgraphs = [], []
    for ei, x in mols:
        g = util_mod.load_dgl_fromPyG(SimpleNamespace(edge_index=torch.from_numpy(ei),
                                                      x=torch.from_numpy(x)))
        graphs.append(g)
        subgraphs.append([D.khop_in_subgraph(g, v, k=k)[0] for v in g.nodes()])
    batch_g = D.batch(graphs)
    ego_g = D.batch(list(chain.from_iterable(subgraphs)))
    batch_x = F_normalize(batch_g.ndata["x"].float())                 # train_molhiv.py
    x_subs = F_normalize(ego_g.ndata["x"].float())
    args = SimpleNamespace(recons_type=cfg["recons_type"], useAtt=cfg["useAtt"],
                           readout_f=cfg["readout_f"], d_transfer=cfg["d_transfer"],
                           device="cpu", batch_size=B, task="graph_classification",
                           dataset="ogbg-molhiv")
    real_load = models.torch.load
    try:
        m = None
        for kind, f_in in reversed(levels):  # innermost first
            if kind == "Mainmodel":
                m = models.Mainmodel(args, f_in, hidden_dim=64, num_layers=4, num_heads=4,
                                     k_transition=k, encoder="GIN")
            else:
                inner = m
                models.torch.load = lambda *a, **kw: inner  # in-memory: nothing is unpickled
                m = models.Mainmodel_continue(args, f_in, hidden_dim=64, num_layers=4,
                                              num_heads=4, k_transition=k,
                                              num_classes=cfg["num_classes"],
                                              cp_filename="<mem>", encoder="GIN")
        pre = m
        for mod in pre.modules():  # the checkpoint's 5-GINConv encoders
            if isinstance(mod, models.GIN):
                _grow_gin(models, mod, L)
        pre.load_state_dict(sd, strict=True)
        models.torch.load = lambda *a, **kw: pre
        model = models.Mainmodel_finetuning(args, F, hidden_dim=64, num_layers=4, num_heads=4,
                                            k_transition=k, num_classes=1,
                                            cp_filename="<mem>", encoder="GIN")
    finally:
        models.torch.load = real_load
    for enc in (model.Encoder1, model.Encoder2):
        _grow_gin(models, enc, L)
    state0 = {kk: v.detach().clone() for kk, v in model.state_dict().items()
              if not kk.startswith("model.")}  # model.*: the checkpoint fixture
    trainable = [kk for kk, p in model.named_parameters() if p.requires_grad]
    targets = torch.randint(0, 2, (B, 1)).float()
    out = {"B": np.array(B), "k": np.array(k), "F": np.array(F), "L": np.array(L),
           "num_classes": np.array(1), "dataset": np.array("ogbg-molhiv"),
           "loss_kind": np.array("bce"), "checkpoint": np.array(CKPT_FIXTURE),
           "batch_num_nodes": batch_g.batch_num_nodes().numpy(),
           "src": batch_g.src.numpy(), "dst": batch_g.dst.numpy(),
           "x_raw": batch_g.ndata["x"].numpy(),
           "ego_batch_num_nodes": ego_g.batch_num_nodes().numpy(),
           "ego_src": ego_g.src.numpy(), "ego_dst": ego_g.dst.numpy(),
           "targets": targets.numpy(), "trainable": np.array(trainable)}
    for mode in ("eval", "train"):  # eval first: the train step updates running stats
        model.train(mode == "train")
        torch.manual_seed(seed + (1000 if mode == "train" else 2000))
        with _NoiseRecorder() as rec:
            scores, *_ = model.forward(batch_g, batch_x, ego_g, x_subs, 1, batch_g.edges(), 2,
                                       "cpu", B)
        draws = rec.draws
        assert len(draws) == 2 * B, len(draws)
        out[f"{mode}_u_gate"] = torch.cat([draws[2 * i].reshape(-1) for i in range(B)]).numpy()
        out[f"{mode}_u_feat"] = torch.cat([draws[2 * i + 1] for i in range(B)]).numpy()
        out[f"{mode}_scores"] = scores.detach().numpy()
        if mode == "train":
            loss = model.loss(scores, targets)
            loss.backward()
            out["loss"] = loss.detach().numpy()
    gptr = np.concatenate([[0], np.cumsum(out["batch_num_nodes"])])
    node_graph = np.repeat(np.arange(B), out["batch_num_nodes"])
    ego_owner = np.repeat(np.arange(len(out["ego_batch_num_nodes"])), out["ego_batch_num_nodes"])
    out["ego_nodes_global"] = ego_g.ndata["_ID"].numpy() + gptr[node_graph[ego_owner]]
    for kk, v in state0.items():
        out["param_" + kk] = v.numpy()
    for kk, p in model.named_parameters():
        if p.grad is not None:
            out["grad_" + kk] = p.grad.numpy()
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **out)
    print(f"wrote {name}.npz  N={len(out['x_raw'])} loss={out['loss']:.6g} "
          f"eval scores[:2]={out['eval_scores'][:2].ravel()} trainable={len(trainable)}")


def gen_domainadapt_golden(models, util_mod, name, *, workload, F, B, k, num_classes, seed,
                           then_finetune=False):
    """Mainmodel_domainadapt (models.py:107-355) on a pretrained
    Mainmodel_continue, as run_domain_adaptation drives it (exp_molhiv.py:50-68,
    train_molhiv.py:74-105): X loss and the gradients of every parameter, with
    recorded noise.  then_finetune: Mainmodel_finetuning on that adapted model
    (exp_molhiv.py:129-157 loads the DA model), whose extract_features is the
    DA model's OWN (models.py:283) — scores, loss and gradients."""
    torch.manual_seed(seed)
    mols = synth.molecules(B, workload, seed=seed, mu=12.0, sigma=4.0, F=F)
    graphs, subgraphs = [], []
    for ei, x in mols:
        g = util_mod.load_dgl_fromPyG(SimpleNamespace(edge_index=torch.from_numpy(ei),
                                                      x=torch.from_numpy(x)))
        graphs.append(g)
        subgraphs.append([D.khop_in_subgraph(g, v, k=k)[0] for v in g.nodes()])
    batch_g = D.batch(graphs)
    ego_g = D.batch(list(chain.from_iterable(subgraphs)))
    batch_x = F_normalize(batch_g.ndata["x"].float())                 # train_molhiv.py:91
    x_subs = F_normalize(ego_g.ndata["x"].float())                    # :92
    args = SimpleNamespace(recons_type="adj", useAtt=1, readout_f="sum", d_transfer=32,
                           device="cpu", batch_size=B, task="graph_classification",
                           dataset="ogbg-molhiv")
    inner = models.Mainmodel(args, F, hidden_dim=64, num_layers=4, num_heads=4,
                             k_transition=k, encoder="GIN")
    real_load = models.torch.load
    try:
        models.torch.load = lambda *a, **kw: inner  # in-memory: nothing is unpickled
        pre = models.Mainmodel_continue(args, F, hidden_dim=64, num_layers=4, num_heads=4,
                                        k_transition=k, num_classes=num_classes,
                                        cp_filename="<mem>", encoder="GIN")
        models.torch.load = lambda *a, **kw: pre
        da = models.Mainmodel_domainadapt(args, F, hidden_dim=64, num_layers=4, num_heads=4,
                                          k_transition=k, num_classes=num_classes,
                                          cp_filename="<mem>", encoder="GIN")
        model = da
        if then_finetune:
            models.torch.load = lambda *a, **kw: da
            model = models.Mainmodel_finetuning(args, F, hidden_dim=64, num_layers=4,
                                                num_heads=4, k_transition=k,
                                                num_classes=num_classes, cp_filename="<mem>",
                                                encoder="GIN")
    finally:
        models.torch.load = real_load
    model.train()
    with torch.no_grad():
        for n_, p_ in model.named_parameters():
            if "batch_norms" in n_ or "compressor.1" in n_:
                p_.add_(0.1 * torch.randn_like(p_))
    state0 = {kk: v.detach().clone() for kk, v in model.state_dict().items()}
    trainable = [kk for kk, p in model.named_parameters() if p.requires_grad]
    targets = torch.randint(0, 2, (B, 1)).float()
    torch.manual_seed(seed + 1000)
    with _NoiseRecorder() as rec:
        if then_finetune:
            scores, *_ = model.forward(batch_g, batch_x, ego_g, x_subs, 1, batch_g.edges(), 2,
                                       "cpu", B)
            loss = model.loss(scores, targets)
        else:
            loss = model.forward(batch_g, batch_x, ego_g, None, x_subs, 1, batch_g.edges(), 2,
                                 "cpu", B)
            scores = None
    loss.backward()
    draws = rec.draws
    assert len(draws) == 2 * B, len(draws)
    u_gate = torch.cat([draws[2 * i].reshape(-1) for i in range(B)])
    u_feat = torch.cat([draws[2 * i + 1] for i in range(B)])
    out = {
        "B": np.array(B), "k": np.array(k), "F": np.array(F),
        "num_classes": np.array(num_classes), "then_finetune": np.array(int(then_finetune)),
        "batch_num_nodes": batch_g.batch_num_nodes().numpy(),
        "src": batch_g.src.numpy(), "dst": batch_g.dst.numpy(),
        "x_raw": batch_g.ndata["x"].numpy(),
        "ego_batch_num_nodes": ego_g.batch_num_nodes().numpy(),
        "ego_src": ego_g.src.numpy(), "ego_dst": ego_g.dst.numpy(),
        "u_gate": u_gate.numpy(), "u_feat": u_feat.numpy(),
        "targets": targets.numpy(), "loss": loss.detach().numpy(),
        "trainable": np.array(trainable),
    }
    if scores is not None:
        out["scores"] = scores.detach().numpy()
    gptr = np.concatenate([[0], np.cumsum(out["batch_num_nodes"])])
    node_graph = np.repeat(np.arange(B), out["batch_num_nodes"])
    ego_owner = np.repeat(np.arange(len(out["ego_batch_num_nodes"])), out["ego_batch_num_nodes"])
    out["ego_nodes_global"] = ego_g.ndata["_ID"].numpy() + gptr[node_graph[ego_owner]]
    for kk, v in state0.items():
        out["param_" + kk] = v.numpy()
    for kk, p in model.named_parameters():
        if p.grad is not None:
            out["grad_" + kk] = p.grad.numpy()
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **out)
    print(f"wrote {name}.npz  N={len(out['x_raw'])} loss={loss.item():.6g} "
          f"trainable={len(trainable)} grads={sum(1 for k_ in out if k_.startswith('grad_'))}")


def F_normalize(x):
    return F.normalize(x)


def main():
    os.makedirs(OUT, exist_ok=True)
    models = refshim.import_reference_models()
    import util  # the reference's util.py (behind the same shim)
    if sys.argv[1:] == ["domainadapt"]:  # only the domain-adaptation goldens
        gen_domain_adaptation(models, util)
        return
    if sys.argv[1:] == ["round2"]:  # only the goldens added in round 2
        gen_round2(models, util)
        return
    if sys.argv[1:] == ["checkpoint"]:  # only the shipped-checkpoint goldens (round 3)
        gen_checkpoint_goldens(models, util)
        return
    gen_ingest_and_ego(util)
    common = dict(B=8, chunk=4)
    gen_model_golden(models, util, "pretrain_L4_k1_qm9", workload="qm9", F=11, L=4, k=1,
                     continue_wrapper=False, seed=1, **common)
    gen_model_golden(models, util, "pretrain_L5_k1_qm9_continue", workload="qm9", F=11, L=5,
                     k=1, continue_wrapper=True, seed=2, **common)
    gen_model_golden(models, util, "pretrain_L5_k2_ogb_continue", workload="pcqm4mv2", F=9,
                     L=5, k=2, continue_wrapper=True, seed=3, **common)
    # logM reconstruction (A15): Mutagenicity's pretraining default
    # (exp_tudataset.py:538), k_transition 2 -> two transition powers
    gen_model_golden(models, util, "pretrain_L4_k2_logm", workload="mutagenicity", F=14, L=4,
                     k=2, continue_wrapper=False, seed=6, recons_type="logM", **common)
    # fine-tune head: Mutagenicity (CE on sigmoid scores, train_tudataset.py:146) and
    # molhiv (BCE, train_molhiv.py:144), k = 1 as hard-coded in exp_tudataset/exp_molhiv
    gen_finetune_golden(models, util, "finetune_mutag_ce", workload="mutagenicity", F=14, B=8,
                        k=1, dataset="Mutagenicity", num_classes=2, loss_kind="ce", seed=4)
    gen_finetune_golden(models, util, "finetune_molhiv_bce", workload="molhiv", F=9, B=8, k=1,
                        dataset="ogbg-molhiv", num_classes=1, loss_kind="bce", seed=5)
    gen_domain_adaptation(models, util)
    gen_round2(models, util)
    gen_checkpoint_goldens(models, util)


def gen_checkpoint_goldens(models, util):
    # BASELINE configs[4]: ogbg-molhiv fine-tune from pre_training_v1_GIN_64_5_1.pt
    gen_checkpoint_finetune_golden(models, util, "finetune_molhiv_ckpt", B=8, seed=11)


def gen_round2(models, util):
    # molpcba-shaped pretrain step (BASELINE configs[2]: k = 1, OGB features F = 9)
    gen_model_golden(models, util, "pretrain_L5_k1_ogb_continue", workload="molpcba", F=9, L=5,
                     k=1, continue_wrapper=True, seed=9, B=8, chunk=4)
    # BASELINE configs[0] names a 5-layer GIN for the Mutagenicity fine-tune
    gen_finetune_golden(models, util, "finetune_mutag_ce_L5", workload="mutagenicity", F=14,
                        B=8, k=1, dataset="Mutagenicity", num_classes=2, loss_kind="ce",
                        seed=10, L=5)


def gen_domain_adaptation(models, util):
    # domain adaptation: molhiv, k = 1 as in exp_molhiv.py
    gen_domainadapt_golden(models, util, "domainadapt_molhiv", workload="molhiv", F=9, B=8, k=1,
                           num_classes=1, seed=7)
    gen_domainadapt_golden(models, util, "finetune_after_da_molhiv", workload="molhiv", F=9, B=8,
                           k=1, num_classes=1, seed=8, then_finetune=True)


if __name__ == "__main__":
    main()

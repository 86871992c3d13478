"""On-disk CSR cache of a molecule dataset.

The reference preprocesses each pretraining dataset into three pickles
(`exp_pretraining.py:171-206`, `:236-287`; `exp_molpcba.py:239-249,
:316-377`):

* `pts/{ds}_k_transition_{k}.bin` — DGL `save_graphs` of every molecule
  (`load_dgl_fromPyG`, `util.py:277-325`) plus the stacked labels;
* `pts/{ds}_subgraphs_khop_{k}.pt` — a pickled list, per molecule, of one
  DGL graph per node (`dgl.khop_in_subgraph`);
* `pts/{ds}_M_khop_{k}.pt` — the logM transition targets (`util.getM_logM`).

Here one directory of flat arrays replaces all three: the bidirected
molecule CSRs (local node ids), features, labels and — only when asked —
the packed logM targets.  Ego-nets are not stored: `graph.egonet_batch`
builds them on the device from the molecule CSR, bit-identical to
`khop_in_subgraph` (tests).  Arrays are `.npy` files opened memory-mapped,
so a cache larger than host memory streams; a batch is collated by slicing
(vectorised, no per-molecule objects).

Kept reference behaviour:

* the A1 skip rule — a record whose feature rows do not match the node count
  inferred from its edges is skipped and counted as missing
  (`exp_pretraining.py:276-278`'s bare ``except``);
* the 100 000-record cap of the pretraining preprocessors
  (`exp_qm9.py:372`, `exp_pcqm4mv2.py:394`, `exp_molpcba.py:333`): records
  with index >= cap are never read, skipped records count towards the cap;
* the dataset-name mismatch: `exp_molpcba.py:373` writes `ogbg-molpcba_*`
  while `exp_pretraining.py:218` reads `mol-PCBA_*`; `resolve` maps the
  pretraining name to the file the preprocessor wrote (`ALIASES`).

Host-side data plumbing (numpy), not on the device hot path.
"""
from __future__ import annotations

import itertools
import json
import os

import numpy as np
import torch

from . import graph as G

FORMAT = "scgib-csr-1"
DEFAULT_CAP = 100_000
# pretraining dataset name (exp_pretraining.py:218) -> preprocessor's name
# (exp_molpcba.py:373)
ALIASES = {"mol-PCBA": "ogbg-molpcba"}
_CHUNK = 4096


def cache_dir(root, name):
    return os.path.join(root, f"{name}.scgib")


def resolve(root, name):
    """Path of the cache for dataset ``name`` under ``root``, following the
    reference's name mismatch (ALIASES) when only the aliased cache exists."""
    p = cache_dir(root, name)
    if os.path.isdir(p):
        return p
    alt = ALIASES.get(name)
    if alt is not None and os.path.isdir(cache_dir(root, alt)):
        return cache_dir(root, alt)
    raise FileNotFoundError(f"no CSR cache for {name!r} under {root!r}")


def _record(rec):
    """(edge_index, x, y) of a PyG-style record or a tuple."""
    if isinstance(rec, (tuple, list)):
        ei, x = rec[0], rec[1]
        y = rec[2] if len(rec) > 2 else None
    else:
        ei, x, y = rec.edge_index, rec.x, getattr(rec, "y", None)
    if isinstance(ei, torch.Tensor):
        ei = ei.numpy()
    if isinstance(x, torch.Tensor):
        x = x.numpy()
    if isinstance(y, torch.Tensor):
        y = y.numpy()
    return np.asarray(ei, np.int64).reshape(2, -1), np.asarray(x), y


def write(records, root, name, *, cap=DEFAULT_CAP, logm_k=(), overwrite=False):
    """Preprocess ``records`` (PyG-style objects with .edge_index / .x / .y,
    or (edge_index, x[, y]) tuples) into ``{root}/{name}.scgib``.  Records with
    index >= cap are not read (cap None: all).  logm_k: transition orders
    whose logM targets are stored (the reference's `_M_khop_{k}.pt`)."""
    path = cache_dir(root, name)
    if os.path.exists(path) and not overwrite:
        raise FileExistsError(path)
    os.makedirs(path, exist_ok=True)
    deg, col, x, y, kept, counts, ecounts = [], [], [], [], [], [], []
    logms = {int(k): [] for k in logm_k}
    seen = missing = 0
    feat_dim = None
    chunk = []

    def flush():
        nonlocal feat_dim
        if not chunk:
            return
        idx = [i for i, _ in chunk]
        mols = [(ei, xx) for _, (ei, xx, _) in chunk]
        g, kept_local = G.collate_pyg(mols)  # A1: to_bidirected + the skip rule
        rp = g.rowptr.numpy().astype(np.int64)
        c = g.col.numpy().astype(np.int64)[: rp[-1]]
        gptr = np.concatenate([[0], np.cumsum(g.batch_num_nodes_host())])
        node_graph = np.repeat(np.arange(len(kept_local)), np.diff(gptr))
        deg.append(np.diff(rp).astype(np.int32))
        col.append((c - gptr[node_graph[np.repeat(np.arange(len(rp) - 1), np.diff(rp))]])
                   .astype(np.int32))
        xx = g.ndata["x"].numpy()
        if feat_dim is None and len(xx):
            feat_dim = xx.shape[1]
        x.append(xx.astype(np.float32))
        counts.append(g.batch_num_nodes_host().astype(np.int64))
        ecounts.append(g.batch_num_edges().numpy().astype(np.int64))
        for j in kept_local:
            kept.append(idx[j])
            yy = chunk[j][1][2]
            y.append(np.asarray(yy if yy is not None else np.zeros(0), np.float32))
        if logms:
            for j, gi in enumerate(_split(g, len(kept_local))):
                for k in logms:
                    logms[k].append(G.trans_logM(gi, k).numpy())
        chunk.clear()

    # islice: record `cap` itself is never pulled (the reference breaks on
    # the index before indexing the dataset)
    for i, rec in enumerate(records if cap is None else itertools.islice(records, cap)):
        seen += 1
        ei, xx, yy = _record(rec)
        chunk.append((i, (ei, xx, yy)))
        if len(chunk) >= _CHUNK:
            flush()
    flush()
    missing = seen - len(kept)
    counts = np.concatenate(counts) if counts else np.zeros(0, np.int64)
    ecounts = np.concatenate(ecounts) if ecounts else np.zeros(0, np.int64)
    arrays = {
        "graph_ptr": np.concatenate([[0], np.cumsum(counts)]).astype(np.int64),
        "edge_ptr": np.concatenate([[0], np.cumsum(ecounts)]).astype(np.int64),
        "deg": np.concatenate(deg) if deg else np.zeros(0, np.int32),
        "col": np.concatenate(col) if col else np.zeros(0, np.int32),
        "x": np.concatenate(x) if x else np.zeros((0, feat_dim or 1), np.float32),
        "y": np.stack(y) if y else np.zeros((0,), np.float32),
        "kept": np.asarray(kept, np.int64),
    }
    for k, ms in logms.items():
        off = np.zeros(len(ms) + 1, np.int64)
        np.cumsum([m.size for m in ms], out=off[1:])
        arrays[f"logm{k}"] = np.concatenate([m.reshape(-1) for m in ms]) if ms else \
            np.zeros(0, np.float32)
        arrays[f"logm{k}_off"] = off
    for key, arr in arrays.items():
        np.save(os.path.join(path, key + ".npy"), arr)
    meta = {"format": FORMAT, "name": name, "num_graphs": int(len(kept)),
            "num_nodes": int(arrays["graph_ptr"][-1]), "num_edges": int(arrays["edge_ptr"][-1]),
            "feat_dim": int(arrays["x"].shape[1]), "records_read": int(seen),
            "missing": int(missing), "cap": cap, "logm_k": sorted(logms)}
    with open(os.path.join(path, "meta.json"), "w") as fh:
        json.dump(meta, fh, indent=1)
    return CSRCache(path)


def _split(g, n_graphs):
    """Per-molecule GraphBatches of a host batch (for logM targets)."""
    rp = g.rowptr.numpy().astype(np.int64)
    c = g.col.numpy().astype(np.int64)
    gptr = np.concatenate([[0], np.cumsum(g.batch_num_nodes_host())])
    for i in range(n_graphs):
        a, b = gptr[i], gptr[i + 1]
        e0, e1 = rp[a], rp[b]
        src = np.repeat(np.arange(b - a), np.diff(rp[a:b + 1]))
        yield G.GraphBatch.from_edges(src, c[e0:e1] - a, int(b - a), True)


class CSRCache:
    """A written cache, memory-mapped.  ``collate(indices)`` returns the
    GraphBatch of those molecules (DGL batch order = the given order), their
    labels and — if stored — their logM targets."""

    def __init__(self, path, mmap=True):
        self.path = path
        with open(os.path.join(path, "meta.json")) as fh:
            self.meta = json.load(fh)
        if self.meta.get("format") != FORMAT:
            raise G.GraphIngestError(f"{path}: not a {FORMAT} cache")
        mode = "r" if mmap else None
        ld = lambda k: np.load(os.path.join(path, k + ".npy"), mmap_mode=mode)  # noqa: E731
        self.graph_ptr, self.edge_ptr = ld("graph_ptr"), ld("edge_ptr")
        self.deg, self.col, self.x, self.y = ld("deg"), ld("col"), ld("x"), ld("y")
        self.kept = ld("kept")
        self.logm = {k: (ld(f"logm{k}"), ld(f"logm{k}_off")) for k in self.meta["logm_k"]}
        # node-level CSR row pointer (global edge offsets), built once
        self.rowptr = np.concatenate([[0], np.cumsum(self.deg, dtype=np.int64)])

    def __len__(self):
        return self.meta["num_graphs"]

    @property
    def num_features(self):
        return self.meta["feat_dim"]

    def collate(self, indices, k_logm=None):
        idx = np.asarray(indices, np.int64)
        a, b = self.graph_ptr[idx], self.graph_ptr[idx + 1]
        n_i = b - a
        ea, eb = self.rowptr[a], self.rowptr[b]
        e_i = eb - ea
        noff = np.concatenate([[0], np.cumsum(n_i)])
        # node rows and edge ranges of the selected molecules, concatenated
        nodes = np.repeat(a - noff[:-1], n_i) + np.arange(noff[-1])
        eoff = np.concatenate([[0], np.cumsum(e_i)])
        edges = np.repeat(ea - eoff[:-1], e_i) + np.arange(eoff[-1])
        col = self.col[edges].astype(np.int64) + np.repeat(noff[:-1], e_i)
        deg = self.deg[nodes].astype(np.int64)
        src = np.repeat(np.arange(noff[-1]), deg)
        g = G.GraphBatch.from_edges(src, col, int(noff[-1]), True, batch_num_nodes=n_i,
                                    batch_num_edges=e_i)
        dict.__setitem__(g.ndata, "x", torch.from_numpy(np.ascontiguousarray(self.x[nodes])))
        labels = torch.from_numpy(np.ascontiguousarray(self.y[idx]))
        logms = None
        if k_logm is not None:
            flat, off = self.logm[int(k_logm)]
            logms = [torch.from_numpy(np.array(flat[off[i]:off[i + 1]]).reshape(
                int(k_logm), int(n), int(n))) for i, n in zip(idx, n_i)]
        return g, labels, logms

    def graph(self, i):
        return self.collate([i])[0]

    def batches(self, batch_size, shuffle=True, seed=None, drop_last=False, k_logm=None):
        order = np.arange(len(self))
        if shuffle:
            np.random.default_rng(seed).shuffle(order)
        for s in range(0, len(order), batch_size):
            sel = order[s:s + batch_size]
            if drop_last and len(sel) < batch_size:
                break
            yield self.collate(sel, k_logm)


def open_cache(root, name, mmap=True):
    """The cache of dataset ``name`` (reference names accepted, see resolve)."""
    return CSRCache(resolve(root, name), mmap=mmap)

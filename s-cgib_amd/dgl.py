"""Drop-in for the DGL calls the S-CGIB pretraining path makes.

Alias it as ``sys.modules["dgl"]`` before importing the reference scripts
(INTEGRATION.md).  Graph objects are ``graph.GraphBatch``.  Semantics follow
DGL 1.1.0 as used at the reference call sites (restated; DGL itself is not
available here):

  graph((u, v))          util.py:317       num_nodes = max id + 1, edges as given
  to_bidirected(g)       util.py:318       reverse edges added, simple graph,
                                           edges sorted by (src, dst)
  batch(graphs)          molecules.py:359, exp_pretraining.py:309
  sum_nodes(g, 'h')      models.py:716, 725, 733 (HIP segment sum)
  khop_in_subgraph(g, v, k)  exp_pretraining.py:271 (host; the device builder
                                           graph.egonet_batch does all nodes at once)
"""
from __future__ import annotations

import numpy as np
import torch

from . import graph as _G
from . import ops as _ops

DGLGraph = _G.GraphBatch
DGLError = _G.GraphIngestError
NID = "_ID"


def graph(data, num_nodes=None, idtype=None, device=None):
    u, v = data
    u = np.asarray(torch.as_tensor(u).cpu(), np.int64).reshape(-1)
    v = np.asarray(torch.as_tensor(v).cpu(), np.int64).reshape(-1)
    if num_nodes is None:
        num_nodes = int(max(u.max(), v.max()) + 1) if u.size else 0
    g = _G.GraphBatch.from_edges(u, v, num_nodes, symmetric_hint=False)
    return g.to(device) if device is not None else g


def to_bidirected(g, copy_ndata=False, readonly=None):
    src, dst = g.to("cpu").edges()
    s, d = _G.bidirected_simple(src.numpy(), dst.numpy(), max(g.num_nodes(), 1))
    out = _G.GraphBatch.from_edges(s, d, g.num_nodes(), symmetric_hint=True)
    if copy_ndata:
        for k, val in g.ndata.items():
            out.ndata[k] = val.cpu()
    return out


def batch(graphs, ndata="__ALL__", edata="__ALL__"):
    return _G.batch(graphs)


def sum_nodes(g, feat, weight=None, ntype=None):
    x = g.ndata[feat]
    if weight is not None:
        x = x * g.ndata[weight]
    return _ops.sum_nodes_graph(g, x)


def khop_in_subgraph(g, nodes, k, *, relabel_nodes=True, store_ids=True, output_device=None):
    """One node's k-hop in-subgraph on the host, DGL order (sorted ball,
    node_subgraph edge order).  Returns (subgraph, seed position)."""
    gc = g.to("cpu") if g.device.type != "cpu" else g
    rp = gc.rowptr.numpy().astype(np.int64)
    col = gc.col.numpy().astype(np.int64)
    seeds = np.asarray(torch.as_tensor(nodes).cpu(), np.int64).reshape(-1)
    ball = set(seeds.tolist())
    frontier = seeds
    for _ in range(k):
        nb = np.unique(np.concatenate([col[rp[u]:rp[u + 1]] for u in frontier] or [np.zeros(0, np.int64)]))
        ball.update(nb.tolist())
        frontier = nb
    ball = np.array(sorted(ball), np.int64)
    pos = {int(u): i for i, u in enumerate(ball)}
    # out-CSR rows in ball order; for a symmetric graph rowptr/col is the out-CSR
    rp_o = gc.rowptr_t.numpy().astype(np.int64)
    col_o = gc.col_t.numpy().astype(np.int64)
    es, ed = [], []
    for r, u in enumerate(ball):
        for w in col_o[rp_o[u]:rp_o[u + 1]]:
            if int(w) in pos:
                es.append(r)
                ed.append(pos[int(w)])
    sg = _G.GraphBatch.from_edges(np.array(es, np.int64), np.array(ed, np.int64), len(ball),
                                  symmetric_hint=gc.symmetric)
    for key, val in gc.ndata.items():
        dict.__setitem__(sg.ndata, key, val[torch.from_numpy(ball)])
    if store_ids:
        dict.__setitem__(sg.ndata, NID, torch.from_numpy(ball))
    inv = torch.tensor([pos[int(s)] for s in seeds])
    if output_device is not None:
        sg = sg.to(output_device)
    return sg, inv

"""CPU restatement of the DGL 1.1.0 primitives the S-CGIB hot path consumes.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import anything under ``oracle/``;
the product path (``s-cgib_amd/``) never does.

DGL 1.1.0 (``/root/reference/environment.yml:25``) is a third-party dependency
that is absent from the reference tree and from this image, so its semantics
are restated here from its published behaviour.  Parity at the DGL boundary
is therefore *unpinned* against real DGL; what is pinned is
the S-CGIB math of the reference's own ``models.py``, which
``oracle/gen_golden.py`` runs on top of these primitives.

Restated semantics (each used by the reference at the cited call site):

* ``graph((u, v))`` – ``num_nodes = max(u, v) + 1`` (0 with no edges);
  edges kept in the given order.                      (util.py:317)
* ``to_bidirected(g)`` – ``add_reverse_edges`` then ``to_simple``; the simple
  graph is rebuilt from a *sorted* CSR, so edges come out lexicographically
  sorted by (src, dst), duplicates removed, node count unchanged. (util.py:318)
* ``g.ndata['x'] = x`` raises when ``len(x) != num_nodes`` – the reason
  molecules with trailing isolated atoms / no edges are skipped
  (util.py:321, exp_pretraining.py:276-278).
* ``batch(gs)`` – concatenation with node-id offsets, per-graph edge order
  kept.                                   (molecules.py:359, exp_pretraining.py:309)
* ``khop_in_subgraph(g, v, k)`` – frontier_{t+1} = unique(in-neighbours of
  frontier_t); node set = unique(cat(all frontiers)) = sorted ball; subgraph =
  ``node_subgraph`` = out-CSR slice, i.e. induced edges ordered by
  (new src, original CSR column order) with monotone relabelling; ``ndata``
  gathered from the parent.                          (exp_pretraining.py:269-272)
* ``sum_nodes`` – per-graph segment sum.           (models.py:716,725,733)
* ``GINConv`` – ``rst = (1 + eps) * feat_dst + sum_{u->v} feat_u``, then
  ``apply_func``; ``eps`` is a non-learnt buffer.              (models.py:63,69)
* ``Set2Set`` – LSTM(2d -> d, n_layers), ``n_iters`` rounds of
  ``e = <feat, q>``, ``softmax_nodes``, ``r = sum_nodes(feat * alpha)``,
  ``q* = [q || r]``.                                        (models.py:565,515)
* ``adj()`` – sparse matrix with A[src, dst] = 1 per edge; ``to_dense()``
  sums duplicates.                                         (models.py:764)
"""
from __future__ import annotations

import contextlib

import numpy as np
import torch
import torch.nn as nn


class DGLError(Exception):
    pass


class _NData(dict):
    """``g.ndata``: validates row counts like DGL's node frame."""

    def __init__(self, graph):
        super().__init__()
        self._g = graph

    def __setitem__(self, key, value):
        if value.shape[0] != self._g.num_nodes():
            raise DGLError(
                "Expect number of features to match number of nodes (len(u))."
                f" Got {value.shape[0]} and {self._g.num_nodes()} instead.")
        super().__setitem__(key, value)


class _Adj:
    def __init__(self, src, dst, n):
        self.src, self.dst, self.n = src, dst, n

    def to_dense(self):
        a = torch.zeros(self.n, self.n, dtype=torch.float32, device=self.src.device)
        a.index_put_((self.src, self.dst), torch.ones_like(self.src, dtype=torch.float32),
                     accumulate=True)
        return a


class Graph:
    """Homogeneous DGLGraph restatement (COO, int64 ids)."""

    def __init__(self, src, dst, num_nodes, batch_num_nodes=None, batch_num_edges=None):
        self.src = torch.as_tensor(src, dtype=torch.int64)
        self.dst = torch.as_tensor(dst, dtype=torch.int64)
        self._n = int(num_nodes)
        self.ndata = _NData(self)
        self.edata = {}
        if batch_num_nodes is None:
            batch_num_nodes = torch.tensor([self._n], dtype=torch.int64)
            batch_num_edges = torch.tensor([self.src.numel()], dtype=torch.int64)
        self._bnn = torch.as_tensor(batch_num_nodes, dtype=torch.int64)
        self._bne = torch.as_tensor(batch_num_edges, dtype=torch.int64)

    # --- queries -----------------------------------------------------------
    def num_nodes(self, ntype=None):
        return self._n

    number_of_nodes = num_nodes

    def num_edges(self, etype=None):
        return int(self.src.numel())

    number_of_edges = num_edges

    def nodes(self, ntype=None):
        return torch.arange(self._n, dtype=torch.int64, device=self.src.device)

    def edges(self, form="uv", order="eid", etype=None):
        return self.src, self.dst

    def batch_num_nodes(self, ntype=None):
        return self._bnn

    def batch_num_edges(self, etype=None):
        return self._bne

    @property
    def batch_size(self):
        return int(self._bnn.numel())

    @property
    def device(self):
        return self.src.device

    def in_edges(self, v, form="uv", etype=None):
        v = torch.as_tensor(v, dtype=torch.int64, device=self.src.device).reshape(-1)
        mask = torch.isin(self.dst, v)
        return self.src[mask], self.dst[mask]

    def adj(self, etype=None, eweight_name=None):
        return _Adj(self.src, self.dst, self._n)

    # --- mutation / movement -----------------------------------------------
    def to(self, device, **kw):
        g = Graph(self.src.to(device), self.dst.to(device), self._n, self._bnn, self._bne)
        for k, v in self.ndata.items():
            dict.__setitem__(g.ndata, k, v.to(device))
        return g

    @contextlib.contextmanager
    def local_scope(self):
        saved = dict(self.ndata)
        try:
            yield
        finally:
            dict.clear(self.ndata)
            for k, v in saved.items():
                dict.__setitem__(self.ndata, k, v)


# ---------------------------------------------------------------------------
# graph construction
# ---------------------------------------------------------------------------
def graph(data, num_nodes=None, idtype=None, device=None):
    u, v = data
    u = torch.as_tensor(u, dtype=torch.int64).reshape(-1)
    v = torch.as_tensor(v, dtype=torch.int64).reshape(-1)
    if num_nodes is None:
        num_nodes = int(max(u.max().item(), v.max().item()) + 1) if u.numel() else 0
    return Graph(u, v, num_nodes)


def to_simple_sorted(src, dst, n):
    """to_simple over a CSR: sort by (src, dst), drop duplicates."""
    if src.numel() == 0:
        return src.clone(), dst.clone()
    key = src * max(n, 1) + dst
    key = torch.unique(key)  # sorted ascending
    return key // max(n, 1), key % max(n, 1)


def to_bidirected(g, copy_ndata=False, readonly=None):
    src = torch.cat([g.src, g.dst])
    dst = torch.cat([g.dst, g.src])
    s, d = to_simple_sorted(src, dst, g.num_nodes())
    out = Graph(s, d, g.num_nodes())
    if copy_ndata:
        for k, val in g.ndata.items():
            out.ndata[k] = val
    return out


def batch(graphs, ndata="__ALL__", edata="__ALL__"):
    graphs = list(graphs)
    srcs, dsts, off = [], [], 0
    bnn, bne = [], []
    for g in graphs:
        srcs.append(g.src + off)
        dsts.append(g.dst + off)
        off += g.num_nodes()
        bnn.append(g.num_nodes())
        bne.append(g.num_edges())
    src = torch.cat(srcs) if srcs else torch.zeros(0, dtype=torch.int64)
    dst = torch.cat(dsts) if dsts else torch.zeros(0, dtype=torch.int64)
    out = Graph(src, dst, off, torch.tensor(bnn, dtype=torch.int64),
                torch.tensor(bne, dtype=torch.int64))
    if graphs:
        for k in graphs[0].ndata.keys():
            out.ndata[k] = torch.cat([g.ndata[k] for g in graphs], 0)
    return out


def node_subgraph(g, nodes, relabel_nodes=True, store_ids=True):
    """Out-CSR slice: rows visited in ``nodes`` order, columns in CSR order."""
    nodes = torch.as_tensor(nodes, dtype=torch.int64)
    n = g.num_nodes()
    pos = torch.full((n,), -1, dtype=torch.int64)
    pos[nodes] = torch.arange(nodes.numel(), dtype=torch.int64)
    # out-CSR of g: rows = src, columns sorted by dst (g's edges are sorted)
    order = torch.argsort(g.src * max(n, 1) + g.dst, stable=True)
    s_sorted, d_sorted, eid_sorted = g.src[order], g.dst[order], order
    ns, nd, ne = [], [], []
    for new_r, r in enumerate(nodes.tolist()):
        m = s_sorted == r
        cols, eids = d_sorted[m], eid_sorted[m]
        keep = pos[cols] >= 0
        ns.append(torch.full((int(keep.sum()),), new_r, dtype=torch.int64))
        nd.append(pos[cols[keep]])
        ne.append(eids[keep])
    src = torch.cat(ns) if ns else torch.zeros(0, dtype=torch.int64)
    dst = torch.cat(nd) if nd else torch.zeros(0, dtype=torch.int64)
    sg = Graph(src, dst, nodes.numel())
    for k, val in g.ndata.items():
        sg.ndata[k] = val[nodes]
    if store_ids:
        dict.__setitem__(sg.ndata, "_ID", nodes)
        sg.edata["_ID"] = torch.cat(ne) if ne else torch.zeros(0, dtype=torch.int64)
    return sg


def khop_in_subgraph(g, nodes, k, *, relabel_nodes=True, store_ids=True, output_device=None):
    seeds = torch.as_tensor(nodes, dtype=torch.int64).reshape(-1)
    hops = [seeds]
    last = seeds
    for _ in range(k):
        in_nbrs, _ = g.in_edges(last)
        last = torch.unique(in_nbrs)
        hops.append(last)
    ball, inverse = torch.unique(torch.cat(hops), return_inverse=True)
    sg = node_subgraph(g, ball, store_ids=store_ids)
    return sg, inverse[: seeds.numel()]


# ---------------------------------------------------------------------------
# readouts / layers
# ---------------------------------------------------------------------------
def _segment_ids(g):
    return torch.repeat_interleave(
        torch.arange(g.batch_size, device=g.device), g.batch_num_nodes().to(g.device))


def sum_nodes(g, feat, weight=None, ntype=None):
    x = g.ndata[feat]
    out = torch.zeros((g.batch_size,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    return out.index_add(0, _segment_ids(g), x)


def mean_nodes(g, feat, weight=None, ntype=None):
    s = sum_nodes(g, feat)
    return s / g.batch_num_nodes().to(s.device).clamp(min=1).unsqueeze(-1).to(s.dtype)


def broadcast_nodes(g, graph_feat):
    return graph_feat[_segment_ids(g)]


def softmax_nodes(g, feat):
    x = g.ndata[feat]
    seg = _segment_ids(g)
    mx = torch.full((g.batch_size,) + tuple(x.shape[1:]), float("-inf"), dtype=x.dtype)
    mx = mx.scatter_reduce(0, seg.view(-1, *([1] * (x.dim() - 1))).expand_as(x), x, "amax")
    e = torch.exp(x - mx[seg])
    den = torch.zeros_like(mx).index_add(0, seg, e)
    return e / den[seg]


class GINConv(nn.Module):
    def __init__(self, apply_func=None, aggregator_type="sum", init_eps=0, learn_eps=False,
                 activation=None):
        super().__init__()
        self.apply_func = apply_func
        self._aggregator_type = aggregator_type
        self.activation = activation
        if learn_eps:
            self.eps = nn.Parameter(torch.FloatTensor([init_eps]))
        else:
            self.register_buffer("eps", torch.FloatTensor([init_eps]))

    def forward(self, graph, feat, edge_weight=None):
        neigh = torch.zeros_like(feat).index_add(0, graph.dst, feat[graph.src])
        rst = (1 + self.eps) * feat + neigh
        if self.apply_func is not None:
            rst = self.apply_func(rst)
        if self.activation is not None:
            rst = self.activation(rst)
        return rst


class Set2Set(nn.Module):
    def __init__(self, input_dim, n_iters, n_layers):
        super().__init__()
        self.input_dim = input_dim
        self.output_dim = 2 * input_dim
        self.n_iters = n_iters
        self.n_layers = n_layers
        self.lstm = torch.nn.LSTM(self.output_dim, self.input_dim, n_layers)
        self.lstm.reset_parameters()

    def forward(self, graph, feat):
        with graph.local_scope():
            bs = graph.batch_size
            h = (feat.new_zeros((self.n_layers, bs, self.input_dim)),
                 feat.new_zeros((self.n_layers, bs, self.input_dim)))
            q_star = feat.new_zeros(bs, self.output_dim)
            for _ in range(self.n_iters):
                q, h = self.lstm(q_star.unsqueeze(0), h)
                q = q.view(bs, self.input_dim)
                e = (feat * broadcast_nodes(graph, q)).sum(dim=-1, keepdim=True)
                dict.__setitem__(graph.ndata, "e", e)
                alpha = softmax_nodes(graph, "e")
                dict.__setitem__(graph.ndata, "r", feat * alpha)
                readout = sum_nodes(graph, "r")
                q_star = torch.cat([q, readout], dim=-1)
            return q_star


class SumPooling(nn.Module):
    def forward(self, graph, feat):
        with graph.local_scope():
            dict.__setitem__(graph.ndata, "h", feat)
            return sum_nodes(graph, "h")


# ---------------------------------------------------------------------------
# convenience for the oracle / fixtures
# ---------------------------------------------------------------------------
def load_from_pyg(edge_index, x):
    """util.load_dgl_fromPyG (util.py:277-325); raises DGLError on the skip rule."""
    g = graph((edge_index[0], edge_index[1]))
    g = to_bidirected(g)
    g.ndata["x"] = torch.as_tensor(x)
    return g


def csr_from_graph(g):
    """(rowptr, col) with row = dst (in-edges), columns sorted — int64 numpy."""
    n = g.num_nodes()
    key = g.dst * max(n, 1) + g.src
    order = torch.argsort(key)
    col = g.src[order].numpy()
    counts = np.bincount(g.dst.numpy(), minlength=n)
    rowptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(counts, out=rowptr[1:])
    return rowptr, col

"""Batched molecular graphs for the S-CGIB hot path (DGL-duck-typed).

Reference surface reproduced: the model consumes a DGL
graph — ``batch_num_nodes()`` (models.py:665), ``ndata`` reads/writes
(exp_pretraining.py:304, models.py:683), ``edges()``, ``.to(device)``,
``adj().to_dense()`` (models.py:764), ``nodes()`` / ``num_nodes()``.

Storage, MI355X-first:
  * ``rowptr`` [N+1] / ``col`` [E] int32: dst-major CSR (row v lists the
    sources of v's in-edges, columns ascending) — the layout the GIN gather
    kernel reads; 4-byte indices halve index traffic vs int64;
  * ``rowptr_t`` / ``col_t``: the src-major CSR (the same tensors when the
    graph is symmetric, i.e. every to_bidirected molecule);
  * ``graph_ptr`` [B+1] int32: node range of every molecule;
  * host copies of the per-graph node/edge counts, so shape decisions never
    synchronise with the device.

Ingest restates ``util.load_dgl_fromPyG`` (util.py:277-325): ``dgl.graph``
infers ``num_nodes = max id + 1``, ``to_bidirected`` adds reverse edges and
rebuilds a simple graph with edges sorted by (src, dst); a molecule whose
``x`` row count differs from that node count (trailing isolated atoms, no
bonds) raises, which the reference's bare ``except`` turns into "skip"
(exp_pretraining.py:276-278).
"""
from __future__ import annotations

import contextlib
import ctypes

import numpy as np
import torch

from . import _lib


class GraphIngestError(ValueError):
    """Raised where DGL raises on ``g.ndata['x'] = x`` (row-count mismatch)."""


class _NData(dict):
    def __init__(self, graph):
        super().__init__()
        self._g = graph

    def __setitem__(self, key, value):
        if value.shape[0] != self._g.num_nodes():
            raise GraphIngestError(
                f"Expect number of features to match number of nodes. Got {value.shape[0]} "
                f"and {self._g.num_nodes()} instead.")
        super().__setitem__(key, value)


class _Adj:
    def __init__(self, g):
        self._g = g

    def to_dense(self):
        src, dst = self._g.edges()
        n = self._g.num_nodes()
        a = torch.zeros(n, n, dtype=torch.float32, device=src.device)
        a[src, dst] = 1.0
        return a


def _csr_from_sorted(keys_major, minor, n):
    """CSR from edges already sorted by (major, minor)."""
    counts = np.bincount(keys_major, minlength=n) if n else np.zeros(0, np.int64)
    rowptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(counts, out=rowptr[1:])
    return rowptr.astype(np.int32), minor.astype(np.int32)


class GraphBatch:
    """A batch of B graphs with N nodes and E directed edges."""

    def __init__(self, rowptr, col, graph_ptr, batch_num_nodes, batch_num_edges=None,
                 rowptr_t=None, col_t=None, max_graph_nodes=None, n_edges=None,
                 host_info=None):
        self.rowptr = rowptr
        self.col = col
        self.rowptr_t = rowptr if rowptr_t is None else rowptr_t
        self.col_t = col if col_t is None else col_t
        self.symmetric = rowptr_t is None
        self.graph_ptr = graph_ptr
        self._bnn = None if batch_num_nodes is None else np.asarray(batch_num_nodes, np.int64)
        self._bne = None if batch_num_edges is None else np.asarray(batch_num_edges, np.int64)
        self._n = int(rowptr.shape[0] - 1)
        self._e = int(col.shape[0]) if n_edges is None else (None if n_edges < 0 else int(n_edges))
        self._B = int(graph_ptr.shape[0] - 1)
        if max_graph_nodes is None:
            max_graph_nodes = int(self._bnn.max()) if self._bnn is not None and len(self._bnn) else 0
        self.max_graph_nodes = int(max_graph_nodes)
        # host-side facts known at construction (no device sync to get them):
        # {"deg": in-degree per node (np.int64), "selfloops": per-node 0/1,
        #  "validated": edges never leave their graph}
        self.host_info = host_info
        # no edge leaves its graph_ptr segment (host-validated, or built so:
        # ego batches, StaticBatch) -- the chunked fused GIN backward needs it
        self.components_closed = bool(host_info is not None and host_info.get("validated"))
        # capacity mode: device int32 [actual nodes, actual edges]; the host
        # sizes above are then capacities (see StaticBatch)
        self.dims = None
        self.ego_caps = None  # (ego nodes cap, ego edges cap) for capacity mode
        self.seg_dims = None  # ego batches: device count of segments (= parent nodes)
        self.ndata = _NData(self)
        self.edata = {}

    # ----- construction ---------------------------------------------------
    @classmethod
    def from_edges(cls, src, dst, num_nodes, symmetric_hint=False, batch_num_nodes=None,
                   batch_num_edges=None):
        """Graph from a COO edge list (kept as a multigraph-free CSR)."""
        src = np.asarray(src, np.int64)
        dst = np.asarray(dst, np.int64)
        n = int(num_nodes)
        order_out = np.lexsort((dst, src))
        rp_t, col_t = _csr_from_sorted(src[order_out], dst[order_out], n)
        if symmetric_hint:
            rp, col, rp_t2, col_t2 = rp_t, col_t, None, None
        else:
            order_in = np.lexsort((src, dst))
            rp, col = _csr_from_sorted(dst[order_in], src[order_in], n)
            rp_t2, col_t2 = torch.from_numpy(rp_t), torch.from_numpy(col_t)
        if batch_num_nodes is None:
            batch_num_nodes = np.array([n], np.int64)
            batch_num_edges = np.array([len(src)], np.int64)
        gptr = np.zeros(len(batch_num_nodes) + 1, np.int64)
        np.cumsum(batch_num_nodes, out=gptr[1:])
        # edges must stay inside their graph (the ego-net builder relies on it)
        owner = np.searchsorted(gptr, np.arange(n), side="right") - 1 if n else np.zeros(0, np.int64)
        validated = bool(len(src) == 0 or (owner[src] == owner[dst]).all())
        sl = np.zeros(n, np.int64)
        np.add.at(sl, src[src == dst], 1)
        info = {"deg": np.diff(rp.astype(np.int64)), "selfloops": sl, "validated": validated}
        return cls(torch.from_numpy(rp), torch.from_numpy(col),
                   torch.from_numpy(gptr.astype(np.int32)), batch_num_nodes, batch_num_edges,
                   rp_t2, col_t2, host_info=info)

    # ----- DGL surface ------------------------------------------------------
    def num_nodes(self, ntype=None):
        return self._n

    number_of_nodes = num_nodes

    def edge_capacity(self):
        """Host edge count to size launches: exact, or the capacity in capacity mode."""
        return int(self.col.shape[0]) if self.dims is not None else self.num_edges()

    def num_edges(self, etype=None):
        if self._e is None:  # ego batches sized by capacity: read the exact count once
            self._e = int(self.rowptr[-1].item())
        return self._e

    number_of_edges = num_edges

    @property
    def batch_size(self):
        return self._B

    @property
    def device(self):
        return self.rowptr.device

    def batch_num_nodes(self, ntype=None):
        if self._bnn is None:
            gp = self.graph_ptr.to("cpu", torch.int64)
            self._bnn = (gp[1:] - gp[:-1]).numpy()
        return torch.from_numpy(self._bnn)

    def batch_num_nodes_host(self):
        """Per-graph node counts as a host numpy array (no device sync)."""
        self.batch_num_nodes()
        return self._bnn

    def batch_num_edges(self, etype=None):
        if self._bne is None:
            rp_t = self.rowptr_t.to("cpu", torch.int64)
            gp = self.graph_ptr.to("cpu", torch.int64)
            self._bne = (rp_t[gp[1:]] - rp_t[gp[:-1]]).numpy()
        return torch.from_numpy(self._bne)

    def nodes(self, ntype=None):
        return torch.arange(self._n, dtype=torch.int64, device=self.device)

    def edges(self, form="uv", order="eid", etype=None):
        """(src, dst) int64 in DGL's order for to_bidirected graphs: (src, dst) sorted."""
        deg = (self.rowptr_t[1:] - self.rowptr_t[:-1]).to(torch.int64)
        src = torch.repeat_interleave(torch.arange(self._n, device=self.device), deg)
        return src, self.col_t[: self.num_edges()].to(torch.int64)

    def in_degrees(self):
        return (self.rowptr[1:] - self.rowptr[:-1]).to(torch.int64)

    def adj(self, etype=None, eweight_name=None):
        return _Adj(self)

    def to(self, device, non_blocking=False):
        def mv(t):
            return None if t is None else t.to(device, non_blocking=non_blocking)

        g = GraphBatch(mv(self.rowptr), mv(self.col), mv(self.graph_ptr), self._bnn, self._bne,
                       None if self.symmetric else mv(self.rowptr_t),
                       None if self.symmetric else mv(self.col_t), self.max_graph_nodes,
                       -1 if self._e is None else self._e, self.host_info)
        g.dims = mv(self.dims)
        g.components_closed = self.components_closed
        g.ego_caps = self.ego_caps
        g.seg_dims = mv(self.seg_dims)
        for k, v in self.ndata.items():
            dict.__setitem__(g.ndata, k, v.to(device, non_blocking=non_blocking))
        return g

    @contextlib.contextmanager
    def local_scope(self):
        saved = dict(self.ndata)
        try:
            yield
        finally:
            dict.clear(self.ndata)
            dict.update(self.ndata, saved)

    def __repr__(self):
        return (f"GraphBatch(num_graphs={self._B}, num_nodes={self._n}, num_edges={self._e}, "
                f"device={self.device})")


# ---------------------------------------------------------------------------
# ingest (A1) and collate (A3)
# ---------------------------------------------------------------------------
def bidirected_simple(src, dst, n):
    """dgl.to_bidirected(dgl.graph((src, dst))) edges: unique, (src, dst)-sorted."""
    src = np.asarray(src, np.int64)
    dst = np.asarray(dst, np.int64)
    if len(src) == 0:
        return src, dst
    key = np.unique(np.concatenate([src * n + dst, dst * n + src]))
    return key // n, key % n


def pyg_num_nodes(edge_index):
    ei = np.asarray(edge_index)
    return int(ei.max()) + 1 if ei.size else 0


def from_pyg(edge_index, x=None):
    """util.load_dgl_fromPyG (util.py:277-325) for one molecule."""
    ei = np.asarray(edge_index, np.int64).reshape(2, -1)
    n = pyg_num_nodes(ei)
    if x is not None and np.asarray(x).shape[0] != n:
        raise GraphIngestError(f"x has {np.asarray(x).shape[0]} rows, graph has {n} nodes")
    s, d = bidirected_simple(ei[0], ei[1], n)
    g = GraphBatch.from_edges(s, d, n, symmetric_hint=True)
    if x is not None:
        g.ndata["x"] = torch.as_tensor(np.asarray(x))
    return g


def collate_pyg(molecules, device=None, skip_invalid=True):
    """Batch a list of PyG-style ``(edge_index, x)`` molecules in one pass.

    Equivalent to ``dgl.batch([load_dgl_fromPyG(m) for m in molecules])`` with
    the reference's skip rule; vectorised over the batch (edges never cross
    molecules, so one global unique == per-molecule to_bidirected).
    Returns (GraphBatch, kept_indices).
    """
    srcs, dsts, xs, counts, kept = [], [], [], [], []
    off = 0
    for i, (ei, x) in enumerate(molecules):
        ei = np.asarray(ei, np.int64).reshape(2, -1)
        n = pyg_num_nodes(ei)
        if np.asarray(x).shape[0] != n:
            if skip_invalid:
                continue
            raise GraphIngestError(f"molecule {i}: x rows != inferred node count")
        srcs.append(ei[0] + off)
        dsts.append(ei[1] + off)
        xs.append(np.asarray(x, np.float32))
        counts.append(n)
        kept.append(i)
        off += n
    counts = np.asarray(counts, np.int64)
    src = np.concatenate(srcs) if srcs else np.zeros(0, np.int64)
    dst = np.concatenate(dsts) if dsts else np.zeros(0, np.int64)
    s, d = bidirected_simple(src, dst, max(off, 1))
    gptr = np.zeros(len(counts) + 1, np.int64)
    np.cumsum(counts, out=gptr[1:])
    e_counts = np.diff(np.searchsorted(s, gptr)) if len(counts) else np.zeros(0, np.int64)
    g = GraphBatch.from_edges(s, d, off, symmetric_hint=True, batch_num_nodes=counts,
                              batch_num_edges=e_counts)
    g.ndata["x"] = torch.from_numpy(np.concatenate(xs) if xs else np.zeros((0, 1), np.float32))
    if device is not None:
        g = g.to(device)
    return g, kept


def batch(graphs):
    """dgl.batch: concatenate GraphBatches with node-id offsets (host side)."""
    graphs = list(graphs)
    rps, cols, rpts, colts, bnn, bne = [], [], [], [], [], []
    noff = eoff = 0
    sym = all(g.symmetric for g in graphs)
    for g in graphs:
        rp = g.rowptr.cpu().numpy().astype(np.int64)
        rps.append(rp[:-1] + eoff)
        cols.append(g.col.cpu().numpy().astype(np.int64)[: g.num_edges()] + noff)
        if not sym:
            rpt = g.rowptr_t.cpu().numpy().astype(np.int64)
            rpts.append(rpt[:-1] + eoff)
            colts.append(g.col_t.cpu().numpy().astype(np.int64)[: g.num_edges()] + noff)
        bnn.append(g.batch_num_nodes_host())
        bne.append(g.batch_num_edges().numpy())
        noff += g.num_nodes()
        eoff += g.num_edges()
    rowptr = np.concatenate(rps + [np.array([eoff])]).astype(np.int32)
    col = (np.concatenate(cols) if cols else np.zeros(0)).astype(np.int32)
    bnn = np.concatenate(bnn) if bnn else np.zeros(0, np.int64)
    bne = np.concatenate(bne) if bne else np.zeros(0, np.int64)
    gptr = np.zeros(len(bnn) + 1, np.int64)
    np.cumsum(bnn, out=gptr[1:])
    rp_t = col_t = None
    if not sym:
        rp_t = torch.from_numpy(np.concatenate(rpts + [np.array([eoff])]).astype(np.int32))
        col_t = torch.from_numpy(np.concatenate(colts).astype(np.int32))
    out = GraphBatch(torch.from_numpy(rowptr), torch.from_numpy(col),
                     torch.from_numpy(gptr.astype(np.int32)), bnn, bne, rp_t, col_t)
    out.components_closed = bool(graphs) and all(g.components_closed for g in graphs)
    if graphs:
        for k in graphs[0].ndata.keys():
            dict.__setitem__(out.ndata, k, torch.cat([g.ndata[k].cpu() for g in graphs], 0))
    dev = graphs[0].device if graphs else None
    return out.to(dev) if dev is not None and dev.type != "cpu" else out


# ---------------------------------------------------------------------------
# on-device ego-net builder (A2 + the per-step dgl.batch of A3)
# ---------------------------------------------------------------------------
def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def egonet_batch(g: GraphBatch, k: int, x=None):
    """All k-hop in-subgraphs of ``g``, batched: ego j <-> node j of ``g``.

    Equivalent to ``dgl.batch(chain(*[[dgl.khop_in_subgraph(m, v, k)[0] for v
    in m.nodes()] for m in molecules]))`` (exp_pretraining.py:269-272,
    308-309).  Runs on ``g``'s HIP device through scgib_egonet_count/fill.  For
    k = 1 on a host-validated graph the output sizes are known on the host
    (no device sync); otherwise one 3-integer device->host read sizes them.
    The result carries ``ndata['_ID']`` (parent node id of every ego node)
    and, if ``x`` is given, ``ndata['x'] = x[_ID]``.
    """
    if g.device.type != "cuda":
        raise _lib.ScgibError("egonet_batch needs the graph on a HIP device (no CPU fallback)")
    if not g.symmetric:
        raise _lib.ScgibError("egonet_batch expects a symmetric (to_bidirected) graph")
    dev = g.device
    n = g.num_nodes()
    i32 = torch.int32
    ego_ptr = torch.empty(n + 1, dtype=i32, device=dev)
    ego_eptr = torch.empty(n + 1, dtype=i32, device=dev)
    ws = torch.empty(int(_lib.query("scgib_egonet_workspace_bytes", n)), dtype=torch.uint8,
                     device=dev)
    info = g.host_info
    if k == 1 and EGO_K1_FAST and n > 0:
        # two-launch k = 1 builder (sorted-list balls, batched loads): needs
        # the max in-degree bound and in-molecule edges, checked on the host
        kmax = int(_lib.query("scgib_egonet_k1_max_degree"))
        fits = g.max_graph_nodes <= int(_lib.query("scgib_egonet_k1_max_graph_nodes"))
        if g.dims is not None:
            caps = g.ego_caps or ()
            fast = fits and len(caps) > 2 and caps[2] <= kmax
        else:
            fast = (fits and info is not None and info["validated"] and
                    (len(info["deg"]) == 0 or int(info["deg"].max()) <= kmax))
        if fast:
            dmax = int(caps[2]) if g.dims is not None else \
                (int(info["deg"].max()) if len(info["deg"]) else 0)
            return _egonet_k1(g, ego_ptr, ego_eptr, ws, x, dmax)
    err = getattr(g, "err_buf", None)
    if err is None:
        err = torch.zeros(1, dtype=i32, device=dev)
    st = _stream()
    mgn = max(g.max_graph_nodes, 1)
    _lib.call("scgib_egonet_count", _ptr(g.rowptr), _ptr(g.col), _ptr(g.graph_ptr), g.batch_size,
              n, k, mgn, _ptr(ego_ptr), _ptr(ego_eptr), _ptr(ws), _ptr(err), _ptr(g.dims), st)
    ego_dims = None
    if g.dims is not None:
        # capacity mode: outputs sized by the graph's capacities, actual sizes
        # stay on the device (ego_dims) — nothing is read back
        if g.ego_caps is None:
            raise _lib.ScgibError("capacity-mode graph without ego capacities (StaticBatch)")
        n_s, e_cap = g.ego_caps[:2]
        e_s = -1
        ego_dims = torch.empty(2, dtype=i32, device=dev)
    elif k == 1 and info is not None and info["validated"] and mgn <= 512:
        # sizes known on the host, no device sync: |ball(v)| = 1 + deg(v) - selfloop(v);
        # the induced-edge count is bounded by sum_{u in ball(v)} deg(u)
        ball = 1 + info["deg"] - info["selfloops"]
        n_s = int(ball.sum())
        e_cap = int((info["deg"] * ball).sum())
        e_s = -1  # exact count read lazily (GraphBatch.num_edges)
    else:
        tot = torch.stack([ego_ptr[n], ego_eptr[n], err[0]]).cpu().tolist()
        n_s, e_s, e_code = int(tot[0]), int(tot[1]), int(tot[2])
        if e_code:
            raise _lib.ScgibError(f"scgib_egonet_count flagged error bits {e_code} "
                                  "(1: edge leaves its graph, 2: graph larger than max_graph_nodes)")
        e_cap = e_s
    ego_nodes = torch.empty(n_s, dtype=i32, device=dev)
    sub_rowptr = torch.empty(n_s + 1, dtype=i32, device=dev)
    sub_col = torch.empty(max(e_cap, 1), dtype=i32, device=dev)
    _lib.call("scgib_egonet_fill", _ptr(g.rowptr), _ptr(g.col), _ptr(g.graph_ptr), g.batch_size, n,
              k, mgn, _ptr(ego_ptr), _ptr(ego_eptr), _ptr(ego_nodes), _ptr(sub_rowptr),
              _ptr(sub_col), _ptr(err), n_s, _ptr(g.dims), _ptr(ego_dims), st)
    ego = GraphBatch(sub_rowptr, sub_col, ego_ptr, None, None, n_edges=e_s,
                     max_graph_nodes=mgn)
    ego.dims = ego_dims
    ego.components_closed = True  # induced subgraphs: edges stay in their ego-net
    ego.seg_dims = g.dims  # the ego batch's segments are g's nodes
    dict.__setitem__(ego.ndata, "_ID", ego_nodes)
    if x is not None:
        dict.__setitem__(ego.ndata, "x", x.index_select(0, ego_nodes))
    return ego


def ego_bounds(g, k):
    """(ego-batch nodes, bound on ego-batch edges, max in-degree) of host
    batch ``g``'s k-hop ego-nets: nodes = sum_v |ball_k(v)|, edges <= sum_v
    sum_{u in ball_k(v)} deg(u).  k = 1: |ball(v)| = 1 + deg(v) - selfloop(v);
    k > 1: boolean reachability (I + A)^k on the host."""
    info = g.host_info
    deg = info["deg"].astype(np.int64)
    dmax = int(deg.max()) if len(deg) else 0
    if k == 1:
        ball = 1 + deg - info["selfloops"]
        return int(ball.sum()), int((deg * ball).sum()), dmax
    import scipy.sparse as sp
    n = g.num_nodes()
    rp = g.rowptr.cpu().numpy().astype(np.int64)
    col = g.col.cpu().numpy()[: rp[-1]].astype(np.int64)
    a = sp.csr_matrix((np.ones(len(col), np.int8), col, rp), shape=(n, n))
    step = (a + sp.identity(n, dtype=np.int8, format="csr")).astype(bool).astype(np.int32)
    r = step
    for _ in range(k - 1):
        r = (r @ step).astype(bool).astype(np.int32)
    return int(r.nnz), int((r @ deg).sum()), dmax


# k = 1 ego-nets through the sorted-list window builders when their bounds
# hold (in-degree <= 12, molecules <= the window), else the bitmap builder.
# On since round 1, session 4 (39 vs 46 us per QM9 B512 build alone; in the
# replayed step it first measured 0.5 % slower, which the later LDS-window
# one-pass form turned into 2.7 % faster).  Module attributes,
# not environment knobs: the tests compare every builder bit for bit.
EGO_K1_FAST = True
# ... in one launch (count + look-back scan + fill, egonet_k1_onepass_k)
# instead of two (count + block scan, fill)
EGO_K1_ONEPASS = True


def _egonet_k1(g, ego_ptr, ego_eptr, ws, x, max_in_degree=12):
    """egonet_batch for k = 1 via scgib_egonet_k1_build (sizes known on the
    host: |ball(v)| = 1 + deg(v) - selfloop(v); capacity mode: g.ego_caps)."""
    dev = g.device
    n = g.num_nodes()
    i32 = torch.int32
    ego_dims = None
    if g.dims is not None:
        n_s, e_cap = g.ego_caps[:2]
        ego_dims = torch.empty(2, dtype=i32, device=dev)
    else:
        info = g.host_info
        ball = 1 + info["deg"] - info["selfloops"]
        n_s = int(ball.sum())
        e_cap = int((info["deg"] * ball).sum())
    ego_nodes = torch.empty(max(n_s, 1), dtype=i32, device=dev)
    sub_rowptr = torch.empty(n_s + 1, dtype=i32, device=dev)
    sub_col = torch.empty(max(e_cap, 1), dtype=i32, device=dev)
    if EGO_K1_ONEPASS:
        from . import ops  # (ops imports this module)
        state = ops.scan_state(dev, "egonet_k1_scan", int(_lib.query("scgib_egonet_k1_scan_words", n)))
        ops._launch("scgib_egonet_k1_build_onepass", {"n": n}, _ptr(g.rowptr), _ptr(g.col), n,
                  int(max_in_degree), _ptr(ego_ptr), _ptr(ego_eptr), _ptr(state), _ptr(ego_nodes),
                  _ptr(sub_rowptr), _ptr(sub_col), n_s, max(e_cap, 1),
                  _ptr(getattr(g, "err_buf", None)), _ptr(g.dims), _ptr(ego_dims), _stream())
    else:
        _lib.call("scgib_egonet_k1_build_deg", _ptr(g.rowptr), _ptr(g.col), n,
                  int(max_in_degree), _ptr(ego_ptr), _ptr(ego_eptr), _ptr(ws), _ptr(ego_nodes),
                  _ptr(sub_rowptr), _ptr(sub_col), n_s, _ptr(g.dims), _ptr(ego_dims), _stream())
    ego = _ego_graph(g, sub_rowptr, sub_col, ego_ptr, ego_nodes, n_s, ego_dims)
    if x is not None:
        dict.__setitem__(ego.ndata, "x", x.index_select(0, ego_nodes[:n_s]))
    return ego


def _ego_graph(g, sub_rowptr, sub_col, ego_ptr, ego_nodes, n_s, ego_dims):
    ego = GraphBatch(sub_rowptr, sub_col, ego_ptr, None, None, n_edges=-1,
                     max_graph_nodes=max(g.max_graph_nodes, 1))
    ego.dims = ego_dims
    ego.components_closed = True
    ego.seg_dims = g.dims
    dict.__setitem__(ego.ndata, "_ID", ego_nodes[:n_s])
    return ego


class StaticBatch:
    """Capacity-sized device buffers of one molecule batch, for HIP-graph
    replay of the training step: every kernel reads the actual node/edge
    counts from ``dims`` (device), so a graph captured on these buffers
    serves every batch of ``B`` molecules that fits the capacities.

    ``load(src)`` copies a padded device batch (``pad(...)``) in with five
    device-to-device copies; nothing is read back to the host.
    """

    def __init__(self, B, n_cap, e_cap, n_feat, max_graph_nodes, ego_caps, device, k=1):
        self.B, self.n_cap, self.e_cap, self.n_feat = B, n_cap, e_cap, n_feat
        self.k = int(k)
        # one byte blob (rowptr | col | graph_ptr | dims | x, 256-B aligned
        # sections) so that loading a batch is a single device copy
        self.blob = torch.zeros(self._layout()[-1], dtype=torch.uint8, device=device)
        self.rowptr, self.col, self.graph_ptr, self.dims, self.err, self.x = \
            self._views(self.blob)
        self.graph = GraphBatch(self.rowptr, self.col, self.graph_ptr, None, None,
                                max_graph_nodes=max_graph_nodes, n_edges=-1)
        self.graph.dims = self.dims
        self.graph.components_closed = True  # pad() refuses batches whose edges leave a molecule
        # ego-net error word, zeroed by every load (no fill launch in the step)
        self.graph.err_buf = self.err
        self.graph.ego_caps = tuple(int(c) for c in ego_caps)

    def _layout(self):
        sizes = [4 * (self.n_cap + 1), 4 * max(self.e_cap, 1), 4 * (self.B + 1), 4 * 4,
                 4 * self.n_cap * self.n_feat]
        offs = [0]
        for sz in sizes:
            offs.append(offs[-1] + (sz + 255) // 256 * 256)
        return offs

    def _views(self, blob):
        o = self._layout()
        i32 = torch.int32
        return (blob[o[0]:o[0] + 4 * (self.n_cap + 1)].view(i32),
                blob[o[1]:o[1] + 4 * max(self.e_cap, 1)].view(i32),
                blob[o[2]:o[2] + 4 * (self.B + 1)].view(i32),
                blob[o[3]:o[3] + 8].view(i32),
                blob[o[3] + 8:o[3] + 12].view(i32),
                blob[o[4]:o[4] + 4 * self.n_cap * self.n_feat].view(torch.float32)
                .view(self.n_cap, self.n_feat))

    @staticmethod
    def capacities(host_batches, k, slack=1.0):
        """(n_cap, e_cap, max_graph_nodes, (ego nodes cap, ego edges cap, max
        in-degree)) covering every host-collated batch given,
        for k-hop ego-nets (k = 1 in closed form, k > 1 from the host
        reachability of each batch, as the reference's offline pass would)."""
        n = max(g.num_nodes() for g in host_batches)
        e = max(g.num_edges() for g in host_batches)
        mgn = max(g.max_graph_nodes for g in host_batches)
        ns = es = dmax = 0
        for g in host_batches:
            bn, be, bd = ego_bounds(g, k)
            ns, es, dmax = max(ns, bn), max(es, be), max(dmax, bd)
        f = lambda v: int(v * slack) + 1  # noqa: E731
        # ego caps: (nodes, edges, max in-degree — selects the k = 1 builder)
        return f(n), f(e), mgn, (f(ns), f(es), dmax if k == 1 else 1 << 30)

    def pad(self, g):
        """Device copy of host batch ``g`` padded to this batch's capacities."""
        n, e = g.num_nodes(), g.num_edges()
        if n > self.n_cap or e > self.e_cap or g.batch_size != self.B:
            raise _lib.ScgibError(f"batch (B={g.batch_size}, N={n}, E={e}) does not fit the "
                                  f"capacities (B={self.B}, N={self.n_cap}, E={self.e_cap})")
        if g.max_graph_nodes > self.graph.max_graph_nodes:
            raise _lib.ScgibError("batch has a larger molecule than the captured bitmap width")
        if not g.host_info["validated"]:
            raise _lib.ScgibError("batch edges leave their molecule")
        ns, es = self.graph.ego_caps[:2]
        bn, be, _ = ego_bounds(g, self.k)
        if bn > ns or be > es:
            raise _lib.ScgibError("batch's ego-nets exceed the ego capacities")
        if len(self.graph.ego_caps) > 2 and len(g.host_info["deg"]) and \
                int(g.host_info["deg"].max()) > self.graph.ego_caps[2]:
            raise _lib.ScgibError("batch's max degree exceeds the captured ego builder's bound")
        if self.B and g.batch_num_nodes_host().min() < 2:
            raise ValueError("Expected more than 1 value per channel when training "
                             "(a molecule with one atom; the reference skips those)")
        blob = np.zeros(self._layout()[-1], np.uint8)
        o = self._layout()
        rp = np.full(self.n_cap + 1, e, np.int32)
        rp[: n + 1] = g.rowptr.cpu().numpy()
        blob[o[0]:o[0] + rp.nbytes] = rp.view(np.uint8)
        col = g.col.cpu().numpy()[:e].astype(np.int32)
        blob[o[1]:o[1] + col.nbytes] = col.view(np.uint8)
        gp = g.graph_ptr.cpu().numpy().astype(np.int32)
        blob[o[2]:o[2] + gp.nbytes] = gp.view(np.uint8)
        blob[o[3]:o[3] + 8] = np.array([n, e], np.int32).view(np.uint8)
        x = np.ascontiguousarray(g.ndata["x"].cpu().numpy().astype(np.float32))
        blob[o[4]:o[4] + x.nbytes] = x.view(np.uint8).reshape(-1)
        dev = self.blob.device
        return {"blob": torch.from_numpy(blob).to(dev), "n": n, "e": e}

    def load(self, padded):
        """Copy a pad()-ed batch into the static buffers (one device copy)."""
        self.blob.copy_(padded["blob"], non_blocking=True)
        self._unload_prefetch()

    def _unload_prefetch(self):
        pf = getattr(self.graph, "ego_prefetch", None)
        if pf is not None:
            pf.loaded = False  # its ego buffers no longer match the static batch

    def pool(self, padded):
        """Device state for load_next over the pad()-ed batches ``padded``: the
        table of their blobs and the cursor (kept alive by the caller along
        with ``padded``)."""
        dev = self.blob.device
        for p in padded:
            if p["blob"].numel() != self.blob.numel():
                raise _lib.ScgibError("pool batch was padded for other capacities")
        table = torch.tensor([p["blob"].data_ptr() for p in padded], dtype=torch.int64, device=dev)
        return {"table": table, "cursor": torch.zeros(2, dtype=torch.int32, device=dev),
                "n": len(padded), "batches": padded}

    def load_next(self, pool, prefetch=None):
        """Copy the pool's next batch in (one kernel, capturable: the replays of
        a graph holding it walk the pool in order, pool(...)[cursor] first).
        With an EgoPrefetch the same launch also moves the ego-nets it built
        for this batch into the step's ego buffers."""
        src2 = dst2 = None
        n2 = 0
        self._unload_prefetch()
        if prefetch is not None:
            if prefetch.pool is not pool:
                raise _lib.ScgibError("EgoPrefetch was made for another pool")
            # a prefetch no backward joined (a forward without backward) must
            # be done with the staging blob before this copy reads it
            prefetch.join()
            src2, dst2, n2 = _ptr(prefetch.staging), _ptr(prefetch.blob), prefetch.blob.numel()
            prefetch.loaded = True
        _lib.call("scgib_pool_copy2", ctypes.c_void_p(pool["table"].data_ptr()), pool["n"],
                  ctypes.c_void_p(pool["cursor"].data_ptr()), ctypes.c_void_p(self.blob.data_ptr()),
                  self.blob.numel(), src2, dst2, n2,
                  ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))

    def blob_offsets(self):
        """Byte offsets of (rowptr, col, graph_ptr, dims) inside each blob."""
        o = self._layout()
        return o[0], o[1], o[2], o[3]

    def ego_error(self):
        """Error bits the ego-net build of the last step flagged (0 = none; see
        egonet_batch) — a device read, for checks outside the timed loop."""
        return int(self.err.item())


class EgoPrefetch:
    """The ego-nets one batch ahead, for a replayed step over a StaticBatch
    pool (bench.py): step t builds the ego-nets of the batch step t + 1 will
    load — straight from that batch's pool blob, on the encoder pair's queue
    while it would otherwise idle through the loss section
    (models._encode_forked) — into a staging blob, and step t + 1's batch load
    (StaticBatch.load_next) moves them into the ego buffers the step reads.
    Every step still builds one batch's ego-nets (the reference's
    khop_in_subgraph pass, exp_pretraining.py:269-272); the build leaves the
    head of the step's critical path.  k = 1 within the one-pass builder's
    bounds: scgib_egonet_k1_build_onepass_pool; otherwise (k >= 2) the
    bitmap builder's count + fill, scgib_egonet_count_pool / _fill_pool.

    ``prime()`` builds the ego-nets of the pool's current batch once before
    the first step (eager).  ``ego`` is the step's ego batch (capacity mode,
    the same layout egonet_batch gives)."""

    def __init__(self, static, pool):
        g = static.graph
        caps = g.ego_caps or ()
        kmax = int(_lib.query("scgib_egonet_k1_max_degree"))
        self.onepass = (static.k == 1 and EGO_K1_FAST and len(caps) > 2 and caps[2] <= kmax and
                        g.max_graph_nodes <= int(_lib.query("scgib_egonet_k1_max_graph_nodes")))
        if len(caps) < 2 or g.max_graph_nodes > 512:
            raise _lib.ScgibError("EgoPrefetch needs ego capacities and molecules of <= 512 atoms")
        self.static, self.pool, self.k = static, pool, static.k
        self.n = g.num_nodes()
        self.n_s, self.e_cap = int(caps[0]), int(caps[1])
        self.dmax = int(caps[2]) if len(caps) > 2 else 0
        dev = static.blob.device
        # ego_ptr | ego_eptr | ego_nodes | sub_rowptr | sub_col | (ego dims, error bits)
        sizes = [4 * (self.n + 1), 4 * (self.n + 1), 4 * max(self.n_s, 1), 4 * (self.n_s + 1),
                 4 * max(self.e_cap, 1), 16]
        offs = [0]
        for sz in sizes:
            offs.append(offs[-1] + (sz + 255) // 256 * 256)
        self._offs, self._sizes = offs, sizes
        self.blob = torch.zeros(offs[-1], dtype=torch.uint8, device=dev)
        self.staging = torch.zeros(offs[-1], dtype=torch.uint8, device=dev)
        self.views = self._views(self.blob)
        self.next_views = self._views(self.staging)
        ego_ptr, _, ego_nodes, sub_rowptr, sub_col, ego_dims, self.err = self.views
        self.ego = _ego_graph(g, sub_rowptr, sub_col, ego_ptr, ego_nodes, self.n_s, ego_dims)
        self.ws = None if self.onepass else torch.empty(
            int(_lib.query("scgib_egonet_workspace_bytes", self.n)), dtype=torch.uint8, device=dev)
        self.loaded = False  # ego holds the static batch's ego-nets (load_next with this)
        self._side = None  # stream of a prefetch not yet joined back (join())
        g.ego_prefetch = self  # models._encode_forked takes ego from here when loaded

    def _views(self, blob):
        i32 = torch.int32
        v = [blob[o:o + sz].view(i32) for o, sz in zip(self._offs, self._sizes)]
        tail = v.pop()
        return (*v, tail[:2], tail[2:3])

    def prefetch(self):
        """Enqueue (current stream) the build of the ego-nets of the pool's
        batch at the cursor — the one the next load_next copies in — into the
        staging blob."""
        ego_ptr, ego_eptr, ego_nodes, sub_rowptr, sub_col, ego_dims, err = self.next_views
        o_rp, o_col, o_gptr, o_dims = self.static.blob_offsets()
        src = (_ptr(self.pool["table"]), self.pool["n"], _ptr(self.pool["cursor"]))
        if self.onepass:
            from . import ops  # (ops imports this module)
            state = ops.scan_state(self.blob.device, "egonet_k1_scan_prefetch",
                                   int(_lib.query("scgib_egonet_k1_scan_words", self.n)))
            _lib.call("scgib_egonet_k1_build_onepass_pool", *src, o_rp, o_col, o_dims, self.n,
                      self.dmax, _ptr(ego_ptr), _ptr(ego_eptr), _ptr(state), _ptr(ego_nodes),
                      _ptr(sub_rowptr), _ptr(sub_col), self.n_s, max(self.e_cap, 1), _ptr(err),
                      _ptr(ego_dims), _stream())
            return
        g = self.static.graph
        mgn = max(g.max_graph_nodes, 1)
        _lib.call("scgib_egonet_count_pool", *src, o_rp, o_col, o_gptr, o_dims, g.batch_size,
                  self.n, self.k, mgn, _ptr(ego_ptr), _ptr(ego_eptr), _ptr(self.ws), _ptr(err),
                  _stream())
        _lib.call("scgib_egonet_fill_pool", *src, o_rp, o_col, o_gptr, o_dims, g.batch_size,
                  self.n, self.k, mgn, _ptr(ego_ptr), _ptr(ego_eptr), _ptr(ego_nodes),
                  _ptr(sub_rowptr), _ptr(sub_col), _ptr(err), self.n_s, _ptr(ego_dims), _stream())

    def error(self):
        """Error bits any prefetched build flagged (sticky; 0 = none; see
        egonet_batch) — a device read, for checks outside the timed loop."""
        return int(self.err.item())

    def prime(self):
        """The ego-nets of the pool's batch at the cursor into staging, before
        the first load_next (eager, current stream)."""
        self.prefetch()

    def __call__(self):
        """The encoder pair's side tail: prefetch on the current stream, which
        the pair's backward joins back (joined()) — else join() does."""
        self.prefetch()
        self._side = torch.cuda.current_stream()

    def joined(self):
        self._side = None

    def join(self):
        """Order the current stream after a prefetch that no backward joined
        (e.g. a forward without backward); no-op otherwise."""
        if self._side is not None:
            torch.cuda.current_stream().wait_stream(self._side)
            self._side = None


# ---------------------------------------------------------------------------
# A15: logM reconstruction targets (host data preparation, like the
# reference's offline pass exp_tudataset.py:416-449)
# ---------------------------------------------------------------------------
def trans_logM(g, kstep):
    """util.getM_logM (util.py:74-91) + GetProbTranMat (:60-71) of one molecule:
    A^1..A^k of the dense adjacency, each column-normalised,
    log(A^i / colsum) - log(1/n), negatives / -inf / NaN set to 0; computed in
    float64 like the reference's numpy and returned as float32 [k, n, n]
    (exp_tudataset.py:433)."""
    n = g.num_nodes()
    A = g.adj().to_dense().cpu().numpy().astype(np.float32)
    Ak = np.identity(n)
    out = []
    with np.errstate(divide="ignore", invalid="ignore"):
        for _ in range(kstep):
            Ak = Ak @ A
            colsum = np.repeat(Ak.sum(axis=0).reshape(1, -1), n, axis=0)
            P = np.log(np.divide(Ak, colsum)) - np.log(1.0 / n)
            P[P < 0] = 0
            P[np.isnan(P)] = 0
            out.append(P)
    return torch.from_numpy(np.array(out)).float()


class LogMBatch:
    """Device form of a batch's logM targets for scgib_recon_logm_*: per molecule
    S = sum_i logM_i ([n, n] fp32, packed at int64 offsets) and
    C = sum_i ||logM_i||_F^2 (fp64); kstep = k."""

    def __init__(self, logms, device):
        logms = [torch.as_tensor(m) for m in logms]
        if not logms:
            raise GraphIngestError("empty logM batch")
        self.kstep = int(logms[0].shape[0])
        sizes, S, C = [], [], []
        for m in logms:
            if m.dim() != 3 or m.shape[0] != self.kstep or m.shape[1] != m.shape[2]:
                raise GraphIngestError(f"logM target of shape {tuple(m.shape)}: expected "
                                       f"[{self.kstep}, n, n]")
            m64 = m.double()
            sizes.append(m.shape[1])
            S.append(m64.sum(0).float().reshape(-1))
            C.append(float((m64 * m64).sum()))
        off = np.zeros(len(sizes) + 1, np.int64)
        np.cumsum(np.asarray(sizes, np.int64) ** 2, out=off[1:])
        self.sizes = np.asarray(sizes, np.int64)
        self.S = torch.cat(S).to(device)
        self.offsets = torch.from_numpy(off).to(device)
        self.C = torch.tensor(C, dtype=torch.float64, device=device)

"""Autograd ops over the C-ABI (include/scgib.h).  HIP only — no fallback.

Each op checks that its tensors are fp32/int32, contiguous and on a HIP
device, launches on torch's current stream (so torch's caching allocator and
stream semantics apply) and raises ``ScgibError`` on any non-zero status.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import weakref

import numpy as np
import torch

from . import _lib
from . import graph as _graph
from ._lib import HIDDEN, PGRAD_STRIDE, STATS_STRIDE

_NULL = None

# Instrumentation hook (bench.py): when set, OBSERVER(name, meta, launch) is
# called instead of launch() for the launches routed through _launch, with
# meta = the sizes needed to price the launch.  None in production.
OBSERVER = None


def _launch(name, meta, *args):
    if OBSERVER is None:
        return _lib.call(name, *args)
    return OBSERVER(name, meta, lambda: _lib.call(name, *args))


# Off-critical-path work (e.g. the compressor-BN running-stat update, which
# nothing later in the step reads): launched on an auxiliary stream forked
# from the current one, joined back by join_aside() (models call it at the
# end of forward, so captured graphs stay closed).
_AUX_STREAMS = {}
_AUX_PENDING = set()
# Design switches (module attributes, not environment knobs: the measured
# alternatives were removed, DESIGN.md §5 keeps their numbers).  Tests set
# them to cover both sides where both are supported:
# deferred BatchNorm finalize in the fused GIN layers (scgib_bn_pending):
# layer l leaves its statistics as group partials, layer l + 1 finishes them
# (off: the producer finishes them; +4 % / +2.5 % step, round 2)
DEFER_BN = True
DEFER_BN_FWD = True
# layer l's weight-gradient slab reduce folded into layer l-1's backward
# statistics launch (extra workgroups, scgib_gin_bwd_stats_bn_fold) instead of
# the chain's final reduce launch; only layer 0's slabs are left for the end
# (bench.py's superbatch pass turns it off to time the statistics kernel alone)
FOLD_SLABS = True
# the GIN layers' hidden activation r = relu(agg W1^T + b1): stored by the
# forward and read by the backward (True), or not stored and recomputed bit
# for bit by the backward from the saved agg (False: scgib_gin_layer_bwd /
# _layer0_bwd with r NULL, gin_bwd5r_k).  Same bits
# either way (test_gin_r_recompute_bitwise).  Measured (profiles/r05_recompute):
# recomputing costs 8192 flop per row on f32 MFMA, more than the 512 B of
# r traffic it saves — step 0.398 -> 0.421 ms, superbatch forward -39 us but
# backward +145 us per layer — so r is stored; False saves 256 B per row and
# layer of saved activations.  (A d_in = 32 layer fed by a given h0, i.e. not
# the transfer_d fold, always stores r.)
STORE_R = True
# the d_in = 64 GIN layers l >= 1 without a saved agg:
# the forward writes only r and z2, the layer backward (scgib_gin_layer_bwd_z)
# writes dz1 instead of d(agg), and the layer below's statistics launch
# (scgib_gin_bwd_stats_z) gathers dz1 and forms d h = g W1 and dW1 = g^T h
# there (g = (I + A)^T dz1, A symmetric).  Needs STORE_R (the recompute path
# reads agg).  False: every layer stores agg (the round-5 path).
AGG_FREE = True
# ... for encoders of at least this many rows: below it the layer's agg rows
# stay in the Infinity Cache / L2 between the forward and the backward, the
# store + reload costs little, and the agg-free statistics launch's two
# dependent GEMM phases lengthen the latency-bound chain instead (QM9 B512,
# ego-nets of 27.9 k rows: 0.389 -> 0.416 ms per step); from molpcba B1024's
# 80 k-row ego-nets up it is neutral to faster (0.907 -> 0.903 ms; PCQM B2048
# k2: 1.432 -> 1.425 ms), and at ZINC scale the agg rows go to HBM and back
# (the d = 64 forward 0.35 -> 0.40 of HBM, the layer backward 715 -> 711 us).
# DESIGN.md §5 "Agg-free layers" has the A/B.
AGG_FREE_MIN_ROWS = 1 << 16


# LATE_FORK (always): launch_aside records an event on the current stream now
# and enqueues the aside work at join_aside() time, after it has waited on
# that event — the same dependencies, but in a captured graph the main chain's
# next kernel is then created first and so keeps the producer's hardware queue
# (the replayed graph puts a node's first-created child on its queue).
# Only inside aside_deferred() (model forwards, which always end with
# join_aside()); elsewhere aside work is enqueued at once.
_AUX_DEFERRED = []
_DEFER_DEPTH = [0]
# the interaction forward's running-stat update, waiting for the loss head's
# launch (take_running_update) or for join_aside
_PENDING_RU = [None]


# Loss-section weight-gradient reduces deferred into the encoder pair's
# backward (the head MLP's, the interaction's and compressor[0]'s slabs are
# summed by Encoder1's final scgib_slab_reduce_multi instead of one reduce
# launch each on the loss chain).  The gradient tensors these backward
# functions return are then written by a launch enqueued LATER in the same
# backward pass, so a deferral is taken only when nothing can read them
# before: every parameter is a contiguous fp32 CUDA leaf whose .grad is None
# (AccumulateGrad takes the tensor without a kernel), no hook of any kind is
# registered on it or on its AccumulateGrad node, and no other encoder-pair
# forward is awaiting its backward (two forwards into one backward would make
# autograd add the two gradients first).  A scope still open when the
# autograd graph task ends (a backward that never reached the encoder pair,
# e.g. autograd.grad over the head parameters only) reduces its jobs inline
# from an engine callback.  Anything else reduces inline, as before.
DEFER_LOSS_REDUCE = True


class SlabScope:
    """Slab-reduce jobs collected between an encoder pair's forward and its
    backward (which drains them into a chain's final reduce)."""

    _live = weakref.WeakSet()
    # the deferred gradients live on the HIP device (a hook for the host tests)
    _device_ok = staticmethod(lambda p: p.is_cuda)

    def __init__(self):
        self.jobs, self.keep, self.later = [], [], []
        self.open, self.ok, self.callback, self.stream = True, True, False, None
        for other in list(SlabScope._live):
            if other.open:  # two forwards awaiting one backward: defer nothing
                other.ok = self.ok = False
        SlabScope._live.add(self)

    def usable(self, params):
        """Whether a loss-section backward may hand autograd gradients that a
        later launch of this scope writes.  Not for: parameters that are not
        contiguous fp32 CUDA leaves (the backward returns an fp32 tensor that
        autograd would cast or copy at once), a .grad to accumulate into, or a
        hook on the tensor.  (A hook registered directly on a parameter's
        AccumulateGrad node is not visible from Python: whoever registers one
        that reads the gradient sets ops.DEFER_LOSS_REDUCE = False; this
        package's GradAllReducer reads .grad only after backward returns.)"""
        return self.open and self.ok and all(
            p is None or (SlabScope._device_ok(p) and p.dtype == torch.float32 and p.is_contiguous() and
                          p.is_leaf and p.grad is None and
                          not getattr(p, "_backward_hooks", None) and
                          not getattr(p, "_post_accumulate_grad_hooks", None))
            for p in params)

    def add(self, slab, wgrad, width, n_slabs):
        self.jobs.append(_lib.SlabJob(slab.data_ptr(), wgrad.data_ptr(), width, n_slabs, 0))
        self.keep += [slab, wgrad]
        self._arm(slab)

    def defer(self, launch, *tensors):
        """A weight-gradient launch nothing before the optimizer reads (the
        Set2Set LSTM's, scgib_set2set_wgrad): enqueued by the encoder pair's
        backward on the current stream after the ego chain's backward, off the
        loss section's serial chain; ``tensors`` stay referenced until then."""
        self.later.append((launch, tensors))
        self._arm(tensors[0])

    def _arm(self, t):
        self.stream = torch.cuda.current_stream() if t.is_cuda else None
        if not self.callback:
            # a backward that never reaches the encoder pair (autograd.grad over
            # the loss-section parameters only, backward(inputs=...)) would never
            # take the jobs: reduce them at the end of the graph task instead
            try:
                torch.autograd.Variable._execution_engine.queue_callback(self._flush)
                self.callback = True
            except RuntimeError:  # not inside a backward pass (host tests)
                pass

    def _flush(self):
        if not self.open or not (self.jobs or self.later):
            return
        later = self.take_later()
        jobs, keep = self.take()
        with torch.cuda.stream(self.stream):
            for launch, _ in later:
                launch()
            if jobs:
                _reduce_jobs(jobs, _stream())
        del keep, later  # the slabs stay allocated until the launches are enqueued

    def take_later(self):
        later, self.later = self.later, []
        return later

    def take(self):
        self.open = False
        jobs, keep = self.jobs, self.keep
        self.jobs, self.keep = [], []
        return jobs, keep


_SLAB_SCOPE = [None]  # the latest encoder pair's scope (captured by later loss ops)


def _slab_scope_for(params):
    """The current scope if a backward may defer its reduce into it."""
    sc = _SLAB_SCOPE[0]  # (autograd Function forwards run with grad mode off)
    return sc if (sc is not None and DEFER_LOSS_REDUCE) else None


@contextlib.contextmanager
def aside_deferred():
    _DEFER_DEPTH[0] += 1
    try:
        yield
    finally:
        _DEFER_DEPTH[0] -= 1


# The library's forked streams (models' side stream, the aux stream above).
# A fork taken FROM one of them while a HIP graph is being captured nests
# forks; torch-ROCm's CUDAGraph::capture_end segfaults on any nested fork,
# even one with no work or allocation on the inner stream, while the same
# sequence of HIP stream/event calls captures, instantiates and replays in
# plain HIP (tools/capture_probe.py, tools/nested_torch_repro.py,
# tools/nested_capture_repro.hip).  check_fork() refuses it with an error
# instead of the crash at the end of the capture.
_FORK_STREAMS = set()


def register_fork_stream(stream):
    _FORK_STREAMS.add((stream.device_index, stream.stream_id))
    return stream


def check_fork(src):
    """Raise if a fork from ``src`` would nest forks inside a HIP-graph capture."""
    if (src.device_index, src.stream_id) in _FORK_STREAMS and \
            torch.cuda.is_current_stream_capturing():
        raise RuntimeError(
            "stream fork from an already-forked stream during HIP-graph capture: "
            "torch-ROCm's capture_end crashes on nested forks (DESIGN.md §3); fork from the "
            "capture's origin stream instead")


def _aux_stream(device):
    key = device.index
    aux = _AUX_STREAMS.get(key)
    if aux is None:
        aux = _AUX_STREAMS[key] = register_fork_stream(torch.cuda.Stream(device))
    return key, aux


def launch_aside(fn, *tensors):
    """Run ``fn`` (work nothing later in the step reads) off the critical path.
    Only inside aside_deferred() — the model forwards, which always end with
    join_aside() — does it go to the auxiliary stream; a standalone op call
    (the C-ABI drop-in surface) runs it inline on the caller's stream, so the
    op's in-place outputs are ordered before the caller's next read."""
    if _DEFER_DEPTH[0] == 0:
        fn()
        return
    main = torch.cuda.current_stream()
    check_fork(main)
    key, _ = _aux_stream(main.device)
    ev = torch.cuda.Event()
    ev.record(main)
    _AUX_DEFERRED.append((key, ev, fn, tensors))
    _AUX_PENDING.add(key)


def discard_aside():
    """Error path of a model forward: drop aside work that was deferred but
    never enqueued (replaying it with the next batch would apply that batch's
    running-stat update twice) and join what already ran on the aux stream."""
    _SLAB_SCOPE[0] = None
    _PENDING_RU[0] = None
    _AUX_DEFERRED.clear()
    if _AUX_PENDING:
        main = torch.cuda.current_stream()
        for key in list(_AUX_PENDING):
            main.wait_stream(_AUX_STREAMS[key])
        _AUX_PENDING.clear()


def aside_guard(fn):
    """Decorator for model forwards that end with join_aside(): an exception
    raised between the deferred launch and the join discards the deferred
    work instead of leaving it for the next forward.  Each call first runs
    check_handoff() (host-side, no sync)."""
    import functools

    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        check_handoff()  # an earlier step's hand-off wait gave up: raise, loud
        try:
            return fn(*args, **kwargs)
        except BaseException:
            discard_aside()
            raise
    return wrapper


def take_running_update():
    """The compressor BatchNorm running update left by the interaction forward
    (a scgib_running_update for the loss head's launch), or None."""
    pend, _PENDING_RU[0] = _PENDING_RU[0], None
    return pend


def join_aside():
    _SLAB_SCOPE[0] = None  # end of a model forward: later standalone ops never defer
    pend = take_running_update()
    if pend is not None:  # no loss-head launch took it: the aux stream
        launch_aside(pend[1], *pend[2])
    if not _AUX_PENDING:
        return
    main = torch.cuda.current_stream()
    for key, ev, fn, tensors in _AUX_DEFERRED:  # LATE_FORK: enqueue now, after ev
        aux = _AUX_STREAMS[key]
        aux.wait_event(ev)
        for t in tensors:
            t.record_stream(aux)
        with torch.cuda.stream(aux):
            fn()
    _AUX_DEFERRED.clear()
    for key in list(_AUX_PENDING):
        main.wait_stream(_AUX_STREAMS[key])
    _AUX_PENDING.clear()


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else _NULL


def _byref(st):
    """Pointer argument for a ctypes Structure (None -> NULL); the C side
    copies it into the kernel arguments before returning."""
    return ctypes.cast(ctypes.pointer(st), ctypes.c_void_p) if st is not None else _NULL


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _f32(t, name):
    if not t.is_cuda:
        raise _lib.ScgibError(f"{name}: tensor is on {t.device}; the S-CGIB ops run on the HIP "
                              "device only (no CPU fallback)")
    if t.dtype != torch.float32:
        t = t.float()
    return t.contiguous()


# ---------------------------------------------------------------------------
# A5: GIN aggregation
# ---------------------------------------------------------------------------
def _aggregate(h, rowptr, col, ope, dims=None):
    n, d = h.shape
    out = torch.empty_like(h)
    _lib.call("scgib_gin_aggregate", _p(h), _p(rowptr), _p(col), n, d, float(ope), _p(out),
              _p(dims), _stream())
    return out


class _GinAggregate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, graph, ope):
        h = _f32(h, "gin_aggregate")
        ctx.graph, ctx.ope = graph, ope
        return _aggregate(h, graph.rowptr, graph.col, ope, graph.dims)

    @staticmethod
    def backward(ctx, g):
        g = _f32(g, "gin_aggregate.backward")
        gr = ctx.graph
        # d/dh of sum_{u->v} h_u is the aggregation over the transposed CSR
        return _aggregate(g, gr.rowptr_t, gr.col_t, ctx.ope, gr.dims), None, None


def gin_aggregate(h, graph, one_plus_eps=1.0):
    """out[v] = (1 + eps) h[v] + sum_{u -> v} h[u]  (DGL GINConv, models.py:69)."""
    return _GinAggregate.apply(h, graph, float(one_plus_eps))


# ---------------------------------------------------------------------------
# A5 fused: the whole GIN encoder (L x GINConv(MLP) + BN + ReLU)
# ---------------------------------------------------------------------------
def _gin_layer_params(gin):
    """Per layer (W1, b1, W2, b2, gamma, beta) of a models.GIN, flattened."""
    out = []
    for conv, bn in zip(gin.ginlayers, gin.batch_norms):
        mlp = conv.apply_func.mlp
        out += [mlp[0].weight, mlp[0].bias, mlp[2].weight, mlp[2].bias, bn.weight, bn.bias]
    return out


def _drain(gen, tag=None):
    """Run a step generator to completion and return its value (``tag``:
    stamps at each of its yields, at stamp level 2)."""
    i = 0
    while True:
        try:
            next(gen)
        except StopIteration as stop:
            return stop.value
        if tag is not None and _STAMPS["level"] >= 2:
            stamp(f"{tag}.{i}")
        i += 1


# ---------------------------------------------------------------------------
# Diagnostics: device wall-clock stamps (scgib_stamp) at the step's chain
# boundaries, for the timeline of a REPLAYED step with its hand-offs on (a
# rocprofv3 kernel trace serialises the queues' submission, so the hand-offs
# are off there: ops.handoff_rule).  Off unless stamps_enable() was called
# (bench.py: SCGIB_STAMPS=1 coarse, =2 also one per GIN layer); each stamp is
# one more 1-thread launch on its stream.
# ---------------------------------------------------------------------------
_STAMPS = {"buf": None, "labels": [], "level": 0}


def stamps_enable(device, level=1, slots=256):
    _STAMPS["buf"] = torch.zeros(slots, dtype=torch.int64, device=device)
    _STAMPS["labels"] = []
    _STAMPS["level"] = int(level)


def stamp(label):
    """The device wall clock when the current stream reaches this point (when
    stamps are enabled; a no-op otherwise)."""
    buf = _STAMPS["buf"]
    if buf is None or len(_STAMPS["labels"]) >= buf.numel():
        return
    _STAMPS["labels"].append(label)
    _lib.call("scgib_stamp", _p(buf), len(_STAMPS["labels"]) - 1, _stream())


def stamps_read():
    """[(label, us after the first stamp)] of the last replay / run, in time order."""
    buf = _STAMPS["buf"]
    if buf is None or not _STAMPS["labels"]:
        return []
    t = buf[:len(_STAMPS["labels"])].cpu().tolist()
    t0 = min(t)
    return sorted(((lab, (v - t0) / 100.0) for lab, v in zip(_STAMPS["labels"], t)),
                  key=lambda e: e[1])


# hipGraphNodeType (hip_runtime_api.h): the node kinds a replayed step holds
_NODE_TYPES = {0: "kernel", 1: "memcpy", 2: "memset", 5: "empty", 6: "wait_event",
               7: "event_record"}


def graph_node_counts(graph):
    """Nodes of a captured torch CUDAGraph made with keep_graph=True, by
    hipGraphNodeType ({"kernel": .., "memcpy": .., "memset": .., ..., "total"}):
    each node of a replayed graph is host enqueue work (~1.6 us
    per node), so this is the step's launch-overhead count."""
    hip = ctypes.CDLL("libamdhip64.so")
    g = ctypes.c_void_p(graph.raw_cuda_graph())
    n = ctypes.c_size_t(0)
    if hip.hipGraphGetNodes(g, None, ctypes.byref(n)) != 0:
        raise _lib.ScgibError("hipGraphGetNodes failed")
    nodes = (ctypes.c_void_p * max(n.value, 1))()
    if hip.hipGraphGetNodes(g, nodes, ctypes.byref(n)) != 0:
        raise _lib.ScgibError("hipGraphGetNodes failed")
    out = {"total": int(n.value)}
    t = ctypes.c_int(0)
    for i in range(n.value):
        if hip.hipGraphNodeGetType(ctypes.c_void_p(nodes[i]), ctypes.byref(t)) != 0:
            raise _lib.ScgibError("hipGraphNodeGetType failed")
        key = _NODE_TYPES.get(t.value, f"type{t.value}")
        out[key] = out.get(key, 0) + 1
    return out


class SplitUnsupported(_lib.ScgibError):
    """scgib_graph_split refused the graph (a non-kernel node, or an in-graph
    hand-off the two lanes cannot keep): replay the captured graph instead."""


_SPLIT_SLOTS = 64  # hand-off slots per split (the pretraining step uses 2-3)
_LIVE_SPLITS = weakref.WeakSet()


class SplitGraph:
    """A captured step graph replayed as two linear lanes (csrc/graph_split.hip,
    include/scgib.h scgib_graph_split): the host enqueues ~6 us per lane
    instead of ~3 us per node of a two-branch graph (tools/graph_launch_probe.hip,
    DESIGN.md §3 "Host enqueue").  Built from a torch.cuda.CUDAGraph captured
    with keep_graph=True; the torch graph is kept (its memory pool holds the
    step's buffers) and never replayed.  Replays go on the stream current at
    construction (the side stream was checked against its hardware queue).  The lanes' waits rely on two
    concurrently running queues like the encoder pair's hand-offs, so callers
    split only when xq_enabled() holds (a kernel trace serialises dispatch)."""

    def __init__(self, graph, device):
        dev = torch.device(device)
        self.graph = graph
        self.words = torch.zeros(4 * _SPLIT_SLOTS, dtype=torch.int32, device=dev)
        self._fault = handoff_fault_word(dev)
        self._host = _host_fault_word(dev)
        # the side lane reads its slots at once: the zero fill must have landed
        torch.cuda.synchronize(dev)
        handle = ctypes.c_void_p()
        info = (ctypes.c_int32 * 8)()
        rc = _lib.load().scgib_graph_split(
            ctypes.c_void_p(graph.raw_cuda_graph()), _p(self.words), _SPLIT_SLOTS, _p(self._fault),
            _p(self._host), _stream(), ctypes.byref(handle), info)
        if rc == -2:
            raise SplitUnsupported("scgib_graph_split: graph not splittable into two lanes")
        if rc != 0:
            raise _lib.ScgibError(f"scgib_graph_split failed: {_lib.load().scgib_strerror(rc).decode()}"
                                  f" (code {rc})")
        self._handle = handle
        self.device = dev
        self._stream_id = torch.cuda.current_stream(dev).cuda_stream
        keys = ("captured", "lane0_kernels", "lane1_kernels", "handoffs", "lane0_nodes",
                "lane1_nodes", "serialised", "slots")
        self.info = dict(zip(keys, (int(v) for v in info)))
        _LIVE_SPLITS.add(self)

    def replay(self):
        if torch.cuda.current_stream(self.device).cuda_stream != self._stream_id:
            raise _lib.ScgibError("SplitGraph.replay: replay on the stream the split was made on "
                                  "(its side stream's hardware queue was checked against that one)")
        _lib.call("scgib_graph_split_launch", self._handle, _stream())

    def timeouts(self):
        """Waits of the added hand-offs that gave up (0 when the lanes overlapped)."""
        return int(self.words.view(-1, 4)[:self.info["slots"], 2].sum().item())

    def close(self):
        if self._handle:
            _lib.call("scgib_graph_split_destroy", self._handle)
            self._handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 (interpreter shutdown)
            pass


# the agg-free layer's weight-gradient row: dW2 [64][64] | db2 | db1 (the
# scgib_gin_layer_bwd_z slab, reduced as one job) | dW1 [64][64] (the
# scgib_gin_bwd_stats_z slab of the layer below)
_Z_SLAB = HIDDEN * HIDDEN + 2 * HIDDEN
_Z_W1_OFF = _Z_SLAB


# The ego chain's final weight-gradient reduce (after the encoder pair's
# backward join) and the optimizer step right after it as ONE launch
# (scgib_adam_step_reduce, optim.Adam.step): inside fuse_final_into_step() the
# pair's backward leaves its final reduce jobs here instead of launching them,
# and the step takes them; whatever no step took is reduced when the context
# ends.  Only where nothing reads the gradients between the backward and the
# step (the benches' replayed steps without a collective).
FUSE_FINAL_ADAM = True
# ... from this many slabs in the largest final job (the ego layer-0 weight-
# gradient slabs).  0: always.  With four Adam elements per thread in the
# fused launch QM9 B = 32 (28 slabs) was slower fused and this stood at 256;
# with one (SCGIB_FUSE_EPT) B = 32 is faster fused too
# (profiles/r06_noise/fuse_adam_ab.txt, fuse_ept_ab.txt)
FUSE_FINAL_MIN_SLABS = 0
_FINAL_ARMED = [False]
_FINAL_PENDING = {}  # device index -> [(jobs, keep)]


@contextlib.contextmanager
def fuse_final_into_step():
    prev = _FINAL_ARMED[0]
    _FINAL_ARMED[0] = FUSE_FINAL_ADAM
    try:
        yield
    finally:
        _FINAL_ARMED[0] = prev
        for idx in list(_FINAL_PENDING):
            for jobs, _keep in _FINAL_PENDING.pop(idx):
                _reduce_jobs(jobs, _stream())


def take_final(device):
    """The pending final reduces of ``device`` (consumed: the caller launches them)."""
    return _FINAL_PENDING.pop(torch.device(device).index or 0, [])


def _reduce_jobs(jobs, st, max_wg=0):
    cap = int(_lib.query("scgib_slab_reduce_max_jobs"))
    for i0 in range(0, len(jobs), cap):
        chunk = jobs[i0:i0 + cap]
        table = (_lib.SlabJob * len(chunk))(*chunk)
        _lib.call("scgib_slab_reduce_multi_ex", ctypes.cast(table, ctypes.c_void_p), len(chunk),
                  int(max_wg), st)


class _GinEncoder(torch.autograd.Function):
    """GIN.forward (models.py:66-72) as fused HIP layers; see gin_layer.hip.

    With ``x`` / ``wt`` given (h0 = None), transfer_d (h0 = x Wt^T,
    models.py:668-669) is folded into layer 0: the kernel gathers the raw
    features — through ``nmap`` (ego -> parent row) when given, so x_subs is
    never materialised — and d Wt comes out of the layer-0 backward."""

    @staticmethod
    def forward(ctx, h0, graph, gin, training, x, wt, nmap, *params, readout=None):
        """readout = (ptr, nseg, seg_dims): also return the segment sums of
        the output (dgl.sum_nodes, fused with the last BN + ReLU); the backward
        then takes (g_out, g_readout)."""
        return _drain(_GinEncoder.forward_steps(ctx, h0, graph, gin, training, x, wt, nmap,
                                                *params, readout=readout))

    @staticmethod
    def forward_steps(ctx, h0, graph, gin, training, x, wt, nmap, *params, readout=None):
        """forward as a generator that yields after each layer's launch, so
        two encoders on two streams can be enqueued (captured) layer by layer
        in alternation (_GinEncoderPair); returns forward's result."""
        pre = x is not None
        if pre:
            x = _f32(x, "gin_encoder x")
            wt = _f32(wt, "transfer_d.weight")
            n = graph.num_nodes()  # the row capacity in capacity mode
            dev = x.device
        else:
            h0 = _f32(h0, "gin_encoder")
            n = h0.shape[0]
            dev = h0.device
        st = _stream()
        L = len(gin.ginlayers)
        ntiles = int(_lib.query("scgib_gin_tiles", n))
        tstats = torch.empty(max(ntiles, 1), 128, dtype=torch.float32, device=dev)
        # training: BN finalize folded into the layer kernel (one counter set
        # per encoder module: the two encoders run on concurrent streams)
        fused = training and n > 0
        # deferred BN finalize (scgib_bn_pending): layer l leaves its statistics
        # as group partials and layer l + 1 finishes them (the last layer's
        # are finished in its own launch: deferring them into the output's
        # BN + ReLU kernel measured neutral to 0.5 % slower)
        defer_ok = fused and DEFER_BN and DEFER_BN_FWD and \
            n <= int(_lib.query("scgib_gin_defer_max_nodes"))
        ws_floats = max(int(_lib.query("scgib_gin_bn_ws_floats", n)), 1)
        bn_wss = [torch.empty(ws_floats, dtype=torch.float32, device=dev)
                  for _ in range(2 if defer_ok else 1)]
        gpart_off = 4 * int(_lib.query("scgib_gin_bn_gpart_offset", n))
        # (keyed by call site and stream: concurrent encoders run on different
        # streams, launches on one stream are ordered and leave the words zero)
        cnt = scan_state(dev, "gin_fwd", int(_lib.query("scgib_gin_counters", n))) \
            if fused else None
        saved, h, stat_prev, aggx, pend = [], h0, None, None, None
        for l in range(L):
            conv, bn = gin.ginlayers[l], gin.batch_norms[l]
            w1, b1, w2, b2, gamma, beta = (_f32(p, "gin param") for p in params[6 * l: 6 * l + 6])
            d_in = w1.shape[1] if (pre and l == 0) else h.shape[1]
            if w1.shape != (HIDDEN, d_in) or w2.shape != (HIDDEN, HIDDEN):
                raise _lib.ScgibError(f"fused GIN layer needs Linear({d_in},64)/Linear(64,64), got "
                                      f"{tuple(w1.shape)}/{tuple(w2.shape)}")
            # agg only where a backward reads it: layer 0, and every layer
            # without AGG_FREE (the agg-free layers' dW1 comes from the layer
            # below's statistics launch, a frozen layer's backward reads none)
            agg_free = AGG_FREE and STORE_R and l >= 1 and d_in == HIDDEN and \
                n >= AGG_FREE_MIN_ROWS
            agg = None if agg_free else torch.empty(n, d_in, dtype=torch.float32, device=dev)
            # r only where the backward cannot recompute it (or STORE_R)
            keep_r = STORE_R or (d_in != HIDDEN and not (pre and l == 0))
            r = torch.empty(n, HIDDEN, dtype=torch.float32, device=dev) if keep_r else None
            z2 = torch.empty(n, HIDDEN, dtype=torch.float32, device=dev)
            meta = {"n": n, "e": graph.edge_capacity(), "d_in": d_in, "r": r is not None,
                    "agg": agg is not None}
            stat = torch.empty(4, HIDDEN, dtype=torch.float32, device=dev)
            track = training and bn.track_running_stats
            momentum = float(bn.momentum if bn.momentum is not None else 0.1)
            rm = _p(bn.running_mean) if track else None
            rv = _p(bn.running_var) if track else None
            nbt = _p(bn.num_batches_tracked) if track else None
            bn_ws = bn_wss[l % len(bn_wss)]
            defer = int(defer_ok and l < L - 1)
            if pre and l == 0:
                aggx = torch.empty(n, 16, dtype=torch.float32, device=dev)
                _launch("scgib_gin_layer0_fwd", meta, _p(x), x.shape[1], _p(nmap), _p(wt),
                        _p(graph.rowptr), _p(graph.col), n, conv._one_plus_eps, _p(w1), _p(b1),
                        _p(w2), _p(b2), _p(agg), _p(aggx), _p(r), _p(z2), _p(gamma), _p(beta),
                        float(bn.eps), momentum, rm, rv, nbt, _p(stat), _p(bn_ws), _p(cnt),
                        _p(graph.dims), defer, st)
            elif fused:
                _launch("scgib_gin_layer_fwd_bn", meta, _p(h), d_in,
                        None if pend is not None else _p(stat_prev),
                        _p(graph.rowptr), _p(graph.col), n, conv._one_plus_eps, _p(w1), _p(b1),
                        _p(w2), _p(b2), _p(agg), _p(r), _p(z2), _p(gamma), _p(beta),
                        float(bn.eps), momentum, rm, rv, nbt, _p(stat), _p(bn_ws), _p(cnt),
                        _p(graph.dims), _byref(pend), defer, st)
            else:
                _launch("scgib_gin_layer_fwd", meta, _p(h), d_in, _p(stat_prev),
                        _p(graph.rowptr), _p(graph.col), n, conv._one_plus_eps, _p(w1), _p(b1),
                        _p(w2), _p(b2), _p(agg), _p(r), _p(z2), _p(tstats), _p(graph.dims), st)
            if not fused:  # eval (running statistics) or untracked: separate finalize
                src = bn_ws if (pre and l == 0) else tstats
                _lib.call("scgib_bn_finalize", _p(src), n, _p(gamma), _p(beta), float(bn.eps),
                          momentum, int(training),
                          _p(bn.running_mean) if (track or not training) else None,
                          _p(bn.running_var) if (track or not training) else None,
                          nbt, _p(stat), _p(graph.dims), st)
            saved += [agg, r, z2, stat]
            h, stat_prev = z2, stat
            pend = _lib.BnPending(
                bn_ws.data_ptr() + gpart_off, gamma.data_ptr(), beta.data_ptr(),
                bn.running_mean.data_ptr() if track else None,
                bn.running_var.data_ptr() if track else None,
                bn.num_batches_tracked.data_ptr() if track else None,
                stat.data_ptr(), float(bn.eps), momentum) if defer else None
            yield
        out = torch.empty(n, HIDDEN, dtype=torch.float32, device=dev)
        ro = seg = None
        if readout is not None:
            ptr, nseg, seg_dims = readout
            ro = torch.empty(nseg, HIDDEN, dtype=torch.float32, device=dev)
            seg = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
            _lib.call("scgib_bn_relu_segment_sum", _p(h), _p(stat_prev), _p(ptr), nseg, n,
                      _p(out), _p(ro), _p(seg), _p(seg_dims), _p(graph.dims), _byref(pend), st)
        else:
            _lib.call("scgib_bn_relu_apply", _p(h), _p(stat_prev), n, _p(out), _p(graph.dims),
                      _byref(pend), st)
        ctx.seg = seg
        ctx.save_for_backward(*saved, *params, *( (aggx,) if pre else ()))
        ctx.graph, ctx.L, ctx.training, ctx.pre = graph, L, training, pre
        ctx.n_feat = x.shape[1] if pre else None
        ctx.opes = [c._one_plus_eps for c in gin.ginlayers]
        ctx.cnt_key = "gin_bwd"
        return out if ro is None else (out, ro)

    @staticmethod
    def backward(ctx, g_out, g_readout=None):
        if not isinstance(ctx, _Ctx):  # (the encoder pair sets its sub-contexts' own)
            ctx.need = ctx.needs_input_grad[7:]
        return _drain(_GinEncoder.backward_steps(ctx, g_out, g_readout),
                      getattr(ctx, "stamp_tag", None))

    @staticmethod
    def backward_steps(ctx, g_out, g_readout=None):
        """backward as a generator (yields after each layer), see forward_steps."""
        L, gr, pre = ctx.L, ctx.graph, ctx.pre
        t = ctx.saved_tensors
        saved, params = t[: 4 * L], t[4 * L: 4 * L + 6 * L]
        aggx = t[-1] if pre else None
        if g_readout is not None and ctx.seg is None:
            raise _lib.ScgibError("gin_encoder.backward: readout gradient without a readout")
        if g_out is not None:
            g_out = _f32(g_out, "gin_encoder.backward")
        elif g_readout is None:  # the output is unused
            g_out = torch.zeros_like(saved[2])
        if g_readout is not None:
            g_readout = _f32(g_readout, "gin_encoder.backward readout")
        n = saved[2].shape[0]
        dev = saved[2].device
        st = _stream()
        bn_ws = torch.empty(int(_lib.query("scgib_gin_bn_ws_floats", n)), dtype=torch.float32,
                            device=dev)
        cnt = scan_state(dev, ctx.cnt_key, int(_lib.query("scgib_gin_counters", n)))
        # deferred BN-backward finalize: each layer's gin_bwd_k finishes the sums
        defer = int(DEFER_BN and n <= int(_lib.query("scgib_gin_defer_max_nodes")))
        gpart = bn_ws.data_ptr() + 4 * int(_lib.query("scgib_gin_bn_gpart_offset", n))
        grads = [None] * (6 * L)
        # which parameters take a gradient (the fine-tune freezing quirk,
        # models.py:424-434, leaves most GIN layers frozen): a layer none of
        # whose W1 / b1 / W2 / b2 does runs its backward without the weight
        # products (scgib_gin_layer_bwd need_w = 0; same data gradients, bitwise)
        need = getattr(ctx, "need", None)
        dagg_next, dwt = None, None
        # an agg-free layer l + 1 hands layer l's statistics launch its dz1,
        # W1 and the row of its weight gradient dW1 lands in
        dz1_next = w1_next = wgrad_next = None  # (wgrad_next None: layer l + 1 is frozen)
        nslab = int(_lib.query("scgib_gin_bwd_slabs", n))
        jobs, keep = [], []
        # slab jobs waiting to be reduced by the next statistics launch's extra
        # workgroups (one for scgib_gin_bwd_stats_bn_fold, two for
        # scgib_gin_bwd_stats_z), with their slabs: released once that launch
        # is enqueued (the allocator may then reuse the blocks for later
        # tensors of this stream); whatever is left goes to the final reduce
        pend_jobs = []
        w1_fold = None  # the dW1 partials job for the agg-free layer backward next

        def take_folds(k):
            got = pend_jobs[:k]
            del pend_jobs[:k]
            return got

        for l in reversed(range(L)):
            agg, r, z2, stat = saved[4 * l: 4 * l + 4]  # r None: recomputed by the kernel
            w1, b1, w2 = params[6 * l], params[6 * l + 1], params[6 * l + 2]
            d_in = agg.shape[1] if agg is not None else HIDDEN  # (agg None: an agg-free layer)
            # (the previous layer's dy and slab are no longer read by anything
            # not yet enqueued: released before the new allocations, whose
            # blocks the captured step can then reuse)
            dy = slab = None
            dy = torch.empty(n, HIDDEN, dtype=torch.float32, device=dev)
            bn_g = torch.empty(2, HIDDEN, dtype=torch.float32, device=dev)  # dgamma, dbeta
            coef = torch.empty(2, HIDDEN, dtype=torch.float32, device=dev)
            # dy, tile sums and the BN-backward finalize in one launch
            if dagg_next is None and dz1_next is None and g_readout is not None:
                # the readout's broadcast backward folded into the last layer
                _launch("scgib_gin_bwd_stats_seg_bn", {"n": n, "e": 0, "d_in": HIDDEN}, _p(g_out), _p(g_readout),
                        _p(ctx.seg), _p(z2), _p(stat), n, int(ctx.training), _p(dy),
                        _p(bn_g[0]), _p(bn_g[1]), _p(coef), _p(bn_ws), _p(cnt), _p(gr.dims),
                        defer, st)
            elif dagg_next is None and dz1_next is None:
                # (first_fold: a loss-section slab job handed over by the encoder
                # pair — reduced in extra workgroups here, its slab then released)
                ff = getattr(ctx, "first_fold", None)
                ctx.first_fold = None
                _launch("scgib_gin_bwd_stats_bn_fold", {"n": n, "e": 0, "d_in": HIDDEN}, _p(g_out),
                        None, None, 1.0, _p(z2), _p(stat), n, int(ctx.training), _p(dy),
                        _p(bn_g[0]), _p(bn_g[1]), _p(coef), _p(bn_ws), _p(cnt), _p(gr.dims),
                        defer, _byref(ff[0] if ff else None), st)
                ff = None
            elif dz1_next is not None:
                # layer l + 1 is agg-free: gather its dz1, d h_l = g W1_{l+1},
                # and dW1_{l+1} = g^T h_l as per-workgroup partials
                nz = int(_lib.query("scgib_gin_bwd_stats_z_slabs", n))
                wgn = wgrad_next is not None
                wslab = torch.empty(nz * HIDDEN * HIDDEN, dtype=torch.float32,
                                    device=dev) if wgn else None
                # (no folds when the walk fills the chip's two slots per CU: the
                # extra workgroups would wait for a second wave; the pending jobs
                # then go to the next agg-free layer backward, or the final reduce)
                room = 2 * 256 - nz
                folds = []
                while pend_jobs and room >= (pend_jobs[0][0].width + 63) // 64:
                    room -= (pend_jobs[0][0].width + 63) // 64
                    folds += take_folds(1)
                table = (_lib.SlabJob * max(len(folds), 1))(*[j for j, _ in folds])
                _launch("scgib_gin_bwd_stats_z", {"n": n, "e": gr.edge_capacity(), "d_in": HIDDEN,
                                                  "z": True, "wg": wgn},
                        _p(dz1_next), _p(gr.rowptr_t), _p(gr.col_t), ctx.opes[l + 1],
                        _p(w1_next), _p(z2), _p(stat), n, int(ctx.training), _p(dy), _p(bn_g[0]),
                        _p(bn_g[1]), _p(coef), _p(bn_ws), _p(cnt), _p(gr.dims), defer,
                        _p(wslab), int(wgn), ctypes.cast(table, ctypes.c_void_p), len(folds), st)
                folds = table = None
                if wgn:  # dW1_{l+1} lands after its dW2 | db2 | db1 (wgrad_next's layout)
                    job = _lib.SlabJob(wslab.data_ptr(), wgrad_next.data_ptr() + 4 * _Z_W1_OFF,
                                       HIDDEN * HIDDEN, nz, 0)
                    # (one partial per walking workgroup — per tile at small batches:
                    # reduced by this layer's agg-free backward, the next launch,
                    # whose grid leaves room; else with the chain's final reduce)
                    if FOLD_SLABS and agg is None:
                        w1_fold = (job, wslab)
                    else:
                        jobs.append(job)
                        keep.append(wslab)
                wslab = dz1_next = w1_next = wgrad_next = None
            else:
                folds = take_folds(1)
                _launch("scgib_gin_bwd_stats_bn_fold", {"n": n, "e": gr.edge_capacity(), "d_in": HIDDEN},
                        _p(dagg_next), _p(gr.rowptr_t),
                        _p(gr.col_t), ctx.opes[l + 1], _p(z2), _p(stat), n, int(ctx.training),
                        _p(dy), _p(bn_g[0]), _p(bn_g[1]), _p(coef), _p(bn_ws), _p(cnt),
                        _p(gr.dims), defer, _byref(folds[0][0] if folds else None), st)
                folds = dagg_next = None
            bpend = _lib.BnBwdPending(gpart, bn_g[0].data_ptr(), bn_g[1].data_ptr(),
                                      int(ctx.training)) if defer else None
            meta = {"n": n, "e": gr.edge_capacity(), "d_in": d_in, "r": r is not None}
            w1c, w2c = _f32(w1, "w1"), _f32(w2, "w2")
            b1c = _f32(b1, "b1") if r is None else None
            # (frozen-weight kernels: stored r, d_in = 64 or the layer-0 fold)
            wg = need is None or any(need[6 * l: 6 * l + 4]) or r is None or \
                (d_in != HIDDEN and not (pre and l == 0))
            meta["wg"] = wg
            grads[6 * l + 4] = bn_g[0]
            grads[6 * l + 5] = bn_g[1]
            if agg is None:
                # agg-free: dz1 out, dW2 | db2 | db1 here, dW1 from layer l - 1's
                # statistics launch (always one: l >= 1); a frozen layer (not
                # wg): the same dz1 chain, no weight products
                meta["z"] = True
                nsz = int(_lib.query("scgib_gin_layer_bwd_z_slabs", n))
                slab = torch.empty(nsz * _Z_SLAB, dtype=torch.float32, device=dev) if wg else None
                dz1 = torch.empty(n, HIDDEN, dtype=torch.float32, device=dev)
                f2 = take_folds(1)  # the previous agg-free layer's dW2 | db slab (pend)
                _launch("scgib_gin_layer_bwd_z", meta, _p(dy), _p(z2), _p(r), _p(stat), _p(coef),
                        _p(w2c), n, _p(dz1), _p(slab), int(wg), _p(gr.dims), _byref(bpend),
                        _byref(w1_fold[0] if w1_fold else None), _byref(f2[0][0] if f2 else None),
                        st)
                w1_fold = f2 = None
                wgrad = None
                if wg:
                    wgrad = torch.empty(_Z_SLAB + HIDDEN * HIDDEN, dtype=torch.float32,
                                        device=dev)
                    pend_jobs.append((_lib.SlabJob(slab.data_ptr(), wgrad.data_ptr(), _Z_SLAB,
                                                   nsz, 0), slab))
                    grads[6 * l + 2] = wgrad[:HIDDEN * HIDDEN].view(HIDDEN, HIDDEN)
                    grads[6 * l + 3] = wgrad[HIDDEN * HIDDEN:HIDDEN * HIDDEN + HIDDEN]
                    grads[6 * l + 1] = wgrad[HIDDEN * HIDDEN + HIDDEN:_Z_SLAB]
                    grads[6 * l + 0] = wgrad[_Z_W1_OFF:].view(HIDDEN, HIDDEN)
                dz1_next, w1_next, wgrad_next = dz1, w1c, wgrad
                slab = dz1 = wgrad = None
                yield
                continue
            if pre and l == 0:
                width = int(_lib.query("scgib_gin_layer0_slab_width"))
                # (dwt_row: one spare row whose d Wt columns another encoder's
                # reduce fills — the pair's core chain — so this encoder's
                # final reduce returns the sum of both, _GinEncoderPair)
                xrow = int(getattr(ctx, "dwt_row", False))
                slab = torch.empty((nslab + xrow) * width, dtype=torch.float32, device=dev)
                _launch("scgib_gin_layer0_bwd", meta, _p(dy), _p(z2), _p(r), _p(agg), _p(aggx),
                        ctx.n_feat, _p(stat), _p(coef), _p(w1c), _p(b1c), _p(w2c), n, _p(slab),
                        int(wg), _p(gr.dims), _byref(bpend), st)
                dagg = None
            else:
                width = HIDDEN * HIDDEN + HIDDEN * d_in + 2 * HIDDEN
                slab = torch.empty(int(_lib.query("scgib_gin_slab_floats", n, d_in)),
                                   dtype=torch.float32, device=dev) if wg else None
                dagg = torch.empty(n, d_in, dtype=torch.float32, device=dev)
                _launch("scgib_gin_layer_bwd", meta, _p(dy), _p(z2), _p(r), _p(agg), d_in,
                        _p(stat), _p(coef), _p(w1c), _p(b1c), _p(w2c), n, _p(dagg), _p(slab),
                        _NULL, int(wg), _p(gr.dims), _byref(bpend), st)
            if not wg:  # no weight gradients: only layer 0's dWt (its slab's tail)
                if pre and l == 0:
                    o = HIDDEN * HIDDEN + HIDDEN * d_in + 2 * HIDDEN
                    into = getattr(ctx, "dwt_into", None)
                    if into is None:
                        dwt = torch.empty(32 * ctx.n_feat, dtype=torch.float32, device=dev)
                    jobs.append(_lib.SlabJob(slab.data_ptr() + 4 * o,
                                             into if into is not None else dwt.data_ptr(),
                                             32 * ctx.n_feat, nslab + xrow, width))
                    keep.append(slab)
                    if xrow:
                        ctx.dwt_row_ptr = slab.data_ptr() + 4 * (nslab * width + o)
                        ctx.dwt_row_slab = slab
                    dwt = dwt.view(32, ctx.n_feat) if into is None else None
                dagg_next = dagg
                yield
                continue
            wgrad = torch.empty(width, dtype=torch.float32, device=dev)
            if pre and l == 0:  # dWt occupies 32 * F of its 512 columns
                o = HIDDEN * HIDDEN + HIDDEN * d_in + 2 * HIDDEN
                into = getattr(ctx, "dwt_into", None)
                if into is None and not xrow:
                    jobs.append(_lib.SlabJob(slab.data_ptr(), wgrad.data_ptr(),
                                             o + 32 * ctx.n_feat, nslab, width))
                else:  # dWt as its own job: into another encoder's row / over the spare row
                    jobs.append(_lib.SlabJob(slab.data_ptr(), wgrad.data_ptr(), o, nslab, width))
                    jobs.append(_lib.SlabJob(slab.data_ptr() + 4 * o,
                                             into if into is not None else wgrad.data_ptr() + 4 * o,
                                             32 * ctx.n_feat, nslab + xrow, width))
                if xrow:
                    ctx.dwt_row_ptr = slab.data_ptr() + 4 * (nslab * width + o)
                    ctx.dwt_row_slab = slab
                keep.append(slab)
            else:  # reduced by the next stats launch, or together at the end
                ns = int(_lib.query("scgib_gin_layer_bwd_slabs", n, d_in))
                job = _lib.SlabJob(slab.data_ptr(), wgrad.data_ptr(), width, ns, 0)
                if FOLD_SLABS and l > 0:
                    pend_jobs.append((job, slab))
                else:
                    jobs.append(job)
                    keep.append(slab)
            o = HIDDEN * HIDDEN
            grads[6 * l + 2] = wgrad[:o].view(HIDDEN, HIDDEN)
            grads[6 * l + 0] = wgrad[o:o + HIDDEN * d_in].view(HIDDEN, d_in)
            o += HIDDEN * d_in
            grads[6 * l + 3] = wgrad[o:o + HIDDEN]
            grads[6 * l + 1] = wgrad[o + HIDDEN:o + 2 * HIDDEN]
            if pre and l == 0 and getattr(ctx, "dwt_into", None) is None:
                o += 2 * HIDDEN
                dwt = wgrad[o:o + 32 * ctx.n_feat].view(32, ctx.n_feat)
            dagg_next = dagg
            yield
        for job, sl in pend_jobs:  # (none past layer 0's statistics launch as a rule)
            jobs.append(job)
            keep.append(sl)
        pend_jobs = None
        extra = getattr(ctx, "extra_jobs", None)
        if extra is not None:  # deferred loss-section slabs (SlabScope), same launch
            ctx.extra_jobs = None
            jobs.extend(extra[0])
            keep.extend(extra[1])
        if jobs and getattr(ctx, "defer_final", False):  # enqueued by the caller (the pair)
            ctx.final = (jobs, keep)
        elif jobs:  # every layer's weight-gradient slabs, one fixed-order reduce launch
            _reduce_jobs(jobs, st)
            del keep  # slabs stay allocated until the launch is enqueued
        if pre:
            return (None, None, None, None, None, dwt, None, *grads)
        # d h0 = (1+eps_0) d(agg_0) + sum over out-edges (transposed aggregation)
        dh0 = _aggregate(dagg_next, gr.rowptr_t, gr.col_t, ctx.opes[0], gr.dims)
        return (dh0, None, None, None, None, None, None, *grads)


def gin_encoder(h, graph, gin):
    """models.GIN.forward on the fused HIP layers (train or eval BN)."""
    if graph.num_nodes() == 0:
        raise _lib.ScgibError("gin_encoder on an empty graph")
    return _GinEncoder.apply(h, graph, gin, bool(gin.training), None, None, None,
                             *_gin_layer_params(gin))


def gin_encoder_x(x, graph, gin, transfer, node_map=None):
    """gin(graph, transfer(x[node_map])) with transfer_d (Linear(F, 32),
    no bias) folded into the first fused layer.  ``x`` holds the raw
    normalised features of the parent rows (F <= 16); ``node_map`` maps the
    graph's rows to rows of ``x`` (ego batches: ego.ndata['_ID'])."""
    if graph.num_nodes() == 0:
        raise _lib.ScgibError("gin_encoder on an empty graph")
    if transfer.bias is not None or transfer.weight.shape != (32, x.shape[1]) \
            or x.shape[1] > 16:
        raise _lib.ScgibError("transfer_d fold needs Linear(F <= 16, 32, bias=False)")
    if x.requires_grad:
        raise _lib.ScgibError("transfer_d fold: no gradient w.r.t. the raw features")
    return _GinEncoder.apply(None, graph, gin, bool(gin.training), x, transfer.weight,
                             node_map, *_gin_layer_params(gin))


def gin_hidden(agg, w1, b1):
    """r = relu(agg W1^T + b1) [n, 64] with the GIN forward's own MFMA chain
    (scgib_gin_hidden): bitwise the r a fused layer computes, and the r its
    backward recomputes when the forward did not store it (STORE_R False).
    Inspection / tests (the hidden ReLU decisions of a step)."""
    agg = _f32(agg, "gin_hidden agg")
    w1, b1 = _f32(w1, "gin_hidden w1"), _f32(b1, "gin_hidden b1")
    n, d_in = agg.shape
    if tuple(w1.shape) != (HIDDEN, d_in) or b1.numel() != HIDDEN:
        raise _lib.ScgibError(f"gin_hidden: agg {tuple(agg.shape)}, w1 {tuple(w1.shape)}")
    r = torch.empty(n, HIDDEN, dtype=torch.float32, device=agg.device)
    _lib.call("scgib_gin_hidden", _p(agg), d_in, _p(w1), _p(b1), n, _p(r), _stream())
    return r


class _Ctx:
    """Stand-in ctx so _GinEncoder's forward/backward can run inside another
    Function (the tensors it saves stay referenced by the outer node)."""

    def save_for_backward(self, *t):
        self.saved_tensors = t


# The encoder pair's two mid-step cross-queue hand-offs (forward join, backward
# fork) as a signal / wait kernel pair instead of a stream dependency: in the
# replayed graph a cross-queue edge stalls the waiting queue several us even
# when the producer finished long before (tools/xq_probe.hip).  The
# step's final join stays a stream dependency (the capture must end joined).
# A replayed graph may order a wait before its signal on the same queue, and
# then only concurrent queues let the signal run: off where kernel dispatch is
# serialised device-wide (PMC counter collection, AMD_SERIALIZE_KERNEL, launch
# blocking) — there a wait would time out (counted, xq_timeouts) instead — and
# under rocprofv3 kernel tracing, whose per-dispatch callbacks submit the
# replay's nodes one queue after the other, so a wait holds its queue until
# the other queue's submission catches up (a 0.74 ms traced step; the kernels
# are the same either way, only the synchronisation packets differ).


def _dispatch_serialised(env=None):
    env = os.environ if env is None else env
    return any(env.get(k, "0") not in ("", "0") for k in (
        "ROCPROF_COUNTER_COLLECTION", "ROCPROF_KERNEL_TRACE", "AMD_SERIALIZE_KERNEL",
        "HIP_LAUNCH_BLOCKING", "CUDA_LAUNCH_BLOCKING"))


def _env_int(env, name, default):
    try:
        return int(env.get(name, "") or default)
    except ValueError:
        return default


def handoff_rule(device_count=None, env=None):
    """(ok, reason): may the encoder pair use the signal / wait hand-offs?

    A wait kernel spins until its signal kernel has run, so the two must sit
    on hardware queues the device runs CONCURRENTLY — a replayed graph may
    order the wait before the signal on one in-order queue, and then the wait
    only ends at its 0.2 s bound (counted, the sticky fault set, an error at
    the next host check: check_handoff).  What the hand-offs rely on
    ("Cross-queue hand-offs"): eagerly, `side` and the current
    stream are distinct HIP streams; a replayed graph runs its parallel
    branches (the two encoder chains) on distinct streams the runtime creates
    per device for graph execution (capped by DEBUG_HIP_FORCE_GRAPH_QUEUES);
    the runtime gives each stream one of the process's GPU_MAX_HW_QUEUES
    hardware queues (4 on the pool's boxes), spreading streams over them; the
    command processor runs distinct hardware queues concurrently.  So the
    rule refuses exactly the settings that break one of those links:
      * dispatch serialised device-wide (PMC counter collection, kernel-trace
        callbacks, AMD_SERIALIZE_KERNEL, blocking launches);
      * GPU_MAX_HW_QUEUES < 2 (every stream of the process on one queue);
      * DEBUG_HIP_FORCE_GRAPH_QUEUES < 2 (a replayed graph on one stream);
      * more local ranks than devices (ranks sharing a GPU are time-sliced
        processes: their queues need not run at the same time) —
        LOCAL_WORLD_SIZE against the local device count, not the global
        world size (a multi-node job keeps its hand-offs).
    Measured support for the rest: every replay of the GPU suite and of the
    benches asserts zero timed-out waits (ops.xq_timeouts)."""
    env = os.environ if env is None else env
    if _dispatch_serialised(env):
        return False, "kernel dispatch is serialised device-wide (profiling / blocking launches)"
    hw = _env_int(env, "GPU_MAX_HW_QUEUES", 4)
    if hw < 2:
        return False, f"GPU_MAX_HW_QUEUES={hw}: every stream shares one hardware queue"
    gq = _env_int(env, "DEBUG_HIP_FORCE_GRAPH_QUEUES", 0)
    if 0 < gq < 2:
        return False, f"DEBUG_HIP_FORCE_GRAPH_QUEUES={gq}: a replayed graph runs on one stream"
    local = _env_int(env, "LOCAL_WORLD_SIZE", 1)
    if device_count is not None and local > max(int(device_count), 1):
        return False, (f"{local} local ranks on {device_count} device(s): ranks sharing a GPU "
                       "are time-sliced, their queues need not run concurrently")
    return True, f"{hw} hardware queues per process, graph branches on distinct streams"


# None: resolved on first use by xq_enabled() — with the local device count,
# so that ranks sharing a GPU (LOCAL_WORLD_SIZE > devices) get stream edges
# whatever entry point they came in by; True / False set by a caller (bench
# --no-handoffs, tests) stands
XQ_FLAGS, XQ_REASON = None, "not resolved yet (xq_enabled)"


def xq_enabled():
    """Whether the encoder pair's hand-offs are signal / wait kernels: the
    rule (handoff_rule) with this process's environment and local device
    count, resolved once, unless a caller set XQ_FLAGS."""
    global XQ_FLAGS, XQ_REASON
    if XQ_FLAGS is None:
        XQ_FLAGS, XQ_REASON = handoff_rule(torch.cuda.device_count())
    return XQ_FLAGS


def _xq_words(device, key):
    """Four zeroed uint32 for one signal / wait pair: the same words whichever
    stream asks (counters() keys by stream)."""
    with torch.cuda.stream(torch.cuda.default_stream(device)):
        return counters(device, ("xq", key), 4)


def handoff_fault_word(device):
    """The device's sticky hand-off fault word: a wait that gave up sets it,
    and the pretraining loss kernels (scgib_mlp2_recon(_contrastive)_fwd)
    report a NaN recon loss while it is set — a pretraining step whose
    kernels may have read unwritten data never yields a finite loss.  The
    fine-tune and domain-adaptation heads end in torch losses (NaN scores
    would trip binary_cross_entropy's device-side range assert): they rely
    on the host check instead (check_handoff, at the next forward / optimizer
    step).  One word per device, whichever stream asks."""
    with torch.cuda.stream(torch.cuda.default_stream(device)):
        return counters(device, "handoff_fault", 1)


_HOST_FAULT = {}  # device index -> pinned int32 [1]: set by a wait that gave up


def _host_fault_word(device):
    """A pinned host word the wait kernel also sets when it gives up (a
    system-scope store): the host reads it without synchronising."""
    idx = torch.device(device).index or 0
    w = _HOST_FAULT.get(idx)
    if w is None:
        if torch.cuda.is_current_stream_capturing():
            raise _lib.ScgibError("hand-off fault words must be created outside graph capture "
                                  "(run one eager step first)")
        w = _HOST_FAULT[idx] = torch.zeros(1, dtype=torch.int32).pin_memory()
    return w


def check_handoff(device=None):
    """Raise ScgibError if a cross-queue hand-off wait has given up on
    ``device`` (every device used so far when None).  Host-side and free (a
    pinned word, no sync), so it runs at every model forward
    (ops.aside_guard) and optimizer step (optim.Adam.step): the first of them
    after a step whose wait timed out raises — that step's own loss is
    already NaN.  After fixing the cause, clear_handoff_fault()."""
    idx = None if device is None else (torch.device(device).index or 0)
    for d, w in _HOST_FAULT.items():
        if (idx is None or d == idx) and int(w[0]) != 0:
            raise _lib.ScgibError(
                f"cuda:{d}: a cross-queue hand-off wait of the GIN encoder pair (ops._xq_handoff: "
                "scgib_stream_signal / scgib_stream_wait) gave up after 0.2 s — its signal "
                "kernel was not scheduled concurrently, so kernels of that step may have read "
                "data before it was written (its loss is NaN).  Hand-off rule: "
                f"{handoff_rule()[1]}; run with ops.XQ_FLAGS = False if this setup time-slices "
                "the queues, then ops.clear_handoff_fault(device)")


def handoff_fault(device):
    """True once a hand-off wait on ``device`` has given up (sticky)."""
    return bool(handoff_fault_word(device).item())


def clear_handoff_fault(device):
    handoff_fault_word(device).zero_()
    _host_fault_word(device).zero_()


def _xq_handoff(producer, consumer, key):
    """Order ``consumer``'s later work after ``producer``'s work so far
    (scgib_stream_signal on producer, scgib_stream_wait on consumer)."""
    w = _xq_words(producer.device, key)
    fault = handoff_fault_word(producer.device)
    host = _host_fault_word(producer.device)
    with torch.cuda.stream(producer):
        _lib.call("scgib_stream_signal", _p(w), _stream())
    with torch.cuda.stream(consumer):
        _lib.call("scgib_stream_wait", _p(w), _p(fault), _p(host), _stream())


def xq_timeouts(device):
    """Waits of the encoder pair's hand-offs that gave up (0 = every wait saw
    its signal; a non-zero count means the two kernels shared a queue)."""
    idx = torch.device(device).index or 0
    split = sum(s.timeouts() for s in list(_LIVE_SPLITS)
                if s._handle and (s.device.index or 0) == idx)
    return split + sum(int(_xq_words(device, k)[2].item()) for k in ("pair_fwd", "pair_bwd"))


class _GinEncoderPair(torch.autograd.Function):
    """Encoder2 (ego-net batch, on ``side``) and Encoder1 (core batch, on the
    current stream) with transfer_d folded into both first layers, as ONE
    autograd node.  Two separate nodes would make the autograd engine run
    Encoder1's backward first (it was created later), and the cross-stream
    event then makes the ego chain — the longer one — wait for all of it.
    Here the ego backward is enqueued first on ``side`` and the two chains
    overlap in both directions; d Wt = d Wt(ego) + d Wt(core)."""

    @staticmethod
    def forward(ctx, x, wt, w0, b0, nmap, ego, core, gin_ego, gin_core, training, side, tails,
                *params):
        main = _torch_stream()
        core_tail, side_tail, bwd_tail = tails
        ctx.side_tail, ctx.bwd_tail = side_tail, bwd_tail
        ne = 6 * len(gin_ego.ginlayers)
        ctx.set_materialize_grads(False)  # unused outputs (e.g. s) get no zero-fill launch
        # the loss-section reduces of this step are deferred into this node's
        # backward (SlabScope); only when the node will have a backward
        grad = any(isinstance(p, torch.Tensor) and p.requires_grad for p in (wt, w0, b0, *params))
        ctx.scope = SlabScope() if (DEFER_LOSS_REDUCE and grad) else None
        _SLAB_SCOPE[0] = ctx.scope
        ctx.sub = (_Ctx(), _Ctx())
        ctx.side, ctx.ne = side, ne
        check_fork(main)
        ctx.lin = w0 is not None
        ctx.lin_leaves = (w0, b0)
        side.wait_stream(main)
        stamp("fwd.fork[main]")
        with torch.cuda.stream(side):
            stamp("fwd.start[side]")
        if core_tail is not None:  # beside the ego-net build
            core_tail()
        # Encoder2 + its readout (dgl.sum_nodes per ego-net) on ``side``,
        # Encoder1 on the current stream, one chain after the other
        ego_steps = _GinEncoder.forward_steps(
            ctx.sub[0], None, ego, gin_ego, training, x, wt, nmap, *params[:ne],
            readout=(ego.graph_ptr, ego.batch_size, ego.seg_dims))
        core_steps = _GinEncoder.forward_steps(ctx.sub[1], None, core, gin_core, training, x, wt,
                                               None, *params[ne:])
        with torch.cuda.stream(side):
            s, ro = _drain(ego_steps, "fwd.ego")
            stamp("fwd.ego_end[side]")
        f = _drain(core_steps, "fwd.core")
        stamp("fwd.core_end[main]")
        outs = (s, ro, f)
        if ctx.lin:  # compressor[0] on the (shorter) core chain, before the join
            w0, b0 = _f32(w0, "compressor.0.weight"), _f32(b0, "compressor.0.bias")
            if tuple(w0.shape) != (HIDDEN, HIDDEN):
                raise _lib.ScgibError("compressor[0] must be Linear(64, 64)")
            t = torch.empty_like(f)
            _lib.call("scgib_linear_fwd", _p(f), f.shape[0], _p(w0), _p(b0), _p(t),
                      _p(core.dims), _stream())
            # (an alias, not the output object itself: ctx -> output -> its
            # grad_fn -> ctx would be a reference cycle that keeps this step's
            # graph, AccumulateGrad nodes included, alive until a gc pass)
            ctx.lin_saved = (f.detach(), w0)
            ctx.core_dims = core.dims
            outs = (s, ro, f, t)
        if xq_enabled():
            _xq_handoff(side, main, "pair_fwd")
        else:
            main.wait_stream(side)
        stamp("fwd.joined[main]")
        if side_tail is not None:
            # after the hand-off: ``side`` idles through the loss section; the
            # backward's core chain follows it there and joins main at its end
            with torch.cuda.stream(side):
                side_tail()
        s.record_stream(main)
        ro.record_stream(main)
        return outs

    @staticmethod
    def backward(ctx, g_s, g_ro, g_f, g_t=None):
        # backward: the ego chain (the longer one) stays on the current stream,
        # where its weight-gradient reduces can fork to the aux stream (a fork
        # from an already-forked stream breaks HIP-graph capture on this
        # runtime, tools/capture_probe.py); Encoder1 runs on ``side``, preceded
        # by compressor[0]'s backward (d f += d t W0, dW0, db0)
        main, side = _torch_stream(), ctx.side
        check_fork(main)
        stamp("bwd.start[main]")
        if xq_enabled():
            _xq_handoff(main, side, "pair_bwd")
        else:
            side.wait_stream(main)
        with torch.cuda.stream(side):
            stamp("bwd.start[side]")
        # Encoder1's final weight-gradient reduce runs beside the ego chain's
        # last layers; it also sums the loss section's deferred slabs
        # (SlabScope: the head MLP's and the interaction's, enqueued on the
        # main stream before this fork, and compressor[0]'s below) — Encoder1's
        # chain ends well before the ego chain's, so they leave the critical path
        scope = ctx.scope if (ctx.scope is not None and ctx.scope.open) else None
        held = None
        need = ctx.needs_input_grad[12:]  # the two encoders' parameters (frozen ones skip dW)
        ctx.sub[0].need, ctx.sub[1].need = need[:ctx.ne], need[ctx.ne:]
        dw0 = db0 = None
        g_f_in = g_f
        # the critical ego chain is captured first: the replayed graph then
        # puts it on the interaction's queue (round 2: 0.4381 -> 0.4326 ms)
        ctx.sub[0].stamp_tag = "bwd.ego"
        # d Wt = d Wt(ego) + d Wt(core) without a separate add after the join:
        # the core chain's reduce writes its d Wt into a spare row of the ego
        # layer-0 slab, and the ego chain's final reduce — enqueued after the
        # join, which costs nothing there (the core chain ends first) — sums
        # it with the ego's rows
        ctx.sub[0].dwt_row = ctx.sub[0].defer_final = True
        later = scope.take_later() if scope is not None else []
        ge = _GinEncoder.backward(ctx.sub[0], g_s, g_ro)
        for launch, _ in later:  # deferred weight-gradient launches, after the ego chain
            launch()
        later = None
        stamp("bwd.ego_end[main]")
        row = getattr(ctx.sub[0], "dwt_row_ptr", None)
        if row is not None:
            ctx.sub[1].dwt_into = row
            ctx.sub[0].dwt_row_slab.record_stream(side)
        with torch.cuda.stream(side):
            if ctx.lin and g_t is not None:
                f, w0 = ctx.lin_saved
                g_t = _f32(g_t, "compressor.0 grad")
                n = f.shape[0]
                slab = torch.empty(int(_lib.query("scgib_linear_slab_floats", n)),
                                   dtype=torch.float32, device=f.device)
                wg = torch.empty(HIDDEN * HIDDEN + HIDDEN, dtype=torch.float32, device=f.device)
                df_total = torch.empty_like(f)
                lin_defer = scope is not None and scope.usable(ctx.lin_leaves)
                _lib.call("scgib_linear_bwd", _p(g_t), _p(f), _p(w0), n,
                          _p(_f32(g_f, "g_f")) if g_f is not None else None, _p(df_total),
                          _p(slab), None if lin_defer else _p(wg), _p(ctx.core_dims), _stream())
                if lin_defer:
                    scope.add(slab, wg, wg.numel(), slab.numel() // wg.numel())
                dw0, db0 = wg[: HIDDEN * HIDDEN].view(HIDDEN, HIDDEN), wg[HIDDEN * HIDDEN:]
                g_f = df_total
            if scope is not None:
                jobs, keep = scope.take()
                for tsr in keep:  # made on the main stream, reduced / written on side
                    tsr.record_stream(side)
                # ... and referenced until after the join below: a block made on
                # main and read on side is not returned to the allocator while
                # later main-stream work could be handed it unordered (in a
                # captured step `record_stream` alone does not order the reuse)
                held = list(keep)
                if jobs and FOLD_SLABS:  # the largest (the head MLP's) into Encoder1's first launch
                    big = max(range(len(jobs)), key=lambda i: jobs[i].width * jobs[i].n_slabs)
                    ctx.sub[1].first_fold = (jobs[big], keep[2 * big: 2 * big + 2])
                    jobs = jobs[:big] + jobs[big + 1:]
                    keep = keep[:2 * big] + keep[2 * big + 2:]
                ctx.sub[1].extra_jobs = (jobs, keep)
            gc = _drain(_GinEncoder.backward_steps(ctx.sub[1], g_f), "bwd.core")
            if ctx.bwd_tail is not None:  # e.g. NoisePrefetch.draw: the next step's noise
                ctx.bwd_tail()
            stamp("bwd.core_end[side]")
        main.wait_stream(side)
        stamp("bwd.joined[main]")
        final = getattr(ctx.sub[0], "final", None)
        if final is not None:  # the ego chain's weight-gradient reduce, d Wt(core) included
            ctx.sub[0].final = None
            if _FINAL_ARMED[0]:  # left to the optimizer step that follows (fuse_final_into_step)
                _FINAL_PENDING.setdefault(main.device_index or 0, []).append(final)
            else:
                _reduce_jobs(final[0], _stream())
            final = None
        ctx.sub[0].dwt_row_slab = None
        if ctx.side_tail is not None and hasattr(ctx.side_tail, "joined"):
            ctx.side_tail.joined()  # ordered before main's later work by the join above
        held = None  # after the join: main-stream reuse is ordered after side's reads
        for g in (*gc, dw0, db0):
            if isinstance(g, torch.Tensor):
                g.record_stream(main)
        if g_f_in is not None:
            g_f_in.record_stream(side)
        if g_t is not None:
            g_t.record_stream(side)
        dwt = ge[5] if gc[5] is None else ge[5] + gc[5]  # (gc[5] None: summed by the reduce)
        return (None, dwt, dw0, db0, None, None, None, None, None, None, None, None, *ge[7:],
                *gc[7:])


def _torch_stream():
    return torch.cuda.current_stream()


def gin_encoder_pair_x(x, ego, gin_ego, core, gin_core, transfer, node_map, side, lin0=None,
                       core_tail=None, side_tail=None, bwd_tail=None):
    """(s, sum_nodes(ego, s), f) with s = gin_ego(ego, transfer(x[node_map])) and
    f = gin_core(core, transfer(x)) — the two encoders of Mainmodel.forward
    with transfer_d folded, and the ego-net readout fused into Encoder2's last
    BN + ReLU; the ego chain on stream ``side`` (forward and backward).  With ``lin0`` (the
    compressor's Linear(64, 64), models.py:596) also returns
    t = lin0(gin_core(...)), computed at the end of the core chain;
    ``core_tail()`` (non-differentiable, e.g. the noise draw) runs first on
    the core chain, beside the ego-net build; ``side_tail()`` (e.g.
    graph.EgoPrefetch: the next batch's ego-net build) runs on ``side`` after
    the ego chain's hand-off, and its ``joined()`` is called once the
    backward has joined ``side`` back; ``bwd_tail()`` (e.g.
    NoisePrefetch.draw) runs on ``side`` at the end of the backward's core
    chain, before that join."""
    if ego.num_nodes() == 0 or core.num_nodes() == 0:
        raise _lib.ScgibError("gin_encoder on an empty graph")
    if transfer.bias is not None or transfer.weight.shape != (32, x.shape[1]) \
            or x.shape[1] > 16:
        raise _lib.ScgibError("transfer_d fold needs Linear(F <= 16, 32, bias=False)")
    if x.requires_grad:
        raise _lib.ScgibError("transfer_d fold: no gradient w.r.t. the raw features")
    if bool(gin_ego.training) != bool(gin_core.training):
        raise _lib.ScgibError("gin_encoder_pair_x: encoders in different train/eval modes")
    w0, b0 = (lin0.weight, lin0.bias) if lin0 is not None else (None, None)
    return _GinEncoderPair.apply(x, transfer.weight, w0, b0, node_map, ego, core, gin_ego,
                                 gin_core, bool(gin_core.training), side,
                                 (core_tail, side_tail, bwd_tail),
                                 *_gin_layer_params(gin_ego), *_gin_layer_params(gin_core))


# ---------------------------------------------------------------------------
# A6: segment sums (dgl.sum_nodes)
# ---------------------------------------------------------------------------
class _SegmentSum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, ptr, nseg, dims):
        x = _f32(x, "segment_sum")
        out = torch.empty(nseg, x.shape[1], dtype=torch.float32, device=x.device)
        _lib.call("scgib_segment_sum", _p(x), _p(ptr), nseg, x.shape[1], _p(out), _p(dims),
                  _stream())
        ctx.ptr, ctx.nrows, ctx.dims = ptr, x.shape[0], dims
        return out

    @staticmethod
    def backward(ctx, g):
        g = _f32(g, "segment_sum.backward")
        out = torch.empty(ctx.nrows, g.shape[1], dtype=torch.float32, device=g.device)
        _lib.call("scgib_segment_broadcast", _p(g), _p(ctx.ptr), g.shape[0], g.shape[1],
                  _p(out), ctx.nrows, _p(ctx.dims), _stream())
        return out, None, None, None


def segment_sum(x, ptr, nseg, dims=None):
    """out[s] = sum of rows [ptr[s], ptr[s+1]) (dgl.sum_nodes); ``dims`` (device,
    capacity mode) holds the actual segment count."""
    return _SegmentSum.apply(x, ptr, int(nseg), dims)


def sum_nodes_graph(graph, x):
    """dgl.sum_nodes(graph, feat) on a GraphBatch."""
    return segment_sum(x, graph.graph_ptr, graph.batch_size)


class _Set2Set(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w_ih, b_ih, w_hh, b_hh, ptr, nseg, n_iters):
        x = _f32(x, "set2set x")
        d = x.shape[1] if x.dim() == 2 else -1
        w_ih, w_hh = _f32(w_ih, "lstm.weight_ih_l0"), _f32(w_hh, "lstm.weight_hh_l0")
        b_ih, b_hh = _f32(b_ih, "lstm.bias_ih_l0"), _f32(b_hh, "lstm.bias_hh_l0")
        if not (1 <= d <= 64) or tuple(w_ih.shape) != (4 * d, 2 * d) or \
                tuple(w_hh.shape) != (4 * d, d) or b_ih.numel() != 4 * d or b_hh.numel() != 4 * d:
            raise _lib.ScgibError(f"set2set: x {tuple(x.shape)} (width <= 64), w_ih "
                                  f"{tuple(w_ih.shape)}, w_hh {tuple(w_hh.shape)}")
        ctx.leaves = (w_ih, b_ih, w_hh, b_hh)
        ctx.scope = _slab_scope_for(ctx.leaves)
        save = torch.empty(max(int(_lib.query("scgib_set2set_save_floats", nseg, d, n_iters)), 1),
                           dtype=torch.float32, device=x.device)
        out = torch.empty(nseg, 2 * d, dtype=torch.float32, device=x.device)
        _lib.call("scgib_set2set_fwd", _p(x), _p(ptr), nseg, d, n_iters, _p(w_ih), _p(b_ih),
                  _p(w_hh), _p(b_hh), _p(save), _p(out), _stream())
        ctx.save_for_backward(x, w_ih, w_hh, save)
        ctx.ptr, ctx.nseg, ctx.n_iters = ptr, nseg, n_iters
        return out

    @staticmethod
    def backward(ctx, g):
        x, w_ih, w_hh, save = ctx.saved_tensors
        g = _f32(g, "set2set.backward")
        d = x.shape[1]
        dx = torch.empty_like(x)
        dgates = torch.empty(max(ctx.nseg * ctx.n_iters * 4 * d, 1), dtype=torch.float32,
                             device=x.device)
        # the four weight gradients as views of one buffer: autograd then takes
        # the views themselves as .grad (a gradient tensor referenced elsewhere
        # is copied at accumulation), while the deferred launch keeps the buffer
        n_ih, n_hh = 4 * d * 2 * d, 4 * d * d
        wbuf = torch.empty(n_ih + n_hh + 8 * d, dtype=torch.float32, device=x.device)
        dw_ih = wbuf[:n_ih].view(4 * d, 2 * d)
        dw_hh = wbuf[n_ih:n_ih + n_hh].view(4 * d, d)
        db_ih = wbuf[n_ih + n_hh:n_ih + n_hh + 4 * d]
        db_hh = wbuf[n_ih + n_hh + 4 * d:]
        ptrs = (dw_ih.data_ptr(), dw_hh.data_ptr(), db_ih.data_ptr(), db_hh.data_ptr())
        # the LSTM weight gradients: deferred past the encoders' backward when
        # the encoder pair's scope can take them (nothing reads them before the
        # optimizer), else in the same call
        scope = getattr(ctx, "scope", None)
        defer = scope is not None and scope.usable(ctx.leaves)
        wg = (None,) * 4 if defer else tuple(ctypes.c_void_p(v) for v in ptrs)
        _lib.call("scgib_set2set_bwd", _p(x), _p(ctx.ptr), ctx.nseg, d, ctx.n_iters, _p(w_ih),
                  _p(w_hh), _p(save), _p(g), _p(dx), x.shape[0], _p(dgates), *wg, _stream())
        if defer:
            args = (_p(save), _p(dgates), ctx.nseg, d, ctx.n_iters,
                    *(ctypes.c_void_p(v) for v in ptrs))
            scope.defer(lambda: _lib.call("scgib_set2set_wgrad", *args, _stream()),
                        save, dgates, wbuf)
        return dx, dw_ih, db_ih, dw_hh, db_hh, None, None, None


def set2set(x, graph, lstm, n_iters):
    """DGL Set2Set(d, n_iters, 1) (models.py:565) on the device: the LSTM
    recurrence and the per-graph softmax attention readouts of all n_iters
    rounds in one launch (scgib_set2set_fwd); ``lstm`` = the module's
    nn.LSTM (its parameters)."""
    return _Set2Set.apply(x, lstm.weight_ih_l0, lstm.bias_ih_l0, lstm.weight_hh_l0,
                          lstm.bias_hh_l0, graph.graph_ptr, int(graph.batch_size), int(n_iters))


# ---------------------------------------------------------------------------
# (f)1: fine-tune prediction head + BCE (models.py:510-523), csrc/head.hip
# ---------------------------------------------------------------------------
class _PredictHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, sigmoid):
        x = _f32(x, "predict head x")
        w1, b1, w2, b2 = (_f32(t, "predict head params") for t in (w1, b1, w2, b2))
        n, k = x.shape
        c = w2.shape[0]
        hid = torch.empty(n, HIDDEN, dtype=torch.float32, device=x.device)
        out = torch.empty(n, c, dtype=torch.float32, device=x.device)
        # the compressor BN running update left by the interaction forward (inside
        # a model forward): one extra workgroup of this launch, not an aux launch
        ru = take_running_update()
        _lib.call("scgib_head_fwd", _p(x), n, k, _p(w1), _p(b1), _p(w2), _p(b2), c, int(sigmoid),
                  _p(hid), _p(out), _byref(ru[0] if ru else None), _stream())
        ctx.save_for_backward(x, hid, out, w1, w2)
        ctx.sigmoid = bool(sigmoid)
        return out

    @staticmethod
    def backward(ctx, g):
        x, hid, out, w1, w2 = ctx.saved_tensors
        g = _f32(g, "predict head grad")
        n, k = x.shape
        c = w2.shape[0]
        dx, dw1, dw2 = torch.empty_like(x), torch.empty_like(w1), torch.empty_like(w2)
        db1 = torch.empty(HIDDEN, dtype=torch.float32, device=x.device)
        db2 = torch.empty(c, dtype=torch.float32, device=x.device)
        _lib.call("scgib_head_bwd", _p(x), _p(hid), _p(out), _p(g), n, k, _p(w1), _p(w2), c,
                  int(ctx.sigmoid), _p(dx), _p(dw1), _p(db1), _p(dw2), _p(db2), _stream())
        return dx, dw1, db1, dw2, db2, None


def predict_head_ok(x, seq):
    """Whether ``seq`` is the fine-tune head the kernels implement:
    Sequential(Linear(K <= 128, 64), ReLU, Linear(64, C <= 16)) on a [B, K]
    HIP tensor, K a multiple of 4."""
    import torch.nn as nn
    return (x.is_cuda and x.dim() == 2 and len(seq) == 3 and isinstance(seq[0], nn.Linear)
            and isinstance(seq[1], nn.ReLU) and isinstance(seq[2], nn.Linear)
            and seq[0].bias is not None and seq[2].bias is not None
            and seq[0].out_features == HIDDEN and seq[2].in_features == HIDDEN
            and x.shape[1] == seq[0].in_features and 1 <= x.shape[1] <= 128
            and x.shape[1] % 4 == 0 and 1 <= seq[2].out_features <= 16)


def predict_head(x, seq, sigmoid):
    """``sigmoid(seq(x))`` (or ``seq(x)``) for the fine-tune head
    Sequential(Linear, ReLU, Linear) (models.py:510-520: predict, then the
    sigmoid unless the dataset is a regression one) in one launch forward
    and one backward (scgib_head_fwd / _bwd) instead of ~12 torch launches."""
    return _PredictHead.apply(x, seq[0].weight, seq[0].bias, seq[2].weight, seq[2].bias,
                              bool(sigmoid))


class _BceMean(torch.autograd.Function):
    @staticmethod
    def forward(ctx, s, t):
        s, t = _f32(s, "bce scores"), _f32(t, "bce targets")
        loss = torch.empty((), dtype=torch.float32, device=s.device)
        _lib.call("scgib_bce_fwd", _p(s), _p(t), s.numel(), _p(loss), _stream())
        ctx.save_for_backward(s, t)
        return loss

    @staticmethod
    def backward(ctx, g):
        s, t = ctx.saved_tensors
        ds = torch.empty_like(s)
        _lib.call("scgib_bce_bwd", _p(s), _p(t), s.numel(), _p(_f32(g.reshape(1), "bce grad")),
                  _p(ds), _stream())
        return ds, None


def bce_mean(scores, targets):
    """F.binary_cross_entropy(scores, targets) (mean) in one launch each way
    (scgib_bce_fwd / _bwd: torch's per-element formula, its log clamp at
    -100 and its backward's 1e-12 floor; fp64 fixed-order sum)."""
    if scores.shape != targets.shape:
        raise _lib.ScgibError(f"bce: scores {tuple(scores.shape)} vs targets {tuple(targets.shape)}")
    return _BceMean.apply(scores, targets)


# ---------------------------------------------------------------------------
# A6-A8: fused core <-> subgraph interaction
# ---------------------------------------------------------------------------
def _interaction_forward(ctx, f, t, s, u_gate, u_feat, gamma, beta, w2, b2, w_att, b_att, graph,
                         bn, training):
    """Launch scgib_interaction_fwd (+ the BN running update); stores on ctx
    what the backward needs and returns (outputs, tensors to save)."""
    u_gate, u_feat = _f32(u_gate, "interaction"), _f32(u_feat, "interaction")
    n, d = f.shape
    if d != HIDDEN:
        raise _lib.ScgibError(f"interaction kernels are built for hidden={HIDDEN}, got {d}")
    B = graph.batch_size
    pad = graph.dims is not None  # capacity mode: n is the row capacity
    n_last = None
    if not pad:
        counts = graph.batch_num_nodes_host()
        if training and B and counts.min() < 2:
            # nn.BatchNorm1d raises on a 1-row batch in train mode (models.py:642)
            raise ValueError("Expected more than 1 value per channel when training "
                             "(a graph with a single node in the per-graph compressor BN)")
        n_last = int(counts[-1]) if B else 0
    dev = f.device
    im = torch.empty(n, 2 * HIDDEN, dtype=torch.float32, device=dev)
    z1 = torch.empty(B, HIDDEN, dtype=torch.float32, device=dev)
    z2 = torch.empty(B, HIDDEN, dtype=torch.float32, device=dev)
    lam = torch.empty(n, dtype=torch.float32, device=dev)
    logit = torch.empty(n, dtype=torch.float32, device=dev)
    stats = torch.empty(max(B, 1), STATS_STRIDE, dtype=torch.float32, device=dev)
    kl = None if pad else torch.empty(2 * n_last, HIDDEN, dtype=torch.float32, device=dev)
    kl_mean = torch.empty((), dtype=torch.float32, device=dev)
    gamma, beta = _f32(gamma, "bn.weight"), _f32(beta, "bn.bias")
    w2, b2 = _f32(w2, "w2"), _f32(b2, "b2")
    w_att, b_att = _f32(w_att, "w_att"), _f32(b_att, "b_att")
    rm, rv = bn.running_mean, bn.running_var
    st = _stream()
    _launch("scgib_interaction_fwd", {"n": n, "B": B}, _p(f), _p(t), _p(s), _p(u_gate), _p(u_feat),
              _p(graph.graph_ptr), B, n, _p(gamma), _p(beta), _p(rm), _p(rv), float(bn.eps),
              int(training), _p(w2), _p(b2), _p(w_att), _p(b_att), _p(im), _p(z1), _p(z2),
              _p(lam), _p(logit), _p(stats), _p(kl), _p(kl_mean), int(pad), st)
    if training and bn.track_running_stats:
        nbt = bn.num_batches_tracked

        def upd():  # B sequential momentum updates in closed form
            _lib.call("scgib_bn_running_update", _p(stats), _p(graph.graph_ptr), B,
                      float(bn.momentum), _p(rm), _p(rv), _p(nbt), _stream())
        # nothing in the step reads them.  Inside a model forward the loss
        # head's launch runs it in one extra workgroup of its finishing kernel
        # (scgib_mlp2_recon_contrastive_fwd: no second stream, no fork / join
        # edges); if no such launch follows, join_aside puts it on the aux
        # stream.  A standalone op call updates inline.
        if _DEFER_DEPTH[0] > 0:
            ru = _lib.RunningUpdate(stats.data_ptr(), graph.graph_ptr.data_ptr(), B,
                                    float(bn.momentum), rm.data_ptr(), rv.data_ptr(),
                                    nbt.data_ptr())
            _PENDING_RU[0] = (ru, upd, (stats, graph.graph_ptr))
        else:
            upd()
    ctx.graph, ctx.training, ctx.pad, ctx.n_last = graph, training, pad, n_last
    ctx.bn_eps = float(bn.eps)
    ctx.rm, ctx.rv = (None, None) if training else (rm.clone(), rv.clone())
    if kl is None:
        kl = torch.zeros(0, HIDDEN, dtype=torch.float32, device=dev)
    return (im, z1, z2, kl, kl_mean), (f, t, s, u_feat, gamma, beta, w2, w_att, z1, lam, logit,
                                       stats)


def _interaction_backward(ctx, saved, g_im, g_z1, g_z2, g_kl, g_klmean):
    """scgib_interaction_bwd + the fixed-order sum of the per-graph parameter
    gradients.  Returns df, dt, ds and the parameter gradients."""
    f, t, s, u_feat, gamma, beta, w2, w_att, z1, lam, logit, stats = saved
    n = f.shape[0]
    B = ctx.graph.batch_size
    dev = f.device
    zeros = lambda *shape: torch.zeros(*shape, dtype=torch.float32, device=dev)  # noqa: E731
    g_im = zeros(n, 2 * HIDDEN) if g_im is None else _f32(g_im, "g_im")
    # (no gradient for a readout: the kernel reads NULL as zero, no fill launch)
    g_z1 = None if g_z1 is None else _f32(g_z1, "g_z1")
    g_z2 = None if g_z2 is None else _f32(g_z2, "g_z2")
    if g_kl is not None and g_kl.numel() == 0:
        g_kl = None
    if g_kl is not None:
        g_kl = _f32(g_kl, "g_kl")
        if g_klmean is not None:  # fold the mean's gradient into the tensor's
            g_kl = g_kl + g_klmean / (2 * ctx.n_last * HIDDEN)
            g_klmean = None
    if g_klmean is not None:
        g_klmean = _f32(g_klmean.reshape(1), "g_klmean")
    df = torch.empty_like(f)
    dt = torch.empty_like(t)
    ds = torch.empty_like(s)
    pgrad = torch.empty(max(B, 1), PGRAD_STRIDE, dtype=torch.float32, device=dev)
    pg = torch.empty(PGRAD_STRIDE, dtype=torch.float32, device=dev)
    scope = getattr(ctx, "scope", None)
    defer = B > 0 and scope is not None and scope.usable(ctx.leaves)
    _launch("scgib_interaction_bwd", {"n": n, "B": B}, _p(g_im), _p(g_z1), _p(g_z2), _p(g_kl), _p(f), _p(t),
              _p(s), _p(u_feat), _p(ctx.graph.graph_ptr), B, n, _p(gamma), _p(beta),
              _p(ctx.rm), _p(ctx.rv), ctx.bn_eps, int(ctx.training), _p(w2), _p(w_att),
              _p(z1), _p(lam), _p(logit), _p(stats), _p(df), _p(dt), _p(ds), _p(pgrad),
              _p(g_klmean), int(ctx.pad), None if defer else _p(pg), _stream())
    if defer:  # the per-graph partials are summed by the encoder pair's backward
        scope.add(pgrad, pg, PGRAD_STRIDE, B)
    grads = (pg[65:129], pg[129:193], pg[0:64].view(1, 64), pg[64:65],
             pg[193:321].view(1, 128), pg[321:322])  # dgamma dbeta dW2 db2 dWatt dbatt
    return df, dt, ds, grads


class _Interaction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, f, t, s, u_gate, u_feat, gamma, beta, w2, b2, w_att, b_att, graph, bn,
                training):
        ctx.set_materialize_grads(False)  # outputs no loss reads (fine-tune: z1, z2, KL): no fills
        ctx.leaves = (gamma, beta, w2, b2, w_att, b_att)
        ctx.scope = _slab_scope_for(ctx.leaves)
        f = _f32(f, "interaction")
        t, s = _f32(t, "interaction"), _f32(s, "interaction")
        outs, saved = _interaction_forward(ctx, f, t, s, u_gate, u_feat, gamma, beta, w2, b2,
                                           w_att, b_att, graph, bn, training)
        ctx.save_for_backward(*saved)
        return outs

    @staticmethod
    def backward(ctx, g_im, g_z1, g_z2, g_kl, g_klmean):
        df, dt, ds, grads = _interaction_backward(ctx, ctx.saved_tensors, g_im, g_z1, g_z2, g_kl,
                                                  g_klmean)
        return (df, dt, ds, None, None) + grads + (None, None, None)


class _InteractionLin(torch.autograd.Function):
    """compressor[0] (Linear 64 -> 64) fused in front of the interaction:
    t = f W0^T + b0 (scgib_linear_fwd); backward d f = df + dt W0 and dW0, db0
    in one pass (scgib_linear_bwd with add = df)."""

    @staticmethod
    def forward(ctx, f, w0, b0, s, u_gate, u_feat, gamma, beta, w2, b2, w_att, b_att, graph, bn,
                training):
        ctx.set_materialize_grads(False)  # outputs no loss reads (fine-tune: z1, z2, KL): no fills
        f = _f32(f, "interaction")
        s = _f32(s, "interaction")
        w0, b0 = _f32(w0, "compressor.0.weight"), _f32(b0, "compressor.0.bias")
        if f.shape[1] != HIDDEN or tuple(w0.shape) != (HIDDEN, HIDDEN):
            raise _lib.ScgibError("compressor[0] must be Linear(64, 64)")
        t = torch.empty_like(f)
        _lib.call("scgib_linear_fwd", _p(f), f.shape[0], _p(w0), _p(b0), _p(t), _p(graph.dims),
                  _stream())
        outs, saved = _interaction_forward(ctx, f, t, s, u_gate, u_feat, gamma, beta, w2, b2,
                                           w_att, b_att, graph, bn, training)
        ctx.save_for_backward(*saved, w0)
        return outs

    @staticmethod
    def backward(ctx, g_im, g_z1, g_z2, g_kl, g_klmean):
        saved = ctx.saved_tensors
        w0 = saved[-1]
        df, dt, ds, grads = _interaction_backward(ctx, saved[:-1], g_im, g_z1, g_z2, g_kl,
                                                  g_klmean)
        f = saved[0]
        n = f.shape[0]
        slab = torch.empty(int(_lib.query("scgib_linear_slab_floats", n)), dtype=torch.float32,
                           device=f.device)
        wg = torch.empty(HIDDEN * HIDDEN + HIDDEN, dtype=torch.float32, device=f.device)
        df_total = torch.empty_like(f)
        _lib.call("scgib_linear_bwd", _p(dt), _p(f), _p(w0), n, _p(df), _p(df_total), _p(slab),
                  _p(wg), _p(ctx.graph.dims), _stream())
        dw0, db0 = wg[: HIDDEN * HIDDEN].view(HIDDEN, HIDDEN), wg[HIDDEN * HIDDEN:]
        return (df_total, dw0, db0, ds, None, None) + grads + (None, None, None)


def interaction(f, t, s, u_gate, u_feat, bn, lin2, attn, graph, training):
    """Fused compression + attention (models.py:595-660, 714-749).

    ``bn`` is the compressor BatchNorm1d (its running stats are updated in
    place in train mode, once per graph), ``lin2`` the compressor's
    Linear(64, 1), ``attn`` the attn_layer Linear(128, 1).
    Returns (interaction_map [N,128], z1 = sum_nodes(noisy) [B,64],
    z2 = sum_nodes(f) [B,64], kl_tensor [2 n_last, 64] (empty in capacity
    mode), kl_mean = mean(kl_tensor) [scalar]).
    """
    return _Interaction.apply(f, t, s, u_gate, u_feat, bn.weight, bn.bias, lin2.weight,
                              lin2.bias, attn.weight, attn.bias, graph, bn, bool(training))


def interaction_lin(f, s, u_gate, u_feat, compressor, attn, graph, training):
    """interaction() with t = compressor[0](f) computed by the fused dense
    kernels (the model's path): ``compressor`` is the Sequential(Linear,
    BatchNorm1d, ReLU, Linear) of models.py:589-592."""
    lin0, bn, lin2 = compressor[0], compressor[1], compressor[3]
    return _InteractionLin.apply(f, lin0.weight, lin0.bias, s, u_gate, u_feat, bn.weight, bn.bias,
                                 lin2.weight, lin2.bias, attn.weight, attn.bias, graph, bn,
                                 bool(training))


# ---------------------------------------------------------------------------
# A12: adjacency reconstruction loss (Gram form)
# ---------------------------------------------------------------------------
class _ReconAdj(torch.autograd.Function):
    @staticmethod
    def forward(ctx, im, graph):
        im = _f32(im, "recon_adj")
        n, d = im.shape
        if d != HIDDEN:
            raise _lib.ScgibError(f"recon kernels are built for width {HIDDEN}, got {d}")
        dev = im.device
        partials = torch.empty(int(_lib.query("scgib_recon_partials_floats", n)),
                               dtype=torch.float32, device=dev)
        gram = torch.empty(HIDDEN * HIDDEN, dtype=torch.float32, device=dev)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        _lib.call("scgib_recon_fwd", _p(im), _p(graph.rowptr), _p(graph.col), n,
                  graph.edge_capacity(), _p(partials), _p(gram), _p(loss), _p(graph.dims),
                  _stream())
        ctx.save_for_backward(im, gram)
        ctx.graph = graph
        return loss

    @staticmethod
    def backward(ctx, g_loss):
        im, gram = ctx.saved_tensors
        gr = ctx.graph
        g_loss = _f32(g_loss.reshape(1), "g_loss")
        out = torch.empty_like(im)
        _lib.call("scgib_recon_bwd", _p(im), _p(gram), _p(gr.rowptr), _p(gr.col), _p(gr.rowptr_t),
                  _p(gr.col_t), im.shape[0], _p(g_loss), _p(out), _p(gr.dims), _stream())
        return out, None


def recon_adj(im, graph):
    """sum((IM IM^T - A)^2) / N without the N x N matrix (models.py:762-768)."""
    return _ReconAdj.apply(im, graph)


# ---------------------------------------------------------------------------
# Arrival counters for last-arriver reductions: one persistent zeroed int32
# buffer per device, carved into fixed ranges per call site.  Kernels leave
# their counters zero, so a range is reused by every launch and graph replay.
# ---------------------------------------------------------------------------
_COUNTER_CAP = 1 << 16
_COUNTERS = {}   # device index -> tensor
_COUNTER_RANGES = {}  # (device index, key) -> (offset, size)


def counters(device, key, n):
    """``n`` zeroed uint32 counters reserved for call site ``key`` on ``device``
    and the current stream (allocate outside graph capture: the first call per
    device allocates).  Keying by stream as well keeps two launches of one call
    site that run concurrently on different streams (e.g. two contrastive ops)
    on disjoint ranges; launches on one stream are ordered, so they share."""
    idx = torch.device(device).index or 0
    buf = _COUNTERS.get(idx)
    if buf is None:
        buf = _COUNTERS[idx] = _zeroed_words(_COUNTER_CAP, device)
    rk = (idx, key, torch.cuda.current_stream(device).cuda_stream)
    off, size = _COUNTER_RANGES.get(rk, (None, 0))
    if size < n:
        used = max((o + s for (d, _, _), (o, s) in _COUNTER_RANGES.items() if d == idx), default=0)
        if used + n > _COUNTER_CAP:
            raise _lib.ScgibError("arrival-counter pool exhausted")
        off, size = used, n
        _COUNTER_RANGES[rk] = (off, size)
    return buf[off: off + n]


_SCAN_STATES = {}  # (device index, key, stream) -> int32 tensor (a range of an arena)
_SCAN_ARENAS = {}  # device index -> [int32 tensors]: zeroed at creation, never freed
_SCAN_NEXT = {}    # device index -> next free word of the newest arena
_SCAN_ARENA_WORDS = 1 << 20  # 4 MB: every key and stream of a process, captures included


def _zeroed_words(n, device):
    """n zeroed int32 on ``device``, the fill COMPLETE before this returns.
    The pool / arena it makes is carved into ranges that kernels on other
    streams use with no ordering edge to the fill (a later carve
    for another stream could otherwise race the memset — e.g. the encoder's
    BatchNorm arrival counters on the main stream against a fill enqueued on
    the side stream, leaving a counter non-zero and every later last-arriver
    reduction miscounting).  Made once per device, before any capture (a
    capture would record the fill into the replayed step instead)."""
    dev = torch.device(device)
    if dev.type == "cuda" and torch.cuda.is_current_stream_capturing():
        raise _lib.ScgibError("arrival-counter / scan-state memory must be created outside "
                              "graph capture (run one eager step first)")
    buf = torch.zeros(n, dtype=torch.int32, device=dev)
    if dev.type == "cuda":
        torch.cuda.current_stream(dev).synchronize()
    return buf


def _scan_carve(idx, device, size):
    """``size`` zeroed words from the device's arena.  The arena is made by the
    first request (an eager step, before any capture), so a key first seen
    while a graph is being captured — a capture runs on its own stream, a new
    key — is carved from memory that is already zero instead of allocating
    (and zero-filling) inside the graph, where the fill would replay every
    step (a 5 us fill at the head of each encoder chain, round 4)."""
    arenas = _SCAN_ARENAS.setdefault(idx, [])
    off = _SCAN_NEXT.get(idx, 0)
    if arenas and off + size <= arenas[-1].numel():
        _SCAN_NEXT[idx] = off + ((size + 63) // 64) * 64  # 256-B aligned ranges
        return arenas[-1][off: off + size]
    words = _SCAN_ARENA_WORDS
    while words < size:
        words *= 2
    arenas.append(_zeroed_words(words, device))
    _SCAN_NEXT[idx] = ((size + 63) // 64) * 64
    return arenas[-1][:size]


def scan_state(device, key, n):
    """``n`` zeroed int32 words of O(n) state (the one-pass ego builder's
    look-back words, a GIN encoder's BatchNorm arrival counters) for call
    site ``key`` on ``device`` and the current stream, separate from the O(1)
    counter pool: it grows on demand to the next power of two (a new zeroed
    range of the device's arena; the outgrown one stays allocated, since a
    captured graph may reference it — at most log2 of the largest size per
    key) and the kernels leave it zeroed for the next launch.  Keys name call
    sites, never objects, so a long-lived process that builds new modules
    reuses the same words."""
    idx = torch.device(device).index or 0
    rk = (idx, key, torch.cuda.current_stream(device).cuda_stream)
    buf = _SCAN_STATES.get(rk)
    if buf is None or buf.numel() < n:
        size = 1024
        while size < n:
            size *= 2
        buf = _SCAN_STATES[rk] = _scan_carve(idx, device, size)
    return buf[:n]


# ---------------------------------------------------------------------------
# Device noise: {seed, offset} (int64) per device for the Philox draws of
# scgib_noise_uniform; the kernel advances the offset itself, so a captured
# step draws fresh noise on every replay.
# ---------------------------------------------------------------------------
_NOISE_STATES = {}  # device index -> int64 [seed, offset]


def noise_state(device):
    """The device's noise state; created on first use with a seed drawn from
    torch's default CPU generator (reproducible under torch.manual_seed).
    Create it outside graph capture (any eager step does)."""
    idx = torch.device(device).index or 0
    st = _NOISE_STATES.get(idx)
    if st is None:
        if torch.cuda.is_current_stream_capturing():
            raise _lib.ScgibError("device noise state must be created outside graph capture "
                                  "(run one eager step or call ops.seed_noise first)")
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        st = _NOISE_STATES[idx] = torch.tensor([seed, 0], dtype=torch.int64, device=device)
    return st


def seed_noise(device, seed, offset=0):
    """Reset the device noise stream (seed, offset) in place."""
    st = noise_state(device)
    st.copy_(torch.tensor([int(seed), int(offset)], dtype=torch.int64))
    return st


def device_noise(n, device):
    """(u_gate [n], u_feat [n, 64]) ~ U[0, 1) drawn on the current stream by
    scgib_noise_uniform from the device's noise state."""
    u_gate = torch.empty(n, dtype=torch.float32, device=device)
    u_feat = torch.empty(n, HIDDEN, dtype=torch.float32, device=device)
    _lib.call("scgib_noise_uniform", _p(u_gate), _p(u_feat), n, _p(noise_state(device)),
              _p(counters(device, "noise", 1)), _stream())
    return u_gate, u_feat


class NoisePrefetch:
    """The compression noise one step ahead, for a replayed step (bench.py):
    the step reads (u_gate, u_feat) from these static buffers and its
    backward draws the next step's into them at the end of the encoder
    pair's core chain — on ``side``, after the interaction backward (the
    buffers' last reader) and beside the longer ego chain — instead of at
    the head of the forward core chain.  The same Philox draws in the same
    order as device_noise per step (one draw of ``n`` rows per step), so a
    replayed step reads the values the inline draw would have given it.
    ``prime()`` draws the first step's (eager); models._encode_forked takes
    the buffers from ``batch_g.noise_prefetch``."""

    def __init__(self, graph, device):
        self.n = graph.num_nodes()
        self.device = torch.device(device)
        self.u_gate = torch.zeros(self.n, dtype=torch.float32, device=device)
        self.u_feat = torch.zeros(self.n, HIDDEN, dtype=torch.float32, device=device)
        graph.noise_prefetch = self

    def draw(self):
        """The next step's noise into the buffers, on the current stream."""
        _lib.call("scgib_noise_uniform", _p(self.u_gate), _p(self.u_feat), self.n,
                  _p(noise_state(self.device)), _p(counters(self.device, "noise", 1)), _stream())

    prime = draw


# ---------------------------------------------------------------------------
# A11: contrastive loss (batched_semi_loss, tau = 1)
# ---------------------------------------------------------------------------
class _Contrastive(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z1, z2):
        z1 = _f32(z1, "contrastive z1")
        z2 = _f32(z2, "contrastive z2")
        B = z1.shape[0]
        if z1.shape != (B, HIDDEN) or z2.shape != (B, HIDDEN):
            raise _lib.ScgibError(f"contrastive: z1 {tuple(z1.shape)} / z2 {tuple(z2.shape)} "
                                  f"must both be [B, {HIDDEN}]")
        ws = torch.empty(int(_lib.query("scgib_contrastive_workspace_floats", B)),
                         dtype=torch.float32, device=z1.device)
        loss = torch.empty((), dtype=torch.float32, device=z1.device)
        cnt = counters(z1.device, "contrastive", int(_lib.query("scgib_contrastive_counters", B)))
        _lib.call("scgib_contrastive_fwd", _p(z1), _p(z2), B, _p(ws), _p(loss), _p(cnt),
                  _stream())
        ctx.save_for_backward(z1, z2, ws)
        return loss

    @staticmethod
    def backward(ctx, g):
        z1, z2, ws = ctx.saved_tensors
        B = z1.shape[0]
        g = _f32(g, "contrastive.backward").reshape(1)
        dz1, dz2 = torch.empty_like(z1), torch.empty_like(z2)
        cnt = counters(z1.device, "contrastive", int(_lib.query("scgib_contrastive_counters", B)))
        _lib.call("scgib_contrastive_bwd", _p(z1), _p(z2), B, _p(ws), _p(g), _p(dz1), _p(dz2),
                  _p(cnt), _stream())
        return dz1, dz2


def contrastive(z1, z2):
    """batched_semi_loss(z1, z2, chunk) with tau = 1 (models.py:606-629); the
    value does not depend on the chunk size."""
    return _Contrastive.apply(z1, z2)


# ---------------------------------------------------------------------------
# A10 head: the interaction-map MLP (Linear(128,64) - ReLU - Linear(64,64))
# ---------------------------------------------------------------------------
class _Mlp2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, dims):
        x = _f32(x, "mlp2")
        n, d_in = x.shape
        if tuple(w1.shape) != (HIDDEN, d_in) or tuple(w2.shape) != (HIDDEN, HIDDEN):
            raise _lib.ScgibError(f"mlp2: expects Linear({d_in},64) - Linear(64,64)")
        # (the fine-tune head's MLP: its weight-gradient reduce is deferred into
        # the encoder pair's backward, off the loss chain, as the pretraining
        # head's is — SlabScope)
        ctx.leaves = (w1, b1, w2, b2)
        ctx.scope = _slab_scope_for(ctx.leaves)
        w1, b1, w2, b2 = (_f32(t, "mlp2 params") for t in (w1, b1, w2, b2))
        r = torch.empty(n, HIDDEN, dtype=torch.float32, device=x.device)
        out = torch.empty(n, HIDDEN, dtype=torch.float32, device=x.device)
        _lib.call("scgib_mlp2_fwd", _p(x), d_in, n, _p(w1), _p(b1), _p(w2), _p(b2), _p(r),
                  _p(out), _p(dims), _stream())
        ctx.save_for_backward(x, r, w1, w2)
        ctx.dims = dims
        return out

    @staticmethod
    def backward(ctx, g):
        x, r, w1, w2 = ctx.saved_tensors
        g = _f32(g, "mlp2.backward")
        n, d_in = x.shape
        dx = torch.empty_like(x)
        slab = torch.empty(int(_lib.query("scgib_mlp2_slab_floats", n, d_in)),
                           dtype=torch.float32, device=x.device)
        wg = torch.empty(HIDDEN * HIDDEN + HIDDEN * d_in + 2 * HIDDEN, dtype=torch.float32,
                         device=x.device)
        defer = ctx.scope is not None and ctx.scope.usable(ctx.leaves)
        _lib.call("scgib_mlp2_bwd", _p(g), _p(x), _p(r), d_in, _p(w1), _p(w2), n, _p(dx),
                  _p(slab), None if defer else _p(wg), _p(ctx.dims), _stream())
        if defer:  # reduced by the encoder pair's backward (SlabScope)
            ctx.scope.add(slab, wg, wg.numel(), slab.numel() // wg.numel())
        o = HIDDEN * HIDDEN
        dw2 = wg[:o].view(HIDDEN, HIDDEN)
        dw1 = wg[o: o + HIDDEN * d_in].view(HIDDEN, d_in)
        db2 = wg[o + HIDDEN * d_in: o + HIDDEN * d_in + HIDDEN]
        db1 = wg[o + HIDDEN * d_in + HIDDEN:]
        return dx, dw1, db1, dw2, db2, None


def mlp2(x, mlp, dims=None):
    """``mlp`` = Sequential(Linear(d, 64), ReLU(), Linear(64, 64)) applied by
    the fused tile kernels (models.py:1055-1057, :1174)."""
    return _Mlp2.apply(x, mlp[0].weight, mlp[0].bias, mlp[2].weight, mlp[2].bias, dims)


class _Mlp2Recon(torch.autograd.Function):
    """loss_recon_adj(MLP(x)) (models.py:1174 then :1256-1262) in two
    launches forward (the MLP tiles also write Gram partials; one kernel
    reduces them, adds the edge term and forms the loss) and one backward
    (the MLP backward forms d IM of its tile itself) + the weight reduce."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, graph):
        x = _f32(x, "mlp2_recon")
        n, d_in = x.shape
        if tuple(w1.shape) != (HIDDEN, d_in) or tuple(w2.shape) != (HIDDEN, HIDDEN):
            raise _lib.ScgibError(f"mlp2_recon: expects Linear({d_in},64) - Linear(64,64)")
        w1, b1, w2, b2 = (_f32(t, "mlp2 params") for t in (w1, b1, w2, b2))
        dev = x.device
        r = torch.empty(n, HIDDEN, dtype=torch.float32, device=dev)
        out = torch.empty(n, HIDDEN, dtype=torch.float32, device=dev)
        ws = torch.empty(int(_lib.query("scgib_mlp2_recon_ws_floats", n)), dtype=torch.float32,
                         device=dev)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        cnt = counters(dev, "mlp2_recon", 3)
        _lib.call("scgib_mlp2_recon_fwd", _p(x), d_in, n, _p(w1), _p(b1), _p(w2), _p(b2), _p(r),
                  _p(out), _p(graph.rowptr), _p(graph.col), graph.edge_capacity(), _p(ws),
                  _p(cnt), _p(loss), _p(graph.dims), _p(handoff_fault_word(dev)), _stream())
        ctx.save_for_backward(x, r, out, ws, w1, w2)
        ctx.graph = graph
        return loss

    @staticmethod
    def backward(ctx, g_loss):
        x, r, out, ws, w1, w2 = ctx.saved_tensors
        gr = ctx.graph
        g_loss = _f32(g_loss.reshape(1), "g_loss")
        n, d_in = x.shape
        dx = torch.empty_like(x)
        slab = torch.empty(int(_lib.query("scgib_mlp2_recon_slab_floats", n, d_in)),
                           dtype=torch.float32, device=x.device)
        wg = torch.empty(HIDDEN * HIDDEN + HIDDEN * d_in + 2 * HIDDEN, dtype=torch.float32,
                         device=x.device)
        sym = gr.symmetric
        _lib.call("scgib_mlp2_recon_bwd", _p(x), _p(r), _p(out), _p(ws), d_in, _p(w1), _p(w2), n,
                  _p(gr.rowptr), _p(gr.col), None if sym else _p(gr.rowptr_t),
                  None if sym else _p(gr.col_t), _p(g_loss), _p(dx), _p(slab), _p(wg),
                  _p(gr.dims), _stream())
        o = HIDDEN * HIDDEN
        dw2 = wg[:o].view(HIDDEN, HIDDEN)
        dw1 = wg[o: o + HIDDEN * d_in].view(HIDDEN, d_in)
        db2 = wg[o + HIDDEN * d_in: o + HIDDEN * d_in + HIDDEN]
        db1 = wg[o + HIDDEN * d_in + HIDDEN:]
        return dx, dw1, db1, dw2, db2, None


class _Mlp2ReconContrastive(torch.autograd.Function):
    """_Mlp2Recon and _Contrastive in the same launches: the contrastive
    loss's workgroups run beside the MLP tiles (forward and backward), so the
    critical chain has one launch each way instead of two."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, graph, z1, z2):
        x = _f32(x, "mlp2_recon")
        n, d_in = x.shape
        if d_in != 2 * HIDDEN or tuple(w1.shape) != (HIDDEN, d_in) or \
                tuple(w2.shape) != (HIDDEN, HIDDEN):
            raise _lib.ScgibError("mlp2_recon_contrastive: expects Linear(128,64) - Linear(64,64)")
        z1, z2 = _f32(z1, "contrastive z1"), _f32(z2, "contrastive z2")
        B = z1.shape[0]
        if z1.shape != (B, HIDDEN) or z2.shape != (B, HIDDEN):
            raise _lib.ScgibError(f"contrastive: z1 {tuple(z1.shape)} / z2 {tuple(z2.shape)} "
                                  f"must both be [B, {HIDDEN}]")
        ctx.leaves = (w1, b1, w2, b2)
        ctx.scope = _slab_scope_for(ctx.leaves)
        w1, b1, w2, b2 = (_f32(t, "mlp2 params") for t in (w1, b1, w2, b2))
        dev = x.device
        r = torch.empty(n, HIDDEN, dtype=torch.float32, device=dev)
        out = torch.empty(n, HIDDEN, dtype=torch.float32, device=dev)
        ws = torch.empty(int(_lib.query("scgib_mlp2_recon_ws_floats", n)), dtype=torch.float32,
                         device=dev)
        cws = torch.empty(int(_lib.query("scgib_contrastive_workspace_floats", B)),
                          dtype=torch.float32, device=dev)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        closs = torch.empty((), dtype=torch.float32, device=dev)
        cnt = counters(dev, "mlp2_recon", 3)
        ccnt = counters(dev, "contrastive", int(_lib.query("scgib_contrastive_counters", B)))
        ru = take_running_update()
        _launch("scgib_mlp2_recon_contrastive_fwd", {"n": n, "d_in": d_in, "B": B}, _p(x), d_in, n,
                _p(w1), _p(b1), _p(w2),
                  _p(b2), _p(r), _p(out), _p(graph.rowptr), _p(graph.col),
                  graph.edge_capacity(), _p(ws), _p(cnt), _p(loss), _p(graph.dims), _p(z1),
                  _p(z2), B, _p(cws), _p(closs), _p(ccnt), _byref(ru[0] if ru else None),
                  _p(handoff_fault_word(dev)), _stream())
        ctx.save_for_backward(x, r, out, ws, w1, w2, z1, z2, cws)
        ctx.graph = graph
        return loss, closs

    @staticmethod
    def backward(ctx, g_loss, g_con):
        x, r, out, ws, w1, w2, z1, z2, cws = ctx.saved_tensors
        gr = ctx.graph
        dev = x.device
        g_loss = _f32(g_loss.reshape(1), "g_loss") if g_loss is not None else \
            torch.zeros(1, dtype=torch.float32, device=dev)
        g_con = _f32(g_con.reshape(1), "g_con") if g_con is not None else \
            torch.zeros(1, dtype=torch.float32, device=dev)
        n, d_in = x.shape
        B = z1.shape[0]
        dx = torch.empty_like(x)
        dz1, dz2 = torch.empty_like(z1), torch.empty_like(z2)
        slab = torch.empty(int(_lib.query("scgib_mlp2_recon_slab_floats", n, d_in)),
                           dtype=torch.float32, device=dev)
        wg = torch.empty(HIDDEN * HIDDEN + HIDDEN * d_in + 2 * HIDDEN, dtype=torch.float32,
                         device=dev)
        ccnt = counters(dev, "contrastive", int(_lib.query("scgib_contrastive_counters", B)))
        sym = gr.symmetric
        defer = ctx.scope is not None and ctx.scope.usable(ctx.leaves)
        _launch("scgib_mlp2_recon_contrastive_bwd", {"n": n, "d_in": d_in, "B": B}, _p(x), _p(r),
                _p(out), _p(ws), d_in,
                  _p(w1), _p(w2), n, _p(gr.rowptr), _p(gr.col),
                  None if sym else _p(gr.rowptr_t), None if sym else _p(gr.col_t), _p(g_loss),
                  _p(dx), _p(slab), None if defer else _p(wg), _p(gr.dims), _p(z1), _p(z2), B,
                  _p(cws), _p(g_con), _p(dz1), _p(dz2), _p(ccnt), _stream())
        if defer:  # reduced by the encoder pair's backward (SlabScope)
            ctx.scope.add(slab, wg, wg.numel(), slab.numel() // wg.numel())
        o = HIDDEN * HIDDEN
        dw2 = wg[:o].view(HIDDEN, HIDDEN)
        dw1 = wg[o: o + HIDDEN * d_in].view(HIDDEN, d_in)
        db2 = wg[o + HIDDEN * d_in: o + HIDDEN * d_in + HIDDEN]
        db1 = wg[o + HIDDEN * d_in + HIDDEN:]
        return dx, dw1, db1, dw2, db2, None, dz1, dz2


def mlp2_recon_contrastive(x, mlp, graph, z1, z2):
    """(recon_adj(mlp2(x, mlp), graph), contrastive(z1, z2)) from the same
    launches (scgib_mlp2_recon_contrastive_fwd / _bwd)."""
    return _Mlp2ReconContrastive.apply(x, mlp[0].weight, mlp[0].bias, mlp[2].weight,
                                       mlp[2].bias, graph, z1, z2)


def mlp2_recon(x, mlp, graph):
    """recon_adj(mlp2(x, mlp), graph) fused (the pretraining model's head);
    the MLP output itself is not returned (nothing else reads it)."""
    return _Mlp2Recon.apply(x, mlp[0].weight, mlp[0].bias, mlp[2].weight, mlp[2].bias, graph)


# ---------------------------------------------------------------------------
# A15: logM reconstruction loss (models.py:770-782)
# ---------------------------------------------------------------------------
class _ReconLogM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, im, graph, logm):
        im = _f32(im, "recon_logm")
        if im.shape[1] != HIDDEN:
            raise _lib.ScgibError(f"recon_logm kernels are built for width {HIDDEN}")
        if graph.dims is not None:
            raise _lib.ScgibError("recon_logm: capacity mode is not supported")
        B = graph.batch_size
        if len(logm.sizes) != B or not np.array_equal(logm.sizes, graph.batch_num_nodes_host()):
            raise _lib.ScgibError("logM targets do not match the molecules of the batch")
        lossg = torch.empty(B, dtype=torch.float32, device=im.device)
        loss = torch.empty((), dtype=torch.float32, device=im.device)
        _lib.call("scgib_recon_logm_fwd", _p(im), _p(graph.graph_ptr), B, _p(logm.S),
                  _p(logm.offsets), _p(logm.C), logm.kstep, _p(lossg), _p(loss), _stream())
        ctx.save_for_backward(im)
        ctx.graph, ctx.logm = graph, logm
        return loss

    @staticmethod
    def backward(ctx, g):
        (im,) = ctx.saved_tensors
        g = _f32(g, "recon_logm.backward").reshape(1)
        grad = torch.empty_like(im)
        lm = ctx.logm
        _lib.call("scgib_recon_logm_bwd", _p(im), _p(ctx.graph.graph_ptr), ctx.graph.batch_size,
                  _p(lm.S), _p(lm.offsets), lm.kstep, _p(g), _p(grad), _stream())
        return grad, None, None


def recon_logm(im, graph, logm):
    """loss_recon (models.py:770-782) on the device.  ``logm`` is a
    graph.LogMBatch or the reference's list of per-molecule [k, n, n]
    targets (packed here)."""
    if not isinstance(logm, _graph.LogMBatch):
        logm = _graph.LogMBatch(list(logm), im.device)
    return _ReconLogM.apply(im, graph, logm)

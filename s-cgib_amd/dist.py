"""Data parallelism for the pretrain step: one process per GPU, RCCL over xGMI.

The reference has no distributed code ("Collectives: none").
Molecules shard naturally: ego-nets never cross molecules, so the ego-net
build, both encoders, compression and attention are rank-local, and the only
exchange is the gradient average (replica mode: every rank
runs the reference's step on its own sub-batch; batch-coupled terms — BN
statistics, contrastive denominators, recon loss, last-graph KL — are taken
over the rank's sub-batch).

The hot-path gradients total ~98k fp32 (~390 KB): one flat bucket, one
all-reduce per step.  At that size an xGMI ring is latency-bound (< 10 us of
link time), so a single bucket beats per-layer buckets and there is nothing
to overlap it with worth the complexity.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Initialise torch.distributed from torchrun's env; returns (rank, world, local_rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:  # SCGIB_DIST_BACKEND=gloo: local multi-rank runs on one GPU
            backend = os.environ.get("SCGIB_DIST_BACKEND") or \
                ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
        elif torch.cuda.is_available():  # gloo with HIP tensors (local rehearsal)
            torch.cuda.set_device(local % torch.cuda.device_count())
        dist.init_process_group(backend=backend)
    return rank, world, local


class GradAllReducer:
    """Averages the gradients of every parameter that received one (and the
    given float buffers), in one flat all-reduce (SUM / world).  The set of parameters with gradients is
    the same on every rank (same model, same path).

    HIP tensors: the gradients are packed into the flat bucket by ONE launch
    (scgib_grad_pack) and unpacked with the 1/world scale by one more
    (scgib_grad_unpack), not a copy launch per tensor; ``pack`` / ``reduce`` /
    ``unpack`` are exposed separately so a captured HIP graph can hold the
    pack (with the backward) and the unpack (with the optimizer step) while
    the RCCL all-reduce runs between the two replays.  CPU tensors (the gloo
    tests) take per-tensor copies."""

    def __init__(self, params, group=None, buffers=()):
        self.params = [p for p in params if p.requires_grad]
        # float buffers averaged with the gradients (BatchNorm running
        # statistics, ``bn_buffers``): every replica then holds the same
        # statistics after each step, so eval and a saved checkpoint do not
        # depend on which rank wrote them
        self.buffers = [b for b in buffers if b.dtype == torch.float32]
        self.group = group
        self._flat = None

    def _world(self):
        if not dist.is_initialized():
            return 1
        return dist.get_world_size(self.group)

    def _grads(self):
        return [p.grad for p in self.params if p.grad is not None] + self.buffers

    def _buffer(self, grads):
        numel = sum(g.numel() for g in grads)
        if self._flat is None or self._flat.numel() != numel or self._flat.device != grads[0].device:
            if grads[0].is_cuda and torch.cuda.is_current_stream_capturing():
                raise RuntimeError("GradAllReducer: run one step outside graph capture first "
                                   "(the flat bucket is allocated then)")
            self._flat = torch.empty(numel, dtype=grads[0].dtype, device=grads[0].device)
        return self._flat

    def _table(self, grads):
        from . import _lib
        out, off = [], 0
        for g in grads:
            if g.dtype != torch.float32 or not g.is_contiguous():
                raise _lib.ScgibError("GradAllReducer: gradients must be contiguous fp32")
            out.append(_lib.GradSlice(g.data_ptr(), g.numel(), off))
            off += g.numel()
        return out

    def _launch(self, name, grads, *extra):
        import ctypes
        from . import _lib
        from . import ops
        ent = self._table(grads)
        cap = int(_lib.query("scgib_grad_pack_max_tensors"))
        for i0 in range(0, len(ent), cap):
            chunk = ent[i0:i0 + cap]
            table = (_lib.GradSlice * len(chunk))(*chunk)
            _lib.call(name, ctypes.cast(table, ctypes.c_void_p), len(chunk), ops._p(self._flat),
                      *extra, ops._stream())

    def pack(self):
        """Gradients -> the flat bucket."""
        grads = self._grads()
        if not grads:
            return
        flat = self._buffer(grads)
        if not flat.is_cuda:
            off = 0
            for g in grads:
                flat[off:off + g.numel()].copy_(g.reshape(-1))
                off += g.numel()
            return
        self._launch("scgib_grad_pack", grads)

    def reduce(self, force=False):
        """All-reduce (SUM) of the flat bucket over the group (``force``: also
        over a 1-rank group, to exercise the collective path on one GPU)."""
        if self._flat is None:
            return
        if self._world() > 1 or (force and dist.is_initialized()):
            dist.all_reduce(self._flat, op=dist.ReduceOp.SUM, group=self.group)

    def unpack(self):
        """The flat bucket / world -> the gradients."""
        grads = self._grads()
        if not grads:
            return
        scale = 1.0 / self._world()
        if not self._flat.is_cuda:
            off = 0
            for g in grads:
                g.copy_(self._flat[off:off + g.numel()].view_as(g) * scale)
                off += g.numel()
            return
        self._launch("scgib_grad_unpack", grads, float(scale))

    def __call__(self):
        if self._world() == 1:
            return
        self.pack()
        self.reduce()
        self.unpack()


def broadcast_replicas(model, src=0, group=None):
    """Rank ``src``'s parameters and buffers to every rank of ``group`` (the
    construction-time sync of a data-parallel replica set): the replicas start
    identical whatever each rank's seed, and the one averaged update per step
    keeps them identical.  No-op in a 1-rank world."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    with torch.no_grad():
        for t in list(model.parameters()) + list(model.buffers()):
            dist.broadcast(t.data, src, group=group)


def bn_buffers(model):
    """The BatchNorm running means / variances of ``model`` (float buffers the
    replicas average each step; num_batches_tracked is equal on every rank)."""
    return [b for name, b in model.named_buffers()
            if name.endswith(("running_mean", "running_var"))]


def shard(items, rank, world):
    """Contiguous, equal-as-possible slice of a list of molecules for ``rank``."""
    n = len(items)
    lo = (n * rank) // world
    hi = (n * (rank + 1)) // world
    return items[lo:hi]

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
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    return rank, world, local


class GradAllReducer:
    """Averages the gradients of every parameter that received one, in one
    flat all-reduce (SUM / world).  The set of parameters with gradients is
    the same on every rank (same model, same path)."""

    def __init__(self, params, group=None):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self._flat = None

    def __call__(self):
        if not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return
        world = dist.get_world_size(self.group)
        grads = [p.grad for p in self.params if p.grad is not None]
        if not grads:
            return
        numel = sum(g.numel() for g in grads)
        if self._flat is None or self._flat.numel() != numel or self._flat.device != grads[0].device:
            self._flat = torch.empty(numel, dtype=grads[0].dtype, device=grads[0].device)
        off = 0
        for g in grads:
            self._flat[off:off + g.numel()].copy_(g.reshape(-1))
            off += g.numel()
        dist.all_reduce(self._flat, op=dist.ReduceOp.SUM, group=self.group)
        self._flat.div_(world)
        off = 0
        for g in grads:
            g.copy_(self._flat[off:off + g.numel()].view_as(g))
            off += g.numel()


def shard(items, rank, world):
    """Contiguous, equal-as-possible slice of a list of molecules for ``rank``."""
    n = len(items)
    lo = (n * rank) // world
    hi = (n * (rank + 1)) // world
    return items[lo:hi]

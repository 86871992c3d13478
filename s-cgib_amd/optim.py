"""Adam on the device in one launch per 80 tensors (scgib_adam_step).

Drop-in for the optimizer every reference script builds,
``torch.optim.Adam(model.parameters(), lr=args.lr, weight_decay=5e-5)``
(exp_pretraining.py, exp_molhiv.py:53/:89/:160 ...): same hyper-parameters,
same per-parameter state (``step`` / ``exp_avg`` / ``exp_avg_sq``, so
state_dicts are interchangeable with torch's), the arithmetic of torch's
fused Adam, and HIP-graph capturable (the tensor table is passed by value in
the kernel arguments; ``step`` stays on the device).  amsgrad, maximize,
decoupled weight decay and sparse gradients are not supported (the reference
does not use them).  HIP only — no CPU fallback.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from . import ops


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 amsgrad=False, maximize=False):
        if amsgrad or maximize:
            raise NotImplementedError("scgib Adam: amsgrad / maximize are not implemented")
        if not 0.0 <= lr or not 0.0 <= eps or not 0.0 <= weight_decay:
            raise ValueError(f"invalid Adam hyper-parameters lr={lr} eps={eps} wd={weight_decay}")
        if not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError(f"invalid betas {betas}")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._max = int(_lib.query("scgib_adam_max_tensors"))

    def _entries(self, group):
        out = []
        for p in group["params"]:
            if p.grad is None:
                continue
            if not p.is_cuda or p.dtype != torch.float32 or not p.is_contiguous():
                raise _lib.ScgibError("scgib Adam: parameters must be contiguous fp32 HIP tensors")
            if p.grad.is_sparse:
                raise _lib.ScgibError("scgib Adam: sparse gradients are not supported")
            if p.grad.dtype != torch.float32 or not p.grad.is_contiguous():
                p.grad = p.grad.float().contiguous()
            st = self.state[p]
            if not st:
                st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            elif st["step"].device != p.device or st["step"].dtype != torch.float32:
                st["step"] = st["step"].to(device=p.device, dtype=torch.float32)
            out.append(_lib.AdamTensor(p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(),
                                       st["exp_avg_sq"].data_ptr(), st["step"].data_ptr(),
                                       p.numel()))
        return out

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        ops.check_handoff()  # an earlier step's hand-off wait gave up: raise before updating
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        pending = []  # the final weight-gradient reduces left to this step (ops.fuse_final_into_step)
        for group in self.param_groups:
            pending += ops.take_final(group["params"][0].device) if group["params"] else []
        fused = False
        for gi, group in enumerate(self.param_groups):
            ent = self._entries(group)
            if not ent:
                continue
            dev = group["params"][0].device
            b1, b2 = group["betas"]
            st = ops._stream()
            jobs = [j for jl, _ in pending for j in jl]
            if (jobs and not fused and len(self.param_groups) == 1 and len(ent) <= self._max
                    and len(jobs) <= int(_lib.query("scgib_adam_reduce_max_jobs"))
                    and max(j.n_slabs for j in jobs) >= ops.FUSE_FINAL_MIN_SLABS):
                # the reduce and this step in one launch (same bits)
                table = (_lib.AdamTensor * len(ent))(*ent)
                jt = (_lib.SlabJob * len(jobs))(*jobs)
                _lib.call("scgib_adam_step_reduce", ctypes.cast(table, ctypes.c_void_p), len(ent),
                          ctypes.cast(jt, ctypes.c_void_p), len(jobs), float(group["lr"]),
                          float(b1), float(b2), float(group["eps"]), float(group["weight_decay"]),
                          ops._p(ops.counters(dev, "adam", 1)), st)
                fused = True
                continue
            if pending and not fused:  # not fusable here: the reduces first, as unfused
                for jl, _ in pending:
                    ops._reduce_jobs(jl, st)
                fused = True
            for li, i0 in enumerate(range(0, len(ent), self._max)):
                chunk = ent[i0:i0 + self._max]
                table = (_lib.AdamTensor * len(chunk))(*chunk)
                # one word per stream (launches on a stream are ordered, and each
                # leaves it zero): not per optimizer, so new optimizers reuse it
                cnt = ops.counters(dev, "adam", 1)
                _lib.call("scgib_adam_step", ctypes.cast(table, ctypes.c_void_p), len(chunk),
                          float(group["lr"]), float(b1), float(b2), float(group["eps"]),
                          float(group["weight_decay"]), ops._p(cnt), st)
        if pending and not fused:  # (no gradients here at all)
            for jl, _ in pending:
                ops._reduce_jobs(jl, ops._stream())
        pending = None  # the slabs stay referenced until the launches are enqueued
        ops.stamp("adam_end")
        return loss

"""S-CGIB hot path, MI355X-native.

The package directory is ``s-cgib_amd`` (not a Python identifier), so import it
with ``importlib.import_module("s-cgib_amd")`` and reach submodules as
attributes (``pkg.models``, ``pkg.graph`` ...) — they load lazily.

Layout:
  csrc/        hand-written HIP kernels for gfx950 + the C-ABI (include/scgib.h)
  _lib.py      ctypes binding of libscgib.so (fails loudly when missing)
  graph.py     DGL-duck-typed graph batch (CSR int32, dst-major) + ingest
  ops.py       autograd Functions over the C-ABI
  models.py    models.py-compatible Mainmodel / Mainmodel_continue /
               Mainmodel_finetuning / GIN / Set2Set
  metrics.py   ROC-AUC (OGB semantics) and TU accuracy of the fine-tune configs
  optim.py     one-launch device Adam (drop-in for torch.optim.Adam as the scripts use it)
  cache.py     on-disk CSR cache of a molecule dataset (replaces the pts/ pickles)
  refckpt.py   the reference's whole-module checkpoints, read weights-only
  dgl.py       drop-in ``dgl`` surface (graph, batch, sum_nodes, khop...)
  dist.py      one-process-per-GPU data parallel (RCCL all-reduce)
  synth.py     seeded synthetic molecules
"""
import importlib

__all__ = ["graph", "ops", "models", "dgl", "dist", "synth", "metrics", "optim", "cache", "refckpt",
           "_lib"]


def __getattr__(name):
    if name in __all__:
        return importlib.import_module(f"{__name__}.{name}")
    raise AttributeError(name)

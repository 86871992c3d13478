"""Stub modules that let the reference's own ``models.py`` be imported here.

TEST INFRASTRUCTURE ONLY (see ``oracle/dgl_semantics.py`` header).  Used by
``oracle/gen_golden.py`` in the build container, where ``/root/reference``
exists.  Nothing on the GPU box imports this.

The reference imports ``dgl``, ``torch_geometric``, ``ogb``, ``pyro`` and
``torch_scatter`` at module scope (``/root/reference/models.py:1-35``); none is
installed.  Each is replaced by a module whose hot-path members are the DGL
restatements in ``dgl_semantics`` and whose other members are inert
placeholders (only touched at import time, never called on the path).
"""
from __future__ import annotations

import sys
import types

from . import dgl_semantics as D

REFERENCE_DIR = "/root/reference"


class _Placeholder:
    def __init__(self, *a, **k):
        raise RuntimeError("placeholder for an unsupported third-party symbol was called")


def _module(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)

    def __getattr__(attr):
        if attr.startswith("__"):
            raise AttributeError(attr)
        return _Placeholder

    m.__getattr__ = __getattr__
    sys.modules[name] = m
    return m


def install():
    """Register the stubs in ``sys.modules`` (idempotent)."""
    if "dgl" in sys.modules and getattr(sys.modules["dgl"], "_scgib_shim", False):
        return
    dgl_fn = _module("dgl.function")
    glob = _module("dgl.nn.pytorch.glob", Set2Set=D.Set2Set, SumPooling=D.SumPooling)
    ginconv = _module("dgl.nn.pytorch.conv.ginconv", GINConv=D.GINConv)
    conv = _module("dgl.nn.pytorch.conv", GINConv=D.GINConv, ginconv=ginconv)
    pt = _module("dgl.nn.pytorch", conv=conv, glob=glob, GINConv=D.GINConv, Set2Set=D.Set2Set)
    nn_ = _module("dgl.nn", pytorch=pt, GINConv=D.GINConv, Set2Set=D.Set2Set)
    sparse = _module("dgl.sparse")
    data = _module("dgl.data")
    dataloading = _module("dgl.dataloading")
    _module("dgl", _scgib_shim=True, nn=nn_, sparse=sparse, function=dgl_fn, data=data,
            dataloading=dataloading, graph=D.graph, batch=D.batch,
            to_bidirected=D.to_bidirected, khop_in_subgraph=D.khop_in_subgraph,
            node_subgraph=D.node_subgraph, sum_nodes=D.sum_nodes, mean_nodes=D.mean_nodes,
            broadcast_nodes=D.broadcast_nodes, softmax_nodes=D.softmax_nodes,
            DGLGraph=D.Graph, DGLError=D.DGLError)
    tg_nn = _module("torch_geometric.nn")
    _module("torch_geometric", nn=tg_nn)
    mol = _module("ogb.graphproppred.mol_encoder")
    gpp = _module("ogb.graphproppred", mol_encoder=mol)
    _module("ogb", graphproppred=gpp)
    _module("pyro")
    _module("torch_scatter")


def import_reference_models():
    """``import models`` from the read-only reference tree, behind the stubs."""
    install()
    if REFERENCE_DIR not in sys.path:
        sys.path.insert(0, REFERENCE_DIR)
    import models  # noqa: E402  (the reference's own file)
    return models

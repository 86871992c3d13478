"""ctypes front-end of oracle/egonet_ref.c (test infrastructure only)."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libegonet_ref.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        p = ctypes.c_void_p
        _lib.egonet_ref.argtypes = [p, p, ctypes.c_int64, ctypes.c_int, p, p, p, p, p]
        _lib.egonet_ref.restype = ctypes.c_int
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def egonets(rowptr, col, k):
    """All ego-nets of a CSR graph (row = node, sorted columns).

    Returns (sizes, ecount, nodes, esrc, edst) as int64 arrays; ``nodes`` are
    the sorted ball members (global ids), ``esrc/edst`` ego-local positions.
    """
    lib = _load()
    rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
    col = np.ascontiguousarray(col, dtype=np.int64)
    n = len(rowptr) - 1
    sizes = np.zeros(n, np.int64)
    ecount = np.zeros(n, np.int64)
    rc = lib.egonet_ref(_ptr(rowptr), _ptr(col), n, k, _ptr(sizes), _ptr(ecount), None, None, None)
    assert rc == 0
    nodes = np.zeros(int(sizes.sum()), np.int64)
    esrc = np.zeros(int(ecount.sum()), np.int64)
    edst = np.zeros(int(ecount.sum()), np.int64)
    rc = lib.egonet_ref(_ptr(rowptr), _ptr(col), n, k, _ptr(sizes), _ptr(ecount), _ptr(nodes),
                        _ptr(esrc), _ptr(edst))
    assert rc == 0
    return sizes, ecount, nodes, esrc, edst

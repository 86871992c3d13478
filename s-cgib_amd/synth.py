"""Seeded synthetic molecule batches of the shapes in SURVEY.md §8(d).

No dataset is reachable offline, so the benchmark and the parity fixtures use
molecules drawn here:

* atom count ``n ~ round(Normal(mu, sigma))`` clipped to ``[2, 4*mu]``;
* a random spanning tree (atom ``i`` bonds to ``randrange(i)``);
* ``n // 8`` ring-closure attempts under a degree cap of 4;
* bonds stored in both directions (PyG ``edge_index`` convention), no
  self-loops, so every molecule survives the reference's skip rule
  (``util.py:317-321``, ``exp_pretraining.py:276-278``);
* features: ``"qm9"`` F=11 floats in [0, 1); ``"ogb"`` F=9 non-negative
  integers in the OGB atom-feature ranges; ``"mutag"`` F=14 one-hot.
"""
from __future__ import annotations

import random

import numpy as np

# (mu, sigma, F, feature kind) per workload
WORKLOADS = {
    "mutagenicity": (30.0, 8.0, 14, "mutag"),
    "qm9": (18.0, 3.0, 11, "qm9"),
    "molpcba": (26.0, 3.0, 9, "ogb"),
    "pcqm4mv2": (14.0, 3.0, 9, "ogb"),
    "molhiv": (25.5, 8.0, 9, "ogb"),
    "zinc": (23.2, 4.5, 9, "ogb"),
}

# OGB atom feature cardinalities (ogb.utils.features.get_atom_feature_dims)
_OGB_ATOM_DIMS = (119, 5, 12, 12, 10, 6, 6, 2, 2)


def molecule(rnd: random.Random, mu: float, sigma: float):
    """One molecule: (n, edge_index int64 [2, E]) with both directions stored."""
    n = int(round(rnd.gauss(mu, sigma)))
    n = max(2, min(n, int(4 * mu)))
    deg = [0] * n
    bonds = set()
    for i in range(1, n):
        j = rnd.randrange(i)
        bonds.add((j, i))
        deg[i] += 1
        deg[j] += 1
    for _ in range(n // 8):
        a, b = rnd.randrange(n), rnd.randrange(n)
        if a == b:
            continue
        key = (min(a, b), max(a, b))
        if key in bonds or deg[a] >= 4 or deg[b] >= 4:
            continue
        bonds.add(key)
        deg[a] += 1
        deg[b] += 1
    bonds = sorted(bonds)
    ei = np.empty((2, 2 * len(bonds)), dtype=np.int64)
    for t, (a, b) in enumerate(bonds):
        ei[0, 2 * t], ei[1, 2 * t] = a, b
        ei[0, 2 * t + 1], ei[1, 2 * t + 1] = b, a
    return n, ei


def features(nprng: np.random.Generator, n: int, F: int, kind: str) -> np.ndarray:
    if kind == "qm9":
        return nprng.random((n, F), dtype=np.float32)
    if kind == "ogb":
        cols = [nprng.integers(0, d, size=n) for d in _OGB_ATOM_DIMS[:F]]
        return np.stack(cols, 1).astype(np.float32)
    if kind == "mutag":
        x = np.zeros((n, F), dtype=np.float32)
        x[np.arange(n), nprng.integers(0, F, size=n)] = 1.0
        return x
    raise ValueError(kind)


def molecules(num: int, workload: str = "qm9", seed: int = 0, mu=None, sigma=None, F=None):
    """List of (edge_index [2,E] int64, x [n,F] float32), PyG ``Data``-shaped."""
    wmu, wsig, wF, kind = WORKLOADS[workload]
    mu = wmu if mu is None else mu
    sigma = wsig if sigma is None else sigma
    F = wF if F is None else F
    rnd = random.Random(seed)
    nprng = np.random.default_rng(seed)
    out = []
    for _ in range(num):
        n, ei = molecule(rnd, mu, sigma)
        out.append((ei, features(nprng, n, F, kind)))
    return out

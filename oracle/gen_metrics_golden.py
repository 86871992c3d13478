"""Golden vectors for the fine-tune metrics (test infrastructure, not product).

Imports the REFERENCE's own /root/reference/metrics.py (torch + sklearn +
numpy only; the OGB Evaluator the molhiv harness calls, train_molhiv.py:50,
109, 158, is absent here — metrics.eval_rocauc at metrics.py:18-37 is its
restatement, copied into the reference from ogb/graphproppred/evaluate.py)
and records its outputs on seeded inputs into tests/golden/metrics.npz:

  eval_rocauc  metrics.py:18-37    multi-task, NaN labels, one-class tasks
  eval_ap      metrics.py:40-61    (train_pep_func.py:126)
  eval_rmse    metrics.py:64-76
  eval_acc     metrics.py:79-87
  rmse         metrics.py:129-137  (train_molsolv.py:180)
  MAE          metrics.py:140-143
  accuracy_TU  metrics.py:146-159  (train_tudataset.py:148)

Run in the survey container (the reference does not exist on the GPU box):
    python oracle/gen_metrics_golden.py
"""
import importlib.util
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/metrics.py"


def load_ref():
    spec = importlib.util.spec_from_file_location("ref_metrics", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def cases(rng):
    """(name, y_true [n, t], y_pred [n, t]) for the ROC/AP/acc/rmse family."""
    out = []
    # molhiv-like: one task, imbalanced labels, continuous scores with ties
    y = (rng.random((500, 1)) < 0.05).astype(np.float64)
    p = np.round(rng.random((500, 1)) + 0.3 * y, 2)
    out.append(("hiv_like", y, p))
    # molpcba-like: many tasks, NaN labels, some tasks with one class only
    y = (rng.random((300, 16)) < 0.2).astype(np.float64)
    y[rng.random((300, 16)) < 0.3] = np.nan
    y[:, 3] = np.where(np.isnan(y[:, 3]), np.nan, 0.0)  # negatives only: skipped
    y[:, 7] = np.where(np.isnan(y[:, 7]), np.nan, 1.0)  # positives only: skipped
    p = rng.standard_normal((300, 16)) + 0.8 * np.nan_to_num(y)
    out.append(("pcba_like", y, p))
    # tiny, perfectly separable and perfectly inverted tasks
    y = np.array([[0, 1], [0, 1], [1, 0], [1, 0]], dtype=np.float64)
    p = np.array([[0.1, 0.9], [0.2, 0.8], [0.9, 0.3], [0.8, 0.2]])
    out.append(("separable", y, p))
    return out


def main():
    ref = load_ref()
    rng = np.random.default_rng(20261016)
    blob = {}
    for name, y, p in cases(rng):
        blob[f"{name}__y_true"] = y
        blob[f"{name}__y_pred"] = p
        blob[f"{name}__rocauc"] = np.float64(ref.eval_rocauc(y, p)["rocauc"])
        blob[f"{name}__ap"] = np.float64(ref.eval_ap(y, p))
        blob[f"{name}__rmse"] = np.float64(ref.eval_rmse(y, p)["rmse"])
        yb = np.where(np.isnan(y), np.nan, (p > 0.5).astype(np.float64))
        blob[f"{name}__acc_pred"] = yb
        blob[f"{name}__acc"] = np.float64(ref.eval_acc(y, yb)["acc"])
    # torch-side metrics of the training loops
    g = torch.Generator().manual_seed(7)
    scores = torch.randn(64, 2, generator=g)
    targets = torch.randint(0, 2, (64, 1), generator=g)
    blob["tu__scores"] = scores.numpy()
    blob["tu__targets"] = targets.numpy()
    blob["tu__accuracy"] = np.float64(ref.accuracy_TU(scores, targets))
    reg_s = torch.randn(40, 1, generator=g)
    reg_t = torch.randn(40, 1, generator=g)
    blob["reg__scores"] = reg_s.numpy()
    blob["reg__targets"] = reg_t.numpy()
    blob["reg__mae"] = np.float64(ref.MAE(reg_s, reg_t))
    blob["reg__rmse"] = np.float64(ref.rmse(reg_s, reg_t))
    out = os.path.join(ROOT, "tests", "golden", "metrics.npz")
    np.savez(out, **blob)
    print("wrote", out, len(blob), "arrays")


if __name__ == "__main__":
    sys.exit(main())

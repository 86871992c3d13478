"""Evaluation metrics of the fine-tune configs (metrics.py of the reference).

  eval_rocauc   metrics.py:18-37   (OGB Evaluator semantics: mean per-task
                                    sklearn roc_auc_score over tasks with both
                                    classes present, NaN labels ignored; the
                                    molhiv harness calls ogb's Evaluator,
                                    train_molhiv.py:109,158, whose rule this is)
  eval_ap       metrics.py:40-61   (mean per-task average precision, same task
                                    rule; returns the bare mean as the reference)
  eval_rmse     metrics.py:64-76   (mean per-task RMSE over labelled rows)
  eval_acc      metrics.py:79-87   (mean per-task accuracy over labelled rows)
  rmse          metrics.py:129-137 (sqrt(MSE + 1e-6), train_molsolv.py:180)
  MAE           metrics.py:140-143
  accuracy_TU   metrics.py:146-159 (argmax over classes, count of matches)
Host-side (numpy / sklearn / torch CPU ops), as in the reference; pinned by
tests/golden/metrics.npz (oracle/gen_metrics_golden.py runs the reference's
own functions).
"""
from __future__ import annotations

import numpy as np
import torch


def _np2(a):
    a = np.asarray(torch.as_tensor(a).detach().cpu(), dtype=np.float64)
    return a[:, None] if a.ndim == 1 else a


def _both_classes(col):
    return np.sum(col == 1) > 0 and np.sum(col == 0) > 0


def eval_rocauc(y_true, y_pred):
    from sklearn.metrics import roc_auc_score
    y_true, y_pred = _np2(y_true), _np2(y_pred)
    scores = []
    for i in range(y_true.shape[1]):
        col = y_true[:, i]
        if _both_classes(col):
            lab = col == col
            scores.append(roc_auc_score(col[lab], y_pred[lab, i]))
    if not scores:
        raise RuntimeError("No positively labeled data available. Cannot compute ROC-AUC.")
    return {"rocauc": sum(scores) / len(scores)}


def eval_ap(y_true, y_pred):
    from sklearn.metrics import average_precision_score
    y_true, y_pred = _np2(y_true), _np2(y_pred)
    aps = []
    for i in range(y_true.shape[1]):
        col = y_true[:, i]
        if _both_classes(col):
            lab = col == col
            aps.append(average_precision_score(col[lab], y_pred[lab, i]))
    if not aps:
        raise RuntimeError(
            "No positively labeled data available. Cannot compute Average Precision.")
    return sum(aps) / len(aps)


def eval_rmse(y_true, y_pred):
    y_true, y_pred = _np2(y_true), _np2(y_pred)
    out = []
    for i in range(y_true.shape[1]):
        lab = y_true[:, i] == y_true[:, i]
        out.append(np.sqrt(((y_true[lab, i] - y_pred[lab, i]) ** 2).mean()))
    return {"rmse": sum(out) / len(out)}


def eval_acc(y_true, y_pred):
    y_true, y_pred = _np2(y_true), _np2(y_pred)
    out = []
    for i in range(y_true.shape[1]):
        lab = y_true[:, i] == y_true[:, i]
        correct = y_true[lab, i] == y_pred[lab, i]
        out.append(float(np.sum(correct)) / len(correct))
    return {"acc": sum(out) / len(out)}


def rmse(scores, targets):
    return torch.sqrt(torch.nn.functional.mse_loss(scores, targets) + 1e-6).detach().item()


def accuracy_TU(scores, targets):
    targets = targets.squeeze(dim=-1)
    pred = scores.argmax(dim=1)
    return (pred.to(float) == targets.to(float)).sum().item()


def MAE(scores, targets):
    return torch.nn.functional.l1_loss(scores, targets).detach().item()

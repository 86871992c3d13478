"""Evaluation metrics of the fine-tune configs (metrics.py of the reference).

  eval_rocauc   metrics.py:18-37  (OGB Evaluator semantics: mean per-task
                                    sklearn roc_auc_score over tasks with both
                                    classes present, NaN labels ignored)
  accuracy_TU   metrics.py:146-159 (argmax over classes, count of matches)
Host-side (numpy / sklearn), as in the reference.
"""
from __future__ import annotations

import numpy as np
import torch


def eval_rocauc(y_true, y_pred):
    from sklearn.metrics import roc_auc_score
    y_true = np.asarray(torch.as_tensor(y_true).detach().cpu(), dtype=np.float64)
    y_pred = np.asarray(torch.as_tensor(y_pred).detach().cpu(), dtype=np.float64)
    if y_true.ndim == 1:
        y_true, y_pred = y_true[:, None], y_pred[:, None]
    scores = []
    for i in range(y_true.shape[1]):
        col = y_true[:, i]
        if np.sum(col == 1) > 0 and np.sum(col == 0) > 0:
            lab = col == col
            scores.append(roc_auc_score(col[lab], y_pred[lab, i]))
    if not scores:
        raise RuntimeError("No positively labeled data available. Cannot compute ROC-AUC.")
    return {"rocauc": sum(scores) / len(scores)}


def accuracy_TU(scores, targets):
    targets = targets.squeeze(dim=-1)
    pred = scores.argmax(dim=1)
    return (pred.to(float) == targets.to(float)).sum().item()


def MAE(scores, targets):
    return torch.nn.functional.l1_loss(scores, targets).detach().item()

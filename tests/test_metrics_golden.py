"""Fine-tune metrics (s-cgib_amd/metrics.py) against the reference's own
metrics.py outputs (tests/golden/metrics.npz, oracle/gen_metrics_golden.py):
ROC-AUC / AP / RMSE / accuracy over multi-task labels with NaNs and
one-class tasks, accuracy_TU, MAE, rmse.  Exact up to float64 rounding."""
import os

import numpy as np
import pytest
import torch

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "metrics.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


@pytest.mark.parametrize("case", ["hiv_like", "pcba_like", "separable"])
def test_task_metrics(pkg, gold, case):
    M = pkg.metrics
    y, p = gold[f"{case}__y_true"], gold[f"{case}__y_pred"]
    assert M.eval_rocauc(y, p)["rocauc"] == pytest.approx(float(gold[f"{case}__rocauc"]), rel=1e-12)
    assert M.eval_ap(y, p) == pytest.approx(float(gold[f"{case}__ap"]), rel=1e-12)
    assert M.eval_rmse(y, p)["rmse"] == pytest.approx(float(gold[f"{case}__rmse"]), rel=1e-12)
    assert M.eval_acc(y, gold[f"{case}__acc_pred"])["acc"] == pytest.approx(
        float(gold[f"{case}__acc"]), rel=1e-12)
    # torch inputs (the harnesses pass tensors) give the same numbers
    assert M.eval_rocauc(torch.from_numpy(y), torch.from_numpy(p))["rocauc"] == pytest.approx(
        float(gold[f"{case}__rocauc"]), rel=1e-12)


def test_rocauc_no_positive_raises(pkg):
    with pytest.raises(RuntimeError):
        pkg.metrics.eval_rocauc(np.zeros((5, 1)), np.ones((5, 1)))


def test_training_loop_metrics(pkg, gold):
    M = pkg.metrics
    s, t = torch.from_numpy(gold["tu__scores"]), torch.from_numpy(gold["tu__targets"])
    assert M.accuracy_TU(s, t) == float(gold["tu__accuracy"])
    rs, rt = torch.from_numpy(gold["reg__scores"]), torch.from_numpy(gold["reg__targets"])
    assert M.MAE(rs, rt) == pytest.approx(float(gold["reg__mae"]), rel=1e-6)
    assert M.rmse(rs, rt) == pytest.approx(float(gold["reg__rmse"]), rel=1e-6)

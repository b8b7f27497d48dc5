"""Evaluator numerics against independent references (scikit-learn and direct numpy definitions).

Reference behaviour: OpBinaryClassificationEvaluator.scala:67-135 (Spark BinaryClassificationMetrics:
trapezoidal ROC / PR over distinct score thresholds, PR curve starting at (0, precision of the first
threshold)), OpMultiClassificationEvaluator.scala:100-125 (weighted precision / recall, F1 of the two),
OpRegressionEvaluator, OpForecastEvaluator (SMAPE, MASE), OPLogLoss, OpBinScoreEvaluator (Brier)."""
import numpy as np
import pytest
import torch
from sklearn import metrics as skm

from transmogrifai_amd.evaluators import metrics as M
from transmogrifai_amd.evaluators.evaluators import (OpBinaryClassificationEvaluator, OpBinScoreEvaluator,
                                                     OpForecastEvaluator, OpLogLossEvaluator,
                                                     OpMultiClassificationEvaluator, OpRegressionEvaluator)


def _binary(n=2000, seed=0, ties=False):
    rng = np.random.default_rng(seed)
    y = (rng.random(n) < 0.3).astype(np.float64)
    s = np.clip(0.35 * y + rng.normal(0.4, 0.2, n), 0, 1)
    if ties:
        s = np.round(s, 2)
    return torch.as_tensor(s), torch.as_tensor(y)


def _spark_pr_area(s, y):
    """Spark areaUnderPR: one point per distinct threshold (descending), first point (0, p1), trapezoid."""
    order = np.argsort(-s, kind="stable")
    s, y = s[order], y[order]
    uniq_end = np.r_[np.nonzero(np.diff(s))[0], len(s) - 1]
    tp = np.cumsum(y)[uniq_end]
    fp = np.cumsum(1 - y)[uniq_end]
    prec = tp / (tp + fp)
    rec = tp / y.sum()
    x = np.r_[0.0, rec]
    yy = np.r_[prec[0], prec]
    return float(np.sum((x[1:] - x[:-1]) * (yy[1:] + yy[:-1]) / 2))


@pytest.mark.parametrize("ties", [False, True])
def test_exact_auroc_matches_sklearn(ties):
    s, y = _binary(ties=ties)
    assert M.au_roc(s, y, 0) == pytest.approx(skm.roc_auc_score(y.numpy(), s.numpy()), abs=1e-12)


@pytest.mark.parametrize("ties", [False, True])
def test_exact_aupr_matches_spark_definition(ties):
    s, y = _binary(ties=ties, seed=1)
    assert M.au_pr(s, y, 0) == pytest.approx(_spark_pr_area(s.numpy(), y.numpy()), abs=1e-12)


def test_binned_aupr_close_to_exact():
    s, y = _binary(n=20000, seed=2)
    assert M.binned_aupr(s, y) == pytest.approx(M.au_pr(s, y, 0), abs=2e-3)
    h = torch.stack([torch.stack([torch.bincount(((1 - s[y == c]) * 65535).long(), minlength=65536)
                                  for c in (0, 1)])]).to(torch.int32)
    assert float(M.binned_aupr_from_counts(h)[0]) == pytest.approx(M.binned_aupr(s, y), abs=1e-6)


def test_binary_evaluator_confusion_metrics():
    s, y = _binary(seed=3)
    pred = (s > 0.5).double()
    prob = torch.stack([1 - s, s], 1)
    out = OpBinaryClassificationEvaluator().evaluate_arrays(y, pred, torch.log(prob), prob)
    yt, yp = y.numpy(), pred.numpy()
    assert out["Precision"] == pytest.approx(skm.precision_score(yt, yp))
    assert out["Recall"] == pytest.approx(skm.recall_score(yt, yp))
    assert out["F1"] == pytest.approx(skm.f1_score(yt, yp))
    assert out["Error"] == pytest.approx(1 - skm.accuracy_score(yt, yp))
    assert out["TP"] + out["TN"] + out["FP"] + out["FN"] == len(yt)
    tm = out["ThresholdMetrics"]
    # Spark's numBins down-sampling: groups of (distinct thresholds // numBins) consecutive thresholds
    d = len(np.unique(s.numpy()))
    assert len(tm["thresholds"]) == -(-d // (d // 100))
    assert tm["thresholds"] == sorted(tm["thresholds"], reverse=True)
    # numBins = 100 down-sampled curves stay close to the exact areas
    assert out["AuROC"] == pytest.approx(skm.roc_auc_score(yt, s.numpy()), abs=5e-3)


def test_binary_evaluator_empty_data():
    e = torch.zeros(0, dtype=torch.float64)
    out = OpBinaryClassificationEvaluator().evaluate_arrays(e, e, torch.zeros(0, 2), torch.zeros(0, 2))
    assert out["AuROC"] == 0.0 and out["ThresholdMetrics"]["thresholds"] == []


def test_multiclass_weighted_metrics_match_sklearn():
    rng = np.random.default_rng(4)
    y = rng.integers(0, 4, 3000)
    p = np.where(rng.random(3000) < 0.6, y, rng.integers(0, 4, 3000))
    prob = np.eye(4)[p] * 0.7 + 0.075
    out = OpMultiClassificationEvaluator().evaluate_arrays(torch.as_tensor(y).double(), torch.as_tensor(p).double(),
                                                           None, torch.as_tensor(prob))
    wp = skm.precision_score(y, p, average="weighted")
    wr = skm.recall_score(y, p, average="weighted")
    assert out["Precision"] == pytest.approx(wp)
    assert out["Recall"] == pytest.approx(wr)
    assert out["F1"] == pytest.approx(2 * wp * wr / (wp + wr))
    assert out["Error"] == pytest.approx(1 - skm.accuracy_score(y, p))
    th = out["ThresholdMetrics"]
    for t in ("1", "3"):
        tot = np.array(th["correctCounts"][t]) + np.array(th["incorrectCounts"][t]) + np.array(th["noPredictionCounts"][t])
        assert (tot == len(y)).all()


def test_regression_metrics_match_sklearn():
    rng = np.random.default_rng(5)
    y = rng.normal(10, 3, 1000)
    p = y + rng.normal(0, 1, 1000)
    out = OpRegressionEvaluator().evaluate_arrays(torch.as_tensor(y), torch.as_tensor(p), None, None)
    assert out["MeanSquaredError"] == pytest.approx(skm.mean_squared_error(y, p))
    assert out["RootMeanSquaredError"] == pytest.approx(np.sqrt(skm.mean_squared_error(y, p)))
    assert out["MeanAbsoluteError"] == pytest.approx(skm.mean_absolute_error(y, p))
    assert out["R2"] == pytest.approx(skm.r2_score(y, p))
    assert sum(out["SignedPercentageErrorHistogram"]["counts"]) == 1000


@pytest.mark.parametrize("metric", ["RootMeanSquaredError", "MeanSquaredError", "MeanAbsoluteError", "R2"])
def test_regression_selection_metric_batch_equals_full_set(metric):
    rng = np.random.default_rng(6)
    y = torch.as_tensor(rng.normal(10, 3, 5000))
    preds = [torch.as_tensor(y.numpy() + rng.normal(0, s, 5000)).float() for s in (0.5, 1.0, 2.0)]
    ev = OpRegressionEvaluator(metric)
    batch = ev.selection_metric_batch(y, [(p, None, None) for p in preds])
    for p, b in zip(preds, batch):
        full = M.regression_metrics(p, y)[metric]
        assert b == pytest.approx(full, rel=1e-12)
        assert ev.selection_metric(y, p, None, None) == pytest.approx(full, rel=1e-12)
    const = torch.full((10,), 2.0, dtype=torch.float64)
    assert OpRegressionEvaluator("R2").selection_metric(const, const + 1, None, None) == 0.0


def test_forecast_smape_mase():
    y = np.array([1.0, 2.0, 4.0, 3.0, 5.0, 6.0])
    p = np.array([1.5, 2.0, 3.0, 3.5, 4.0, 6.5])
    out = OpForecastEvaluator(seasonal_window=1).evaluate_arrays(torch.as_tensor(y), torch.as_tensor(p), None, None)
    smape = np.mean(2 * np.abs(p - y) / (np.abs(p) + np.abs(y)))
    se = np.mean(np.abs(y[1:] - y[:-1]))
    assert out["SMAPE"] == pytest.approx(smape)
    assert out["SeasonalError"] == pytest.approx(se)
    assert out["MASE"] == pytest.approx(np.mean(np.abs(p - y)) / se)


def test_log_loss_and_brier_match_sklearn():
    rng = np.random.default_rng(6)
    y = rng.integers(0, 3, 500)
    prob = rng.dirichlet([1, 1, 1], 500)
    ll = OpLogLossEvaluator().evaluate_arrays(torch.as_tensor(y).double(), torch.as_tensor(prob.argmax(1)).double(),
                                              None, torch.as_tensor(prob))
    val = ll if isinstance(ll, float) else ll[next(iter(ll))]
    assert val == pytest.approx(skm.log_loss(y, prob, labels=[0, 1, 2]))
    s, yb = _binary(seed=7)
    out = OpBinScoreEvaluator().evaluate_arrays(yb, (s > 0.5).double(), None, torch.stack([1 - s, s], 1))
    assert out["BrierScore"] == pytest.approx(skm.brier_score_loss(yb.numpy(), s.numpy()))
    assert sum(out["numberOfDataPoints"]) == len(yb)


def test_binary_areas_batch_matches_per_curve():
    """One segmented sort for J score sets gives each set's exact AuPR / AuROC (ties, constant scores, all
    positives / negatives included)."""
    import torch
    from transmogrifai_amd.evaluators import metrics as M
    g = torch.Generator().manual_seed(0)
    n = 3000
    y = (torch.rand(n, generator=g) < 0.3).double()
    S = torch.stack([torch.rand(n, generator=g, dtype=torch.float64),
                     torch.round(torch.rand(n, generator=g, dtype=torch.float64) * 10) / 10,   # heavy ties
                     torch.full((n,), 0.5, dtype=torch.float64),                            # one run
                     y + 0.01 * torch.rand(n, generator=g, dtype=torch.float64),           # perfect
                     -y])                                                                  # inverted
    aupr, auroc = M.binary_areas_batch(S, y, chunk_elems=2 * n)
    for j in range(S.shape[0]):
        c = M.binary_curves(S[j], y, 0)
        assert abs(float(aupr[j]) - c["AuPR"]) < 1e-12, (j, float(aupr[j]), c["AuPR"])
        assert abs(float(auroc[j]) - c["AuROC"]) < 1e-12, (j, float(auroc[j]), c["AuROC"])


def test_binary_areas_batch_fp32_packed_key():
    """fp32 score sets take the packed (row, float-order) key sort: negative, zero, tied and extreme
    scores give the same areas as the per-curve fp64 path."""
    import torch
    from transmogrifai_amd.evaluators import metrics as M
    g = torch.Generator().manual_seed(1)
    n = 2500
    y = (torch.rand(n, generator=g) < 0.4).double()
    S = torch.stack([torch.randn(n, generator=g) * 3,
                     torch.round(torch.randn(n, generator=g) * 4) / 4,               # ties around 0, -0.0
                     torch.where(y > 0, torch.tensor(3.0e38), torch.tensor(-3.0e38)),   # extremes
                     -torch.rand(n, generator=g)]).to(torch.float32)
    S[1, :7] = -0.0
    aupr, auroc = M.binary_areas_batch(S, y)
    for j in range(S.shape[0]):
        c = M.binary_curves(S[j].double(), y, 0)
        assert abs(float(aupr[j]) - c["AuPR"]) < 1e-12, (j, float(aupr[j]), c["AuPR"])
        assert abs(float(auroc[j]) - c["AuROC"]) < 1e-12, (j, float(auroc[j]), c["AuROC"])

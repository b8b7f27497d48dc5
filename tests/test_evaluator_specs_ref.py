"""OpBinScoreEvaluatorTest, OpForecastEvaluatorTest (the closed-form cases) and OPLogLossTest
(``core/src/test/.../evaluators/`` and ``stages/impl/evaluator/``) with the reference's numbers."""
import math

import pytest
import torch

from transmogrifai_amd.evaluators.evaluators import OpBinScoreEvaluator, OpForecastEvaluator, OpLogLossEvaluator


def _t(x):
    return torch.tensor(x, dtype=torch.float64)


def _bin(num_bins, rows):
    """rows: (prediction, raw, prob, label)"""
    y = _t([r[3] for r in rows])
    pred = _t([r[0] for r in rows])
    raw = _t([r[1] for r in rows]) if rows and rows[0][1] else torch.zeros(len(rows), 0, dtype=torch.float64)
    prob = _t([r[2] for r in rows]) if rows and rows[0][2] else torch.zeros(len(rows), 0, dtype=torch.float64)
    return OpBinScoreEvaluator(num_bins=num_bins).evaluate_arrays(y, pred, raw, prob)


def _check(m, brier, size, centers, counts, positives, avg_score, avg_conv):
    assert m["BrierScore"] == pytest.approx(brier, rel=1e-9, abs=1e-15)
    assert m["binSize"] == pytest.approx(size, rel=1e-12)
    assert m["binCenters"] == pytest.approx(centers, rel=1e-12)
    assert m["numberOfDataPoints"] == counts and m["numberOfPositiveLabels"] == positives
    assert m["averageScore"] == pytest.approx(avg_score, rel=1e-12, abs=1e-15)
    assert m["averageConversionRate"] == pytest.approx(avg_conv, rel=1e-12)


def test_bin_metrics():
    rows = [(1.0, [10.0, 10.0], [0.0001, 0.99999], 1.0), (1.0, [10.0, 10.0], [0.0001, 0.99999], 1.0),
            (1.0, [10.0, 10.0], [0.99560, 0.00541], 0.0), (1.0, [10.0, 10.0], [0.30, 0.70], 0.0),
            (0.0, [10.0, 10.0], [0.999, 0.001], 0.0)]
    _check(_bin(4, rows), 0.09800605366, 0.25, [0.125, 0.375, 0.625, 0.875], [2, 0, 1, 2], [0, 0, 0, 2],
           [0.003205, 0.0, 0.7, 0.99999], [0.0, 0.0, 0.0, 1.0])


def test_bin_metrics_scores_outside_unit_interval():
    """Without probabilities the class-1 raw score is binned over [min(0, min), max(1, max)]."""
    rows = [(1.0, [0.0001, -0.99999], [], 0.0), (1.0, [0.0001, 1.99999], [], 1.0), (1.0, [0.0001, 12.0], [], 1.0)]
    _check(_bin(4, rows), 40.999986666733335, 3.2499975, [0.62500875, 3.87500625, 7.125003749999999, 10.37500125],
           [2, 0, 0, 1], [1, 0, 0, 1], [0.49999999999999994, 0.0, 0.0, 12.0], [0.5, 0.0, 0.0, 1.0])


def test_bin_metrics_invalid_bins_and_empty():
    with pytest.raises(ValueError, match="numOfBins must be positive"):
        OpBinScoreEvaluator(num_bins=0)
    m = _bin(10, [])
    assert m == {"BrierScore": 0.0, "binSize": 0.0, "binCenters": [], "numberOfDataPoints": [],
                 "numberOfPositiveLabels": [], "averageScore": [], "averageConversionRate": []}


def test_bin_metrics_skewed_and_default_metric():
    rows = [(1.0, [10.0, 10.0], [0.0001, 0.99999], 1.0), (1.0, [10.0, 10.0], [0.0001, 0.99999], 1.0),
            (1.0, [10.0, 10.0], [0.001, 0.9987], 1.0), (1.0, [10.0, 10.0], [0.0541, 0.946], 1.0)]
    _check(_bin(5, rows), 7.294225500000013e-4, 0.2, [0.1, 0.30000000000000004, 0.5, 0.7, 0.9], [0, 0, 0, 0, 4],
           [0, 0, 0, 0, 4], [0.0, 0.0, 0.0, 0.0, 0.98617], [0.0, 0.0, 0.0, 0.0, 1.0])
    ev = OpBinScoreEvaluator(num_bins=4)
    assert ev.metric == "BrierScore" and not ev.is_larger_better


def _sine(n=100):
    y = _t([math.sin(x / n * 2.0 * math.pi) for x in range(n)])
    return y, 1.2 * y


def test_forecast_metrics():
    y, p = _sine()
    m = OpForecastEvaluator(seasonal_window=25).evaluate_arrays(y, p, None, None)
    assert m["SMAPE"] == pytest.approx(0.18, abs=1e-3)
    assert m["MASE"] == pytest.approx(0.16395, abs=1e-5)
    assert m["SeasonalError"] == pytest.approx(0.77634, abs=1e-5)


def test_forecast_metrics_window_too_large_and_empty():
    y, p = _sine()
    m = OpForecastEvaluator(seasonal_window=101).evaluate_arrays(y, p, None, None)
    assert m["SMAPE"] == pytest.approx(0.18, abs=1e-3) and m["MASE"] == 0.0 and m["SeasonalError"] == 0.0
    e = torch.zeros(0, dtype=torch.float64)
    m = OpForecastEvaluator().evaluate_arrays(e, e, None, None)
    assert (m["SMAPE"], m["MASE"], m["SeasonalError"]) == (0.0, 0.0, 0.0)


def test_log_loss():
    rows = [(1.0, [0.8, 0.1, 0.1]), (0.0, [1.0, 0.0, 0.0]), (0.0, [0.5, 0.4, 0.1]), (1.0, [0.1, 0.8, 0.1]),
            (2.0, [0.0, 0.0, 1.0]), (2.0, [0.0, 0.0, 1.0]), (1.0, [0.1, 0.4, 0.5]), (0.0, [0.1, 0.6, 0.3]),
            (1.0, [0.5, 0.4, 0.1]), (2.0, [0.5, 0.4, 0.1])]
    y = _t([r[0] for r in rows])
    prob = _t([r[1] for r in rows])
    ev = OpLogLossEvaluator()
    m = ev.evaluate_arrays(y, prob.argmax(1).double(), prob, prob)
    expected = -math.log(0.1 * 0.5 * 0.8 * 0.4 * 0.1 * 0.4 * 0.1) / 10.0
    assert ev.metric == "MultiClasslogLoss" and not ev.is_larger_better
    assert m["MultiClasslogLoss"] == pytest.approx(expected, rel=1e-14)
    assert OpLogLossEvaluator(binary=True).metric == "BinarylogLoss"
    with pytest.raises(ValueError, match="requirement failed: Dataset is empty, log loss cannot be calculated"):
        ev.evaluate_arrays(torch.zeros(0), torch.zeros(0), torch.zeros(0, 3), torch.zeros(0, 3))


# ------------------------------------------------------------------------- OpMultiClassificationEvaluatorTest
def _multi_const(n=1000):
    y = torch.ones(n, dtype=torch.float64)
    prob = _t([[0.70, 0.25, 0.05, 0.0, 0.0]] * n)
    return y, torch.zeros(n, dtype=torch.float64), prob


def test_multiclass_threshold_counts_default():
    from transmogrifai_amd.evaluators.evaluators import OpMultiClassificationEvaluator
    n = 1000
    y, pred, prob = _multi_const(n)
    tm = OpMultiClassificationEvaluator().evaluate_arrays(y, pred, prob, prob)["ThresholdMetrics"]
    T_ = 101
    assert tm["topNs"] == [1, 3] and tm["thresholds"] == [i / 100 for i in range(101)]
    assert tm["correctCounts"] == {"1": [0] * T_, "3": [n] * 26 + [0] * (T_ - 26)}
    assert tm["incorrectCounts"] == {"1": [n] * 71 + [0] * (T_ - 71), "3": [0] * 26 + [n] * 45 + [0] * (T_ - 71)}
    assert tm["noPredictionCounts"] == {"1": [0] * 71 + [n] * (T_ - 71), "3": [0] * 71 + [n] * (T_ - 71)}


def test_multiclass_settable_thresholds_and_top_ns():
    from transmogrifai_amd.evaluators.evaluators import OpMultiClassificationEvaluator
    n = 1000
    y, pred, prob = _multi_const(n)
    ev = OpMultiClassificationEvaluator().set_thresholds([0.1, 0.2, 0.5, 0.8, 0.9, 1.0]).set_top_ns([1, 4, 12])
    tm = ev.evaluate_arrays(y, pred, prob, prob)["ThresholdMetrics"]
    assert tm["correctCounts"] == {"1": [0] * 6, "4": [n, n, 0, 0, 0, 0], "12": [n, n, 0, 0, 0, 0]}
    assert tm["incorrectCounts"] == {"1": [n, n, n, 0, 0, 0], "4": [0, 0, n, 0, 0, 0], "12": [0, 0, n, 0, 0, 0]}
    assert tm["noPredictionCounts"] == {k: [0, 0, 0, n, n, n] for k in ("1", "4", "12")}


@pytest.mark.parametrize("ties", [False, True])
def test_multiclass_random_probabilities(ties):
    from transmogrifai_amd.evaluators.evaluators import OpMultiClassificationEvaluator
    g = torch.Generator().manual_seed(3)
    n, k = 1000, (200 if ties else 100)
    if ties:
        raw = torch.full((n, k), 1e-10, dtype=torch.float64)
        raw[torch.arange(n), torch.randint(0, k, (n,), generator=g)] = 4.0
    else:
        raw = torch.rand(n, k, generator=g, dtype=torch.float64)
    prob = torch.softmax(raw, 1)
    pred = prob.argmax(1).double()
    y = torch.where(torch.rand(n, generator=g) < 0.3, pred, torch.ones(n, dtype=torch.float64)) if ties else \
        torch.randint(0, k, (n,), generator=g).double()
    m = OpMultiClassificationEvaluator().set_top_ns([1, 3, 5, 10] if ties else [1, 3]).evaluate_arrays(y, pred, raw, prob)
    tm = m["ThresholdMetrics"]
    assert tm["correctCounts"]["1"][0] / n + m["Error"] == pytest.approx(1.0)
    for c, i, z in zip(tm["correctCounts"]["1"], tm["incorrectCounts"]["1"], tm["noPredictionCounts"]["1"]):
        assert c + i + z == n
    assert all(v[0] == 0 for v in tm["noPredictionCounts"].values())


# --------------------------------------------------------------------------------- OpRegressionEvaluatorTest
_REAL = [(-10.0, -11.0), (-4.0, -8.0), (-2.0, 0.1), (0.0, -0.1), (0.0, 0.0), (0.0, 0.0), (0.0, 0.1), (2.0, 0.0),
         (4.0, 4.0), (10.0, 100.0)]
INF = float("inf")


def _reg(ev, rows):
    from transmogrifai_amd.evaluators.evaluators import OpRegressionEvaluator  # noqa: F401
    y, p = _t([r[0] for r in rows]), _t([r[1] for r in rows])
    return ev.evaluate_arrays(y, p, None, None)


def _reg_ev():
    from transmogrifai_amd.evaluators.evaluators import OpRegressionEvaluator
    return OpRegressionEvaluator()


def test_regression_param_validation():
    for bad in ([], [1.0, 0.0, 2.0]):
        with pytest.raises(ValueError):
            _reg_ev().set_percentage_error_histogram_bins(bad)
    with pytest.raises(ValueError):
        _reg_ev().set_scaled_error_cutoff(-1.0)
    with pytest.raises(ValueError):
        _reg_ev().set_smart_cutoff_ratio(-1.0)


def test_regression_histogram_cases():
    fine = [-INF] + [round(-1.0 + 0.1 * i, 10) for i in range(21)] + [INF]
    m = _reg(_reg_ev().set_percentage_error_histogram_bins(fine), [])
    assert m["SignedPercentageErrorHistogram"]["counts"] == [0] * (len(fine) - 1)
    m = _reg(_reg_ev(), _REAL)
    h = m["SignedPercentageErrorHistogram"]
    assert sum(h["counts"]) == len(_REAL) and len(h["bins"]) == 23
    m = _reg(_reg_ev().set_percentage_error_histogram_bins(fine), _REAL)
    assert m["SignedPercentageErrorHistogram"]["bins"] == fine and len(m["SignedPercentageErrorHistogram"]["counts"]) == 22
    m = _reg(_reg_ev().set_percentage_error_histogram_bins([-INF, -500.0, -100.0, 0.0, 100.0, 500.0, INF])
             .set_scaled_error_cutoff(10000.0), _REAL)
    assert m["SignedPercentageErrorHistogram"]["counts"] == [0, 0, 4, 6, 0, 0]
    m = _reg(_reg_ev().set_percentage_error_histogram_bins([-10.0, 0.0, 10.0]), _REAL)
    assert m["SignedPercentageErrorHistogram"]["counts"] == [1, 3]
    m = _reg(_reg_ev().set_percentage_error_histogram_bins([-INF, -1000.0, -10.0, 0.0, 10.0, 1000.0, INF]), _REAL)
    assert m["SignedPercentageErrorHistogram"]["counts"] == [1, 2, 1, 3, 2, 1]
    m = _reg(_reg_ev().set_percentage_error_histogram_bins([-INF, -100.0, 0.0, 100.0, INF]), [(1.0, 1.0)] * 5)
    assert m["SignedPercentageErrorHistogram"]["counts"] == [0, 0, 5, 0]


def test_regression_smart_cutoff_and_nans():
    ev = _reg_ev().set_smart_cutoff_ratio(0.1)
    _reg(ev, _REAL)
    assert ev.scaled_error_cutoff == pytest.approx(0.1 * sum(abs(r[0]) for r in _REAL) / len(_REAL))
    ev = _reg_ev().set_smart_cutoff_ratio(0.1)
    _reg(ev, [(0.0, 0.1), (0.0, 0.0), (0.0, 0.1), (0.0, 0.0), (0.0, 0.0)])
    assert ev.scaled_error_cutoff == 1e-3
    nan = float("nan")
    m = _reg(_reg_ev(), [(-2.0, 0.1), (nan, 0.0), (0.0, nan), (2.0, 0.0), (2.0, 0.0)])
    assert sum(m["SignedPercentageErrorHistogram"]["counts"]) == 3

"""Expectations ported from ``PercentileCalibratorTest.scala`` (estimator spec, 0..99 range, every bucket
used, uniformity, order preservation, the split / scaled-split summary metadata) and
``IsotonicRegressionCalibratorTest.scala`` (isotonic and antitonic fits: predictions, boundaries, model
predictions)."""
import numpy as np
import pytest
import torch
from scipy import stats

from transmogrifai_amd import dsl  # noqa: F401
from transmogrifai_amd.features import types as T
from transmogrifai_amd.stages.feature import math_stages as M
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder


def _calibrate(vals, **kw):
    ds, (f,) = TestFeatureBuilder.of(("score", T.RealNN, list(vals)))
    est = M.PercentileCalibrator(**kw).set_input(f)
    model = est.fit(ds)
    return est, model, model.transform(ds)[model.get_output_feature_name()].values.double().numpy()


def test_estimator_spec():
    _, _, out = _calibrate([10.0, 100.0, 1000.0])
    assert out.tolist() == [33.0, 66.0, 99.0]


def test_split_metadata_three_points():
    vals = [0.7231742029971469, 0.25329310557439133, 0.9908988967772393]
    est, _, _ = _calibrate(vals)
    summ = est.metadata["summary"]
    assert summ[M.ORIG_SPLITS_KEY] == ["-Infinity", "0.25329310557439133", "0.7231742029971469",
                                       "0.9908988967772393", "Infinity"]
    assert summ[M.SCALED_SPLITS_KEY] == ["0.0", "33.0", "66.0", "99.0", "99.0"]


@pytest.mark.parametrize("n", [1000, 30])
def test_range_buckets_uniformity_and_order(n):
    rng = np.random.default_rng(n)
    vals = rng.random(n)
    _, _, out = _calibrate(vals)
    assert out.max() == 99.0       # with fewer rows than buckets the reference pins only the maximum
    if n == 1000:
        assert out.min() == 0.0
        assert set(out.tolist()) == set(float(i) for i in range(100))
        counts = np.bincount(out.astype(int), minlength=100)
        assert stats.chisquare(counts).pvalue > 0.5
    # same order when sorted by score or by (percentile, score)
    by_prob = np.argsort(vals, kind="stable")
    by_perc = np.lexsort((vals, out))
    assert (by_prob == by_perc).all()


def test_to_percentile_shortcut():
    ds, (f,) = TestFeatureBuilder.of(("score", T.RealNN, list(np.linspace(0, 1, 500))))
    p = f.to_percentile()
    assert isinstance(p.origin_stage, M.PercentileCalibrator)
    out = p.origin_stage.fit(ds).transform(ds)[p.name].values.double().numpy()
    assert out.min() == 0.0 and out.max() == 99.0 and (np.diff(out) >= 0).all()


def _iso(labels, isotonic):
    ds, (y, x) = TestFeatureBuilder.of(("label", T.RealNN, [float(v) for v in labels]),
                                       ("score", T.RealNN, [float(i) for i in range(len(labels))]), response="label")
    est = M.IsotonicRegressionCalibrator(isotonic=isotonic).set_input(y, x)
    model = est.fit(ds)
    return model, model.transform(ds)[model.get_output_feature_name()].values.double().tolist()


def test_isotonic_calibration():
    model, pred = _iso([1, 2, 3, 1, 6, 17, 16, 17, 18], True)
    assert pred == [1, 2, 2, 2, 6, 16.5, 16.5, 17, 18]
    assert model.boundaries == [0, 1, 3, 4, 5, 6, 7, 8]
    assert model.predictions == [1, 2, 2, 6, 16.5, 16.5, 17.0, 18.0]


def test_antitonic_calibration():
    model, pred = _iso([7, 5, 3, 5, 1], False)
    assert pred == [7.0, 5.0, 4.0, 4.0, 1.0]
    assert model.boundaries == [0, 1, 2, 3, 4]
    assert model.predictions == [7.0, 5.0, 4.0, 4.0, 1.0]


def test_isotonic_shortcut():
    ds, (y, x) = TestFeatureBuilder.of(("label", T.RealNN, [1.0, 2.0, 3.0, 1.0, 6.0, 17.0, 16.0, 17.0, 18.0]),
                                       ("score", T.RealNN, [float(i) for i in range(9)]), response="label")
    c = x.to_isotonic_calibrated(y)
    out = c.origin_stage.fit(ds).transform(ds)[c.name].values.double().tolist()
    assert out == [1, 2, 2, 2, 6, 16.5, 16.5, 17, 18]


def test_percentile_model_roundtrip_ctor_args():
    m = M.PercentileCalibratorModel([float("-inf"), 1.0, 2.0, float("inf")], 4, 100)
    m2 = M.PercentileCalibratorModel()
    m2.load_ctor_args(m.ctor_args())
    x = torch.tensor([0.5, 1.0, 1.5, 3.0], dtype=torch.float64)
    assert m2.calibrate(x).tolist() == m.calibrate(x).tolist() == [50.0, 50.0, 99.0, 99.0]

"""``DecisionTreeNumericBucketizerTest.scala`` ported: the estimator spec rows (:53-67), the response flag of the
output (:107-120), no splits on random data (:122-128), null-only and empty data (:130-140), the ``autoBucketize``
shortcut (:142-150), uniform currency data with four label bands (:152-159) and label leakage through an
expected-revenue column (:161-192), each checked as the spec's ``assertBucketizer`` (:194-268): the fitted
model's flags, the splits within the relative tolerance (one extra split allowed), the vector size and the
metadata column count."""
import math

import numpy as np
import pytest

from transmogrifai_amd.features import types as T
from transmogrifai_amd.stages.feature.bucketizers import (DecisionTreeNumericBucketizer,
                                                          DecisionTreeNumericBucketizerModel)
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.testkit.random_data import RandomBinary, RandomReal

INF = float("inf")


def _assert_splits(splits, expected, tol):
    assert len(splits) in (len(expected), len(expected) + 1), (splits, expected)
    for s, e in zip(splits, expected):
        d = abs((s - e) / max(s, e)) if max(s, e) != 0 else math.nan
        if math.isfinite(d):
            assert d <= tol, (splits, expected)


def _assert_bucketizer(est, ds, should_split, track_nulls, track_invalid, expected_splits, tol):
    model = est.fit(ds)
    assert isinstance(model, DecisionTreeNumericBucketizerModel)
    assert model.uid == est.uid and model.operation_name == est.operation_name
    assert model.should_split == should_split
    assert model.track_nulls == track_nulls
    assert model.track_invalid == track_invalid
    _assert_splits(model.splits, expected_splits, tol)
    out = model.transform(ds)[model.get_output_feature_name()].values.double().numpy()
    n_split = 1 if should_split else 0
    size = len(model.splits) - n_split + (1 if track_nulls else 0) + (n_split if track_invalid else 0)
    assert out.shape[1] == size
    assert np.isin(out, (0.0, 1.0)).all()          # nominal columns (assertNominal)
    assert len(model.metadata["vector_metadata"].columns) == size
    return model, out


def _normal(seed=0):
    num = RandomReal.normal().with_probability_of_empty(0.2).reset(seed).take(1000)
    lab = [1.0 if b else 0.0 for b in RandomBinary(0.4).reset(seed + 1).take(1000)]
    ds, (numeric, label) = TestFeatureBuilder.of(("numeric", T.Real, num), ("label", T.RealNN, lab))
    return ds, numeric, label


def test_estimator_spec_rows():
    ds, (numeric, label) = TestFeatureBuilder.of(("numeric", T.Real, [1.0, 18.0, None, -1.23, 0.0]),
                                                 ("label", T.RealNN, [1.0, 1.0, 0.0, 0.0, 1.0]))
    est = DecisionTreeNumericBucketizer().set_input(label, numeric)
    model = est.fit(ds)
    out = model.transform(ds)[model.get_output_feature_name()].values.double().tolist()
    assert out == [[0, 1, 0], [0, 1, 0], [0, 0, 1], [1, 0, 0], [0, 1, 0]]


def test_output_is_response_only_when_both_inputs_are():
    _, numeric, label = _normal()
    for lr, nr in [(False, False), (True, False), (False, True)]:
        f = DecisionTreeNumericBucketizer().set_input(label._with_response(lr), numeric._with_response(nr))
        assert f.get_output().is_response is False
    f = DecisionTreeNumericBucketizer().set_input(label._with_response(True), numeric._with_response(True))
    assert f.get_output().is_response is True


def test_no_splits_on_random_data():
    ds, numeric, label = _normal()
    est = DecisionTreeNumericBucketizer(track_nulls=False).set_input(label, numeric)
    _assert_bucketizer(est, ds, False, False, False, [], 0.0)


def test_null_only_and_empty_data():
    ds, (label, numeric) = TestFeatureBuilder.of(("label", T.RealNN, [0.0]), ("numeric", T.Real, [None]))
    est = DecisionTreeNumericBucketizer(track_nulls=False).set_input(label, numeric)
    _assert_bucketizer(est, ds, False, False, False, [], 0.0)
    empty, (l2, n2) = TestFeatureBuilder.of(("label", T.RealNN, []), ("numeric", T.Real, []))
    est = DecisionTreeNumericBucketizer(track_nulls=False).set_input(l2, n2)
    with pytest.raises(ValueError, match="Dataset is empty, buckets cannot be computed"):
        est.fit(empty)


def test_auto_bucketize_shortcut():
    ds, numeric, label = _normal()
    out = numeric.auto_bucketize(label, track_nulls=True)
    assert isinstance(out.origin_stage, DecisionTreeNumericBucketizer)
    _assert_bucketizer(out.origin_stage, ds, False, True, False, [], 0.0)


def test_uniform_currency_label_bands():
    cur = [x * 100.0 / 1000 for x in range(1000)]
    lab = [0.0 if v < 15 else 1.0 if v < 26 else 2.0 if v < 91 else 3.0 for v in cur]
    ds, (currency, label) = TestFeatureBuilder.of(("currency", T.Currency, cur), ("label", T.RealNN, lab))
    out = currency.auto_bucketize(label, track_nulls=True, track_invalid=True, min_info_gain=0.1)
    _assert_bucketizer(out.origin_stage, ds, True, True, True, [-INF, 15, 26, 91, INF], 0.15)


def test_label_leakage_through_expected_revenue():
    b = RandomBinary(0.5).with_probability_of_empty(0.3).reset(3).take(1000)
    cur = RandomReal.log_normal(10.0, 1.0, ftype=T.Currency).reset(4).take(1000)
    er = [None if x is None else (1.0 if x else 0.0) * c for x, c in zip(b, cur)]
    lab = [1.0 if x else 0.0 for x in b]
    ds, (rb, rc, rer, label) = TestFeatureBuilder.of(
        ("binary", T.Binary, b), ("currency", T.Currency, cur), ("expectedRevenue", T.Currency, er),
        ("label", T.RealNN, lab))
    split_value = min(v for v in er if v is not None and v > 0) / 2.0
    out = rer.auto_bucketize(label, track_nulls=True, track_invalid=True)
    _assert_bucketizer(out.origin_stage, ds, True, True, True, [-INF, split_value, INF], 0.15)

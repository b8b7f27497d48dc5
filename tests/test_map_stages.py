"""Map vectorizers (``OPMapVectorizerTest``, ``TextMapPivotVectorizerTest``, ``DateMapToUnitCircleVectorizerTest``,
``TextMapLenEstimatorTest``, ``TextMapNullEstimatorTest``, ``DecisionTreeNumericMapBucketizerTest``)."""
import numpy as np
import pytest

from transmogrifai_amd.features import types as T
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.testkit.spec import check_estimator
from transmogrifai_amd.stages.feature import maps as MP
from transmogrifai_amd.stages.feature.bucketizers import DecisionTreeNumericMapBucketizer


def test_real_map_vectorizer_mean_fill():
    ds, (m,) = TestFeatureBuilder.of(("m", T.RealMap, [{"a": 1.0, "b": 2.0}, {"a": 3.0}, {}]))
    st = MP.RealMapVectorizer(track_nulls=True).set_input(m)
    model, out = check_estimator(st, ds, check_rows=False)
    assert out[0] == [1.0, 0.0, 2.0, 0.0] and out[1] == [3.0, 0.0, 2.0, 1.0] and out[2] == [2.0, 1.0, 2.0, 1.0]


def test_text_map_pivot():
    ds, (m,) = TestFeatureBuilder.of(("m", T.PickListMap, [{"c": "x"}, {"c": "y"}, {"c": "x"}, {}]))
    model, out = check_estimator(MP.TextMapPivotVectorizer(min_support=1, clean_text=False).set_input(m), ds,
                                 check_rows=False)
    names = [c.indicator_value for c in model.metadata["vector_metadata"].columns]
    assert names == ["x", "y", "OTHER", "NullIndicatorValue"] and out[3] == [0, 0, 0, 1]


def test_date_map_unit_circle():
    hour = 3_600_000
    ds, (m,) = TestFeatureBuilder.of(("m", T.DateMap, [{"k": 0}, {"k": 6 * hour}, {}]))
    model, out = check_estimator(MP.DateMapToUnitCircleVectorizer(time_period="HourOfDay").set_input(m), ds,
                                 check_rows=False)
    assert np.allclose(out[0], [1, 0]) and np.allclose(out[1], [0, 1], atol=1e-12) and out[2] == [0, 0]


def test_text_map_len_and_null():
    ds, (m,) = TestFeatureBuilder.of(("m", T.TextMap, [{"a": "hello world"}, {"b": "x"}, {}]))
    _, lens = check_estimator(MP.TextMapLenEstimator().set_input(m), ds, check_rows=False)
    assert lens[0] == [10.0, 0.0] and lens[1] == [0.0, 1.0]
    _, nulls = check_estimator(MP.TextMapNullEstimator().set_input(m), ds, check_rows=False)
    assert nulls[0] == [0.0, 1.0] and nulls[2] == [1.0, 1.0]


def test_dt_numeric_map_bucketizer():
    rng = np.random.default_rng(0)
    x = rng.uniform(0, 10, 300)
    y = (x > 5).astype(float)
    maps = [{"k": float(v)} if i % 10 else {} for i, v in enumerate(x)]
    ds, (lab, m) = TestFeatureBuilder.of(("y", T.RealNN, list(y)), ("m", T.RealMap, maps), response="y")
    model, out = check_estimator(DecisionTreeNumericMapBucketizer().set_input(lab, m), ds, check_rows=False)
    assert model.splits[0] and 4.0 < model.splits[0][1] < 6.0
    assert out[0][-1] == 1.0 and sum(out[1]) == 1.0

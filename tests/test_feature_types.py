"""Feature type system, UIDs and the feature DAG (FeatureTypeValueTest.scala, FeatureTypeFactoryTest,
ConcurrentCheck.scala:39-80, FeatureLikeTest / FeatureBuilderTest, UIDTest)."""
import math
import threading

import numpy as np
import pandas as pd
import pytest

from transmogrifai_amd import uid as UID
from transmogrifai_amd.features import types as T
from transmogrifai_amd.features.builder import FeatureBuilder
from transmogrifai_amd.features.feature import FeatureCycleException


def test_registry_has_53_types_and_resolves_names():
    assert len(T.ALL_TYPES) == 53
    for t in T.ALL_TYPES:
        assert T.feature_type_from_name(t.__name__) is t
        assert T.feature_type_from_name(t.type_name()) is t
        assert t.type_name() == f"com.salesforce.op.features.types.{t.__name__}"
    with pytest.raises(ValueError):
        T.feature_type_from_name("NoSuchType")


def test_hierarchy_matches_reference():
    assert T.is_subtype(T.RealNN, T.Real) and T.is_subtype(T.Percent, T.Real) and T.is_subtype(T.Currency, T.Real)
    assert T.is_subtype(T.DateTime, T.Date) and T.is_subtype(T.Date, T.Integral)
    for t in (T.Email, T.Base64, T.Phone, T.ID, T.URL, T.TextArea, T.PickList, T.ComboBox, T.Country, T.State,
              T.PostalCode, T.City, T.Street):
        assert T.is_subtype(t, T.Text)
    assert T.is_subtype(T.Prediction, T.RealMap) and T.is_subtype(T.DateTimeMap, T.DateMap)
    assert len(T.MAP_TYPES) == 25
    assert T.PickList.categorical and T.MultiPickList.categorical and T.Binary.categorical
    assert T.Geolocation.location and not T.RealNN.nullable and not T.Prediction.nullable


@pytest.mark.parametrize("t", T.ALL_TYPES, ids=lambda t: t.__name__)
def test_empty_values_and_defaults(t):
    if not t.nullable:
        with pytest.raises(T.NonNullableEmptyException):
            t(None)
        return
    e = t(None)
    assert e.is_empty and not e.non_empty
    assert e == t.empty()
    d = T.default_value(t)
    assert t(d).is_empty


def test_value_conversions():
    assert T.Real(float("nan")).is_empty and T.Real(3).value == 3.0
    assert T.Integral(4.0).value == 4 and isinstance(T.Integral(4.0).value, int)
    assert T.Binary(1).value is True and T.Binary(0).to_double() == 0.0 and T.Binary(None).to_double() is None
    assert T.MultiPickList(["a", "b", "a"]).value == frozenset({"a", "b"})
    assert T.TextList(None).value == [] and T.OPVector([1, 2]).value.dtype == np.float64
    g = T.Geolocation([37.7, -122.4, 2.0])
    assert (g.lat, g.lon, g.accuracy) == (37.7, -122.4, 2.0)
    with pytest.raises(ValueError):
        T.Geolocation([100.0, 0.0, 1.0])
    with pytest.raises(ValueError):
        T.Geolocation([1.0, 2.0])
    with pytest.raises(T.NonNullableEmptyException):
        T.RealNN(float("nan"))


def test_prediction_keys():
    p = T.Prediction(prediction=1.0, raw_prediction=[-2.0, 2.0], probability=[0.1, 0.9])
    assert p.prediction == 1.0 and p.raw_prediction == [-2.0, 2.0] and p.probability == [0.1, 0.9]
    assert set(p.value) == {"prediction", "rawPrediction_0", "rawPrediction_1", "probability_0", "probability_1"}
    assert p.score == [0.1, 0.9] and T.Prediction(prediction=3.5).score == [3.5]
    with pytest.raises(T.NonNullableEmptyException):
        T.Prediction({"probability_0": 1.0})


def test_equality_and_hash():
    assert T.Real(1.0) == T.Real(1.0) and T.Real(1.0) != T.Percent(1.0)
    assert T.Real(float("nan")) == T.Real(None)
    assert len({T.TextMap({"a": "x"}), T.TextMap({"a": "x"}), T.PickList("x")}) == 2
    assert T.OPVector([1.0, 2.0]) == T.OPVector(np.array([1.0, 2.0]))


def test_concurrent_construction():
    """ConcurrentCheck: type constructors hammered from 10 threads give the same values."""
    errors = []

    def work(k):
        try:
            for i in range(2000):
                v = T.Real(i * 0.5)
                assert v.value == i * 0.5
                assert T.MultiPickList([str(i), str(k)]).value == frozenset({str(i), str(k)})
                assert T.Prediction(prediction=float(i)).prediction == float(i)
        except Exception as e:     # pragma: no cover - reported below
            errors.append(e)

    th = [threading.Thread(target=work, args=(k,)) for k in range(10)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors


def test_uid_format_and_reset():
    UID.reset()
    a = UID.make_uid("RealVectorizer")
    b = UID.make_uid(T.Real)
    assert a == "RealVectorizer_000000000001" and b == "Real_000000000002"
    assert UID.from_string(a) == ("RealVectorizer", "000000000001")
    UID.reset()
    assert UID.make_uid("X") == "X_000000000001"


def test_feature_builder_and_dag():
    age = FeatureBuilder.Real("age").extract(lambda r: r["age"]).as_predictor()
    sex = FeatureBuilder.PickList("sex").extract(lambda r: r["sex"]).as_predictor()
    label = FeatureBuilder.RealNN("survived").extract(lambda r: r["survived"]).as_response()
    assert label.is_response and not age.is_response and age.is_raw
    from transmogrifai_amd.dsl import transmogrify
    vec = transmogrify([age, sex])
    assert {f.name for f in vec.raw_features()} == {"age", "sex"}
    stages = vec.parent_stages()
    assert min(stages.values()) == 0          # the combiner producing vec is at distance 0
    assert vec.origin_stage in stages and stages[vec.origin_stage] == 0
    js = vec.to_json()
    assert js["typeName"].endswith("OPVector") and js["parents"]
    assert vec.history().origin_features == ("age", "sex")


def test_feature_builder_from_dataframe_infers_types():
    df = pd.DataFrame({"y": [0.0, 1.0, 1.0], "x": [1.5, None, 2.0], "n": [1, 2, 3], "s": ["a", "b", None],
                       "b": [True, False, True]})
    resp, preds = FeatureBuilder.from_dataframe(df, response="y")
    assert resp.name == "y" and resp.is_response and resp.wtype is T.RealNN
    kinds = {f.name: f.wtype for f in preds}
    assert kinds["x"] is T.Real and kinds["n"] is T.Integral and kinds["b"] is T.Binary
    assert issubclass(kinds["s"], T.Text)


def test_cycle_detection():
    a = FeatureBuilder.Real("a").extract(lambda r: r["a"]).as_predictor()
    b = a + 1.0
    # forge a cycle a <- b <- a through the parents list
    a.parents = (b,)
    with pytest.raises((FeatureCycleException, ValueError)):
        b.parent_stages()

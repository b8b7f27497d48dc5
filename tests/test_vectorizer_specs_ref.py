"""Expected vectors and metadata of the reference's BinaryVectorizerTest and IntegralVectorizerTest
(``core/src/test/.../stages/impl/feature/``), through the OpTransformerSpec / OpEstimatorSpec contract."""
import pytest

from transmogrifai_amd.data.vector_metadata import NULL_STRING
from transmogrifai_amd.features import types as T
from transmogrifai_amd.stages.feature import vectorizers as V
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.testkit.spec import check_estimator, check_transformer

_BIN = [(False, False), (False, True), (True, False), (True, True), (None, False), (None, True), (False, None),
        (True, None), (None, None)]


def _meta(st, ds):
    return [(c.parent_feature_name[0], c.indicator_value)
            for c in st.transform(ds)[st.get_output().name].metadata.columns]


@pytest.mark.parametrize("track,fill,expected", [
    (True, False, [[0, 0, 0, 0], [0, 0, 1, 0], [1, 0, 0, 0], [1, 0, 1, 0], [0, 1, 0, 0], [0, 1, 1, 0], [0, 0, 0, 1],
                   [1, 0, 0, 1], [0, 1, 0, 1]]),
    (True, True, [[0, 0, 0, 0], [0, 0, 1, 0], [1, 0, 0, 0], [1, 0, 1, 0], [1, 1, 0, 0], [1, 1, 1, 0], [0, 0, 1, 1],
                  [1, 0, 1, 1], [1, 1, 1, 1]]),
    (False, False, [[0, 0], [0, 1], [1, 0], [1, 1], [0, 0], [0, 1], [0, 0], [1, 0], [0, 0]]),
    (False, True, [[0, 0], [0, 1], [1, 0], [1, 1], [1, 0], [1, 1], [0, 1], [1, 1], [1, 1]]),
])
def test_binary_vectorizer(track, fill, expected):
    ds, (f1, f2) = TestFeatureBuilder.of(("f1", T.Binary, [a for a, _ in _BIN]), ("f2", T.Binary, [b for _, b in _BIN]))
    st = V.BinaryVectorizer(track_nulls=track, fill_value=fill).set_input(f1, f2)
    check_transformer(st, ds, expected=expected)
    per = [None, NULL_STRING] if track else [None]
    assert _meta(st, ds) == [(f, v) for f in ("f1", "f2") for v in per]


def _integral_data(ftype):
    rows = [(4, 2, 2, None), (4, None, 1, None), (2, 4, 1, None), (None, 2, 2, None), (None, None, None, None)]
    return TestFeatureBuilder.of(*[(n, ftype, [r[k] for r in rows]) for k, n in enumerate(("inA", "inB", "inC", "inD"))])


def test_integral_vectorizer_fill_constant():
    ds, fs = _integral_data(T.Integral)
    est = V.IntegralVectorizer(fill_with_constant=True, fill_value=3, track_nulls=False).set_input(*fs)
    check_estimator(est, ds, expected=[[4, 2, 2, 3], [4, 3, 1, 3], [2, 4, 1, 3], [3, 2, 2, 3], [3, 3, 3, 3]])


@pytest.mark.parametrize("ftype", [T.Integral, T.Date, T.DateTime])
def test_integral_vectorizer_fill_mode(ftype):
    """The mode of each column (ties -> the smaller value; a column without values -> 0); Date and DateTime
    columns vectorize as Integral ones."""
    ds, fs = _integral_data(ftype)
    est = V.IntegralVectorizer(fill_with_mode=True, fill_with_constant=False, track_nulls=False).set_input(*fs)
    check_estimator(est, ds, expected=[[4, 2, 2, 0], [4, 2, 1, 0], [2, 4, 1, 0], [4, 2, 2, 0], [4, 2, 1, 0]])


def test_integral_vectorizer_tracked_nulls():
    ds, fs = _integral_data(T.Integral)
    est = V.IntegralVectorizer(fill_with_constant=True, fill_value=0, track_nulls=True).set_input(*fs)
    model, _ = check_estimator(est, ds, expected=[[4, 0, 2, 0, 2, 0, 0, 1], [4, 0, 0, 1, 1, 0, 0, 1],
                                                  [2, 0, 4, 0, 1, 0, 0, 1], [0, 1, 2, 0, 2, 0, 0, 1],
                                                  [0, 1, 0, 1, 0, 1, 0, 1]])
    assert _meta(model, ds) == [(f, v) for f in ("inA", "inB", "inC", "inD") for v in (None, NULL_STRING)]
    est = V.IntegralVectorizer(fill_with_mode=True, fill_with_constant=False, track_nulls=True).set_input(*fs)
    check_estimator(est, ds, expected=[[4, 0, 2, 0, 2, 0, 0, 1], [4, 0, 2, 1, 1, 0, 0, 1], [2, 0, 4, 0, 1, 0, 0, 1],
                                       [4, 1, 2, 0, 2, 0, 0, 1], [4, 1, 2, 1, 1, 1, 0, 1]])


def test_realnn_vectorizer_and_shortcut():
    vals = [-1.0, -4.0, 5.0, -5.5, 0.1, 2.0, 0.0]
    ds, (f1,) = TestFeatureBuilder.of(("f1", T.RealNN, vals))
    check_transformer(V.RealNNVectorizer().set_input(f1), ds, expected=[[v] for v in vals])
    assert isinstance(f1.vectorize().origin_stage, V.RealNNVectorizer)


# ------------------------------------------------------------------------------ GeolocationVectorizerTest
_GEO = [((32.4, -100.2, 3.0), (38.6, -110.4, 2.0), (39.1, -111.3, 3.0), None),
        ((40.1, -120.3, 4.0), (42.5, -95.4, 4.0), None, None),
        ((45.0, -105.5, 4.0), None, None, None)]


def _geo_ds():
    return TestFeatureBuilder.of(*[(n, T.Geolocation, [None if r[k] is None else list(r[k]) for r in _GEO])
                                  for k, n in enumerate(("inA", "inB", "inC", "inD"))])


def test_geolocation_vectorizer_fill_constant():
    ds, fs = _geo_ds()
    est = V.GeolocationVectorizer(fill_with_constant=True, fill_value=[50.0, 50.0, 4.0], track_nulls=False)
    est.set_input(*fs)
    c = [50.0, 50.0, 4.0]
    check_estimator(est, ds, expected=[[32.4, -100.2, 3.0, 38.6, -110.4, 2.0, 39.1, -111.3, 3.0] + c,
                                       [40.1, -120.3, 4.0, 42.5, -95.4, 4.0] + c + c,
                                       [45.0, -105.5, 4.0] + c + c + c])


@pytest.mark.parametrize("track", [False, True])
def test_geolocation_vectorizer_fill_mean(track):
    """Fill with each column's geographic mean (midpoint on the sphere, accuracy of the mean as the reference
    prints it): inB -> (40.79, -103.12, 0.0), inC -> its one value, inD (no values) -> (0, 0, 0); with null
    tracking each location gets a fourth, null-indicator column."""
    import numpy as np
    ds, fs = _geo_ds()
    est = V.GeolocationVectorizer(fill_with_constant=False, track_nulls=track).set_input(*fs)
    model, out = check_estimator(est, ds)
    m1, m2, m3 = [40.79, -103.12, 0.0], [39.1, -111.3, 3.0], [0.0, 0.0, 0.0]
    rows = [[[32.4, -100.2, 3.0], [38.6, -110.4, 2.0], [39.1, -111.3, 3.0], m3],
            [[40.1, -120.3, 4.0], [42.5, -95.4, 4.0], m2, m3],
            [[45.0, -105.5, 4.0], m1, m2, m3]]
    nulls = [[0, 0, 0, 1], [0, 0, 1, 1], [0, 1, 1, 1]]
    for got, exp, nl in zip(out, rows, nulls):
        want = [v for k, g in enumerate(exp) for v in (g + [float(nl[k])] if track else g)]
        assert np.allclose(got, want, atol=0.01), (got, want)


# -------------------------------------------------------------------- MonoidAggregatorDefaultsTest (geolocation)
def test_geolocation_midpoint_aggregator():
    """MonoidAggregatorDefaultsTest.scala:275-290: the midpoint of the base locations is (40.04, -106.33) with
    Unknown accuracy (the box spans thousands of miles); one location is its own midpoint."""
    import numpy as np
    from transmogrifai_amd.features.aggregators import Event, default_aggregator
    base = [[32.4, -100.2, 3.0], [38.6, -110.4, 2.0], [], [40.1, -120.3, 4.0], [42.5, -95.4, 4.0], [],
            [45.0, -105.5, 4.0]]
    agg = default_aggregator(T.Geolocation)
    assert np.allclose(agg.aggregate([Event(0, v) for v in base]), [40.04, -106.33, 0.0], atol=0.01)
    assert np.allclose(agg.aggregate([Event(0, base[0])]), base[0], atol=0.01)


def test_geolocation_map_midpoint_aggregator():
    """:363-400: per-key midpoints; keys a and b get State accuracy (their boxes span tens of miles), c keeps
    its one location's."""
    import numpy as np
    from transmogrifai_amd.features.aggregators import Event, default_aggregator
    rows = [{"a": [38.4, -110.2, 3.0]}, {"a": [38.6, -110.4, 2.0]}, {"a": []}, {"a": [39.1, -110.3, 4.0]},
            {"a": [38.5, -110.45, 4.0]}, {"a": []}, {"a": [39.0, -109.55, 4.0]}, {"b": [43.8, -108.7, 2.0]},
            {"b": [43.9, -109.6, 3.0]}, {"b": [43.4, -109.3, 2.0]}, {"b": []}, {"c": [40.4, -116.3, 2.0]},
            {"c": []}]
    got = default_aggregator(T.GeolocationMap).aggregate([Event(0, r) for r in rows])
    exp = {"a": [38.72, -110.18, 10.0], "b": [43.7, -109.2, 10.0], "c": [40.4, -116.3, 2.0]}
    assert set(got) == set(exp)
    for k, v in exp.items():
        assert np.allclose(got[k], v, atol=0.01), (k, got[k])

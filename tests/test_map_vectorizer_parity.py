"""Expected vectors and metadata ported from the reference map-vectorizer specs:
``IntegralMapVectorizerTest.scala`` (fills, null tracking, allow / block lists given as raw keys and cleaned
like the map keys), ``BinaryMapVectorizerTest.scala``, ``MultiPickListMapVectorizerTest.scala`` (same data
as the text-map pivot spec) and ``DecisionTreeNumericMapBucketizerTest.scala`` (the estimator spec rows and
the correlated-currency splits with ``trackInvalid``)."""
import numpy as np
import pytest

from transmogrifai_amd.data.vector_metadata import NULL_STRING, OTHER_STRING
from transmogrifai_amd.features import types as T
from transmogrifai_amd.stages.feature import maps as MP
from transmogrifai_amd.stages.feature.bucketizers import DecisionTreeNumericMapBucketizer
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder

INF = float("inf")


def _dense(size, idx, vals=None):
    v = [0.0] * size
    for k, i in enumerate(idx):
        v[i] = 1.0 if vals is None else float(vals[k])
    return v


def _fit_out(est, ds):
    m = est.fit(ds)
    return m, m.transform(ds)[m.get_output_feature_name()].values.double().tolist()


def _meta(m):
    return [(c.grouping, c.indicator_value) for c in m.metadata["vector_metadata"].columns]


def _int_data():
    m1 = [{"a": 1, "b": 5}, {"c": 11}, {}]
    m2 = [{"z": 10}, {"y": 3, "x": 0}, {}]
    return TestFeatureBuilder.of(("m1", T.IntegralMap, m1), ("m2", T.IntegralMap, m2))


def test_integral_map_vectorizer_expected_vectors():
    ds, (f1, f2) = _int_data()
    m, out = _fit_out(MP.IntegralMapVectorizer(track_nulls=False, clean_keys=True).set_input(f1, f2), ds)
    assert out == [[1.0, 5.0, 0.0, 0.0, 0.0, 10.0], _dense(6, [2, 4], [11.0, 3.0]), [0.0] * 6]
    assert _meta(m) == [("A", None), ("B", None), ("C", None), ("X", None), ("Y", None), ("Z", None)]
    m, out = _fit_out(MP.IntegralMapVectorizer(track_nulls=True, clean_keys=True).set_input(f1, f2), ds)
    assert out == [_dense(12, [0, 2, 5, 7, 9, 10], [1, 5, 1, 1, 1, 10]),
                   _dense(12, [1, 3, 4, 8, 11], [1, 1, 11, 3, 1]),
                   _dense(12, [1, 3, 5, 7, 9, 11])]
    assert _meta(m)[:2] == [("A", None), ("A", NULL_STRING)]


def test_integral_map_vectorizer_fill_value():
    ds, (f1, f2) = _int_data()
    _, out = _fit_out(MP.IntegralMapVectorizer(track_nulls=False, clean_keys=True, fill_value=100).set_input(f1, f2),
                      ds)
    assert out == [[1.0, 5.0, 100.0, 100.0, 100.0, 10.0], [100.0, 100.0, 11.0, 0.0, 3.0, 100.0], [100.0] * 6]
    _, out = _fit_out(MP.IntegralMapVectorizer(track_nulls=True, clean_keys=True, fill_value=100).set_input(f1, f2),
                      ds)
    assert out == [[1.0, 0.0, 5.0, 0.0, 100.0, 1.0, 100.0, 1.0, 100.0, 1.0, 10.0, 0.0],
                   [100.0, 1.0, 100.0, 1.0, 11.0, 0.0, 0.0, 0.0, 3.0, 0.0, 100.0, 1.0],
                   [100.0, 1.0] * 6]


def test_integral_map_vectorizer_allow_and_block_lists():
    ds, (f1, f2) = _int_data()
    m, out = _fit_out(MP.IntegralMapVectorizer(track_nulls=False, clean_keys=True, allow_keys=["a", "b", "z"])
                      .set_input(f1, f2), ds)
    assert out == [[1.0, 5.0, 10.0], [0.0] * 3, [0.0] * 3]
    assert _meta(m) == [("A", None), ("B", None), ("Z", None)]
    _, out = _fit_out(MP.IntegralMapVectorizer(track_nulls=True, clean_keys=True, allow_keys=["a", "b", "z"])
                      .set_input(f1, f2), ds)
    assert out == [_dense(6, [0, 2, 4], [1, 5, 10]), _dense(6, [1, 3, 5]), _dense(6, [1, 3, 5])]
    m, out = _fit_out(MP.IntegralMapVectorizer(track_nulls=False, clean_keys=True, block_keys=["a", "z"])
                      .set_input(f1, f2), ds)
    assert out == [_dense(4, [0], [5]), [0.0, 11.0, 0.0, 3.0], [0.0] * 4]
    assert _meta(m) == [("B", None), ("C", None), ("X", None), ("Y", None)]
    _, out = _fit_out(MP.IntegralMapVectorizer(track_nulls=True, clean_keys=True, block_keys=["a", "z"])
                      .set_input(f1, f2), ds)
    assert out == [_dense(8, [0, 3, 5, 7], [5, 1, 1, 1]), _dense(8, [1, 2, 6], [1, 11, 3]), _dense(8, [1, 3, 5, 7])]


def test_binary_map_vectorizer_expected_vectors():
    m1 = [{"a": False, "b": True}, {"c": False}, {}]
    m2 = [{"z": False}, {"y": True, "x": True}, {}]
    ds, (f1, f2) = TestFeatureBuilder.of(("m1", T.BinaryMap, m1), ("m2", T.BinaryMap, m2))
    m, out = _fit_out(MP.BinaryMapVectorizer(track_nulls=False, clean_keys=True).set_input(f1, f2), ds)
    assert out == [_dense(6, [1]), _dense(6, [3, 4]), [0.0] * 6]
    assert _meta(m) == [("A", None), ("B", None), ("C", None), ("X", None), ("Y", None), ("Z", None)]
    m, out = _fit_out(MP.BinaryMapVectorizer(track_nulls=True, clean_keys=True).set_input(f1, f2), ds)
    assert out == [_dense(12, [2, 5, 7, 9]), _dense(12, [1, 3, 6, 8, 11]), _dense(12, [1, 3, 5, 7, 9, 11])]
    assert [v for _, v in _meta(m)] == [None, NULL_STRING] * 6


_MPL_TOP = [{"a": {"d"}, "b": {"d"}}, {"a": {"e"}}, {"c": {"D"}}, {"c": {"d"}, "a": {"d"}}]
_MPL_BOT = [{"x": {"W"}}, {"z": {"w"}, "y": {"v"}}, {"x": {"w"}, "y": {"V"}}, {"z": {"v"}}]


@pytest.mark.parametrize("track_nulls,width,expected", [
    (False, 14, [[2, 5, 7], [3, 9, 12], [0, 7, 9], [0, 2, 11]]),
    (True, 20, [[2, 3, 7, 10, 15, 19], [2, 4, 9, 12, 13, 17], [0, 6, 9, 10, 13, 19], [0, 3, 9, 12, 15, 16]]),
])
def test_multi_pick_list_map_vectorizer_expected_vectors(track_nulls, width, expected):
    """MultiPickListMapVectorizerTest.scala (topK 10, minSupport 0, clean keys). The reference orders the
    keys of a map as Scala's Map iteration does (top: C, A, B); ours are sorted -- the columns are compared
    after placing ours in the reference key order, the values of a key keep their count-then-value order."""
    ds, (t, b) = TestFeatureBuilder.of(("top", T.MultiPickListMap, _MPL_TOP), ("bot", T.MultiPickListMap, _MPL_BOT))
    m = MP.MultiPickListMapVectorizer(clean_keys=True, min_support=0, top_k=10, track_nulls=track_nulls) \
        .set_input(t, b).fit(ds)
    out = np.asarray(m.transform(ds)[m.get_output_feature_name()].values.double())
    assert out.shape[1] == width
    cols = m.metadata["vector_metadata"].columns
    rank = {"top": "cab", "bot": "xyz"}
    order = sorted(range(len(cols)), key=lambda i: (cols[i].parent_feature_name[0] != "top",
                                                    rank[cols[i].parent_feature_name[0]].index(cols[i].grouping.lower()),
                                                    i))
    assert [sorted(order.index(j) for j in np.flatnonzero(r)) for r in out] == expected
    got = [(cols[i].grouping, cols[i].indicator_value) for i in order]
    ref = [("C", "D"), ("C", OTHER_STRING), ("A", "D"), ("A", "E"), ("A", OTHER_STRING), ("B", "D"),
           ("B", OTHER_STRING), ("X", "W"), ("X", OTHER_STRING), ("Y", "V"), ("Y", OTHER_STRING), ("Z", "V"),
           ("Z", "W"), ("Z", OTHER_STRING)]
    assert [g for g in got if g[1] != NULL_STRING] == ref


def test_dt_numeric_map_bucketizer_estimator_spec():
    """The estimator spec of DecisionTreeNumericMapBucketizerTest.scala: keys a, b, c; a splits once, b
    once, c (one row) not at all; null indicators tracked."""
    maps = [{"a": 1.0, "b": 1.0}, {"a": 18.0}, {"b": 0.0}, {"a": -1.23, "b": 1.0}, {"a": -1.23, "b": 1.0, "c": 117.0}]
    labels = [1.0, 1.0, 0.0, 0.0, 1.0]
    ds, (lab, m) = TestFeatureBuilder.of(("label", T.RealNN, labels), ("num", T.RealMap, maps), response="label")
    _, out = _fit_out(DecisionTreeNumericMapBucketizer().set_input(lab, m), ds)
    assert out == [_dense(7, [1, 4, 6]), _dense(7, [1, 5, 6]), _dense(7, [2, 3, 6]), _dense(7, [0, 4, 6]),
                   _dense(7, [0, 4])]


def test_dt_numeric_map_bucketizer_correlated_currency_splits():
    """'correctly bucketize when labels are specified': two map keys carry x in [0, 100) with the label a step
    function of x (steps at 15, 26, 91), one key carries uniform noise; minInfoGain 0.1, trackInvalid."""
    total = 1000
    rng = np.random.default_rng(3)
    x = [i * 100.0 / total for i in range(total)]
    noise = [None if rng.random() < 0.1 else float(rng.uniform(0, 100)) for _ in range(total)]
    lab = [0.0 if v < 15 else 1.0 if v < 26 else 2.0 if v < 91 else 3.0 for v in x]
    maps = [{k: v for k, v in (("f1", a), ("f2", b), ("f3", a)) if v is not None} for a, b in zip(x, noise)]
    ds, (y, m) = TestFeatureBuilder.of(("label", T.RealNN, lab), ("cur", T.CurrencyMap, maps), response="label")
    est = DecisionTreeNumericMapBucketizer(min_info_gain=0.1, track_nulls=True, track_invalid=True).set_input(y, m)
    model = est.fit(ds)
    assert model.keys == ["f1", "f2", "f3"]
    sp = dict(zip(model.keys, model.splits))
    assert sp["f2"] == []
    for k in ("f1", "f3"):
        assert sp[k][0] == -INF and sp[k][-1] == INF and len(sp[k]) == 5
        # the reference's assertSplits: relative difference per split <= expectedTolerance (0.15)
        for got, exp in zip(sp[k][1:-1], [15.0, 26.0, 91.0]):
            assert abs(got - exp) / max(got, exp) <= 0.15
    labels = [v for g, v in _meta(model) if g == "f1"]
    assert labels[-2:] == [OTHER_STRING, NULL_STRING] and len(labels) == 6
    assert [v for g, v in _meta(model) if g == "f2"] == [NULL_STRING]


def test_dt_numeric_map_bucketizer_clean_keys_and_lists():
    maps = [{"Key one": float(i % 7), "b": float(i)} for i in range(60)]
    labels = [float(i % 7 > 3) for i in range(60)]
    ds, (lab, m) = TestFeatureBuilder.of(("label", T.RealNN, labels), ("num", T.RealMap, maps), response="label")
    model = DecisionTreeNumericMapBucketizer(clean_keys=True, allow_keys=["key one"]).set_input(lab, m).fit(ds)
    assert model.keys == ["KeyOne"]
    out = model.transform(ds)[model.get_output_feature_name()].values.double().numpy()
    assert out.shape == (60, 3) and (out[:, :2].sum(1) == 1).all()
    model = DecisionTreeNumericMapBucketizer(block_keys=["b"]).set_input(lab, m).fit(ds)
    assert model.keys == ["Key one"]

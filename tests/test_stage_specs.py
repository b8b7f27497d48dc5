"""Every stage agrees across batch / row / key-value / reloaded-checkpoint paths
(the ``OpTransformerSpec`` / ``OpEstimatorSpec`` contract), plus expected values
mirroring the reference unit tests (``core/src/test/.../stages/impl/feature/*Test.scala``)."""
import math

import numpy as np
import pytest

from transmogrifai_amd.features import types as T
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.testkit.spec import check_estimator, check_transformer
from transmogrifai_amd.stages.feature import vectorizers as V
from transmogrifai_amd.stages.feature import math_stages as MS
from transmogrifai_amd.stages.feature import text_stages as TS
from transmogrifai_amd.data.vector_metadata import NULL_STRING


def test_real_vectorizer_mean_fill_and_nulls():
    # RealVectorizerTest: fill with mean of non-nulls, null indicator columns
    ds, (a, b) = TestFeatureBuilder.of(("a", T.Real, [4.0, None, 2.0, None]),
                                       ("b", T.Real, [1.0, 2.0, None, 3.0]))
    est = V.RealVectorizer(fill_with_constant=False, track_nulls=True).set_input(a, b)
    model, out = check_estimator(est, ds, expected=[[4, 0, 1, 0], [3, 1, 2, 0], [2, 0, 2, 1], [3, 1, 3, 0]])
    meta = model.metadata["vector_metadata"]
    assert [c.indicator_value for c in meta.columns] == [None, NULL_STRING, None, NULL_STRING]


def test_real_vectorizer_constant_fill_no_nulls():
    ds, (a,) = TestFeatureBuilder.of(("a", T.Real, [4.0, None, 2.0]))
    est = V.RealVectorizer(fill_value=-1.0, fill_with_constant=True, track_nulls=False).set_input(a)
    check_estimator(est, ds, expected=[[4], [-1], [2]])


def test_integral_vectorizer_mode_fill():
    ds, (a,) = TestFeatureBuilder.of(("a", T.Integral, [1, 3, 3, None, 2, 2]))
    est = V.IntegralVectorizer(fill_with_mode=True, fill_with_constant=False, track_nulls=True).set_input(a)
    # mode ties -> smallest value (2 and 3 both twice -> 2)
    check_estimator(est, ds, expected=[[1, 0], [3, 0], [3, 0], [2, 1], [2, 0], [2, 0]])


def test_binary_vectorizer():
    ds, (a,) = TestFeatureBuilder.of(("a", T.Binary, [True, None, False]))
    st = V.BinaryVectorizer(fill_value=False, track_nulls=True).set_input(a)
    check_transformer(st, ds, expected=[[1, 0], [0, 1], [0, 0]])


def test_realnn_vectorizer():
    ds, (a, b) = TestFeatureBuilder.of(("a", T.RealNN, [1.0, 2.0]), ("b", T.RealNN, [3.0, 4.0]))
    check_transformer(V.RealNNVectorizer().set_input(a, b), ds, expected=[[1, 3], [2, 4]])


def test_pivot_vectorizer_topk_other_null():
    vals = ["a"] * 5 + ["b"] * 3 + ["c"] * 1 + [None]
    ds, (f,) = TestFeatureBuilder.of(("f", T.PickList, vals))
    est = V.OpTextPivotVectorizer(top_k=2, min_support=2, clean_text=False, track_nulls=True).set_input(f)
    model, out = check_estimator(est, ds)
    meta = model.metadata["vector_metadata"]
    assert [c.indicator_value for c in meta.columns] == ["a", "b", "OTHER", NULL_STRING]
    assert out[0] == [1, 0, 0, 0] and out[5] == [0, 1, 0, 0] and out[8] == [0, 0, 1, 0] and out[9] == [0, 0, 0, 1]


def test_set_vectorizer():
    vals = [{"x", "y"}, {"x"}, set(), {"z"}, {"x", "z"}]
    ds, (f,) = TestFeatureBuilder.of(("f", T.MultiPickList, vals))
    est = V.OpSetVectorizer(top_k=10, min_support=1, clean_text=False, track_nulls=True).set_input(f)
    model, out = check_estimator(est, ds)
    names = [c.indicator_value for c in model.metadata["vector_metadata"].columns]
    assert names[:3] == ["x", "z", "y"] and names[-1] == NULL_STRING
    assert out[2][-1] == 1.0


def test_hashing_vectorizer_shapes():
    ds, (f,) = TestFeatureBuilder.of(("f", T.TextList, [["a", "b", "a"], [], ["c"]]))
    st = V.OPCollectionHashingVectorizer(num_features=16).set_input(f)
    out = check_transformer(st, ds)
    assert len(out[0]) == 16 and sum(out[0]) == 3 and sum(out[1]) == 0


def test_smart_text_vectorizer_pivot_vs_hash():
    cats = ["red", "blue", "green"] * 10
    free = [f"word{i} other{i % 7} thing" for i in range(30)]
    ds, (c, t) = TestFeatureBuilder.of(("c", T.Text, cats), ("t", T.Text, free))
    est = V.SmartTextVectorizer(max_cardinality=5, num_features=32, min_support=1, top_k=5).set_input(c, t)
    model, out = check_estimator(est, ds)
    assert model.metadata["text_methods"][0].lower().startswith("pivot")
    assert model.metadata["text_methods"][1].lower().startswith("hash")


def test_date_to_unit_circle():
    hour = 3600 * 1000
    ds, (d,) = TestFeatureBuilder.of(("d", T.DateTime, [0, 6 * hour, None]))
    st = V.DateToUnitCircleTransformer(time_period="HourOfDay").set_input(d)
    out = check_transformer(st, ds)
    assert np.allclose(out[0], [1.0, 0.0], atol=1e-9)
    assert np.allclose(out[1], [0.0, 1.0], atol=1e-9)
    assert np.allclose(out[2], [0.0, 0.0])


def test_date_list_vectorizer_since_last():
    day = 86_400_000
    ref = 10 * day
    ds, (d,) = TestFeatureBuilder.of(("d", T.DateList, [[1 * day, 3 * day], [], [9 * day]]))
    st = V.DateListVectorizer(pivot="SinceLast", reference_date=ref, track_nulls=True).set_input(d)
    out = check_transformer(st, ds)
    assert out[0] == [7.0, 0.0] and out[1][1] == 1.0 and out[2] == [1.0, 0.0]


def test_geolocation_vectorizer():
    ds, (g,) = TestFeatureBuilder.of(("g", T.Geolocation, [[10.0, 20.0, 1.0], None, [30.0, 40.0, 3.0]]))
    model, out = check_estimator(V.GeolocationVectorizer(track_nulls=True).set_input(g), ds)
    assert len(out[0]) == 4 and out[1][-1] == 1.0


def test_vectors_combiner_concatenates_metadata():
    ds, (a, b) = TestFeatureBuilder.of(("a", T.Real, [1.0, None]), ("b", T.PickList, ["x", "y"]))
    va = V.RealVectorizer(track_nulls=True).set_input(a).get_output()
    vb = V.OpTextPivotVectorizer(min_support=1).set_input(b).get_output()
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    comb = V.VectorsCombiner().set_input(va, vb).get_output()
    m = OpWorkflow().set_result_features(comb).set_input_dataset(ds).train()
    out = m.score()
    vec = out[comb.name]
    assert vec.values.shape[1] == 2 + 4
    assert vec.metadata.size == 6


@pytest.mark.parametrize("op,expected", [("plus", [5.0, None, None]), ("minus", [-3.0, None, None]),
                                         ("multiply", [4.0, None, None]), ("divide", [0.25, None, None])])
def test_binary_math(op, expected):
    ds, (a, b) = TestFeatureBuilder.of(("a", T.Real, [1.0, None, 2.0]), ("b", T.Real, [4.0, 3.0, None]))
    st = MS.BinaryMathTransformer(op).set_input(a, b)
    out = check_transformer(st, ds)
    assert out[0] == pytest.approx(expected[0])


@pytest.mark.parametrize("op", ["abs", "ceil", "floor", "round", "exp", "sqrt", "log"])
def test_unary_math(op):
    ds, (a,) = TestFeatureBuilder.of(("a", T.Real, [1.5, None, 4.0, 0.2]))
    check_transformer(MS.UnaryMathTransformer(op).set_input(a), ds)


def test_scalar_math():
    ds, (a,) = TestFeatureBuilder.of(("a", T.Real, [1.5, None]))
    out = check_transformer(MS.ScalarMathTransformer("multiply", 2.0).set_input(a), ds)
    assert out[0] == 3.0 and out[1] is None


def test_fill_missing_with_mean():
    ds, (a,) = TestFeatureBuilder.of(("a", T.Real, [1.0, None, 3.0]))
    check_estimator(MS.FillMissingWithMean().set_input(a), ds, expected=[1.0, 2.0, 3.0])


def test_standard_scaler():
    ds, (a,) = TestFeatureBuilder.of(("a", T.Real, [1.0, 2.0, 3.0]))
    model, out = check_estimator(MS.OpScalarStandardScaler().set_input(a), ds)
    assert out == pytest.approx([-1.0, 0.0, 1.0])


def test_numeric_bucketizer():
    ds, (a,) = TestFeatureBuilder.of(("a", T.Real, [-1.0, 0.5, 10.0, None]))
    st = MS.NumericBucketizer(splits=[float("-inf"), 0.0, 1.0, float("inf")], track_nulls=True).set_input(a)
    out = check_transformer(st, ds)
    assert out[0][:3] == [1, 0, 0] and out[1][:3] == [0, 1, 0] and out[2][:3] == [0, 0, 1] and out[3][-1] == 1


def test_percentile_calibrator_monotone():
    vals = [float(v) for v in np.random.default_rng(0).normal(size=200)]
    ds, (a,) = TestFeatureBuilder.of(("a", T.RealNN, vals))
    model, out = check_estimator(MS.PercentileCalibrator(expected_num_buckets=10).set_input(a), ds)
    order = np.argsort(vals)
    assert all(out[order[i]] <= out[order[i + 1]] for i in range(len(vals) - 1))


def test_isotonic_calibrator_monotone():
    rng = np.random.default_rng(1)
    x = rng.uniform(size=100)
    y = (rng.uniform(size=100) < x).astype(float)
    ds, (lab, f) = TestFeatureBuilder.of(("y", T.RealNN, list(y)), ("x", T.RealNN, list(x)), response="y")
    model, out = check_estimator(MS.IsotonicRegressionCalibrator().set_input(lab, f), ds)
    o = np.asarray(out)[np.argsort(x)]
    assert np.all(np.diff(o) >= -1e-12)


def test_text_tokenizer():
    ds, (t,) = TestFeatureBuilder.of(("t", T.Text, ["Hello, World! the cat", None, "A b"]))
    out = check_transformer(TS.TextTokenizer().set_input(t), ds)
    assert "hello" in out[0] and "world" in out[0]


def test_text_len_and_null():
    ds, (t,) = TestFeatureBuilder.of(("t", T.Text, ["abc", None, ""]))
    out = check_transformer(TS.TextLenTransformer().set_input(t), ds)
    assert out[0] == [3.0]


def test_hashing_tf_idf():
    ds, (t,) = TestFeatureBuilder.of(("t", T.TextList, [["a", "b"], ["a"], ["c", "c"]]))
    tf = TS.OpHashingTF(num_features=8).set_input(t)
    out = check_transformer(tf, ds)
    assert sum(out[2]) == 2
    tfo = tf.get_output()
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    idf = TS.IDF().set_input(tfo).get_output()
    m = OpWorkflow().set_result_features(idf).set_input_dataset(ds).train()
    res = m.score()[idf.name].values
    assert res.shape == (3, 8)


def test_valid_email():
    ds, (e,) = TestFeatureBuilder.of(("e", T.Email, ["a@b.com", "nope", None]))
    out = check_transformer(TS.ValidEmailTransformer().set_input(e), ds)
    assert out[0] is True and out[1] is False


def test_string_indexer_roundtrip():
    from transmogrifai_amd.stages.feature.indexers import OpStringIndexerNoFilter
    ds, (t,) = TestFeatureBuilder.of(("t", T.Text, ["b", "a", "b", "c", None]))
    model, out = check_estimator(OpStringIndexerNoFilter().set_input(t), ds)
    assert out[0] == 0.0 and out[2] == 0.0


def test_random_dataset_transmogrify_roundtrip(tmp_path):
    """All common feature types through transmogrify -> save -> load -> score gives identical vectors."""
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.workflow.workflow import OpWorkflow, OpWorkflowModel
    ds, feats = TestFeatureBuilder.random(40)
    vec = transmogrify(feats)
    m = OpWorkflow().set_result_features(vec).set_input_dataset(ds).train()
    a = m.score()[vec.name].values
    m.save(str(tmp_path / "m"))
    m2 = OpWorkflowModel.load(str(tmp_path / "m"))
    b = m2.score(ds)[vec.name].values
    assert a.shape == b.shape
    assert np.allclose(a.numpy(), b.numpy())

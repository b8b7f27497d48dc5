"""SanityChecker scenarios (SanityCheckerTest.scala:149-635): the 6-row eye-colour fixture, parameter
validation, sample-size guard, Spearman vs Pearson, drop-everything guard, duplicate features, label-only
correlations on a wide vector, and identical statistics for identical inputs.

Fixture values are the reference's (label isBlueEyed; columns age, height, height_null, gender,
testFeatNegCor): age is constant (zero variance, NaN correlation), gender equals the label and
testFeatNegCor its negation, so with maxCorrelation 0.99 those three are dropped."""
import math

import numpy as np
import pytest
import torch

from transmogrifai_amd.data.vector_metadata import OpVectorColumnMetadata, OpVectorMetadata
from transmogrifai_amd.features import types as T
from transmogrifai_amd.stages.preparators.sanity_checker import SanityChecker
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder

NAMES = ["age", "height", "height_null", "gender", "testFeatNegCor"]
ROWS = [  # isBlueEyed, age, height, height_null, gender, testFeatNegCor
    (1, 32, 5.0, 0, 0.5, 0), (0, 32, 4.0, 1, 0, 0.1), (1, 32, 6.0, 1, 0.5, 0),
    (1, 32, 5.5, 0, 0.5, 0), (0, 32, 5.4, 1, 0, 0.1), (0, 32, 5.4, 1, 0, 0.1)]


def _meta(name, names):
    return OpVectorMetadata(name, [OpVectorColumnMetadata((n,), (T.Real.type_name(),)) for n in names])


def _fixture(rows=ROWS, names=NAMES):
    ds, (label, vec) = TestFeatureBuilder.of(("isBlueEye", T.RealNN, [float(r[0]) for r in rows]),
                                             ("features", T.OPVector, [list(map(float, r[1:])) for r in rows]),
                                             response="isBlueEye")
    ds["features"].metadata = _meta(vec.name, names)
    return ds, label, vec


def _checker(label, vec, **kw):
    return SanityChecker(**kw).set_input(label, vec)


def test_removes_trouble_features():
    ds, label, vec = _fixture()
    sc = _checker(label, vec, max_correlation=0.99, min_variance=0.0, check_sample=1.0, remove_bad_features=True)
    model = sc.fit(ds)
    summ = model.metadata["summary"]
    cols = [c.make_col_name() for c in ds["features"].metadata.columns]
    assert summ["dropped"] == sorted([cols[0], cols[3], cols[4]])
    assert summ["names"] == cols + [label.name]
    corr = dict(zip(summ["correlationsWLabel"]["featuresIn"], summ["correlationsWLabel"]["values"]))
    assert corr[cols[0]] is None                         # constant column: NaN correlation
    assert corr[cols[3]] == pytest.approx(1.0) and corr[cols[4]] == pytest.approx(-1.0)
    out = model.transform(ds)[sc.get_output_feature_name()]
    assert out.values.shape == (6, 2)
    np.testing.assert_allclose(out.values.numpy(), np.array([r[2:4] for r in ROWS], float))
    assert out.metadata.size + len(summ["dropped"]) == len(NAMES)


def test_keeps_everything_when_not_removing():
    ds, label, vec = _fixture()
    model = _checker(label, vec, max_correlation=0.99, min_variance=0.0).fit(ds)
    assert model.metadata["summary"]["dropped"] == []
    out = model.transform(ds)[model.get_output_feature_name()]
    np.testing.assert_allclose(out.values.numpy(), ds["features"].values.numpy())


def test_param_validation_and_defaults():
    sc = SanityChecker()
    for name, bad in [("check_sample", -1.0), ("check_sample", 0.0), ("check_sample", 2.0),
                      ("min_correlation", -1.0), ("min_correlation", 2.0), ("max_correlation", -1.0),
                      ("max_correlation", 2.0), ("sample_upper_limit", -1), ("sample_lower_limit", -1)]:
        with pytest.raises(ValueError):
            sc.set(name, bad)
    p = SanityChecker().params
    assert (p["sample_lower_limit"], p["sample_upper_limit"], p["check_sample"]) == (1000, 1_000_000, 1.0)
    assert (p["max_correlation"], p["min_variance"], p["min_correlation"]) == (0.95, 1e-5, 0.0)
    assert (p["max_feature_correlation"], p["correlation_type"], p["remove_bad_features"]) == (0.99, "pearson", False)


def test_response_feature_vector_rejected():
    ds, label, vec = _fixture()
    with pytest.raises(ValueError, match="should not contain any response features"):
        SanityChecker().set_input(label, vec.as_response())


def test_zero_sample_size_fails():
    ds, label, vec = _fixture()
    sc = _checker(label, vec, remove_bad_features=True, check_sample=0.99999, sample_lower_limit=0,
                  sample_upper_limit=0)
    with pytest.raises(ValueError, match="Sample size cannot be zero"):
        sc.fit(ds)


def test_spearman_beats_pearson_on_monotone_nonlinear():
    x = np.arange(1.0, 21.0)
    rows = [(xi, xi ** 5) for xi in x]
    ds, (label, vec) = TestFeatureBuilder.of(("label", T.RealNN, [r[0] for r in rows]),
                                             ("features", T.OPVector, [[r[1]] for r in rows]), response="label")
    ds["features"].metadata = _meta(vec.name, ["feature"])

    def corr(kind):
        m = _checker(label, vec, correlation_type=kind, check_sample=0.99999).fit(ds)
        return m.metadata["summary"]["correlationsWLabel"]["values"][0]

    assert corr("spearman") == pytest.approx(1.0)
    assert corr("spearman") > corr("pearson")


def test_all_features_removed_fails():
    ds, label, vec = _fixture()
    sc = _checker(label, vec, max_correlation=0.000001, min_variance=1000, check_sample=0.999999,
                  remove_bad_features=True)
    with pytest.raises(ValueError, match="dropped all of your features"):
        sc.fit(ds)


def test_duplicate_features_above_max_feature_correlation():
    rng = np.random.default_rng(0)
    n = 400
    y = (rng.random(n) < 0.5).astype(float)
    a = y * 0.3 + rng.normal(0, 1, n)
    b = rng.normal(0, 1, n)
    rows = [(y[i], a[i], b[i], a[i]) for i in range(n)]          # column 2 duplicates column 0
    ds, (label, vec) = TestFeatureBuilder.of(("label", T.RealNN, [r[0] for r in rows]),
                                             ("features", T.OPVector, [list(r[1:]) for r in rows]), response="label")
    ds["features"].metadata = _meta(vec.name, ["a", "b", "a_copy"])
    m = _checker(label, vec, remove_bad_features=True, categorical_label=False).fit(ds)
    cols = [c.make_col_name() for c in ds["features"].metadata.columns]
    assert m.metadata["summary"]["dropped"] == [cols[2]]          # the later duplicate goes


def test_label_only_correlations_on_wide_vector():
    rng = np.random.default_rng(1)
    n, d = 200, 5000
    X = rng.normal(0, 1, (n, d))
    y = (X[:, 7] + 0.1 * rng.normal(0, 1, n) > 0).astype(float)
    ds, (label, vec) = TestFeatureBuilder.of(("label", T.RealNN, y.tolist()),
                                             ("features", T.OPVector, list(X)), response="label")
    ds["features"].metadata = _meta(vec.name, [f"f{i}" for i in range(d)])
    m = _checker(label, vec, feature_feature_corr_level="Off", categorical_label=False).fit(ds)
    vals = m.metadata["summary"]["correlationsWLabel"]["values"]
    assert len(vals) == d + 1
    assert int(np.nanargmax(np.abs(np.array(vals[:d], float)))) == 7
    ref = np.corrcoef(X[:, 7], y)[0, 1]
    assert vals[7] == pytest.approx(ref, rel=1e-9)


def test_same_statistics_for_same_inputs():
    ds, label, vec = _fixture()
    s1 = _checker(label, vec, min_variance=0.0).fit(ds).metadata["summary"]
    s2 = _checker(label, vec, min_variance=0.0).fit(ds).metadata["summary"]
    for k in ("correlationsWLabel", "featuresStatistics", "dropped"):
        assert s1[k] == s2[k]
    fs = s1["featuresStatistics"]
    X = np.array([r[1:] + (r[0],) for r in ROWS], float)
    np.testing.assert_allclose(fs["mean"], X.mean(0))
    np.testing.assert_allclose(fs["variance"], X.var(0, ddof=1))
    assert not any(math.isnan(v) for v in fs["max"])


# ------------------------------------------------------------------- text-map fixture (SanityCheckerTest.scala:77-98)
TEXT_ROWS = [
    ("0", 1.0, {"color": "red", "fruit": "berry", "beverage": "tea"}),
    ("1", 1.0, {"color": "orange", "fruit": "berry", "beverage": "coffee"}),
    ("2", 1.0, {"color": "yello", "fruit": "berry", "beverage": "water"}),
    ("3", 1.0, {"color": "green", "fruit": "berry"}),
    ("4", 1.0, {"color": "blue", "fruit": "berry"}),
    ("5", 1.0, {"color": "indigo", "fruit": "berry"}),
    ("6", 0.0, {"fruit": "peach"}),
    ("7", 0.0, {"fruit": "peach"}),
    ("8", 0.0, {"fruit": "mango"}),
    ("9", 0.0, {"beverage": "tea"}),
    ("10", 0.0, {"beverage": "coffee"}),
    ("11", 0.0, {"beverage": "water"})]


def _text_fixture():
    ds, (ident, target, tm) = TestFeatureBuilder.of(
        ("id", T.Text, [r[0] for r in TEXT_ROWS]), ("target", T.RealNN, [r[1] for r in TEXT_ROWS]),
        ("textMap", T.TextMap, [r[2] for r in TEXT_ROWS]), response="target")
    return ds, ident, target, tm


def _train_summary(ds, vec, checked):
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    model = OpWorkflow().set_result_features(vec, checked).set_input_dataset(ds).train()
    return model.get_origin_stage_of(checked).metadata["summary"]


def _validate(summ, names, dropped, nan_corr, ignored=(), feature_feature=None):
    """``SanityCheckerTest.validateTransformerOutput``."""
    assert sorted(summ["names"][:-1]) == sorted(names)
    corr = summ["correlationsWLabel"]
    assert sorted(n for n, v in zip(corr["featuresIn"], corr["values"]) if v is None or v != v) == sorted(nan_corr)
    assert sorted(corr["featuresIn"]) == sorted([n for n in names if n not in set(ignored)] + [summ["names"][-1]])
    assert sorted(summ["dropped"]) == sorted(dropped)
    if feature_feature is not None:
        assert bool(summ.get("correlationsWFeatures")) == feature_feature


def _smart_map(tm, strategy, num_features):
    from transmogrifai_amd.stages.feature.maps import SmartTextMapVectorizer
    return SmartTextMapVectorizer(max_cardinality=2, num_features=num_features, min_support=1, top_k=2,
                                  prepend_feature_name=True, coverage_pct=1.0,
                                  hash_space_strategy=strategy).set_input(tm).get_output()


SHARED_NAMES = [f"textMap_{i}" for i in range(8)] + ["textMap_color_NullIndicatorValue_8",
                                                       "textMap_fruit_NullIndicatorValue_9",
                                                       "textMap_beverage_NullIndicatorValue_10"]


def test_removes_individual_text_hash_features_independently():
    """SanityCheckerTest.scala:359-391: shared hash space; protected shared hashes are judged one by one."""
    ds, _, target, tm = _text_fixture()
    vec = _smart_map(tm, "shared", 8)
    checked = SanityChecker(check_sample=1.0, remove_bad_features=True, remove_feature_group=True,
                            protect_text_shared_hash=True, min_correlation=0.0, max_correlation=0.8,
                            max_cramers_v=0.8).set_input(target, vec).get_output()
    summ = _train_summary(ds, vec, checked)
    _validate(summ, SHARED_NAMES, ["textMap_4", "textMap_7", "textMap_color_NullIndicatorValue_8"], ["textMap_7"])


def test_removes_text_hash_features_as_groups():
    """SanityCheckerTest.scala:393-434: separate hash spaces per key; a bad key's whole hash group goes."""
    ds, _, target, tm = _text_fixture()
    vec = _smart_map(tm, "separate", 4)
    checked = SanityChecker(check_sample=1.0, remove_bad_features=True, remove_feature_group=True,
                            protect_text_shared_hash=True, min_correlation=0.0, max_correlation=0.8,
                            max_cramers_v=0.8).set_input(target, vec).get_output()
    summ = _train_summary(ds, vec, checked)
    names = ([f"textMap_color_{i}" for i in range(4)] + [f"textMap_fruit_{i}" for i in range(4, 8)] +
             [f"textMap_beverage_{i}" for i in range(8, 12)] +
             ["textMap_color_NullIndicatorValue_12", "textMap_fruit_NullIndicatorValue_13",
              "textMap_beverage_NullIndicatorValue_14"])
    dropped = ["textMap_color_0", "textMap_color_1", "textMap_color_2", "textMap_color_3", "textMap_fruit_4",
               "textMap_fruit_5", "textMap_fruit_6", "textMap_fruit_7", "textMap_beverage_8", "textMap_beverage_9",
               "textMap_color_NullIndicatorValue_12", "textMap_fruit_NullIndicatorValue_13"]
    nan = ["textMap_color_1", "textMap_color_2", "textMap_fruit_4", "textMap_beverage_8", "textMap_beverage_9"]
    _validate(summ, names, dropped, nan)


def test_no_correlations_on_hashed_text_smart_map():
    """SanityCheckerTest.scala:436-471: CorrelationExclusion.HashedText leaves the shared hash columns out of the
    correlations (and so out of the correlation-based removals)."""
    ds, _, target, tm = _text_fixture()
    vec = _smart_map(tm, "shared", 8)
    checked = SanityChecker(check_sample=1.0, remove_bad_features=True, remove_feature_group=True,
                            protect_text_shared_hash=True, correlation_exclusion="HashedText", min_correlation=0.0,
                            max_correlation=0.8, max_feature_correlation=1.0, max_cramers_v=0.8).set_input(
        target, vec).get_output()
    summ = _train_summary(ds, vec, checked)
    _validate(summ, SHARED_NAMES, ["textMap_7", "textMap_color_NullIndicatorValue_8"], [],
              ignored=[f"textMap_{i}" for i in range(8)])


def test_no_correlations_on_hashed_text_vectorizer():
    """SanityCheckerTest.scala:502-533: the same exclusion through ``textMap.vectorize`` (512 shared hashes + per-key
    null indicators, keys sorted)."""
    ds, _, target, tm = _text_fixture()
    vec = tm.vectorize(clean_text=True)
    checked = SanityChecker(check_sample=1.0, remove_bad_features=True, remove_feature_group=True,
                            protect_text_shared_hash=True, correlation_exclusion="HashedText", min_variance=-0.1,
                            min_correlation=0.0, max_correlation=0.8, max_feature_correlation=1.0,
                            max_cramers_v=0.8).set_input(target, vec).get_output()
    summ = _train_summary(ds, vec, checked)
    hashed = [f"textMap_{i}" for i in range(512)]
    names = hashed + ["textMap_beverage_NullIndicatorValue_512", "textMap_color_NullIndicatorValue_513",
                      "textMap_fruit_NullIndicatorValue_514"]
    _validate(summ, names, ["textMap_color_NullIndicatorValue_513"], [], ignored=hashed)


def test_maps_with_the_same_keys():
    """SanityCheckerTest.scala:617-633: two pick-list maps with the same keys and a real map: nothing dropped, one
    categorical group per (map, key) pivot, 2 labels in every contingency matrix."""
    from transmogrifai_amd.dsl import transmogrify
    rng = np.random.default_rng(0)
    ds, (ident, target, m1, m2, dm) = TestFeatureBuilder.of(
        ("id", T.Text, [r[0] for r in TEXT_ROWS]), ("target", T.RealNN, [r[1] for r in TEXT_ROWS]),
        ("textMap1", T.PickListMap, [r[2] for r in TEXT_ROWS]), ("textMap2", T.PickListMap, [r[2] for r in TEXT_ROWS]),
        ("doubleMap", T.RealMap, [{k: float(rng.random()) for k in r[2]} for r in TEXT_ROWS]))
    feats = transmogrify([ident, target, m1, m2, dm])          # the target also as a predictor, as the reference
    checked = target.as_response().sanity_check(feats, categorical_label=True)
    summ = _train_summary(ds, feats, checked)
    assert summ["dropped"] == []
    cats = summ["categoricalStats"]
    assert len(cats) == 10
    assert all(len((c.get("contingencyMatrix") or c["contingency"])["0"]) == 2 for c in cats)


def test_tiny_check_sample_still_fits():
    """``SanityCheckerTest.scala:237-249``: a 1e-6 check sample on 6 rows is lifted to the sample lower limit; the
    fit runs through."""
    ds, label, vec = _fixture()
    _checker(label, vec, max_correlation=0.99, min_variance=0.0, check_sample=0.000001,
             remove_bad_features=True).fit(ds)


def test_missing_vector_metadata_is_an_error():
    """``SanityCheckerTest.scala:257-277``: a feature vector without OpVectorMetadata cannot be checked (the
    column names and groups come from it)."""
    rows = [(32, [5.0, 1, 1, 0]), (32, [4.0, 0, 0, 1]), (34, [6.0, 1, 1, 0]), (32, [5.5, 1, 1, 0]),
            (30, [5.4, 0, 0, 1]), (32, [5.4, 0, 0, 1])]
    ds, (label, vec) = TestFeatureBuilder.of(("label", T.RealNN, [float(r[0]) for r in rows]),
                                             ("features", T.OPVector, [r[1] for r in rows]), response="label")
    ds["features"].metadata = None
    sc = _checker(label, vec, remove_bad_features=True, check_sample=1.0)
    with pytest.raises(ValueError):
        sc.fit(ds).transform(ds)

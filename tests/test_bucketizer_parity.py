"""Expectations ported from ``NumericBucketizerTest.scala`` (explicit labels, derived left / right labels,
null and invalid tracking, param validation, out-of-bounds errors, the ``bucketize`` shortcut on reals and
integrals) and ``DecisionTreeNumericMapBucketizerTest.scala`` (the map ``autoBucketize`` shortcut)."""
import numpy as np
import pytest

from transmogrifai_amd import dsl  # noqa: F401  (registers the DSL methods)
from transmogrifai_amd.data.vector_metadata import NULL_STRING, OTHER_STRING
from transmogrifai_amd.features import types as T
from transmogrifai_amd.stages.feature.bucketizers import DecisionTreeNumericMapBucketizer
from transmogrifai_amd.stages.feature.math_stages import NumericBucketizer
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder

INF = float("inf")
NUMBERS = [10.0, None, 3.0, 5.0, 6.0, None, 1.0, 0.0]
SPLITS = [0.0, 1.0, 5.0, 10.0, INF]
LABELS = ["0-1", "1-5", "5-10", "10-Infinity"]
EXPECTED = [[0, 0, 0, 1], [0, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, 0], [0, 0, 1, 0], [0, 0, 0, 0], [0, 1, 0, 0],
            [1, 0, 0, 0]]
EXPECTED_RIGHT = [[0, 0, 0, 1], [0, 0, 0, 0], [0, 0, 1, 0], [0, 0, 1, 0], [0, 0, 0, 1], [0, 0, 0, 0], [0, 1, 0, 0],
                  [1, 0, 0, 0]]


def _run(stage, ds):
    out = stage.transform(ds)[stage.get_output_feature_name()].values.double().tolist()
    return out, [c.indicator_value for c in stage.metadata["vector_metadata"].columns]


@pytest.mark.parametrize("ftype", [T.Real, T.Integral])
def test_explicit_labels_and_null_tracking(ftype):
    vals = NUMBERS if ftype is T.Real else [None if v is None else int(v) for v in NUMBERS]
    ds, (num,) = TestFeatureBuilder.of(("num", ftype, vals))
    out, meta = _run(NumericBucketizer(track_nulls=False).set_buckets(SPLITS, LABELS).set_input(num), ds)
    assert out == EXPECTED and meta == LABELS
    out, meta = _run(NumericBucketizer(track_nulls=True).set_buckets(SPLITS, LABELS).set_input(num), ds)
    assert out == [e + [1.0 if v is None else 0.0] for e, v in zip(EXPECTED, NUMBERS)]
    assert meta == LABELS + [NULL_STRING]
    out, meta = _run(NumericBucketizer(track_nulls=False).set_buckets(SPLITS).set_input(num), ds)
    assert meta == ["[0.0-1.0)", "[1.0-5.0)", "[5.0-10.0)", "[10.0-Infinity)"]
    # the DSL shortcut
    f = num.bucketize(track_nulls=False, splits=SPLITS, bucket_labels=LABELS)
    assert f.origin_stage.transform(ds)[f.name].values.double().tolist() == EXPECTED
    f = num.bucketize(track_nulls=False, splits=[-INF, 0.0, 1.0, 5.0, 10.0], split_inclusion="Right")
    assert f.origin_stage.transform(ds)[f.name].values.double().tolist() == EXPECTED_RIGHT


def test_param_validation_and_label_updates():
    b = NumericBucketizer()
    with pytest.raises(ValueError):
        b.set_buckets([0, 1, 5, 10], ["0-1K", "1K-5K"])        # not enough labels
    with pytest.raises(ValueError):
        b.set_buckets([10, 1, 5], ["0-1K", "1K-5K"])            # not increasing
    with pytest.raises(ValueError):
        b.set_buckets([0, 1], ["0-1K"])                          # fewer than 3 points
    with pytest.raises(ValueError):
        b.set_buckets([0, float("nan"), 100], ["0-1K", "1K-5K"])
    b.set_buckets([7.0, 8.0, 10.0, 11.0])
    assert b.get_splits() == [7.0, 8.0, 10.0, 11.0]
    assert b.get_bucket_labels() == ["[7.0-8.0)", "[8.0-10.0)", "[10.0-11.0)"]
    b.set("split_inclusion", "Right")
    assert b.get_bucket_labels() == ["(7.0-8.0]", "(8.0-10.0]", "(10.0-11.0]"]
    b.set_buckets([7.0, 8.0, 10.0, 11.0], ["A", "B", "C"])
    assert b.get_bucket_labels() == ["A", "B", "C"]


def test_out_of_bounds_without_track_invalid_raises():
    ds, (num,) = TestFeatureBuilder.of(("num", T.Real, [INF, float("nan"), -1.0, -100.0]))
    with pytest.raises(ValueError, match="outside the bounds"):
        NumericBucketizer(track_invalid=False).set_buckets(SPLITS).set_input(num).transform(ds)


def test_track_invalid():
    """The reference rows are (empty, NaN, -Inf, +Inf, 10.0) -> (null, invalid, invalid, invalid, invalid).
    Here NaN is read as an empty value (docs/PARITY.md, deliberate deviations), so its row is the null one."""
    ds, (num,) = TestFeatureBuilder.of(("num", T.Real, [None, float("nan"), -INF, INF, 10.0]))
    f = num.bucketize(track_nulls=True, track_invalid=True, splits=[0.0, 1.0, 5.0])
    out = f.origin_stage.transform(ds)[f.name].values.double().tolist()
    assert out == [[0, 0, 0, 1], [0, 0, 0, 1], [0, 0, 1, 0], [0, 0, 1, 0], [0, 0, 1, 0]]
    assert [c.indicator_value for c in f.origin_stage.metadata["vector_metadata"].columns] == \
        ["[0.0-1.0)", "[1.0-5.0)", OTHER_STRING, NULL_STRING]


def test_random_reals_sign_buckets():
    rng = np.random.default_rng(11)
    vals = [0.0] + [None if rng.random() < 0.3 else float(rng.uniform(-1e7, 1e7)) for _ in range(1000)]
    ds, (num,) = TestFeatureBuilder.of(("num", T.Real, vals))
    f = num.bucketize(track_nulls=True, splits=[-INF, 0.0, INF], split_inclusion="Left")
    out = f.origin_stage.transform(ds)[f.name].values.double().tolist()
    for v, r in zip(vals, out):
        assert r == ([0, 0, 1] if v is None else [0, 1, 0] if v >= 0 else [1, 0, 0])


def test_map_auto_bucketize_shortcut():
    rng = np.random.default_rng(2)
    x = rng.uniform(0, 100, 600)
    lab = [float(v >= 40) for v in x]
    maps = [{"k": float(v), "noise": float(rng.uniform())} for v in x]
    ds, (y, m) = TestFeatureBuilder.of(("label", T.RealNN, lab), ("m", T.CurrencyMap, maps), response="label")
    out = m.auto_bucketize(y, track_nulls=True, min_info_gain=0.1)
    st = out.origin_stage
    assert isinstance(st, DecisionTreeNumericMapBucketizer)
    model = st.fit(ds)
    sp = dict(zip(model.keys, model.splits))
    assert sp["noise"] == [] and len(sp["k"]) == 3 and abs(sp["k"][1] - 40.0) < 1.0

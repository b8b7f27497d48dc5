"""RawFeatureFilter on the reference's passenger fixture: ports of ``RawFeatureFilterTest.scala:64-386`` (feature
statistics, cleaned data and blocklists, response / protected / JS-protected features, null-label leakage at four
correlation thresholds). Training reader = the aggregated passengers (6 keys), scoring reader = the 8 raw records."""
import pytest

from transmogrifai_amd import uid
from transmogrifai_amd.features.builder import FeatureBuilder
from transmogrifai_amd.filters.raw_feature_filter import RawFeatureFilter
from transmogrifai_amd.testkit import passenger as PF

pytestmark = pytest.mark.skipif(not PF.available(), reason="reference test data not mounted")


@pytest.fixture
def fx():
    uid.reset(0)
    return PF.PassengerFeatures()


def _names(fs):
    return sorted(f.name for f in fs)


def _surv_pred(fx):
    """``survived.copy(isResponse = false)``: a predictor over the response's generator stage (aggregated with the
    response's event window, as the reference's stage-built aggregator does)."""
    from transmogrifai_amd.features.feature import FeatureLike
    s = fx.survived
    return FeatureLike(s.name, s.wtype, False, s.origin_stage, [], uid=s.uid)


def _check_distributions(res, total):
    """``assertFeatureDistributions``: training then scoring distributions, half each."""
    ds = res.rawFeatureDistributions
    assert len(ds) == total
    tr = [d for d in ds if d.type == "Training"]
    sc = [d for d in ds if d.type == "Scoring"]
    assert len(tr) == total // 2 and len(sc) == total // 2
    assert ds == tr + sc


def _map_keys(cleaned, name):
    keys = set()
    for v in cleaned[name].to_list():
        keys |= set((v or {}).keys())
    return keys


def test_clean_dataset_and_blocklists(fx):
    """``:270-294``: nothing dropped at permissive thresholds; with minFill 0.5 / maxFillDifference 0.5 the
    predictor copy of the label and the maps' "Male" key go, the cleaned maps keep "Female" only."""
    surv = _surv_pred(fx)
    feats = [surv, fx.age, fx.gender, fx.height, fx.weight, fx.description, fx.boarded, fx.stringMap,
             fx.numericMap, fx.booleanMap]
    rff = RawFeatureFilter(PF.data_reader(), PF.simple_reader(), bins=10, min_fill_rate=0.0, max_fill_difference=1.0,
                           max_fill_ratio_diff=float("inf"), max_js_divergence=1.0, max_correlation=1.0,
                           min_scoring_rows=0)
    cleaned, drop, keys, res = rff.generate_filtered_raw(feats)
    assert drop == [] and not keys
    assert set(cleaned.columns) == {f.name for f in feats}
    _check_distributions(res, 26)
    rff1 = RawFeatureFilter(PF.data_reader(), PF.simple_reader(), bins=10, min_fill_rate=0.5, max_fill_difference=0.5,
                            max_fill_ratio_diff=float("inf"), max_js_divergence=1.0, max_correlation=1.0,
                            min_scoring_rows=0)
    cleaned1, drop1, keys1, res1 = rff1.generate_filtered_raw(feats)
    assert _names(drop1) == ["survived"]
    assert {k: set(v) for k, v in keys1.items()} == {"numericMap": {"Male"}, "booleanMap": {"Male"},
                                                     "stringMap": {"Male"}}
    assert "survived" not in cleaned1.columns
    assert _map_keys(cleaned1, "stringMap") <= {"Female"}


def test_response_features_are_never_dropped(fx):
    """``:296-308``."""
    feats = fx.raw_features
    rff = RawFeatureFilter(PF.data_reader(), PF.simple_reader(), bins=10, min_fill_rate=0.5, max_fill_difference=0.5,
                           max_fill_ratio_diff=float("inf"), max_js_divergence=1.0, max_correlation=1.0,
                           min_scoring_rows=0)
    cleaned, drop, keys, res = rff.generate_filtered_raw(feats)
    assert drop == []
    assert set(cleaned.columns) == {f.name for f in feats}
    assert _map_keys(cleaned, "stringMap") <= {"Female"}
    _check_distributions(res, 26)


def test_protected_features_are_kept(fx):
    """``:310-331``."""
    feats = [fx.survived, fx.age, fx.gender, fx.height, fx.weight, fx.description, fx.boarded]
    kw = dict(bins=10, min_fill_rate=0.1, max_fill_difference=0.1, max_fill_ratio_diff=2, max_js_divergence=0.2,
              max_correlation=0.9, min_scoring_rows=0)
    rff = RawFeatureFilter(PF.data_reader(), PF.simple_reader(), protected_features=[fx.age.name], **kw)
    cleaned, drop, keys, res = rff.generate_filtered_raw(feats)
    assert _names(drop) == _names([fx.gender, fx.height, fx.weight, fx.description, fx.boarded])
    assert set(cleaned.columns) == {"survived", "age"}
    _check_distributions(res, 14)
    rff2 = RawFeatureFilter(PF.data_reader(), PF.simple_reader(), protected_features=[fx.age.name, fx.gender.name],
                            **kw)
    cleaned2, drop2, _, _ = rff2.generate_filtered_raw(feats)
    assert _names(drop2) == _names([fx.height, fx.weight, fx.description, fx.boarded])
    assert set(cleaned2.columns) == {"survived", "age", "gender"}


def test_js_divergence_protected_features(fx):
    """``:333-356``: with maxJSDivergence 0 every distribution shift drops a feature, except the protected ones."""
    feats = [fx.survived, fx.age, fx.gender, fx.height, fx.weight, fx.description, fx.boarded, fx.boardedTime,
             fx.boardedTimeAsDateTime]
    rff = RawFeatureFilter(PF.data_reader(), PF.simple_reader(), bins=10, min_fill_rate=0.0, max_fill_difference=1.0,
                           max_fill_ratio_diff=float("inf"), max_js_divergence=0.0, max_correlation=1.0,
                           protected_js_features=[fx.boardedTime.name, fx.boardedTimeAsDateTime.name],
                           min_scoring_rows=0)
    cleaned, drop, keys, res = rff.generate_filtered_raw(feats)
    assert _names(drop) == _names([fx.age, fx.gender, fx.height, fx.weight, fx.description, fx.boarded])
    assert set(cleaned.columns) == {"survived", "boardedTime", "boardedTimeAsDateTime"}
    _check_distributions(res, 18)


@pytest.mark.parametrize("max_corr,dropped,map_keys,dropped_keys", [
    (0.9, ["boarded", "weight", "gender"], {"Female", "Male"}, {}),
    (0.6, ["boarded", "weight", "gender", "age"], {"Female", "Male"}, {}),
    (0.4, ["boarded", "weight", "gender", "age", "description"], {"Male"},
     {"booleanMap": {"Female"}, "stringMap": {"Female"}, "numericMap": {"Female"}}),
    (0.3, ["boarded", "weight", "gender", "age", "description", "booleanMap", "numericMap", "stringMap"], set(), {}),
])
def test_null_label_leakage(fx, max_corr, dropped, map_keys, dropped_keys):
    """``:358-385`` (``nullLabelCorrelationTest``)."""
    feats = fx.raw_features
    rff = RawFeatureFilter(PF.data_reader(), PF.simple_reader(), bins=10, min_fill_rate=0.0, max_fill_difference=1.0,
                           max_fill_ratio_diff=float("inf"), max_js_divergence=1.0, max_correlation=max_corr,
                           min_scoring_rows=0)
    cleaned, drop, keys, res = rff.generate_filtered_raw(feats)
    _check_distributions(res, 26)
    assert _names(drop) == sorted(dropped)
    assert {k: set(v) for k, v in keys.items()} == dropped_keys
    assert set(cleaned.columns) == {f.name for f in feats} - set(dropped)
    for m in ("booleanMap", "numericMap", "stringMap"):
        if map_keys:
            assert _map_keys(cleaned, m) == map_keys
        else:
            assert m not in cleaned.columns

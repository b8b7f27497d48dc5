"""RawFeatureFilter exclusion rules on fixed distributions: ports of ``RawFeatureFilterTest.scala:156-268`` with the
reference's ``FiltersTestData`` summaries (features A, B and the map features C, D with keys "1" / "2")."""
import math

import numpy as np
import pytest

from transmogrifai_amd.filters.raw_feature_filter import FeatureDistribution, RawFeatureFilter


def _fd(name, key, count, nulls, dist, typ="Training"):
    return FeatureDistribution(name, key, count, nulls, np.asarray(dist, float), [], type=typ)


TRAIN = [_fd("A", None, 10, 1, [1, 4, 0, 0, 6]), _fd("B", None, 20, 20, [2, 8, 0, 0, 12]),
         _fd("C", "1", 10, 1, [1, 4, 0, 0, 6]), _fd("C", "2", 20, 19, [2, 8, 0, 0, 12]),
         _fd("D", "1", 10, 9, [1, 4, 0, 0, 6]), _fd("D", "2", 20, 19, [2, 8, 0, 0, 12])]
SCORE = [_fd("A", None, 10, 8, [1, 4, 0, 0, 6], "Scoring"), _fd("B", None, 20, 20, [2, 8, 0, 0, 12], "Scoring"),
         _fd("C", "1", 10, 1, [0, 0, 10, 10, 0], "Scoring"), _fd("C", "2", 20, 19, [2, 8, 0, 0, 12], "Scoring"),
         _fd("D", "1", 0, 0, [0, 0, 0, 0, 0], "Scoring"), _fd("D", "2", 0, 0, [0, 0, 0, 0, 0], "Scoring")]


def _rff(min_fill, max_fill_diff, max_ratio, max_js, max_corr=1.0):
    return RawFeatureFilter(None, None, bins=10, min_fill_rate=min_fill, max_fill_difference=max_fill_diff,
                            max_fill_ratio_diff=max_ratio, max_js_divergence=max_js, max_correlation=max_corr)


def test_metrics_without_correlations_or_scoring():
    m, _, _, _ = _rff(0.2, 1.0, math.inf, 1.0).features_to_exclude(TRAIN, [], {})
    assert [x.trainingFillRate for x in m] == pytest.approx([0.9, 0.0, 0.9, 0.05, 0.1, 0.05])
    assert all(x.trainingNullLabelAbsoluteCorr is None for x in m)
    assert all(x.scoringFillRate is None and x.jsDivergence is None and x.fillRateDiff is None
               and x.fillRatioDiff is None for x in m)


def test_metrics_with_scoring_distributions():
    m, _, _, _ = _rff(0.2, 1.0, math.inf, 1.0).features_to_exclude(TRAIN, SCORE, {})
    assert [x.name for x in m] == ["A", "B", "C", "C", "D", "D"]
    assert [x.key for x in m] == [None, None, "1", "2", "1", "2"]
    assert [x.scoringFillRate for x in m] == pytest.approx([0.2, 0.0, 0.9, 0.05, 0.0, 0.0])
    js = [x.jsDivergence for x in m]
    assert js[:4] == pytest.approx([0.0, 0.0, 1.0, 0.0])
    assert all(math.isnan(v) for v in js[4:])                # empty scoring distributions
    assert [x.fillRateDiff for x in m] == pytest.approx([0.7, 0.0, 0.0, 0.0, 0.1, 0.05])
    assert [x.fillRatioDiff for x in m] == pytest.approx([4.5, math.inf, 1.0, 1.0, math.inf, math.inf])


def test_exclusion_by_training_fill_rate():
    _, reasons, drop, keys = _rff(0.2, 1.0, math.inf, 1.0).features_to_exclude(TRAIN, [], {})
    assert set(drop) == {"B", "D"}
    assert {k: set(v) for k, v in keys.items()} == {"C": {"2"}}
    assert {r.name for r in reasons if r.trainingUnfilledState} == {"B", "C", "D"}
    assert [r.name for r in reasons] == ["A", "B", "C", "C", "D", "D"]
    assert [r.key for r in reasons] == [None, None, "1", "2", "1", "2"]


def test_exclusion_by_training_and_scoring_fill_rate():
    _, reasons, drop, keys = _rff(0.2, 1.0, math.inf, 1.0).features_to_exclude(TRAIN, SCORE, {})
    assert set(drop) == {"B", "D"}
    assert {k: set(v) for k, v in keys.items()} == {"C": {"2"}}
    assert {r.name for r in reasons if r.trainingUnfilledState or r.scoringUnfilledState} == {"B", "C", "D"}


def test_exclusion_by_fill_rate_difference():
    _, reasons, drop, keys = _rff(0.0, 0.5, math.inf, 1.0).features_to_exclude(TRAIN, SCORE, {})
    assert set(drop) == {"A"} and not keys
    assert {r.name for r in reasons if r.fillRateDiffMismatch} == {"A"}


def test_exclusion_by_fill_ratio():
    _, reasons, drop, keys = _rff(0.0, 1.0, 2.0, 1.0).features_to_exclude(TRAIN, SCORE, {})
    assert set(drop) == {"A", "B", "D"} and not keys
    assert {r.name for r in reasons if r.fillRatioDiffMismatch} == {"A", "B", "D"}


def test_exclusion_by_js_divergence():
    _, reasons, drop, keys = _rff(0.0, 1.0, math.inf, 0.5).features_to_exclude(TRAIN, SCORE, {})
    assert not drop
    assert {k: set(v) for k, v in keys.items()} == {"C": {"1"}}
    assert {r.name for r in reasons if r.excluded} == {"C"}


def test_exclusion_by_all_rules():
    _, reasons, drop, keys = _rff(0.1, 0.5, math.inf, 0.5).features_to_exclude(TRAIN, SCORE, {})
    assert set(drop) == {"A", "B", "C", "D"} and not keys
    assert {r.name for r in reasons if r.excluded} == {"A", "B", "C", "D"}

"""``FeatureHistoryTest.scala`` ported: a history to / from its metadata (JSON) form, merging two histories
(distinct, sorted), and the per-feature map form."""
import json

from transmogrifai_amd.data.vector_metadata import FeatureHistory


def test_to_metadata():
    h = FeatureHistory(("feature1", "feature2"), ("stage1", "stage2"))
    meta = json.loads(json.dumps(h.to_json()))
    assert meta["originFeatures"] == ["feature1", "feature2"] and meta["stages"] == ["stage1", "stage2"]
    assert FeatureHistory.from_json(meta) == h


def test_merge():
    h = FeatureHistory(("feature1",), ("stage1",)).merge(FeatureHistory(("feature2",), ("stage2",)))
    assert h.origin_features == ("feature1", "feature2") and h.stages == ("stage1", "stage2")
    h2 = FeatureHistory(("b", "a"), ("s",)).merge(FeatureHistory(("a",), ("s", "r")))
    assert h2.origin_features == ("a", "b") and h2.stages == ("r", "s")


def test_map_metadata():
    m = {"1": FeatureHistory(("feature1",), ("stage1",)), "2": FeatureHistory(("feature2",), ("stage2",))}
    meta = json.loads(json.dumps(FeatureHistory.map_to_json(m)))
    assert set(meta) == {"1", "2"}
    assert meta["1"] == {"originFeatures": ["feature1"], "stages": ["stage1"]}
    assert meta["2"] == {"originFeatures": ["feature2"], "stages": ["stage2"]}
    assert FeatureHistory.map_from_json(meta) == m

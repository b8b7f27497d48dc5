"""``TransientFeatureTest.scala`` ported: built from a raw and a derived feature (history kept), built from fields
without a feature (``get_feature`` raises), equality and the uid hash, casting back, serialization dropping the
live feature, and the JSON form."""
import json
import pickle

import pytest

from transmogrifai_amd import dsl  # noqa: F401
from transmogrifai_amd.features import types as T
from transmogrifai_amd.features.feature import TransientFeature
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder


def _feats():
    _, (height, weight) = TestFeatureBuilder.of(("height", T.Real, [1.0]), ("weight", T.Real, [2.0]))
    return height, weight


def _compare(tf, f):
    h = f.history()
    assert (tf.name, tf.uid, tf.is_response, tf.is_raw, tf.type_name) == \
        (f.name, f.uid, f.is_response, f.is_raw, f.type_name)
    assert list(tf.origin_features) == list(h.origin_features) and list(tf.stages) == list(h.stages)


def test_from_features():
    height, weight = _feats()
    tf = TransientFeature.of(height)
    _compare(tf, height)
    assert tf.get_feature() is height and tf.as_feature_like() is height
    density = weight / height
    _compare(TransientFeature.of(density), density)


def test_without_a_feature():
    height, _ = _feats()
    t = TransientFeature(height.name, height.uid, height.is_response, height.is_raw, height.type_name,
                         [height.name], [])
    _compare(t, height)
    with pytest.raises(RuntimeError):
        t.get_feature()


def test_equality_and_hash():
    height, weight = _feats()
    tf = TransientFeature.of(height)
    assert tf == tf and tf == TransientFeature.of(height)
    assert tf != TransientFeature.of(weight)
    assert hash(tf) == hash(tf.uid)


def test_serialization_drops_the_feature():
    height, _ = _feats()
    tf2 = pickle.loads(pickle.dumps(TransientFeature.of(height)))
    _compare(tf2, height)
    with pytest.raises(RuntimeError):
        tf2.get_feature()
    with pytest.raises(RuntimeError):
        tf2.as_feature_like()


def test_json():
    height, _ = _feats()
    tf = TransientFeature.of(height)
    j = json.loads(json.dumps(tf.to_json()))
    assert (j["name"], j["isResponse"], j["isRaw"], j["uid"], j["typeName"]) == \
        (height.name, height.is_response, height.is_raw, height.uid, height.type_name)
    assert TransientFeature.from_json(j) == tf

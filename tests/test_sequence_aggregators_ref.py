"""SequenceAggregatorsTest.scala (``core/src/test/.../utils/spark/``): the per-key mean of real maps and the
per-key mode of integral maps (ties -> the smallest value), as the map vectorizers compute their fills, and the
mode of nullable integral columns."""
import pytest

from transmogrifai_amd.features import types as T
from transmogrifai_amd.stages.feature import maps as MV
from transmogrifai_amd.stages.feature import vectorizers as V
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder


def _fills(est, rows, ftype):
    ds, (f1, f2) = TestFeatureBuilder.of(("f1", ftype, [r[0] for r in rows]), ("f2", ftype, [r[1] for r in rows]))
    model = est.set_input(f1, f2).fit(ds)
    keys = model.keys if hasattr(model, "keys") else None
    return model, keys


def _key_fills(model):
    """{key: fill} per input of a fitted map vectorizer model."""
    out = []
    for keys, fills in zip(model.keys, model.fills):
        out.append(dict(zip(keys, fills)))
    return out


@pytest.mark.parametrize("rows,expected", [
    ([({"a": 1.0, "b": 5.0}, {"z": 10.0}), ({"c": 11.0}, {"y": 3.0, "x": 0.0}), ({}, {})],
     [{"a": 1.0, "c": 11.0, "b": 5.0}, {"z": 10.0, "y": 3.0, "x": 0.0}]),
    ([({"a": 1.0, "b": 5.0}, {"y": 4.0, "x": 0.0, "z": 10.0}), ({"a": -3.0, "b": 3.0, "c": 11.0}, {"y": 3.0, "x": 0.0}),
      ({"a": 1.0, "b": 5.0}, {"y": 1.0, "x": 0.0, "z": 5.0})],
     [{"a": -1.0 / 3, "c": 11.0, "b": 13.0 / 3}, {"z": 7.5, "y": 8.0 / 3, "x": 0.0}]),
])
def test_mean_by_key(rows, expected):
    model, _ = _fills(MV.RealMapVectorizer(fill_with_mean=True), rows, T.RealMap)
    got = _key_fills(model)
    for g, e in zip(got, expected):
        assert g.keys() == e.keys() and all(g[k] == pytest.approx(v, rel=1e-12) for k, v in e.items())


@pytest.mark.parametrize("rows,expected", [
    ([({"a": 1, "b": 5}, {"z": 10}), ({"c": 11}, {"y": 3, "x": 0}), ({}, {})],
     [{"a": 1, "b": 5, "c": 11}, {"x": 0, "y": 3, "z": 10}]),
    ([({"a": 1, "b": 5}, {"y": 4, "x": 0, "z": 10}), ({"a": -3, "b": 3, "c": 11}, {"y": 3, "x": 0}),
      ({"a": 1, "b": 5}, {"y": 1, "x": 0, "z": 5})],
     [{"a": 1, "b": 5, "c": 11}, {"x": 0, "y": 1, "z": 5}]),
])
def test_mode_by_key(rows, expected):
    model, _ = _fills(MV.IntegralMapVectorizer(fill_with_mode=True), rows, T.IntegralMap)
    assert [{k: int(v) for k, v in g.items()} for g in _key_fills(model)] == expected


def test_mode_of_nullable_columns():
    ds, (f1, f2) = TestFeatureBuilder.of(("f1", T.Integral, [3, 3, 1]), ("f2", T.Integral, [None, 2, 5]))
    model = V.IntegralVectorizer(fill_with_mode=True, fill_with_constant=False, track_nulls=False).set_input(f1, f2)
    m = model.fit(ds)
    out = m.transform(ds)[m.get_output().name].values.tolist()
    assert out[0] == [3.0, 2.0]          # f2's missing value filled with its mode (2 and 5 tie -> 2)

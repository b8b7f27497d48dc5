"""OpSetVectorizer expectations ported from ``OpSetVectorizerTest.scala`` (core/src/test/.../feature): default
settings, clean text off, topK, minSupport, fitting on empty sets then scoring unseen values (with and
without null tracking) and an all-empty input. Values are one-hot counts per kept value plus OTHER
(count of non-kept values) and the null indicator (``OpSetVectorizer.scala:60-180``)."""
import pytest

from transmogrifai_amd.data.vector_metadata import NULL_STRING
from transmogrifai_amd.features import types as T
from transmogrifai_amd.stages.feature import vectorizers as V
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.testkit.spec import check_estimator

TOP = [{"a", "b"}, {"a"}, {"c"}, {"C ", "A."}]
BOT = [{"x"}, {"z", "y"}, {"x", "y"}, {"Z"}]


def _sparse(size, idx):
    v = [0.0] * size
    for i in idx:
        v[i] = 1.0
    return v


def _data():
    return TestFeatureBuilder.of(("top", T.MultiPickList, TOP), ("bot", T.MultiPickList, BOT))


def _names(model):
    return [c.indicator_value for c in model.metadata["vector_metadata"].columns]


def test_default_settings():
    ds, (top, bot) = _data()
    est = V.OpSetVectorizer(min_support=0, top_k=10).set_input(top, bot)
    model, _ = check_estimator(est, ds, expected=[_sparse(10, [0, 2, 5]), _sparse(10, [0, 6, 7]),
                                                  _sparse(10, [1, 5, 6]), _sparse(10, [0, 1, 7])])
    assert _names(model) == ["A", "C", "B", "OTHER", NULL_STRING, "X", "Y", "Z", "OTHER", NULL_STRING]


def test_clean_text_off():
    ds, (top, bot) = _data()
    est = V.OpSetVectorizer(min_support=0, top_k=10, clean_text=False).set_input(top, bot)
    model, _ = check_estimator(est, ds, expected=[_sparse(13, [0, 3, 7]), _sparse(13, [0, 8, 10]),
                                                  _sparse(13, [4, 7, 8]), _sparse(13, [1, 2, 9])])
    assert _names(model) == ["a", "A.", "C ", "b", "c", "OTHER", NULL_STRING,
                             "x", "y", "Z", "z", "OTHER", NULL_STRING]


EXPECTED_TOP1 = [[1, 1, 0, 1, 0, 0], [1, 0, 0, 0, 2, 0], [0, 1, 0, 1, 1, 0], [1, 1, 0, 0, 1, 0]]


def test_top_k():
    ds, (top, bot) = _data()
    est = V.OpSetVectorizer(min_support=0, top_k=1).set_input(top, bot)
    check_estimator(est, ds, expected=EXPECTED_TOP1)
    with pytest.raises((ValueError, AssertionError)):
        V.OpSetVectorizer(top_k=0)


def test_min_support():
    ds, (top, bot) = _data()
    est = V.OpSetVectorizer(min_support=3, top_k=10).set_input(top, bot)
    check_estimator(est, ds, expected=[[1, 1, 0, 1, 0], [1, 0, 0, 2, 0], [0, 1, 0, 2, 0], [1, 1, 0, 1, 0]])


@pytest.mark.parametrize("track", [True, False])
def test_fit_on_empty_then_unseen(track):
    ds_empty, (top, bot) = TestFeatureBuilder.of(("top", T.MultiPickList, [{"a", "b"}, {"a"}, set()]),
                                                 ("bot", T.MultiPickList, [set(), set(), set()]))
    est = V.OpSetVectorizer(min_support=0, top_k=10, track_nulls=track).set_input(top, bot)
    if track:
        exp = [[1, 1, 0, 0, 0, 1], [1, 0, 0, 0, 0, 1], [0, 0, 0, 1, 0, 1]]
        names = ["A", "B", "OTHER", NULL_STRING, "OTHER", NULL_STRING]
        exp2 = [[1, 1, 0, 0, 1, 0], [1, 0, 0, 0, 2, 0], [0, 0, 1, 0, 2, 0], [1, 0, 1, 0, 1, 0]]
    else:
        exp = [[1, 1, 0, 0], [1, 0, 0, 0], [0, 0, 0, 0]]
        names = ["A", "B", "OTHER", "OTHER"]
        exp2 = [[1, 1, 0, 1], [1, 0, 0, 2], [0, 0, 1, 2], [1, 0, 1, 1]]
    model, _ = check_estimator(est, ds_empty, expected=exp)
    assert _names(model) == names
    ds, _ = _data()
    out = model.transform(ds)[model.get_output().name].to_list()
    assert [list(map(float, r)) for r in out] == [list(map(float, r)) for r in exp2]


def test_all_empty():
    ds, (top,) = TestFeatureBuilder.of(("top", T.MultiPickList, [set(), set(), set()]))
    model, _ = check_estimator(V.OpSetVectorizer(top_k=10).set_input(top), ds, expected=[[0, 1]] * 3)
    assert _names(model) == ["OTHER", NULL_STRING]


def test_picklist_like_sets_expand_by_two():
    ds, (f,) = TestFeatureBuilder.of(("f", T.MultiPickList, [{v} for v in "abbaabbca"]))
    model, out = check_estimator(V.OpSetVectorizer(top_k=20, min_support=0, track_nulls=True).set_input(f), ds)
    assert all(len(r) == 5 for r in out)

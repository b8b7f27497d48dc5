"""Generic transformers (``core/src/test/.../stages/impl/feature/*Test.scala`` for Alias, Exists, Filter,
Replace, ToOccur, Substring, JaccardSimilarity, NGramSimilarity, TimePeriod*, MultiLabelJoiner, FilterMap)."""
import numpy as np
import pytest

from transmogrifai_amd.features import types as T
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.testkit.spec import check_transformer
from transmogrifai_amd.stages.feature import misc_stages as M


def is_big(v):
    return v > 2.0


def test_alias_exists_filter_replace_occur():
    ds, (a,) = TestFeatureBuilder.of(("a", T.Real, [1.0, 3.0, None]))
    al = M.AliasTransformer("renamed").set_input(a)
    assert al.get_output().name == "renamed"
    check_transformer(al, ds, expected=[1.0, 3.0, None])
    check_transformer(M.ExistsTransformer(is_big).set_input(a), ds.take([0, 1]), expected=[False, True])
    check_transformer(M.FilterTransformer(is_big, -1.0).set_input(a), ds, expected=[-1.0, 3.0, -1.0])
    check_transformer(M.ReplaceTransformer(old_value=1.0, new_value=7.0).set_input(a), ds, expected=[7.0, 3.0, None])
    check_transformer(M.ToOccurTransformer().set_input(a), ds, expected=[1.0, 1.0, 0.0])


def test_dsl_uses_serializable_stages():
    ds, (a,) = TestFeatureBuilder.of(("a", T.Real, [1.0, 3.0]))
    f = a.exists(is_big)
    assert type(f.origin_stage).__name__ == "ExistsTransformer"
    from transmogrifai_amd.testkit.spec import roundtrip
    st2 = roundtrip(f.origin_stage)
    assert st2.fn is is_big


def test_substring_and_similarities():
    ds, (s, t) = TestFeatureBuilder.of(("s", T.Text, ["Cat", "dog", None]), ("t", T.Text, ["the cat sat", "cow", "x"]))
    check_transformer(M.SubstringTransformer().set_input(s, t), ds, expected=[True, False, None])
    sim = check_transformer(M.TextNGramSimilarity().set_input(s, t), ds)
    assert 0.0 < sim[0] < 1.0 and sim[2] == 0.0
    assert M.ngram_distance("abcdef", "abcdef") == pytest.approx(1.0)
    assert M.ngram_distance("abc", "xyz") == pytest.approx(0.0)
    assert M.ngram_distance("ab", "ac") == pytest.approx(0.5)
    ds2, (x, y) = TestFeatureBuilder.of(("x", T.MultiPickList, [{"a", "b"}, set(), {"a"}]),
                                        ("y", T.MultiPickList, [{"b", "c"}, set(), {"z"}]))
    check_transformer(M.JaccardSimilarity().set_input(x, y), ds2, expected=[1 / 3, 1.0, 0.0])
    check_transformer(M.SetNGramSimilarity().set_input(x, y), ds2)


def test_time_period_transformers():
    day = 86_400_000
    # 1970-01-01 was a Thursday (ISO day 4); 1970-01-05 a Monday
    ds, (d, l, m) = TestFeatureBuilder.of(("d", T.Date, [0, 4 * day, None]),
                                          ("l", T.DateList, [[0, 4 * day], [], [day]]),
                                          ("m", T.DateMap, [{"k": 0}, {}, {"k": 4 * day}]))
    check_transformer(M.TimePeriodTransformer(period="DayOfWeek").set_input(d), ds, expected=[4, 1, None])
    out = check_transformer(M.TimePeriodListTransformer(period="DayOfWeek").set_input(l), ds, check_rows=False)
    assert out[0] == [4.0, 1.0]
    check_transformer(M.TimePeriodMapTransformer(period="DayOfWeek").set_input(m), ds,
                      expected=[{"k": 4}, {}, {"k": 1}])


def test_label_joiners_and_filter_map():
    ds, (lab, p) = TestFeatureBuilder.of(("lab", T.RealNN, [0.0, 1.0]), ("p", T.OPVector, [[0.2, 0.7, 0.1], [0.5, 0.1, 0.4]]),
                                         response="lab")
    mj = M.MultiLabelJoiner(labels=["a", "b", "c"]).set_input(lab, p)
    out = check_transformer(mj, ds)
    assert out[0] == {"a": 0.2, "b": 0.7, "c": 0.1}
    tj = M.TopNLabelJoiner(labels=["a", "b", "c"], top_n=2).set_input(lab, p)
    assert check_transformer(tj, ds)[1] == {"a": 0.5, "c": 0.4}
    ds3, (mp,) = TestFeatureBuilder.of(("mp", T.TextMap, [{"k1": "v", "k2": "w"}, {}]))
    check_transformer(M.FilterMap(block_list_keys=["k2"]).set_input(mp), ds3, expected=[{"k1": "v"}, {}])


def test_prediction_descaler_inverts_scaler():
    """``DescalerTransformerTest`` / ``PredictionDescalerTransformerTest``: descaling a scaled label (and a
    prediction made on the scaled label) recovers the original scale."""
    import torch
    from transmogrifai_amd.data.columns import NumericColumn, PredictionColumn
    from transmogrifai_amd.data.dataset import Dataset
    from transmogrifai_amd.dsl.core import descale_prediction
    from transmogrifai_amd.features import types as T
    from transmogrifai_amd.features.builder import FeatureBuilder
    from transmogrifai_amd.stages.feature.math_stages import PredictionDescaler
    y = FeatureBuilder.Real("y").as_predictor()
    scaled = y.scale("Linear", slope=2.0, intercept=1.0)
    back = y.descale(scaled)
    vals = torch.tensor([1.0, 2.5, -3.0], dtype=torch.float64)
    ds = Dataset({"y": NumericColumn(T.Real, vals)})
    ds = scaled.origin_stage.transform(ds)
    assert torch.allclose(ds[scaled.name].values, 2 * vals + 1)
    ds2 = back.origin_stage.transform(ds.with_column("y", NumericColumn(T.Real, ds[scaled.name].values)))
    assert torch.allclose(ds2[back.name].values, vals)
    # prediction descaler
    pcol = PredictionColumn(2 * vals + 1, None, None)
    pd = PredictionDescaler(scaling_type="Linear", slope=2.0, intercept=1.0)
    out = pd.transform_columns(pcol, ds[scaled.name])
    assert torch.allclose(out.values, vals)
    assert pd.transform_row({"prediction": 7.0}, None) == 3.0
    pred_feat = FeatureBuilder.Real("p").as_predictor()
    d = descale_prediction(pred_feat, scaled)
    assert isinstance(d.origin_stage, PredictionDescaler)

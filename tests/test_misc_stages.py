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
    # cleanText defaults to true (TransmogrifierDefaults.CleanText): "v" -> "V"
    check_transformer(M.FilterMap(block_list_keys=["k2"]).set_input(mp), ds3, expected=[{"k1": "V"}, {}])
    check_transformer(M.FilterMap(block_list_keys=["k2"], clean_text=False).set_input(mp), ds3,
                      expected=[{"k1": "v"}, {}])


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


def _ms(y, mo, d, h=0, mi=0):
    import datetime as _dt
    return int(_dt.datetime(y, mo, d, h, mi, tzinfo=_dt.timezone.utc).timestamp() * 1000)


_TP_DATES = [_ms(1879, 3, 14), _ms(1955, 11, 12, 10, 4), _ms(1999, 3, 8, 12), None, _ms(2019, 4, 30, 13)]
_TP_EXPECTED = {   # TimePeriodTransformerTest.scala "correctly transform for all TimePeriod types" (UTC)
    "DayOfMonth": [14, 12, 8, None, 30], "DayOfWeek": [5, 6, 1, None, 2], "DayOfYear": [73, 316, 67, None, 120],
    "HourOfDay": [0, 10, 12, None, 13], "MonthOfYear": [3, 11, 3, None, 4], "WeekOfMonth": [3, 2, 2, None, 5],
    "WeekOfYear": [11, 46, 11, None, 18],
}


@pytest.mark.parametrize("period", sorted(_TP_EXPECTED))
def test_time_period_reference_table(period):
    from transmogrifai_amd import dsl  # noqa: F401
    ds, (d,) = TestFeatureBuilder.of(("d", T.Date, _TP_DATES))
    check_transformer(M.TimePeriodTransformer(period=period).set_input(d), ds, expected=_TP_EXPECTED[period])
    f = d.to_time_period(period)
    col = f.origin_stage.transform(ds)[f.name]
    assert [None if not ok else int(v) for v, ok in zip(col.values.tolist(), col.valid.tolist())] == \
        _TP_EXPECTED[period]


def test_time_period_list_and_map_reference():
    """TimePeriodListTransformerTest / TimePeriodMapTransformerTest: day of month of the four dates; the
    shortcuts on DateList / DateTimeList and DateMap / DateTimeMap."""
    from transmogrifai_amd import dsl  # noqa: F401
    dates = [v for v in _TP_DATES if v is not None]
    ds, (l, m) = TestFeatureBuilder.of(("l", T.DateList, [dates]),
                                       ("m", T.DateMap, [dict(zip(["n1", "n2", "n3", "n4"], dates))]))
    out = check_transformer(M.TimePeriodListTransformer(period="DayOfMonth").set_input(l), ds, check_rows=False)
    assert out[0] == [14.0, 12.0, 8.0, 30.0]
    check_transformer(M.TimePeriodMapTransformer(period="DayOfMonth").set_input(m), ds,
                      expected=[{"n1": 14, "n2": 12, "n3": 8, "n4": 30}])
    ds2, (d1, d2, m1, m2) = TestFeatureBuilder.of(("d1", T.DateList, [[dates[0]]]), ("d2", T.DateTimeList, [[dates[0]]]),
                                                  ("m1", T.DateMap, [{"n1": dates[0]}]),
                                                  ("m2", T.DateTimeMap, [{"n1": dates[0]}]))
    for f in (d1, d2):
        g = f.to_time_period("DayOfMonth")
        assert g.origin_stage.transform(ds2)[g.name].values.double().tolist() == [[14.0]]
    for f in (m1, m2):
        g = f.to_time_period("DayOfMonth")
        assert g.origin_stage.transform(ds2)[g.name].values.tolist() == [{"n1": 14}]

"""MonoidAggregatorDefaultsTest.scala (features/src/test/.../aggregators/): every default aggregator and the named
alternatives on the reference's base data, and the monoid laws of the logical ops."""
import itertools
import math

import numpy as np
import pytest

from transmogrifai_amd.features import aggregators as A
from transmogrifai_amd.features import types as T
from transmogrifai_amd.features.aggregators import Event, default_aggregator

DOUBLE = [-1.0, None, 0.25, 0.1, 0.7, 2.5]
LONG = [1, None, 11110, 250, 10, 1234324234]
BOOL = [True, None, False, True, None]
SETS = [{"a", "b", "c"}, {"d", "e"}, {"d", "a"}, set()]
PICK = ["A", "B", "B", "A", None, "A", None, "C"]
PICK_BAL = ["C", "B", None, "D"]
TEXT = ["My name is Joe", "And I work in a button factory", "One day my boss said to me", "Are you busy, I said no",
        "Then push the button with your right hand", None, None]
DOUBLE_MAP = [{"a": 1.0, "b": 1.0}, {"b": 1.0, "c": 1.0, "e": 0.0}, {"a": 0.5, "d": 0.3, "e": 0.0}, {}]
LONG_MAP = [{"a": 1, "b": 1}, {"b": 1, "c": 1, "e": 0}, {"a": 2, "d": 2, "e": 0}, {}]
BOOL_MAP = [{"a": True, "b": False, "c": True}, {"a": True, "b": False, "c": False}, {}]
TEXT_MAP = [{"a": "Mo' money", "b": "Been spending all their lives", "d": ""},
            {"a": "mo' problems", "b": "livin' in the gangsta's paradise", "c": "Does this take you back?"},
            {"d": ""}, {}]
SET_MAP = [{"a": {"a", "b"}, "b": {"a", "b"}}, {"a": {"c"}, "d": set()}, {"b": {"a", "c"}, "c": {"a"}}, {}]


def agg(a, values):
    return a.aggregate([Event(0, v) for v in values])


def dflt(t, values):
    return agg(default_aggregator(t), values)


def _flat(xs):
    return [x for x in xs if x is not None]


def test_unknown_type_is_an_error():
    with pytest.raises(ValueError):
        default_aggregator(T.FeatureType)


def test_sum_numeric_defaults():
    for t in (T.Real, T.RealNN, T.Currency):
        assert dflt(t, DOUBLE if t is not T.RealNN else [v or 0.0 for v in DOUBLE]) == pytest.approx(sum(_flat(DOUBLE)))
    assert dflt(T.Integral, LONG) == sum(_flat(LONG))


def test_min_max_numeric():
    assert agg(A.MaxNumeric(), DOUBLE) == max(_flat(DOUBLE))
    assert agg(A.MinNumeric(), DOUBLE) == min(_flat(DOUBLE))
    assert agg(A.MaxNumeric(), LONG) == max(_flat(LONG))
    assert agg(A.MinNumeric(), LONG) == min(_flat(LONG))
    assert dflt(T.Date, LONG) == max(_flat(LONG)) and dflt(T.DateTime, LONG) == max(_flat(LONG))
    nn = [v or 0.0 for v in DOUBLE]
    assert agg(A.MaxRealNN(), nn) == 2.5 and agg(A.MinRealNN(), nn) == -1.0


def test_mean_numeric_and_percent():
    vals = _flat(DOUBLE)
    assert agg(A.MeanNumeric(), DOUBLE) == pytest.approx(sum(v / len(vals) for v in vals))
    nn = [v if v is not None else 0.0 for v in DOUBLE]
    assert agg(A.MeanRealNN(), nn) == pytest.approx(sum(nn) / len(nn))
    # MeanPercent clips to [0, 1] before averaging: (0 + .25 + .1 + .7 + 1) / 5
    assert dflt(T.Percent, DOUBLE) == pytest.approx(0.41, abs=5e-3)
    assert dflt(T.Percent, DOUBLE) == pytest.approx((0 + .25 + .1 + .7 + 1) / 5)


def test_union_multi_pick_list():
    assert set(dflt(T.MultiPickList, SETS)) == {"a", "b", "c", "d", "e"}


@pytest.mark.parametrize("t,sep", [(T.Base64, ","), (T.ComboBox, ","), (T.Email, ","), (T.ID, ","), (T.Phone, ","),
                                   (T.Text, " "), (T.TextArea, " "), (T.URL, ","), (T.Country, ","), (T.State, ","),
                                   (T.City, ","), (T.PostalCode, ","), (T.Street, ",")])
def test_concat_text_with_separator(t, sep):
    assert dflt(t, TEXT) == sep.join(_flat(TEXT))


def test_concat_text_empty_strings():
    """TextUtils.concat: an empty side adds no separator; all-empty stays a present ""."""
    a = A.ConcatText(",")
    assert agg(a, ["x", "", "y"]) == "x,y" and agg(a, ["", ""]) == "" and agg(a, [None, None]) is None


def test_mode_pick_list():
    assert dflt(T.PickList, PICK) == "A"
    assert dflt(T.PickList, PICK_BAL) == "B"      # ties -> the smallest value


def test_concat_and_min_max_lists():
    assert dflt(T.TextList, [["a"], ["b"], ["c"]]) == ["a", "b", "c"]
    longs = [[v] for v in _flat(LONG)]
    assert dflt(T.DateList, longs) == _flat(LONG) and dflt(T.DateTimeList, longs) == _flat(LONG)
    assert agg(A.MinMaxList(False, "MaxDateList"), longs) == [max(_flat(LONG))]
    assert agg(A.MinMaxList(True, "MinDateTimeList"), longs) == [min(_flat(LONG))]


def test_logical_ops():
    assert dflt(T.Binary, BOOL) is True and agg(A.LogicalOr(), BOOL) is True
    assert agg(A.LogicalXor(), BOOL) is False
    assert agg(A.LogicalAnd(), BOOL) is False


@pytest.mark.parametrize("m", [A.LogicalOr(), A.LogicalXor(), A.LogicalAnd()])
def test_logical_ops_are_monoids(m):
    vals = [True, False, None]
    for a, b, c in itertools.product(vals, repeat=3):
        assert m.plus(m.zero_value(), a) == a and m.plus(a, m.zero_value()) == a
        assert m.plus(m.plus(a, b), c) == m.plus(a, m.plus(b, c))


def test_union_sum_numeric_map():
    exp_d = {"a": 1.5, "b": 2.0, "c": 1.0, "d": 0.3, "e": 0.0}
    for t in (T.RealMap, T.CurrencyMap):
        got = dflt(t, DOUBLE_MAP)
        assert got.keys() == exp_d.keys() and all(got[k] == pytest.approx(v) for k, v in exp_d.items())
    assert dflt(T.IntegralMap, LONG_MAP) == {"a": 3, "b": 2, "c": 1, "d": 2, "e": 0}


def test_union_mean_map():
    exp = {"a": 0.75, "b": 1.0, "c": 1.0, "d": 0.3, "e": 0.0}
    assert agg(A.UnionMeanMap("UnionMeanRealMap"), DOUBLE_MAP) == pytest.approx(exp)
    assert dflt(T.PercentMap, DOUBLE_MAP) == pytest.approx(exp)
    # a true mean, not a running pairwise average
    assert agg(A.UnionMeanMap(), [{"a": 1.0}, {"a": 2.0}, {"a": 6.0}]) == {"a": 3.0}


def test_union_min_max_numeric_map():
    assert agg(A.UnionMinMaxMap(False, "UnionMaxRealMap"), DOUBLE_MAP) == {"a": 1.0, "b": 1.0, "c": 1.0, "d": 0.3,
                                                                              "e": 0.0}
    assert agg(A.UnionMinMaxMap(True, "UnionMinRealMap"), DOUBLE_MAP) == {"a": 0.5, "b": 1.0, "c": 1.0, "d": 0.3,
                                                                             "e": 0.0}
    lmax = {"a": 2, "b": 1, "c": 1, "d": 2, "e": 0}
    assert dflt(T.DateMap, LONG_MAP) == lmax and dflt(T.DateTimeMap, LONG_MAP) == lmax
    assert agg(A.UnionMinMaxMap(True, "UnionMinDateMap"), LONG_MAP) == {"a": 1, "b": 1, "c": 1, "d": 2, "e": 0}


@pytest.mark.parametrize("t,sep", [(T.Base64Map, ","), (T.ComboBoxMap, ","), (T.EmailMap, ","), (T.IDMap, ","),
                                   (T.PhoneMap, ","), (T.PickListMap, ","), (T.TextMap, " "), (T.TextAreaMap, " "),
                                   (T.URLMap, ","), (T.CountryMap, ","), (T.StateMap, ","), (T.CityMap, ","),
                                   (T.PostalCodeMap, ","), (T.StreetMap, ",")])
def test_union_concat_text_map(t, sep):
    exp = {"a": f"Mo' money{sep}mo' problems",
           "b": f"Been spending all their lives{sep}livin' in the gangsta's paradise",
           "c": "Does this take you back?", "d": ""}
    assert dflt(t, TEXT_MAP) == exp


def test_union_binary_and_set_maps():
    assert dflt(T.BinaryMap, BOOL_MAP) == {"a": True, "b": False, "c": True}
    got = dflt(T.MultiPickListMap, SET_MAP)
    assert {k: set(v) for k, v in got.items()} == {"a": {"a", "b", "c"}, "b": {"a", "b", "c"}, "c": {"a"}, "d": set()}


def test_vectors():
    assert list(dflt(T.OPVector, [[0.1, 0.2], [1.0], [0.2]])) == [0.1, 0.2, 1.0, 0.2]
    assert np.allclose(agg(A.SumVector(), [[0.1, 0.2], [1.0, -1.5], [0.2, 0.0]]), [1.3, -1.3])
    with pytest.raises(ValueError, match=r"Vectors must have same length: x.length == y.length \(1 != 2\)"):
        agg(A.SumVector(), [[0.1, 0.2], [1.0]])


def test_custom_monoid_aggregator():
    custom = A.CustomMonoidAggregator(None, lambda a, b: b if a is None else a if b is None else a + b)
    assert agg(custom, DOUBLE) == pytest.approx(sum(_flat(DOUBLE)))


def test_aggregators_round_trip_json():
    for a in (A.LogicalXor(), A.MeanPercent(), A.UnionMeanMap("UnionMeanPercentMap", clip=True),
              A.UnionMinMaxMap(True, "UnionMinDateMap"), A.UnionConcatTextMap(" "), A.MinMaxList(False, "MaxDateList"),
              A.UnionGeolocationMidpointMap(), A.SumVector()):
        b = A.aggregator_from_json({"value": a.to_json()})
        assert type(b) is type(a) and b.to_json() == a.to_json()

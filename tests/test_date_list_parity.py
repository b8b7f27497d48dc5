"""DateListVectorizer expectations ported from ``DateListVectorizerTest.scala`` (core/src/test/.../feature):
SinceFirst with/without null tracking, a reference date in the past, the stage's default pivot (``first``
defaults to true, ``DateListVectorizer.scala:110-115``) and the ModeDay / ModeMonth / ModeHour one-hot pivots,
on the same two data sets (dates around 1998-07-12 22:45 UTC and around the reference date)."""
from datetime import datetime, timezone

import numpy as np
import pytest

from transmogrifai_amd.data.vector_metadata import NULL_STRING
from transmogrifai_amd.features import types as T
from transmogrifai_amd.stages.feature import vectorizers as V
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.testkit.spec import check_transformer

DAY = 86_400_000
HOUR = 3_600_000
MONTH = 2_628_000_000            # the test's monthsToMilliseconds
DEFAULT_DATE = int(datetime(1998, 7, 12, 22, 45, tzinfo=timezone.utc).timestamp() * 1000)
REF = int(datetime(2026, 1, 5, 13, 7, 11, 123000, tzinfo=timezone.utc).timestamp() * 1000)
NOW = REF - 1                    # "make date time be in the past"


def _data():
    d = DEFAULT_DATE
    return TestFeatureBuilder.of(
        ("clicks", T.DateList, [[d, d + 7 * DAY, d + 12 * MONTH], [d, d - 3 * DAY, d + 4 * DAY],
                                [d, d + 7 * DAY, d + DAY, d + 8 * DAY], []]),
        ("opens", T.DateList, [[d + DAY, d, d + 8 * DAY], [d - MONTH, d + 11 * MONTH],
                               [d, d + 24 * MONTH, d - 2 * MONTH, d + 10 * MONTH], []]),
        ("purchases", T.DateList, [[d], [d - 3 * HOUR, d + 21 * HOUR],
                                   [d, d + 24 * HOUR, d - 6 * HOUR, d + 18 * HOUR], []]))


def _data_current():
    n = NOW
    return TestFeatureBuilder.of(
        ("clicks", T.DateList, [[], [n - 2 * DAY, n - 3 * DAY, n], [n - 1],
                                [n, n - 34, n - 2 * DAY, n + 2 * DAY + 600_000]]),
        ("opens", T.DateList, [[], [n, n + 2 * DAY + 600_000, n + DAY], [n],
                               [n + 2 * DAY + HOUR, n - DAY + 1]]),
        ("purchases", T.DateList, [[], [n], [n, n + 4 * DAY + 600_000], [n + DAY + 600_000]]))


def _one_row(*lists):
    return TestFeatureBuilder.of(*[(f"c{i}", T.DateList, [l]) for i, l in enumerate(lists)])


def _sparse(size, idx):
    v = [0.0] * size
    for i in idx:
        v[i] = 1.0
    return v


def test_default_pivot_is_since_first_with_nulls():
    ds, feats = _data_current()
    st = V.DateListVectorizer(reference_date=REF).set_input(*feats)
    assert st.params["pivot"] == "SinceFirst" and st.params["track_nulls"] is True
    check_transformer(st, ds, expected=[[0, 1, 0, 1, 0, 1], [3, 0, 0, 0, 0, 0], [0, 0, 0, 0, 0, 0],
                                        [2, 0, 1, 0, -1, 0]])


def test_since_first_no_nulls():
    ds, feats = _data_current()
    st = V.DateListVectorizer(pivot="SinceFirst", track_nulls=False, reference_date=REF).set_input(*feats)
    check_transformer(st, ds, expected=[[0, 0, 0], [3, 0, 0], [0, 0, 0], [2, 1, -1]])
    meta = st.metadata["vector_metadata"]
    assert [c.indicator_value for c in meta.columns] == [None, None, None]
    ds1, f1 = _one_row([NOW - DAY, NOW], [NOW - 20 * DAY, NOW - DAY], [NOW])
    st1 = V.DateListVectorizer(pivot="SinceFirst", track_nulls=False, reference_date=REF).set_input(*f1)
    check_transformer(st1, ds1, expected=[[1, 20, 0]])


def test_since_first_track_nulls_single_row():
    ds1, f1 = _one_row([NOW - DAY, NOW], [NOW - 20 * DAY, NOW - DAY], [NOW], [])
    st = V.DateListVectorizer(pivot="SinceFirst", track_nulls=True, reference_date=REF).set_input(*f1)
    check_transformer(st, ds1, expected=[[1, 0, 20, 0, 0, 0, 0, 1]])
    meta = st.metadata["vector_metadata"]
    assert [c.indicator_value for c in meta.columns] == [None, NULL_STRING] * 4


def test_since_first_reference_date_in_past():
    ref = REF - 30 * DAY - 2
    ds, feats = _data_current()
    st = V.DateListVectorizer(pivot="SinceFirst", track_nulls=False, reference_date=ref).set_input(*feats)
    check_transformer(st, ds, expected=[[0, 0, 0], [-27, -30, -30], [-30, -30, -30], [-28, -29, -31]])
    ds1, f1 = _one_row([NOW - DAY, NOW], [NOW - 20 * DAY, NOW - DAY], [NOW])
    st1 = V.DateListVectorizer(pivot="SinceFirst", track_nulls=False, reference_date=ref).set_input(*f1)
    check_transformer(st1, ds1, expected=[[-29, -10, -30]])


@pytest.mark.parametrize("pivot,track,width,single,rows", [
    ("ModeDay", False, 21, [6, 7, 15], [[6, 7, 20], [3, 11, 14], [0, 8, 14], []]),
    ("ModeDay", True, 24, [6, 8, 17], [[6, 8, 22], [3, 12, 16], [0, 9, 16], [7, 15, 23]]),
    ("ModeMonth", False, 36, [6, 18, 27], [[6, 18, 30], [6, 17, 30], [6, 16, 30], []]),
    ("ModeHour", False, 72, [22, 46, 48], [[22, 46, 70], [22, 36, 67], [22, 26, 64], []]),
])
def test_mode_pivots(pivot, track, width, single, rows):
    ds, feats = _data()
    st = V.DateListVectorizer(pivot=pivot, track_nulls=track).set_input(*feats)
    check_transformer(st, ds, expected=[_sparse(width, r) for r in rows])
    names = [c.indicator_value for c in st.metadata["vector_metadata"].columns]
    per = {"ModeDay": ["Monday", "Tuesday", "Wednesday", "Thursday", "Friday", "Saturday", "Sunday"],
           "ModeMonth": ["January", "February", "March", "April", "May", "June", "July", "August",
                         "September", "October", "November", "December"],
           "ModeHour": [f"{h}:00" for h in range(24)]}[pivot] + ([NULL_STRING] if track else [])
    assert names == per * 3
    d = DEFAULT_DATE
    step = {"ModeDay": DAY, "ModeMonth": MONTH, "ModeHour": HOUR}[pivot]
    ds1, f1 = _one_row([d], [d + step, d], [d, d + 2 * step, d + 9 * step])
    st1 = V.DateListVectorizer(pivot=pivot, track_nulls=track).set_input(*f1)
    check_transformer(st1, ds1, expected=[_sparse(width, single)])

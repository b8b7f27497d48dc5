"""``DateTimeVectorizerTest.scala`` ported: three DateTime features vectorized together against a reference date
(days since, truncated toward zero like the reference's ``Long`` division and ``getStandardDays``), with and
without null tracking and with the default circular representations (3 x 8 circular + 3 x 2 = 30 columns), at a
fixed test date and at "now minus an hour"."""
import datetime as dt

import pytest

from transmogrifai_amd import dsl  # noqa: F401
from transmogrifai_amd.features import types as T
from transmogrifai_amd.stages.feature.transmogrifier import TransmogrifierDefaults as D
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.workflow.workflow import OpWorkflow

DAY = 86_400_000
UTC = dt.timezone.utc


def _ms(*a):
    return int(dt.datetime(*a, tzinfo=UTC).timestamp() * 1000)


DEFAULT_DATE = _ms(1998, 7, 12, 22, 45)     # Sunday July 12th 1998 at 22:45


def _tdiv(a, b):
    q = abs(a) // b
    return q if a >= 0 else -q


def _expected(m):
    return [[_tdiv(m - 1, DAY), 0, _tdiv(m, DAY)],
            [_tdiv(m - 1, DAY), _tdiv(m - DEFAULT_DATE, DAY), _tdiv(m - 3 * DAY, DAY)],
            [0, _tdiv(m, DAY), -100]]


def _score(vec, ds):
    out = OpWorkflow().set_result_features(vec).set_input_dataset(ds).train().score()
    return out[vec.name].values.double().tolist(), None


@pytest.mark.parametrize("moment", [_ms(2017, 9, 28, 15, 45, 39),
                                    int((dt.datetime.now(UTC) - dt.timedelta(hours=1)).timestamp() * 1000)])
def test_vectorize_dates_at(moment):
    ds, (f1, f2, f3) = TestFeatureBuilder.of(
        ("f1", T.DateTime, [1, 1, None]),
        ("f2", T.DateTime, [None, DEFAULT_DATE, 0]),
        ("f3", T.DateTime, [0, 3 * DAY, moment + 100 * DAY + 60_000]))
    v1 = f1.vectorize(date_list_pivot=D.DateListDefault, reference_date=moment, track_nulls=False,
                      circular_date_reps=(), others=[f2, f3])
    out, _ = _score(v1, ds)
    assert out == [[float(x) for x in r] for r in _expected(moment)]
    assert len(v1.origin_stage.metadata["vector_metadata"].columns) == 3

    v2 = f1.vectorize(date_list_pivot=D.DateListDefault, reference_date=moment, track_nulls=True,
                      circular_date_reps=(), others=[f2, f3])
    out2, _ = _score(v2, ds)
    assert len(out2[0]) == 6
    assert [r[0::2] for r in out2] == [[float(x) for x in r] for r in _expected(moment)]
    assert [r[1::2] for r in out2] == [[0, 1, 0], [0, 0, 0], [1, 0, 0]]      # the nominal null columns

    v3 = f1.vectorize(date_list_pivot=D.DateListDefault, reference_date=moment, others=[f2, f3])
    out3, _ = _score(v3, ds)
    assert len(out3[0]) == 30
    # the last 6 columns are (days since, null) per feature; the null indicators are nominal
    assert [r[-5::2] for r in out3] == [[0, 1, 0], [0, 0, 0], [1, 0, 0]]


# ---- DateMapVectorizerTest.scala: the same days-since values keyed a / b / c in one DateTimeMap ----
def _map_ds(moment):
    return TestFeatureBuilder.of(("f1", T.DateTimeMap, [
        {"a": 1, "b": DEFAULT_DATE, "c": 3 * DAY},
        {"a": 1, "c": 0},
        {"b": 0, "c": moment + 100 * DAY + 60_000}]))


def _map_expected(m):
    return [[_tdiv(m - 1, DAY), _tdiv(m - DEFAULT_DATE, DAY), _tdiv(m - 3 * DAY, DAY)],
            [_tdiv(m - 1, DAY), 0, _tdiv(m, DAY)],
            [0, _tdiv(m, DAY), -100]]


@pytest.mark.parametrize("moment", [_ms(2017, 9, 28, 15, 45, 39), _ms(1901, 1, 1, 0, 0, 0),
                                    int((dt.datetime.now(UTC) - dt.timedelta(hours=1)).timestamp() * 1000)])
def test_date_map_vectorize_at(moment):
    ds, (f1,) = _map_ds(moment)
    v1 = f1.vectorize(default_value=0, reference_date=moment, track_nulls=False, circular_date_reps=())
    out, _ = _score(v1, ds)
    assert out == [[float(x) for x in r] for r in _map_expected(moment)]
    cols = v1.origin_stage.metadata["vector_metadata"].columns
    assert sorted(c.grouping for c in cols) == ["a", "b", "c"]

    v2 = f1.vectorize(default_value=0, reference_date=moment, track_nulls=True, circular_date_reps=())
    out2, _ = _score(v2, ds)
    assert len(out2[0]) == 6
    assert [r[1::2] for r in out2] == [[0, 0, 0], [0, 1, 0], [1, 0, 0]]

    v3 = f1.vectorize(default_value=0)
    out3, _ = _score(v3, ds)
    assert len(out3[0]) == 30


def test_date_map_vectorizer_serializes(tmp_path):
    from transmogrifai_amd.stages.feature.maps import DateMapVectorizer
    from transmogrifai_amd.workflow.workflow import OpWorkflowModel
    moment = int((dt.datetime.now(UTC) - dt.timedelta(hours=1)).timestamp() * 1000)
    ds, (f1,) = _map_ds(moment)
    st = DateMapVectorizer(fill_value=0.0, reference_date=moment, track_nulls=False).set_input(f1)
    wf = OpWorkflow().set_input_dataset(ds).set_result_features(st.get_output())
    model = wf.train()
    model.save(str(tmp_path / "m"))
    loaded = wf.load_model(str(tmp_path / "m"))
    assert st.uid in [s.uid for s in loaded.get_stages()]

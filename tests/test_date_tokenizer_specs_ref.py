"""DateVectorizerTest.scala and TextTokenizerRegexTest.scala (``core/src/test/.../stages/impl/feature/``)."""
import datetime as dt

import pytest

from transmogrifai_amd import dsl  # noqa: F401
from transmogrifai_amd.features import types as T
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.testkit.spec import check_transformer
from transmogrifai_amd.workflow.workflow import OpWorkflow

DAY = 86_400_000


def _ms(*a):
    return int(dt.datetime(*a, tzinfo=dt.timezone.utc).timestamp() * 1000)


DEFAULT_DATE = _ms(1998, 7, 12, 22, 45)


def _data(moment):
    rows = [(1, None, 0), (1, DEFAULT_DATE, 3 * DAY), (None, 0, moment + 100 * DAY + 60_000)]
    return TestFeatureBuilder.of(*[(n, T.Date, [r[k] for r in rows]) for k, n in enumerate(("f1", "f2", "f3"))])


def _expected(moment):
    """Whole days since each date at the reference moment (a date in the future counts negative days)."""
    def days(d):
        return float(int((moment - d) / DAY)) if moment >= d else -float(int((d - moment) / DAY))
    return [[days(1), 0.0, days(0)], [days(1), days(DEFAULT_DATE), days(3 * DAY)],
            [0.0, days(0), days(moment + 100 * DAY)]]


def _check_at(moment):
    ds, (f1, f2, f3) = _data(moment)
    vec = f1.vectorize(date_list_pivot="SinceLast", reference_date=moment, track_nulls=False, circular_date_reps=(),
                       others=[f2, f3])
    out = OpWorkflow().set_result_features(vec).set_input_dataset(ds).train().score()[vec.name]
    assert out.values.tolist() == _expected(moment)
    assert out.metadata.size == 3 and len(out.metadata.history) == 3
    vec2 = f1.vectorize(date_list_pivot="SinceLast", reference_date=moment, track_nulls=True, circular_date_reps=(),
                        others=[f2, f3])
    out2 = OpWorkflow().set_result_features(vec2).set_input_dataset(ds).train().score()[vec2.name]
    assert out2.values.shape[1] == 6 and out2.metadata.size == 6 and len(out2.metadata.history) == 3
    vec3 = f1.vectorize(date_list_pivot="SinceLast", others=[f2, f3])       # default circular reps + since-last
    out3 = OpWorkflow().set_result_features(vec3).set_input_dataset(ds).train().score()[vec3.name]
    assert out3.values.shape[1] == 30 and out3.metadata.size == 30


@pytest.mark.parametrize("hour", [0, 5, 11, 17, 23])
def test_vectorize_dates_at_moments(hour):
    _check_at(_ms(2017, 9, 27, hour, 45, 39))


def test_vectorize_dates_now():
    import time
    _check_at(int(time.time() * 1000))


def test_tokenize_regex():
    texts = ["I've got a lovely bunch of coconuts", "There they are, all standing in a row",
             "Big ones, small ones, some as big as your head",
             "<body>Big ones, small <h1>ones</h1>, some as big as your head</body>", "two  words", "   ehh,   Fluff     ",
             ""]
    ds, (english,) = TestFeatureBuilder.of(("english", T.Text, texts))
    st = english.tokenize_regex(pattern=r"\s+", min_token_length=5, to_lowercase=False).origin_stage
    check_transformer(st, ds, expected=[["lovely", "bunch", "coconuts"], ["There", "standing"],
                                        ["ones,", "small", "ones,"],
                                        ["<body>Big", "ones,", "small", "<h1>ones</h1>,", "head</body>"], ["words"],
                                        ["Fluff"], []])

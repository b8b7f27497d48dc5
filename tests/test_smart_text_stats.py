"""SmartTextVectorizer TextStats: capped monoid, token / full-entry length distributions, stripHtml and the
row-sharded (2-rank) fit. Expected values ported from ``SmartTextVectorizerTest.scala:579-720``."""
import math
from collections import Counter

import numpy as np
import pytest
import torch

from transmogrifai_amd.data.columns import column_from_values
from transmogrifai_amd.features import types as T
from transmogrifai_amd.stages.feature.vectorizers import TextStats, reduce_text_stats

STRING = "I have got a LovEly buncH of cOcOnuts. Here they are ALL standing in a row."


def _col(vals):
    return column_from_values(T.Text, vals, "cpu")


def _std(seq):
    m = sum(seq) / len(seq)
    return math.sqrt(sum((x - m) ** 2 for x in seq) / len(seq))


def test_text_stats_from_string_with_cleaning_tokens():
    st = TextStats.of_column(_col([STRING]), clean=True, token_lengths=True, max_card=50)
    assert st.value_counts == Counter({"IHaveGotALovelyBunchOfCoconutsHereTheyAreAllStandingInARow": 1})
    assert st.length_counts == Counter({6: 1, 3: 2, 5: 1, 8: 2})
    assert abs(st.length_std - _std([6, 3, 3, 5, 8, 8])) < 1e-12


def test_text_stats_from_string_without_cleaning():
    st = TextStats.of_column(_col([STRING]), clean=False, token_lengths=True, max_card=50)
    assert st.value_counts == Counter({STRING: 1})
    assert st.length_counts == Counter({6: 1, 3: 2, 5: 1, 8: 2})


def test_text_stats_respects_max_cardinality_in_token_lengths():
    # lengths fold got(3), lovely(6), bunch(5) -> 3 keys > 2: frozen
    st = TextStats.of_column(_col([STRING]), clean=False, token_lengths=True, max_card=2)
    assert st.length_counts == Counter({6: 1, 3: 1, 5: 1})
    assert abs(st.length_std - _std([6, 3, 5])) < 1e-12


def test_text_stats_full_entry_length():
    st = TextStats.of_column(_col([STRING]), clean=True, token_lengths=False, max_card=50)
    assert st.length_counts == Counter({58: 1})


def test_text_stats_monoid():
    l1 = TextStats(Counter({"hello": 1, "world": 2}), Counter({5: 3}))
    r1 = TextStats(Counter({"hello": 1, "world": 1}), Counter({5: 2}))
    e1 = l1.plus(r1, 2)
    assert e1.value_counts == Counter({"hello": 2, "world": 3}) and e1.length_counts == Counter({5: 5})
    l2 = TextStats(Counter({"hello": 1, "world": 2, "ocean": 3}), Counter({5: 6}))
    r2 = TextStats(Counter({"hello": 1}), Counter({5: 1}))
    e2 = l2.plus(r2, 2)
    assert e2.value_counts == Counter({"hello": 1, "world": 2, "ocean": 3}) and e2.length_counts == Counter({5: 7})


def test_text_stats_length_statistics():
    ts = TextStats(Counter({"hello": 2, "joe": 2, "woof": 1}), Counter({3: 2, 4: 1, 5: 2}))
    assert abs(ts.length_std - math.sqrt(0.8)) < 1e-12
    assert math.isnan(TextStats(Counter({"the": 10}), Counter()).length_std)


def test_value_counts_freeze_after_max_cardinality_plus_one_values():
    """Left fold of one-value maps: counting stops once max_card + 1 distinct values were seen."""
    vals = ["a", "b", "a", "c", None, "d", "a", "b", "e", "c"]
    st = TextStats.of_column(_col(vals), clean=False, token_lengths=False, max_card=2)
    # a, b, a, c -> 3 distinct at row 3: frozen there
    assert st.value_counts == Counter({"a": 2, "b": 1, "c": 1})
    # the same fold written out with the monoid
    acc = TextStats(Counter(), Counter())
    for v in vals:
        if v is not None:
            acc = acc.plus(TextStats(Counter({v: 1}), Counter({len(v): 1})), 2)
    assert acc.value_counts == st.value_counts
    # partitions merged in order: the frozen left side wins
    parts = [[TextStats.of_column(_col(vals[:5]), False, False, 2)], [TextStats.of_column(_col(vals[5:]), False, False, 2)]]
    merged = reduce_text_stats(parts, 2)[0]
    assert merged.value_counts == Counter({"a": 2, "b": 1, "c": 1})


def test_smart_text_model_strip_html_tokens():
    from transmogrifai_amd.stages.feature.vectorizers import SmartTextVectorizerModel, HashingParams
    html = "<body>Big ones, small <h1>ones</h1>, some as big as your head</body>"
    c = _col([html])
    m = SmartTextVectorizerModel(["hash"], [[]], True, False, HashingParams(num_features=64, num_inputs=1,
                                 prepend_feature_name=False), strip_html=True)
    m2 = SmartTextVectorizerModel(["hash"], [[]], True, False, HashingParams(num_features=64, num_inputs=1,
                                  prepend_feature_name=False), strip_html=False)
    a = m.transform_columns(c).values
    b = m2.transform_columns(c).values
    # the html tag names (body, h1) are hashed only without stripping
    assert float(b.sum()) > float(a.sum())
    from transmogrifai_amd.utils import text as TU
    assert sorted(TU.tokenize(TU.strip_html(html))) == sorted(["big", "ones", "small", "ones", "big", "head"])


def test_text_length_type_tokens_ignores_constant_token_length_ids():
    """Machine-generated ids (fixed 6-digit tokens) have token-length std 0 and are ignored with
    textLengthType = Tokens (SmartTextVectorizerTest.scala:212-246)."""
    from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
    from transmogrifai_amd.stages.feature.vectorizers import SmartTextVectorizer
    rng = np.random.default_rng(3)
    ids = [None if rng.random() < 0.2 else "%06d" % (40230 + int(rng.integers(1, 1000))) for _ in range(1000)]
    words = ["alpha", "be", "gamma", "delta", "epsilonic", "z"]
    text = [None if rng.random() < 0.2 else " ".join(rng.choice(words, size=int(rng.integers(1, 8))))
            for _ in range(1000)]
    ds, (fi, ft) = TestFeatureBuilder.of(("textId", T.Text, ids), ("text", T.Text, text))
    st = SmartTextVectorizer(max_cardinality=10, num_features=5, min_support=10, top_k=3, min_length_std_dev=0.5,
                             text_length_type="Tokens", track_text_len=True)
    st.set_input(fi, ft)
    model = st.fit(ds)
    assert model.methods == ["ignore", "hash"]
    with pytest.raises(ValueError):
        SmartTextVectorizer(text_length_type="Words").set_input(fi).fit(ds)


def test_native_clean_batch_equals_clean_string():
    """ops/csrc/host/text_clean.cpp: ASCII strings cleaned natively, the rest through clean_string; ids in
    first-appearance order of equal cleaned values, lengths in characters."""
    import numpy as np
    from transmogrifai_amd.utils import text as TU
    rng = np.random.default_rng(0)
    alpha = list("abcXYZ ,.-_!?'\t09Éßİ")
    vals = ["".join(rng.choice(alpha, size=rng.integers(0, 12))) for _ in range(5000)] + ["", "İstanbul", "ǅ x"]
    cb = TU.clean_batch(vals, True)
    py = [TU.clean_string(v) for v in vals]
    ids = {}
    exp = [ids.setdefault(v, len(ids)) for v in py]
    assert [cb.value(j) for j in range(len(vals))] == py
    assert cb.ids.tolist() == exp and cb.n_ids == len(ids)
    assert cb.char_len.tolist() == [len(v) for v in py]
    raw = TU.clean_batch(vals, False)
    ids = {}
    assert raw.ids.tolist() == [ids.setdefault(v, len(ids)) for v in vals]

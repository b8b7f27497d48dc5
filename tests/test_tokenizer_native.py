"""Native multithreaded tokenizer (ops/csrc/host/tokenizer.cpp) against the Python spec
``utils/text.py:tokenize`` (TextTokenizer.scala:160-188 default analyzer rules)."""
import random

import numpy as np
import pytest

from transmogrifai_amd.utils import text as TU

ALPH = (list("abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789_ .,'-!?") * 4 +
        list("ÀÉÎõüßçñ²¼µ") + list("ΑΣσςβДжЁ") + list("東京中文タワーー한국") + list("٣٤۵") + ["😀", "İ", "　"])


def _rand_strings(n, seed):
    r = random.Random(seed)
    out = []
    for _ in range(n):
        if r.random() < 0.05:
            out.append(None)
            continue
        words = []
        for _ in range(r.randint(0, 12)):
            if r.random() < 0.3:
                words.append(r.choice(sorted(TU.ENGLISH_STOPWORDS)).upper() if r.random() < 0.2 else
                             r.choice(sorted(TU.ENGLISH_STOPWORDS)))
            else:
                words.append("".join(r.choice(ALPH) for _ in range(r.randint(1, 9))))
        out.append(" ".join(words))
    return out


@pytest.mark.parametrize("lower,min_len", [(True, 1), (False, 1), (True, 3)])
def test_native_tokenizer_matches_python(lower, min_len):
    ss = _rand_strings(5000, 7)   # > 2048 strings: the OpenMP path
    tb = TU.tokenize_batch(ss, lower, min_len)
    assert tb.lists() == [TU.tokenize(s, lower, min_len) for s in ss]


def test_native_tokenizer_no_stopwords_and_lengths():
    ss = _rand_strings(300, 11)
    tb = TU.tokenize_batch(ss, stopwords=frozenset())
    ref = [TU.tokenize(s, stopwords=frozenset()) for s in ss]
    assert tb.lists() == ref
    np.testing.assert_array_equal(tb.counts(), [len(t) for t in ref])
    np.testing.assert_array_equal(tb.char_lengths(), [sum(len(x) for x in t) for t in ref])


def test_long_tokens_capped():
    s = "a" * 255 + " " + "b" * 256 + " ok"
    assert TU.tokenize_batch([s]).lists() == [TU.tokenize(s)] == [["a" * 255, "ok"]]

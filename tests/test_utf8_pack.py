"""Native UTF-8 packing of str lists (ops/csrc/host/utf8_pack.cpp) equals str.encode + join, falls back on what
str.encode rejects."""
import random

import numpy as np
import pytest

from transmogrifai_amd.utils import text as T


def _ref(strings):
    enc = [s.encode("utf-8") if s else b"" for s in strings]
    offs = np.zeros(len(enc) + 1, np.int64)
    np.cumsum([len(e) for e in enc], out=offs[1:])
    return np.frombuffer(b"".join(enc) or b"\0", np.uint8), offs


def test_utf8_pack_matches_encode():
    rnd = random.Random(3)
    alphabet = ["a", "Z", " ", "é", "ß", "ÿ", "Ω", "中", "テ", "😀", "Ā", "￿", "\U0010ffff"]
    strings = ["".join(rnd.choice(alphabet) for _ in range(rnd.randint(0, 40))) for _ in range(3000)]
    strings += ["", None, "plain ascii", "latin-1 only: é à ü"]
    buf, offs = T._encode_batch_impl(strings)
    rb, ro = _ref(strings)
    assert np.array_equal(offs, ro)
    assert np.array_equal(buf[:len(rb)], rb)


def test_utf8_pack_falls_back():
    with pytest.raises(UnicodeEncodeError):          # a lone surrogate: the Python path raises as str.encode does
        T._encode_batch_impl(["ok", "a\ud800"])
    buf, offs = T._encode_batch_impl(["", None])
    assert list(offs) == [0, 0, 0]

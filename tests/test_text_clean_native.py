"""Native batch cleaning and first-appearance grouping (ops/csrc/host/text_clean.cpp): the parallel paths
(batches above 65536 strings) give exactly the serial results -- TextUtils.cleanString per value and ids in order
of first appearance."""
import random
import string

import numpy as np

from transmogrifai_amd.utils import text as TU


def _strings(n, seed):
    rng = random.Random(seed)
    words = ["".join(rng.choices(string.ascii_letters, k=rng.randint(1, 9))) for _ in range(3000)]
    out = []
    for i in range(n):
        r = rng.random()
        if r < 0.05:
            out.append(None)
        elif r < 0.08:
            out.append("Ünïcode " + rng.choice(words))          # Python fallback path
        else:
            out.append(rng.choice(" -.,!?").join(rng.choices(words, k=rng.randint(1, 4))))
    return out


def _first_ids(values):
    seen, ids = {}, []
    for v in values:
        ids.append(seen.setdefault(v, len(seen)))
    return np.asarray(ids), len(seen)


def test_clean_batch_matches_clean_string_and_first_appearance_ids():
    for n in (1000, 150_000):                                   # serial and parallel paths
        strs = _strings(n, seed=n)
        TU.clear_batch_cache()
        cb = TU.clean_batch(strs, clean=True)
        want = [TU.clean_string(s or "") for s in strs]
        got = [cb.value(j) for j in range(n)]
        assert got == want
        assert np.array_equal(cb.char_len, [len(w) for w in want])
        ids, k = _first_ids(want)
        assert cb.n_ids == k and np.array_equal(cb.ids, ids)
        raw = TU.clean_batch(strs, clean=False)
        ids, k = _first_ids([s or "" for s in strs])
        assert raw.n_ids == k and np.array_equal(raw.ids, ids)

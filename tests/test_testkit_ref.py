"""The testkit's random generators (``testkit/src/test/.../testkit/``): RandomRealTest, RandomIntegralTest,
RandomTextTest, RandomBinaryTest, RandomListTest, RandomSetTest, RandomMapTest, RandomVectorTest,
RandomStreamTest / InfiniteStreamTest -- distribution moments, null fractions, domains, sizes and reproducibility."""
import math
import statistics

import pytest

from transmogrifai_amd.features import types as T
from transmogrifai_amd.testkit import random_data as R


def _null_frac(xs):
    return sum(1 for x in xs if x is None) / len(xs)


def _vals(xs):
    return [x for x in xs if x is not None]


@pytest.mark.parametrize("gen,p,mean,tol", [
    (lambda: R.RandomReal.normal(1.0, 0.1), 0.1, 1.0, 0.02),
    (lambda: R.RandomReal.uniform(1.0, 2.0), 0.5, 1.5, 0.03),
    (lambda: R.RandomReal.poisson(4.0), 0.2, 4.0, 0.15),
    (lambda: R.RandomReal.exponential(1.0), 0.01, 1.0, 0.08),
    (lambda: R.RandomReal.gamma(5.0, 1.0), 0.0, 5.0, 0.2),
])
def test_random_real_distributions(gen, p, mean, tol):
    """RandomRealTest: the requested mean and null fraction."""
    xs = gen().with_probability_of_empty(p).take(5000)
    assert abs(_null_frac(xs) - p) < 0.03
    assert abs(statistics.fmean(_vals(xs)) - mean) < tol


def test_random_real_ranges_and_types():
    u = _vals(R.RandomReal.uniform(1.0, 2.0).take(2000))
    assert all(1.0 <= x < 2.0 for x in u)
    assert all(x > 0 for x in _vals(R.RandomReal.log_normal(0.25, 0.1).take(500)))
    assert R.RandomReal.normal(0.0, 1.0, T.RealNN).ftype is T.RealNN


def test_random_integral_and_dates():
    xs = R.RandomIntegral.integrals(10, 20).with_probability_of_empty(0.2).take(3000)
    v = _vals(xs)
    assert all(10 <= x < 20 for x in v) and len(set(v)) == 10 and abs(_null_frac(xs) - 0.2) < 0.03
    start = 1_500_000_000_000
    ds = _vals(R.RandomIntegral.dates(start, 86_400_000, 100).take(500))
    assert all(d >= start and (d - start) % 86_400_000 == 0 for d in ds)
    dts = _vals(R.RandomIntegral.datetimes(start, start + 10_000).take(500))
    assert all(start <= d < start + 10_000 for d in dts)


def test_random_binary():
    xs = R.RandomBinary(0.3).with_probability_of_empty(0.1).take(5000)
    v = _vals(xs)
    assert abs(sum(v) / len(v) - 0.3) < 0.03 and abs(_null_frac(xs) - 0.1) < 0.02


def test_random_text_generators():
    s = _vals(R.RandomText.strings(3, 8).take(500))
    assert all(3 <= len(x) < 8 for x in s) and len(set(s)) > 400
    dom = ["A", "B", "C"]
    assert set(_vals(R.RandomText.text_from_domain(dom).take(300))) <= set(dom)
    picks = R.RandomText.pick_lists(dom, [0.7, 0.2, 0.1]).take(5000)
    assert abs(picks.count("A") / 5000 - 0.7) < 0.03
    emails = _vals(R.RandomText.emails("example.com").take(100))
    assert all(e.endswith("@example.com") for e in emails)
    assert all(T.URL(u).is_valid() for u in _vals(R.RandomText.urls().take(100)))
    assert all(len(x) == 5 and x.isdigit() for x in _vals(R.RandomText.postal_codes().take(100)))
    ids = _vals(R.RandomText.unique_ids().take(1000))
    assert len(set(ids)) == 1000
    assert len(_vals(R.RandomText.ids().take(200))) == 200                    # no empty IDs by default


def test_random_lists_sets_maps_vectors():
    lists = R.RandomList.of_texts(R.RandomText.strings(1, 5), 2, 6).take(300)
    assert all(2 <= len(x) < 6 for x in lists)
    sets = R.RandomSet.of(R.RandomText.text_from_domain(["a", "b", "c", "d"]), 1, 3).take(300)
    assert all(set(x) <= {"a", "b", "c", "d"} for x in sets)
    maps = R.RandomMap.of(R.RandomText.strings(1, 5), 0, 3).take(300)
    assert all(len(m) < 3 and set(m) <= {"k0", "k1"} for m in maps)
    vecs = R.RandomVector.dense(R.RandomReal.uniform(0.0, 1.0), 7).take(50)
    assert all(len(v) == 7 and all(0 <= x < 1 for x in v) for v in vecs)
    sparse = R.RandomVector.sparse(R.RandomReal.normal().with_probability_of_empty(0.5), 40).take(200)
    zeros = sum(x == 0.0 for v in sparse for x in v) / (200 * 40)
    assert abs(zeros - 0.5) < 0.05


def test_streams_are_reproducible_and_resettable():
    a = R.RandomReal.normal(seed=7).take(20) if "seed" in R.RandomReal.normal.__code__.co_varnames else None
    g = R.RandomReal.normal()
    first = g.take(20)
    g.reset(42)
    again = g.take(20)
    assert first == again                     # default seed 42: reset(42) replays the stream
    g.reset(43)
    assert g.take(20) != first
    assert len(list(R.RandomIntegral.integrals(0, 5).limit(17))) == 17
    del a

"""Streaming histogram (native C++) against the reference's fixtures
(utils/src/test/scala/com/salesforce/op/utils/stats/StreamingHistogramTest.scala)."""
import numpy as np

from transmogrifai_amd.utils.stats import StreamingHistogram, density
from transmogrifai_amd.utils.version import version_info


def _reference_histogram():
    h = StreamingHistogram(5, 0, 1)
    for v in (23, 19, 10, 16, 36, 2, 9):
        h.update(v)
    h2 = StreamingHistogram(5, 0, 1)
    h2.update([32, 30, 45])
    return h.merge(h2)


def test_histogram_bins():
    bins = [(round(p, 2), c) for p, c in _reference_histogram().padded_bins(0.5)]
    assert sorted(bins) == sorted([(1.5, 0.0), (2.0, 1), (9.5, 2), (19.33, 3), (32.67, 3), (45.0, 1), (45.5, 0.0)])


def test_histogram_sum():
    h = _reference_histogram()
    exp = {0: 0.0, 2: 0.5, 9.5: 2.0, 15: 3.28, 20: 4.65, 35: 8.03, 45: 10.0, 46: 10.0}
    for b, v in exp.items():
        assert round(h.sum(b), 2) == v


def test_histogram_merge_of_partitions():
    a = StreamingHistogram(15, 500, 1).update(np.arange(0, 6, dtype=float))
    b = StreamingHistogram(15, 500, 1).update(np.arange(6, 11, dtype=float))
    bins = a.merge(b).padded_bins(0.5)
    assert sorted(bins) == sorted([(float(k), 1.0) for k in range(11)] + [(-0.5, 0.0), (10.5, 0.0)])


def test_histogram_density():
    h = StreamingHistogram(10, 500, 1)
    for pt, ct in ((0.0, 1), (2.0, 3), (3.0, 3), (4.0, 1)):
        h.update(pt, ct)
    pdf = h.density(0.5)
    exp = {-1.0: 0.0, -0.5: 0.0625, 0.0: 0.25, 1.0: 0.25, 2.0: 0.375, 2.5: 0.375, 3.0: 0.25, 3.5: 0.25,
           4.0: 0.0625, 4.5: 0.0, 5.0: 0.0}
    for x, v in exp.items():
        assert abs(pdf(x) - v) < 1e-12, (x, pdf(x), v)


def test_histogram_normal_approximation():
    rng = np.random.default_rng(0)
    x = rng.normal(size=1000)
    h = StreamingHistogram(75, 100, 1).update(x)
    assert len(h.bins()) == 75
    assert abs(h.sum(0.0) / 1000 - 0.5) < 0.05
    assert abs(sum(p * c for p, c in h.bins()) / 1000 - x.mean()) < 1e-9     # merges keep the mean


def test_version_info():
    v = version_info()
    assert v.version and isinstance(v.to_dict(), dict)

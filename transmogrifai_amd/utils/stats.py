"""Streaming histogram (native host C++) and its density / bin helpers.

Reference: ``StreamingHistogram`` / ``StreamingHistogramBuilder``
(``utils/src/main/java/com/salesforce/op/utils/stats/StreamingHistogram.java:30-299``) and
``RichStreamingHistogram`` (``utils/.../stats/RichStreamingHistogram.scala:39-100``: padded bins and
the histogram density estimator). The bin bookkeeping lives in
``ops/csrc/host/streaming_histogram.cpp``; this module is the ctypes-facing Python surface.
"""
from __future__ import annotations

import ctypes as C
from typing import Callable, Iterable, List, Optional, Tuple

import numpy as np

from ..ops import _native as N


class StreamingHistogram:
    """``StreamingHistogram(max_bins, max_spool=0, round_to=1)``; ``update`` points (optionally with
    counts), ``merge`` another histogram, read ``bins()`` / ``sum(b)`` / ``density(padding)``."""

    def __init__(self, max_bins: int, max_spool: int = 0, round_to: int = 1):
        self.max_bins, self.max_spool, self.round_to = int(max_bins), int(max_spool), int(round_to)
        self._h = N.host().tmog_shist_new(self.max_bins, self.max_spool, self.round_to)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                N.host().tmog_shist_free(h)
            except Exception:   # interpreter shutdown
                pass
            self._h = None

    def update(self, points, counts=None) -> "StreamingHistogram":
        p = np.ascontiguousarray(np.atleast_1d(np.asarray(points, np.float64)))
        c = None if counts is None else np.ascontiguousarray(np.broadcast_to(np.asarray(counts, np.int64), p.shape))
        N.host().tmog_shist_update(self._h, p.ctypes.data, None if c is None else c.ctypes.data, p.size)
        return self

    def merge(self, other: "StreamingHistogram") -> "StreamingHistogram":
        if other is not None:
            N.host().tmog_shist_merge(self._h, other._h)
        return self

    def bins(self) -> List[Tuple[float, int]]:
        n = int(N.host().tmog_shist_size(self._h))
        pts = np.empty(n, np.float64)
        cts = np.empty(n, np.int64)
        if n:
            N.host().tmog_shist_bins(self._h, pts.ctypes.data, cts.ctypes.data)
        return list(zip(pts.tolist(), cts.tolist()))

    def sum(self, b: float) -> float:
        """Estimated number of points in ``(-inf, b]``."""
        return float(N.host().tmog_shist_sum(self._h, C.c_double(float(b))))

    def padded_bins(self, padding: float = 0.1) -> List[Tuple[float, float]]:
        return padded_bins([(p, float(c)) for p, c in self.bins()], padding)

    def density(self, padding: float = 0.1) -> Callable[[float], float]:
        return density(self.padded_bins(padding))


def padded_bins(bins: List[Tuple[float, float]], padding: float) -> List[Tuple[float, float]]:
    if not bins:
        return []
    pts = [p for p, _ in bins]
    return [(min(pts) - padding, 0.0)] + list(bins) + [(max(pts) + padding, 0.0)]


def density(bins: List[Tuple[float, float]]) -> Callable[[float], float]:
    """Histogram density estimator over consecutive bin pairs (trapezoid masses)."""
    if len(bins) == 1:
        return lambda x: 1.0
    lo = np.array([b[0] for b in bins[:-1]])
    hi = np.array([b[0] for b in bins[1:]])
    mass = np.array([(a[1] + b[1]) / 2 for a, b in zip(bins[:-1], bins[1:])])
    total = float(mass.sum())

    def pdf(x: float) -> float:
        if total == 0.0:
            return 0.0
        return float(mass[(x >= lo) & (x < hi)].sum() / total)
    return pdf

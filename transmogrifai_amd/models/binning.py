"""Feature quantization for the histogram tree engine.

Split candidates follow Spark MLlib ``RandomForest.findSplits`` / ``findSplitsForContinuousFeature``
(2.4): a row sample of ``max(maxBins^2, 10000)`` rows, distinct values with counts, and midpoints
picked by the stride rule (native host kernel ``tmog_find_splits_cpu``). A value ``x`` falls in bin
``#{thresholds < x}`` so the tree split "bin <= b" is exactly Spark's "x <= threshold_b".
XGBoost-style missing handling reserves the last bin for missing values (``missing`` value or NaN).
"""
from __future__ import annotations

import os

from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from ..ops import _native as N


@dataclass
class BinSpec:
    thresholds: np.ndarray      # float64 [F, max_splits] padded with +inf
    n_thresh: np.ndarray        # int32 [F]
    B: int                      # histogram width (bins per feature incl. a missing bin)
    missing_bin: int = -1       # bin index of missing values, -1 = no missing handling
    missing_value: Optional[float] = None   # value treated as missing (XGBoost ``missing``), NaN always is

    @property
    def n_bins(self) -> np.ndarray:
        return (self.n_thresh + 1).astype(np.int32)

    @property
    def n_features(self) -> int:
        return self.thresholds.shape[0]

    def to_state(self):
        return {"thresholds": self.thresholds, "n_thresh": self.n_thresh, "B": self.B,
                "missing_bin": self.missing_bin, "missing_value": self.missing_value}

    @staticmethod
    def from_state(d) -> "BinSpec":
        return BinSpec(np.asarray(d["thresholds"], np.float64), np.asarray(d["n_thresh"], np.int32), int(d["B"]),
                       int(d.get("missing_bin", -1)), d.get("missing_value"))

    def threshold(self, f: int, b: int) -> float:
        return float(self.thresholds[f, b])


def sample_rows(n: int, max_bins: int, seed: int = 0, device="cpu") -> torch.Tensor:
    k = max(max_bins * max_bins, 10000)
    if n <= k:
        return torch.arange(n, device=device)
    # O(k) sampling without replacement (a full randperm of n rows costs ~0.3 s at n = 10M)
    idx = np.sort(np.random.default_rng(seed).choice(n, size=k, replace=False))
    return torch.as_tensor(idx, dtype=torch.int64, device=device)


def find_splits(X: torch.Tensor, max_bins: int = 32, seed: int = 0, missing_value: Optional[float] = None,
                reserve_missing: bool = False, rows: Optional[torch.Tensor] = None) -> BinSpec:
    """Compute per-feature thresholds from a row sample of ``X [N, F]``."""
    n, F = int(X.shape[0]), int(X.shape[1])
    idx = sample_rows(n if rows is None else int(rows.numel()), max_bins, seed, X.device)
    if rows is not None:
        idx = rows[idx]
    samp = X[idx].to(torch.float64)
    if missing_value is not None:
        samp = torch.where(samp == missing_value, torch.full_like(samp, float("nan")), samp)
    samp = samp.cpu().numpy()
    samp = np.ascontiguousarray(samp)
    nb = max_bins - 1 if reserve_missing else max_bins
    max_splits = max(1, min(nb, max(2, samp.shape[0])) - 1)
    out = np.empty((F, max_splits), np.float64)
    n_out = np.empty(F, np.int32)
    N.check(N.host().tmog_find_splits_cpu(samp.ctypes.data, samp.shape[0], F, max_splits, out.ctypes.data,
                                          n_out.ctypes.data), "find_splits")
    B = max_bins
    return BinSpec(out, n_out, B, (B - 1) if reserve_missing else -1, missing_value)


def quantize(X: torch.Tensor, spec: BinSpec, chunk_rows: int = 1 << 20) -> torch.Tensor:
    """``uint8 [N, F]`` bins of ``X`` (float) under ``spec`` (row chunks bound the temporaries). A contiguous fp32
    device matrix takes one HIP pass (``ops/csrc/hip/quantize_kernels.hip``; same bins as the torch path:
    ``searchsorted(side="left")`` on the fp32 thresholds, NaN after every threshold, the missing bin)."""
    dev = X.device
    n, F = int(X.shape[0]), int(X.shape[1])
    ms = int(spec.thresholds.shape[1]) if spec.thresholds.ndim == 2 else 0
    if (X.is_cuda and X.dtype == torch.float32 and X.is_contiguous() and 1 <= ms <= 255 and F > 0 and n > 0
            and os.environ.get("TMOG_HIP_QUANTIZE", "1") != "0"):
        from ..ops import _native as N_
        thr32 = torch.as_tensor(np.ascontiguousarray(spec.thresholds, np.float32), device=dev)
        out = torch.empty(n, F, dtype=torch.uint8, device=dev)
        mv = spec.missing_value
        N_.check(N_.hip().tmog_hip_quantize(N_.ptr(X), n, F, N_.ptr(thr32), ms, int(spec.missing_bin),
                                            int(mv is not None), float(mv) if mv is not None else 0.0, N_.ptr(out),
                                            N_.stream(dev)), "quantize")
        return out
    thr = torch.as_tensor(spec.thresholds, device=dev)
    out = torch.empty(n, F, dtype=torch.uint8, device=dev)
    thr_t = thr.to(torch.float32 if X.dtype == torch.float32 else torch.float64).contiguous()
    for a in range(0, n, chunk_rows):
        b = min(n, a + chunk_rows)
        xt = X[a:b].to(thr_t.dtype).t().contiguous()           # [F, rows]
        bins = torch.searchsorted(thr_t, xt, side="left")       # #thresholds < x
        if spec.missing_bin >= 0:
            miss = torch.isnan(xt)
            if spec.missing_value is not None:
                miss |= xt == spec.missing_value
            bins = torch.where(miss, torch.full_like(bins, spec.missing_bin), bins)
        out[a:b] = bins.t().to(torch.uint8)
    return out

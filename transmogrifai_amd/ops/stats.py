"""Column statistics kernels.

* :func:`col_stats` -- Spark ``Statistics.colStats`` (count, mean, unbiased variance, min, max, nnz)
  in one pass; fp32 data is accumulated in fp64 on the device.
* :func:`corr_matrix` -- Pearson (or Spearman via rank transform) correlation of every column pair:
  mean-centered Gram ``Xc^T Xc`` on the matrix cores (fp32 GEMM), normalized in fp64.
* :func:`label_column_sums` -- label x column contingency sums ``onehot(y)^T X`` (skinny GEMM).
"""
from __future__ import annotations

from typing import Dict

import torch

from . import _native as N


def col_stats(X: torch.Tensor) -> Dict[str, torch.Tensor]:
    n = X.shape[0]
    if X.is_cuda and X.dtype == torch.float32 and n > 0 and X.is_contiguous():
        d = X.shape[1]
        out = torch.empty(6, d, dtype=torch.float64, device=X.device)
        N.check(N.hip().tmog_hip_col_stats(N.ptr(X), None, n, d, d, N.ptr(out), N.stream(X.device)), "col_stats")
        s1, s2, mn, mx, nnz = out[0], out[1], out[2], out[3], out[4]
        mean = s1 / max(n, 1)
        var = (s2 - n * mean * mean) / max(n - 1, 1)
        return {"count": n, "mean": mean, "variance": var.clamp_min(0), "min": mn, "max": mx, "numNonzeros": nnz}
    Xd = X.to(torch.float64)
    mean = Xd.mean(0) if n else torch.zeros(X.shape[1], dtype=torch.float64)
    var = Xd.var(0, unbiased=True) if n > 1 else torch.zeros(X.shape[1], dtype=torch.float64)
    return {"count": n, "mean": mean, "variance": var, "min": Xd.min(0).values if n else mean,
            "max": Xd.max(0).values if n else mean, "numNonzeros": (Xd != 0).sum(0).to(torch.float64)}


def _rank_columns(X: torch.Tensor) -> torch.Tensor:
    """Average ranks per column (ties share the mean rank), as Spark's Spearman correlation."""
    n, d = X.shape
    out = torch.empty(n, d, dtype=torch.float64, device=X.device)
    for j in range(d):
        v = X[:, j].to(torch.float64)
        s, order = torch.sort(v, stable=True)
        uniq, inv, cnt = torch.unique_consecutive(s, return_inverse=True, return_counts=True)
        ends = torch.cumsum(cnt, 0).to(torch.float64)
        avg = ends - (cnt.to(torch.float64) - 1) / 2.0
        r = torch.empty(n, dtype=torch.float64, device=X.device)
        r[order] = avg[inv]
        out[:, j] = r
    return out


def corr_matrix(X: torch.Tensor, method: str = "pearson", mean=None) -> torch.Tensor:
    """``(d x d)`` correlation matrix; NaN where a column has zero variance (Spark semantics)."""
    if method == "spearman":
        X = _rank_columns(X)
        mean = None
    n = X.shape[0]
    if mean is None:
        mean = X.to(torch.float64).mean(0)
    Xc = (X - mean.to(X.dtype)[None, :])
    G = (Xc.t() @ Xc).to(torch.float64) / max(n - 1, 1)
    sd = torch.sqrt(torch.diag(G))
    C = G / (sd[:, None] * sd[None, :])
    C = torch.where((sd[:, None] == 0) | (sd[None, :] == 0), torch.full_like(C, float("nan")), C)
    C.fill_diagonal_(1.0)
    return C


def label_column_sums(X: torch.Tensor, y: torch.Tensor):
    """(sorted distinct labels, ``[L, d]`` per-label column sums, ``[L]`` counts)."""
    labels, inv = torch.unique(y.to(torch.float64), return_inverse=True)
    L = labels.numel()
    oh = torch.zeros(X.shape[0], L, dtype=X.dtype, device=X.device)
    oh[torch.arange(X.shape[0], device=X.device), inv] = 1
    sums = (oh.t() @ X).to(torch.float64)
    return labels, sums, oh.sum(0).to(torch.float64)

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


def _col_partials(X: torch.Tensor):
    """(sum, sum of squares, min, max, non-zeros) per column, fp64, in one pass (HIP kernel on fp32 device data)."""
    n, d = X.shape[0], X.shape[1]
    if X.is_cuda and X.dtype == torch.float32 and n > 0 and X.is_contiguous():
        out = torch.empty(6, d, dtype=torch.float64, device=X.device)
        N.check(N.hip().tmog_hip_col_stats(N.ptr(X), None, n, d, d, N.ptr(out), N.stream(X.device)), "col_stats")
        return out[0], out[1], out[2], out[3], out[4]
    Xd = X.to(torch.float64)
    if n == 0:
        z = torch.zeros(d, dtype=torch.float64, device=X.device)
        return z, z.clone(), torch.full_like(z, float("inf")), torch.full_like(z, float("-inf")), z.clone()
    return Xd.sum(0), (Xd * Xd).sum(0), Xd.min(0).values, Xd.max(0).values, (Xd != 0).sum(0).to(torch.float64)


def col_stats(X: torch.Tensor) -> Dict[str, torch.Tensor]:
    """Spark ``Statistics.colStats``. In a row-sharded fit the per-rank partials are all-reduced (one packed
    SUM of count / sums / non-zeros plus a MIN and a MAX, ``SanityChecker.scala:407``)."""
    from ..parallel import dp
    s1, s2, mn, mx, nnz = _col_partials(X)
    n_t = torch.tensor([float(X.shape[0])], dtype=torch.float64, device=s1.device)
    if dp.active():
        n_t, s1, s2, nnz = dp.sum_([n_t, s1, s2, nnz])
        mn, mx = dp.min_(mn), dp.max_(mx)
    n = int(n_t.item())
    mean = s1 / max(n, 1)
    if not dp.active() and not (X.is_cuda and X.dtype == torch.float32) and n > 1:
        var = X.to(torch.float64).var(0, unbiased=True)      # host reference path: two-pass variance
    else:
        var = ((s2 - n * mean * mean) / max(n - 1, 1)).clamp_min(0)
    if n == 0:
        mn, mx = mean, mean
    return {"count": n, "mean": mean, "variance": var, "min": mn, "max": mx, "numNonzeros": nnz}


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
    """``(d x d)`` correlation matrix; NaN where a column has zero variance (Spark semantics).

    Row-sharded fits: Pearson centres every shard on the global mean and all-reduces the partial
    Gramians (``SanityChecker.scala:468``, one ``(d x d)`` SUM); Spearman needs global ranks, so the
    (already down-sampled) rows are gathered first."""
    from ..parallel import dp
    if method == "spearman":
        if dp.active():
            X = dp.rows(X)
            with dp.local_only():
                return corr_matrix(X, method)
        X = _rank_columns(X)
        mean = None
    n = dp.count(X.shape[0])
    if mean is None:
        s, = dp.sum_([X.to(torch.float64).sum(0)])
        mean = s / max(n, 1)
    Xc = (X - mean.to(X.dtype)[None, :])
    G, = dp.sum_([(Xc.t() @ Xc).to(torch.float64)])
    G = G / max(n - 1, 1)
    sd = torch.sqrt(torch.diag(G))
    C = G / (sd[:, None] * sd[None, :])
    C = torch.where((sd[:, None] == 0) | (sd[None, :] == 0), torch.full_like(C, float("nan")), C)
    C.fill_diagonal_(1.0)
    return C


def label_column_sums(X: torch.Tensor, y: torch.Tensor):
    """(sorted distinct labels, ``[L, d]`` per-label column sums, ``[L]`` counts): the skinny GEMM
    ``onehot(y)^T X``. Row-sharded fits use the global label set and all-reduce the sums
    (``SanityChecker.scala:272,280`` ``reduceByKey(label)``)."""
    from ..parallel import dp
    labels = dp.unique_values(y.to(torch.float64))
    inv = torch.searchsorted(labels, y.to(torch.float64))
    L = labels.numel()
    oh = torch.zeros(X.shape[0], L, dtype=X.dtype, device=X.device)
    oh[torch.arange(X.shape[0], device=X.device), inv] = 1
    sums, cnt = dp.sum_([(oh.t() @ X).to(torch.float64), oh.sum(0).to(torch.float64)])
    return labels, sums, cnt

"""Column statistics kernels.

* :func:`col_stats` -- Spark ``Statistics.colStats`` (count, mean, unbiased variance, min, max, nnz)
  in one pass; fp32 data is accumulated in fp64 on the device.
* :func:`corr_matrix` -- Pearson (or Spearman via rank transform) correlation of every column pair:
  mean-centered Gram ``Xc^T Xc`` on the matrix cores (fp32 GEMM), normalized in fp64.
* :func:`label_column_sums` -- label x column contingency sums ``onehot(y)^T X`` (skinny GEMM).
"""
from __future__ import annotations

import os

from typing import Dict, Optional

import torch

from . import _native as N


def _col_partials(X: torch.Tensor):
    """(count, mean, M2, min, max, non-zeros) per column in fp64, one pass. fp32 device data runs the HIP
    shifted-sum / Chan-merge kernel; host data the two-pass reference."""
    n, d = X.shape[0], X.shape[1]
    if X.is_cuda and X.dtype == torch.float32 and n > 0 and X.stride(1) == 1:
        out = torch.empty(6, d, dtype=torch.float64, device=X.device)
        N.check(N.hip().tmog_hip_col_stats(N.ptr(X), None, n, d, X.stride(0), N.ptr(out), N.stream(X.device)),
                "col_stats")
        return n, out[5], out[1], out[2], out[3], out[4]
    Xd = X.to(torch.float64)
    if n == 0:
        z = torch.zeros(d, dtype=torch.float64, device=X.device)
        return 0, z, z.clone(), torch.full_like(z, float("inf")), torch.full_like(z, float("-inf")), z.clone()
    mean = Xd.mean(0)
    m2 = (Xd - mean).pow(2).sum(0)
    return n, mean, m2, Xd.min(0).values, Xd.max(0).values, (Xd != 0).sum(0).to(torch.float64)


def col_stats(X: torch.Tensor) -> Dict[str, torch.Tensor]:
    """Spark ``Statistics.colStats`` with a numerically stable variance (per-chunk shifted sums merged with
    Chan's update on the device; ``SanityChecker.scala:407``). Row-sharded fits gather every rank's
    (count, mean, M2) and merge them the same way, plus a MIN / MAX / SUM of the rest."""
    from ..parallel import dp
    n, mean, m2, mn, mx, nnz = _col_partials(X)
    if dp.active():
        d = mean.numel()
        part = torch.cat([torch.tensor([float(n)], dtype=torch.float64, device=mean.device), mean, m2])[None, :]
        allp = dp.rows(part)                      # [world, 1 + 2d]
        ns, means, m2s = allp[:, 0], allp[:, 1:1 + d], allp[:, 1 + d:]
        tot = float(ns.sum().item())
        gmean = (ns[:, None] * means).sum(0) / max(tot, 1.0)
        m2 = (m2s + ns[:, None] * (means - gmean[None, :]).pow(2)).sum(0)
        mean, n = gmean, int(tot)
        nnz, = dp.sum_([nnz])
        mn, mx = dp.min_(mn), dp.max_(mx)
    var = (m2 / max(n - 1, 1)).clamp_min(0)
    if n == 0:
        mn, mx = mean, mean
    return {"count": n, "mean": mean, "variance": var, "min": mn, "max": mx, "numNonzeros": nnz}


def _rank_columns(X: torch.Tensor, chunk: int = 256) -> torch.Tensor:
    """Average ranks per column (ties share the mean rank), as Spark's Spearman correlation: one batched
    column sort per chunk of columns, tie groups from run starts / ends (cummax / reversed cummin)."""
    n, d = X.shape
    out = torch.empty(n, d, dtype=torch.float64, device=X.device)
    if n == 0:
        return out
    pos = torch.arange(n, device=X.device, dtype=torch.int64)[:, None]
    for a in range(0, d, chunk):
        v = X[:, a:a + chunk].to(torch.float64)
        s, order = torch.sort(v, dim=0, stable=True)
        first = torch.ones_like(s, dtype=torch.bool)
        first[1:] = s[1:] != s[:-1]
        last = torch.ones_like(s, dtype=torch.bool)
        last[:-1] = first[1:]
        start = torch.where(first, pos, torch.zeros_like(pos)).cummax(0).values
        big = torch.full_like(pos, n - 1)
        end = torch.where(last, pos, big).flip(0).cummin(0).values.flip(0)
        avg = (start + end).to(torch.float64) / 2.0 + 1.0
        out[:, a:a + chunk].scatter_(0, order, avg)
    return out


def gram_centered(X: torch.Tensor, mean: torch.Tensor, y_codes: Optional[torch.Tensor] = None,
                  n_labels: int = 0) -> torch.Tensor:
    """``G = A^T A`` with ``A = [X - mean | onehot(y_codes)]`` (fp64 ``[d + L, d + L]``, this rank's rows).

    fp32 device data runs the MFMA ``gram_aug_kernel`` (one pass: centred Gramian, label x column sums and
    label counts); otherwise an fp64 torch reference."""
    n, d = X.shape
    L = int(n_labels)
    if X.is_cuda and X.dtype == torch.float32 and X.stride(1) == 1 and n > 0 and \
            os.environ.get("TMOG_GRAM_BF16", "1") != "0":
        return _gram_centered_bf16(X, mean, y_codes, L)
    if X.is_cuda and X.dtype == torch.float32 and X.stride(1) == 1 and n > 0:
        G = torch.empty(d + L, d + L, dtype=torch.float64, device=X.device)
        mu = mean.to(device=X.device, dtype=torch.float32).contiguous()
        yc = None if L == 0 else y_codes.to(device=X.device, dtype=torch.int32).contiguous()
        N.check(N.hip().tmog_hip_gram_aug(N.ptr(X), n, d, X.stride(0), N.ptr(mu), N.ptr(yc), L, N.ptr(G),
                                          N.stream(X.device)), "gram_aug")
        return G
    A = X.to(torch.float64) - mean.to(device=X.device, dtype=torch.float64)[None, :]
    if L:
        oh = torch.zeros(n, L, dtype=torch.float64, device=X.device)
        oh[torch.arange(n, device=X.device), y_codes.to(X.device).long()] = 1.0
        A = torch.cat([A, oh], 1)
    return A.t() @ A


def bf16_exact_columns(X: torch.Tensor) -> torch.Tensor:
    """``[d]`` bool: every value of the column is exact in bf16 (``stats_kernels.hip`` col_bf16_exact_kernel)."""
    n, d = X.shape
    bits = torch.empty(d, dtype=torch.int32, device=X.device)
    N.check(N.hip().tmog_hip_col_bf16_exact(N.ptr(X), n, d, X.stride(0), N.ptr(bits), N.stream(X.device)),
            "col_bf16_exact")
    return bits == 0


# bf16_pack_kernel column modes
PACK_ZERO, PACK_ONE, PACK_RAW, PACK_HI, PACK_MID, PACK_LO, PACK_LABEL = range(7)


def bf16_pack(X: torch.Tensor, src, mode, mu, sc, ldb: int, rows: Optional[int] = None, y=None) -> torch.Tensor:
    """``B [rows, ldb]`` bf16 built from the fp32 rows of ``X`` per output column (``stats_kernels.hip``
    bf16_pack_kernel: zero / one / raw / hi, mid, lo parts of ``(x - mu) * sc`` / label indicator); output columns
    past ``len(src)`` and rows past ``X``'s are zero."""
    n = X.shape[0]
    dev = X.device
    rows = n if rows is None else rows
    k = len(src)

    def col(v, dtype):
        t = torch.zeros(ldb, dtype=dtype, device=dev)
        if k:
            t[:k] = torch.as_tensor(v, dtype=dtype).to(dev) if not isinstance(v, torch.Tensor) else v.to(dev, dtype)
        return t
    src_t, mode_t = col(src, torch.int32), col(mode, torch.int32)
    mu_t, sc_t = col(mu, torch.float32), col(sc, torch.float32)
    B = torch.empty(rows, ldb, dtype=torch.bfloat16, device=dev)
    if rows > n:
        B[n:].zero_()
    yc = None if y is None else y.to(device=dev, dtype=torch.int32).contiguous()
    N.check(N.hip().tmog_hip_bf16_pack(N.ptr(X), n, X.stride(0), N.ptr(yc), N.ptr(src_t), N.ptr(mode_t), N.ptr(mu_t),
                                       N.ptr(sc_t), N.ptr(B), ldb, N.stream(dev)), "bf16_pack")
    return B


def _gram_centered_bf16(X: torch.Tensor, mean: torch.Tensor, y_codes, L: int) -> torch.Tensor:
    """``gram_centered`` on the bf16 matrix cores (``stats_kernels.hip`` gram_bf16_kernel) at fp32-accumulation
    accuracy: the Gramian of ``B = [X_E | 1 | C_hi | C_mid | C_lo | onehot(y)]`` where ``E`` are the columns whose
    values are exact in bf16 (kept raw) and ``C = X_R - mean_R`` the other columns centred in fp32 as the fp32 kernel
    does and split into three bf16 parts that sum to it exactly (one packing pass, ``bf16_pack``). Every single
    product is exact; the products are summed in fp32 over 256-row slices (so the result carries fp32 rounding of
    those partial sums, like the fp32 kernel, but is not bit-identical to it), then in fp64 across slices; the
    centred blocks of the original columns are assembled from ``B^T B`` in fp64 (the ones column gives the raw
    column sums and the row count), re-centred from the fp32-rounded mean the packing used onto the fp64 mean.
    ``tests/test_sanity_kernels_gpu.py`` bounds it against the fp64 Gramian."""
    n, d = X.shape
    dev = X.device
    exact = bf16_exact_columns(X)
    E = torch.nonzero(exact).reshape(-1)
    R = torch.nonzero(~exact).reshape(-1)
    nE, nR = int(E.numel()), int(R.numel())
    mu64 = mean.to(device=dev, dtype=torch.float64)
    mu32 = mu64.to(torch.float32)
    D = nE + 1 + 3 * nR + L
    lda = ((D + 127) // 128) * 128
    zi = torch.zeros(1, dtype=torch.int64, device=dev)
    src = torch.cat([E, zi, R, R, R, torch.arange(L, device=dev)])
    mode = torch.cat([torch.full((nE,), PACK_RAW, device=dev), torch.full((1,), PACK_ONE, device=dev),
                      torch.full((nR,), PACK_HI, device=dev), torch.full((nR,), PACK_MID, device=dev),
                      torch.full((nR,), PACK_LO, device=dev), torch.full((L,), PACK_LABEL, device=dev)])
    zf = torch.zeros(nE + 1, dtype=torch.float32, device=dev)
    muR = mu32.index_select(0, R)
    mu_cols = torch.cat([zf, muR, muR, muR, torch.zeros(L, dtype=torch.float32, device=dev)])
    sc_cols = torch.ones(D, dtype=torch.float32, device=dev)
    B = bf16_pack(X, src, mode, mu_cols, sc_cols, lda, y=y_codes if L else None)
    GA = torch.empty(D, D, dtype=torch.float64, device=dev)
    N.check(N.hip().tmog_hip_gram_bf16(N.ptr(B), n, lda, D, N.ptr(GA), N.stream(dev)), "gram_bf16")
    del B
    ie = torch.arange(nE, device=dev)
    io = nE
    iH = nE + 1
    iY = iH + 3 * nR
    parts = [torch.arange(iH + k * nR, iH + (k + 1) * nR, device=dev) for k in range(3)]
    iy = torch.arange(iY, iY + L, device=dev)

    def blk(a, b):
        return GA.index_select(0, a).index_select(1, b)

    muE = mu64.index_select(0, E)
    sE = GA[io].index_select(0, ie)                     # raw column sums of the exact columns
    cnt = GA[io, io]
    SR = sum(GA[io].index_select(0, p) for p in parts)  # sums of the centred other columns
    # the other columns were centred on the fp32-rounded mean (C = x - mu32, exact in fp32); re-centre on the fp64
    # mean in fp64: sum (C_i - dl_i)(C_j - dl_j) with dl = mu64 - mu32 -- for a large-offset, small-spread column
    # the rounding of the mean is a sizeable fraction of its spread, and the variance would carry n dl^2
    dl = mu64.index_select(0, R) - muR.to(torch.float64)
    G = torch.empty(d + L, d + L, dtype=torch.float64, device=dev)
    G_EE = blk(ie, ie) - muE[:, None] * sE[None, :] - sE[:, None] * muE[None, :] + cnt * muE[:, None] * muE[None, :]
    G_ER = sum(blk(ie, p) for p in parts) - muE[:, None] * SR[None, :] - (sE - cnt * muE)[:, None] * dl[None, :]
    G_RR = sum(blk(p, q) for p in parts for q in parts) - SR[:, None] * dl[None, :] - dl[:, None] * SR[None, :] + \
        cnt * dl[:, None] * dl[None, :]
    G[E[:, None], E[None, :]] = G_EE
    G[E[:, None], R[None, :]] = G_ER
    G[R[:, None], E[None, :]] = G_ER.t()
    G[R[:, None], R[None, :]] = G_RR
    if L:
        ly = torch.arange(d, d + L, device=dev)
        nl = GA[iy, io]
        G_YE = blk(iy, ie) - nl[:, None] * muE[None, :]
        G_YR = sum(blk(iy, p) for p in parts) - nl[:, None] * dl[None, :]
        G[ly[:, None], E[None, :]] = G_YE
        G[E[:, None], ly[None, :]] = G_YE.t()
        G[ly[:, None], R[None, :]] = G_YR
        G[R[:, None], ly[None, :]] = G_YR.t()
        G[ly[:, None], ly[None, :]] = blk(iy, iy)
    return G


def _corr_from_gram(G: torch.Tensor, n: int) -> torch.Tensor:
    G = G / max(n - 1, 1)
    sd = torch.sqrt(torch.diag(G).clamp_min(0))
    C = G / (sd[:, None] * sd[None, :])
    C = torch.where((sd[:, None] == 0) | (sd[None, :] == 0), torch.full_like(C, float("nan")), C)
    C.fill_diagonal_(1.0)
    return C


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
    if X.dtype == torch.float64 and X.is_cuda:      # ranks: centred fp64 GEMM on the device
        Xc = X - mean.to(X.dtype)[None, :]
        G = Xc.t() @ Xc
    else:
        G = gram_centered(X, mean)
    G, = dp.sum_([G])
    return _corr_from_gram(G, n)


def _shift(mean: torch.Tensor, mn: Optional[torch.Tensor], mx: Optional[torch.Tensor]) -> torch.Tensor:
    """Per-column centring shift: the nearest integer to the mean for integer-bounded columns (one-hot,
    null indicators, counts: ``x - shift`` and every fp32 product / partial sum stay exact), else the
    fp32-rounded mean."""
    s = mean.to(torch.float32).to(torch.float64)
    if mn is None or mx is None:
        return s
    mn, mx = mn.to(mean.device, torch.float64), mx.to(mean.device, torch.float64)
    integral = (mn == torch.round(mn)) & (mx == torch.round(mx)) & ((mx - mn) < 2 ** 20)
    return torch.where(integral, torch.round(mean), s)


def corr_and_label_sums(X: torch.Tensor, y: torch.Tensor, mean: torch.Tensor, mn: Optional[torch.Tensor] = None,
                        mx: Optional[torch.Tensor] = None):
    """Pearson correlation matrix of ``X`` plus the label contingency of its columns from ONE Gramian pass
    (``SanityChecker.scala:464-470`` + ``categoricalTests:252-348``): returns ``(C [d, d], labels [L],
    sums [L, d] = onehot(y)^T X, counts [L])``. Row-sharded: global labels, one SUM of the partial Gramian.

    The kernel centres on a per-column shift ``s`` (``_shift``); the centred Gramian is recovered in fp64 as
    ``G_s - n (mean - s)(mean - s)^T`` and the label sums as ``onehot^T (X - s) + n_l s`` -- exact for
    indicator / count columns, whose contingency tables feed Cramér's V."""
    from ..parallel import dp
    labels = dp.unique_values(y.to(torch.float64))
    codes = torch.searchsorted(labels, y.to(torch.float64))
    L = labels.numel()
    d = X.shape[1]
    mean = mean.to(torch.float64)
    sh = _shift(mean, mn, mx)
    G = gram_centered(X, sh, codes, L)
    G, = dp.sum_([G])
    n = dp.count(X.shape[0])
    delta = (mean - sh).to(G.device)
    Gx = G[:d, :d] - n * delta[:, None] * delta[None, :]
    C = _corr_from_gram(Gx, n)
    counts = torch.diag(G[d:, d:]).clone()
    sums = G[d:, :d] + counts[:, None] * sh.to(G.device)[None, :]
    return C, labels, sums, counts


def class_column_sums(X: torch.Tensor, codes: torch.Tensor, n_classes: int) -> torch.Tensor:
    """``[P, L, d]`` fp64 sums of the rows of ``X`` per problem ``p`` and class ``c`` (``codes[p, r] == c``;
    -1 leaves row r out of problem p): the label x column contingency / NaiveBayes class feature sums.
    fp32 device data with ``P * L <= 64`` runs the deterministic HIP ``class_colsum_kernel``."""
    P, n = codes.shape
    d = X.shape[1]
    L = int(n_classes)
    if X.is_cuda and X.dtype == torch.float32 and X.stride(1) == 1 and n > 0 and P * L <= 64:
        out = torch.empty(P, L, d, dtype=torch.float64, device=X.device)
        cd = codes.to(device=X.device, dtype=torch.int32).contiguous()
        N.check(N.hip().tmog_hip_class_colsum(N.ptr(X), n, d, X.stride(0), N.ptr(cd), P, L, N.ptr(out),
                                              N.stream(X.device)), "class_colsum")
        return out
    Xd = X.to(torch.float64)
    out = torch.zeros(P, L, d, dtype=torch.float64, device=X.device)
    for p in range(P):
        c = codes[p].to(X.device).long()
        m = c >= 0
        out[p].index_add_(0, c[m], Xd[m])
    return out


def label_column_sums(X: torch.Tensor, y: torch.Tensor):
    """(sorted distinct labels, ``[L, d]`` per-label column sums, ``[L]`` counts): the skinny GEMM
    ``onehot(y)^T X``. Row-sharded fits use the global label set and all-reduce the sums
    (``SanityChecker.scala:272,280`` ``reduceByKey(label)``)."""
    from ..parallel import dp
    labels = dp.unique_values(y.to(torch.float64))
    inv = torch.searchsorted(labels, y.to(torch.float64))
    L = labels.numel()
    sums = class_column_sums(X, inv[None, :], L)[0]
    cnt = torch.bincount(inv, minlength=L).to(torch.float64)
    sums, cnt = dp.sum_([sums, cnt])
    return labels, sums, cnt


def weighted_gram(X: torch.Tensor, W: torch.Tensor, Y: Optional[torch.Tensor] = None,
                  chunk: int = 1 << 18) -> torch.Tensor:
    """``[K, D, D]`` fp64 weighted Grams ``A_k^T diag(W[:, k]) A_k`` with ``A_k = [X | 1 | Y_k]`` (``D = d + 1``,
    ``+ 1`` with ``Y``): the normal-equation statistics of the linear learners (Spark WeightedLeastSquares /
    IRLS). ``Y`` is ``[n]`` (one response shared by every weight column) or ``[n, K]`` (one per column, the
    IRLS working responses). fp32 device ``X`` runs the HIP fp64-MFMA kernel (``stats_kernels.hip``
    ``wgram_kernel``: X read once per tile pair for 4 weight columns, exact fp64 products); otherwise the
    row-chunked fp64 torch reference."""
    n, d = int(X.shape[0]), int(X.shape[1])
    K = int(W.shape[1])
    dev = X.device
    D = d + 1 + (0 if Y is None else 1)
    per_weight = Y is not None and Y.dim() == 2
    if Y is not None and Y.dim() == 2 and int(Y.shape[1]) != K:
        raise ValueError("Y must be [n] or [n, K]")
    if dev.type == "cuda" and X.dtype == torch.float32 and X.stride(1) == 1 and n > 0 and d > 0 and K > 0:
        Wd = W.to(torch.float64).contiguous()
        Yd = None if Y is None else Y.to(torch.float64).contiguous()
        G = torch.empty(K, D, D, dtype=torch.float64, device=dev)
        N.check(N.hip().tmog_hip_wgram(N.ptr(X), n, d, X.stride(0), N.ptr(Wd), K, K, N.ptr(Yd),
                                       (K if per_weight else 1) if Yd is not None else 0, int(per_weight),
                                       N.ptr(G), N.stream(dev)), "wgram")
        return G
    G = torch.zeros(K, D, D, dtype=torch.float64, device=dev)
    for a in range(0, n, chunk):
        Xc = X[a:a + chunk].to(torch.float64)
        m = Xc.shape[0]
        base = torch.cat([Xc, torch.ones(m, 1, dtype=torch.float64, device=dev)], 1)
        Wc = W[a:a + chunk].to(torch.float64)
        for k in range(K):
            if Y is None:
                A = base
            else:
                yk = (Y[a:a + chunk, k] if per_weight else Y[a:a + chunk]).to(torch.float64)
                A = torch.cat([base, yk[:, None]], 1)
            G[k] += A.t() @ (A * Wc[:, k:k + 1])
    return G

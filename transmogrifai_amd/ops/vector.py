"""Vectorizer column kernels (fill / null-indicator blocks, one-hot scatter, hashed TF scatter).

Device tensors go to the fused HIP kernels in ``csrc/hip/vector_kernels.hip`` when they are
available for the shape; host tensors use the torch reference path, which is also the numerics
spec the HIP kernels are tested against.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np
import torch

from ..data.columns import NumericColumn
from . import _native as N
from .staging import Pack, to_device


def column_means(cols: Sequence[NumericColumn]) -> List[float]:
    """Mean of non-null values per column; 0 when a column is all null (``MeanSeqNullNum``).

    All columns reduce in one batched pass and one host read; in a row-sharded fit the (sum, count)
    pairs of every column are all-reduced in one collective (``RealVectorizer.scala:84``)."""
    from ..parallel import dp
    if not cols:
        return []
    dev = cols[0].values.device
    if dev.type == "cuda" and all(c.values.dtype in (torch.float32, torch.float64) and c.values.dim() == 1
                                  and len(c) == len(cols[0]) for c in cols) and len(cols[0]) > 0:
        sums, cnts = _masked_colsums_hip(cols, dev)
    else:
        sums = torch.stack([torch.where(c.valid, c.values.to(torch.float64),
                                        torch.zeros((), dtype=torch.float64, device=c.values.device)).sum()
                            for c in cols])
        cnts = torch.stack([c.valid.sum().to(torch.float64) for c in cols])
    sums, cnts = dp.sum_([sums, cnts])
    s, n = sums.cpu().numpy(), cnts.cpu().numpy()
    return [float(a / b) if b > 0 else float(a) for a, b in zip(s, n)]


def _masked_colsums_hip(cols: Sequence[NumericColumn], dev):
    """(sums, counts) fp64 of the valid values of every column: one ``masked_colsum_kernel`` launch over all
    of them (vector_kernels.hip) instead of ~5 torch launches per column."""
    n = len(cols[0])
    vals = [c.values.contiguous() for c in cols]
    oks = [c.valid.contiguous() if c.valid is not None else None for c in cols]
    rpc = max(1 << 16, -(-n // max(1, 2048 // len(cols))))       # >= ~2048 workgroups in all
    chunks = -(-n // rpc)
    part = torch.empty(len(cols), chunks, 2, dtype=torch.float64, device=dev)
    pk = Pack(dev)
    i_v = pk.add(np.array([t.data_ptr() for t in vals], np.int64))
    i_o = pk.add(np.array([t.data_ptr() if t is not None else 0 for t in oks], np.int64))
    i_d = pk.add(np.array([1 if t.dtype == torch.float64 else 0 for t in vals], np.int32))
    d = pk.ship()
    N.check(N.hip().tmog_hip_masked_colsum(N.ptr(d[i_v]), N.ptr(d[i_o]), N.ptr(d[i_d]), len(cols), n, rpc,
                                           N.ptr(part), N.stream(dev)), "masked_colsum")
    tot = part.sum(1)
    return tot[:, 0].contiguous(), tot[:, 1].contiguous()


_MODE_RANGE = 1 << 20


def column_modes(cols: Sequence[NumericColumn]) -> List[float]:
    """Mode of non-null values per column, ties -> smallest value, 0 if empty (``ModeSeqNullInt``,
    ``IntegralVectorizer.scala:79``).

    Columns whose (global) value range spans at most 2^20 values are offset-coded and counted by the
    HIP ``code_count_kernel`` (LDS-privatised histogram) in one launch, the counts all-reduced over
    ranks in one collective; the first maximum of the dense count table is the smallest modal value.
    Wider columns go through a sort-based ``unique`` whose (value, count) tables are merged over ranks."""
    from ..parallel import dp
    from .text import code_counts
    if not cols:
        return []
    dev = cols[0].values.device
    big = torch.tensor(2 ** 62, dtype=torch.int64, device=dev)
    vals = [c.values.to(torch.int64) for c in cols]
    lo = torch.stack([torch.where(c.valid, v, big).min() if len(c) else big for c, v in zip(cols, vals)])
    hi = torch.stack([torch.where(c.valid, v, -big).max() if len(c) else -big for c, v in zip(cols, vals)])
    lo, hi = dp.min_(lo), dp.max_(hi)
    lo_h, hi_h = lo.cpu().numpy(), hi.cpu().numpy()
    out: List[float] = [0.0] * len(cols)
    dense = [j for j in range(len(cols)) if lo_h[j] <= hi_h[j] and hi_h[j] - lo_h[j] < _MODE_RANGE]
    wide = [j for j in range(len(cols)) if lo_h[j] <= hi_h[j] and hi_h[j] - lo_h[j] >= _MODE_RANGE]
    if dense:
        codes = [torch.where(cols[j].valid, vals[j] - int(lo_h[j]), torch.full_like(vals[j], -1)).to(torch.int32)
                 for j in dense]
        nv = [int(hi_h[j] - lo_h[j]) + 1 for j in dense]
        counts = code_counts(codes, nv)
        summed = np.concatenate([c[:-1] for c in counts])
        if dp.active():
            summed = dp.sum_([torch.as_tensor(summed, device=dev)])[0].cpu().numpy()
        o = 0
        for j, v in zip(dense, nv):
            seg = summed[o:o + v]
            o += v
            out[j] = float(int(lo_h[j]) + int(np.argmax(seg)))
    if wide:
        tables = []
        for j in wide:
            u, cnt = torch.unique(vals[j][cols[j].valid], return_counts=True)
            tables.append((u.cpu().numpy(), cnt.cpu().numpy()))
        parts = dp.objects(tables)
        for k, j in enumerate(wide):
            u = np.concatenate([p[k][0] for p in parts])
            c = np.concatenate([p[k][1] for p in parts])
            uu, inv = np.unique(u, return_inverse=True)
            tot = np.bincount(inv, weights=c)
            out[j] = float(uu[int(np.argmax(tot))])
    return out


def gather_rows_cols(blocks, rows, n: int) -> torch.Tensor:
    """Dense ``[len(rows), width]`` gather of the selected rows (all ``n`` when ``rows`` is None) from a
    blocked vector (list of ``(block, column index or None)``). fp32 device blocks use the HIP
    ``gather_rows_cols_kernel`` (one pass, no per-block temporaries); otherwise torch index ops."""
    dev = blocks[0][0].device
    dtype = blocks[0][0].dtype
    widths = [int(t.shape[1]) if ci is None else int(ci.numel()) for t, ci in blocks]
    k = sum(widths)
    m = n if rows is None else int(rows.numel())
    if dev.type == "cuda" and all(t.dtype == torch.float32 and t.stride(1) == 1 for t, _ in blocks):
        out = torch.empty(m, k, dtype=torch.float32, device=dev)
        if m == 0 or k == 0:
            return out
        base, ld = [], []
        for (t, ci), w in zip(blocks, widths):
            cols = np.arange(w, dtype=np.int64) if ci is None else ci.cpu().numpy().astype(np.int64)
            base.append(t.data_ptr() + 4 * cols)
            ld.append(np.full(w, t.stride(0), np.int64))
        pk = Pack(dev)
        i_b, i_l = pk.add(np.concatenate(base)), pk.add(np.concatenate(ld))
        d = pk.ship()
        r = None if rows is None else rows.to(device=dev, dtype=torch.int64).contiguous()
        N.check(N.hip().tmog_hip_gather_rows_cols(N.ptr(d[i_b]), N.ptr(d[i_l]), N.ptr(r), m, k, N.ptr(out),
                                                  N.stream(dev)), "gather_rows_cols")
        return out
    parts = []
    for t, ci in blocks:
        x = t if rows is None else t.index_select(0, rows.to(t.device))
        parts.append(x if ci is None else x.index_select(1, ci.to(t.device)))
    return torch.cat([p.to(dtype) for p in parts], 1) if parts else torch.zeros(m, 0, dtype=dtype, device=dev)


def fill_and_track(cols: Sequence[NumericColumn], fills: Sequence[float], track_nulls: bool,
                   dtype: torch.dtype) -> torch.Tensor:
    """``[N, F]`` (or ``[N, 2F]`` interleaved with null flags) filled value block."""
    if not cols:
        return torch.zeros(0, 0, dtype=dtype)
    dev = cols[0].values.device
    n = len(cols[0])
    F = len(cols)
    W = F * (2 if track_nulls else 1)
    if dev.type == "cuda" and dtype == torch.float32 and n > 0:
        out = torch.empty(n, W, dtype=dtype, device=dev)
        vals = [c.values.to(torch.float32).contiguous() for c in cols]
        oks = [c.valid.contiguous() for c in cols]
        pk = Pack(dev)
        i_v = pk.add(np.array([t.data_ptr() for t in vals], np.int64))
        i_o = pk.add(np.array([t.data_ptr() for t in oks], np.int64))
        i_f = pk.add(np.asarray(list(fills), np.float32))
        d = pk.ship()
        vp, op, fl = d[i_v], d[i_o], d[i_f]
        N.check(N.hip().tmog_hip_vectorize_numeric(
            N.ptr(vp), N.ptr(op), N.ptr(fl), n, F, None, None, None, N.ptr(out), W, int(track_nulls),
            N.stream(dev)), "vectorize_numeric")
        del vals, oks
        return out
    vals = torch.stack([c.values.to(dtype) for c in cols], 1)
    ok = torch.stack([c.valid for c in cols], 1)
    fill = to_device(np.asarray(list(fills), np.float64), dev).to(dtype)[None, :]
    filled = torch.where(ok, vals, fill)
    if not track_nulls:
        return filled.contiguous()
    return torch.stack([filled, (~ok).to(dtype)], 2).reshape(n, W)


def onehot_pivot(out: torch.Tensor, codes: Sequence[torch.Tensor], luts: Sequence[np.ndarray],
                 offs: Sequence[int]) -> None:
    """All categorical columns of a pivot block in one HIP launch (``onehot_pivot_kernel``) when ``out``
    is an fp32 device matrix; otherwise column by column through ``onehot_scatter``."""
    if not codes:
        return
    dev = out.device
    if dev.type == "cuda" and out.dtype == torch.float32 and out.is_contiguous():
        cs = [c.to(device=dev, dtype=torch.int32).contiguous() for c in codes]
        ls = [np.ascontiguousarray(l, np.int32) for l in luts]
        pk = Pack(dev)
        i_l = [pk.add(l) for l in ls]
        i_n, i_o = pk.add(np.array([l.size for l in ls], np.int32)), pk.add(np.asarray(offs, np.int64))
        d = pk.ship()
        lp = [d[i] for i in i_l]
        pk2 = Pack(dev)
        i_c, i_lp = pk2.add(np.array([c.data_ptr() for c in cs], np.int64)), pk2.add(
            np.array([t.data_ptr() for t in lp], np.int64))
        d2 = pk2.ship()
        N.check(N.hip().tmog_hip_onehot_pivot(N.ptr(d2[i_c]), N.ptr(d2[i_lp]), N.ptr(d[i_n]), N.ptr(d[i_o]), len(cs),
                                              int(out.shape[0]), N.ptr(out), int(out.shape[1]), N.stream(dev)),
                "onehot_pivot")
        return
    for c, l, o in zip(codes, luts, offs):
        onehot_scatter(out, c, torch.as_tensor(np.asarray(l, np.int64), device=dev), o)


def onehot_scatter(out: torch.Tensor, codes: torch.Tensor, lut: torch.Tensor, off: int) -> None:
    """``out[r, off + lut[codes[r]]] += 1`` (code -1 uses the last lut entry; slot -1 = skip)."""
    n = codes.shape[0]
    if n == 0:
        return
    idx = torch.where(codes >= 0, codes.long(), torch.full_like(codes.long(), lut.numel() - 1))
    slot = lut[idx]
    rows = torch.arange(n, device=codes.device)
    m = slot >= 0
    out.index_put_((rows[m], slot[m] + off), torch.ones(int(m.sum()), dtype=out.dtype, device=out.device),
                   accumulate=True)


def csr_rows_scatter_add(out: torch.Tensor, codes: torch.Tensor, indptr: np.ndarray, idx: np.ndarray,
                         vals: np.ndarray) -> None:
    """For each row r with code c >= 0 add the sparse vector ``c`` (CSR) into ``out[r]``."""
    dev = out.device
    if idx.size == 0:
        return
    ip = torch.as_tensor(indptr, device=dev)
    ix = torch.as_tensor(idx, device=dev)
    vx = torch.as_tensor(vals, dtype=out.dtype, device=dev)
    c = codes.long()
    ok = c >= 0
    rows = torch.arange(codes.shape[0], device=dev)[ok]
    c = c[ok]
    starts = ip[c]
    cnt = ip[c + 1] - starts
    total = int(cnt.sum())
    if total == 0:
        return
    r_rep = torch.repeat_interleave(rows, cnt)
    base = torch.repeat_interleave(starts - (torch.cumsum(cnt, 0) - cnt), cnt)
    g = base + torch.arange(total, device=dev)
    out.index_put_((r_rep, ix[g]), vx[g], accumulate=True)

"""Text / categorical / calendar vectorizer ops.

Device tensors run the HIP kernels of ``csrc/hip/text_kernels.hip``; host tensors run the torch /
numpy reference path, which is the numerics spec the GPU tests compare against. Every writer takes
a 2-D ``out`` that may be a column slice of a wider feature matrix (``big[:, a:b]``): kernels write
through ``out.stride(0)``, so producers fill the combined matrix in place (K1).
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..utils import text as TU
from . import _native as N


def _dev_copy(a: np.ndarray, dev) -> torch.Tensor:
    a = np.ascontiguousarray(a)
    if a.size == 0:
        a = np.zeros(1, a.dtype)
    return torch.from_numpy(a).to(dev)


def _check_out(out: torch.Tensor):
    if out.dim() != 2 or out.stride(1) != 1:
        raise ValueError("vectorizer output must be a row-major 2-D block (unit column stride)")


# ----------------------------------------------------------------------------------------- hashing TF
class HashInput:
    """One hashed feature: ``codes`` maps each row to a distinct value (``None`` = row i is value i),
    ``tokens`` holds each distinct value's terms, ``prefix`` is the feature-name hash prepended as
    ``"<prefix>_<term>"`` (``OPCollectionHashingVectorizer.scala:284-305``) or ``None``."""

    def __init__(self, codes: Optional[torch.Tensor], tokens: TU.TokenBatch, prefix: Optional[int]):
        self.codes, self.tokens, self.prefix = codes, tokens, prefix


def _host_indices(tb: TU.TokenBatch, prefix: Optional[int], num_features: int) -> np.ndarray:
    if tb.n_tokens == 0:
        return np.zeros(0, np.int32)
    data, offs = tb.data, tb.tok_offs
    if prefix is not None:      # "<prefix>_" || token, laid out contiguously for the murmur3 batch
        pre = np.frombuffer(f"{prefix}_".encode(), np.uint8)
        lens = np.diff(tb.tok_offs)
        offs = np.zeros(tb.n_tokens + 1, np.int64)
        np.cumsum(lens + pre.size, out=offs[1:])
        data = np.empty(int(offs[-1]), np.uint8)
        starts = offs[:-1]
        for k in range(pre.size):
            data[starts + k] = pre[k]
        nbytes = int(lens.sum())
        src = np.arange(nbytes) + int(tb.tok_offs[0])
        data[np.repeat(starts + pre.size - tb.tok_offs[:-1], lens) + src] = tb.data[src]
    out = np.empty(tb.n_tokens, np.int32)
    buf = np.ascontiguousarray(data) if data.size else np.zeros(1, np.uint8)
    N.check(N.host().tmog_hash_index_batch(buf.ctypes.data, np.ascontiguousarray(offs).ctypes.data, tb.n_tokens, 42,
                                           num_features, out.ctypes.data), "hash_index_batch")
    return out


def hashed_tf(out: torch.Tensor, inputs: Sequence[HashInput], num_features: int, shared: bool, binary: bool) -> None:
    """Write the hashed term-frequency block of ``inputs`` into ``out`` (``[n, W]``; W = num_features when
    the hash space is shared, else ``len(inputs) * num_features``, feature k at ``k * num_features``)."""
    _check_out(out)
    n, W = out.shape
    need = num_features if shared else num_features * len(inputs)
    if W != need:
        raise ValueError(f"hashed block width {W} != {need}")
    if n == 0:
        return
    if out.device.type == "cuda":
        _hashed_tf_hip(out, inputs, num_features, shared, binary)
        return
    acc = torch.zeros(n, W, dtype=torch.float64)
    for k, h in enumerate(inputs):
        idx = torch.as_tensor(_host_indices(h.tokens, h.prefix, num_features).astype(np.int64)
                              + (0 if shared else k * num_features))
        codes = torch.arange(n, dtype=torch.int64) if h.codes is None else h.codes.to(torch.int64).cpu()
        rp = torch.as_tensor(h.tokens.row_ptr)
        ok = codes >= 0
        rows = torch.arange(n)[ok]
        c = codes[ok]
        cnt = rp[c + 1] - rp[c]
        tot = int(cnt.sum())
        if tot == 0:
            continue
        r_rep = torch.repeat_interleave(rows, cnt)
        t = torch.repeat_interleave(rp[c] - (torch.cumsum(cnt, 0) - cnt), cnt) + torch.arange(tot)
        acc.index_put_((r_rep, idx[t]), torch.ones(tot, dtype=torch.float64), accumulate=True)
    if binary:
        acc.clamp_(max=1.0)
    out.copy_(acc)


def _hashed_tf_hip(out, inputs, num_features, shared, binary):
    dev = out.device
    lib = N.hip()
    st = N.stream(dev)
    keep = []
    triples = []
    for k, h in enumerate(inputs):
        tb = h.tokens
        data = _dev_copy(tb.data, dev)
        toffs = _dev_copy(tb.tok_offs, dev)
        rp = _dev_copy(tb.row_ptr, dev)
        idx = torch.empty(max(tb.n_tokens, 1), dtype=torch.int32, device=dev)
        pre = f"{h.prefix}_".encode() if h.prefix is not None else b""
        pb = np.frombuffer(pre or b"\0", np.uint8).copy()
        N.check(lib.tmog_hip_hash_tokens(N.ptr(data), N.ptr(toffs), tb.n_tokens, pb.ctypes.data, len(pre), 42,
                                         num_features, 0 if shared else k * num_features, N.ptr(idx), st),
                "hash_tokens")
        codes = None
        if h.codes is not None:
            if h.codes.shape[0] != out.shape[0]:
                raise ValueError("hash input codes do not match the output rows")
            if len(tb) == 0:
                continue
            codes = h.codes.to(device=dev, dtype=torch.int32).contiguous()
            if int(codes.max()) >= len(tb):
                raise ValueError("dictionary code out of range of the tokenized values")
        elif len(tb) != out.shape[0]:
            raise ValueError("token lists do not match the output rows")
        keep += [data, toffs, rp, idx, codes]
        triples.append((N.ptr(codes) or 0, N.ptr(rp), N.ptr(idx)))
    if not triples:
        out.zero_()
        return
    assert lib.tmog_hip_hash_feat_bytes() == 24
    tab = torch.as_tensor(np.asarray(triples, np.int64).reshape(-1), device=dev)
    W = out.shape[1]
    if 4 * W * 4 > 64 * 1024:
        out.zero_()
    N.check(lib.tmog_hip_hash_tf_rows(N.ptr(tab), len(triples), out.shape[0], W, int(binary), N.ptr(out),
                                      out.stride(0), 0, st), "hash_tf_rows")
    del keep    # stream-ordered frees: the caching allocator reuses these only after the kernels above


# ------------------------------------------------------------------------------------------ counting
def code_counts(codes: Sequence[torch.Tensor], n_values: Sequence[int]) -> List[np.ndarray]:
    """Per column: counts of each code ``0..n_values-1`` plus the null count (code -1) in the last slot
    (``OpOneHotVectorizer.scala:75-124`` value counts; LDS-privatised HIP histogram on device)."""
    if not codes:
        return []
    dev = codes[0].device
    if dev.type != "cuda":
        out = []
        for c, v in zip(codes, n_values):
            cl = c.to(torch.int64)
            cl = torch.where((cl < 0) | (cl >= v), torch.full_like(cl, v), cl)
            out.append(torch.bincount(cl, minlength=v + 1).numpy().astype(np.int64))
        return out
    cs = [c.to(dtype=torch.int32).contiguous() for c in codes]
    total = sum(v + 1 for v in n_values)
    buf = torch.zeros(total, dtype=torch.int64, device=dev)
    offs = np.concatenate([[0], np.cumsum([v + 1 for v in n_values])[:-1]]).astype(np.int64)
    cptr = torch.as_tensor(np.array([c.data_ptr() for c in cs], np.int64), device=dev)
    optr = torch.as_tensor(np.array([buf.data_ptr() + 8 * int(o) for o in offs], np.int64), device=dev)
    nv = torch.as_tensor(np.asarray(n_values, np.int32), device=dev)
    n = cs[0].shape[0]
    if any(c.shape[0] != n for c in cs):
        raise ValueError("code columns differ in length")
    N.check(N.hip().tmog_hip_code_count(N.ptr(cptr), N.ptr(nv), int(max(n_values)), len(cs), n, N.ptr(optr),
                                        N.stream(dev)), "code_count")
    h = buf.cpu().numpy()
    return [h[o:o + v + 1] for o, v in zip(offs, n_values)]


# ---------------------------------------------------------------------------------------- bucketize
def bucketize_into(out: torch.Tensor, x: torch.Tensor, ok: torch.Tensor, splits: Sequence[float], track_nulls: bool,
                   track_invalid: bool, left_inclusive: bool) -> None:
    """One-hot bucket block (``NumericBucketizer.bucketize:219-265``) written into a zeroed ``out``."""
    _check_out(out)
    n = x.shape[0]
    nb = len(splits) - 1
    width = nb + int(track_invalid) + int(track_nulls)
    if out.shape != (n, width):
        raise ValueError(f"bucket block shape {tuple(out.shape)} != {(n, width)}")
    dev = x.device
    if n == 0:
        return
    s = torch.as_tensor(list(map(float, splits)), dtype=torch.float64, device=dev)
    if dev.type == "cuda":
        xd = x.to(torch.float64).contiguous()
        okd = ok.to(torch.uint8).contiguous()
        bad = torch.full((1,), -1, dtype=torch.int64, device=dev)    # ULLONG_MAX
        N.check(N.hip().tmog_hip_bucketize(N.ptr(xd), N.ptr(okd), n, N.ptr(s), len(splits), int(left_inclusive),
                                           int(track_invalid), int(track_nulls), N.ptr(out), out.stride(0), 0, width,
                                           N.ptr(bad), N.stream(dev)), "bucketize")
        r = int(bad.item())
        if r != -1:
            raise ValueError(f"Numeric value {xd[r].item()} falls outside the bounds of the specified buckets")
        return
    x64 = x.to(torch.float64)
    idx = torch.searchsorted(s, x64, right=left_inclusive) - 1
    invalid = (idx < 0) | (idx >= nb) | ~torch.isfinite(x64)
    if (invalid & ok).any() and not track_invalid:
        bad = x64[ok & invalid][0].item()
        raise ValueError(f"Numeric value {bad} falls outside the bounds of the specified buckets")
    rows = torch.arange(n)
    good = ok & ~invalid
    out[rows[good], idx[good]] = 1.0
    if track_invalid:
        out[rows[ok & invalid], nb] = 1.0
    if track_nulls:
        out[rows[~ok], width - 1] = 1.0


# ------------------------------------------------------------------------------------------- dates
_PERIOD_ID = {"DayOfMonth": 0, "DayOfWeek": 1, "DayOfYear": 2, "HourOfDay": 3, "MonthOfYear": 4, "WeekOfMonth": 5,
              "WeekOfYear": 6}


def date_unit_circle_into(out: torch.Tensor, ms: torch.Tensor, ok: torch.Tensor, period: str) -> None:
    """(cos, sin) of ``period`` for every row into ``out[:, 0:2]`` (``DateToUnitCircleTransformer.scala:77-121``)."""
    from ..utils.dates import TIME_PERIODS, period_values
    _check_out(out)
    lo, hi = TIME_PERIODS[period]
    n = ms.shape[0]
    if out.shape != (n, 2):
        raise ValueError("unit-circle block must be [n, 2]")
    if n == 0:
        return
    dev = ms.device
    if dev.type == "cuda":
        m = ms.to(torch.int64).contiguous()
        o = ok.to(torch.uint8).contiguous()
        N.check(N.hip().tmog_hip_date_unit_circle(N.ptr(m), N.ptr(o), n, _PERIOD_ID[period], 1 if lo == 1 else 0, hi,
                                                  N.ptr(out), out.stride(0), 0, N.stream(dev)), "date_unit_circle")
        return
    val, size = period_values(ms.to(torch.int64), period)
    rad = 2 * np.pi * val.to(torch.float64) / size
    out[:, 0] = torch.where(ok, torch.cos(rad), torch.zeros_like(rad)).to(out.dtype)
    out[:, 1] = torch.where(ok, torch.sin(rad), torch.zeros_like(rad)).to(out.dtype)

"""Numeric raw-column statistics for the RawFeatureFilter (``csrc/hip/rff_kernels.hip``).

``numeric_summary`` -> ``[F, 9]`` float64: count, nulls, min, max, sum, sum^2, sum^3, sum^4, and
sum(label over null rows) (the cross term of the null-indicator / label correlation).
``numeric_hist`` -> ``[F, bins]`` counts with the reference bucketing (``FeatureDistribution.histValues``).
Device columns run on the HIP kernels (pointer arrays, no staging copy); host columns use the torch
reference below, which is the numerics spec the kernels are tested against.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
import torch

from . import _native as N
from .staging import Pack

NSTAT = 9
_DT = {torch.float32: 0, torch.float64: 1, torch.int64: 2, torch.bool: 3, torch.uint8: 3}


def _prep(values: Sequence[torch.Tensor], valids: Sequence[Optional[torch.Tensor]]):
    dev = values[0].device
    keep = []
    vals = []
    oks = []
    dts = []
    for v, ok in zip(values, valids):
        if v.dtype not in _DT:
            v = v.to(torch.float64)
        v = v.contiguous()
        keep.append(v)
        vals.append(v.data_ptr())
        dts.append(_DT[v.dtype])
        if ok is None:
            oks.append(0)
        else:
            o = ok.to(torch.uint8).contiguous()
            keep.append(o)
            oks.append(o.data_ptr())
    pk = Pack(dev)
    i_v, i_o, i_d = pk.add(np.asarray(vals, np.int64)), pk.add(np.asarray(oks, np.int64)), pk.add(np.asarray(dts, np.int32))
    d = pk.ship()
    vp, op, dt = d[i_v], d[i_o], d[i_d]
    return vp, op, dt, keep


def numeric_summary(values: Sequence[torch.Tensor], valids: Sequence[Optional[torch.Tensor]],
                    label: Optional[torch.Tensor] = None) -> torch.Tensor:
    F = len(values)
    if F == 0:
        return torch.zeros(0, NSTAT, dtype=torch.float64)
    dev = values[0].device
    n = int(values[0].shape[0])
    if dev.type == "cuda":
        vp, op, dt, keep = _prep(values, valids)
        out = torch.empty(F, NSTAT, dtype=torch.float64, device=dev)
        lab = None
        ldt = 0
        if label is not None:
            lab = label if label.dtype in _DT else label.to(torch.float64)
            lab = lab.contiguous()
            ldt = _DT[lab.dtype]
        N.check(N.hip().tmog_hip_rff_summary(N.ptr(vp), N.ptr(op), N.ptr(dt), n, F, N.ptr(lab), ldt, N.ptr(out),
                                             N.stream(dev)), "rff_summary")
        del keep
        return out
    rows = []
    yl = None if label is None else label.to(torch.float64)
    for v, ok in zip(values, valids):
        x = v.to(torch.float64)
        m = torch.ones(n, dtype=torch.bool) if ok is None else ok.to(torch.bool)
        xv = x[m]
        c = float(xv.numel())
        rows.append([c, float(n - c), float(xv.min()) if c else float("inf"), float(xv.max()) if c else float("-inf"),
                     float(xv.sum()), float((xv ** 2).sum()), float((xv ** 3).sum()), float((xv ** 4).sum()),
                     float(yl[~m].sum()) if yl is not None else 0.0])
    return torch.tensor(rows, dtype=torch.float64)


def numeric_hist(values: Sequence[torch.Tensor], valids: Sequence[Optional[torch.Tensor]], lo: torch.Tensor,
                 hi: torch.Tensor, bins: int) -> torch.Tensor:
    F = len(values)
    if F == 0:
        return torch.zeros(0, bins, dtype=torch.float64)
    dev = values[0].device
    n = int(values[0].shape[0])
    if dev.type == "cuda" and bins <= 16384:
        vp, op, dt, keep = _prep(values, valids)
        out = torch.zeros(F, bins, dtype=torch.int32, device=dev)
        lo_d = lo.to(device=dev, dtype=torch.float64).contiguous()
        hi_d = hi.to(device=dev, dtype=torch.float64).contiguous()
        N.check(N.hip().tmog_hip_rff_hist(N.ptr(vp), N.ptr(op), N.ptr(dt), n, F, N.ptr(lo_d), N.ptr(hi_d), bins,
                                          N.ptr(out), N.stream(dev)), "rff_hist")
        del keep
        return out.to(torch.float64)
    out = torch.zeros(F, bins, dtype=torch.float64)
    for f, (v, ok) in enumerate(zip(values, valids)):
        x = v.to(torch.float64).cpu()
        if ok is not None:
            x = x[ok.cpu().to(torch.bool)]
        mn, mx = float(lo[f]), float(hi[f])
        if not mn < mx:
            out[f, 0] = float((x == mx).sum())
            out[f, 1] = float((x != mx).sum())
            continue
        step = (mx - mn) / (bins - 2.0)
        splits = torch.tensor([mn + step * b for b in range(bins)], dtype=torch.float64)
        b = torch.searchsorted(splits, x, right=True) - 1          # Left inclusion: [s_i, s_{i+1})
        b = torch.where((x >= splits[0]) & (x < splits[-1]), b, torch.full_like(b, bins - 1))
        out[f] = torch.bincount(b, minlength=bins).to(torch.float64)[:bins]
    return out

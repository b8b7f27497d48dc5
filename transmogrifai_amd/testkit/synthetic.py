"""Synthetic tabular datasets generated directly in device memory.

Used by ``bench.py`` for the headline config (10M-row binary-class tabular, BASELINE.json) and by
tests. The table is built column by column on the target device with a seeded generator, so every
rank of a job produces the identical table without any host round trip (no 10M-row host arrays).

Column mix (defaults): ``n_real`` ``Real`` columns (a few with nulls), ``n_int`` ``Integral`` columns
(small counts), ``n_pick`` ``PickList`` columns (dictionary-coded categories, a few with nulls) and a
``RealNN`` binary label drawn from a logistic model with interactions and a categorical effect, so
that both linear models and trees have signal to find and AuPR is a meaningful quality check.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import List, Tuple

import torch

from ..data.columns import NumericColumn, TextColumn
from ..data.dataset import Dataset
from ..features import types as T
from ..features.builder import FeatureBuilder


def binary_table(n_rows: int, n_real: int = 170, n_int: int = 15, n_pick: int = 15, n_cats: int = 8,
                 null_frac: float = 0.1, n_null_cols: int = 20, seed: int = 7, device="cpu",
                 chunk: int = 1 << 21) -> Tuple[Dataset, object, List[object]]:
    """Return ``(dataset, label_feature, predictor_features)``."""
    dev = torch.device(device)
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    n_inf = min(n_real, 24)
    cols: "OrderedDict[str, object]" = OrderedDict()
    # label model weights
    wg = torch.Generator(device="cpu")
    wg.manual_seed(seed + 1)
    w_real = torch.randn(n_inf, generator=wg, dtype=torch.float32) * 0.6
    w_cat = torch.randn(max(n_pick, 1), n_cats, generator=wg, dtype=torch.float32) * 0.5
    logit = torch.zeros(n_rows, dtype=torch.float32, device=dev)
    reals = []
    for j in range(n_real):
        x = torch.randn(n_rows, generator=g, device=dev, dtype=torch.float32)
        if j % 7 == 3:
            x = torch.exp(0.5 * x)                      # skewed, positive
        if j < n_inf:
            logit += w_real[j].item() * (x if j % 7 != 3 else torch.log(x))
        reals.append(x)
    # a few nonlinear terms only trees capture well
    if n_real >= 4:
        logit += 0.8 * (reals[0] * reals[1] > 0).float() - 0.4
        logit += 0.6 * torch.tanh(2.0 * reals[2]) * (reals[3] > 0.5).float()
    for j, x in enumerate(reals):
        valid = None
        if j < n_null_cols:
            valid = torch.rand(n_rows, generator=g, device=dev) >= null_frac
            x = torch.where(valid, x, torch.zeros_like(x))
        cols[f"real_{j:03d}"] = NumericColumn(T.Real, x.to(torch.float64) if dev.type == "cpu" else x, valid)
    for j in range(n_int):
        lam = 1.0 + (j % 5)
        x = torch.poisson(torch.full((n_rows,), lam, device=dev), generator=g).to(torch.int64)
        if j < 2:
            logit += 0.15 * (x.float() - lam)
        cols[f"int_{j:03d}"] = NumericColumn(T.Integral, x, None)
    for j in range(n_pick):
        # zipf-ish category frequencies
        p = torch.tensor([1.0 / (k + 1) for k in range(n_cats)], device=dev)
        codes = torch.multinomial(p / p.sum(), n_rows, replacement=True, generator=g).to(torch.int32)
        if j < 3:
            logit += w_cat[j].to(dev)[codes.long()]
        if j % 4 == 1:
            nul = torch.rand(n_rows, generator=g, device=dev) < null_frac
            codes = torch.where(nul, torch.full_like(codes, -1), codes)
        cols[f"cat_{j:03d}"] = TextColumn(T.PickList, codes, [f"c{j}_{k}" for k in range(n_cats)])
    u = torch.rand(n_rows, generator=g, device=dev)
    y = (u < torch.sigmoid(logit - 0.7)).to(torch.float64 if dev.type == "cpu" else torch.float32)
    cols["label"] = NumericColumn(T.RealNN, y, None)
    ds = Dataset(cols, None, n_rows)
    label = FeatureBuilder.RealNN("label").as_response()
    preds = []
    for name, c in cols.items():
        if name == "label":
            continue
        preds.append(FeatureBuilder.of(c.ftype, name).as_predictor())
    return ds, label, preds

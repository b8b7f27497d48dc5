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


def _topic_docs(n_docs: int, n_topics: int, n_words: int, seed: int) -> Tuple[List[str], "torch.Tensor"]:
    """``n_docs`` distinct short documents, each written mostly from its topic's word slice."""
    import numpy as np
    r = np.random.default_rng(seed)
    words = np.array([f"w{k:04d}" for k in range(n_words)] + ["the", "and", "of", "a", "to", "in"])
    topic = r.integers(0, n_topics, n_docs)
    lens = r.integers(3, 14, n_docs)
    per = n_words // n_topics
    docs = []
    for d in range(n_docs):
        on = r.random(lens[d]) < 0.55
        w = np.where(on, topic[d] * per + r.integers(0, per, lens[d]), r.integers(0, len(words), lens[d]))
        docs.append(" ".join(words[w]))
    return docs, torch.as_tensor(topic)


def multiclass_text_table(n_rows: int, n_classes: int = 6, n_real: int = 20, n_pick: int = 6, n_text: int = 2,
                          n_docs: int = 200_000, n_cities: int = 300, seed: int = 11,
                          device="cpu") -> Tuple[Dataset, object, List[object]]:
    """BASELINE config 4 shape: multi-class label with numeric, categorical and text columns.

    * ``n_real`` ``Real`` and ``n_pick`` ``PickList`` columns (device generated);
    * one medium-cardinality ``Text`` column (``city``, ``n_cities`` values: SmartText pivots it);
    * ``n_text`` free ``Text`` columns drawn from ``n_docs`` distinct topic documents (cardinality far above
      SmartText's 1000: tokenized and murmur3-hashed); a row of class c picks a document of topic c with
      probability 0.6, so the text carries label signal only through its words.
    """
    dev = torch.device(device)
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    wg = torch.Generator(device="cpu")
    wg.manual_seed(seed + 1)
    cols: "OrderedDict[str, object]" = OrderedDict()
    score = torch.zeros(n_rows, n_classes, device=dev)
    wr = torch.randn(n_real, n_classes, generator=wg) * 0.5
    for j in range(n_real):
        x = torch.randn(n_rows, generator=g, device=dev)
        if j < 8:
            score += x[:, None] * wr[j].to(dev)[None, :]
        valid = (torch.rand(n_rows, generator=g, device=dev) >= 0.1) if j % 5 == 0 else None
        if valid is not None:
            x = torch.where(valid, x, torch.zeros_like(x))
        cols[f"real_{j:03d}"] = NumericColumn(T.Real, x.to(torch.float64) if dev.type == "cpu" else x, valid)
    for j in range(n_pick):
        nc = 12
        codes = torch.randint(0, nc, (n_rows,), generator=g, device=dev, dtype=torch.int32)
        if j < 2:
            score += (torch.randn(nc, n_classes, generator=wg) * 0.6).to(dev)[codes.long()]
        cols[f"cat_{j:03d}"] = TextColumn(T.PickList, codes, [f"k{j}_{k}" for k in range(nc)])
    y = torch.argmax(score + torch.randn(n_rows, n_classes, generator=g, device=dev) * 1.5, dim=1)
    p = torch.tensor([1.0 / (k + 1) ** 0.8 for k in range(n_cities)], device=dev)
    city = torch.multinomial(p / p.sum(), n_rows, replacement=True, generator=g).to(torch.int32)
    cols["city"] = TextColumn(T.Text, city, [f"City {k}" for k in range(n_cities)])
    nd = min(n_docs, max(n_rows // 2, 1))
    for t in range(n_text):
        docs, topic = _topic_docs(nd, n_classes, 3000, seed + 10 + t)
        topic = topic.to(dev)
        order = torch.argsort(topic, stable=True)
        counts = torch.bincount(topic, minlength=n_classes)
        starts = torch.cumsum(counts, 0) - counts
        pick_same = torch.rand(n_rows, generator=g, device=dev) < 0.6
        r_same = starts[y] + (torch.rand(n_rows, generator=g, device=dev) * counts[y]).long().clamp(max=nd - 1)
        r_any = torch.randint(0, nd, (n_rows,), generator=g, device=dev)
        code = torch.where(pick_same, order[r_same.clamp(max=nd - 1)], r_any).to(torch.int32)
        nul = torch.rand(n_rows, generator=g, device=dev) < 0.05
        code = torch.where(nul, torch.full_like(code, -1), code)
        cols[f"text_{t}"] = TextColumn(T.Text, code, docs)
    cols["label"] = NumericColumn(T.RealNN, y.to(torch.float64 if dev.type == "cpu" else torch.float32), None)
    ds = Dataset(cols, None, n_rows)
    label = FeatureBuilder.RealNN("label").as_response()
    preds = [FeatureBuilder.of(c.ftype, name).as_predictor() for name, c in cols.items() if name != "label"]
    return ds, label, preds


def regression_table(n_rows: int, n_real: int = 30, n_int: int = 5, n_pick: int = 5, seed: int = 13,
                     device="cpu") -> Tuple[Dataset, object, List[object]]:
    """BASELINE config 5 shape: a real-valued label with a linear + nonlinear signal over numeric and
    categorical columns (device generated, chunk free)."""
    dev = torch.device(device)
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    wg = torch.Generator(device="cpu")
    wg.manual_seed(seed + 1)
    cols: "OrderedDict[str, object]" = OrderedDict()
    w = torch.randn(n_real, generator=wg)
    y = torch.zeros(n_rows, device=dev)
    xs = []
    for j in range(n_real):
        x = torch.randn(n_rows, generator=g, device=dev)
        if j < 12:
            y += float(w[j]) * x
        xs.append(x)
        valid = (torch.rand(n_rows, generator=g, device=dev) >= 0.1) if j % 6 == 0 else None
        if valid is not None:
            x = torch.where(valid, x, torch.zeros_like(x))
        cols[f"real_{j:03d}"] = NumericColumn(T.Real, x.to(torch.float64) if dev.type == "cpu" else x, valid)
    if n_real >= 3:
        y += 2.0 * torch.sin(xs[0] * xs[1]) + (xs[2] > 0.5).float() * 1.5
    for j in range(n_int):
        x = torch.poisson(torch.full((n_rows,), 2.0 + j, device=dev), generator=g).to(torch.int64)
        if j == 0:
            y += 0.3 * x.float()
        cols[f"int_{j:03d}"] = NumericColumn(T.Integral, x, None)
    for j in range(n_pick):
        codes = torch.randint(0, 10, (n_rows,), generator=g, device=dev, dtype=torch.int32)
        if j == 0:
            y += (torch.randn(10, generator=wg) * 1.0).to(dev)[codes.long()]
        cols[f"cat_{j:03d}"] = TextColumn(T.PickList, codes, [f"r{j}_{k}" for k in range(10)])
    y += torch.randn(n_rows, generator=g, device=dev)
    cols["label"] = NumericColumn(T.RealNN, y.to(torch.float64) if dev.type == "cpu" else y, None)
    ds = Dataset(cols, None, n_rows)
    label = FeatureBuilder.RealNN("label").as_response()
    preds = [FeatureBuilder.of(c.ftype, name).as_predictor() for name, c in cols.items() if name != "label"]
    return ds, label, preds

"""Label-aware numeric bucketizers.

Reference: ``DecisionTreeNumericBucketizer`` (``core/.../impl/feature/DecisionTreeNumericBucketizer.scala:60-300``:
one depth-5 / 32-bin / gini decision tree per numeric feature over its non-missing values, bucket
edges = the tree's split thresholds, right-inclusive buckets + null indicator) and the map variant
(``DecisionTreeNumericMapBucketizer.scala:56-170``). The 1-D tree runs on the same batched histogram
engine as the model-selector forests.
"""
from __future__ import annotations

import math
from typing import List

import numpy as np
import torch

from ...config import vector_dtype
from ...data.columns import VectorColumn
from ...data.vector_metadata import FeatureHistory, OpVectorMetadata
from ...features import types as T
from ...models import tree_engine as TE
from ...models.binning import find_splits, quantize
from ..base import BinaryEstimator, BinaryTransformer, register_stage
from .math_stages import bucket_labels, bucket_metadata, bucketize_column, check_splits


def tree_splits(x: torch.Tensor, y: torch.Tensor, max_depth=5, max_bins=32, min_instances=1, min_info_gain=0.01,
                impurity="gini") -> list:
    """Sorted distinct thresholds of a single-feature classification tree (grown by the batched tree
    engine; the reference for :func:`tree_splits_dp`)."""
    if x.numel() == 0:
        return []
    X = x.to(torch.float64)[:, None]
    spec = find_splits(X, max_bins)
    Xb = quantize(X, spec)
    yl = y.to(torch.float64)
    uniq, yi = torch.unique(yl, return_inverse=True)
    K = max(2, uniq.numel())
    job = TE.TreeJob(0, TE.TreeParams(max_depth=max_depth, min_instances=min_instances,
                                      min_info_gain=min_info_gain), torch.arange(x.numel(), device=x.device))
    f = TE.grow_forest(Xb, spec.n_bins, [job], mode=TE.MODE_CLS, kind=TE.KINDS[impurity], n_classes=K,
                       y=yi.to(torch.float32), B=max_bins)
    internal = f.nodes[:, 2] >= 0
    bins = sorted(set(int(b) for b in f.nodes[internal, 1]))
    return [float(spec.thresholds[0, b]) for b in bins]


def _impurity(st: np.ndarray, kind: str):
    """(impurity, count) with the tree engine's operation order (ops/csrc/host/tree_cpu.cpp impurity)."""
    n = 0.0
    for v in st:
        n += float(v)
    if n <= 0:
        return 0.0, n
    imp = 1.0 if kind == "gini" else 0.0
    for v in st:
        p = float(v) / n
        if kind == "gini":
            imp -= p * p
        elif p > 0:
            imp -= p * math.log2(p)
    return imp, n


def table_tree_splits(table: np.ndarray, max_depth=5, min_instances=1.0, min_info_gain=0.01,
                      impurity="gini") -> List[int]:
    """Split bins of a single-feature classification tree grown from its ``(bin, class)`` count table.

    On one feature every node is a contiguous bin range and its statistics are sums of table rows, so the
    whole tree follows from the ``B x K`` table: the same candidates, gains (engine operation order,
    float64) and tie-breaking (first best bin) as the histogram engine growing it from the rows. A
    row-sharded fit all-reduces the table (a few hundred bytes) instead of gathering the column."""
    B = table.shape[0]
    cum = np.vstack([np.zeros((1, table.shape[1]), np.int64), np.cumsum(table.astype(np.int64), 0)])
    out = set()
    level = [(0, B - 1)]
    for depth in range(max_depth + 1):
        nxt = []
        for lo, hi in level:
            tot = cum[hi + 1] - cum[lo]
            tcount = float(tot.sum())
            if not (depth < max_depth and tcount >= 2 and tcount >= 2 * min_instances - 1e-9):
                continue
            pimp, tc = _impurity(tot, impurity)
            best, bb = -math.inf, -1
            for b in range(lo, hi):
                left = cum[b + 1] - cum[lo]
                right = tot - left
                li, lc = _impurity(left, impurity)
                ri, rc = _impurity(right, impurity)
                if lc < min_instances or rc < min_instances or lc <= 0 or rc <= 0:
                    continue
                gain = pimp - (lc / tc) * li - (rc / tc) * ri
                if gain < min_info_gain:
                    continue
                if gain > best:
                    best, bb = gain, b
            if bb >= 0 and np.float32(best) > 0.0:
                out.add(bb)
                nxt += [(lo, bb), (bb + 1, hi)]
        level = nxt
        if not level:
            break
    return sorted(out)


def _global_sample(x: torch.Tensor, max_bins: int) -> torch.Tensor:
    """The rows of ``x`` (concatenated over the ranks in rank order) that ``find_splits`` samples: each rank
    contributes its part of the global sample, so thresholds equal the single-process ones."""
    from ...parallel import dp
    from ...parallel import dist as D
    from ...models.binning import sample_rows
    n_loc = int(x.numel())
    counts = dp.objects(n_loc)
    me = D.rank() if dp.active() else 0
    off, n = sum(counts[:me]), sum(counts)
    idx = sample_rows(n, max_bins)
    mine = idx[(idx >= off) & (idx < off + n_loc)] - off
    part = x.detach().to("cpu", torch.float64)[mine].numpy()
    parts = dp.objects(part)
    return torch.as_tensor(np.concatenate(parts) if parts else part, dtype=torch.float64)


def tree_splits_dp(x: torch.Tensor, y: torch.Tensor, max_depth=5, max_bins=32, min_instances=1,
                   min_info_gain=0.01, impurity="gini") -> list:
    """:func:`tree_splits` over every rank's rows with no column gather: the global binning sample, global
    label classes, and one all-reduced ``(bin, class)`` count table."""
    from ...parallel import dp
    n = dp.count(int(x.numel()))
    if n == 0:
        return []
    samp = _global_sample(x, max_bins)
    spec = find_splits(samp[:, None], max_bins)
    uniq = dp.unique_values(y.to(torch.float64))
    K = max(2, int(uniq.numel()))
    B = int(spec.n_bins[0])
    if x.numel():
        bins = quantize(x.to(torch.float64)[:, None], spec)[:, 0].to(torch.int64)
        yi = torch.searchsorted(uniq.to(y.device), y.to(torch.float64).contiguous())
        tab = torch.bincount(bins * K + yi, minlength=B * K).to(torch.float64)
    else:
        tab = torch.zeros(B * K, dtype=torch.float64, device=x.device)
    tab = dp.sum_([tab])[0].reshape(B, K).cpu().numpy().round().astype(np.int64)
    split_bins = table_tree_splits(tab, max_depth, float(min_instances), float(min_info_gain), impurity)
    return [float(spec.thresholds[0, b]) for b in split_bins]


@register_stage
class DecisionTreeNumericBucketizerModel(BinaryTransformer):
    operation_name = "dtNumBuck"
    output_type = T.OPVector
    allow_label_as_input = True

    def __init__(self, should_split=False, splits=None, track_nulls=True, track_invalid=False, uid=None, **kw):
        super().__init__(None, uid=uid, **kw)
        self.should_split = should_split
        self.splits = list(splits or [])
        self.track_nulls = track_nulls
        self.track_invalid = track_invalid

    def transform_columns(self, label, a, ds=None):
        x = a.values.to(torch.float64)
        ok = a.valid
        dtype = vector_dtype(x.device)
        if self.should_split:
            out = bucketize_column(x, ok, self.splits, self.track_nulls, self.track_invalid, "Right", dtype)
        elif self.track_nulls:
            out = (~ok).to(dtype)[:, None]
        else:
            out = torch.zeros(x.shape[0], 0, dtype=dtype, device=x.device)
        return VectorColumn(out, self.metadata.get("vector_metadata"))

    def ctor_args(self):
        return {"shouldSplit": self.should_split, "splits": self.splits, "trackNulls": self.track_nulls,
                "trackInvalid": self.track_invalid}

    def load_ctor_args(self, a):
        self.should_split, self.splits = a["shouldSplit"], list(a["splits"])
        self.track_nulls, self.track_invalid = a["trackNulls"], a["trackInvalid"]


@register_stage
class DecisionTreeNumericBucketizer(BinaryEstimator):
    operation_name = "dtNumBuck"
    output_type = T.OPVector
    allow_label_as_input = True
    _defaults = {"max_depth": 5, "max_bins": 32, "min_instances_per_node": 1, "min_info_gain": 0.01,
                 "impurity": "gini", "track_nulls": True, "track_invalid": False}
    dp_aware = True     # global binning sample + one all-reduced (bin, class) table (tree_splits_dp)

    def fit_columns(self, label, a, ds=None):
        from ...parallel import dp
        p = self.params
        ok = a.valid
        if dp.count(int(ok.shape[0])) == 0:       # DecisionTreeNumericBucketizer.scala:77
            raise ValueError("requirement failed: Dataset is empty, buckets cannot be computed.")
        x = a.values.to(torch.float64)[ok]
        y = label.values[ok]
        sp = tree_splits_dp(x, y, p["max_depth"], p["max_bins"], p["min_instances_per_node"], p["min_info_gain"],
                            p["impurity"])
        splits = [float("-inf")] + sp + [float("inf")]
        should = check_splits(splits)
        final = splits if should else []
        labels = bucket_labels(final, "Right") if should else []
        t = self.get_transient_features()[1]
        cols = bucket_metadata(t, labels, p["track_nulls"], should and p["track_invalid"])
        self.metadata["vector_metadata"] = OpVectorMetadata(
            self.get_output_feature_name(), cols,
            {t.name: FeatureHistory(tuple(t.origin_features), tuple(t.stages) + (self.stage_name(),))})
        return DecisionTreeNumericBucketizerModel(should, final, p["track_nulls"], should and p["track_invalid"])


# ------------------------------------------------------------------------------------ map variant
@register_stage
class DecisionTreeNumericMapBucketizerModel(BinaryTransformer):
    operation_name = "dtNumMapBuck"
    output_type = T.OPVector
    allow_label_as_input = True

    def __init__(self, keys=None, splits=None, track_nulls=True, track_invalid=False, clean_keys=False, uid=None,
                 **kw):
        super().__init__(None, uid=uid, **kw)
        self.keys = list(keys or [])
        self.splits = [list(s) for s in (splits or [])]
        self.track_nulls = track_nulls
        self.track_invalid = track_invalid
        self.clean_keys = clean_keys

    def transform_columns(self, label, m, ds=None):
        from ...config import default_device
        from .maps import map_coo
        dev = default_device()
        coo = map_coo(m, "real", self.clean_keys, dev)
        dtype = vector_dtype(dev)
        last = coo.last_entry(self.keys)
        blocks = []
        for j, sp in enumerate(self.splits):
            e = last[:, j]
            ok = e >= 0
            x = coo.num[e.clamp_min(0)] if coo.nnz else torch.zeros(coo.n, dtype=torch.float64, device=dev)
            if sp:
                blocks.append(bucketize_column(x, ok, sp, self.track_nulls, self.track_invalid, "Right", dtype))
            elif self.track_nulls:
                blocks.append((~ok).to(dtype)[:, None])
        out = torch.cat(blocks, 1) if blocks else torch.zeros(coo.n, 0, dtype=dtype, device=dev)
        return VectorColumn(out, self.metadata.get("vector_metadata"))

    def ctor_args(self):
        return {"keys": self.keys, "splits": self.splits, "trackNulls": self.track_nulls,
                "trackInvalid": self.track_invalid, "shouldCleanKeys": self.clean_keys}

    def load_ctor_args(self, a):
        self.keys, self.splits, self.track_nulls = list(a["keys"]), [list(s) for s in a["splits"]], a["trackNulls"]
        self.track_invalid = bool(a.get("trackInvalid", False))
        self.clean_keys = bool(a.get("shouldCleanKeys", False))


@register_stage
class DecisionTreeNumericMapBucketizer(BinaryEstimator):
    """One label-aware tree per numeric map key (``DecisionTreeNumericMapBucketizer.scala:56-170``)."""
    operation_name = "dtNumMapBuck"
    output_type = T.OPVector
    allow_label_as_input = True
    # cleanKeys / allow / block lists: MapPivotParams + Transmogrifier.scala filterKeys
    _defaults = dict(DecisionTreeNumericBucketizer._defaults, clean_keys=False, allow_keys=None, block_keys=None)
    dp_aware = True     # key union + per-key tree_splits_dp

    def fit_columns(self, label, m, ds=None):
        from ...data.vector_metadata import OpVectorColumnMetadata, NULL_STRING, OTHER_STRING
        p = self.params
        from ...config import default_device
        from .maps import _filter_keys, _global_keys, map_coo
        dev = default_device()
        coo = map_coo(m, "real", p["clean_keys"], dev)
        y_all = label.values.to(device=dev, dtype=torch.float64)
        used = torch.unique(coo.key).cpu().numpy() if coo.nnz else np.zeros(0, np.int64)
        keys = _filter_keys(_global_keys([[coo.keys[int(i)] for i in used]])[0], p["allow_keys"], p["block_keys"],
                            p["clean_keys"])
        last = coo.last_entry(keys)
        t = self.get_transient_features()[1]
        splits, cols = [], []
        for j, k in enumerate(keys):
            e = last[:, j]
            rows = torch.nonzero(e >= 0).reshape(-1)
            x = coo.num[e[rows]] if coo.nnz else torch.zeros(0, dtype=torch.float64, device=dev)
            sp = tree_splits_dp(x, y_all[rows], p["max_depth"], p["max_bins"], p["min_instances_per_node"],
                                p["min_info_gain"], p["impurity"])
            full = [float("-inf")] + sp + [float("inf")]
            ok = check_splits(full)
            splits.append(full if ok else [])
            if ok:
                for lab in bucket_labels(full, "Right"):
                    cols.append(OpVectorColumnMetadata((t.name,), (t.type_name,), k, lab))
                if p["track_invalid"]:
                    cols.append(OpVectorColumnMetadata((t.name,), (t.type_name,), k, OTHER_STRING))
            if p["track_nulls"]:
                cols.append(OpVectorColumnMetadata((t.name,), (t.type_name,), k, NULL_STRING))
        self.metadata["vector_metadata"] = OpVectorMetadata(
            self.get_output_feature_name(), cols,
            {t.name: FeatureHistory(tuple(t.origin_features), tuple(t.stages) + (self.stage_name(),))})
        return DecisionTreeNumericMapBucketizerModel(keys, splits, p["track_nulls"], p["track_invalid"],
                                                     p["clean_keys"])

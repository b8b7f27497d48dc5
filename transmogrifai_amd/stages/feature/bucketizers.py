"""Label-aware numeric bucketizers.

Reference: ``DecisionTreeNumericBucketizer`` (``core/.../impl/feature/DecisionTreeNumericBucketizer.scala:60-300``:
one depth-5 / 32-bin / gini decision tree per numeric feature over its non-missing values, bucket
edges = the tree's split thresholds, right-inclusive buckets + null indicator) and the map variant
(``DecisionTreeNumericMapBucketizer.scala:56-170``). The 1-D tree runs on the same batched histogram
engine as the model-selector forests.
"""
from __future__ import annotations

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
    """Sorted distinct thresholds of a single-feature classification tree."""
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

    def fit_columns(self, label, a, ds=None):
        p = self.params
        ok = a.valid
        x = a.values.to(torch.float64)[ok]
        y = label.values[ok]
        sp = tree_splits(x, y, p["max_depth"], p["max_bins"], p["min_instances_per_node"], p["min_info_gain"],
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

    def __init__(self, keys=None, splits=None, track_nulls=True, uid=None, **kw):
        super().__init__(None, uid=uid, **kw)
        self.keys = list(keys or [])
        self.splits = [list(s) for s in (splits or [])]
        self.track_nulls = track_nulls

    def transform_columns(self, label, m, ds=None):
        vals = m.to_list()
        dtype = vector_dtype(torch.device("cpu"))
        blocks = []
        for k, sp in zip(self.keys, self.splits):
            x = torch.as_tensor([float(r[k]) if (r and r.get(k) is not None) else 0.0 for r in vals],
                                dtype=torch.float64)
            ok = torch.as_tensor([bool(r) and r.get(k) is not None for r in vals], dtype=torch.bool)
            if sp:
                blocks.append(bucketize_column(x, ok, sp, self.track_nulls, False, "Right", dtype))
            elif self.track_nulls:
                blocks.append((~ok).to(dtype)[:, None])
        out = torch.cat(blocks, 1) if blocks else torch.zeros(len(vals), 0, dtype=dtype)
        return VectorColumn(out, self.metadata.get("vector_metadata"))

    def ctor_args(self):
        return {"keys": self.keys, "splits": self.splits, "trackNulls": self.track_nulls}

    def load_ctor_args(self, a):
        self.keys, self.splits, self.track_nulls = list(a["keys"]), [list(s) for s in a["splits"]], a["trackNulls"]


@register_stage
class DecisionTreeNumericMapBucketizer(BinaryEstimator):
    """One label-aware tree per numeric map key (``DecisionTreeNumericMapBucketizer.scala:56-170``)."""
    operation_name = "dtNumMapBuck"
    output_type = T.OPVector
    allow_label_as_input = True
    _defaults = dict(DecisionTreeNumericBucketizer._defaults)

    def fit_columns(self, label, m, ds=None):
        from ...data.vector_metadata import OpVectorColumnMetadata, NULL_STRING
        p = self.params
        vals = m.to_list()
        y_all = label.values.to(torch.float64).cpu()
        keys = sorted({k for r in vals for k, v in (r or {}).items() if v is not None})
        t = self.get_transient_features()[1]
        splits, cols = [], []
        for k in keys:
            rows = [i for i, r in enumerate(vals) if r and r.get(k) is not None]
            x = torch.as_tensor([float(vals[i][k]) for i in rows], dtype=torch.float64)
            sp = tree_splits(x, y_all[rows], p["max_depth"], p["max_bins"], p["min_instances_per_node"],
                             p["min_info_gain"], p["impurity"])
            full = [float("-inf")] + sp + [float("inf")]
            ok = check_splits(full)
            splits.append(full if ok else [])
            if ok:
                for lab in bucket_labels(full, "Right"):
                    cols.append(OpVectorColumnMetadata((t.name,), (t.type_name,), k, lab))
            if p["track_nulls"]:
                cols.append(OpVectorColumnMetadata((t.name,), (t.type_name,), k, NULL_STRING))
        self.metadata["vector_metadata"] = OpVectorMetadata(
            self.get_output_feature_name(), cols,
            {t.name: FeatureHistory(tuple(t.origin_features), tuple(t.stages) + (self.stage_name(),))})
        return DecisionTreeNumericMapBucketizerModel(keys, splits, p["track_nulls"])

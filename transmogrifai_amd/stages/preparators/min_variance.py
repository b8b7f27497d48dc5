"""MinVarianceFilter (``core/.../impl/preparators/MinVarianceFilter.scala:58-159``): label-free removal of
near-constant vector columns using one column-moment pass (K14)."""
from __future__ import annotations

import torch

from ...data.columns import VectorColumn
from ...features import types as T
from ...ops import stats as ST
from ..base import OpTransformer, UnaryEstimator, register_stage


@register_stage
class MinVarianceFilterModel(OpTransformer):
    operation_name = "minVarianceFilter"
    output_type = T.OPVector
    arity = 1

    def __init__(self, indices_to_keep=None, remove_bad_features=True, uid=None, **kw):
        super().__init__(uid=uid, **kw)
        self.indices_to_keep = list(indices_to_keep or [])
        self.remove_bad_features = remove_bad_features

    def transform_columns(self, v, ds=None):
        if not self.remove_bad_features:
            return VectorColumn(v.values, v.metadata)
        idx = torch.as_tensor(self.indices_to_keep, dtype=torch.long, device=v.values.device)
        return VectorColumn(v.values.index_select(1, idx), self.metadata.get("vector_metadata"))

    def ctor_args(self):
        return {"indicesToKeep": self.indices_to_keep, "removeBadFeatures": self.remove_bad_features}

    def load_ctor_args(self, a):
        self.indices_to_keep, self.remove_bad_features = list(a["indicesToKeep"]), a["removeBadFeatures"]


@register_stage
class MinVarianceFilter(UnaryEstimator):
    operation_name = "minVarianceFilter"
    output_type = T.OPVector
    _defaults = {"min_variance": 1e-5, "remove_bad_features": True}

    def fit_columns(self, v, ds=None):
        cs = ST.col_stats(v.values.contiguous())
        var = cs["variance"].cpu().numpy()
        keep = [i for i in range(len(var)) if var[i] > self.params["min_variance"]]
        meta = v.metadata
        if meta is not None:
            self.metadata["vector_metadata"] = meta.select(keep if self.params["remove_bad_features"]
                                                           else range(meta.size), self.get_output_feature_name())
        self.metadata["summary"] = {"dropped": [meta.columns[i].make_col_name() for i in range(len(var))
                                                if i not in set(keep)] if meta else [],
                                    "featuresStatistics": {"count": cs["count"], "mean": cs["mean"].tolist(),
                                                           "variance": cs["variance"].tolist(),
                                                           "min": cs["min"].tolist(), "max": cs["max"].tolist()}}
        return MinVarianceFilterModel(keep, self.params["remove_bad_features"])

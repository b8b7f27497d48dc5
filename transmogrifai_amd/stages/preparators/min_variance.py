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
            return VectorColumn(v.values, self.metadata.get("vector_metadata", v.metadata))
        idx = torch.as_tensor(self.indices_to_keep, dtype=torch.long, device=v.values.device)
        return VectorColumn(v.values.index_select(1, idx), self.metadata.get("vector_metadata"))

    def ctor_args(self):
        return {"indicesToKeep": self.indices_to_keep, "removeBadFeatures": self.remove_bad_features}

    def load_ctor_args(self, a):
        self.indices_to_keep, self.remove_bad_features = list(a["indicesToKeep"]), a["removeBadFeatures"]


@register_stage
class MinVarianceFilter(UnaryEstimator):
    """Drop vector columns whose variance is at or below ``min_variance`` (``MinVarianceFilter.scala:84-140``):
    the input needs its vector metadata and at least one row; with ``remove_bad_features`` off nothing is
    dropped; the summary names every input column, the dropped ones and the column statistics."""
    operation_name = "minVarianceFilter"
    output_type = T.OPVector
    _defaults = {"min_variance": 1e-5, "remove_bad_features": False}     # MinVarianceFilter.MinVariance / ...

    def fit_columns(self, v, ds=None):
        X = v.values
        if X.shape[0] == 0:
            raise ValueError("requirement failed: Sample size cannot be zero")
        if X.shape[1] == 0:
            raise ValueError("requirement failed: Feature vector passed in is empty, check your vectorizers")
        meta = v.metadata
        if meta is None:
            raise ValueError("Vector input metadata is malformed: no vector metadata on the input feature")
        if meta.size != X.shape[1]:
            raise ValueError(f"requirement failed: Number of columns in vector metadata ({meta.size}) did not match "
                             f"number of columns in data({X.shape[1]}), check your vectorizers")
        cs = ST.col_stats(X.contiguous())
        var = cs["variance"].cpu().numpy()
        remove = bool(self.params["remove_bad_features"])
        drop = {i for i in range(len(var)) if var[i] <= self.params["min_variance"]} if remove else set()
        keep = [i for i in range(len(var)) if i not in drop]
        names = [c.make_col_name() for c in meta.columns]
        self.metadata["vector_metadata"] = meta.select(keep, self.get_output_feature_name())
        self.metadata["summary"] = {"dropped": [names[i] for i in sorted(drop)], "names": names,
                                    "featuresStatistics": {"count": cs["count"], "mean": cs["mean"].tolist(),
                                                           "variance": cs["variance"].tolist(),
                                                           "min": cs["min"].tolist(), "max": cs["max"].tolist()}}
        if not keep:
            raise ValueError("requirement failed: The minimum variance filter has dropped all of your features, "
                             "check your input data or your threshold")
        return MinVarianceFilterModel(keep, remove)

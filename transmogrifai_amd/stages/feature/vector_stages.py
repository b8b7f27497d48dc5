"""Vector-level transformers (``DropIndicesByTransformer``, ``RichVectorFeature.scala:57-167``)."""
from __future__ import annotations

import torch

from ...data.columns import VectorColumn
from ...features import types as T
from ..base import OpTransformer, register_stage


@register_stage
class DropIndicesByTransformer(OpTransformer):
    """Drop vector columns whose metadata matches a predicate."""
    operation_name = "dropIndicesBy"
    output_type = T.OPVector
    arity = 1

    def __init__(self, match_fn=None, uid=None, **kw):
        super().__init__(uid=uid, **kw)
        self.match_fn = match_fn
        self.keep = None

    def transform_columns(self, v, ds=None):
        meta = v.metadata
        if self.keep is None:
            self.keep = [c.index for c in meta.columns if not self.match_fn(c)]
            self.metadata["vector_metadata"] = meta.select(self.keep, self.get_output_feature_name())
        idx = torch.as_tensor(self.keep, dtype=torch.long, device=v.values.device)
        return VectorColumn(v.values.index_select(1, idx), self.metadata["vector_metadata"])

    def ctor_args(self):
        return {"keep": self.keep}

    def load_ctor_args(self, a):
        self.keep = a["keep"]

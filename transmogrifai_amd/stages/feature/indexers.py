"""String indexing (``OpStringIndexerNoFilter.scala:48-80``, ``OpIndexToStringNoFilter``)."""
from __future__ import annotations

from collections import Counter

import numpy as np
import torch

from ...data.columns import NumericColumn, TextColumn
from ...features import types as T
from ..base import UnaryEstimator, UnaryTransformer, register_stage


@register_stage
class OpStringIndexerNoFilterModel(UnaryTransformer):
    operation_name = "str2idx"
    output_type = T.RealNN

    def __init__(self, labels=None, unseen_name="UnseenLabel", uid=None, **kw):
        super().__init__(None, uid=uid, **kw)
        self.labels = list(labels or [])
        self.unseen_name = unseen_name

    def transform_columns(self, c, ds=None):
        idx = {v: i for i, v in enumerate(self.labels)}
        unseen = float(len(self.labels))
        if isinstance(c, TextColumn):
            lut = np.array([idx.get(s, unseen) for s in c.vocab] + [unseen], dtype=np.float64)
            codes = torch.where(c.codes >= 0, c.codes.long(), torch.full_like(c.codes.long(), len(c.vocab)))
            vals = torch.as_tensor(lut, device=c.codes.device)[codes]
            return NumericColumn(T.RealNN, vals, torch.ones_like(codes, dtype=torch.bool))
        vals = [idx.get(v, unseen) if v is not None else unseen for v in c.to_list()]
        return NumericColumn.from_values(T.RealNN, vals)

    def ctor_args(self):
        return {"labels": self.labels, "unseenName": self.unseen_name}

    def load_ctor_args(self, a):
        self.labels, self.unseen_name = list(a["labels"]), a["unseenName"]


@register_stage
class OpStringIndexerNoFilter(UnaryEstimator):
    """Index strings by descending frequency (ties by value); unseen / null -> last index."""
    operation_name = "str2idx"
    output_type = T.RealNN
    _defaults = {"unseen_name": "UnseenLabel"}

    dp_aware = True     # value counts merged over the ranks (one object all-gather)

    def fit_columns(self, c, ds=None):
        from ...parallel import dp
        if isinstance(c, TextColumn):
            from ...ops.text import code_counts
            n = code_counts([c.codes], [len(c.vocab)])[0][:-1] if c.vocab else []
            cnt = Counter({v: int(k) for v, k in zip(c.vocab, n) if k})
        else:
            cnt = Counter(v for v in c.to_list() if v is not None)
        cnt = dp.merge_counters([cnt])[0]
        labels = [v for v, _ in sorted(cnt.items(), key=lambda kv: (-kv[1], kv[0]))]
        self.metadata["labels"] = labels + [self.params["unseen_name"]]
        return OpStringIndexerNoFilterModel(labels, self.params["unseen_name"])


@register_stage
class OpIndexToStringNoFilter(UnaryTransformer):
    operation_name = "idx2str"
    output_type = T.Text
    _defaults = {"labels": [], "unseen_name": "UnseenIndex"}

    def _labels(self):
        """Given labels, else the fitted string indexer's labels from the input's origin stage metadata
        (``OpIndexToStringNoFilter``: "if not provided or empty, metadata from input feature is used")."""
        labels = list(self.params["labels"] or [])
        if not labels and self._inputs:
            st = self._inputs[0].origin_stage
            md = getattr(st, "metadata", {}) or {}
            labels = list(md.get("labels") or [])
            if labels and isinstance(st, OpStringIndexerNoFilter):
                labels = labels[:-1]              # the indexer's unseen label is not an index target
            if not labels:
                labels = list(getattr(st, "labels", []) or [])
        return labels

    def transform_fn(self, v):
        labels = self._labels()
        if v is None:
            return self.params["unseen_name"]
        i = int(v)
        return labels[i] if 0 <= i < len(labels) else self.params["unseen_name"]


@register_stage
class OpIndexToString(OpIndexToStringNoFilter):
    """Spark ``IndexToString``: an index without a label is an error (handleInvalid = Error)."""
    operation_name = "idx2strStrict"

    def transform_fn(self, v):
        labels = self._labels()
        if v is None:
            raise ValueError("OpIndexToString: null index")
        i = int(v)
        if not 0 <= i < len(labels):
            raise ValueError(f"OpIndexToString: index {i} has no label (labels: {len(labels)})")
        return labels[i]

"""Generic, serializable transformers of the stage catalog.

Reference files (``core/.../stages/impl/feature/``): ``AliasTransformer.scala``, ``ExistsTransformer.scala``,
``FilterTransformer.scala``, ``ReplaceTransformer.scala``, ``ToOccurTransformer.scala``,
``SubstringTransformer.scala``, ``JaccardSimilarity.scala``, ``NGramSimilarity.scala`` (Lucene
``NGramDistance``), ``TimePeriod{,List,Map}Transformer.scala``, ``MultiLabelJoiner.scala``
(``TopNLabelJoiner`` / ``TopNLabelProbMap``), ``FilterMap.scala``, ``OPCollectionTransformer.scala``,
``EmailToPickListMapTransformer.scala`` / ``UrlMapToPickListMapTransformer.scala`` and
``preparators/PredictionDeIndexer.scala``.

User functions (``exists`` / ``filter`` predicates, collection maps) are stored by importable name
(``module.qualname``) in the checkpoint so a module-level function survives a save/load, the analogue
of the reference's reflectively re-instantiated function classes.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, Optional

import numpy as np
import torch

from ...data.columns import NumericColumn, ObjectColumn, TextColumn, column_from_values
from ...features import types as T
from ...utils.text import clean_string, email_domain, url_domain
from ..base import BinaryTransformer, UnaryEstimator, UnaryTransformer, register_stage
from ..generator import _fn_name, load_extract_fn, require_function


def _v(x):
    return x.value if isinstance(x, T.FeatureType) else x


class _FnStage(UnaryTransformer):
    """Unary stage whose behaviour is a user function saved by importable name."""

    def __init__(self, fn: Optional[Callable] = None, uid=None, **kw):
        super().__init__(fn, uid=uid, **kw)
        if fn is not None:
            _fn_name(fn)                 # registers module-level functions for checkpoint reloads

    def ctor_args(self):
        return {"fn": _fn_name(self.fn)}

    def load_ctor_args(self, a):
        self.fn = load_extract_fn(a.get("fn"))


@register_stage
class AliasTransformer(UnaryTransformer):
    """Identity with a user-chosen output name (``AliasTransformer.scala``)."""
    operation_name = "alias"

    def __init__(self, name: Optional[str] = None, uid=None, **kw):
        super().__init__(None, uid=uid, **kw)
        self.alias_name = name

    def set_input(self, *features):
        super().set_input(*features)
        self.output_type = self._inputs[0].wtype
        if self.alias_name:
            self._output_name = self.alias_name
        return self

    def transform_fn(self, v):
        return v

    def transform_columns(self, *cols, ds=None):
        return cols[0]

    def ctor_args(self):
        return {"name": self.alias_name}

    def load_ctor_args(self, a):
        self.alias_name = a.get("name")


@register_stage
class ExistsTransformer(_FnStage):
    operation_name = "exists"
    output_type = T.Binary

    def transform_fn(self, v):
        return bool(self.fn(v))


@register_stage
class FilterTransformer(_FnStage):
    operation_name = "filter"

    def __init__(self, fn=None, default=None, uid=None, **kw):
        super().__init__(fn, uid=uid, **kw)
        self.default = default

    def set_input(self, *features):
        super().set_input(*features)
        self.output_type = self._inputs[0].wtype
        return self

    def transform_fn(self, v):
        return v if (v is not None and self.fn(v)) else self.default

    def ctor_args(self):
        return {"fn": _fn_name(self.fn), "default": self.default}

    def load_ctor_args(self, a):
        self.fn = load_extract_fn(a.get("fn"))
        self.default = a.get("default")


@register_stage
class ReplaceTransformer(UnaryTransformer):
    operation_name = "replaceWith"
    _defaults = {"old_value": None, "new_value": None}

    def set_input(self, *features):
        super().set_input(*features)
        self.output_type = self._inputs[0].wtype
        return self

    def transform_fn(self, v):
        return self.params["new_value"] if v == self.params["old_value"] else v


def default_matches(v) -> bool:
    """``ToOccurTransformer.DefaultMatches``: numeric > 0, non-empty text, non-empty collection."""
    if v is None:
        return False
    if isinstance(v, bool):
        return v
    if isinstance(v, (int, float, np.number)):
        return float(v) > 0.0
    if isinstance(v, str):
        return len(v) > 0
    try:
        return len(v) > 0
    except TypeError:
        return False


@register_stage
class ToOccurTransformer(_FnStage):
    operation_name = "toOccur"
    output_type = T.RealNN

    def __init__(self, fn: Optional[Callable] = None, uid=None, **kw):
        super().__init__(fn or default_matches, uid=uid, **kw)

    def transform_fn(self, v):
        return 1.0 if self.fn(v) else 0.0

    def load_ctor_args(self, a):
        self.fn = load_extract_fn(a.get("fn")) or default_matches


@register_stage
class SubstringTransformer(BinaryTransformer):
    """(sub: Text, full: Text) -> Binary: ``full.contains(sub)`` (``SubstringTransformer.scala``)."""
    operation_name = "substring"
    output_type = T.Binary
    _defaults = {"to_lowercase": True}

    def transform_fn(self, sub, full):
        if sub is None or full is None:
            return None
        if self.params["to_lowercase"]:
            sub, full = sub.lower(), full.lower()
        return sub in full


def jaccard(a, b) -> float:
    """``JaccardSim``: |a ∩ b| / |a ∪ b|, 1.0 when both are empty."""
    a, b = set(a or ()), set(b or ())
    if not a and not b:
        return 1.0
    return len(a & b) / float(len(a | b))


@register_stage
class JaccardSimilarity(BinaryTransformer):
    operation_name = "jacSim"
    output_type = T.RealNN

    def transform_fn(self, a, b):
        return jaccard(a, b)


def ngram_distance(source: str, target: str, n: int = 3) -> float:
    """Lucene ``NGramDistance.getDistance`` (Kondrak n-gram edit similarity), float32 arithmetic."""
    f32 = np.float32
    sl, tl = len(source), len(target)
    if sl == 0 or tl == 0:
        return 1.0 if sl == tl else 0.0
    if sl < n or tl < n:
        cost = sum(1 for i in range(min(sl, tl)) if source[i] == target[i])
        return float(f32(cost) / f32(max(sl, tl)))
    sa = ["\0"] * (n - 1) + list(source)
    p = np.arange(sl + 1, dtype=np.float32)
    d = np.zeros(sl + 1, dtype=np.float32)
    for j in range(1, tl + 1):
        if j < n:
            t_j = ["\0"] * (n - j) + list(target[:j])
        else:
            t_j = list(target[j - n:j])
        d[0] = f32(j)
        for i in range(1, sl + 1):
            cost = 0
            tn = n
            for ni in range(n):
                if sa[i - 1 + ni] != t_j[ni]:
                    cost += 1
                elif sa[i - 1 + ni] == "\0":
                    tn -= 1
            ec = f32(cost) / f32(tn)
            d[i] = min(min(d[i - 1] + f32(1), p[i] + f32(1)), p[i - 1] + ec)
        p, d = d, p
    return float(f32(1.0) - p[sl] / f32(max(tl, sl)))


class _NGramSimilarity(BinaryTransformer):
    output_type = T.RealNN
    _defaults = {"to_lowercase": True, "n_gram_size": 3}

    def _str(self, v) -> str:
        raise NotImplementedError

    def transform_fn(self, a, b):
        lc = self.params["to_lowercase"]
        sa, sb = self._str(a).strip(), self._str(b).strip()
        if lc:
            sa, sb = sa.lower(), sb.lower()
        if not sa or not sb:
            return 0.0
        return ngram_distance(sa, sb, int(self.params["n_gram_size"]))


@register_stage
class TextNGramSimilarity(_NGramSimilarity):
    operation_name = "nGramText"

    def _str(self, v):
        return v or ""


@register_stage
class SetNGramSimilarity(_NGramSimilarity):
    operation_name = "nGramSet"

    def _str(self, v):
        return " ".join(v or ())


def _period(ms, period):
    from ...utils.dates import period_values
    return int(period_values(torch.as_tensor([int(ms)], dtype=torch.int64), period, raw=True)[0][0])


@register_stage
class TimePeriodTransformer(UnaryTransformer):
    operation_name = "dateToTimePeriod"
    output_type = T.Integral
    _defaults = {"period": "DayOfWeek"}

    def transform_columns(self, *cols, ds=None):
        from ...utils.dates import period_values
        c = cols[0]
        v, _ = period_values(c.values.to(torch.int64), self.params["period"], raw=True)
        return NumericColumn(T.Integral, v.to(torch.int64), c.valid)

    def transform_fn(self, v):
        return None if v is None else _period(v, self.params["period"])


@register_stage
class TimePeriodListTransformer(UnaryTransformer):
    operation_name = "dateListToTimePeriod"
    output_type = T.OPVector
    _defaults = {"period": "DayOfWeek"}

    def transform_fn(self, v):
        return np.asarray([float(_period(t, self.params["period"])) for t in (v or [])], np.float64)

    def transform_columns(self, *cols, ds=None):
        rows = [self.transform_fn(v) for v in cols[0].to_list()]
        width = max((len(r) for r in rows), default=0)
        out = np.zeros((len(rows), width))
        for i, r in enumerate(rows):
            out[i, :len(r)] = r
        from ...data.columns import VectorColumn
        return VectorColumn(torch.as_tensor(out))


@register_stage
class TimePeriodMapTransformer(UnaryTransformer):
    operation_name = "dateMapToTimePeriod"
    output_type = T.IntegralMap
    _defaults = {"period": "DayOfWeek"}

    def transform_fn(self, v):
        return {k: _period(t, self.params["period"]) for k, t in (v or {}).items()}


@register_stage
class MultiLabelJoiner(BinaryTransformer):
    """(indexed label, probability vector) -> RealMap label -> probability (``MultiLabelJoiner.scala``)."""
    operation_name = "MultiLabelJoiner"
    output_type = T.RealMap
    allow_label_as_input = True
    _defaults = {"labels": []}

    def _labels(self):
        """The given labels, else the class names of the indexed input's string indexer, read from its fitted
        metadata (``MultiLabelJoiner.scala``: the ``ml_attr`` values of the class-index column)."""
        if self.params["labels"] or not self._inputs:
            return list(self.params["labels"])
        st = self._inputs[0].origin_stage
        labels = (getattr(st, "metadata", None) or {}).get("labels") if st is not None else None
        return list(labels or [])

    def transform_fn(self, idx, probs):
        p = np.asarray(probs if probs is not None else [], np.float64).reshape(-1)
        return {l: float(x) for l, x in zip(self._labels(), p)}


@register_stage
class TopNLabelJoiner(MultiLabelJoiner):
    operation_name = "TopNLabelJoiner"
    _defaults = {"labels": [], "top_n": 3, "unseen_name": "UnseenLabel"}

    def transform_fn(self, idx, probs):
        m = super().transform_fn(idx, probs)
        m = {k: v for k, v in m.items() if k != self.params["unseen_name"]}
        return dict(sorted(m.items(), key=lambda kv: -kv[1])[:int(self.params["top_n"])])


@register_stage
class TopNLabelProbMap(UnaryTransformer):
    operation_name = "TopNLabelProbMap"
    output_type = T.RealMap
    _defaults = {"top_n": 3}

    def transform_fn(self, m):
        return dict(sorted((m or {}).items(), key=lambda kv: -kv[1])[:int(self.params["top_n"])])


@register_stage
class FilterMap(UnaryTransformer):
    """Keep / drop map keys and optionally clean keys / values (``FilterMap.scala``; ``filterKeys`` and
    ``cleanMap``, Transmogrifier.scala:532-625): the map is cleaned first (keys with ``clean_keys``, string values
    and string-collection values with ``clean_text``; defaults false / true as TransmogrifierDefaults), the
    allow / block lists are cleaned like the keys, then a non-empty allow list keeps its keys minus the block
    list, else a non-empty block list drops its keys."""
    operation_name = "filterMap"
    _defaults = {"allow_list_keys": [], "block_list_keys": [], "clean_keys": False, "clean_text": True}

    def set_input(self, *features):
        super().set_input(*features)
        self.output_type = self._inputs[0].wtype
        return self

    def transform_fn(self, m):
        p = self.params
        ck, cv = bool(p["clean_keys"]), bool(p["clean_text"])

        def clean(x, on):
            return clean_string(x) if on else x

        def value(v):
            if isinstance(v, str):
                return clean(v, cv)
            if isinstance(v, (set, frozenset, list, tuple)) and v and all(isinstance(e, str) for e in v):
                out = [clean(e, cv) for e in v]
                return type(v)(out) if not isinstance(v, frozenset) else frozenset(out)
            return v

        m = {clean(k, ck): value(v) for k, v in (m or {}).items()}
        allow = {clean(k, ck) for k in p["allow_list_keys"]}
        block = {clean(k, ck) for k in p["block_list_keys"]}
        if allow:
            return {k: v for k, v in m.items() if k in allow and k not in block}
        if block:
            return {k: v for k, v in m.items() if k not in block}
        return m


@register_stage
class OPCollectionTransformer(_FnStage):
    """Apply a value function element-wise to a list / set / map (``OPCollectionTransformer.scala``)."""
    operation_name = "opCollectionMap"

    def __init__(self, fn=None, output_type=None, uid=None, **kw):
        super().__init__(fn, uid=uid, **kw)
        if output_type is not None:
            self.output_type = output_type

    def transform_fn(self, v):
        if v is None:
            return None
        if isinstance(v, dict):
            return {k: self.fn(x) for k, x in v.items()}
        if isinstance(v, (set, frozenset)):
            return frozenset(self.fn(x) for x in v)
        return [self.fn(x) for x in v]


@register_stage
class EmailToPickListMapTransformer(UnaryTransformer):
    operation_name = "emailToPickListMap"
    output_type = T.PickListMap

    def transform_fn(self, m):
        return {k: d for k, d in ((k, email_domain(v)) for k, v in (m or {}).items()) if d is not None}


@register_stage
class UrlMapToPickListMapTransformer(UnaryTransformer):
    operation_name = "urlMapToPickListMap"
    output_type = T.PickListMap

    def transform_fn(self, m):
        return {k: d for k, d in ((k, url_domain(v)) for k, v in (m or {}).items()) if d is not None}


@register_stage
class PredictionDeIndexer(BinaryTransformer):
    """(indexed response, prediction) -> Text label of the predicted index (``PredictionDeIndexer.scala``);
    the labels come from the response's ``OpStringIndexer`` metadata."""
    operation_name = "predictionDeIndexer"
    output_type = T.Text
    allow_label_as_input = True
    _defaults = {"labels": [], "unseen_name": "UnseenIndex"}

    def _resolve_labels(self):
        """The response's string-indexer labels (minus its unseen label), read from its origin stage's metadata
        once that stage has been fitted."""
        if self.params["labels"] or not self._inputs:
            return
        st = self._inputs[0].origin_stage
        labels = (getattr(st, "metadata", None) or {}).get("labels") if st is not None else None
        if labels:
            self.params["labels"] = [l for l in labels if l != "UnseenLabel"]

    def set_input(self, *features):
        super().set_input(*features)
        self._resolve_labels()
        return self

    def transform_columns(self, *cols, ds=None):
        self._resolve_labels()
        return super().transform_columns(*cols, ds=ds)

    def transform_fn(self, label, pred):
        p = pred.get("prediction") if isinstance(pred, dict) else pred
        if p is None:
            return None
        labels = self.params["labels"]
        if not labels:      # PredictionDeIndexer.scala:60-66: the response carries no indexer labels
            name = self._inputs[0].name if self._inputs else "response"
            raise ValueError(f"The feature {name} does not contain any label/index mapping in its metadata")
        i = int(p)
        return labels[i] if 0 <= i < len(labels) else self.params["unseen_name"]


@register_stage
class MapTransformer(_FnStage):
    """``feature.map(fn)``: a unary value function with an explicit output type (serialized by name)."""
    operation_name = "map"

    def __init__(self, fn=None, output_type=None, operation_name=None, uid=None, **kw):
        super().__init__(fn, uid=uid, **kw)
        if output_type is not None:
            self.output_type = output_type
        if operation_name is not None:
            self.operation_name = operation_name

    def transform_fn(self, v):
        return require_function(self.fn, f"transform function of {self.uid}")(v)


@register_stage
class TextToMultiPickList(UnaryTransformer):
    """Text -> MultiPickList holding the one value (``TextToMultiPickList``, RichTextFeature.scala:53)."""
    operation_name = "textToMultiPickList"
    output_type = T.MultiPickList

    def transform_fn(self, v):
        return set() if v is None else {v}


@register_stage
class DateToListTransformer(UnaryTransformer):
    """Date -> DateList (DateTime -> DateTimeList) of the one date (``RichDateFeatureLambdas.ToDateList``,
    RichDateFeature.scala:55)."""
    operation_name = "dateToList"
    output_type = T.DateList

    def transform_fn(self, v):
        return [] if v is None else [int(v)]

    def transform_columns(self, *cols, ds=None):
        c = cols[0]
        if isinstance(c, NumericColumn):
            vals = c.values.to(torch.int64).cpu().numpy()
            ok = c.valid.cpu().numpy()
            return column_from_values(self.output_type, [[int(v)] if o else [] for v, o in zip(vals, ok)],
                                      "cpu")
        return super().transform_columns(*cols, ds=ds)

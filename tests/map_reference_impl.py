"""Per-row host reference of the map vectorizers (the round-2 implementation), kept as the test oracle
for the COO / device path in ``stages/feature/maps.py``.

Map vectorizers: one block of columns per (map feature, key).

Reference: ``OPMapVectorizer`` family (``core/.../impl/feature/OPMapVectorizer.scala:60-468``: RealMap / IntegralMap /
BinaryMap / DateMap / TextMapHashing; key discovery, per-key mean / mode / constant fill and null
tracking), ``TextMapPivotVectorizer`` (``:53-145``), ``MultiPickListMapVectorizer`` (``:49-122``),
``SmartTextMapVectorizer`` (``:57-418``), ``GeolocationMapVectorizer`` (``:42-129``) and
``DateMapToUnitCircleVectorizer`` (``:63-134``). Maps are ragged host data (COO of row, key, value);
every key becomes a dense device column block.
"""
from __future__ import annotations

from collections import Counter
from typing import Dict, List, Optional

import numpy as np
import torch

from transmogrifai_amd.config import vector_dtype
from transmogrifai_amd.data.columns import ObjectColumn
from transmogrifai_amd.data.vector_metadata import NULL_STRING, OTHER_STRING, OpVectorColumnMetadata
from transmogrifai_amd.features import types as T
from transmogrifai_amd.utils import text as TU
from transmogrifai_amd.stages.base import SequenceEstimator, SequenceTransformer, register_stage
from transmogrifai_amd.stages.feature.vectorizers import VectorizerMixin, top_values


def _clean_key(k, clean):
    return TU.clean_string(k) if clean else k


def _kind_of(t) -> str:
    if issubclass(t, T.BinaryMap):
        return "binary"
    if issubclass(t, T.DateMap):
        return "date"
    if issubclass(t, T.IntegralMap):
        return "integral"
    if issubclass(t, T.RealMap):
        return "real"
    if issubclass(t, T.MultiPickListMap):
        return "set"
    if issubclass(t, T.GeolocationMap):
        return "geo"
    if issubclass(t, (T.TextMap, T.TextAreaMap)) and t in (T.TextMap, T.TextAreaMap):
        return "smarttext"
    return "pivot"


class MapVectorizerModel(VectorizerMixin, SequenceTransformer):
    operation_name = "vecMap"

    def __init__(self, kind="real", keys=None, fills=None, tops=None, clean_keys=False, clean_text=True,
                 track_nulls=True, reference_date=None, methods=None, num_features=512, uid=None, **kw):
        super().__init__(uid=uid, **kw)
        self.kind = kind
        self.keys = [list(k) for k in (keys or [])]
        self.fills = [list(f) for f in (fills or [])]
        self.tops = [[list(t) for t in tt] for tt in (tops or [])]
        self.clean_keys = clean_keys
        self.clean_text = clean_text
        self.track_nulls = track_nulls
        self.reference_date = reference_date
        self.methods = [list(m) for m in (methods or [])]
        self.num_features = num_features

    def transform_columns(self, *cols, ds=None):
        n = len(cols[0]) if cols else 0
        blocks = []
        for ci, c in enumerate(cols):
            vals = c.values if isinstance(c, ObjectColumn) else np.array(c.to_list(), dtype=object)
            keys = self.keys[ci]
            kidx = {k: i for i, k in enumerate(keys)}
            if self.kind in ("real", "integral", "binary", "date"):
                per = 2 if self.track_nulls else 1
                b = np.zeros((n, len(keys) * per))
                seen = np.zeros((n, len(keys)), bool)
                for r, m in enumerate(vals):
                    for k, v in (m or {}).items():
                        j = kidx.get(_clean_key(k, self.clean_keys))
                        if j is None or v is None:
                            continue
                        if self.kind == "date":
                            v = float((int(self.reference_date) - int(v)) // 86400000)
                        elif self.kind == "binary":
                            v = 1.0 if v else 0.0
                        b[r, j * per] = float(v)
                        seen[r, j] = True
                for j in range(len(keys)):
                    miss = ~seen[:, j]
                    b[miss, j * per] = self.fills[ci][j]
                    if self.track_nulls:
                        b[:, j * per + 1] = miss.astype(np.float64)
                blocks.append(b)
            elif self.kind == "geo":
                per = 4 if self.track_nulls else 3
                b = np.zeros((n, len(keys) * per))
                for j in range(len(keys)):
                    b[:, j * per:j * per + 3] = self.fills[ci][j] if self.fills[ci][j] else [0.0, 0.0, 0.0]
                    if self.track_nulls:
                        b[:, j * per + 3] = 1.0
                for r, m in enumerate(vals):
                    for k, v in (m or {}).items():
                        j = kidx.get(_clean_key(k, self.clean_keys))
                        if j is None or not v:
                            continue
                        b[r, j * per:j * per + 3] = v
                        if self.track_nulls:
                            b[r, j * per + 3] = 0.0
                blocks.append(b)
            else:  # pivot / set / smarttext (pivot or hash per key)
                parts = []
                for j, k in enumerate(keys):
                    method = self.methods[ci][j] if self.methods else "pivot"
                    top = self.tops[ci][j]
                    if method == "hash":
                        w = self.num_features + (1 if self.track_nulls else 0)
                        bb = np.zeros((n, w))
                        for r, m in enumerate(vals):
                            v = _get(m, k, self.clean_keys)
                            toks = TU.tokenize(v) if isinstance(v, str) else []
                            if toks:
                                idx = TU.hash_terms(toks, self.num_features)
                                np.add.at(bb[r], idx, 1.0)
                            elif self.track_nulls:
                                bb[r, -1] = 1.0
                        parts.append(bb)
                        continue
                    w = len(top) + 1 + (1 if self.track_nulls else 0)
                    bb = np.zeros((n, w))
                    ix = {v: i for i, v in enumerate(top)}
                    for r, m in enumerate(vals):
                        v = _get(m, k, self.clean_keys)
                        items = ([] if v is None else (list(v) if isinstance(v, (set, frozenset, list)) else [v]))
                        if not items:
                            if self.track_nulls:
                                bb[r, -1] = 1.0
                            continue
                        for it in items:
                            s = TU.clean_string(str(it)) if self.clean_text else str(it)
                            bb[r, ix.get(s, len(top))] += 1.0
                    parts.append(bb)
                blocks.append(np.concatenate(parts, 1) if parts else np.zeros((n, 0)))
        dev = cols[0].device if cols else torch.device("cpu")
        out = np.concatenate(blocks, 1) if blocks else np.zeros((n, 0))
        return self._vec(torch.as_tensor(out, dtype=vector_dtype(dev), device=dev))

    def ctor_args(self):
        return {"kind": self.kind, "keys": self.keys, "fills": self.fills, "tops": self.tops,
                "cleanKeys": self.clean_keys, "cleanText": self.clean_text, "trackNulls": self.track_nulls,
                "referenceDate": self.reference_date, "methods": self.methods, "numFeatures": self.num_features}

    def load_ctor_args(self, a):
        self.__init__(a["kind"], a["keys"], a["fills"], a["tops"], a["cleanKeys"], a["cleanText"], a["trackNulls"],
                      a.get("referenceDate"), a.get("methods"), a.get("numFeatures", 512), uid=self.uid)


def _get(m, k, clean):
    if not m:
        return None
    if k in m:
        return m[k]
    if clean:
        for kk, v in m.items():
            if TU.clean_string(kk) == k:
                return v
    return None


class MapVectorizer(VectorizerMixin, SequenceEstimator):
    operation_name = "vecMap"
    _defaults = {"kind": "real", "clean_keys": False, "clean_text": True, "track_nulls": True,
                 "fill_with_mean": True, "fill_with_mode": True, "fill_value": 0.0, "top_k": 20, "min_support": 10,
                 "reference_date": None, "max_cardinality": 30, "num_features": 512, "allow_keys": None,
                 "block_keys": None}

    def fit_columns(self, *cols, ds=None):
        from transmogrifai_amd.utils.dates import now_ms
        p = self.params
        kind = p["kind"]
        ref = p["reference_date"] or now_ms()
        self.params["reference_date"] = ref
        all_keys, fills, tops, methods = [], [], [], []
        colsm = []
        for c, t in zip(cols, self.get_transient_features()):
            vals = c.values if isinstance(c, ObjectColumn) else c.to_list()
            per_key: Dict[str, list] = {}
            for m in vals:
                for k, v in (m or {}).items():
                    if v is None:
                        continue
                    per_key.setdefault(_clean_key(k, p["clean_keys"]), []).append(v)
            keys = sorted(per_key)
            if p["allow_keys"]:
                keys = [k for k in keys if k in set(p["allow_keys"])]
            if p["block_keys"]:
                keys = [k for k in keys if k not in set(p["block_keys"])]
            all_keys.append(keys)
            f_col, t_col, m_col = [], [], []
            for k in keys:
                vs = per_key[k]
                if kind == "real":
                    f_col.append(float(np.mean(vs)) if p["fill_with_mean"] else float(p["fill_value"]))
                elif kind == "integral":
                    if p["fill_with_mode"]:
                        cnt = Counter(int(v) for v in vs)
                        f_col.append(float(min(cnt.items(), key=lambda kv: (-kv[1], kv[0]))[0]))
                    else:
                        f_col.append(float(p["fill_value"]))
                elif kind in ("binary", "date"):
                    f_col.append(float(p["fill_value"]))
                elif kind == "geo":
                    from transmogrifai_amd.features.aggregators import Event, GeolocationMidpoint
                    f_col.append(GeolocationMidpoint().aggregate(Event(0, v) for v in vs))
                else:
                    cnt: Counter = Counter()
                    for v in vs:
                        items = list(v) if isinstance(v, (set, frozenset, list)) else [v]
                        cnt.update(TU.clean_string(str(i)) if p["clean_text"] else str(i) for i in items)
                    method = "pivot"
                    if kind == "smarttext" and len(cnt) > p["max_cardinality"]:
                        method = "hash"
                    m_col.append(method)
                    t_col.append(top_values(cnt, p["top_k"], p["min_support"]) if method == "pivot" else [])
            fills.append(f_col)
            tops.append(t_col)
            methods.append(m_col)
            for j, k in enumerate(keys):
                base = dict(parent_feature_name=(t.name,), parent_feature_type=(t.type_name,), grouping=k)
                if kind in ("real", "integral", "binary", "date"):
                    colsm.append(OpVectorColumnMetadata(**base))
                    if p["track_nulls"]:
                        colsm.append(OpVectorColumnMetadata(indicator_value=NULL_STRING, **base))
                elif kind == "geo":
                    colsm += [OpVectorColumnMetadata(descriptor_value=d, **base) for d in ("lat", "lon", "accuracy")]
                    if p["track_nulls"]:
                        colsm.append(OpVectorColumnMetadata(indicator_value=NULL_STRING, **base))
                elif m_col[j] == "hash":
                    colsm += [OpVectorColumnMetadata(**base) for _ in range(p["num_features"])]
                    if p["track_nulls"]:
                        colsm.append(OpVectorColumnMetadata(indicator_value=NULL_STRING, **base))
                else:
                    vals2 = t_col[j] + [OTHER_STRING] + ([NULL_STRING] if p["track_nulls"] else [])
                    colsm += [OpVectorColumnMetadata(indicator_value=v, **base) for v in vals2]
        self.metadata["vector_metadata"] = self.vector_metadata(colsm)
        return MapVectorizerModel(kind, all_keys, fills, tops, p["clean_keys"], p["clean_text"], p["track_nulls"],
                                  ref, methods, p["num_features"])


def map_vectorize(t, feats, label, D) -> list:
    kind = _kind_of(t)
    if t is T.PhoneMap or t is T.EmailMap or t is T.URLMap or t is T.Base64Map:
        kind = "pivot"
    st = MapVectorizer(kind=kind, clean_keys=D.CleanKeys, clean_text=D.CleanText, track_nulls=D.TrackNulls,
                       top_k=D.TopK, min_support=D.MinSupport, reference_date=D.ReferenceDate,
                       max_cardinality=D.MaxCategoricalCardinality, num_features=D.DefaultNumOfFeatures,
                       fill_value=float(D.FillValue))
    return [st.set_input(feats).get_output()]


# ------------------------------------------------------------------------ date map unit circle
class DateMapToUnitCircleVectorizerModel(VectorizerMixin, SequenceTransformer):
    operation_name = "dateMapToUnitCircle"

    def __init__(self, keys=None, time_period="HourOfDay", uid=None, **kw):
        super().__init__(uid=uid, **kw)
        self.keys = [list(k) for k in (keys or [])]
        self.time_period = time_period

    def transform_columns(self, *cols, ds=None):
        from transmogrifai_amd.utils.dates import period_values
        n = len(cols[0]) if cols else 0
        blocks = []
        for ci, c in enumerate(cols):
            vals = c.to_list()
            keys = self.keys[ci]
            b = np.zeros((n, 2 * len(keys)))
            for j, k in enumerate(keys):
                rows = [r for r, m in enumerate(vals) if m and m.get(k) is not None]
                if not rows:
                    continue
                ms = torch.as_tensor([int(vals[r][k]) for r in rows], dtype=torch.int64)
                v, size = period_values(ms, self.time_period)
                rad = 2 * np.pi * v.to(torch.float64).numpy() / size
                b[rows, 2 * j] = np.cos(rad)
                b[rows, 2 * j + 1] = np.sin(rad)
            blocks.append(b)
        dev = cols[0].device if cols else torch.device("cpu")
        out = np.concatenate(blocks, 1) if blocks else np.zeros((n, 0))
        return self._vec(torch.as_tensor(out, dtype=vector_dtype(dev), device=dev))

    def ctor_args(self):
        return {"keys": self.keys, "timePeriod": self.time_period}

    def load_ctor_args(self, a):
        self.keys, self.time_period = [list(k) for k in a["keys"]], a["timePeriod"]


class DateMapToUnitCircleVectorizer(VectorizerMixin, SequenceEstimator):
    """(cos, sin) of a time period per map key (``DateMapToUnitCircleVectorizer.scala:63-134``)."""
    operation_name = "dateMapToUnitCircle"
    _defaults = {"time_period": "HourOfDay", "clean_keys": False}

    def fit_columns(self, *cols, ds=None):
        all_keys, colsm = [], []
        tp = self.params["time_period"]
        for c, t in zip(cols, self.get_transient_features()):
            keys = sorted({k for m in c.to_list() for k, v in (m or {}).items() if v is not None})
            all_keys.append(keys)
            for k in keys:
                for d in ("x", "y"):
                    colsm.append(OpVectorColumnMetadata((t.name,), (t.type_name,), k, None, f"{d}_{tp}"))
        self.metadata["vector_metadata"] = self.vector_metadata(colsm)
        return DateMapToUnitCircleVectorizerModel(all_keys, tp)


# ------------------------------------------------------------------------ text map length / null
class TextMapLenModel(VectorizerMixin, SequenceTransformer):
    operation_name = "textMapLen"

    def __init__(self, keys=None, clean_keys=False, uid=None, **kw):
        super().__init__(uid=uid, **kw)
        self.keys = [list(k) for k in (keys or [])]
        self.clean_keys = clean_keys

    def _block(self, ci, vals, fn):
        keys = self.keys[ci]
        b = np.zeros((len(vals), len(keys)))
        for r, m in enumerate(vals):
            for j, k in enumerate(keys):
                b[r, j] = fn(_get(m, k, self.clean_keys))
        return b

    def _len(self, v):
        return float(sum(len(t) for t in TU.tokenize(v))) if isinstance(v, str) else 0.0

    def transform_columns(self, *cols, ds=None):
        n = len(cols[0]) if cols else 0
        blocks = [self._block(ci, c.to_list(), self._len) for ci, c in enumerate(cols)]
        dev = cols[0].device if cols else torch.device("cpu")
        out = np.concatenate(blocks, 1) if blocks else np.zeros((n, 0))
        return self._vec(torch.as_tensor(out, dtype=vector_dtype(dev), device=dev))

    def ctor_args(self):
        return {"keys": self.keys, "cleanKeys": self.clean_keys}

    def load_ctor_args(self, a):
        self.keys, self.clean_keys = [list(k) for k in a["keys"]], a["cleanKeys"]


class TextMapNullModel(TextMapLenModel):
    operation_name = "textMapNull"

    def _len(self, v):
        return 0.0 if isinstance(v, str) and v else 1.0


class _TextMapKeysEstimator(VectorizerMixin, SequenceEstimator):
    model_cls = TextMapLenModel
    descriptor = "TextLen"
    _defaults = {"clean_keys": False}

    def fit_columns(self, *cols, ds=None):
        all_keys, colsm = [], []
        for c, t in zip(cols, self.get_transient_features()):
            keys = sorted({_clean_key(k, self.params["clean_keys"]) for m in c.to_list()
                           for k, v in (m or {}).items() if v is not None})
            all_keys.append(keys)
            for k in keys:
                if self.descriptor == "TextLen":
                    colsm.append(OpVectorColumnMetadata((t.name,), (t.type_name,), k, None, "TextLen"))
                else:
                    colsm.append(OpVectorColumnMetadata((t.name,), (t.type_name,), k, NULL_STRING))
        self.metadata["vector_metadata"] = self.vector_metadata(colsm)
        return self.model_cls(all_keys, self.params["clean_keys"])


class TextMapLenEstimator(_TextMapKeysEstimator):
    """Token-length per text-map key (``TextMapLenEstimator.scala``)."""
    operation_name = "textMapLen"
    model_cls = TextMapLenModel
    descriptor = "TextLen"


class TextMapNullEstimator(_TextMapKeysEstimator):
    """Null indicator per text-map key (``TextMapNullEstimator.scala``)."""
    operation_name = "textMapNull"
    model_cls = TextMapNullModel
    descriptor = "Null"

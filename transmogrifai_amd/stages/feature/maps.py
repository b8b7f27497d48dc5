"""Map vectorizers: one block of columns per (map feature, key).

Reference: ``OPMapVectorizer`` family (``core/.../impl/feature/OPMapVectorizer.scala:60-468``: RealMap / IntegralMap /
BinaryMap / DateMap / TextMapHashing; key discovery, per-key mean / mode / constant fill and null
tracking), ``TextMapPivotVectorizer`` (``:53-145``), ``MultiPickListMapVectorizer`` (``:49-122``),
``SmartTextMapVectorizer`` (``:57-418``), ``GeolocationMapVectorizer`` (``:42-129``),
``DateMapToUnitCircleVectorizer`` (``:63-134``) and ``TextMapLenEstimator`` / ``TextMapNullEstimator``.

MI355X design: a map column is flattened ONCE into a COO view (:class:`MapCOO`: entry e =
``(row[e], key[e], value[e])`` as device tensors, keys and text values dictionary-coded; the only
per-element host work is that flattening of the Python dicts). Every fit statistic is a segmented
device reduction over the entries -- per-key sums / counts, ``(key, value)`` pair counts -- reduced over
the ranks of a row-sharded fit with one collective (``dp_aware``; reference reductions
``OPMapVectorizer.scala:134,238,280``), and every transform densifies the entries of the model's keys
with one scatter (last value wins for keys that collide after cleaning, as a dict update does) and
feeds the dense per-key columns to the same fill / one-hot pivot / hashing kernels as the scalar
vectorizers (``ops/vector.py``, ``ops/text.py``).
"""
from __future__ import annotations

from collections import Counter
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ...config import default_device, vector_dtype
from ...data.columns import ObjectColumn, TextColumn
from ...data.vector_metadata import NULL_STRING, OTHER_STRING, OpVectorColumnMetadata
from ...features import types as T
from ...utils import text as TU
from ..base import SequenceEstimator, SequenceTransformer, register_stage
from .vectorizers import VectorizerMixin, pivot_columns, top_values


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


_VALUE_KIND = {"real": "num", "binary": "num", "integral": "int", "date": "int", "geo": "geo", "set": "set",
               "pivot": "text", "smarttext": "text"}


# ------------------------------------------------------------------------------------------- COO view
class MapCOO:
    """Entries of a map column with a non-null value.

    ``row`` / ``key`` are int64 device tensors over the entries (``key`` indexes ``keys``, the cleaned key
    strings); the value is one of ``num`` (float64), ``ival`` (int64: integral / date millis), ``vcode``
    (int64 codes into ``vocab``: text), ``geo`` (float64 ``[nnz, 3]``) or, for sets, ``item_entry`` /
    ``item_code`` (one row per set element: its entry and its code into ``vocab``)."""

    def __init__(self, n, row, key, keys, device):
        self.n, self.row, self.key, self.keys, self.device = n, row, key, keys, device
        self.num = self.ival = self.vcode = self.geo = self.item_entry = self.item_code = None
        self.vocab: List[str] = []

    @property
    def nnz(self) -> int:
        return int(self.row.numel())

    def slots(self, model_keys: Sequence[str]) -> torch.Tensor:
        """``[len(keys)]`` int64: this column's key id -> position in ``model_keys`` (-1 = not a model key)."""
        pos = {k: i for i, k in enumerate(model_keys)}
        return torch.as_tensor(np.fromiter((pos.get(k, -1) for k in self.keys), np.int64, len(self.keys)),
                               device=self.device)

    def last_entry(self, model_keys: Sequence[str]) -> torch.Tensor:
        """``[n, K]`` int64: the entry holding (row, model key k), -1 if the row has none (the last one when
        several raw keys clean to the same key)."""
        K = len(model_keys)
        out = torch.full((self.n * max(K, 1),), -1, dtype=torch.int64, device=self.device)
        if K and self.nnz:
            s = self.slots(model_keys)[self.key]
            sel = s >= 0
            flat = self.row[sel] * K + s[sel]
            out.scatter_reduce_(0, flat, torch.nonzero(sel).reshape(-1), reduce="amax")
        return out.view(self.n, max(K, 1))[:, :K]


def _flatten(vals) -> tuple:
    n = len(vals)
    lens = np.fromiter((len(m) if m else 0 for m in vals), np.int64, n)
    ks = [k for m in vals if m for k in m]
    vs = [v for m in vals if m for v in m.values()]
    row = np.repeat(np.arange(n, dtype=np.int64), lens)
    return n, row, ks, vs


def map_coo(col, kind: str, clean_keys: bool, device=None) -> MapCOO:
    """The :class:`MapCOO` of a map column (cached on the column object per ``(kind, clean_keys, device)``)."""
    dev = torch.device(device) if device is not None else default_device()
    vkind = _VALUE_KIND[kind]
    cache = getattr(col, "_coo_cache", None)
    if cache is None:
        cache = {}
        try:
            col._coo_cache = cache
        except AttributeError:
            pass
    ck = (vkind, bool(clean_keys), str(dev))
    if ck in cache:
        return cache[ck]
    vals = col.values if isinstance(col, ObjectColumn) else col.to_list()
    n, row, ks, vs = _flatten(vals)
    if vkind == "geo":
        keep = np.fromiter((bool(v) for v in vs), bool, len(vs))
    else:
        keep = np.fromiter((v is not None for v in vs), bool, len(vs))
    row = row[keep]
    ks = [k for k, o in zip(ks, keep) if o]
    vs = [v for v, o in zip(vs, keep) if o]
    raw: Dict[str, int] = {}
    kc = np.fromiter((raw.setdefault(k, len(raw)) for k in ks), np.int64, len(ks))
    clean: Dict[str, int] = {}
    lut = np.fromiter((clean.setdefault(_clean_key(k, clean_keys), len(clean)) for k in raw), np.int64, len(raw))
    key = lut[kc] if kc.size else kc
    coo = MapCOO(n, torch.as_tensor(row, device=dev), torch.as_tensor(key, device=dev), list(clean), dev)
    if vkind == "num":
        coo.num = torch.as_tensor(np.fromiter((float(v) for v in vs), np.float64, len(vs)), device=dev)
    elif vkind == "int":
        coo.ival = torch.as_tensor(np.fromiter((int(v) for v in vs), np.int64, len(vs)), device=dev)
    elif vkind == "geo":
        g = np.asarray([list(v)[:3] for v in vs], np.float64).reshape(-1, 3)
        coo.geo = torch.as_tensor(g, device=dev)
    elif vkind == "text":
        voc: Dict[str, int] = {}
        coo.vcode = torch.as_tensor(np.fromiter((voc.setdefault(str(v), len(voc)) for v in vs), np.int64, len(vs)),
                                    device=dev)
        coo.vocab = list(voc)
    else:   # set: one item row per element
        items = [list(v) if isinstance(v, (set, frozenset, list, tuple)) else [v] for v in vs]
        ilen = np.fromiter((len(i) for i in items), np.int64, len(items))
        voc = {}
        codes = np.fromiter((voc.setdefault(str(x), len(voc)) for i in items for x in i), np.int64, int(ilen.sum()))
        coo.item_entry = torch.as_tensor(np.repeat(np.arange(len(items), dtype=np.int64), ilen), device=dev)
        coo.item_code = torch.as_tensor(codes, device=dev)
        coo.vocab = list(voc)
    cache[ck] = coo
    return coo


def _global_keys(local_keys: Sequence[Sequence[str]]) -> List[List[str]]:
    """Per column: sorted union of the keys of every rank (one object all-gather for all columns)."""
    from ...parallel import dp
    parts = dp.objects([sorted(k) for k in local_keys])
    return [sorted(set().union(*[set(p[i]) for p in parts])) for i in range(len(local_keys))]


def _filter_keys(keys, allow, block, clean: bool = False):
    """Allow / block lists (Transmogrifier.scala ``filterKeys``): the lists are cleaned like the map keys."""
    allow = {_clean_key(k, clean) for k in allow} if allow else None
    block = {_clean_key(k, clean) for k in block} if block else set()
    return [k for k in keys if (allow is None or k in allow) and k not in block]


def _key_sums(coo: MapCOO, keys: Sequence[str], values: torch.Tensor) -> torch.Tensor:
    """``[K, C]`` float64 sums over the entries of each model key of ``values [nnz, C]``."""
    K = len(keys)
    out = torch.zeros(K, values.shape[1], dtype=torch.float64, device=coo.device)
    if coo.nnz and K:
        s = coo.slots(keys)[coo.key]
        sel = s >= 0
        out.index_add_(0, s[sel], values[sel].to(torch.float64))
    return out


def _pair_counts(keys_of: torch.Tensor, codes: torch.Tensor, n_codes: int) -> tuple:
    """Distinct ``(key id, code)`` pairs with counts (device unique, one host read)."""
    if keys_of.numel() == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.int64)
    pair = keys_of * max(n_codes, 1) + codes
    u, c = torch.unique(pair, return_counts=True)
    u, c = u.cpu().numpy(), c.cpu().numpy()
    return u // max(n_codes, 1), u % max(n_codes, 1), c


def _per_key_text_columns(coo: MapCOO, keys: Sequence[str]) -> List[TextColumn]:
    """One dictionary-coded column per model key: row -> value code of (row, key), -1 when absent."""
    last = coo.last_entry(keys)
    out = []
    for j in range(len(keys)):
        e = last[:, j]
        codes = torch.where(e >= 0, coo.vcode[e.clamp_min(0)], torch.full_like(e, -1)) if coo.nnz else e
        out.append(TextColumn(T.PickList, codes.to(torch.int32), coo.vocab))
    return out


# --------------------------------------------------------------------------------------------- model
@register_stage
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

    def _numeric_block(self, coo: MapCOO, keys, fills, dtype) -> torch.Tensor:
        K, n, dev = len(keys), coo.n, coo.device
        last = coo.last_entry(keys)
        present = last >= 0
        e = last.clamp_min(0)
        if self.kind == "date":
            ms = coo.ival[e] if coo.nnz else torch.zeros(n, K, dtype=torch.int64, device=dev)
            v = torch.div(int(self.reference_date) - ms, 86400000, rounding_mode="trunc").to(torch.float64)
        elif self.kind == "integral":
            v = (coo.ival[e] if coo.nnz else torch.zeros(n, K, dtype=torch.int64, device=dev)).to(torch.float64)
        else:
            v = coo.num[e] if coo.nnz else torch.zeros(n, K, dtype=torch.float64, device=dev)
            if self.kind == "binary":
                v = (v != 0).to(torch.float64)
        f = torch.as_tensor(np.asarray(fills, np.float64).reshape(-1), device=dev)
        x = torch.where(present, v, f[None, :])
        if not self.track_nulls:
            return x.to(dtype)
        return torch.stack([x, (~present).to(torch.float64)], 2).reshape(n, 2 * K).to(dtype)

    def _geo_block(self, coo: MapCOO, keys, fills, dtype) -> torch.Tensor:
        K, n, dev = len(keys), coo.n, coo.device
        last = coo.last_entry(keys)
        present = last >= 0
        g = coo.geo[last.clamp_min(0)] if coo.nnz else torch.zeros(n, K, 3, dtype=torch.float64, device=dev)
        f = torch.as_tensor(np.asarray([fl if fl else [0.0, 0.0, 0.0] for fl in fills], np.float64).reshape(K, 3),
                            device=dev)
        x = torch.where(present[:, :, None], g, f[None, :, :])
        if self.track_nulls:
            x = torch.cat([x, (~present).to(torch.float64)[:, :, None]], 2)
        return x.reshape(n, K * (4 if self.track_nulls else 3)).to(dtype)

    def _set_block(self, coo: MapCOO, keys, tops, dtype) -> torch.Tensor:
        n, dev = coo.n, coo.device
        widths = [len(t) + 1 + (1 if self.track_nulls else 0) for t in tops]
        offs = np.concatenate([[0], np.cumsum(widths)]).astype(np.int64)
        out = torch.zeros(n, int(offs[-1]), dtype=dtype, device=dev)
        if not keys:
            return out
        has = torch.zeros(n, len(keys), dtype=torch.bool, device=dev)
        if coo.item_code is not None and coo.item_code.numel():
            s = coo.slots(keys)[coo.key]                         # per entry
            es = s[coo.item_entry]                               # per item
            sel = es >= 0
            # (slot, code) -> column inside the slot's block, built once per distinct pair on the host
            ks_, cs_, _ = _pair_counts(es[sel], coo.item_code[sel], len(coo.vocab))
            idx = [{v: i for i, v in enumerate(t)} for t in tops]
            col_of = np.empty(ks_.size, np.int64)
            for i, (k, c) in enumerate(zip(ks_, cs_)):
                v = coo.vocab[int(c)]
                v = TU.clean_string(v) if self.clean_text else v
                col_of[i] = offs[int(k)] + idx[int(k)].get(v, len(tops[int(k)]))
            pair_ids = torch.as_tensor(ks_ * max(len(coo.vocab), 1) + cs_, device=dev)
            mine = es[sel] * max(len(coo.vocab), 1) + coo.item_code[sel]
            cols = torch.as_tensor(col_of, device=dev)[torch.searchsorted(pair_ids, mine)]
            rows = coo.row[coo.item_entry[sel]]
            out.view(-1).index_put_((rows * out.shape[1] + cols,), torch.ones_like(rows, dtype=dtype), accumulate=True)
            has[rows, es[sel]] = True
        if self.track_nulls:
            for j in range(len(keys)):
                out[:, int(offs[j + 1]) - 1] = (~has[:, j]).to(dtype)
        return out

    def _text_block(self, coo: MapCOO, keys, tops, methods, dtype) -> torch.Tensor:
        from ...ops.text import HashInput, hashed_tf
        n, dev = coo.n, coo.device
        cols = _per_key_text_columns(coo, keys)
        toks = None
        parts = []
        for j, c in enumerate(cols):
            if methods and methods[j] == "hash":
                if toks is None:
                    toks = TU.tokenize_batch(coo.vocab)
                blk = torch.zeros(n, self.num_features + (1 if self.track_nulls else 0), dtype=dtype, device=dev)
                hashed_tf(blk[:, :self.num_features], [HashInput(c.codes, toks, None)], self.num_features, False,
                          False)
                if self.track_nulls:
                    cnt = torch.as_tensor(np.append(toks.counts(), 0), dtype=torch.int64, device=dev)
                    cc = c.codes.to(torch.int64)
                    blk[:, -1] = (cnt[torch.where(cc >= 0, cc, torch.full_like(cc, cnt.numel() - 1))] == 0).to(dtype)
                parts.append(blk)
            else:
                parts.append(pivot_columns([c], [tops[j]], self.clean_text, self.track_nulls, dtype))
        return torch.cat(parts, 1) if parts else torch.zeros(n, 0, dtype=dtype, device=dev)

    def transform_columns(self, *cols, ds=None):
        dev = default_device()
        dtype = vector_dtype(dev)
        n = len(cols[0]) if cols else 0
        blocks = []
        for ci, c in enumerate(cols):
            coo = map_coo(c, self.kind, self.clean_keys, dev)
            keys = self.keys[ci]
            if self.kind in ("real", "integral", "binary", "date"):
                blocks.append(self._numeric_block(coo, keys, self.fills[ci], dtype))
            elif self.kind == "geo":
                blocks.append(self._geo_block(coo, keys, self.fills[ci], dtype))
            elif self.kind == "set":
                blocks.append(self._set_block(coo, keys, self.tops[ci], dtype))
            else:
                blocks.append(self._text_block(coo, keys, self.tops[ci], self.methods[ci] if self.methods else None,
                                               dtype))
        out = torch.cat(blocks, 1) if blocks else torch.zeros(n, 0, dtype=dtype, device=dev)
        return self._vec(out)

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


# ------------------------------------------------------------------------------------------ estimator
@register_stage
class MapVectorizer(VectorizerMixin, SequenceEstimator):
    operation_name = "vecMap"
    _defaults = {"kind": "real", "clean_keys": False, "clean_text": True, "track_nulls": True,
                 "fill_with_mean": False, "fill_with_mode": False, "fill_value": 0.0, "top_k": 20, "min_support": 10,
                 "reference_date": None, "max_cardinality": 30, "num_features": 512, "allow_keys": None,
                 "block_keys": None, "max_pct_cardinality": 1.0}
    # row-sharded fits reduce per-key statistics over the ranks: key union and (key, value) counts in one
    # object all-gather, per-key sums in one all-reduce -- no map column is gathered
    dp_aware = True

    def fit_columns(self, *cols, ds=None):
        from ...parallel import dp
        from ...utils.dates import now_ms
        p = self.params
        kind = p["kind"]
        ref = p["reference_date"] or now_ms()
        self.params["reference_date"] = ref
        dev = default_device()
        coos = [map_coo(c, kind, p["clean_keys"], dev) for c in cols]
        # keys with at least one value on some rank
        present = []
        for coo in coos:
            used = torch.unique(coo.key).cpu().numpy() if coo.nnz else np.zeros(0, np.int64)
            present.append([coo.keys[int(i)] for i in used])
        all_keys = [_filter_keys(k, p["allow_keys"], p["block_keys"], p["clean_keys"]) for k in _global_keys(present)]
        fills: List[list] = [[] for _ in cols]
        tops: List[list] = [[] for _ in cols]
        methods: List[list] = [[] for _ in cols]
        if kind == "real":
            if p["fill_with_mean"]:
                sums = [_key_sums(coo, keys, torch.stack([coo.num, torch.ones_like(coo.num)], 1))
                        for coo, keys in zip(coos, all_keys)]
                red = dp.sum_(sums) if sums else []
                for i, r in enumerate(red):
                    r = r.cpu().numpy()
                    fills[i] = [float(a / b) if b > 0 else float(p["fill_value"]) for a, b in r]
            else:
                fills = [[float(p["fill_value"])] * len(k) for k in all_keys]
        elif kind == "integral":
            if p["fill_with_mode"]:
                counters = []
                for coo in coos:
                    cnt: Counter = Counter()
                    if coo.nnz:
                        u, c = torch.unique(torch.stack([coo.key, coo.ival], 1), dim=0, return_counts=True)
                        for (k, v), n_ in zip(u.cpu().numpy().tolist(), c.cpu().numpy().tolist()):
                            cnt[(coo.keys[k], v)] += n_
                    counters.append(cnt)
                merged = dp.merge_counters(counters)
                for i, keys in enumerate(all_keys):
                    per: Dict[str, list] = {}
                    for (k, v), n_ in merged[i].items():
                        per.setdefault(k, []).append((v, n_))
                    fills[i] = [float(min(per[k], key=lambda vc: (-vc[1], vc[0]))[0]) if k in per
                                else float(p["fill_value"]) for k in keys]
            else:
                fills = [[float(p["fill_value"])] * len(k) for k in all_keys]
        elif kind in ("binary", "date"):
            fills = [[float(p["fill_value"])] * len(k) for k in all_keys]
        elif kind == "geo":      # per-key geographic midpoint (features/geo.py monoid, reduced over the ranks)
            from ...features import geo
            stats = []
            for coo, keys in zip(coos, all_keys):
                if coo.nnz:
                    s = coo.slots(keys)[coo.key]
                    sel = s >= 0
                    stats.append(geo.reduce_by_key(geo.prepare(coo.geo[sel]), s[sel], len(keys)))
                else:
                    stats.append(geo.reduce_by_key(torch.zeros(0, 3, dtype=torch.float64, device=dev),
                                                   torch.zeros(0, dtype=torch.long, device=dev), len(keys)))
            for i, keys in enumerate(all_keys):
                S = geo.all_reduce(stats[i]).cpu()
                fills[i] = [geo.present(S[j]) for j in range(len(keys))]
        else:
            counters = []
            for coo in coos:
                cnt = Counter()
                if kind == "set":
                    if coo.item_code is not None and coo.item_code.numel():
                        k_, c_, n_ = _pair_counts(coo.key[coo.item_entry], coo.item_code, len(coo.vocab))
                    else:
                        k_ = c_ = n_ = np.zeros(0, np.int64)
                elif coo.nnz:
                    k_, c_, n_ = _pair_counts(coo.key, coo.vcode, len(coo.vocab))
                else:
                    k_ = c_ = n_ = np.zeros(0, np.int64)
                for k, c, m in zip(k_.tolist(), c_.tolist(), n_.tolist()):
                    v = coo.vocab[c]
                    cnt[(coo.keys[k], TU.clean_string(v) if p["clean_text"] else v)] += m
                counters.append(cnt)
            merged = dp.merge_counters(counters)
            pct = float(p.get("max_pct_cardinality", 1.0))
            n_rows = dp.count(len(cols[0]) if cols else 0) if pct < 1.0 else 0
            for i, keys in enumerate(all_keys):
                per: Dict[str, Counter] = {}
                for (k, v), m in merged[i].items():
                    per.setdefault(k, Counter())[v] += m
                if pct < 1.0 and n_rows > 0 and kind in ("pivot", "set"):
                    # OpOneHotVectorizer.scala:291-313 filterByMaxCardinality: a key whose distinct-value count
                    # reaches pct of the rows loses all its values before the fit, so it never becomes a key
                    # (distinct counts are exact here, the reference estimates them with an HLL)
                    keys = [k for k in keys if len(per.get(k, ())) / n_rows < pct]
                    all_keys[i] = keys
                for k in keys:
                    cnt = per.get(k, Counter())
                    method = "pivot"
                    if kind == "smarttext" and len(cnt) > p["max_cardinality"]:
                        method = "hash"
                    methods[i].append(method)
                    tops[i].append(top_values(cnt, p["top_k"], p["min_support"]) if method == "pivot" else [])
        colsm = []
        for i, t in enumerate(self.get_transient_features()):
            for j, k in enumerate(all_keys[i]):
                base = dict(parent_feature_name=(t.name,), parent_feature_type=(t.type_name,), grouping=k)
                if kind in ("real", "integral", "binary", "date"):
                    colsm.append(OpVectorColumnMetadata(**base))
                    if p["track_nulls"]:
                        colsm.append(OpVectorColumnMetadata(indicator_value=NULL_STRING, **base))
                elif kind == "geo":
                    colsm += [OpVectorColumnMetadata(descriptor_value=d, **base) for d in ("lat", "lon", "accuracy")]
                    if p["track_nulls"]:
                        colsm.append(OpVectorColumnMetadata(indicator_value=NULL_STRING, **base))
                elif methods[i] and methods[i][j] == "hash":
                    colsm += [OpVectorColumnMetadata(**base) for _ in range(p["num_features"])]
                    if p["track_nulls"]:
                        colsm.append(OpVectorColumnMetadata(indicator_value=NULL_STRING, **base))
                else:
                    vals2 = tops[i][j] + [OTHER_STRING] + ([NULL_STRING] if p["track_nulls"] else [])
                    colsm += [OpVectorColumnMetadata(indicator_value=v, **base) for v in vals2]
        self.metadata["vector_metadata"] = self.vector_metadata(colsm)
        return MapVectorizerModel(kind, all_keys, fills, tops, p["clean_keys"], p["clean_text"], p["track_nulls"],
                                  ref, methods, p["num_features"])


# RichMapFeature.vectorize argument names -> MapVectorizer params
_MAP_ARGS = {"default_value": "fill_value", "fill_value": "fill_value", "fill_with_mean": "fill_with_mean",
             "fill_with_mode": "fill_with_mode", "clean_keys": "clean_keys", "clean_text": "clean_text",
             "track_nulls": "track_nulls", "top_k": "top_k", "min_support": "min_support",
             "white_list_keys": "allow_keys", "allow_keys": "allow_keys", "black_list_keys": "block_keys",
             "block_keys": "block_keys", "reference_date": "reference_date",
             "max_categorical_cardinality": "max_cardinality", "num_hashes": "num_features",
             "allow_list_keys": "allow_keys", "block_list_keys": "block_keys",
             "max_pct_cardinality": "max_pct_cardinality"}


def map_vectorize(t, feats, label, D, **overrides) -> list:
    """The Transmogrifier's map vectorizer (Transmogrifier.scala:140-215: fill real maps with the mean and
    integral maps with the mode, pivot the categorical maps, smart-vectorize the free-text maps);
    ``overrides`` take the RichMapFeature.vectorize argument names.

    Four map types are converted before their vectorizer, as RichMapFeature does:
      * ``EmailMap`` -> ``EmailToPickListMapTransformer`` (domains) -> pivot (RichMapFeature.scala:1039-1058)
      * ``URLMap`` -> ``UrlMapToPickListMapTransformer`` (domains of valid URLs) -> pivot (:1067-1100)
      * ``PhoneMap`` -> ``IsValidPhoneMapDefaultCountry`` -> ``BinaryMapVectorizer`` (:979-1013)
      * ``Base64Map`` -> ``MimeTypeMapDetector`` -> ``TextMapPivotVectorizer`` (:121-179)
    """
    kind = _kind_of(t)
    ov = dict(overrides)
    circular = tuple(ov.pop("circular_date_reps", getattr(D, "CircularDateRepresentations", ())))
    region = ov.pop("default_region", D.DefaultRegion)
    strict = ov.pop("is_strict", False)
    type_hint = ov.pop("type_hint", None)
    feats = list(feats)
    if issubclass(t, T.EmailMap):
        from .misc_stages import EmailToPickListMapTransformer
        feats = [EmailToPickListMapTransformer().set_input(f).get_output() for f in feats]
        kind = "pivot"
    elif issubclass(t, T.URLMap):
        from .misc_stages import UrlMapToPickListMapTransformer
        feats = [UrlMapToPickListMapTransformer().set_input(f).get_output() for f in feats]
        kind = "pivot"
    elif issubclass(t, T.Base64Map):
        from .nlp_stages import MimeTypeMapDetector
        feats = [MimeTypeMapDetector(type_hint=type_hint or "").set_input(f).get_output() for f in feats]
        kind = "pivot"
    elif issubclass(t, T.PhoneMap):
        from .nlp_stages import IsValidPhoneMapDefaultCountry
        feats = [IsValidPhoneMapDefaultCountry(default_region=region, strict=strict).set_input(f).get_output()
                 for f in feats]
        kind = "binary"
    params = dict(kind=kind, clean_keys=D.CleanKeys, clean_text=D.CleanText, track_nulls=D.TrackNulls,
                  top_k=D.TopK, min_support=D.MinSupport, reference_date=D.ReferenceDate,
                  max_cardinality=D.MaxCategoricalCardinality, num_features=D.DefaultNumOfFeatures,
                  fill_value=float(D.FillValue), fill_with_mean=D.FillWithMean, fill_with_mode=D.FillWithMode,
                  max_pct_cardinality=float(getattr(D, "MaxPercentCardinality", 1.0)))
    if kind == "binary":   # RichBinaryMapFeature.vectorize: constant fill only
        params.update(fill_with_mean=False, fill_with_mode=False)
    for k, v in ov.items():
        if k not in _MAP_ARGS:
            raise TypeError(f"map vectorize got an unexpected argument {k!r}")
        params[_MAP_ARGS[k]] = v
    if kind == "smarttext":         # RichTextMapFeature.smartVectorize (Transmogrifier.scala:214-232)
        keep = ("clean_keys", "clean_text", "track_nulls", "top_k", "min_support", "max_cardinality", "num_features",
                "allow_keys", "block_keys")
        sp = {k: v for k, v in params.items() if k in keep}
        sp.update(track_text_len=bool(getattr(D, "TrackTextLen", False)),
                  hash_space_strategy=getattr(D, "HashSpaceStrategy", "auto"),
                  prepend_feature_name=bool(getattr(D, "PrependFeatureName", True)),
                  min_length_std_dev=float(getattr(D, "MinLengthStdDev", 0.0)))
        return [SmartTextMapVectorizer(**sp).set_input(feats).get_output()]
    cls = {"pivot": TextMapPivotVectorizer, "binary": BinaryMapVectorizer}.get(kind, MapVectorizer)
    st = cls(**params) if kind in ("pivot", "binary") and t is not T.OPMap else MapVectorizer(**params)
    out = st.set_input(feats).get_output()
    if kind == "date" and circular and t is not T.OPMap:
        # RichDateMapFeature / RichDateTimeMapFeature.vectorize (RichMapFeature.scala:776-797, :861-882): one
        # unit-circle vectorizer per circular representation, then the days-since block, combined
        from .vectorizers import VectorsCombiner
        circ = [DateMapToUnitCircleVectorizer(time_period=tp, clean_keys=params["clean_keys"]).set_input(feats)
                .get_output() for tp in circular]
        out = VectorsCombiner().set_input(circ + [out]).get_output()
    return [out]


# ---------------------------------------------------------------------- named map vectorizers (catalog)
def _named(name: str, op: str, kind: str):
    cls = type(name, (MapVectorizer,), {"operation_name": op, "_defaults": dict(MapVectorizer._defaults, kind=kind),
                                        "__doc__": f"``{name}`` (kind={kind!r}) of ``OPMapVectorizer.scala``."})
    return register_stage(cls)


RealMapVectorizer = _named("RealMapVectorizer", "vecRealMap", "real")
IntegralMapVectorizer = _named("IntegralMapVectorizer", "vecIntMap", "integral")
BinaryMapVectorizer = _named("BinaryMapVectorizer", "vecBinMap", "binary")
DateMapVectorizer = _named("DateMapVectorizer", "vecDateMap", "date")
TextMapPivotVectorizer = _named("TextMapPivotVectorizer", "vecPivotTextMap", "pivot")


def _first_keys(coo: "MapCOO") -> List[str]:
    """The map column's keys holding a value, in order of first appearance (row order, then key order)."""
    if not coo.nnz:
        return []
    k = coo.key.cpu().numpy()
    _, first = np.unique(k, return_index=True)
    return [coo.keys[int(k[i])] for i in np.sort(first)]


@register_stage
class SmartTextMapVectorizerModel(VectorizerMixin, SequenceTransformer):
    """Transform of :class:`SmartTextMapVectorizer` (``SmartTextMapVectorizerModel``, SmartTextMapVectorizer.scala:
    327-420): ``[categorical pivots | hashed text | text lengths | text null indicators]``."""
    operation_name = "smartTxtMapVec"

    def __init__(self, keys=None, methods=None, tops=None, clean_keys=False, clean_text=True, track_nulls=True,
                 track_text_len=False, hashing=None, uid=None, **kw):
        from .vectorizers import HashingParams
        super().__init__(uid=uid, **kw)
        self.keys = [list(k) for k in (keys or [])]
        self.methods = [list(m) for m in (methods or [])]
        self.tops = [[list(t) for t in tt] for tt in (tops or [])]
        self.clean_keys, self.clean_text = clean_keys, clean_text
        self.track_nulls, self.track_text_len = track_nulls, track_text_len
        self.hashing = hashing if isinstance(hashing, HashingParams) else HashingParams(**(hashing or {}))

    def transform_columns(self, *cols, ds=None):
        from ...ops.text import HashInput
        from .vectorizers import _vocab_lut, hash_text_columns
        dev = default_device()
        dtype = vector_dtype(dev)
        n = len(cols[0]) if cols else 0
        kcols = []
        for i, c in enumerate(cols):
            coo = map_coo(c, "pivot", self.clean_keys, dev)
            kcols.append((coo, _per_key_text_columns(coo, self.keys[i])))
        piv = [(i, j) for i in range(len(cols)) for j, m in enumerate(self.methods[i]) if m == "pivot"]
        hsh = [(i, j) for i in range(len(cols)) for j, m in enumerate(self.methods[i]) if m == "hash"]
        text = [(i, j) for i in range(len(cols)) for j, m in enumerate(self.methods[i]) if m in ("hash", "ignore")]
        toks = {}
        for i, _ in text:
            if i not in toks:
                voc = kcols[i][0].vocab
                toks[i] = TU.tokenize_batch(voc) if voc else TU.TokenBatch.from_lists([])
        blocks = []
        if piv:
            blocks.append(pivot_columns([kcols[i][1][j] for i, j in piv], [self.tops[i][j] for i, j in piv],
                                        self.clean_text, self.track_nulls, dtype))
        if hsh:
            hp = self.hashing
            ins = [HashInput(kcols[i][1][j].codes, toks[i], int(TU.hash_terms([self.keys[i][j]], hp.num_features)[0])
                             if hp.prepend_feature_name else None) for i, j in hsh]
            shared = hp.shared(len(hsh))
            from .vectorizers import HashingParams
            hp2 = HashingParams(hp.num_features, len(hsh), hp.max_num_features, hp.binary, hp.prepend_feature_name,
                                "shared" if shared else "separate", hp.hash_with_index)
            blocks.append(hash_text_columns([kcols[i][1][j] for i, j in hsh], None, hp2, None, dtype, inputs=ins))
        if text and self.track_text_len:
            blocks.append(torch.stack([_vocab_lut(kcols[i][1][j], toks[i].char_lengths().astype(np.float64), 0.0,
                                                  dtype) for i, j in text], 1))
        if text and self.track_nulls:
            blocks.append(torch.stack([_vocab_lut(kcols[i][1][j], (toks[i].counts() == 0).astype(np.float64), 1.0,
                                                  dtype) for i, j in text], 1))
        out = torch.cat(blocks, 1) if blocks else torch.zeros(n, 0, dtype=dtype, device=dev)
        return self._vec(out)

    def ctor_args(self):
        return {"keys": self.keys, "methods": self.methods, "tops": self.tops, "cleanKeys": self.clean_keys,
                "cleanText": self.clean_text, "trackNulls": self.track_nulls, "trackTextLen": self.track_text_len,
                "hashingParams": self.hashing.to_json()}

    def load_ctor_args(self, a):
        from .vectorizers import HashingParams
        self.keys = [list(k) for k in a["keys"]]
        self.methods = [list(m) for m in a["methods"]]
        self.tops = [[list(t) for t in tt] for tt in a["tops"]]
        self.clean_keys, self.clean_text = a["cleanKeys"], a["cleanText"]
        self.track_nulls, self.track_text_len = a["trackNulls"], a.get("trackTextLen", False)
        self.hashing = HashingParams.from_json(a["hashingParams"])


@register_stage
class SmartTextMapVectorizer(VectorizerMixin, SequenceEstimator):
    """``SmartTextMapVectorizer`` (SmartTextMapVectorizer.scala:58-270): every key of every text map is a text
    feature of its own, vectorized by the SmartTextVectorizer rule -- pivoted when its cardinality is at most
    ``max_cardinality`` (or its top-K values with min support cover ``coverage_pct`` of it), ignored when its
    length spread is below ``min_length_std_dev``, hashed otherwise (all hashed keys in one space of
    ``num_features`` columns, or one space each: ``hash_space_strategy``, keys' names prepended to their
    tokens). Keys come in order of first appearance. Output layout: categorical pivots, hashed columns, text
    lengths (``track_text_len``), null indicators of the hashed / ignored keys."""
    operation_name = "smartTxtMapVec"
    _defaults = {"max_cardinality": 30, "top_k": 20, "min_support": 10, "clean_text": True, "clean_keys": False,
                 "track_nulls": True, "track_text_len": False, "num_features": 512, "hash_space_strategy": "auto",
                 "prepend_feature_name": True, "binary_freq": False, "coverage_pct": 1.0,
                 "min_length_std_dev": 0.0, "allow_keys": None, "block_keys": None,
                 "max_pct_cardinality": 1.0, "unseen_name": OTHER_STRING}
    dp_aware = True

    def fit_columns(self, *cols, ds=None):
        from ...parallel import dp
        from .vectorizers import HashingParams, TextStats, hash_metadata  # noqa: F401
        p = self.params
        dev = default_device()
        max_card = int(p["max_cardinality"])
        allow = set(p["allow_keys"]) if p["allow_keys"] else None
        block = set(p["block_keys"] or ())
        local = []
        for c in cols:
            coo = map_coo(c, "pivot", p["clean_keys"], dev)
            keys = [k for k in _first_keys(coo) if (allow is None or k in allow) and k not in block]
            kc = _per_key_text_columns(coo, keys)
            local.append([(k, TextStats.of_column(col, p["clean_text"], False, max_card)) for k, col in zip(keys, kc)])
        merged: List[Dict[str, "TextStats"]] = [dict() for _ in cols]
        for part in dp.objects(local):                    # ranks in order: first appearance across the ranks
            for i, kv in enumerate(part):
                for k, st in kv:
                    merged[i][k] = merged[i][k].plus(st, max_card) if k in merged[i] else st
        keys, methods, tops = [], [], []
        for i in range(len(cols)):
            ks, ms, ts = [], [], []
            for k, st in merged[i].items():
                vc = st.value_counts
                total = sum(vc.values())
                filt = {v: m for v, m in vc.items() if m >= p["min_support"]}
                sv = sorted(filt.values(), reverse=True)
                cum = np.cumsum(sv) if sv else np.zeros(0)
                kk = min(p["top_k"], cum.size)
                coverage = (cum[kk - 1] / total) if (kk > 0 and total > 0) else 0.0
                card = len(vc)
                if card > max_card and card > p["top_k"] and coverage >= p["coverage_pct"]:
                    m = "pivot"
                elif card <= max_card:
                    m = "pivot"
                elif st.length_std < p["min_length_std_dev"]:
                    m = "ignore"
                else:
                    m = "hash"
                ks.append(k)
                ms.append(m)
                ts.append(top_values(Counter(filt), p["top_k"], 0) if m == "pivot" else [])
            keys.append(ks)
            methods.append(ms)
            tops.append(ts)
        tfs = self.get_transient_features()
        hp = HashingParams(p["num_features"], len(cols), 1 << 17, p["binary_freq"], p["prepend_feature_name"],
                           p["hash_space_strategy"])
        colsm = []
        for i, t in enumerate(tfs):                       # categorical keys
            for k, m, top in zip(keys[i], methods[i], tops[i]):
                if m != "pivot":
                    continue
                vals = list(top) + [p["unseen_name"]] + ([NULL_STRING] if p["track_nulls"] else [])
                colsm += [OpVectorColumnMetadata((t.name,), (t.type_name,), k, v) for v in vals]
        n_hash = sum(m == "hash" for ms in methods for m in ms)
        if n_hash:                                        # hashed keys (MapHashingFun.makeVectorColumnMetadata)
            if hp.shared(n_hash):
                hf = [t for i, t in enumerate(tfs) if "hash" in methods[i]]
                colsm += [OpVectorColumnMetadata(tuple(t.name for t in hf), tuple(t.type_name for t in hf), None, None)
                          for _ in range(p["num_features"])]
            else:
                for i, t in enumerate(tfs):
                    for k, m in zip(keys[i], methods[i]):
                        if m == "hash":
                            colsm += [OpVectorColumnMetadata((t.name,), (t.type_name,), k, None)
                                      for _ in range(p["num_features"])]
        text = [(t, k) for i, t in enumerate(tfs) for k, m in zip(keys[i], methods[i]) if m in ("hash", "ignore")]
        if p["track_text_len"]:
            colsm += [OpVectorColumnMetadata((t.name,), (t.type_name,), k, None, "TextLen") for t, k in text]
        if p["track_nulls"]:
            colsm += [OpVectorColumnMetadata((t.name,), (t.type_name,), k, NULL_STRING) for t, k in text]
        self.metadata["vector_metadata"] = self.vector_metadata(colsm)
        return SmartTextMapVectorizerModel(keys, methods, tops, p["clean_keys"], p["clean_text"], p["track_nulls"],
                                           p["track_text_len"], hp)

MultiPickListMapVectorizer = _named("MultiPickListMapVectorizer", "vecCatMap", "set")
GeolocationMapVectorizer = _named("GeolocationMapVectorizer", "vecGeoMap", "geo")


@register_stage
class TextMapHashingVectorizer(VectorizerMixin, SequenceTransformer):
    """``TextMapHashingVectorizer`` (OPMapVectorizer.scala:411-470): the tokens of every value of every input map
    (allow / block lists on the cleaned keys) are combined into ONE token list per row and hashed into one space of
    ``num_features`` columns (``numInputs = 1``), the first input's name prepended to the terms. Null / length
    tracking is done outside, per key, by :class:`TextMapNullEstimator` / :class:`TextMapLenEstimator`, as
    ``RichTextMapFeature.vectorize`` wires it."""
    operation_name = "vecHashTextMap"
    _defaults = {"num_features": 512, "clean_keys": False, "clean_text": True, "prepend_feature_name": True,
                 "allow_keys": None, "block_keys": None}

    def transform_columns(self, *cols, ds=None):
        from ...ops.text import HashInput, hashed_tf
        from .vectorizers import col_meta
        p = self.params
        tfs = self.get_transient_features()
        nf = int(p["num_features"])
        if len(tfs) == 1:
            cm = [col_meta(tfs[0]) for _ in range(nf)]
        else:
            cm = [OpVectorColumnMetadata(tuple(t.name for t in tfs), tuple(t.type_name for t in tfs), None, None,
                                         None) for _ in range(nf)]
        self.metadata["vector_metadata"] = self.vector_metadata(cm)
        dev = default_device()
        n = len(cols[0]) if cols else 0
        allow = set(p["allow_keys"]) if p["allow_keys"] else None
        block = set(p["block_keys"] or ())
        rows: List[List[str]] = [[] for _ in range(n)]
        for c in cols:
            coo = map_coo(c, "pivot", p["clean_keys"], torch.device("cpu"))
            if not coo.nnz:
                continue
            toks = TU.tokenize_batch(coo.vocab).lists() if coo.vocab else []
            ok = [(allow is None or k in allow) and k not in block for k in coo.keys]
            for r, k, v in zip(coo.row.tolist(), coo.key.tolist(), coo.vcode.tolist()):
                if ok[k]:
                    rows[r].extend(toks[v])
        prefix = int(TU.hash_terms([tfs[0].name], nf)[0]) if (p["prepend_feature_name"] and tfs) else None
        out = torch.empty(n, nf, dtype=vector_dtype(dev), device=dev)
        hashed_tf(out, [HashInput(None, TU.TokenBatch.from_lists(rows), prefix)], nf, True, False)
        return self._vec(out)


def _present_keys(cols, kind: str, clean: bool) -> List[List[str]]:
    """Global (all ranks) sorted keys that hold a value, per column."""
    local = []
    for c in cols:
        coo = map_coo(c, kind, clean)
        used = torch.unique(coo.key).cpu().numpy() if coo.nnz else np.zeros(0, np.int64)
        local.append([coo.keys[int(i)] for i in used])
    return _global_keys(local)


# ------------------------------------------------------------------------ date map unit circle
@register_stage
class DateMapToUnitCircleVectorizerModel(VectorizerMixin, SequenceTransformer):
    operation_name = "dateMapToUnitCircle"

    def __init__(self, keys=None, time_period="HourOfDay", uid=None, **kw):
        super().__init__(uid=uid, **kw)
        self.keys = [list(k) for k in (keys or [])]
        self.time_period = time_period

    def transform_columns(self, *cols, ds=None):
        from ...utils.dates import period_values
        dev = default_device()
        n = len(cols[0]) if cols else 0
        blocks = []
        for ci, c in enumerate(cols):
            coo = map_coo(c, "date", False, dev)
            keys = self.keys[ci]
            last = coo.last_entry(keys)
            present = last >= 0
            b = torch.zeros(n, len(keys), 2, dtype=torch.float64, device=dev)
            if coo.nnz and bool(present.any()):
                ms = coo.ival[last[present]]
                v, size = period_values(ms, self.time_period)
                rad = 2 * np.pi * v.to(torch.float64) / size
                b[present] = torch.stack([torch.cos(rad), torch.sin(rad)], 1)
            blocks.append(b.reshape(n, 2 * len(keys)))
        out = torch.cat(blocks, 1) if blocks else torch.zeros(n, 0, dtype=torch.float64, device=dev)
        return self._vec(out.to(vector_dtype(dev)))

    def ctor_args(self):
        return {"keys": self.keys, "timePeriod": self.time_period}

    def load_ctor_args(self, a):
        self.keys, self.time_period = [list(k) for k in a["keys"]], a["timePeriod"]


@register_stage
class DateMapToUnitCircleVectorizer(VectorizerMixin, SequenceEstimator):
    """(cos, sin) of a time period per map key (``DateMapToUnitCircleVectorizer.scala:63-134``)."""
    operation_name = "dateMapToUnitCircle"
    _defaults = {"time_period": "HourOfDay", "clean_keys": False}
    dp_aware = True     # key union only

    def fit_columns(self, *cols, ds=None):
        colsm = []
        tp = self.params["time_period"]
        all_keys = _present_keys(cols, "date", False)
        for keys, t in zip(all_keys, self.get_transient_features()):
            for k in keys:
                for d in ("x", "y"):
                    colsm.append(OpVectorColumnMetadata((t.name,), (t.type_name,), k, None, f"{d}_{tp}"))
        self.metadata["vector_metadata"] = self.vector_metadata(colsm)
        return DateMapToUnitCircleVectorizerModel(all_keys, tp)


# ------------------------------------------------------------------------ text map length / null
@register_stage
class TextMapLenModel(VectorizerMixin, SequenceTransformer):
    operation_name = "textMapLen"

    def __init__(self, keys=None, clean_keys=False, uid=None, **kw):
        super().__init__(uid=uid, **kw)
        self.keys = [list(k) for k in (keys or [])]
        self.clean_keys = clean_keys

    def _per_value(self, vocab: List[str]) -> np.ndarray:
        """Token-length sum of each distinct value (``TextMapLenEstimator``)."""
        return TU.tokenize_batch(vocab).char_lengths().astype(np.float64) if vocab else np.zeros(0)

    absent_value = 0.0

    def transform_columns(self, *cols, ds=None):
        dev = default_device()
        n = len(cols[0]) if cols else 0
        blocks = []
        for ci, c in enumerate(cols):
            coo = map_coo(c, "pivot", self.clean_keys, dev)
            keys = self.keys[ci]
            lut = torch.as_tensor(np.append(self._per_value(coo.vocab), self.absent_value), device=dev)
            b = torch.full((n, len(keys)), self.absent_value, dtype=torch.float64, device=dev)
            for j, tc in enumerate(_per_key_text_columns(coo, keys)):
                cc = tc.codes.to(torch.int64)
                b[:, j] = lut[torch.where(cc >= 0, cc, torch.full_like(cc, lut.numel() - 1))]
            blocks.append(b)
        out = torch.cat(blocks, 1) if blocks else torch.zeros(n, 0, dtype=torch.float64, device=dev)
        return self._vec(out.to(vector_dtype(dev)))

    def ctor_args(self):
        return {"keys": self.keys, "cleanKeys": self.clean_keys}

    def load_ctor_args(self, a):
        self.keys, self.clean_keys = [list(k) for k in a["keys"]], a["cleanKeys"]


@register_stage
class TextMapNullModel(TextMapLenModel):
    operation_name = "textMapNull"
    absent_value = 1.0

    def _per_value(self, vocab):
        return np.asarray([0.0 if v else 1.0 for v in vocab], np.float64)


class _TextMapKeysEstimator(VectorizerMixin, SequenceEstimator):
    model_cls = TextMapLenModel
    descriptor = "TextLen"
    _defaults = {"clean_keys": False}
    dp_aware = True     # key union only

    def fit_columns(self, *cols, ds=None):
        colsm = []
        all_keys = _present_keys(cols, "pivot", self.params["clean_keys"])
        for keys, t in zip(all_keys, self.get_transient_features()):
            for k in keys:
                if self.descriptor == "TextLen":
                    colsm.append(OpVectorColumnMetadata((t.name,), (t.type_name,), k, None, "TextLen"))
                else:
                    colsm.append(OpVectorColumnMetadata((t.name,), (t.type_name,), k, NULL_STRING))
        self.metadata["vector_metadata"] = self.vector_metadata(colsm)
        return self.model_cls(all_keys, self.params["clean_keys"])


@register_stage
class TextMapLenEstimator(_TextMapKeysEstimator):
    """Token-length per text-map key (``TextMapLenEstimator.scala``)."""
    operation_name = "textMapLen"
    model_cls = TextMapLenModel
    descriptor = "TextLen"


@register_stage
class TextMapNullEstimator(_TextMapKeysEstimator):
    """Null indicator per text-map key (``TextMapNullEstimator.scala``)."""
    operation_name = "textMapNull"
    model_cls = TextMapNullModel
    descriptor = "Null"

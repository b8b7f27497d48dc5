"""Type-driven vectorizers used by ``transmogrify``.

Reference stages: ``RealVectorizer`` (``impl/feature/RealVectorizer.scala:49-121``),
``IntegralVectorizer`` (``IntegralVectorizer.scala:49-116``), ``BinaryVectorizer`` (``:57-94``),
``RealNNVectorizer`` (``:43-57``), ``OpSetVectorizer`` / ``OpTextPivotVectorizer``
(``OpOneHotVectorizer.scala:61-438``), ``SmartTextVectorizer`` (``SmartTextVectorizer.scala:60-418``),
``OPCollectionHashingVectorizer`` (``:59-405``), ``DateToUnitCircleTransformer`` (``:77-121``),
``DateListVectorizer`` (``:60-309``), ``GeolocationVectorizer`` (``:49-156``) and ``VectorsCombiner``
(``VectorsCombiner.scala:51-89``).

Every transform is a whole-column (batch) operation: numerics are fused fill + null-indicator
kernels over ``[N, F]`` blocks, categoricals are dictionary-code gathers into a one-hot block
(string work happens once per *distinct* value on the host), hashing builds a per-distinct-value
sparse term vector and scatters it by code. On a GPU dataset these run as device kernels
(:mod:`transmogrifai_amd.ops.vector`), on the host as the torch/C++ reference path.
"""
from __future__ import annotations

from collections import Counter
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ...config import vector_dtype
from ...data.columns import NumericColumn, ObjectColumn, TextColumn, VectorColumn, GeoColumn
from ...data.vector_metadata import (NULL_STRING, OTHER_STRING, TEXT_LEN_STRING, FeatureHistory,
                                     OpVectorColumnMetadata, OpVectorMetadata)
from ...features import types as T
from ...ops import vector as V
from ...utils import text as TU
from ...utils.dates import TIME_PERIODS, period_values
from ..base import (GT0, GTEQ0, UNIT, OpEstimator, OpTransformer, SequenceEstimator, SequenceTransformer,
                    register_stage)


# ----------------------------------------------------------------------------------------- helpers
def col_meta(tf, is_null=False, descriptor=None, indicator=None, grouping="__default__"):
    if grouping == "__default__":
        grouping = tf.name if (is_null or descriptor is not None or indicator is not None) else None
    return OpVectorColumnMetadata((tf.name,), (tf.type_name,), grouping,
                                  NULL_STRING if is_null else indicator, descriptor)


def input_history(tfs, stage_name) -> Dict[str, FeatureHistory]:
    """``Transmogrifier.inputFeaturesToHistory`` (``Transmogrifier.scala:361-362``)."""
    return {t.name: FeatureHistory(tuple(t.origin_features), tuple(list(t.stages) + [stage_name])) for t in tfs}


class VectorizerMixin:
    output_type = T.OPVector

    def vector_metadata(self, columns) -> OpVectorMetadata:
        return OpVectorMetadata(self.get_output_feature_name(), list(columns),
                                input_history(self.get_transient_features(), self.stage_name()))

    def _vec(self, values: torch.Tensor) -> VectorColumn:
        return VectorColumn(values, self.metadata.get("vector_metadata"))


def _device(cols):
    for c in cols:
        d = c.device
        if d.type != "cpu":
            return d
    return torch.device("cpu")


# ------------------------------------------------------------------------------------------ numerics
@register_stage
class RealVectorizerModel(VectorizerMixin, SequenceTransformer):
    operation_name = "vecReal"

    def __init__(self, fill_values=None, track_nulls=True, uid=None, **kw):
        super().__init__(uid=uid, **kw)
        self.fill_values = list(fill_values or [])
        self.track_nulls = track_nulls

    def transform_columns(self, *cols, ds=None):
        dev = _device(cols)
        out = V.fill_and_track(cols, self.fill_values, self.track_nulls, vector_dtype(dev))
        return self._vec(out)

    def ctor_args(self):
        return {"fillValues": self.fill_values, "trackNulls": self.track_nulls}

    def load_ctor_args(self, a):
        self.fill_values, self.track_nulls = list(a["fillValues"]), a["trackNulls"]


@register_stage
class RealVectorizer(VectorizerMixin, SequenceEstimator):
    """Fill missing reals with the column mean (or a constant) plus a null indicator."""
    operation_name = "vecReal"
    _defaults = {"fill_value": 0.0, "fill_with_constant": True, "track_nulls": True}
    dp_aware = True     # means / modes reduce over the ranks (ops/vector.py)

    def set_fill_with_mean(self):
        return self.set("fill_with_constant", False)

    def set_fill_with_constant(self, v):
        self.set("fill_value", float(v))
        return self.set("fill_with_constant", True)

    def _meta(self):
        tfs = self.get_transient_features()
        cols = []
        for t in tfs:
            cols.append(col_meta(t))
            if self.params["track_nulls"]:
                cols.append(col_meta(t, is_null=True))
        return self.vector_metadata(cols)

    def fit_columns(self, *cols, ds=None):
        if self.params["fill_with_constant"]:
            fills = [float(self.params["fill_value"])] * len(cols)
        else:
            fills = V.column_means(cols)
        self.metadata["vector_metadata"] = self._meta()
        return RealVectorizerModel(fills, self.params["track_nulls"])


@register_stage
class IntegralVectorizer(RealVectorizer):
    """Fill missing integrals with the column mode (ties -> smallest value)."""
    operation_name = "vecInt"
    _defaults = {"fill_value": 0.0, "fill_with_constant": True, "fill_with_mode": False, "track_nulls": True}

    def set_fill_with_mode(self):
        self.set("fill_with_constant", False)
        return self.set("fill_with_mode", True)

    def fit_columns(self, *cols, ds=None):
        if self.params["fill_with_constant"] and not self.params["fill_with_mode"]:
            fills = [float(self.params["fill_value"])] * len(cols)
        else:
            fills = V.column_modes(cols)
        self.metadata["vector_metadata"] = self._meta()
        m = RealVectorizerModel(fills, self.params["track_nulls"])
        m.operation_name = self.operation_name
        return m


@register_stage
class BinaryVectorizer(VectorizerMixin, SequenceTransformer):
    operation_name = "vecBin"
    _defaults = {"fill_value": False, "track_nulls": True}

    def _meta(self):
        cols = []
        for t in self.get_transient_features():
            cols.append(col_meta(t))
            if self.params["track_nulls"]:
                cols.append(col_meta(t, is_null=True))
        return self.vector_metadata(cols)

    def transform_columns(self, *cols, ds=None):
        self.metadata["vector_metadata"] = self._meta()
        dev = _device(cols)
        fill = 1.0 if self.params["fill_value"] else 0.0
        return self._vec(V.fill_and_track(cols, [fill] * len(cols), self.params["track_nulls"], vector_dtype(dev)))


@register_stage
class RealNNVectorizer(VectorizerMixin, SequenceTransformer):
    operation_name = "vecNum"   # RealNNVectorizer.scala:46

    def transform_columns(self, *cols, ds=None):
        self.metadata["vector_metadata"] = self.vector_metadata([col_meta(t) for t in self.get_transient_features()])
        dev = _device(cols)
        return self._vec(V.fill_and_track(cols, [0.0] * len(cols), False, vector_dtype(dev)))


# -------------------------------------------------------------------------------------- categorical
def _text_counts(col: TextColumn, clean: bool) -> Counter:
    """Counts of (cleaned) non-null values: device bincount over codes, string work per vocab entry."""
    if len(col.vocab) == 0:
        return Counter()
    from ...ops.text import code_counts
    cnt = code_counts([col.codes], [len(col.vocab)])[0][:-1]
    out: Counter = Counter()
    for s, c in zip(col.vocab, cnt):
        if c:
            out[TU.clean_string(s) if clean else s] += int(c)
    return out


def _set_counts(col: ObjectColumn, clean: bool) -> Counter:
    out: Counter = Counter()
    for v in col.values:
        if v:
            out.update({(TU.clean_string(str(x)) if clean else str(x)) for x in v})
    return out


def top_values(counts: Counter, top_k: int, min_support: int) -> List[str]:
    """TopK by (-count, value) with min support (``OpOneHotVectorizer.scala:95-103``)."""
    items = [(v, c) for v, c in counts.items() if c >= min_support]
    items.sort(key=lambda vc: (-vc[1], vc[0]))
    return [v for v, _ in items[:top_k]]


def pivot_metadata(tfs, tops, track_nulls, unseen=OTHER_STRING):
    cols = []
    for t, top in zip(tfs, tops):
        vals = list(top) + [unseen] + ([NULL_STRING] if track_nulls else [])
        for v in vals:
            cols.append(OpVectorColumnMetadata((t.name,), (t.type_name,), t.name, v, None))
    return cols


def pivot_columns(cols, tops, clean, track_nulls, dtype) -> torch.Tensor:
    """One-hot block: per feature ``len(top)`` slots + OTHER (+ NULL) (``OpOneHotVectorizer.scala:416-437``)."""
    dev = _device(cols)
    n = len(cols[0]) if cols else 0
    widths = [len(t) + 1 + (1 if track_nulls else 0) for t in tops]
    out = torch.zeros(n, sum(widths), dtype=dtype, device=dev)
    off = 0
    p_codes, p_luts, p_offs = [], [], []     # dictionary-coded columns: one batched pivot launch
    for c, top, w in zip(cols, tops, widths):
        if isinstance(c, TextColumn):
            idx = {v: i for i, v in enumerate(top)}
            lut = np.empty(len(c.vocab) + 1, np.int64)
            for j, s in enumerate(c.vocab):
                k = TU.clean_string(s) if clean else s
                lut[j] = idx.get(k, len(top))
            lut[-1] = len(top) + 1 if track_nulls else -1
            p_codes.append(c.codes)
            p_luts.append(lut)
            p_offs.append(off)
        else:
            vals = c.values if isinstance(c, ObjectColumn) else c.to_list()
            block = np.zeros((n, w))
            idx = {v: i for i, v in enumerate(top)}
            for r, sv in enumerate(vals):
                if not sv:
                    if track_nulls:
                        block[r, len(top) + 1] = 1.0
                    continue
                grp = Counter(TU.clean_string(str(x)) if clean else str(x) for x in sv)
                for k, cnt in grp.items():
                    block[r, idx.get(k, len(top))] += cnt
            out[:, off:off + w] = torch.as_tensor(block, dtype=dtype, device=dev)
        off += w
    V.onehot_pivot(out, p_codes, p_luts, p_offs)
    return out


@register_stage
class OpOneHotVectorizerModel(VectorizerMixin, SequenceTransformer):
    operation_name = "pivotText"

    def __init__(self, top_values=None, clean_text=True, track_nulls=True, uid=None, **kw):
        super().__init__(uid=uid, **kw)
        self.top_values = [list(t) for t in (top_values or [])]
        self.clean_text = clean_text
        self.track_nulls = track_nulls

    def transform_columns(self, *cols, ds=None):
        return self._vec(pivot_columns(cols, self.top_values, self.clean_text, self.track_nulls,
                                       vector_dtype(_device(cols))))

    def ctor_args(self):
        return {"topValues": self.top_values, "shouldCleanText": self.clean_text,
                "shouldTrackNulls": self.track_nulls}

    def load_ctor_args(self, a):
        self.top_values, self.clean_text, self.track_nulls = a["topValues"], a["shouldCleanText"], \
            a["shouldTrackNulls"]


@register_stage
class OpTextPivotVectorizer(VectorizerMixin, SequenceEstimator):
    """One-hot pivot of text/categorical values (topK by count with min support).

    ``max_pct_cardinality`` drops a column whose distinct-value count reaches that fraction of the rows
    (OpOneHotVectorizer.scala:75-124). The reference estimates the cardinality with an Algebird
    HyperLogLog of ``hll_bits`` bits (~1.04 / sqrt(2^bits) error); here the distinct count comes exactly
    from the (all-reduced) value counts the fit already holds, so ``hll_bits`` is accepted for parity
    and has no effect."""
    operation_name = "pivotText"
    _defaults = {"top_k": 20, "min_support": 10, "clean_text": True, "track_nulls": True,
                 "unseen_name": OTHER_STRING, "max_pct_cardinality": 1.0, "hll_bits": 12}
    # Transmogrifier.scala:556-575 (topK > 0, minSupport >= 0), OpOneHotVectorizer.scala:250-266
    _param_domains = {"top_k": GT0, "min_support": GTEQ0, "max_pct_cardinality": UNIT,
                      "hll_bits": (4, 31, True, True)}

    def _counts(self, c):
        return _text_counts(c, self.params["clean_text"]) if isinstance(c, TextColumn) else \
            _set_counts(c, self.params["clean_text"])

    dp_aware = True

    def fit_columns(self, *cols, ds=None):
        from ...parallel import dp
        p = self.params
        tops = []
        n = dp.count(len(cols[0]) if cols else 0)
        # per-rank value counts folded over the process group (OpOneHotVectorizer.scala:97)
        for counts in dp.merge_counters([self._counts(c) for c in cols]):
            if p["max_pct_cardinality"] < 1.0 and n > 0 and len(counts) / n >= p["max_pct_cardinality"]:
                counts = Counter()
            tops.append(top_values(counts, p["top_k"], p["min_support"]))
        self.metadata["vector_metadata"] = self.vector_metadata(
            pivot_metadata(self.get_transient_features(), tops, p["track_nulls"], p["unseen_name"]))
        m = OpOneHotVectorizerModel(tops, p["clean_text"], p["track_nulls"])
        return m


@register_stage
class OpSetVectorizer(OpTextPivotVectorizer):
    operation_name = "vecSet"


# ------------------------------------------------------------------------------------------ hashing
class HashingParams:
    def __init__(self, num_features=512, num_inputs=1, max_num_features=1 << 17, binary=False,
                 prepend_feature_name=True, hash_space_strategy="auto", hash_with_index=False):
        self.num_features = num_features
        self.num_inputs = num_inputs
        self.max_num_features = max_num_features
        self.binary = binary
        self.prepend_feature_name = prepend_feature_name
        self.hash_space_strategy = hash_space_strategy
        self.hash_with_index = hash_with_index

    def shared(self, n_feats=None) -> bool:
        """``HashingFun.isSharedHashSpace`` (``OPCollectionHashingVectorizer.scala:191-199``)."""
        s = self.hash_space_strategy.lower()
        if s == "shared":
            return True
        if s == "separate":
            return False
        return self.num_features * (n_feats if n_feats is not None else self.num_inputs) > self.max_num_features

    def to_json(self):
        return dict(self.__dict__)

    @staticmethod
    def from_json(d):
        return HashingParams(**d)


def hash_metadata(tfs, hp: HashingParams):
    if hp.shared():
        return [OpVectorColumnMetadata(tuple(t.name for t in tfs), tuple(t.type_name for t in tfs), None, None, None)
                for _ in range(hp.num_features)]
    return [col_meta(t) for t in tfs for _ in range(hp.num_features)]


def hash_inputs(cols, tfs, hp: HashingParams, tok_params: Optional[Tuple[bool, int]]):
    """Per feature: dictionary codes + the tokens of each distinct value (native tokenizer) + the
    feature-name prefix. ``tok_params`` = (to_lowercase, min_token_length), or ``None`` when the values
    are already terms (lists / sets / maps)."""
    from ...ops.text import HashInput
    out = []
    for c, t in zip(cols, tfs):
        prefix = int(TU.hash_terms([t.name], hp.num_features)[0]) if hp.prepend_feature_name else None
        if isinstance(c, TextColumn):
            tb = TU.tokenize_batch(c.vocab, *tok_params) if tok_params is not None else \
                TU.TokenBatch.from_lists([[s] for s in c.vocab])
            out.append(HashInput(c.codes, tb, prefix))
        else:
            lists = [[str(x) for x in v] if v else [] for v in c.to_list()]
            out.append(HashInput(None, TU.TokenBatch.from_lists(lists), prefix))
    return out


def hash_text_columns(cols, tfs, hp: HashingParams, tok_params, dtype, inputs=None) -> torch.Tensor:
    """Hashed TF block of the columns, shared or per-feature hash space (HIP ``hash_tf_rows`` on device)."""
    from ...ops.text import hashed_tf
    dev = _device(cols)
    n = len(cols[0]) if cols else 0
    shared = hp.shared()
    width = hp.num_features if shared else hp.num_features * len(cols)
    out = torch.empty(n, width, dtype=dtype, device=dev)
    hashed_tf(out, inputs if inputs is not None else hash_inputs(cols, tfs, hp, tok_params), hp.num_features,
              shared, hp.binary)
    return out


@register_stage
class OPCollectionHashingVectorizer(VectorizerMixin, SequenceTransformer):
    """Hashing TF of lists / sets / maps (Spark ``HashingTF`` murmur3, seed 42)."""
    operation_name = "vecColHash"
    _defaults = {"num_features": 512, "binary_freq": False, "prepend_feature_name": True,
                 "hash_space_strategy": "auto", "hash_with_index": False}

    def _hp(self):
        p = self.params
        return HashingParams(p["num_features"], len(self._inputs), 1 << 17, p["binary_freq"],
                             p["prepend_feature_name"], p["hash_space_strategy"], p["hash_with_index"])

    def transform_columns(self, *cols, ds=None):
        hp = self._hp()
        tfs = self.get_transient_features()
        self.metadata["vector_metadata"] = self.vector_metadata(hash_metadata(tfs, hp))
        conv = []
        for c in cols:
            if isinstance(c, ObjectColumn) and issubclass(c.ftype, T.OPMap):
                conv.append(ObjectColumn(c.ftype, [[str(x) for x in v.values()] if v else [] for v in c.values]))
            else:
                conv.append(c)
        return self._vec(hash_text_columns(conv, tfs, hp, None, vector_dtype(_device(cols))))


# --------------------------------------------------------------------------------------- smart text
def _capped_plus(a: Counter, b: Counter, max_card: int) -> Counter:
    """``TextStats.additionHelper`` (SmartTextVectorizer.scala:231-235): once a map holds more than
    ``max_card`` keys it stops absorbing others."""
    if len(a) > max_card:
        return a
    if len(b) > max_card:
        return b
    out = Counter(a)
    out.update(b)
    return out


def _prefix_cutoff(first_seen: np.ndarray, max_card: int) -> Optional[int]:
    """Row (inclusive) after which a left fold of one-key maps under :func:`_capped_plus` is frozen: the row
    of the ``max_card + 1``-th distinct key; ``None`` while there are at most ``max_card`` keys."""
    if first_seen.size <= max_card:
        return None
    return int(np.partition(first_seen, max_card)[max_card])


class TextStats:
    """Value counts and length counts of one text feature (``TextStats``, SmartTextVectorizer.scala:200-300),
    with the reference's capped monoid: :meth:`of_column` folds a partition's rows in order, :meth:`plus`
    merges partitions (ranks) in order."""

    def __init__(self, value_counts: Counter, length_counts: Counter):
        self.value_counts = value_counts
        self.length_counts = length_counts

    @property
    def length_std(self) -> float:
        n = sum(self.length_counts.values())
        if n == 0:
            return float("nan")
        mean = sum(k * v for k, v in self.length_counts.items()) / n
        var = sum(v * (k - mean) ** 2 for k, v in self.length_counts.items()) / n
        return var ** 0.5

    def plus(self, other: "TextStats", max_card: int) -> "TextStats":
        return TextStats(_capped_plus(self.value_counts, other.value_counts, max_card),
                         _capped_plus(self.length_counts, other.length_counts, max_card))

    @staticmethod
    def of_column(col: TextColumn, clean: bool, token_lengths: bool, max_card: int) -> "TextStats":
        """The left fold ``rows.map(computeTextStats).reduce(plus)`` of one partition, computed from
        per-value counts and first occurrences (device histogram over the dictionary codes): values seen
        after the ``max_card + 1``-th distinct value are not counted (the reference's frozen map)."""
        V = len(col.vocab)
        if V == 0:
            return TextStats(Counter(), Counter())
        from ...ops.text import code_counts
        # cleaned values of the whole vocabulary in one native pass (first-appearance ids of equal cleaned
        # strings, character lengths); Python strings only for the values that end up counted
        cb = TU.clean_batch(col.vocab, clean)
        lut = cb.ids
        full = code_counts([col.codes], [V])[0][:-1]
        codes = col.codes
        n = int(codes.shape[0])
        first = None
        if cb.n_ids > max_card:
            c = codes.to(torch.int64)
            ok = c >= 0
            rid = torch.arange(n, device=c.device)
            fv = torch.full((V,), n, dtype=torch.int64, device=c.device).scatter_reduce_(
                0, c[ok], rid[ok], reduce="amin")
            first = fv.cpu().numpy()
            first_id = np.full(cb.n_ids, n, np.int64)
            np.minimum.at(first_id, lut, first)
            cut = _prefix_cutoff(first_id, max_card)
            counts = code_counts([codes[:cut + 1]], [V])[0][:-1]
        else:
            counts = full
        vc: Counter = Counter()
        nzc = np.flatnonzero(counts)
        if nzc.size:
            per_id = np.bincount(lut[nzc], weights=counts[nzc], minlength=cb.n_ids)
            first_j = np.full(cb.n_ids, V, np.int64)
            np.minimum.at(first_j, lut[nzc], nzc)
            live = np.flatnonzero(per_id)
            for i in live[np.argsort(first_j[live], kind="stable")]:     # insertion order: first counted value
                vc[cb.value(int(first_j[i]))] = int(per_id[i])
        # length counts: every row of the partition (their own cap applies to distinct lengths)
        lc: Counter = Counter()
        if token_lengths:
            # TextTokenizer.tokenizeString with the default analyzer; each row's map folds its token lengths
            # under the same cap (textStatsFromString)
            tb = TU.tokenize_batch(col.vocab)
            tl = tb.token_char_lengths()
            rp = tb.row_ptr
            maps = []
            for j in range(V):
                m: Counter = Counter()
                for L in tl[rp[j]:rp[j + 1]]:
                    m = _capped_plus(m, Counter({int(L): 1}), max_card)
                maps.append(m)
            present = [j for j in np.flatnonzero(full)]
            union = set().union(*[maps[j].keys() for j in present]) if present else set()
            if len(union) <= max_card:
                for j in present:
                    for L, c in maps[j].items():
                        lc[L] += c * int(full[j])
            else:               # the cap triggers: fold the rows in order (rare: > max_card token lengths)
                for code in codes.cpu().numpy():
                    if code >= 0:
                        lc = _capped_plus(lc, maps[int(code)], max_card)
            return TextStats(vc, lc)
        else:
            nzf = np.flatnonzero(full)
            if nzf.size:
                bl = np.bincount(cb.char_len[nzf], weights=full[nzf])
                for L in np.flatnonzero(bl):
                    lc[int(L)] = int(bl[L])
        if len(lc) > max_card:
            # same prefix rule over the rows' lengths (first occurrence of each length value)
            if first is None:
                c = codes.to(torch.int64)
                ok = c >= 0
                rid = torch.arange(n, device=c.device)
                first = torch.full((V,), n, dtype=torch.int64, device=c.device).scatter_reduce_(
                    0, c[ok], rid[ok], reduce="amin").cpu().numpy()
            lens = cb.char_len
            uniq, inv = np.unique(lens, return_inverse=True)
            first_len = np.full(uniq.size, n, np.int64)
            np.minimum.at(first_len, inv, first)
            cut = _prefix_cutoff(first_len, max_card)
            pc = code_counts([codes[:cut + 1]], [V])[0][:-1]
            lc = Counter()
            for j in np.flatnonzero(pc):
                lc[int(lens[j])] += int(pc[j])
        return TextStats(vc, lc)


def reduce_text_stats(parts: Sequence[List["TextStats"]], max_card: int) -> List["TextStats"]:
    """Merge per-partition (per-rank) stats lists in partition order."""
    acc = list(parts[0])
    for p in parts[1:]:
        acc = [a.plus(b, max_card) for a, b in zip(acc, p)]
    return acc


@register_stage
class SmartTextVectorizerModel(VectorizerMixin, SequenceTransformer):
    operation_name = "smartTxtVec"

    def __init__(self, methods=None, top_values=None, clean_text=True, track_nulls=True, hashing=None,
                 track_text_len=False, min_token_length=1, to_lowercase=True, strip_html=False, uid=None, **kw):
        super().__init__(uid=uid, **kw)
        self.strip_html = strip_html
        self.methods = list(methods or [])
        self.top_values = [list(t) for t in (top_values or [])]
        self.clean_text = clean_text
        self.track_nulls = track_nulls
        self.hashing = hashing if isinstance(hashing, HashingParams) else HashingParams(**(hashing or {}))
        self.track_text_len = track_text_len
        self.min_token_length = min_token_length
        self.to_lowercase = to_lowercase

    def transform_columns(self, *cols, ds=None):
        dtype = vector_dtype(_device(cols))
        tfs = self.get_transient_features() if self._inputs else [None] * len(cols)
        piv = [i for i, m in enumerate(self.methods) if m == "pivot"]
        hsh = [i for i, m in enumerate(self.methods) if m == "hash"]
        ign = [i for i, m in enumerate(self.methods) if m == "ignore"]
        rest = hsh + ign
        # one native tokenizer pass per hashed / ignored column, over its distinct values
        toks = {i: TU.tokenize_batch([TU.strip_html(v) for v in cols[i].vocab] if self.strip_html else cols[i].vocab,
                                     self.to_lowercase, self.min_token_length) for i in rest}
        blocks = []
        if piv:
            blocks.append(pivot_columns([cols[i] for i in piv], [self.top_values[i] for i in piv], self.clean_text,
                                        self.track_nulls, dtype))
        if hsh:
            from ...ops.text import HashInput
            hp = self.hashing
            ins = [HashInput(cols[i].codes, toks[i], int(TU.hash_terms([tfs[i].name], hp.num_features)[0])
                             if hp.prepend_feature_name else None) for i in hsh]
            blocks.append(hash_text_columns([cols[i] for i in hsh], None, hp, None, dtype, inputs=ins))
        if rest and self.track_text_len:
            blocks.append(torch.stack([_vocab_lut(cols[i], toks[i].char_lengths().astype(np.float64), 0.0, dtype)
                                       for i in rest], 1))
        if rest and self.track_nulls:
            blocks.append(torch.stack([_vocab_lut(cols[i], (toks[i].counts() == 0).astype(np.float64), 1.0, dtype)
                                       for i in rest], 1))
        dev = _device(cols)
        out = torch.cat(blocks, 1) if blocks else torch.zeros(len(cols[0]), 0, dtype=dtype, device=dev)
        return self._vec(out)

    def ctor_args(self):
        return {"vectorizationMethods": self.methods, "topValues": self.top_values,
                "shouldCleanText": self.clean_text, "shouldTrackNulls": self.track_nulls,
                "hashingParams": self.hashing.to_json(), "trackTextLen": self.track_text_len,
                "minTokenLength": self.min_token_length, "toLowercase": self.to_lowercase,
                "stripHtml": self.strip_html}

    def load_ctor_args(self, a):
        self.methods, self.top_values = a["vectorizationMethods"], a["topValues"]
        self.clean_text, self.track_nulls = a["shouldCleanText"], a["shouldTrackNulls"]
        self.hashing = HashingParams.from_json(a["hashingParams"])
        self.track_text_len = a.get("trackTextLen", False)
        self.min_token_length = a.get("minTokenLength", 1)
        self.to_lowercase = a.get("toLowercase", True)
        self.strip_html = a.get("stripHtml", False)


def _vocab_lut(c: TextColumn, per_value: np.ndarray, null_value: float, dtype) -> torch.Tensor:
    """Row values from a per-distinct-value table (null rows take ``null_value``)."""
    lut = torch.as_tensor(np.append(per_value, null_value), dtype=dtype, device=c.codes.device)
    idx = torch.where(c.codes >= 0, c.codes.long(), torch.full_like(c.codes.long(), len(c.vocab)))
    return lut[idx]


@register_stage
class SmartTextVectorizer(VectorizerMixin, SequenceEstimator):
    """Pivot low-cardinality text, hash free text, ignore constant-length text
    (``SmartTextVectorizer.scala:79-152``)."""
    operation_name = "smartTxtVec"
    _defaults = {"max_cardinality": 1000, "top_k": 20, "min_support": 10, "clean_text": True, "track_nulls": True,
                 "num_features": 512, "hash_space_strategy": "auto", "prepend_feature_name": True,
                 "binary_freq": False, "coverage_pct": 0.90, "min_length_std_dev": 0.0, "track_text_len": False,
                 "min_token_length": 1, "to_lowercase": True, "unseen_name": OTHER_STRING,
                 "text_length_type": "FullEntry", "strip_html": False}
    # SmartTextVectorizer.scala:378-405 + the shared topK / minSupport validators
    _param_domains = {"top_k": GT0, "min_support": GTEQ0, "max_cardinality": (1, 1000, True, True),
                      "coverage_pct": (0.0, 1.0, False, True), "min_length_std_dev": (0.0, 100.0, True, True)}
    # Row-sharded fits: every rank folds its own rows into capped TextStats (<= max_cardinality + 1 values
    # per feature) and the ranks' stats are merged in rank order -- one small object all-gather, the
    # reference's ``valueStats.reduce(_ + _)`` (SmartTextVectorizer.scala:87-91) with ranks as partitions
    dp_aware = True

    def fit_columns(self, *cols, ds=None):
        from ...parallel import dp
        p = self.params
        tlt = str(p["text_length_type"]).lower()
        if tlt not in ("fullentry", "tokens"):
            raise ValueError(f"textLengthType must be FullEntry or Tokens, got {p['text_length_type']!r}")
        max_card = int(p["max_cardinality"])
        local = [TextStats.of_column(c, p["clean_text"], tlt == "tokens", max_card) for c in cols]
        stats_all = reduce_text_stats(dp.objects(local), max_card)
        methods, tops = [], []
        for stats in stats_all:
            vc = stats.value_counts
            total = sum(vc.values())
            filt = {k: v for k, v in vc.items() if v >= p["min_support"]}
            sv = sorted(filt.values(), reverse=True)
            cum = np.cumsum(sv) if sv else np.zeros(0)
            k = min(p["top_k"], cum.size)
            coverage = (cum[k - 1] / total) if (k > 0 and total > 0) else 0.0
            card = len(vc)
            if card > max_card and card > p["top_k"] and coverage >= p["coverage_pct"]:
                m = "pivot"
            elif card <= max_card:
                m = "pivot"
            elif stats.length_std < p["min_length_std_dev"]:
                m = "ignore"
            else:
                m = "hash"
            methods.append(m)
            tops.append(top_values(Counter(filt), p["top_k"], 0))
        hp = HashingParams(p["num_features"], len(cols), 1 << 17, p["binary_freq"], p["prepend_feature_name"],
                           p["hash_space_strategy"])
        tfs = self.get_transient_features()
        piv = [i for i, m in enumerate(methods) if m == "pivot"]
        hsh = [i for i, m in enumerate(methods) if m == "hash"]
        rest = hsh + [i for i, m in enumerate(methods) if m == "ignore"]
        colsm = pivot_metadata([tfs[i] for i in piv], [tops[i] for i in piv], p["track_nulls"], p["unseen_name"])
        if hsh:
            colsm += hash_metadata([tfs[i] for i in hsh], hp)
        if p["track_text_len"]:
            colsm += [col_meta(tfs[i], descriptor=TEXT_LEN_STRING) for i in rest]
        if p["track_nulls"]:
            colsm += [col_meta(tfs[i], is_null=True) for i in rest]
        self.metadata["vector_metadata"] = self.vector_metadata(colsm)
        self.metadata["text_methods"] = methods
        return SmartTextVectorizerModel(methods, tops, p["clean_text"], p["track_nulls"], hp, p["track_text_len"],
                                        p["min_token_length"], p["to_lowercase"], p["strip_html"])


# --------------------------------------------------------------------------------------------- dates
@register_stage
class DateToUnitCircleTransformer(VectorizerMixin, SequenceTransformer):
    """(cos, sin) of a calendar period of each date (``DateToUnitCircleTransformer.scala:77-121``)."""
    operation_name = "dateToUnitCircle"
    _defaults = {"time_period": "HourOfDay"}

    def transform_columns(self, *cols, ds=None):
        tp = self.params["time_period"]
        tfs = self.get_transient_features() if self._inputs else []
        self.metadata["vector_metadata"] = OpVectorMetadata(
            self.get_output_feature_name() if self._inputs else "v",
            [col_meta(t, descriptor=d, grouping=None) for t in tfs for d in (f"x_{tp}", f"y_{tp}")],
            {t.name: FeatureHistory(tuple(t.origin_features), tuple(t.stages)) for t in tfs})
        dev = _device(cols)
        dtype = vector_dtype(dev)
        from ...ops.text import date_unit_circle_into
        if not cols:
            return self._vec(torch.zeros(0, 0))
        out = torch.empty(len(cols[0]), 2 * len(cols), dtype=dtype, device=dev)
        for k, c in enumerate(cols):     # HIP date_unit_circle_kernel on device
            date_unit_circle_into(out[:, 2 * k:2 * k + 2], c.values, c.valid, tp)
        return self._vec(out)


@register_stage
class DateListVectorizer(VectorizerMixin, SequenceTransformer):
    """Days since first/last date vs a reference date, or mode day/month/hour pivots
    (``DateListVectorizer.scala:60-309``). Accepts ``DateList`` or single ``Date`` columns."""
    operation_name = "vecDateList"
    _defaults = {"pivot": "SinceFirst", "reference_date": None, "track_nulls": True, "fill_value": 0.0}
    _param_domains = {"reference_date": GTEQ0}          # DateListVectorizer.scala:150-155

    def _ref(self):
        r = self.params["reference_date"]
        if r is None:
            from ...utils.dates import now_ms
            r = now_ms()
            self.params["reference_date"] = r
        return int(r)

    def transform_columns(self, *cols, ds=None):
        p = self.params
        pv = p["pivot"]
        tfs = self.get_transient_features() if self._inputs else []
        dev = _device(cols)
        dtype = vector_dtype(dev)
        tn = p["track_nulls"]
        if pv in ("SinceLast", "SinceFirst"):
            cm = []
            for t in tfs:
                cm.append(col_meta(t))
                if tn:
                    cm.append(col_meta(t, is_null=True))
            self.metadata["vector_metadata"] = self.vector_metadata(cm) if tfs else None
            ref = self._ref()
            parts = []
            for c in cols:
                d, ok = _date_reduce(c, pv == "SinceFirst", dev)
                days = torch.div(ref - d, 86400000, rounding_mode="trunc").to(torch.float64)
                parts.append(torch.where(ok, days, torch.full_like(days, float(p["fill_value"]))))
                if tn:
                    parts.append((~ok).to(torch.float64))
            return self._vec(torch.stack(parts, 1).to(dtype))
        # mode pivots
        names = {"ModeDay": ["Monday", "Tuesday", "Wednesday", "Thursday", "Friday", "Saturday", "Sunday"],
                 "ModeMonth": ["January", "February", "March", "April", "May", "June", "July", "August",
                               "September", "October", "November", "December"],
                 "ModeHour": [f"{h}:00" for h in range(24)]}[pv]
        allnames = names + ([NULL_STRING] if tn else [])
        self.metadata["vector_metadata"] = self.vector_metadata(
            [OpVectorColumnMetadata((t.name,), (t.type_name,), t.name, v, None) for t in tfs for v in allnames]) \
            if tfs else None
        blocks = []
        for c in cols:
            lists = c.to_list() if not isinstance(c, NumericColumn) else [[v] if v is not None else []
                                                                          for v in c.to_list()]
            b = np.zeros((len(lists), len(allnames)))
            for r, l in enumerate(lists):
                if not l:
                    if tn:
                        b[r, -1] = 1.0
                    continue
                vals = period_values(torch.as_tensor(l, dtype=torch.int64),
                                     {"ModeDay": "DayOfWeek", "ModeMonth": "MonthOfYear",
                                      "ModeHour": "HourOfDay"}[pv], raw=True)[0].tolist()
                cnt = Counter(vals)
                mode = min(cnt.items(), key=lambda kv: (-kv[1], kv[0]))[0]
                b[r, mode - (0 if pv == "ModeHour" else 1)] = 1.0
            blocks.append(torch.as_tensor(b, dtype=dtype, device=dev))
        return self._vec(torch.cat(blocks, 1))


def _date_reduce(c, first: bool, dev):
    if isinstance(c, NumericColumn):
        return c.values.to(torch.int64), c.valid
    vals = c.to_list()
    ok = np.array([bool(v) for v in vals], dtype=bool)
    d = np.array([(min(v) if first else max(v)) if v else 0 for v in vals], np.int64)
    return torch.as_tensor(d, device=dev), torch.as_tensor(ok, device=dev)


# ------------------------------------------------------------------------------------------------ geo
GEO_NAMES = ("lat", "lon", "accuracy")


@register_stage
class GeolocationVectorizerModel(VectorizerMixin, SequenceTransformer):
    operation_name = "vecGeo"

    def __init__(self, fill_values=None, track_nulls=True, uid=None, **kw):
        super().__init__(uid=uid, **kw)
        self.fill_values = [list(f) for f in (fill_values or [])]
        self.track_nulls = track_nulls

    def transform_columns(self, *cols, ds=None):
        dev = _device(cols)
        parts = []
        for c, f in zip(cols, self.fill_values):
            fill = torch.as_tensor(f if f else [0.0, 0.0, 0.0], dtype=torch.float64, device=dev)
            v = torch.where(c.valid[:, None], c.values.to(torch.float64), fill[None, :])
            parts.append(v)
            if self.track_nulls:
                parts.append((~c.valid).to(torch.float64)[:, None])
        return self._vec(torch.cat(parts, 1).to(vector_dtype(dev)))

    def ctor_args(self):
        return {"fillValues": self.fill_values, "trackNulls": self.track_nulls}

    def load_ctor_args(self, a):
        self.fill_values, self.track_nulls = a["fillValues"], a["trackNulls"]


@register_stage
class GeolocationVectorizer(VectorizerMixin, SequenceEstimator):
    operation_name = "vecGeo"
    _defaults = {"fill_with_constant": False, "fill_value": [0.0, 0.0, 0.0], "track_nulls": True}
    # the geographic midpoint is a monoid (features/geo.py: WGS84 point sums, count, accuracy box): partial results
    # reduce over the ranks as one sum, one min and one max (GeolocationVectorizer.scala:80-92)
    dp_aware = True

    def fit_columns(self, *cols, ds=None):
        from ...features import geo
        fills = []
        if cols:
            stats = geo.all_reduce(torch.stack([geo.reduce_rows(geo.prepare(c.values[c.valid])) for c in cols]))
            stats = stats.cpu()
        for i, c in enumerate(cols):
            if self.params["fill_with_constant"]:
                fills.append(list(self.params["fill_value"]))
                continue
            fills.append(geo.present(stats[i]))
        cm = []
        for t in self.get_transient_features():
            cm += [col_meta(t, descriptor=nm) for nm in GEO_NAMES]
            if self.params["track_nulls"]:
                cm.append(col_meta(t, is_null=True))
        self.metadata["vector_metadata"] = self.vector_metadata(cm)
        return GeolocationVectorizerModel(fills, self.params["track_nulls"])


# ------------------------------------------------------------------------------------------ combiner
@register_stage
class VectorsCombinerModel(VectorizerMixin, SequenceTransformer):
    operation_name = "combVec"

    def transform_columns(self, *cols, ds=None):
        dev = _device(cols)
        dtype = vector_dtype(dev)
        meta = self.metadata.get("vector_metadata")
        if meta is None:
            metas = [c.metadata for c in cols]
            if all(m is not None for m in metas):
                meta = OpVectorMetadata.flatten(self.get_output_feature_name(), metas)
                self.metadata["vector_metadata"] = meta
        if not cols:
            return VectorColumn(torch.zeros(0, 0), meta)
        # concatenation as a blocked view of the inputs' own storage: no copy of the feature matrix
        blocks = [(t if t.dtype == dtype else t.to(dtype), ci) for c in cols for t, ci in c.blocks]
        return VectorColumn(metadata=meta, blocks=blocks)


@register_stage
class VectorsCombiner(VectorizerMixin, SequenceEstimator):
    """Concatenate vectors and merge their column metadata (``VectorsCombiner.scala:51-89``)."""
    operation_name = "combVec"
    dp_aware = True     # metadata only: nothing to reduce

    def fit_columns(self, *cols, ds=None):
        metas = []
        for c, t in zip(cols, self.get_transient_features()):
            if c.metadata is not None:
                metas.append(c.metadata)
            else:
                metas.append(OpVectorMetadata(t.name, [OpVectorColumnMetadata((t.name,), (t.type_name,), t.name)
                                                       for _ in range(c.width)], {}))
        self.metadata["vector_metadata"] = OpVectorMetadata.flatten(self.get_output_feature_name(), metas)
        return VectorsCombinerModel()

"""Joined readers: combine the raw features of two readers on the record key.

Reference: ``JoinedDataReader`` (``readers/.../JoinedDataReader.scala:54-442``; inner / left / outer joins,
``JoinKeys``, ``TimeBasedFilter`` for joined aggregate readers) and ``Reader.innerJoin/leftOuterJoin/
outerJoin`` (``Reader.scala:96-168``). Each side produces its own columnar dataset (for the raw features
it owns); the join is a key -> row-index mapping applied as gathers on the columns, so device columns
never leave the device.
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np
import torch

from ..data.columns import column_from_values
from ..data.dataset import Dataset
from .base import DataReader


class JoinTypes:
    Inner, LeftOuter, Outer = "inner", "left", "outer"


KEY_FIELD = "key"
COMBINED_KEY = "combinedKey"


@dataclass(frozen=True)
class JoinKeys:
    """Join keys (``JoinedDataReader.scala:97-126``): ``left_key`` / ``right_key`` name the record key
    (``"key"``) or a raw feature column holding the other side's key; ``result_key`` is ``"key"`` for
    parent-child / child-parent joins and ``"combinedKey"`` for two tables describing the same object."""
    left_key: str = KEY_FIELD
    right_key: str = KEY_FIELD
    result_key: str = COMBINED_KEY

    @property
    def is_parent_child(self) -> bool:
        return self.result_key == KEY_FIELD and self.left_key == KEY_FIELD and self.right_key != KEY_FIELD

    @property
    def is_child_parent(self) -> bool:
        return self.result_key == KEY_FIELD and self.left_key != KEY_FIELD and self.right_key == KEY_FIELD

    @property
    def is_combined(self) -> bool:
        return self.result_key == COMBINED_KEY and self.left_key == KEY_FIELD and self.right_key == KEY_FIELD


@dataclass(frozen=True)
class TimeColumn:
    """A time column of the joined data (``JoinedDataReader.scala:54-60``); ``keep=False`` drops it from
    the aggregated result."""
    name: str
    keep: bool = True


@dataclass(frozen=True)
class TimeBasedFilter:
    """Conditional aggregation filter after a join (``JoinedDataReader.scala:69-74``): an event of a
    predictor counts when ``condition - window < primary < condition``, an event of a response when
    ``condition <= primary < condition + window`` (``JoinedConditionalAggregator.update``)."""
    condition: TimeColumn
    primary: TimeColumn
    time_window_ms: int


def _name_of(f):
    return f if isinstance(f, str) else f.name


def _owned(reader: DataReader, feats, names: Optional[Sequence[str]]):
    if names is not None:
        s = set(names)
        return [f for f in feats if f.name in s]
    return None


class JoinedReader(DataReader):
    def __init__(self, left: DataReader, right: DataReader, join_type: str = JoinTypes.LeftOuter,
                 right_features: Optional[Sequence[str]] = None, left_features: Optional[Sequence[str]] = None,
                 device=None, join_keys: Optional[JoinKeys] = None):
        super().__init__(None, device or left.device)
        if join_type not in (JoinTypes.Inner, JoinTypes.LeftOuter, JoinTypes.Outer):
            raise ValueError(f"unknown join type {join_type}")
        self.left, self.right = left, right
        self.join_type = join_type
        self.right_features = right_features
        self.left_features = left_features
        self.join_keys = join_keys or JoinKeys()
        jk = self.join_keys
        if not (jk.is_combined or jk.is_parent_child or jk.is_child_parent):
            raise ValueError(f"Invalid key combination: {jk}")

    def inner_join(self, other: DataReader, **kw) -> "JoinedReader":
        return JoinedReader(self, other, JoinTypes.Inner, **kw)

    def left_join(self, other: DataReader, **kw) -> "JoinedReader":
        return JoinedReader(self, other, JoinTypes.LeftOuter, **kw)

    def outer_join(self, other: DataReader, **kw) -> "JoinedReader":
        return JoinedReader(self, other, JoinTypes.Outer, **kw)

    def with_secondary_aggregation(self, time_filter: TimeBasedFilter) -> "JoinedAggregateReader":
        """Aggregate the joined rows per result key (``JoinedDataReader.withSecondaryAggregation``)."""
        return JoinedAggregateReader(self.left, self.right, self.join_type, self.right_features,
                                     self.left_features, self.device, self.join_keys, time_filter)

    def _split(self, raw_features):
        rf = _owned(self.right, raw_features, self.right_features)
        lf = _owned(self.left, raw_features, self.left_features)
        if rf is None and lf is None:
            raise ValueError("JoinedReader needs right_features (or left_features) to assign raw features")
        if rf is None:
            rf = [f for f in raw_features if f not in lf]
        if lf is None:
            lf = [f for f in raw_features if f not in rf]
        return lf, rf

    def _join_index(self, L: Dataset, R: Dataset):
        """(result keys, left row per result row or -1, right row per result row or -1): a relational join
        (every matching pair of rows) on the configured keys."""
        jk = self.join_keys

        def keys_of(ds, k):
            if k == KEY_FIELD:
                if ds.key is None:
                    raise ValueError("both sides of a join need record keys")
                return [None if v is None else str(v) for v in ds.key]
            return [None if v is None else str(v) for v in ds[k].to_list()]

        lk, rk = keys_of(L, jk.left_key), keys_of(R, jk.right_key)
        rpos: dict = {}
        for i, k in enumerate(rk):
            if k is not None:
                rpos.setdefault(k, []).append(i)
        keys, li, ri = [], [], []
        matched_r = set()
        lkeys_res = keys_of(L, KEY_FIELD) if jk.is_child_parent else lk
        for i, k in enumerate(lk):
            ms = rpos.get(k, []) if k is not None else []
            if ms:
                for j in ms:
                    keys.append(lkeys_res[i])
                    li.append(i)
                    ri.append(j)
                    matched_r.add(j)
            elif self.join_type in (JoinTypes.LeftOuter, JoinTypes.Outer):
                keys.append(lkeys_res[i])
                li.append(i)
                ri.append(-1)
        if self.join_type == JoinTypes.Outer:
            rkeys_res = rk if jk.is_combined else keys_of(R, KEY_FIELD)
            for j in range(len(rk)):
                if j not in matched_r:
                    keys.append(rkeys_res[j] if jk.is_combined else (rk[j] if jk.is_parent_child else rkeys_res[j]))
                    li.append(-1)
                    ri.append(j)
        return keys, np.asarray(li, np.int64), np.asarray(ri, np.int64)

    def _joined(self, raw_features, params=None):
        lf, rf = self._split(list(raw_features))
        jk = self.join_keys
        extra_l = [jk.left_key] if jk.left_key != KEY_FIELD and jk.left_key not in {f.name for f in lf} else []
        extra_r = [jk.right_key] if jk.right_key != KEY_FIELD and jk.right_key not in {f.name for f in rf} else []
        if extra_l or extra_r:
            raise ValueError(f"join key column(s) {extra_l + extra_r} must be raw features of their reader")
        L = self.left.generate_dataset(lf, params)
        R = self.right.generate_dataset(rf, params)
        keys, li, ri = self._join_index(L, R)
        cols = OrderedDict()
        for ds, idx, feats in ((L, li, lf), (R, ri, rf)):
            for f in feats:
                c = ds[f.name]
                if idx.size and (idx >= 0).all():
                    cols[f.name] = c.take(torch.as_tensor(idx))
                else:
                    vals = c.to_list()
                    cols[f.name] = column_from_values(f.wtype, [vals[i] if i >= 0 else None for i in idx], c.device)
        return keys, cols, lf, rf

    def generate_dataset(self, raw_features, params=None) -> Dataset:
        keys, cols, _, _ = self._joined(raw_features, params)
        return Dataset(cols, np.asarray(keys, dtype=object), len(keys))


class JoinedAggregateReader(JoinedReader):
    """Join, then aggregate the joined rows per result key with each raw feature's monoid under a
    :class:`TimeBasedFilter` (``JoinedAggregateDataReader``, ``JoinedDataReader.scala:234-330``):
    right (child) features and, for combined joins, left features use the conditional aggregator; the
    left (parent) features of a parent-child join keep one copy per key."""

    def __init__(self, left, right, join_type=JoinTypes.LeftOuter, right_features=None, left_features=None,
                 device=None, join_keys=None, time_filter: Optional[TimeBasedFilter] = None):
        super().__init__(left, right, join_type, right_features, left_features, device, join_keys)
        if time_filter is None:
            raise ValueError("JoinedAggregateReader needs a TimeBasedFilter")
        self.time_filter = time_filter

    def generate_dataset(self, raw_features, params=None) -> Dataset:
        from ..features import aggregators as A
        from ..features.aggregators import Event
        keys, cols, lf, rf = self._joined(raw_features, params)
        tf = self.time_filter
        for tc in (tf.condition, tf.primary):
            if tc.name not in cols:
                raise ValueError(f"time column {tc.name} is not a raw feature of the join")
        n = len(keys)
        prim = [0 if v is None else int(v) for v in cols[tf.primary.name].to_list()]
        cond = [0 if v is None else int(v) for v in cols[tf.condition.name].to_list()]
        order: "OrderedDict[str, list]" = OrderedDict()
        for i, k in enumerate(keys):
            order.setdefault(k, []).append(i)
        gkeys = list(order.keys())
        dummy_left = not self.join_keys.is_combined
        out = OrderedDict()
        dev = self.device
        for f in list(lf) + list(rf):
            vals = cols[f.name].to_list()
            if f in lf and dummy_left:
                res = [vals[rows[-1]] for rows in order.values()]
            else:
                st = f.origin_stage
                agg = st.aggregator or A.default_aggregator(f.wtype)
                win = st.aggregate_window if st.aggregate_window is not None else tf.time_window_ms
                res = []
                for rows in order.values():
                    evs = []
                    for i in rows:
                        t, c = prim[i], cond[i]
                        ok = (t >= c and t < c + win) if f.is_response else (t < c and t > c - win)
                        if ok and vals[i] is not None:
                            evs.append(Event(t, vals[i], f.is_response))
                    res.append(agg.aggregate(evs))
            out[f.name] = column_from_values(f.wtype, res, dev or cols[f.name].device)
        for tc in (tf.condition, tf.primary):
            if not tc.keep:
                out.pop(tc.name, None)
        return Dataset(out, np.asarray(gkeys, dtype=object), len(gkeys))

"""Joined readers: combine the raw features of two readers on the record key.

Reference: ``JoinedDataReader`` (``readers/.../JoinedDataReader.scala:54-442``; inner / left / outer joins,
``JoinKeys``, ``TimeBasedFilter`` for joined aggregate readers) and ``Reader.innerJoin/leftOuterJoin/
outerJoin`` (``Reader.scala:96-168``). Each side produces its own columnar dataset (for the raw features
it owns); the join is a key -> row-index mapping applied as gathers on the columns, so device columns
never leave the device.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Optional, Sequence

import numpy as np
import torch

from ..data.columns import column_from_values
from ..data.dataset import Dataset
from .base import DataReader


class JoinTypes:
    Inner, LeftOuter, Outer = "inner", "left", "outer"


def _owned(reader: DataReader, feats, names: Optional[Sequence[str]]):
    if names is not None:
        s = set(names)
        return [f for f in feats if f.name in s]
    return None


class JoinedReader(DataReader):
    def __init__(self, left: DataReader, right: DataReader, join_type: str = JoinTypes.LeftOuter,
                 right_features: Optional[Sequence[str]] = None, left_features: Optional[Sequence[str]] = None,
                 device=None):
        super().__init__(None, device or left.device)
        if join_type not in (JoinTypes.Inner, JoinTypes.LeftOuter, JoinTypes.Outer):
            raise ValueError(f"unknown join type {join_type}")
        self.left, self.right = left, right
        self.join_type = join_type
        self.right_features = right_features
        self.left_features = left_features

    def inner_join(self, other: DataReader, **kw) -> "JoinedReader":
        return JoinedReader(self, other, JoinTypes.Inner, **kw)

    def left_join(self, other: DataReader, **kw) -> "JoinedReader":
        return JoinedReader(self, other, JoinTypes.LeftOuter, **kw)

    def outer_join(self, other: DataReader, **kw) -> "JoinedReader":
        return JoinedReader(self, other, JoinTypes.Outer, **kw)

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

    def generate_dataset(self, raw_features, params=None) -> Dataset:
        lf, rf = self._split(list(raw_features))
        L = self.left.generate_dataset(lf, params)
        R = self.right.generate_dataset(rf, params)
        if L.key is None or R.key is None:
            raise ValueError("both sides of a join need record keys")
        lk = [str(k) for k in L.key]
        rk = [str(k) for k in R.key]
        rpos = {}
        for i, k in enumerate(rk):
            rpos.setdefault(k, i)
        lset = set(lk)
        if self.join_type == JoinTypes.Inner:
            keys = [k for k in lk if k in rpos]
        elif self.join_type == JoinTypes.LeftOuter:
            keys = list(lk)
        else:
            keys = list(lk) + sorted(set(rk) - lset)
        lpos = {}
        for i, k in enumerate(lk):
            lpos.setdefault(k, i)
        li = np.asarray([lpos.get(k, -1) for k in keys], np.int64)
        ri = np.asarray([rpos.get(k, -1) for k in keys], np.int64)
        cols = OrderedDict()
        for side, ds, idx, feats in ((0, L, li, lf), (1, R, ri, rf)):
            for f in feats:
                c = ds[f.name]
                if (idx >= 0).all():
                    cols[f.name] = c.take(torch.as_tensor(idx))
                else:
                    vals = c.to_list()
                    cols[f.name] = column_from_values(f.wtype, [vals[i] if i >= 0 else None for i in idx], c.device)
        return Dataset(cols, np.asarray(keys, dtype=object), len(keys))

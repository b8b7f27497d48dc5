"""Columnar dataset: the replacement for a Spark ``DataFrame`` with a ``key`` column.

A :class:`Dataset` is an ordered mapping ``feature name -> Column`` plus an optional record key
(reference key column name ``key``, ``readers/.../DataFrameFieldNames.scala:37``). Columns of a
dataset that lives on a GPU keep their tensors in HBM; host-only kinds (ragged collections,
vocabularies) stay on the host.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, Iterable, Optional

import numpy as np
import torch

from .columns import Column, column_from_values

KEY_FIELD = "key"


class Dataset:
    def __init__(self, columns: Optional[Dict[str, Column]] = None, key: Optional[np.ndarray] = None,
                 n_rows: Optional[int] = None, row_ids: Optional[torch.Tensor] = None):
        self.columns: "OrderedDict[str, Column]" = OrderedDict(columns or {})
        lens = {len(c) for c in self.columns.values()}
        if len(lens) > 1:
            raise ValueError(f"columns have different lengths: { {k: len(c) for k, c in self.columns.items()} }")
        if n_rows is None:
            n_rows = lens.pop() if lens else (0 if key is None else len(key))
        self.n_rows = int(n_rows)
        if key is not None and len(key) != self.n_rows:
            raise ValueError("key length mismatch")
        self.key = key
        # global row ids (stable across shards / subsets): drive every seeded per-row decision
        self._row_ids = row_ids
        # True when this is one rank's row shard of a table split across a process group
        # (parallel/dp.py): estimator fits then reduce their statistics over the ranks
        self.sharded = False

    @property
    def row_ids(self) -> torch.Tensor:
        if self._row_ids is None:
            self._row_ids = torch.arange(self.n_rows, device=self.device)
        return self._row_ids

    def __len__(self):
        return self.n_rows

    def __contains__(self, name):
        return name in self.columns

    def __getitem__(self, name) -> Column:
        try:
            return self.columns[name]
        except KeyError:
            raise KeyError(f"column '{name}' not in dataset (has {list(self.columns)})") from None

    @property
    def names(self):
        return list(self.columns.keys())

    @property
    def device(self):
        for c in self.columns.values():
            d = c.device
            if d.type != "cpu":
                return d
        return torch.device("cpu")

    def with_column(self, name: str, col: Column) -> "Dataset":
        if len(col) != self.n_rows:
            raise ValueError(f"column '{name}' has {len(col)} rows, dataset has {self.n_rows}")
        cols = OrderedDict(self.columns)
        cols[name] = col
        return self._like(Dataset(cols, self.key, self.n_rows, self._row_ids))

    def with_columns(self, new: Dict[str, Column]) -> "Dataset":
        cols = OrderedDict(self.columns)
        for k, v in new.items():
            if len(v) != self.n_rows:
                raise ValueError(f"column '{k}' has {len(v)} rows, dataset has {self.n_rows}")
            cols[k] = v
        return self._like(Dataset(cols, self.key, self.n_rows, self._row_ids))

    def select(self, names: Iterable[str]) -> "Dataset":
        return self._like(Dataset(OrderedDict((n, self.columns[n]) for n in names), self.key, self.n_rows,
                                  self._row_ids))

    def drop(self, names: Iterable[str]) -> "Dataset":
        names = set(names)
        return self._like(Dataset(OrderedDict((k, v) for k, v in self.columns.items() if k not in names), self.key,
                                  self.n_rows, self._row_ids))

    def _like(self, other: "Dataset") -> "Dataset":
        other.sharded = self.sharded
        return other

    def shard(self, rank: int, world: int) -> "Dataset":
        """Contiguous row shard ``rank`` of ``world`` with the global row ids kept, marked ``sharded``: the
        data-parallel layout of SURVEY.md §2.8 (each GPU holds ``N / world`` rows, fit statistics are
        all-reduced, see parallel/dp.py)."""
        n = self.n_rows
        a, b = (n * rank) // world, (n * (rank + 1)) // world
        idx = torch.arange(a, b, device=self.row_ids.device)
        cols = OrderedDict((k, v.take(idx)) for k, v in self.columns.items())
        key = None if self.key is None else self.key[a:b]
        out = Dataset(cols, key, b - a, self.row_ids[a:b])
        out.sharded = world > 1
        return out

    def take(self, idx) -> "Dataset":
        if isinstance(idx, torch.Tensor):
            idx_np = idx.detach().cpu().numpy()
        else:
            idx_np = np.asarray(idx, dtype=np.int64)
        cols = OrderedDict((k, v.take(idx)) for k, v in self.columns.items())
        key = None if self.key is None else self.key[idx_np]
        rid = self.row_ids
        return self._like(Dataset(cols, key, len(idx_np), rid[torch.as_tensor(idx_np, device=rid.device)]))

    def to(self, device) -> "Dataset":
        return self._like(Dataset(OrderedDict((k, v.to(device)) for k, v in self.columns.items()), self.key,
                                  self.n_rows, None if self._row_ids is None else self._row_ids.to(device)))

    @staticmethod
    def concat(parts) -> "Dataset":
        parts = list(parts)
        names = parts[0].names
        cols = OrderedDict((n, Column.concat([p[n] for p in parts])) for n in names)
        keys = None if any(p.key is None for p in parts) else np.concatenate([p.key for p in parts])
        rids = torch.cat([p.row_ids.to(parts[0].row_ids.device) for p in parts])
        return Dataset(cols, keys, row_ids=rids)

    # ------------------------------------------------------------------------------------ conversion
    @staticmethod
    def from_rows(rows, features, device="cpu", key=None) -> "Dataset":
        """Build from a list of ``{feature name: python value}`` dicts."""
        cols = OrderedDict()
        for f in features:
            cols[f.name] = column_from_values(f.wtype, [r.get(f.name) for r in rows], device)
        return Dataset(cols, None if key is None else np.asarray(key, dtype=object), len(rows))

    def row(self, i: int, names=None) -> dict:
        names = names or self.names
        return {n: self.columns[n].row(i) for n in names}

    def to_rows(self, names=None):
        names = names or self.names
        lists = {n: self.columns[n].to_list() for n in names}
        return [{n: lists[n][i] for n in names} for i in range(self.n_rows)]

    def to_pandas(self, names=None):
        import pandas as pd
        names = names or self.names
        data = OrderedDict()
        if self.key is not None:
            data[KEY_FIELD] = list(self.key)
        for n in names:
            data[n] = self.columns[n].to_list()
        return pd.DataFrame(data)

    def __repr__(self):
        return f"Dataset(n_rows={self.n_rows}, columns={self.names})"

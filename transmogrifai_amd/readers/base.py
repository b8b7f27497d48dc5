"""Data readers: records / DataFrames / files -> columnar raw-feature datasets.

Reference: ``Reader`` / ``DataReader`` (``readers/.../Reader.scala:42-180``, ``DataReader.scala:57-198``):
``generateDataFrame`` produces a ``key`` column plus one column per raw feature by applying each raw
feature's extract function. Here that is columnar: when a raw feature has no custom extract
function its column is taken directly (vectorized) from the source table; otherwise the extract
function runs per record on the host. The resulting columns can be placed on a GPU in one copy.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Any, Callable, Iterable, List, Optional, Sequence

import numpy as np
import torch

from ..config import default_device
from ..data.columns import Column, NumericColumn, TextColumn, column_from_values
from ..data.dataset import Dataset
from ..features import types as T


def column_from_series(ftype, series, device) -> Column:
    """Vectorized pandas Series -> Column conversion for numeric / text types."""
    import pandas as pd
    if ftype.kind == "numeric":
        if issubclass(ftype, T.Binary):
            vals = series.map(lambda v: None if v is None or (isinstance(v, float) and v != v) else bool(v))
            valid = vals.notna().to_numpy()
            arr = vals.fillna(False).astype(bool).to_numpy()
            return NumericColumn(ftype, torch.as_tensor(arr, device=device), torch.as_tensor(valid, device=device))
        if pd.api.types.is_datetime64_any_dtype(series.dtype):
            valid = series.notna().to_numpy()
            arr = series.astype("int64").to_numpy() // 1_000_000
            return NumericColumn(ftype, torch.as_tensor(arr, device=device), torch.as_tensor(valid, device=device))
        num = pd.to_numeric(series, errors="coerce")
        valid = num.notna().to_numpy()
        if issubclass(ftype, T.Integral):
            arr = num.fillna(0).to_numpy().astype(np.int64)
        else:
            arr = num.fillna(0.0).to_numpy().astype(np.float64)
        if not ftype.nullable and not valid.all():
            raise T.NonNullableEmptyException(f"{ftype.__name__} column '{series.name}' contains empty values")
        return NumericColumn(ftype, torch.as_tensor(arr, device=device), torch.as_tensor(valid, device=device))
    if ftype.kind == "text":
        s = series.astype(object).where(series.notna(), None)
        s = s.map(lambda v: v if v is None else (str(int(v)) if isinstance(v, float) and v.is_integer() else str(v)))
        codes, uniq = pd.factorize(s, use_na_sentinel=True)
        return TextColumn(ftype, torch.as_tensor(codes.astype(np.int32), device=device), [str(u) for u in uniq])
    return column_from_values(ftype, list(series), device)


class DataReader:
    """Base reader. Subclasses implement :meth:`read_records` or :meth:`read_frame`."""

    # the record type the reader reads (the reference's ``Reader.typeName``): when set, only the OpParams reader
    # params under that key apply to this reader (``Reader.getReaderParams``, Reader.scala:69); unset, the first
    # reader params entry does
    type_name: Optional[str] = None

    def __init__(self, key: Optional[Callable] = None, device=None):
        self.key_fn = key
        self.device = torch.device(device) if device is not None else None

    def reader_params_of(self, op_params):
        """This reader's ``ReaderParams`` from a workflow's ``OpParams`` (None when none apply)."""
        rps = getattr(op_params, "reader_params", None) or {}
        if not rps:
            return None
        tn = self.type_name or getattr(getattr(self, "source", None), "type_name", None)
        if tn is not None:
            return rps.get(tn)
        return next(iter(rps.values()))

    def read_records(self, params=None) -> Optional[List[Any]]:
        return None

    def read_frame(self, params=None):
        return None

    def read_dataset(self, params=None) -> Optional[Dataset]:
        return None

    def generate_dataset(self, raw_features: Sequence, params=None) -> Dataset:
        dev = self.device or default_device()
        ds = self.read_dataset(params)
        if ds is not None:
            return _select_raw(ds, raw_features, dev)
        frame = self.read_frame(params)
        if frame is not None:
            return dataset_from_frame(frame, raw_features, dev, self.key_fn)
        recs = self.read_records(params)
        if recs is None:
            raise ValueError("reader produced no data")
        return dataset_from_records(recs, raw_features, dev, self.key_fn)


def _select_raw(ds: Dataset, raw_features, dev) -> Dataset:
    cols = OrderedDict()
    for f in raw_features:
        st = f.origin_stage
        name = getattr(st, "column", None) or f.name
        if name not in ds:
            raise KeyError(f"raw feature '{f.name}' (column '{name}') not in input dataset")
        c = ds[name]
        cols[f.name] = c if c.device == torch.device(dev) or c.device.type == "cpu" and dev.type == "cpu" else c.to(dev)
    return ds._like(Dataset(cols, ds.key, ds.n_rows, ds._row_ids))


def dataset_from_frame(df, raw_features, dev, key_fn=None) -> Dataset:
    cols = OrderedDict()
    records = None
    for f in raw_features:
        st = f.origin_stage
        if st.extract_fn is None and st.column in df.columns:
            cols[f.name] = column_from_series(f.wtype, df[st.column], dev)
        else:
            if records is None:
                records = df.to_dict("records")
            cols[f.name] = column_from_values(f.wtype, [st.extract(r) for r in records], dev)
    key = None
    if key_fn is not None:
        if records is None:
            records = df.to_dict("records")
        key = np.asarray([str(key_fn(r)) for r in records], dtype=object)
    elif "key" in df.columns:
        key = df["key"].astype(str).to_numpy(dtype=object)
    return Dataset(cols, key, len(df))


def dataset_from_records(records, raw_features, dev, key_fn=None) -> Dataset:
    records = list(records)
    cols = OrderedDict()
    for f in raw_features:
        st = f.origin_stage
        cols[f.name] = column_from_values(f.wtype, [st.extract(r) for r in records], dev)
    key = None if key_fn is None else np.asarray([str(key_fn(r)) for r in records], dtype=object)
    return Dataset(cols, key, len(records))


class InMemoryReader(DataReader):
    """``CustomReader``: records, a pandas DataFrame or a columnar :class:`Dataset`."""

    def __init__(self, data, key=None, device=None):
        super().__init__(key, device)
        self.data = data

    def read_dataset(self, params=None):
        return self.data if isinstance(self.data, Dataset) else None

    def read_frame(self, params=None):
        try:
            import pandas as pd
            if isinstance(self.data, pd.DataFrame):
                return self.data
        except ImportError:
            pass
        return None

    def read_records(self, params=None):
        return list(self.data)

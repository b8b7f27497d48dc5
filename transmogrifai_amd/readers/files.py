"""File readers: CSV (explicit schema or headers), CSV with schema inference, Parquet, Avro.

Reference: ``CSVReaders.scala:54-122``, ``CSVAutoReaders.scala:57-142``, ``ParquetProductReader.scala:47-90``,
``AvroReaders.scala:55-134`` and the ``DataReaders`` factory (``DataReaders.scala:44-278``). Parsing goes
through pandas/pyarrow's native CSV/Parquet engines into a DataFrame, then column-wise into the
columnar dataset (see :mod:`.base`). Avro container files are decoded by :mod:`.avro`.
"""
from __future__ import annotations

import torch

from typing import Callable, List, Optional, Sequence, Tuple

from .base import DataReader


def _require_path(path):
    """The reader's path, the reader params' path overriding it (``DataReader.readPath``: "The path is not
    set" when neither is)."""
    if not path:
        raise ValueError("requirement failed: The path is not set")
    return path


class CSVReader(DataReader):
    """CSV with column names from ``schema`` (``[(name, kind)]`` or names) or the file header."""

    # storage type of real-valued columns: float64 (the reference's double) unless a float32 source is declared --
    # a file written from float32 data (shortest float32 decimals) then reads back bit-identical to it
    real_dtype = torch.float64

    def __init__(self, path: Optional[str] = None, schema: Optional[Sequence] = None, has_header: bool = False,
                 key: Optional[Callable] = None, device=None, separator: str = ","):
        super().__init__(key, device)
        self.path = path
        self.schema = schema
        self.has_header = has_header
        self.separator = separator

    def _names(self):
        if self.schema is None:
            return None
        return [s[0] if isinstance(s, (tuple, list)) else s for s in self.schema]

    def read_frame(self, params=None):
        import pandas as pd
        path = self.path
        if params is not None and getattr(params, "path", None):
            path = params.path
        path = _require_path(path)
        names = self._names()
        dtype = None
        if self.schema is not None and all(isinstance(s, (tuple, list)) for s in self.schema):
            m = {"string": str, "text": str}
            dtype = {n: m[k] for n, k in self.schema if k in m}
        # round-trip float parsing: correctly rounded like Java's Double.parseDouble under Spark's CSV reader
        # (pandas' default fast parser can be one ulp off) and like the Arrow parser of the columnar path
        df = pd.read_csv(path, header=0 if self.has_header else None, names=names, sep=self.separator,
                         dtype=dtype, keep_default_na=True, skipinitialspace=False, float_precision="round_trip")
        return df

    def _path(self, params):
        return _require_path(params.path if (params is not None and getattr(params, "path", None)) else self.path)

    def generate_dataset(self, raw_features, params=None):
        """Columnar fast path (readers/columnar.py csv_dataset: pyarrow's multi-threaded parser -> Arrow columns ->
        pinned row-slice copies -> device) when every raw feature is a plain numeric / string column; the pandas
        path otherwise (TMOG_COLUMNAR=0)."""
        import os
        from ..config import default_device
        path = self._path(params)
        if os.environ.get("TMOG_COLUMNAR", "1") != "0" and isinstance(path, str) and os.path.isfile(path):
            from .columnar import csv_dataset
            text = [n for n, k in self.schema if k in ("string", "text")] \
                if (self.schema is not None and all(isinstance(s, (tuple, list)) for s in self.schema)) else []
            dev = torch.device(self.device or default_device())
            ds = None
            if dev.type == "cuda":          # the whole parse on the device (readers/gpu_csv.py)
                from .gpu_csv import gpu_csv_dataset
                ds = gpu_csv_dataset(path, raw_features, dev, self._names(), self.has_header, self.separator,
                                     self.key_fn, text_columns=text, real_dtype=self.real_dtype)
            if ds is None:
                ds = csv_dataset(path, raw_features, dev, self._names(), self.has_header, self.separator, text,
                                 self.key_fn)
                if ds is not None and self.real_dtype != torch.float64:
                    ds = _cast_reals(ds, self.real_dtype)
            if ds is not None:
                return ds
        return super().generate_dataset(raw_features, params)


def _cast_reals(ds, dtype):
    from ..data.columns import NumericColumn
    for name, c in list(ds.columns.items()):
        if isinstance(c, NumericColumn) and c.values.is_floating_point() and c.values.dtype != dtype:
            ds.columns[name] = NumericColumn(c.ftype, c.values.to(dtype), c.valid)
    return ds


class CSVAutoReader(CSVReader):
    """CSV with a header row and schema inference (``CSVAutoReaders``)."""

    def __init__(self, path=None, key=None, device=None, separator=","):
        super().__init__(path, None, True, key, device, separator)


class ParquetReader(DataReader):
    def __init__(self, path: Optional[str] = None, key=None, device=None):
        super().__init__(key, device)
        self.path = path

    def _path(self, params):
        return _require_path(params.path if (params is not None and getattr(params, "path", None)) else self.path)

    def read_frame(self, params=None):
        import pandas as pd
        return pd.read_parquet(self._path(params))

    def generate_dataset(self, raw_features, params=None):
        """Columnar fast path (readers/columnar.py: Arrow buffers -> pinned row-group copies -> device) when
        every raw feature is a plain numeric / string column; the pandas path otherwise (TMOG_COLUMNAR=0)."""
        import os
        from ..config import default_device
        path = self._path(params)
        if os.environ.get("TMOG_COLUMNAR", "1") != "0" and isinstance(path, str) and os.path.isfile(path):
            from .columnar import parquet_dataset
            ds = parquet_dataset(path, raw_features, self.device or default_device(), self.key_fn)
            if ds is not None:
                return ds
        return super().generate_dataset(raw_features, params)


class AvroReader(DataReader):
    def __init__(self, path: Optional[str] = None, key=None, device=None):
        super().__init__(key, device)
        self.path = path

    def read_records(self, params=None):
        from .avro import read_avro
        path = params.path if (params is not None and getattr(params, "path", None)) else self.path
        return read_avro(_require_path(path))


class DataReaders:
    """``DataReaders.Simple`` / ``.Aggregate`` / ``.Conditional`` factories."""

    class Simple:
        @staticmethod
        def csv(path=None, schema=None, key=None, has_header=False, device=None):
            return CSVReader(path, schema, has_header, key, device)

        @staticmethod
        def csv_case(path=None, schema=None, key=None, device=None):
            return CSVReader(path, schema, False, key, device)

        @staticmethod
        def csv_auto(path=None, key=None, device=None):
            return CSVAutoReader(path, key, device)

        @staticmethod
        def parquet(path=None, key=None, device=None):
            return ParquetReader(path, key, device)

        @staticmethod
        def avro(path=None, key=None, device=None):
            return AvroReader(path, key, device)

        @staticmethod
        def custom(data, key=None, device=None):
            from .base import InMemoryReader
            return InMemoryReader(data, key, device)

    class Aggregate:
        @staticmethod
        def csv(path=None, schema=None, key=None, aggregate_params=None, has_header=False, device=None):
            from .aggregate import AggregateReader
            return AggregateReader(CSVReader(path, schema, has_header, None, device), key, aggregate_params)

        @staticmethod
        def avro(path=None, key=None, aggregate_params=None, device=None):
            from .aggregate import AggregateReader
            return AggregateReader(AvroReader(path, None, device), key, aggregate_params)

        @staticmethod
        def parquet(path=None, key=None, aggregate_params=None, device=None):
            from .aggregate import AggregateReader
            return AggregateReader(ParquetReader(path, None, device), key, aggregate_params)

        @staticmethod
        def custom(data, key=None, aggregate_params=None, device=None):
            from .aggregate import AggregateReader
            from .base import InMemoryReader
            return AggregateReader(InMemoryReader(data, None, device), key, aggregate_params)

    class Conditional:
        @staticmethod
        def csv(path=None, schema=None, key=None, conditional_params=None, has_header=False, device=None):
            from .aggregate import ConditionalReader
            return ConditionalReader(CSVReader(path, schema, has_header, None, device), key, conditional_params)

        @staticmethod
        def avro(path=None, key=None, conditional_params=None, device=None):
            from .aggregate import ConditionalReader
            return ConditionalReader(AvroReader(path, None, device), key, conditional_params)

        @staticmethod
        def parquet(path=None, key=None, conditional_params=None, device=None):
            from .aggregate import ConditionalReader
            return ConditionalReader(ParquetReader(path, None, device), key, conditional_params)

        @staticmethod
        def custom(data, key=None, conditional_params=None, device=None):
            from .aggregate import ConditionalReader
            from .base import InMemoryReader
            return ConditionalReader(InMemoryReader(data, None, device), key, conditional_params)

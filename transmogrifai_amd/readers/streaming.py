"""Streaming readers: micro-batches for ``StreamingScore`` runs.

Reference: ``StreamingReader`` / ``StreamingReaders`` (``readers/.../StreamingReader.scala:40-57``,
``StreamingReaders.scala``) backed by Spark streaming file sources (``AvroReaders.scala:110``). Here a
streaming reader yields columnar micro-batches: new files appearing in a directory (CSV, Parquet,
JSON lines or Avro), or chunks of an in-memory record iterator. Each batch is scored by the
fitted model through the same columnar (device) transforms as batch scoring.
"""
from __future__ import annotations

import glob
import os
import time
from typing import Any, Callable, Iterable, Iterator, List, Optional, Sequence


class StreamingReader:
    def stream(self, params=None) -> Iterator[Any]:
        raise NotImplementedError


class IterableStreamingReader(StreamingReader):
    """Chunks an iterable of records (dicts) into micro-batches of ``batch_size``."""

    def __init__(self, records: Iterable[dict], batch_size: int = 1000):
        self.records = records
        self.batch_size = batch_size

    def stream(self, params=None):
        buf: List[dict] = []
        for r in self.records:
            buf.append(r)
            if len(buf) >= self.batch_size:
                yield buf
                buf = []
        if buf:
            yield buf


class FileStreamingReader(StreamingReader):
    """Treat every new file in ``path`` (matching ``pattern``) as one micro-batch (pandas frame).

    ``poll_secs`` > 0 keeps watching the directory until ``timeout_secs`` elapses without new files
    (``awaitTerminationTimeoutSecs``); with 0 the files present now are read once.
    """

    def __init__(self, path: Optional[str] = None, pattern: str = "*", fmt: Optional[str] = None,
                 poll_secs: float = 0.0, timeout_secs: float = 0.0, schema: Optional[Sequence] = None):
        self.path = path
        self.pattern = pattern
        self.fmt = fmt
        self.poll_secs = poll_secs
        self.timeout_secs = timeout_secs
        self.schema = schema

    def _read(self, f: str):
        import pandas as pd
        fmt = self.fmt or os.path.splitext(f)[1].lstrip(".").lower()
        if fmt in ("csv", "txt"):
            names = None if self.schema is None else [s[0] if isinstance(s, (list, tuple)) else s for s in self.schema]
            return pd.read_csv(f, header=None if names else 0, names=names)
        if fmt in ("parquet", "pq"):
            return pd.read_parquet(f)
        if fmt in ("json", "jsonl"):
            return pd.read_json(f, lines=True)
        if fmt == "avro":
            from .avro import read_avro_records
            return pd.DataFrame(read_avro_records(f))
        raise ValueError(f"unsupported streaming file format {fmt}")

    def stream(self, params=None):
        path = self.path
        if params is not None and getattr(params, "reader_params", None):
            rp = next(iter(params.reader_params.values()))
            path = rp.path or path
        seen = set()
        last_new = time.time()
        while True:
            files = sorted(f for f in glob.glob(os.path.join(path, self.pattern)) if os.path.isfile(f))
            new = [f for f in files if f not in seen]
            for f in new:
                seen.add(f)
                yield self._read(f)
            if new:
                last_new = time.time()
            if self.poll_secs <= 0 or time.time() - last_new > self.timeout_secs:
                return
            time.sleep(self.poll_secs)

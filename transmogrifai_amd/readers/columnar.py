"""Columnar Parquet / CSV -> device ingest (the fast paths of :class:`~.files.ParquetReader` and
:class:`~.files.CSVReader`).

Reference: ``ParquetProductReader.scala:47-90`` / ``DataReader.generateDataFrame`` (``DataReader.scala:57-198``)
read Parquet into a Spark DataFrame of one column per raw feature. The generic path here (:mod:`.base`) goes
through a pandas DataFrame and converts each column on the host (``to_numeric``, ``fillna``, float64), then
copies it to the device -- at 10M x 200 that is tens of seconds of single-threaded host work.

This path keeps the data in Arrow's columnar buffers end to end:

* row groups are decoded by pyarrow's multi-threaded C++ reader, the next one on a prefetch thread while the
  current one is copied;
* each numeric column chunk is copied as its raw value buffer (float32 stays float32 on the GPU -- the
  precision the GPU vectorizers run at) and, when it has nulls, its packed validity bitmap (1 bit per row);
  the chunks of a row group are packed into one pinned host buffer (memcpys on a thread pool) and sent with one
  asynchronous host-to-device copy on a copy stream, double-buffered against the next row group's packing;
* on the device the bitmaps are unpacked, null slots zeroed (the pandas path's ``fillna(0)``) and the values
  scattered into the preallocated columns;
* text columns are dictionary-encoded by Arrow (first-appearance order and -1 for null, exactly
  ``pandas.factorize``), integral columns keep int64.

Columns the fast path does not cover (custom extract functions, Binary / date types, text stored as
non-strings, integral stored as floats) make :func:`parquet_dataset` return ``None`` and the reader falls back
to the pandas path. ``tests/test_columnar_ingest.py`` checks both paths give identical datasets."""
from __future__ import annotations

import concurrent.futures as cf
import os
import time
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..data.columns import NumericColumn, TextColumn
from ..data.dataset import Dataset
from ..features import types as T


def _plan(schema, raw_features):
    """``[(feature, column, kind)]`` with kind in {"real", "int", "text"}, or None if any feature needs the
    generic path."""
    import pyarrow as pa
    out = []
    for f in raw_features:
        st = f.origin_stage
        if st.extract_fn is not None or st.column is None or st.column not in schema.names:
            return None
        at = schema.field(st.column).type
        ft = f.wtype
        if ft.kind == "numeric":
            if issubclass(ft, T.Binary) or not (pa.types.is_floating(at) or pa.types.is_integer(at)):
                return None
            if issubclass(ft, T.Integral):
                if not pa.types.is_integer(at):
                    return None
                out.append((f, st.column, "int"))
            else:
                out.append((f, st.column, "real"))
        elif ft.kind == "text":
            vt = at.value_type if pa.types.is_dictionary(at) else at
            if not (pa.types.is_string(vt) or pa.types.is_large_string(vt)):
                return None
            out.append((f, st.column, "text"))
        else:
            return None
    return out


def _real_dtype(at, dev):
    import pyarrow as pa
    if dev.type == "cuda" and pa.types.is_float32(at):
        return torch.float32
    return torch.float64


def _bitmap_bytes(n):
    return (n + 7) // 8


class _Slot:
    """One pinned staging buffer, the device buffer it is copied into, and the event that marks the copy done."""

    def __init__(self, nbytes, dev):
        self.host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        self.dev = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        self.event = None


class _ParquetSource:
    """Row groups of a Parquet file (decoded on demand by pyarrow's multi-threaded reader)."""

    def __init__(self, path):
        import pyarrow.parquet as pq
        import threading
        self.path = path
        self.text_cols: List[str] = []
        self._tl = threading.local()
        self.pf = pq.ParquetFile(path)
        self.schema = self.pf.schema_arrow
        self.n = self.pf.metadata.num_rows
        self.n_chunks = self.pf.metadata.num_row_groups

    def read(self, i, cols):
        # a ParquetFile is not safe for concurrent reads: every prefetch thread decodes through its own
        import pyarrow.parquet as pq
        pf = getattr(self._tl, "pf", None)
        if pf is None:      # string columns keep their dictionaries (no per-row string materialisation)
            pf = self._tl.pf = pq.ParquetFile(self.path, read_dictionary=self.text_cols or None)
        return pf.read_row_group(i, columns=cols, use_threads=True)

    def read_all(self, cols):
        return self.pf.read(columns=cols, use_threads=True)

    def read_text(self, cols):
        """String columns with their Parquet dictionaries kept (no per-row string materialisation)."""
        import pyarrow.parquet as pq
        return pq.ParquetFile(self.path, read_dictionary=cols).read(columns=cols, use_threads=True)


class _TableSource:
    """An in-memory Arrow table (e.g. a parsed CSV file) fed to the device pipeline in slices of ``rows``."""

    def __init__(self, table, rows: int = 1 << 20):
        self.table = table
        self.schema = table.schema
        self.n = table.num_rows
        self.rows = max(1, rows)
        self.n_chunks = (self.n + self.rows - 1) // self.rows

    def read(self, i, cols):
        return self.table.select(cols).slice(i * self.rows, self.rows)

    def read_all(self, cols):
        return self.table.select(cols)

    read_text = read_all


def parquet_dataset(path: str, raw_features: Sequence, dev, key_fn=None, threads: Optional[int] = None
                    ) -> Optional[Dataset]:
    """Dataset of ``raw_features`` from the Parquet file ``path`` on ``dev``, or None (use the generic path)."""
    try:
        import pyarrow  # noqa: F401
    except ImportError:
        return None
    if key_fn is not None:
        return None
    return _arrow_dataset(_ParquetSource(path), raw_features, torch.device(dev), threads)


# pandas.read_csv's default NA strings (keep_default_na=True): the CSV fast path marks the same cells missing
_PANDAS_NA = ["", "#N/A", "#N/A N/A", "#NA", "-1.#IND", "-1.#QNAN", "-NaN", "-nan", "1.#IND", "1.#QNAN", "<NA>",
              "N/A", "NA", "NULL", "NaN", "None", "n/a", "nan", "null"]


def csv_dataset(path: str, raw_features: Sequence, dev, names: Optional[Sequence[str]] = None,
                has_header: bool = True, separator: str = ",", text_columns: Sequence[str] = (),
                key_fn=None, threads: Optional[int] = None) -> Optional[Dataset]:
    """Dataset of ``raw_features`` from the CSV file ``path`` (``CSVReaders.scala:54-122`` / ``CSVAutoReaders``)
    on ``dev``, or None (use the pandas path): pyarrow's multi-threaded CSV parser builds the Arrow columns,
    which then take the same pinned, double-buffered copy pipeline as Parquet row groups. Numeric features
    parse as float64 / int64 (the pandas path's dtypes), pandas' NA strings are nulls, and a text feature is
    taken only when Arrow types its column as strings (a numeric-looking column keeps the pandas path's
    number-to-text rendering)."""
    try:
        import pyarrow as pa
        import pyarrow.csv as pacsv
    except ImportError:
        return None
    if key_fn is not None:
        return None
    dev = torch.device(dev)
    want = {}
    for f in raw_features:
        st = f.origin_stage
        if st.extract_fn is not None or st.column is None:
            return None
        if f.wtype.kind == "numeric" and not issubclass(f.wtype, T.Binary):
            want[st.column] = pa.int64() if issubclass(f.wtype, T.Integral) else pa.float64()
        elif f.wtype.kind == "text":
            if st.column in text_columns:
                want[st.column] = pa.dictionary(pa.int32(), pa.string())
        else:
            return None
    ro = pacsv.ReadOptions(column_names=list(names) if (names is not None and not has_header) else None,
                           autogenerate_column_names=False, use_threads=True, block_size=1 << 24)
    if names is not None and has_header:
        ro = pacsv.ReadOptions(column_names=list(names), skip_rows=1, use_threads=True, block_size=1 << 24)
    if names is None:               # header names (the first line), to know whether a key column exists
        import csv
        with open(path, newline="") as fh:
            names = next(csv.reader(fh, delimiter=separator), [])
    cols = list(dict.fromkeys(f.origin_stage.column for f in raw_features))
    if any(c not in names for c in cols):
        return None
    co = pacsv.ConvertOptions(column_types=want, null_values=_PANDAS_NA, strings_can_be_null=True,
                              include_columns=cols + (["key"] if "key" in names and "key" not in cols else []))
    try:
        table = pacsv.read_csv(path, read_options=ro, parse_options=pacsv.ParseOptions(delimiter=separator),
                               convert_options=co)
    except (pa.ArrowInvalid, pa.ArrowTypeError, KeyError, ValueError):
        return None            # unparsable numbers, missing columns, ...: the pandas path decides
    return _arrow_dataset(_TableSource(table), raw_features, dev, threads)


def _arrow_dataset(source, raw_features: Sequence, dev: torch.device, threads: Optional[int] = None
                   ) -> Optional[Dataset]:
    import pyarrow as pa
    import pyarrow.compute as pc
    schema = source.schema
    plan = _plan(schema, raw_features)
    if plan is None:
        return None
    n = source.n
    num = [(f, c, k) for f, c, k in plan if k in ("real", "int")]
    txt = [(f, c, k) for f, c, k in plan if k == "text"]
    ncols = list(dict.fromkeys(c for _, c, _ in num))
    tcols = [c for c in dict.fromkeys(c for _, c, _ in txt) if c not in ncols]
    source.text_cols = tcols
    text_chunks: Dict[str, list] = {c: [] for c in tcols}
    types = {c: schema.field(c).type for c in ncols}
    dtype = {c: (torch.int64 if any(k == "int" and cc == c for _, cc, k in num) else _real_dtype(types[c], dev))
             for c in ncols}
    vals = {c: torch.empty(n, dtype=dtype[c], device=dev) for c in ncols}
    valid = {c: None for c in ncols}
    gpu = dev.type == "cuda"
    threads = threads or min(16, os.cpu_count() or 4)
    pool = cf.ThreadPoolExecutor(threads)
    prefetch = cf.ThreadPoolExecutor(max(1, int(os.environ.get("TMOG_INGEST_PREFETCH", "3"))))
    n_rg = source.n_chunks
    t_start = time.perf_counter()
    prof = {"wait_decode": 0.0, "pack": 0.0, "copy_wait": 0.0}

    def read(i):     # numeric and text columns of one row group (text decoded on the prefetch threads too)
        return source.read(i, ncols + tcols) if (ncols or tcols) else None

    def host_chunk(arr, c):
        """(values ndarray in the column's device dtype, validity bitmap bytes or None, bit offset)."""
        want = dtype[c]
        npd = {torch.float32: np.float32, torch.float64: np.float64, torch.int64: np.int64}[want]
        bufs = arr.buffers()
        v = np.frombuffer(bufs[1], dtype=arr.type.to_pandas_dtype(), count=len(arr) + arr.offset)[arr.offset:]
        if v.dtype != npd:
            v = v.astype(npd)
        bm = None
        if arr.null_count > 0:
            bm = np.frombuffer(bufs[0], dtype=np.uint8, count=_bitmap_bytes(len(arr) + arr.offset))
        return v, bm, arr.offset

    slots: List[Optional[_Slot]] = [None, None]
    copy_stream = torch.cuda.Stream(device=dev) if gpu else None
    if gpu:
        # float columns: validity also drops non-null NaNs, decided on the device; columns that turn out
        # all-valid lose their mask after the copies (one host read for all of them)
        for c in ncols:
            if dtype[c].is_floating_point:
                valid[c] = torch.ones(n, dtype=torch.bool, device=dev)
        # the copy stream writes buffers allocated on the caller's stream: order after its queued work
        copy_stream.wait_stream(torch.cuda.current_stream(dev))
    depth = max(1, int(os.environ.get("TMOG_INGEST_PREFETCH", "3")))     # row groups decoded ahead
    futs = [prefetch.submit(read, g) for g in range(min(depth, n_rg))]
    row0 = 0
    try:
        for g in range(n_rg):
            t_w = time.perf_counter()
            tab = futs.pop(0).result()
            prof["wait_decode"] += time.perf_counter() - t_w
            if g + depth < n_rg:
                futs.append(prefetch.submit(read, g + depth))
            if tab is None:
                continue
            for c in tcols:
                text_chunks[c].extend(tab.column(c).chunks)
            rows = tab.num_rows
            pieces = []                  # (column, row offset, values ndarray, bitmap, bit offset)
            for c in ncols:
                r = row0
                for ch in tab.column(c).chunks:
                    pieces.append((c, r) + host_chunk(ch, c))
                    r += len(ch)
            if not gpu:
                for c, r, v, bm, bo in pieces:
                    dst = vals[c][r:r + len(v)]
                    dst.copy_(torch.from_numpy(v))
                    ok = None
                    if bm is not None:
                        ok = torch.from_numpy(np.unpackbits(bm, bitorder="little")[bo:bo + len(v)].astype(bool))
                    if dst.is_floating_point():         # a non-null NaN is missing too (pandas path: notna)
                        fin = ~torch.isnan(dst)
                        if not bool(fin.all()):
                            ok = fin if ok is None else ok & fin
                    if ok is not None:
                        if valid[c] is None:
                            valid[c] = torch.ones(n, dtype=torch.bool)
                        valid[c][r:r + len(v)] = ok
                        dst.masked_fill_(~ok, 0)
                row0 += rows
                continue
            # pack the row group into one pinned buffer (8-byte aligned pieces), one async H2D copy
            layout, off = [], 0
            for c, r, v, bm, bo in pieces:
                vo = off
                off += (v.nbytes + 7) // 8 * 8
                bmo = None
                if bm is not None:
                    bmo = off
                    off += (bm.nbytes + 7) // 8 * 8
                layout.append((c, r, v, bm, bo, vo, bmo))
            k = g & 1
            s = slots[k]
            if s is None or s.host.numel() < off:
                if s is not None and s.event is not None:
                    s.event.synchronize()
                s = slots[k] = _Slot(max(off, 1), dev)
            elif s.event is not None:
                s.event.synchronize()          # the copy of row group g - 2 has left this buffer
            hb = s.host.numpy()

            def pack(item):
                c, r, v, bm, bo, vo, bmo = item
                hb[vo:vo + v.nbytes] = v.view(np.uint8)
                if bm is not None:
                    hb[bmo:bmo + bm.nbytes] = bm

            t_p = time.perf_counter()
            list(pool.map(pack, layout))
            prof["pack"] += time.perf_counter() - t_p
            for c, r, v, bm, bo, vo, bmo in layout:
                if bm is not None and valid[c] is None:     # on the caller's stream, like vals
                    valid[c] = torch.ones(n, dtype=torch.bool, device=dev)
            with torch.cuda.stream(copy_stream):
                s.dev[:off].copy_(s.host[:off], non_blocking=True)
                for c, r, v, bm, bo, vo, bmo in layout:
                    m = len(v)
                    src = s.dev[vo:vo + v.nbytes].view(vals[c].dtype)
                    dst = vals[c][r:r + m]
                    ok = None
                    if bm is not None:
                        bits = s.dev[bmo:bmo + bm.nbytes]
                        ok = ((bits[:, None] >> torch.arange(8, device=dev, dtype=torch.uint8)) & 1).reshape(-1)
                        ok = ok[bo:bo + m].bool()
                    if src.is_floating_point():         # a non-null NaN is missing too (pandas path: notna)
                        fin = ~torch.isnan(src)
                        ok = fin if ok is None else ok & fin
                    if ok is None:
                        dst.copy_(src)
                    else:
                        valid[c][r:r + m] = ok
                        dst.copy_(torch.where(ok, src, torch.zeros_like(src)))
                s.event = torch.cuda.Event()
                s.event.record(copy_stream)
            row0 += rows
        if gpu:
            torch.cuda.current_stream(dev).wait_stream(copy_stream)
            for c in ncols:            # allocated on the caller's stream, written on the copy stream
                vals[c].record_stream(copy_stream)
                if valid[c] is not None:
                    valid[c].record_stream(copy_stream)
            t_c = time.perf_counter()
            for s in slots:
                if s is not None and s.event is not None:
                    s.event.synchronize()
            prof["copy_wait"] += time.perf_counter() - t_c
            masked = [c for c in ncols if valid[c] is not None]
            if masked:
                full = torch.stack([valid[c].all() for c in masked]).tolist()
                for c, f in zip(masked, full):
                    if f:
                        valid[c] = None
    finally:
        pool.shutdown(wait=False)
        prefetch.shutdown(wait=False)
    cols = OrderedDict()
    for f, c, k in plan:
        if k == "text":
            continue
        ok = valid[c]
        if not f.wtype.nullable and ok is not None and not bool(ok.all()):
            raise T.NonNullableEmptyException(f"{f.wtype.__name__} column '{c}' contains empty values")
        cols[f.name] = NumericColumn(f.wtype, vals[c], ok)
    if txt:
        t_t = time.perf_counter()
        enc = {}
        for f, c, _ in txt:
            if c not in enc:
                if c in text_chunks:
                    ch = pa.chunked_array(text_chunks[c]) if text_chunks[c] else pa.chunked_array([], pa.string())
                else:       # a column also read as numbers: its strings separately
                    ch = source.read_all([c]).column(c)
                enc[c] = _encode_text(ch, dev)
            cols[f.name] = TextColumn(f.wtype, *enc[c])
        prof["text"] = time.perf_counter() - t_t
    order = OrderedDict((f.name, cols[f.name]) for f in raw_features)
    key = None
    if "key" in schema.names:
        key = source.read_all(["key"]).column("key").to_pandas().astype(str).to_numpy(dtype=object)
    if os.environ.get("TMOG_INGEST_PROFILE") == "1":
        import sys
        prof["total"] = time.perf_counter() - t_start
        sys.stderr.write("[ingest-profile] " + " ".join(f"{k}={v:.3f}" for k, v in prof.items()) + "\n")
    return Dataset(order, key, n)


def _encode_text(chunked, dev):
    """``(codes, vocab)`` of a string column in ``pandas.factorize`` semantics -- codes in order of first appearance
    over the rows, -1 for null, unused dictionary entries dropped. Dictionary-encoded input (Parquet string columns
    read with their dictionaries, CSV columns parsed as dictionaries) is unified across chunks and its indices are
    reordered by first appearance on the device (a scatter-min of row positions per code), so no per-string
    hashing runs on the host; plain strings are dictionary-encoded by Arrow first."""
    import pyarrow as pa
    import pyarrow.compute as pc
    if not pa.types.is_dictionary(chunked.type):
        chunked = pc.dictionary_encode(chunked)
    chunked = chunked.unify_dictionaries()
    dictionary = chunked.chunk(0).dictionary if chunked.num_chunks else pa.array([], pa.string())
    idx = np.concatenate([pc.fill_null(ch.indices.cast(pa.int32()), -1).to_numpy(zero_copy_only=False)
                          for ch in chunked.chunks]) if chunked.num_chunks else np.zeros(0, np.int32)
    K = len(dictionary)
    codes = torch.as_tensor(idx.astype(np.int32, copy=False), device=dev)
    n = int(codes.numel())
    if K == 0 or n == 0:
        return codes, []
    ok = codes >= 0
    # first appearance of every used code: a stable radix sort of the valid rows' codes (a scatter-min onto the K
    # codes would pile millions of atomics onto a few addresses); each run's first element is its first row
    rows = torch.nonzero(ok).squeeze(1)
    sc, perm = torch.sort(codes[rows], stable=True)
    starts = torch.ones_like(sc, dtype=torch.bool)
    if sc.numel() > 1:
        starts[1:] = sc[1:] != sc[:-1]
    first_row = rows[perm[starts]]
    order = sc[starts][torch.argsort(first_row)].to(torch.int64)      # used codes, by first appearance
    used = int(order.numel())
    remap = torch.full((K,), -1, dtype=torch.int32, device=dev)
    remap[order] = torch.arange(used, dtype=torch.int32, device=dev)
    out = torch.where(ok, remap[codes.clamp_min(0).to(torch.int64)], codes)
    vocab = dictionary.take(pa.array(order.cpu().numpy())).to_pylist()
    return out, [str(u) for u in vocab]


def dataset_to_parquet(ds: Dataset, path: str, row_group_rows: int = 1 << 20, names: Optional[Sequence[str]] = None,
                       compression: str = "snappy") -> None:
    """Write the numeric and text columns of ``ds`` (nulls kept) to a Parquet file, one row group per
    ``row_group_rows`` rows, streaming from the device one row group at a time. Text columns are written
    dictionary-encoded. Used by ``bench.py --ingest parquet`` to put the benchmark table on disk."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    names = list(names) if names is not None else list(ds.columns)
    writer = None
    try:
        for r0 in range(0, ds.n_rows, row_group_rows):
            r1 = min(ds.n_rows, r0 + row_group_rows)
            arrays = []
            for nm in names:
                c = ds[nm]
                if isinstance(c, TextColumn):
                    codes = c.codes[r0:r1].cpu().numpy().astype(np.int32)
                    arrays.append(pa.DictionaryArray.from_arrays(pa.array(codes, mask=codes < 0),
                                                                 pa.array(c.vocab, type=pa.string())))
                else:
                    v = c.values[r0:r1].cpu().numpy()
                    ok = c.valid[r0:r1].cpu().numpy()
                    arrays.append(pa.array(v, mask=None if ok.all() else ~ok))
            tab = pa.Table.from_arrays(arrays, names=names)
            if writer is None:
                writer = pq.ParquetWriter(path, tab.schema, compression=compression)
            writer.write_table(tab, row_group_size=r1 - r0)
    finally:
        if writer is not None:
            writer.close()


def dataset_to_csv(ds: Dataset, path: str, row_group_rows: int = 1 << 20, names: Optional[Sequence[str]] = None) -> None:
    """Write the numeric and text columns of ``ds`` to a CSV file with a header (empty cells for nulls), streaming
    one slice of rows at a time through pyarrow's CSV writer. Used by ``bench.py --ingest csv``."""
    import pyarrow as pa
    import pyarrow.csv as pacsv
    names = list(names) if names is not None else list(ds.columns)
    writer = None
    try:
        for r0 in range(0, ds.n_rows, row_group_rows):
            r1 = min(ds.n_rows, r0 + row_group_rows)
            arrays = []
            for nm in names:
                c = ds[nm]
                if isinstance(c, TextColumn):
                    codes = c.codes[r0:r1].cpu().numpy().astype(np.int64)
                    vocab = np.asarray(list(c.vocab) + [None], dtype=object)
                    arrays.append(pa.array(vocab[np.where(codes < 0, len(c.vocab), codes)], type=pa.string()))
                else:
                    v = c.values[r0:r1].cpu().numpy()
                    ok = c.valid[r0:r1].cpu().numpy()
                    arrays.append(pa.array(v, mask=None if ok.all() else ~ok))
            tab = pa.Table.from_arrays(arrays, names=names)
            if writer is None:
                writer = pacsv.CSVWriter(path, tab.schema)
            writer.write_table(tab)
    finally:
        if writer is not None:
            writer.close()

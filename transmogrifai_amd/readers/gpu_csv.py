"""CSV files parsed on the GPU (the reference's default readers are CSV: ``CSVReaders.scala:54-122``,
``DataReader.scala:173-197``).

The host only moves bytes: the file is read in large chunks (parallel ``preadv`` into pinned buffers, the next chunk
while the device parses the current one), each chunk is cut at its last newline and copied to the device, and
``ops/csrc/hip/csv_kernels.hip`` finds the rows (one ``torch.nonzero`` of the newlines), the fields of every row (one
wave per row, quote-aware ballots) and converts every numeric cell in parallel -- exactly (decimal strings of up to 19
significant digits and ``|exponent| <= 22`` are one correctly rounded IEEE operation; the rare others go to the host's
``float``). Text columns are dictionary-encoded on the device: a 64-bit hash per cell, ``torch.unique`` per column,
codes ordered by first appearance (``pandas.factorize`` semantics, as the Arrow path's ``_encode_text``); only the
distinct strings' bytes come back to the host.

Same dataset as :func:`readers.columnar.csv_dataset` (pyarrow): float64 reals, int64 integers, pandas' NA strings and
empty cells missing, text codes by first appearance. Returns None when the file needs the generic path (a key
function, extract functions, rows with a different field count, types the parser does not produce).
"""
from __future__ import annotations

import concurrent.futures as cf
import csv
import io
import os
import time
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..data.columns import NumericColumn, TextColumn
from ..data.dataset import Dataset
from ..features import types as T

CHUNK = 256 << 20          # bytes per chunk (two pinned + two device buffers)
_READ_SPLIT = 8 << 20      # bytes per parallel pread


def _plan(raw_features, names):
    plan = []
    for f in raw_features:
        st = f.origin_stage
        if st.extract_fn is not None or st.column is None or st.column not in names:
            return None
        ft = f.wtype
        if ft.kind == "numeric" and not issubclass(ft, T.Binary):
            plan.append((f, st.column, "int" if issubclass(ft, T.Integral) else "real"))
        elif ft.kind == "text":
            plan.append((f, st.column, "text"))
        else:
            return None
    return plan


class _Chunk:
    def __init__(self, nbytes, dev):
        self.host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        self.np = self.host.numpy()
        self.dev = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        self.copied = None
        self.n = 0


def _pread_into(fd, arr: np.ndarray, off: int, n: int, pool) -> int:
    """Read ``n`` bytes at file offset ``off`` into ``arr[:n]`` with parallel ``preadv`` calls; returns bytes read."""
    parts = [(o, min(_READ_SPLIT, n - o)) for o in range(0, n, _READ_SPLIT)]

    def one(p):
        o, m = p
        mv = memoryview(arr)[o:o + m]
        got = 0
        while got < m:
            k = os.preadv(fd, [mv[got:]], off + o + got)
            if k <= 0:
                break
            got += k
        return got
    return sum(pool.map(one, parts)) if len(parts) > 1 else one(parts[0]) if parts else 0


def gpu_csv_dataset(path: str, raw_features: Sequence, dev, names: Optional[Sequence[str]] = None,
                    has_header: bool = True, separator: str = ",", key_fn=None,
                    chunk_bytes: int = CHUNK, text_columns: Sequence[str] = ()) -> Optional[Dataset]:
    dev = torch.device(dev)
    if dev.type != "cuda" or key_fn is not None or len(separator) != 1 or os.environ.get("TMOG_GPU_CSV") == "0":
        return None
    from ..ops import _native as N
    lib = N.hip()
    t_start = time.perf_counter()
    with open(path, "rb") as fh:
        first = fh.readline()
    skip = 0
    if has_header:
        header = next(csv.reader(io.StringIO(first.decode("utf-8")), delimiter=separator), [])
        skip = len(first)
        if names is None:
            names = header
    if names is None:
        return None
    names = list(names)
    plan = _plan(raw_features, names)
    if plan is None:
        return None
    ncols = len(names)
    num_cols = list(dict.fromkeys(c for _, c, k in plan if k in ("real", "int")))
    txt_cols = list(dict.fromkeys(c for _, c, k in plan if k == "text"))
    kind_of = {c: ("int" if any(k == "int" and cc == c for _, cc, k in plan) else "real") for c in num_cols}
    if any(c in txt_cols for c in num_cols):
        return None                     # a column read both as numbers and as text: the generic path
    cidx = {c: i for i, c in enumerate(names)}
    ncol_t = torch.tensor([cidx[c] for c in num_cols], dtype=torch.int32, device=dev)
    kind_t = torch.tensor([1 if kind_of[c] == "int" else 0 for c in num_cols], dtype=torch.int32, device=dev)
    tcol_t = torch.tensor([cidx[c] for c in txt_cols], dtype=torch.int32, device=dev)
    size = os.path.getsize(path)
    carry_max = 1 << 20
    bufs = [_Chunk(chunk_bytes + carry_max, dev) for _ in range(2)]
    copy_stream = torch.cuda.Stream(device=dev)
    cur = torch.cuda.current_stream(dev)
    pool = cf.ThreadPoolExecutor(max(1, min(16, os.cpu_count() or 4)))
    reader = cf.ThreadPoolExecutor(1)
    num_vals: List[torch.Tensor] = []
    num_ok: List[torch.Tensor] = []
    txt_hash: List[torch.Tensor] = []
    vocab: List[Dict[int, str]] = [dict() for _ in txt_cols]
    prof = {"read_wait": 0.0, "parse": 0.0, "host_fix": 0.0}
    fd = os.open(path, os.O_RDONLY)

    def fill(k, off, carry: bytes):
        b = bufs[k]
        if b.copied is not None:
            b.copied.synchronize()      # its previous chunk's copy to the device has finished
        c = len(carry)
        if c:
            b.np[:c] = np.frombuffer(carry, np.uint8)
        got = _pread_into(fd, b.np[c:], off, min(chunk_bytes, size - off), pool) if off < size else 0
        b.n = c + got
        return off + got

    try:
        off = skip
        k = 0
        fut = reader.submit(fill, 0, off, b"")
        while True:
            t0 = time.perf_counter()
            off = fut.result()
            prof["read_wait"] += time.perf_counter() - t0
            b = bufs[k]
            L = b.n
            if L == 0:
                break
            eof = off >= size
            if eof:
                end = L                     # (the last row may lack its newline: _parse_chunk adds its end)
            else:
                tail = b.np[max(0, L - carry_max):L]
                nl = np.flatnonzero(tail == 10)
                if nl.size == 0:
                    return None             # a row longer than the carry window: generic path
                end = max(0, L - carry_max) + int(nl[-1]) + 1
            carry = b.np[end:L].tobytes() if end < L else b""
            if not eof:                     # read the next chunk while this one is parsed
                fut = reader.submit(fill, k ^ 1, off, carry)
            t1 = time.perf_counter()
            copy_stream.wait_stream(cur)        # the kernels of the chunk that last used this device buffer
            with torch.cuda.stream(copy_stream):
                b.dev[:end].copy_(b.host[:end], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(copy_stream)
            b.copied = ev
            cur.wait_event(ev)
            res = _parse_chunk(lib, N, b, end, ncols, separator, ncol_t, kind_t, tcol_t, dev, vocab, prof)
            if res is None:
                return None
            nv, ok, th = res
            num_vals.append(nv)
            num_ok.append(ok)
            txt_hash.append(th)
            prof["parse"] += time.perf_counter() - t1
            if eof:
                break
            k ^= 1
    finally:
        os.close(fd)
        reader.shutdown(wait=True)
        pool.shutdown(wait=False)
        for b in bufs:
            if b.copied is not None:
                b.copied.synchronize()
    n = sum(int(v.shape[1]) for v in num_vals) if num_vals else sum(int(h.shape[1]) for h in txt_hash)
    cols = OrderedDict()
    for j, c in enumerate(num_cols):
        v = torch.cat([x[j] for x in num_vals]) if num_vals else torch.empty(0, dtype=torch.int64, device=dev)
        ok = torch.cat([x[j] for x in num_ok]).bool() if num_ok else torch.empty(0, dtype=torch.bool, device=dev)
        vals = v if kind_of[c] == "int" else v.view(torch.float64)
        cols[c] = (vals, None if bool(ok.all()) else ok)
    for j, c in enumerate(txt_cols):
        # a text feature whose cells all look like numbers is read as numbers and rendered back by the generic
        # path (the Arrow path takes a text column only when Arrow types it as strings)
        if c not in text_columns and vocab[j] and all(_numeric_literal(v) for v in vocab[j].values()):
            return None
        h = torch.cat([x[j] for x in txt_hash])
        cols[c] = _encode_hashes(h, vocab[j], dev)
    out = OrderedDict()
    for f, c, k in plan:
        if k == "text":
            codes, voc = cols[c]
            out[f.name] = TextColumn(f.wtype, codes, voc)
        else:
            vals, ok = cols[c]
            if not f.wtype.nullable and ok is not None:
                raise T.NonNullableEmptyException(f"{f.wtype.__name__} column '{c}' contains empty values")
            out[f.name] = NumericColumn(f.wtype, vals, ok)
    if os.environ.get("TMOG_INGEST_PROFILE") == "1":
        import sys
        prof["total"] = time.perf_counter() - t_start
        sys.stderr.write("[gpu-csv] " + " ".join(f"{a}={b:.3f}" for a, b in prof.items()) + f" rows={n}\n")
    return Dataset(OrderedDict((f.name, out[f.name]) for f in raw_features), None, n)


def _parse_chunk(lib, N, b: _Chunk, end: int, ncols: int, sep: str, ncol_t, kind_t, tcol_t, dev, vocab, prof):
    buf = b.dev[:end]
    ends = torch.nonzero(buf == 10).squeeze(1)
    if end and (ends.numel() == 0 or int(ends[-1]) != end - 1):     # a final row without its newline
        ends = torch.cat([ends, torch.tensor([end], dtype=torch.int64, device=dev)])
    starts = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), ends[:-1] + 1]) if ends.numel() else ends
    # empty lines are skipped (pyarrow ignore_empty_lines); "\r" alone counts as empty
    length = ends - starts
    blank = (length == 0) | ((length == 1) & (buf[starts.clamp_max(max(end - 1, 0))] == 13))
    if bool(blank.any()):
        keep = ~blank
        starts, ends = starts[keep], ends[keep]
    nrows = int(starts.numel())
    fstart = torch.empty(nrows, ncols + 1, dtype=torch.int64, device=dev)
    nf = torch.empty(nrows, dtype=torch.int32, device=dev)
    st = N.stream(dev)
    N.check(lib.tmog_hip_csv_fields(N.ptr(buf), N.ptr(starts), N.ptr(ends), nrows, ncols, ord(sep), N.ptr(fstart),
                                    N.ptr(nf), st), "csv_fields")
    if nrows and bool((nf != ncols).any()):
        return None                         # ragged rows: pyarrow / pandas decide
    nn, nt = int(ncol_t.numel()), int(tcol_t.numel())
    vals = torch.empty(nn, nrows, dtype=torch.int64, device=dev)
    ok = torch.empty(nn, nrows, dtype=torch.uint8, device=dev)
    slow = torch.empty(nn, nrows, dtype=torch.uint8, device=dev)
    if nn:
        N.check(lib.tmog_hip_csv_parse_num(N.ptr(buf), N.ptr(fstart), N.ptr(nf), nrows, ncols, N.ptr(ncol_t),
                                           N.ptr(kind_t), nn, N.ptr(vals), N.ptr(ok), N.ptr(slow), st),
                "csv_parse_num")
        idx = torch.nonzero(slow.view(-1)).squeeze(1)
        if idx.numel():                     # the host parses the rare fields the device fast path leaves
            t0 = time.perf_counter()
            if not _host_fix(b, fstart, vals, ok, idx, nrows, ncol_t, kind_t):
                return None
            prof["host_fix"] += time.perf_counter() - t0
    th = torch.empty(nt, nrows, dtype=torch.int64, device=dev)
    if nt:
        span = torch.empty(nt, nrows, 2, dtype=torch.int64, device=dev)
        N.check(lib.tmog_hip_csv_hash_text(N.ptr(buf), N.ptr(fstart), N.ptr(nf), nrows, ncols, N.ptr(tcol_t), nt,
                                           N.ptr(th), N.ptr(span), st), "csv_hash_text")
        for j in range(nt):                 # this chunk's new distinct strings: their first cell's bytes
            h = th[j]
            u, inv = torch.unique(h, return_inverse=True)
            first = torch.full((int(u.numel()),), nrows, dtype=torch.int64, device=dev)
            first.scatter_reduce_(0, inv, torch.arange(nrows, device=dev), reduce="amin")
            hs, rows = u.cpu().tolist(), first.cpu()
            new = [i for i, x in enumerate(hs) if x != 0 and x not in vocab[j]]
            if new:
                sp = span[j].index_select(0, rows[new].to(dev)).cpu().numpy()
                for i, (a, e) in zip(new, sp):
                    vocab[j][hs[i]] = b.np[a:e].tobytes().decode("utf-8", "replace").replace('""', '"')
    return vals, ok, th


def _host_fix(b: _Chunk, fstart, vals, ok, idx, nrows, ncol_t, kind_t) -> bool:
    j = (idx // nrows).cpu().numpy()
    r = (idx % nrows).cpu().numpy()
    cols = ncol_t.cpu().numpy()
    kinds = kind_t.cpu().numpy()
    fs = fstart.cpu().numpy()
    out_v = np.empty(len(idx), np.int64)
    out_ok = np.empty(len(idx), np.uint8)
    for t, (jj, rr) in enumerate(zip(j, r)):
        c = int(cols[jj])
        s = b.np[fs[rr, c]:fs[rr, c + 1] - 1].tobytes().decode("utf-8", "replace").strip()
        if len(s) >= 2 and s[0] == '"' and s[-1] == '"':
            s = s[1:-1]
        try:
            if kinds[jj] == 1:
                out_v[t] = int(s)
            else:
                out_v[t] = np.float64(float(s)).view(np.int64)
            out_ok[t] = 1
            if kinds[jj] == 0 and np.isnan(np.float64(float(s))):
                out_ok[t] = 0               # a NaN is missing (the Arrow path: notna)
        except ValueError:
            return False                    # unparsable cell: the generic path reports it
    dev = vals.device
    vals.view(-1)[idx] = torch.as_tensor(out_v, device=dev)
    ok.view(-1)[idx] = torch.as_tensor(out_ok, device=dev)
    return True


def _numeric_literal(s: str) -> bool:
    try:
        float(s)
        return True
    except ValueError:
        return False


def _encode_hashes(h: torch.Tensor, vocab: Dict[int, str], dev):
    """``(codes int32, vocab)`` from per-row 64-bit hashes (0 = missing), codes by first appearance."""
    n = int(h.numel())
    if n == 0:
        return torch.empty(0, dtype=torch.int32, device=dev), []
    u, inv = torch.unique(h, return_inverse=True)
    first = torch.full((int(u.numel()),), n, dtype=torch.int64, device=dev)
    first.scatter_reduce_(0, inv, torch.arange(n, device=dev), reduce="amin")
    present = u != 0
    order = torch.argsort(torch.where(present, first, torch.full_like(first, n + 1)))
    n_used = int(present.sum())
    rank = torch.empty_like(order)
    rank[order] = torch.arange(int(order.numel()), device=dev)
    codes = torch.where(h == 0, torch.full_like(inv, -1), rank[inv]).to(torch.int32)
    hs = u[order[:n_used]].cpu().tolist()
    return codes, [vocab[x] for x in hs]

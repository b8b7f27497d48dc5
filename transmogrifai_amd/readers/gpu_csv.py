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


class _Host:
    def __init__(self, nbytes):
        self.host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        self.np = self.host.numpy()
        self.copied = None          # event: this buffer's last device copy has finished reading it
        self.n = 0
        self.base = 0               # file offset of byte 0


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
                    chunk_bytes: int = CHUNK, text_columns: Sequence[str] = (),
                    real_dtype: torch.dtype = torch.float64) -> Optional[Dataset]:
    """The CSV file as device columns (None: the generic path decides). ``real_dtype`` is the storage type of the
    real-valued columns (float64, the reference's double; float32 for a file written from float32 data, whose
    shortest decimals then read back bit-identically)."""
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
    # three pinned host buffers (chunk i is read while chunk i - 1 parses and chunk i - 2's bytes stay readable for
    # its host fix-ups), two device buffers (chunk i + 1 is copied while chunk i parses)
    hosts = [_Host(chunk_bytes + carry_max) for _ in range(3)]
    devs = [torch.empty(chunk_bytes + carry_max, dtype=torch.uint8, device=dev) for _ in range(2)]
    dev_free = [None, None]             # event: the kernels of the chunk that last used the device buffer are done
    copy_stream = torch.cuda.Stream(device=dev)
    cur = torch.cuda.current_stream(dev)
    pool = cf.ThreadPoolExecutor(max(1, min(16, os.cpu_count() or 4)))
    reader = cf.ThreadPoolExecutor(1)
    num_vals: List[torch.Tensor] = []
    num_ok: List[torch.Tensor] = []
    txt_hash: List[torch.Tensor] = []
    txt_span: List[torch.Tensor] = []
    prof = {"read_wait": 0.0, "loop": 0.0, "host_fix": 0.0, "sync": 0.0}
    fd = os.open(path, os.O_RDONLY)

    def fill(k, off, carry: bytes):
        h = hosts[k]
        if h.copied is not None:
            h.copied.synchronize()      # its previous chunk's copy to the device has finished
        c = len(carry)
        if c:
            h.np[:c] = np.frombuffer(carry, np.uint8)
        got = _pread_into(fd, h.np[c:], off, min(chunk_bytes, size - off), pool) if off < size else 0
        h.n = c + got
        h.base = off - c
        return off + got

    pending = None                      # the previous chunk: (host buffer, fstart, flags) awaiting its checks
    try:
        t_loop = time.perf_counter()
        off = skip
        i = 0
        fut = reader.submit(fill, 0, off, b"")
        while True:
            t0 = time.perf_counter()
            off = fut.result()
            prof["read_wait"] += time.perf_counter() - t0
            h = hosts[i % 3]
            L = h.n
            if L == 0:
                break
            eof = off >= size
            if eof:
                end = L                     # (the last row may lack its newline: its end is added below)
            else:
                tail = h.np[max(0, L - carry_max):L]
                nl = np.flatnonzero(tail == 10)
                if nl.size == 0:
                    return None             # a row longer than the carry window: generic path
                end = max(0, L - carry_max) + int(nl[-1]) + 1
            carry = h.np[end:L].tobytes() if end < L else b""
            if not eof:                     # read the next chunk while this one is copied and parsed
                fut = reader.submit(fill, (i + 1) % 3, off, carry)
            d = i % 2
            with torch.cuda.stream(copy_stream):
                if dev_free[d] is not None:
                    copy_stream.wait_event(dev_free[d])
                devs[d][:end].copy_(h.host[:end], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(copy_stream)
            h.copied = ev
            cur.wait_event(ev)
            final_nl = end > 0 and int(h.np[end - 1]) == 10
            res = _parse_chunk(lib, N, devs[d], h, end, final_nl, ncols, separator, ncol_t, kind_t, tcol_t, dev,
                               prof, pending)
            if res is None:
                return None
            nv, ok, th, sp, pending = res
            done = torch.cuda.Event()
            done.record(cur)
            dev_free[d] = done
            num_vals.append(nv)
            num_ok.append(ok)
            if th is not None:
                txt_hash.append(th)
                txt_span.append(sp)
            i += 1
            if eof:
                break
        if pending is not None and not _check_pending(pending, N, prof):
            return None
        prof["loop"] = time.perf_counter() - t_loop
    finally:
        os.close(fd)
        reader.shutdown(wait=True)
        pool.shutdown(wait=False)
        for h in hosts:
            if h.copied is not None:
                h.copied.synchronize()
    t_fin = time.perf_counter()
    n = sum(int(v.shape[1]) for v in num_vals) if num_vals else sum(int(t.shape[1]) for t in txt_hash)
    cols = OrderedDict()
    if num_cols:
        # one block per storage type, filled chunk by chunk (a few large copies instead of one concatenation
        # and conversion per column); every column is a row of its block
        ri = [j for j, c in enumerate(num_cols) if kind_of[c] == "real"]
        ii = [j for j, c in enumerate(num_cols) if kind_of[c] == "int"]
        R = torch.empty(len(ri), n, dtype=real_dtype, device=dev)
        I = torch.empty(len(ii), n, dtype=torch.int64, device=dev)
        OK = torch.empty(len(num_cols), n, dtype=torch.bool, device=dev)
        ri_t = torch.tensor(ri, dtype=torch.long, device=dev)
        ii_t = torch.tensor(ii, dtype=torch.long, device=dev)
        r0 = 0
        for v, o in zip(num_vals, num_ok):
            r1 = r0 + int(v.shape[1])
            if ri:
                R[:, r0:r1] = v.index_select(0, ri_t).view(torch.float64)
            if ii:
                I[:, r0:r1] = v.index_select(0, ii_t)
            OK[:, r0:r1] = o
            r0 = r1
        del num_vals, num_ok
        all_ok = OK.all(1).cpu().tolist() if n else [True] * len(num_cols)      # one read for every column
        pos = {j: k for k, j in enumerate(ri)}
        pos.update({j: k for k, j in enumerate(ii)})
        for j, c in enumerate(num_cols):
            v = R[pos[j]] if kind_of[c] == "real" else I[pos[j]]
            cols[c] = (v, None if all_ok[j] else OK[j])
    prof["finish_num"] = time.perf_counter() - t_fin
    if txt_cols:
        Hh = torch.cat(txt_hash, 1) if len(txt_hash) > 1 else txt_hash[0]           # [nt, n]
        Sp = torch.cat(txt_span, 1) if len(txt_span) > 1 else txt_span[0]           # [nt, n, 2] file offsets
        import mmap
        with open(path, "rb") as fh, mmap.mmap(fh.fileno(), 0, access=mmap.ACCESS_READ) as mm:
            for j, c in enumerate(txt_cols):
                codes, voc = _encode_hashes_spans(Hh[j], Sp[j], mm, dev)
                # a text feature whose cells all look like numbers is read as numbers and rendered back by the
                # generic path (the Arrow path takes a text column only when Arrow types it as strings)
                if c not in text_columns and voc and all(_numeric_literal(v) for v in voc):
                    return None
                cols[c] = (codes, voc)
        prof["finish_txt"] = time.perf_counter() - t_fin - prof.get("finish_num", 0.0)
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
        torch.cuda.synchronize(dev)
        prof["finish"] = time.perf_counter() - t_fin
        prof["total"] = time.perf_counter() - t_start
        sys.stderr.write("[gpu-csv] " + " ".join(f"{a}={b:.3f}" for a, b in prof.items()) + f" rows={n} chunks={i}\n")
    return Dataset(OrderedDict((f.name, out[f.name]) for f in raw_features), _key_column(path, names, has_header,
                                                                                        separator, n), n)


def _key_column(path: str, names: Sequence[str], has_header: bool, separator: str, n: int):
    """The file's ``key`` column as strings (the columnar / pandas paths' record keys), or None without one."""
    if "key" not in names:
        return None
    import pyarrow as pa
    import pyarrow.csv as pcsv
    tab = pcsv.read_csv(path, read_options=pcsv.ReadOptions(column_names=list(names), skip_rows=1 if has_header else 0),
                        parse_options=pcsv.ParseOptions(delimiter=separator),
                        convert_options=pcsv.ConvertOptions(include_columns=["key"], column_types={"key": pa.string()}))
    key = tab.column("key").to_pandas().astype(str).to_numpy(dtype=object)
    return key if len(key) == n else None


def _check_pending(pending, N, prof) -> bool:
    """The previous chunk's checks, read after its kernels have run: ragged rows -> the generic path; cells the
    device parser left to the host are parsed from the chunk's (still intact) host bytes."""
    h, fstart, flags, vals, ok, slow, nrows, ncol_t, kind_t = pending
    t0 = time.perf_counter()
    f = flags.cpu().tolist()             # [ragged rows, slow cells]: one small read
    prof["sync"] += time.perf_counter() - t0
    if f[0]:
        return False                    # ragged rows: pyarrow / pandas decide
    if f[1]:
        idx = torch.nonzero(slow.view(-1)).squeeze(1)
        t0 = time.perf_counter()
        if not _host_fix(h, fstart, vals, ok, idx, nrows, ncol_t, kind_t):
            return False
        prof["host_fix"] += time.perf_counter() - t0
    return True


def _parse_chunk(lib, N, buf_all, h: _Host, end: int, final_nl: bool, ncols: int, sep: str, ncol_t, kind_t, tcol_t,
                 dev, prof, pending):
    buf = buf_all[:end]
    ends = torch.nonzero(buf == 10).squeeze(1)
    if end and not final_nl:            # a final row without its newline
        ends = torch.cat([ends, torch.tensor([end], dtype=torch.int64, device=dev)])
    # the nonzero above synchronised with this chunk's copy and the previous chunk's kernels: the previous chunk's
    # flags are ready -- read them now (no extra wait)
    if pending is not None and not _check_pending(pending, N, prof):
        return None
    starts = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), ends[:-1] + 1]) if ends.numel() else ends
    # empty lines are skipped (pyarrow ignore_empty_lines); "\r" alone counts as empty
    length = ends - starts
    blank = (length == 0) | ((length == 1) & (buf[starts.clamp_max(max(end - 1, 0))] == 13))
    keep = torch.nonzero(~blank).squeeze(1)
    if int(keep.numel()) != int(starts.numel()):
        starts, ends = starts[keep], ends[keep]
    nrows = int(starts.numel())
    fstart = torch.empty(nrows, ncols + 1, dtype=torch.int64, device=dev)
    nf = torch.empty(nrows, dtype=torch.int32, device=dev)
    st = N.stream(dev)
    N.check(lib.tmog_hip_csv_fields(N.ptr(buf), N.ptr(starts), N.ptr(ends), nrows, ncols, ord(sep), N.ptr(fstart),
                                    N.ptr(nf), st), "csv_fields")
    nn, nt = int(ncol_t.numel()), int(tcol_t.numel())
    # the kernels write row-major tiles (a wave reads one row's fields); transposed to column-major here
    vals_rm = torch.empty(nrows, nn, dtype=torch.int64, device=dev)
    ok_rm = torch.empty(nrows, nn, dtype=torch.uint8, device=dev)
    slow_rm = torch.empty(nrows, nn, dtype=torch.uint8, device=dev)
    if nn:
        N.check(lib.tmog_hip_csv_parse_num(N.ptr(buf), N.ptr(fstart), N.ptr(nf), nrows, ncols, N.ptr(ncol_t),
                                           N.ptr(kind_t), nn, N.ptr(vals_rm), N.ptr(ok_rm), N.ptr(slow_rm), st),
                "csv_parse_num")
    vals, ok, slow = vals_rm.t().contiguous(), ok_rm.t().contiguous(), slow_rm.t().contiguous()
    del vals_rm, ok_rm, slow_rm
    th = sp = None
    if nt:
        th_rm = torch.empty(nrows, nt, dtype=torch.int64, device=dev)
        sp_rm = torch.empty(nrows, nt, 2, dtype=torch.int64, device=dev)
        N.check(lib.tmog_hip_csv_hash_text(N.ptr(buf), N.ptr(fstart), N.ptr(nf), nrows, ncols, N.ptr(tcol_t), nt,
                                           N.ptr(th_rm), N.ptr(sp_rm), st), "csv_hash_text")
        th = th_rm.t().contiguous()
        sp = sp_rm.transpose(0, 1).contiguous()
        sp += h.base                    # chunk offsets -> file offsets (the bytes are re-read from the file)
    ragged = (nf != ncols).sum() if nrows else torch.zeros((), dtype=torch.int64, device=dev)
    nslow = slow.sum(dtype=torch.int64) if nn and nrows else torch.zeros((), dtype=torch.int64, device=dev)
    flags = torch.stack([ragged.to(torch.int64), nslow])
    return vals, ok, th, sp, (h, fstart, flags, vals, ok, slow, nrows, ncol_t, kind_t)


def _host_fix(h: _Host, fstart, vals, ok, idx, nrows, ncol_t, kind_t) -> bool:
    j = (idx // nrows).cpu().numpy()
    r = (idx % nrows).cpu().numpy()
    cols = ncol_t.cpu().numpy()
    kinds = kind_t.cpu().numpy()
    fs = fstart.cpu().numpy()
    out_v = np.empty(len(idx), np.int64)
    out_ok = np.empty(len(idx), np.uint8)
    for t, (jj, rr) in enumerate(zip(j, r)):
        c = int(cols[jj])
        s = h.np[fs[rr, c]:fs[rr, c + 1] - 1].tobytes().decode("utf-8", "replace").strip()
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


def _encode_hashes_spans(h: torch.Tensor, span: torch.Tensor, mm, dev):
    """``(codes int32, vocab)`` from per-row 64-bit hashes (0 = missing) and the cells' file byte ranges: codes by
    first appearance; each distinct string read once from the file (memory-mapped) at its first cell. One stable
    sort: a group's first sorted position holds its first row (no scatter-min onto the few groups of a pick list,
    whose atomics would contend on a handful of addresses)."""
    n = int(h.numel())
    if n == 0:
        return torch.empty(0, dtype=torch.int32, device=dev), []
    hs, idx = torch.sort(h, stable=True)
    new = torch.ones(n, dtype=torch.bool, device=dev)
    new[1:] = hs[1:] != hs[:-1]
    starts = torch.nonzero(new).squeeze(1)                  # first sorted position of every distinct hash
    gid = torch.cumsum(new.to(torch.int32), 0) - 1          # group of every sorted position
    first = idx.index_select(0, starts)                     # its first row (the sort is stable)
    present = hs.index_select(0, starts) != 0
    order = torch.argsort(torch.where(present, first, torch.full_like(first, n + 1)))
    n_used = int(present.sum())
    rank = torch.empty_like(order)
    rank[order] = torch.arange(int(order.numel()), device=dev)
    grank = torch.where(present, rank, torch.full_like(rank, -1)).to(torch.int32)
    codes = torch.empty(n, dtype=torch.int32, device=dev)
    codes[idx] = grank.index_select(0, gid.long())
    rows = first.index_select(0, order[:n_used])
    spans = span.index_select(0, rows).cpu().numpy()
    voc = [mm[a:b].decode("utf-8", "replace").replace('""', '"') for a, b in spans]
    return codes, voc

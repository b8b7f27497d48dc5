"""Avro object-container file reader / writer (no external dependency).

Reference: ``AvroReaders`` (``readers/.../AvroReaders.scala:55-134``) and the Avro IO helpers
(``utils/.../io/avro/AvroInOut.scala``). Implements the Avro 1.x binary encoding for the schema
subset used by tabular data: null, boolean, int, long, float, double, bytes, string, record, enum,
array, map, union and fixed; container codecs ``null`` and ``deflate``. Decoding yields plain dicts.
"""
from __future__ import annotations

import glob
import io
import json
import os
import struct
import zlib
from typing import Any, Dict, Iterator, List, Optional

MAGIC = b"Obj\x01"


class _Reader:
    def __init__(self, data: bytes):
        self.b = data
        self.p = 0

    def read(self, n: int) -> bytes:
        s = self.b[self.p:self.p + n]
        if len(s) != n:
            raise EOFError("unexpected end of avro data")
        self.p += n
        return s

    def long(self) -> int:
        shift = 0
        acc = 0
        while True:
            c = self.b[self.p]
            self.p += 1
            acc |= (c & 0x7F) << shift
            if not c & 0x80:
                break
            shift += 7
        return (acc >> 1) ^ -(acc & 1)

    def eof(self) -> bool:
        return self.p >= len(self.b)


def _named(schema, names: Dict[str, Any], ns: Optional[str] = None):
    if isinstance(schema, dict) and schema.get("type") in ("record", "enum", "fixed"):
        nm = schema["name"]
        space = schema.get("namespace", ns)
        full = nm if "." in nm or not space else f"{space}.{nm}"
        names[full] = schema
        names[nm] = schema
        if schema["type"] == "record":
            for f in schema["fields"]:
                _named(f["type"], names, space)
    elif isinstance(schema, list):
        for s in schema:
            _named(s, names, ns)
    elif isinstance(schema, dict) and schema.get("type") in ("array", "map"):
        _named(schema.get("items") or schema.get("values"), names, ns)


def _decode(r: _Reader, schema, names) -> Any:
    if isinstance(schema, str):
        if schema in names:
            return _decode(r, names[schema], names)
        t = schema
        schema = {"type": t}
    elif isinstance(schema, list):
        idx = r.long()
        return _decode(r, schema[idx], names)
    t = schema["type"]
    if isinstance(t, (dict, list)):
        return _decode(r, t, names)
    if t == "null":
        return None
    if t == "boolean":
        return r.read(1) != b"\x00"
    if t in ("int", "long"):
        return r.long()
    if t == "float":
        return struct.unpack("<f", r.read(4))[0]
    if t == "double":
        return struct.unpack("<d", r.read(8))[0]
    if t == "bytes":
        return r.read(r.long())
    if t == "string":
        return r.read(r.long()).decode("utf-8")
    if t == "record":
        return {f["name"]: _decode(r, f["type"], names) for f in schema["fields"]}
    if t == "enum":
        return schema["symbols"][r.long()]
    if t == "fixed":
        return r.read(schema["size"])
    if t in ("array", "map"):
        out: Any = [] if t == "array" else {}
        while True:
            n = r.long()
            if n == 0:
                break
            if n < 0:
                n = -n
                r.long()   # block byte size
            for _ in range(n):
                if t == "array":
                    out.append(_decode(r, schema["items"], names))
                else:
                    k = r.read(r.long()).decode("utf-8")
                    out[k] = _decode(r, schema["values"], names)
        return out
    if t in names:
        return _decode(r, names[t], names)
    raise ValueError(f"unsupported avro type {t}")


def snappy_decompress(buf: bytes) -> bytes:
    """Raw snappy format: a varint uncompressed length, then literal / back-reference elements whose tag
    byte's low 2 bits select literal (0) or copy with a 1- (1), 2- (2) or 4-byte (3) offset."""
    n, shift, i = 0, 0, 0
    while True:
        b = buf[i]
        i += 1
        n |= (b & 0x7F) << shift
        shift += 7
        if b < 0x80:
            break
    out = bytearray()
    end = len(buf)
    while i < end:
        tag = buf[i]
        i += 1
        kind = tag & 3
        if kind == 0:
            ln = tag >> 2
            if ln >= 60:
                nb = ln - 59
                ln = int.from_bytes(buf[i:i + nb], "little")
                i += nb
            ln += 1
            out += buf[i:i + ln]
            i += ln
            continue
        if kind == 1:
            ln = ((tag >> 2) & 7) + 4
            off = ((tag >> 5) << 8) | buf[i]
            i += 1
        elif kind == 2:
            ln = (tag >> 2) + 1
            off = int.from_bytes(buf[i:i + 2], "little")
            i += 2
        else:
            ln = (tag >> 2) + 1
            off = int.from_bytes(buf[i:i + 4], "little")
            i += 4
        if off == 0 or off > len(out):
            raise ValueError("corrupt snappy stream (bad back-reference)")
        start = len(out) - off
        if off >= ln:
            out += out[start:start + ln]
        else:                       # overlapping copy: repeat the last `off` bytes
            for k in range(ln):
                out.append(out[start + k])
    if len(out) != n:
        raise ValueError(f"corrupt snappy stream ({len(out)} bytes, header says {n})")
    return bytes(out)


def read_avro_file(path: str) -> Iterator[Dict[str, Any]]:
    with open(path, "rb") as f:
        data = f.read()
    r = _Reader(data)
    if r.read(4) != MAGIC:
        raise ValueError(f"{path} is not an avro container file")
    meta = _decode(r, {"type": "map", "values": "bytes"}, {})
    sync = r.read(16)
    schema = json.loads(meta["avro.schema"].decode("utf-8"))
    codec = meta.get("avro.codec", b"null").decode("utf-8")
    names: Dict[str, Any] = {}
    _named(schema, names)
    while not r.eof():
        count = r.long()
        size = r.long()
        block = r.read(size)
        if codec == "deflate":
            block = zlib.decompress(block, -15)
        elif codec == "snappy":      # raw snappy block + big-endian CRC32 of the uncompressed bytes
            body, crc = block[:-4], int.from_bytes(block[-4:], "big")
            block = snappy_decompress(body)
            if zlib.crc32(block) & 0xFFFFFFFF != crc:
                raise ValueError(f"{path}: snappy block CRC mismatch")
        elif codec != "null":
            raise ValueError(f"unsupported avro codec {codec}")
        br = _Reader(block)
        for _ in range(count):
            yield _decode(br, schema, names)
        if r.read(16) != sync:
            raise ValueError("avro sync marker mismatch")


def read_avro(path: str) -> List[Dict[str, Any]]:
    """All records of one file, or of every ``*.avro`` file in a directory / glob."""
    if os.path.isdir(path):
        files = sorted(glob.glob(os.path.join(path, "*.avro")))
    elif any(c in path for c in "*?["):
        files = sorted(glob.glob(path))
    else:
        files = [path]
    out: List[Dict[str, Any]] = []
    for f in files:
        out.extend(read_avro_file(f))
    return out


read_avro_records = read_avro


def read_avro_schema(path: str) -> Dict[str, Any]:
    """Schema of an ``.avsc`` JSON file or of an avro container file."""
    if path.endswith(".avsc"):
        with open(path) as f:
            return json.load(f)
    with open(path, "rb") as f:
        data = f.read()
    r = _Reader(data)
    if r.read(4) != MAGIC:
        raise ValueError(f"{path} is not an avro container file")
    meta = _decode(r, {"type": "map", "values": "bytes"}, {})
    return json.loads(meta["avro.schema"].decode("utf-8"))


# --------------------------------------------------------------------------------------------- writer
def _zz(n: int) -> bytes:
    n = (n << 1) ^ (n >> 63)
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _encode(buf: io.BytesIO, schema, v, names):
    if isinstance(schema, str):
        if schema in names:
            return _encode(buf, names[schema], v, names)
        schema = {"type": schema}
    elif isinstance(schema, list):
        for i, s in enumerate(schema):
            st = s if isinstance(s, str) else s.get("type")
            if (v is None) == (st == "null"):
                if v is None or _fits(st, v):
                    buf.write(_zz(i))
                    return _encode(buf, s, v, names)
        raise ValueError(f"value {v!r} does not match union {schema}")
    t = schema["type"]
    if isinstance(t, (dict, list)):
        return _encode(buf, t, v, names)
    if t == "null":
        return
    if t == "boolean":
        buf.write(b"\x01" if v else b"\x00")
    elif t in ("int", "long"):
        buf.write(_zz(int(v)))
    elif t == "float":
        buf.write(struct.pack("<f", float(v)))
    elif t == "double":
        buf.write(struct.pack("<d", float(v)))
    elif t in ("bytes", "string"):
        b = v if isinstance(v, bytes) else str(v).encode("utf-8")
        buf.write(_zz(len(b)))
        buf.write(b)
    elif t == "record":
        for f in schema["fields"]:
            _encode(buf, f["type"], v.get(f["name"]), names)
    elif t == "enum":
        buf.write(_zz(schema["symbols"].index(v)))
    elif t == "array":
        if v:
            buf.write(_zz(len(v)))
            for x in v:
                _encode(buf, schema["items"], x, names)
        buf.write(b"\x00")
    elif t == "map":
        if v:
            buf.write(_zz(len(v)))
            for k, x in v.items():
                kb = str(k).encode("utf-8")
                buf.write(_zz(len(kb)))
                buf.write(kb)
                _encode(buf, schema["values"], x, names)
        buf.write(b"\x00")
    else:
        raise ValueError(f"unsupported avro type {t}")


def _fits(t, v) -> bool:
    if t == "boolean":
        return isinstance(v, bool)
    if t in ("int", "long"):
        return isinstance(v, int) and not isinstance(v, bool)
    if t in ("float", "double"):
        return isinstance(v, (int, float)) and not isinstance(v, bool)
    if t == "string":
        return isinstance(v, str)
    if t == "bytes":
        return isinstance(v, bytes)
    if t == "array":
        return isinstance(v, (list, tuple))
    if t == "map":
        return isinstance(v, dict)
    return True


def write_avro(path: str, schema: Dict[str, Any], records: List[Dict[str, Any]], codec: str = "deflate") -> None:
    names: Dict[str, Any] = {}
    _named(schema, names)
    sync = os.urandom(16)
    body = io.BytesIO()
    for rec in records:
        _encode(body, schema, rec, names)
    block = body.getvalue()
    if codec == "deflate":
        c = zlib.compressobj(6, zlib.DEFLATED, -15)
        block = c.compress(block) + c.flush()
    out = io.BytesIO()
    out.write(MAGIC)
    meta = {"avro.schema": json.dumps(schema).encode("utf-8"), "avro.codec": codec.encode("utf-8")}
    _encode(out, {"type": "map", "values": "bytes"}, meta, {})
    out.write(sync)
    if records:
        out.write(_zz(len(records)))
        out.write(_zz(len(block)))
        out.write(block)
        out.write(sync)
    with open(path, "wb") as f:
        f.write(out.getvalue())

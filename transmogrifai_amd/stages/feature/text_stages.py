"""Text transformers: value maps, tokenizer, hashing TF / IDF, validators, detectors.

Reference: ``TextTokenizer`` (``core/.../impl/feature/TextTokenizer.scala:125-234``), ``OpHashingTF``
and ``IDF`` Spark wrappers (``RichListFeature.scala:57-80``, ``RichVectorFeature.scala:57-60``),
``EmailDomainToPickList`` / ``URLDomainToPickList`` map functions (``RichTextFeature.scala:617-680``),
``ValidEmailTransformer``, ``MimeTypeDetector`` (Tika, ``RichTextFeature.scala:712-731``),
``PhoneNumberParser.isValidPhoneDefaultCountry`` (``PhoneNumberParser.scala:143-255``),
``TextLenTransformer`` (``TextLenTransformer.scala:45``), ``TextListNullTransformer`` (``:48``).

Text maps run once per *distinct* value of a dictionary-encoded column (``TextColumn.map_vocab``).
"""
from __future__ import annotations

import base64
import re
from typing import Callable, Dict, Optional

import numpy as np
import torch

from ...config import vector_dtype
from ...data.columns import NumericColumn, ObjectColumn, TextColumn, VectorColumn, column_from_values
from ...data.vector_metadata import OpVectorColumnMetadata
from ...features import types as T
from ...utils import text as TU
from ..base import (BinaryTransformer, OpEstimator, OpTransformer, SequenceTransformer, UnaryEstimator, UnaryTransformer,
                    register_stage)
from .vectorizers import (HashingParams, VectorizerMixin, hash_metadata, col_meta)
from ...ops import vector as V

# ------------------------------------------------------------------------------- named value maps
VALUE_FNS: Dict[str, Callable] = {}


def value_fn(name):
    def deco(fn):
        VALUE_FNS[name] = fn
        return fn
    return deco


@value_fn("EmailDomainToPickList")
def _email_domain(s):
    return TU.email_domain(s)


@value_fn("EmailPrefixToText")
def _email_prefix(s):
    return TU.email_prefix(s)


@value_fn("URLDomainToPickList")
def _url_domain_valid(s):
    return TU.url_domain(s) if TU.is_valid_url(s) else None


@value_fn("URLDomainToText")
def _url_domain(s):
    return TU.url_domain(s)


@value_fn("URLProtocolToText")
def _url_protocol(s):
    return TU.url_protocol(s)


@value_fn("Identity")
def _ident(s):
    return s


@value_fn("CleanText")
def _clean(s):
    return TU.clean_string(s)


_MAGIC = [(b"%PDF", "application/pdf"), (b"\x89PNG", "image/png"), (b"\xff\xd8\xff", "image/jpeg"),
          (b"GIF8", "image/gif"), (b"PK\x03\x04", "application/zip"), (b"ID3", "audio/mpeg"),
          (b"<?xml", "application/xml"), (b"\x1f\x8b", "application/gzip"),
          (b"BM", "image/bmp"), (b"OggS", "audio/ogg"), (b"fLaC", "audio/x-flac"), (b"<html", "text/html"),
          (b"<!DOCTYPE html", "text/html"), (b"\x7fELF", "application/x-executable"),
          (b"\xd0\xcf\x11\xe0\xa1\xb1\x1a\xe1", "application/x-tika-msoffice")]
# MPEG audio frame sync (Tika's audio/mpeg magic: 0xFFFA / FB / F2 / F3 / E3)
_MPEG_SYNC = (b"\xff\xfb", b"\xff\xfa", b"\xff\xf3", b"\xff\xf2", b"\xff\xe3")
# RIFF containers: the form type at offset 8 (Tika 1.x names)
_RIFF = {b"WAVE": "audio/vnd.wave", b"AVI ": "video/x-msvideo", b"WEBP": "image/webp"}
_CONTROL = set(range(0x00, 0x09)) | set(range(0x0E, 0x1B)) | set(range(0x1C, 0x20))


def _looks_like_text(raw: bytes) -> bool:
    """Tika's TextDetector: no control bytes, and mostly printable ASCII or valid UTF-8 (an empty stream is not
    text -- Tika answers application/octet-stream)."""
    if not raw:
        return False
    if any(b in _CONTROL for b in raw):
        return False
    ascii_ = sum(1 for b in raw if 0x20 <= b < 0x7F or b in (0x09, 0x0A, 0x0B, 0x0C, 0x0D, 0x1B))
    if ascii_ * 10 >= len(raw) * 9:
        return True
    try:
        raw.decode("utf-8")
        return True
    except UnicodeDecodeError:
        try:        # a multi-byte character cut by the byte limit
            raw[:-3].decode("utf-8")
            return len(raw) > 3
        except UnicodeDecodeError:
            return False


@value_fn("MimeTypeDetector")
def detect_mime(s, max_bytes: int = 1024, type_hint: str = ""):
    """Magic-byte MIME detection of base64 content (Tika ``DefaultDetector`` replacement; expectations of
    ``MimeTypeDetectorTest.scala`` pinned in ``tests/test_nlp_stages.py``). Only the first ``max_bytes`` decoded
    bytes are examined (``BoundedInputStream``, MimeTypeDetector.scala:94); a ``type_hint`` refines the generic
    answers (``application/octet-stream``, ``text/plain``) the way Tika lets the declared content type
    specialise its magic match. ``None`` stays ``None``; an empty value is ``application/octet-stream``."""
    if s is None:
        return None
    try:
        raw = base64.b64decode(s, validate=False)
    except Exception:
        return None
    raw = raw[:max(0, int(max_bytes))] if max_bytes is not None else raw
    for sig, mime in _MAGIC:
        if raw[:len(sig)] == sig or (sig[:1].isalpha() and raw[:len(sig)].lower() == sig.lower()):
            return mime
    if raw[:2] in _MPEG_SYNC:
        return "audio/mpeg"
    if raw[:4] == b"RIFF" and raw[8:12] in _RIFF:
        return _RIFF[raw[8:12]]
    found = "text/plain" if _looks_like_text(raw) else "application/octet-stream"
    if type_hint and _specialises(type_hint.strip().lower(), found):
        return type_hint
    return found


# text/plain subtypes in Tika's type registry that a declared type may pick for plain-text content
_TEXT_FAMILY = ("application/json", "application/xml", "application/javascript", "application/x-javascript",
                "application/ecmascript", "application/x-sh", "application/sql", "application/rtf")


def _specialises(hint: str, detected: str) -> bool:
    """Tika takes a declared content type only when it specialises the magic-detected one (MimeTypes registry
    supertypes): anything refines application/octet-stream; text/plain is refined by text/* and the
    JSON / XML / script family. Other combinations keep the detected type: plain text declared image/png stays
    text/plain, a PNG declared text/plain stays image/png. Beyond the reference's MimeTypeDetectorTest fixtures
    (application/json over text): parity unpinned."""
    if detected == "application/octet-stream":
        return True
    if detected == "text/plain":
        return hint.startswith("text/") or hint in _TEXT_FAMILY or hint.endswith("+xml") or hint.endswith("+json")
    return False


def is_valid_phone(s: Optional[str], region: str = "US", strict: bool = False) -> Optional[bool]:
    """``PhoneNumberParser.validate`` for one region (``utils/phone.py``: numbering-plan table in place of
    libphonenumber metadata; parity unpinned beyond the reference's test vectors)."""
    from ...utils import phone as PH
    return PH.validate(s, region, strict)


@register_stage
class TextMapTransformer(UnaryTransformer):
    """Applies a named value function to each distinct text value (map[PickList] etc.)."""
    operation_name = "map"

    def __init__(self, fn_name: str = "Identity", output_type=T.Text, uid=None, operation_name=None, **kw):
        super().__init__(None, uid=uid, operation_name=operation_name or fn_name, output_type=output_type, **kw)
        self.fn_name = fn_name

    def transform_fn(self, v):
        return VALUE_FNS[self.fn_name](v)

    def transform_columns(self, *cols, ds=None):
        c = cols[0]
        if isinstance(c, TextColumn) and issubclass(self.output_type, T.Text):
            return c.map_vocab(VALUE_FNS[self.fn_name], self.output_type)
        return super().transform_columns(*cols, ds=ds)

    def ctor_args(self):
        return {"fnName": self.fn_name, "tto": self.output_type.__name__}

    def load_ctor_args(self, a):
        self.fn_name = a["fnName"]
        self.output_type = T.feature_type_from_name(a["tto"])


@register_stage
class ValidEmailTransformer(UnaryTransformer):
    operation_name = "isValidEmail"
    output_type = T.Binary

    def transform_fn(self, v):
        return None if v is None else TU.is_valid_email(v)


@register_stage
class PhoneValidator(UnaryTransformer):
    operation_name = "isValidPhoneDefaultCountry"
    output_type = T.Binary
    _defaults = {"default_region": "US", "strict": False}

    def transform_fn(self, v):
        return is_valid_phone(v, self.params["default_region"], self.params["strict"])

    def transform_columns(self, *cols, ds=None):
        c = cols[0]
        if isinstance(c, TextColumn):       # once per distinct value, then a device gather
            res = [is_valid_phone(s, self.params["default_region"], self.params["strict"]) for s in c.vocab]
            lut = np.array([1.0 if r else 0.0 for r in res] + [0.0])
            okv = np.array([r is not None for r in res] + [False])
            idx = torch.where(c.codes >= 0, c.codes.long(), torch.full_like(c.codes.long(), len(c.vocab)))
            vals = torch.as_tensor(lut, device=c.codes.device)[idx] > 0.5
            return NumericColumn(T.Binary, vals, torch.as_tensor(okv, device=c.codes.device)[idx])
        return super().transform_columns(*cols, ds=ds)


@register_stage
class IsValidPhoneNumber(BinaryTransformer):
    """(Phone, region Text) -> Binary (``IsValidPhoneNumber``, PhoneNumberParser.scala:198-214): the region comes
    from the region feature -- a region code, or the closest country name -- and ``+`` numbers are parsed
    internationally."""
    operation_name = "validatePhone"
    output_type = T.Binary
    _defaults = {"default_region": "US", "strict": False, "codes_and_countries": None}

    def transform_fn(self, phone, region):
        from ...utils import phone as PH
        return PH.validate_with_region(phone, region, self.params["default_region"], self.params["strict"],
                                       self.params["codes_and_countries"])


@register_stage
class ParsePhoneNumberWithRegion(BinaryTransformer):
    """(Phone, region Text) -> Phone in E.164 (``ParsePhoneNumber``, PhoneNumberParser.scala:160-196)."""
    operation_name = "parsePhone"
    output_type = T.Phone
    _defaults = {"default_region": "US", "strict": False, "codes_and_countries": None}

    def transform_fn(self, phone, region):
        from ...utils import phone as PH
        return PH.parse_with_region(phone, region, self.params["default_region"], self.params["strict"],
                                    self.params["codes_and_countries"])


@register_stage
class TextTokenizer(UnaryTransformer):
    """Lowercase + StandardAnalyzer tokenization + min token length -> TextList."""
    operation_name = "textToken"
    output_type = T.TextList
    _defaults = {"to_lowercase": True, "min_token_length": 1, "auto_detect_language": False,
                 "strip_html": False, "default_language": "Unknown", "auto_detect_threshold": 0.99}

    def _language_aware(self) -> bool:
        p = self.params
        return bool(p["auto_detect_language"]) or p["default_language"] not in ("Unknown", None, "en")

    def transform_fn(self, v):
        if v is None:
            return []
        p = self.params
        s = TU.strip_html(v) if p["strip_html"] else v
        if self._language_aware():
            # TextTokenizer.scala:160-188: detected language above the threshold, else the default; its
            # analyzer (utils/lang.py: stop words + elisions of that language)
            from ...utils import lang as LG
            lang = LG.best_language(s, float(p["auto_detect_threshold"]), p["default_language"]) \
                if p["auto_detect_language"] else p["default_language"]
            return LG.analyze(s, lang, p["to_lowercase"], p["min_token_length"])
        return TU.tokenize(s, p["to_lowercase"], p["min_token_length"])

    def transform_columns(self, *cols, ds=None):
        c = cols[0]
        if isinstance(c, TextColumn):
            p = self.params
            if self._language_aware():
                toks = [self.transform_fn(s) for s in c.vocab]
            else:
                vocab = [TU.strip_html(s) for s in c.vocab] if p["strip_html"] else c.vocab
                toks = TU.tokenize_batch(vocab, p["to_lowercase"], p["min_token_length"]).lists()
            codes = c.codes.cpu().numpy()
            out = np.empty(len(codes), dtype=object)
            for i, k in enumerate(codes):
                out[i] = list(toks[k]) if k >= 0 else []
            return ObjectColumn(T.TextList, out)
        return super().transform_columns(*cols, ds=ds)


@register_stage
class TextLenTransformer(VectorizerMixin, SequenceTransformer):
    operation_name = "textLen"

    def transform_columns(self, *cols, ds=None):
        tfs = self.get_transient_features()
        self.metadata["vector_metadata"] = self.vector_metadata(
            [col_meta(t, descriptor="TextLenValue") for t in tfs])
        dev = cols[0].device
        parts = []
        for c in cols:
            if isinstance(c, TextColumn):
                lens = torch.as_tensor(np.append(TU.tokenize_batch(c.vocab).char_lengths().astype(np.float64), 0.0),
                                       device=dev)
                idx = torch.where(c.codes >= 0, c.codes.long(), torch.full_like(c.codes.long(), len(c.vocab)))
                parts.append(lens[idx])
            else:
                parts.append(torch.as_tensor([float(sum(len(x) for x in (v or []))) for v in c.to_list()],
                                             device=dev))
        return self._vec(torch.stack(parts, 1).to(vector_dtype(dev)))


@register_stage
class TextListNullTransformer(VectorizerMixin, SequenceTransformer):
    operation_name = "textListNull"

    def transform_columns(self, *cols, ds=None):
        tfs = self.get_transient_features()
        self.metadata["vector_metadata"] = self.vector_metadata([col_meta(t, is_null=True) for t in tfs])
        dev = cols[0].device
        parts = [c.null_mask().to(dev).to(torch.float64) for c in cols]
        return self._vec(torch.stack(parts, 1).to(vector_dtype(dev)))


@register_stage
class OpHashingTF(VectorizerMixin, OpTransformer):
    """Hashing term frequency of a TextList (Spark ``HashingTF``, murmur3 seed 42, no name prefix)."""
    operation_name = "hashingTF"
    arity = 1
    _defaults = {"num_features": 512, "binary": False}

    def transform_columns(self, *cols, ds=None):
        c = cols[0]
        hp = HashingParams(self.params["num_features"], 1, 1 << 30, self.params["binary"], False, "separate")
        tfs = self.get_transient_features()
        self.metadata["vector_metadata"] = self.vector_metadata(hash_metadata(tfs, hp))
        from ...ops.text import HashInput, hashed_tf
        lists = [[str(x) for x in (v or [])] for v in c.to_list()]
        dev = c.device
        out = torch.empty(len(lists), hp.num_features, dtype=vector_dtype(dev), device=dev)
        hashed_tf(out, [HashInput(None, TU.TokenBatch.from_lists(lists), None)], hp.num_features, True, hp.binary)
        return self._vec(out)


@register_stage
class IDFModel(VectorizerMixin, OpTransformer):
    operation_name = "idf"
    arity = 1

    def __init__(self, idf=None, uid=None, **kw):
        super().__init__(uid=uid, **kw)
        self.idf = None if idf is None else np.asarray(idf, np.float64)

    def transform_columns(self, *cols, ds=None):
        c = cols[0]
        w = torch.as_tensor(self.idf, dtype=c.values.dtype, device=c.values.device)
        return VectorColumn(c.values * w[None, :], c.metadata if self.metadata.get("vector_metadata") is None
                            else self.metadata["vector_metadata"])

    def ctor_args(self):
        return {"idf": self.idf.tolist()}

    def load_ctor_args(self, a):
        self.idf = np.asarray(a["idf"], np.float64)


@register_stage
class IDF(VectorizerMixin, UnaryEstimator):
    """Spark IDF: ``log((m + 1) / (df + 1))``, zeroed for terms with df < minDocFreq."""
    operation_name = "idf"
    _defaults = {"min_doc_freq": 0}
    dp_aware = True     # document frequencies and the row count are all-reduced (one packed collective)

    def fit_columns(self, *cols, ds=None):
        from ...parallel import dp
        x = cols[0].values
        m_t, df_t = dp.sum_([torch.tensor([float(x.shape[0])], dtype=torch.float64, device=x.device),
                             (x != 0).sum(0).to(torch.float64)])
        m = float(m_t.item())
        df = df_t.cpu().numpy()
        idf = np.log((m + 1.0) / (df + 1.0))
        idf[df < self.params["min_doc_freq"]] = 0.0
        if cols[0].metadata is not None:
            self.metadata["vector_metadata"] = cols[0].metadata.with_name(self.get_output_feature_name())
        return IDFModel(idf)


@register_stage
class TextRegexTokenizer(UnaryTransformer):
    """``tokenizeRegex`` (``RichTextFeature.scala:375-392``, ``LuceneRegexTextAnalyzer``): with ``group < 0``
    the text is split on ``pattern`` (empty tokens dropped); otherwise every match's ``group`` is a
    token. Lowercasing and the minimum token length apply as in ``TextTokenizer``."""
    operation_name = "textToken"
    output_type = T.TextList
    _defaults = {"pattern": r"\s+", "group": -1, "min_token_length": 1, "to_lowercase": True}

    def transform_fn(self, v):
        import re
        if v is None:
            return []
        p = self.params
        s = v.lower() if p["to_lowercase"] else v
        rx = re.compile(p["pattern"])
        g = int(p["group"])
        toks = [t for t in rx.split(s) if t] if g < 0 else [m.group(g) for m in rx.finditer(s) if m.group(g)]
        return [t for t in toks if len(t) >= int(p["min_token_length"])]


@register_stage
class ValidUrlTransformer(UnaryTransformer):
    """``URL.isValidUrl`` (``RichTextFeature.scala:651``): Binary flag of a well-formed http/https/ftp URL,
    empty for an empty input."""
    operation_name = "isValidUrl"
    output_type = T.Binary

    def transform_fn(self, v):
        return None if v is None else TU.is_valid_url(v)

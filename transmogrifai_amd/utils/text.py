"""Text utilities: cleaning, tokenization and Spark-compatible murmur3 hashing.

* :func:`clean_string` -- ``TextUtils.cleanString`` (``utils/.../text/TextUtils.scala:39-46``).
* :func:`tokenize` -- ``TextTokenizer.tokenizeString`` (``core/.../TextTokenizer.scala:160-188``) with the
  default analyzer ``StandardAnalyzer(english snowball stopwords)``
  (``core/.../utils/text/LuceneTextAnalyzer.scala:160-166``): a UAX#29-style word tokenizer
  (letters/digits/underscore words, ``'`` and ``.`` joining letters, ``.`` and ``,`` joining digits),
  lowercasing and stopword removal, max token length 255.
* :func:`hash_terms` -- bit-exact Spark ``HashingTF`` murmur3 indices (native host library).
"""
from __future__ import annotations

import re
from typing import Iterable, List, Optional, Sequence
from urllib.parse import urlparse

import numpy as np

_PUNCT = re.compile(r"[!\"#$%&'()*+,\-./:;<=>?@\[\\\]^_`{|}~]")
_SPACES = re.compile(" +")


def clean_string(raw: str, split_on: str = " ") -> str:
    s = raw.lower()
    s = _PUNCT.sub(split_on, s)
    s = re.sub(re.escape(split_on) + "+", split_on, s)
    parts = s.split(split_on)
    # Java's String.split drops trailing empty strings; capitalize() of "" is ""
    return "".join(p[:1].upper() + p[1:] for p in parts)


def clean_opt(raw: Optional[str], should_clean: bool = True) -> Optional[str]:
    if raw is None:
        return None
    return clean_string(raw) if should_clean else raw


# Snowball English stop words (Lucene's english_stop.txt, used by LuceneTextAnalyzer.DefaultAnalyzer)
ENGLISH_STOPWORDS = frozenset("""
i me my myself we our ours ourselves you your yours yourself yourselves he him his himself she her hers
herself it its itself they them their theirs themselves what which who whom this that these those am is
are was were be been being have has had having do does did doing would should could ought i'm you're
he's she's it's we're they're i've you've we've they've i'd you'd he'd she'd we'd they'd i'll you'll he'll
she'll we'll they'll isn't aren't wasn't weren't hasn't haven't hadn't doesn't don't didn't won't wouldn't
shan't shouldn't can't cannot couldn't mustn't let's that's who's what's here's there's when's where's
why's how's a an the and but if or because as until while of at by for with about against between into
through during before after above below to from up down in out on off over under again further then once
here there when where why how all any both each few more most other some such no nor not only own same so
than too very
""".split())



def _mark_class() -> str:
    """Regex class of the BMP combining marks (Mn, Mc, Me) and ZWJ / ZWNJ: UAX#29 Extend characters continue
    the word they follow (Devanagari vowel signs, Arabic harakat ...); scripts/gen/gen_unicode_tables.py gives
    the native tokenizer the same set."""
    import unicodedata
    runs, start = [], None
    for cp in range(0x10000):
        m = unicodedata.category(chr(cp)) in ("Mn", "Mc", "Me") or cp in (0x200C, 0x200D)
        if m and start is None:
            start = cp
        elif not m and start is not None:
            runs.append((start, cp - 1))
            start = None
    return "[" + "".join(f"\\u{a:04x}" if a == b else f"\\u{a:04x}-\\u{b:04x}" for a, b in runs) + "]"


_MARKS = _mark_class()
# word = runs of letters/digits/underscore (and the combining marks that follow them), letters may be joined by
# ' or . , digits by . or ,
_WORD = re.compile(
    r"[^\W\d_](?:[\w]|" + _MARKS + r"|['.](?=[^\W\d_]))*"          # letter-led word (may contain digits)
    r"|\d(?:[\w]|" + _MARKS + r"|[.,](?=\d))*"                      # number-led token
    r"|_+(?:\w|" + _MARKS + r")*",
    re.UNICODE)
_CJK = re.compile(r"[぀-ヿ㐀-䶿一-鿿가-힯]")

# CJK script classes (the code-point ranges of _CJK; ops/csrc/host/tokenizer.cpp uses the same)
HAN, HIRAGANA, KATAKANA, HANGUL = 1, 2, 3, 4


def cjk_class(ch: str) -> int:
    o = ord(ch)
    if 0x4E00 <= o <= 0x9FFF or 0x3400 <= o <= 0x4DBF:
        return HAN
    if 0x3040 <= o <= 0x309F:
        return HIRAGANA
    if 0x30A0 <= o <= 0x30FF:
        return KATAKANA
    if 0xAC00 <= o <= 0xD7AF:
        return HANGUL
    return 0


def _segments(tok: str):
    """StandardTokenizer (UAX#29) split of a word holding CJK characters: every ideograph and every hiragana
    is a token of its own, katakana and hangul runs are words, the other characters form ordinary words.
    Yields (text, is_cjk)."""
    i, n = 0, len(tok)
    while i < n:
        c = cjk_class(tok[i])
        j = i + 1
        if c in (KATAKANA, HANGUL):
            while j < n and cjk_class(tok[j]) == c:
                j += 1
        elif c == 0:
            while j < n and cjk_class(tok[j]) == 0:
                j += 1
        yield tok[i:j], c != 0
        i = j


def _plain(tok: str, stopwords, max_len: int, out: List[str]) -> None:
    tok = tok.lower()
    if len(tok) <= max_len and tok not in stopwords:
        out.append(tok)


def analyze(text: str, stopwords=ENGLISH_STOPWORDS, max_len: int = 255) -> List[str]:
    """StandardAnalyzer-style analysis (lowercase + stop filter) of an already lowercased or raw string."""
    out = []
    for m in _WORD.finditer(text):
        tok = m.group(0)
        if _CJK.search(tok):
            for seg, cjk in _segments(tok):
                if cjk:
                    if len(seg) <= max_len:
                        out.append(seg)
                elif _WORD.fullmatch(seg):
                    _plain(seg, stopwords, max_len, out)
                else:
                    for m2 in _WORD.finditer(seg):
                        _plain(m2.group(0), stopwords, max_len, out)
            continue
        _plain(tok, stopwords, max_len, out)
    return out


# CJKWidthFilter: full-width ASCII variants -> ASCII
_FULLWIDTH = {c: c - 0xFEE0 for c in range(0xFF01, 0xFF5F)}
_FULLWIDTH[0x3000] = 0x20


def analyze_cjk_bigrams(text: str, stopwords=ENGLISH_STOPWORDS, max_len: int = 255) -> List[str]:
    """Lucene ``CJKAnalyzer`` (``LuceneTextAnalyzer.scala``: Korean, Simplified and Traditional Chinese; English
    stop words): StandardTokenizer, CJKWidthFilter, lowercase, CJKBigramFilter over all four CJK scripts,
    stop filter. Adjacent CJK characters -- with no character between them in the text -- form one run; a run
    emits its overlapping bigrams, a run of one character the character itself. Other tokens pass through
    (``TextTokenizerTest.scala:145-181``: sliding 2-grams that do not cross spaces or punctuation)."""
    text = text.translate(_FULLWIDTH)
    out: List[str] = []
    for m in _WORD.finditer(text):
        tok = m.group(0)
        if not _CJK.search(tok):
            _plain(tok, stopwords, max_len, out)
            continue
        run = ""
        for seg, cjk in _segments(tok):
            if cjk:
                run += seg
                continue
            _flush_bigrams(run, out)
            run = ""
            for m2 in _WORD.finditer(seg):
                _plain(m2.group(0), stopwords, max_len, out)
        _flush_bigrams(run, out)
    return out


def _flush_bigrams(run: str, out: List[str]) -> None:
    if len(run) == 1:
        out.append(run)
    else:
        out.extend(run[k:k + 2] for k in range(len(run) - 1))


def tokenize(text: Optional[str], to_lowercase: bool = True, min_token_length: int = 1,
             stopwords=ENGLISH_STOPWORDS) -> List[str]:
    if text is None:
        return []
    s = text.lower() if to_lowercase else text
    return [t for t in analyze(s, stopwords) if len(t) >= min_token_length]


class TokenBatch:
    """Flat token list of a batch of strings: token ``t`` of string ``i`` is
    ``data[tok_offs[row_ptr[i] + t] : tok_offs[row_ptr[i] + t + 1]]`` (UTF-8)."""

    __slots__ = ("data", "tok_offs", "row_ptr")

    def __init__(self, data: np.ndarray, tok_offs: np.ndarray, row_ptr: np.ndarray):
        self.data, self.tok_offs, self.row_ptr = data, tok_offs, row_ptr

    def __len__(self):
        return self.row_ptr.size - 1

    @property
    def n_tokens(self) -> int:
        return self.tok_offs.size - 1

    def counts(self) -> np.ndarray:
        return np.diff(self.row_ptr)

    def token_char_lengths(self) -> np.ndarray:
        """Per-token length in characters (UTF-8 continuation bytes excluded), flat over the batch."""
        lead = (self.data & 0xC0) != 0x80
        cum = np.zeros(self.data.size + 1, np.int64)
        np.cumsum(lead, out=cum[1:])
        return cum[self.tok_offs[1:]] - cum[self.tok_offs[:-1]]

    def char_lengths(self) -> np.ndarray:
        """Per-string total token length in characters (UTF-8 continuation bytes excluded)."""
        tok_chars = self.token_char_lengths()
        tc = np.zeros(tok_chars.size + 1, np.int64)
        np.cumsum(tok_chars, out=tc[1:])
        return tc[self.row_ptr[1:]] - tc[self.row_ptr[:-1]]

    def lists(self) -> List[List[str]]:
        b = self.data.tobytes()
        o, r = self.tok_offs, self.row_ptr
        return [[b[o[t]:o[t + 1]].decode("utf-8") for t in range(r[i], r[i + 1])] for i in range(len(self))]

    @staticmethod
    def from_lists(lists: Sequence[Sequence[str]]) -> "TokenBatch":
        enc = [t.encode("utf-8") for l in lists for t in l]
        lens = np.fromiter((len(e) for e in enc), dtype=np.int64, count=len(enc))
        offs = np.zeros(len(enc) + 1, np.int64)
        np.cumsum(lens, out=offs[1:])
        rp = np.zeros(len(lists) + 1, np.int64)
        np.cumsum([len(l) for l in lists], out=rp[1:])
        return TokenBatch(np.frombuffer(b"".join(enc), dtype=np.uint8).copy(), offs, rp)


# Results of the batch text functions for the vocabularies they last ran on: SmartText's fit and transform (and the
# hashing of the same columns) clean / tokenise the same vocabulary list objects. Keyed by the list object itself
# (held, so its id cannot be reused) and the parameters; lists are never mutated after a column is built.
_BATCH_CACHE: "OrderedDict[tuple, tuple]" = None
_BATCH_CACHE_SIZE = 24


def clear_batch_cache() -> None:
    """Forget every cached batch result (``OpWorkflow.train`` starts each train with an empty cache)."""
    global _BATCH_CACHE
    _BATCH_CACHE = None


def _cached(strings, kind, params, fn):
    global _BATCH_CACHE
    from collections import OrderedDict
    if _BATCH_CACHE is None:
        _BATCH_CACHE = OrderedDict()
    if not isinstance(strings, list) or len(strings) < 1024:
        return fn()
    key = (id(strings), len(strings), kind, params)
    hit = _BATCH_CACHE.get(key)
    if hit is not None and hit[0] is strings:
        _BATCH_CACHE.move_to_end(key)
        return hit[1]
    out = fn()
    _BATCH_CACHE[key] = (strings, out)
    while len(_BATCH_CACHE) > _BATCH_CACHE_SIZE:
        _BATCH_CACHE.popitem(last=False)
    return out


def _encode_batch(strings: Sequence[Optional[str]]):
    return _cached(strings, "utf8", (), lambda: _encode_batch_impl(strings))


def _encode_batch_impl(strings: Sequence[Optional[str]]):
    if isinstance(strings, list) and strings:
        # straight from the str objects (ops/csrc/host/utf8_pack.cpp); -1 (a non-str item, a lone surrogate)
        # falls through to the encode-and-join path
        from ..ops import _native as N
        lib = N.pyhost()
        offs = np.empty(len(strings) + 1, np.int64)
        tot = int(lib.tmog_utf8_offsets(strings, offs.ctypes.data))
        if tot >= 0:
            buf = np.empty(max(tot, 1), np.uint8)
            if tot == 0:
                buf[0] = 0
            if lib.tmog_utf8_copy(strings, offs.ctypes.data, buf.ctypes.data) == 0:
                return buf, offs
    enc = [s.encode("utf-8") if s else b"" for s in strings]
    offs = np.zeros(len(enc) + 1, np.int64)
    np.cumsum(np.fromiter((len(e) for e in enc), dtype=np.int64, count=len(enc)), out=offs[1:])
    return np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8), offs


class CleanedBatch:
    """:func:`clean_string` (or the raw value) of every string of a vocabulary, kept as one UTF-8 buffer with
    per-string byte ranges, plus the first-appearance id of each cleaned value (equal cleaned strings share
    an id) and its length in characters. Strings are decoded only when :meth:`value` asks for them."""

    def __init__(self, buf: np.ndarray, starts: np.ndarray, ends: np.ndarray, ids: np.ndarray, n_ids: int,
                 char_len: np.ndarray):
        self.buf, self.starts, self.ends = buf, starts, ends
        self.ids, self.n_ids, self.char_len = ids, n_ids, char_len

    def value(self, j: int) -> str:
        return self.buf[self.starts[j]:self.ends[j]].tobytes().decode("utf-8")


def clean_batch(strings: Sequence[Optional[str]], clean: bool = True) -> CleanedBatch:
    """Native batch of :func:`clean_string` (``ops/csrc/host/text_clean.cpp``): ASCII strings are cleaned in
    C++, the rest (Unicode case mapping) by :func:`clean_string`; ids by exact cleaned bytes."""
    return _cached(strings, "clean", (bool(clean),), lambda: _clean_batch_impl(strings, clean))


def _clean_batch_impl(strings: Sequence[Optional[str]], clean: bool = True) -> CleanedBatch:
    from ..ops import _native as N
    lib = N.host()
    n = len(strings)
    buf, offs = _encode_batch(strings)
    if clean:
        out = np.empty(max(int(offs[-1]), 1), np.uint8)
        lens = np.empty(max(n, 1), np.int64)
        fb = np.zeros(max(n, 1), np.uint8)
        # cleaned string i in place of its input bytes (never longer), in parallel
        lib.tmog_clean_ascii_lens(buf.ctypes.data, offs.ctypes.data, n, out.ctypes.data, lens.ctypes.data,
                                  fb.ctypes.data)
        starts = offs[:-1].copy()
        ends = starts + lens[:n]
        char_len = lens[:n].copy()
        bad = np.flatnonzero(fb[:n])
        if bad.size:
            extra = [clean_string(strings[i] or "").encode("utf-8") for i in bad]
            base = int(offs[-1])
            lens = np.fromiter((len(e) for e in extra), dtype=np.int64, count=bad.size)
            starts[bad] = base + np.concatenate([[0], np.cumsum(lens)[:-1]])
            ends[bad] = starts[bad] + lens
            out = np.concatenate([out[:base], np.frombuffer(b"".join(extra) or b"\0", np.uint8)])
            char_len[bad] = [len(e.decode("utf-8")) for e in extra]
    else:
        out, starts, ends = buf, offs[:-1].copy(), offs[1:].copy()
        char_len = np.fromiter((len(s) if s else 0 for s in strings), dtype=np.int64, count=n)
    ids = np.empty(max(n, 1), np.int64)
    n_ids = int(lib.tmog_first_ids(out.ctypes.data, starts.ctypes.data, ends.ctypes.data, n, ids.ctypes.data))
    return CleanedBatch(out, starts, ends, ids[:n], n_ids, char_len)


def tokenize_batch(strings: Sequence[Optional[str]], to_lowercase: bool = True, min_token_length: int = 1,
                   stopwords=ENGLISH_STOPWORDS) -> TokenBatch:
    """:func:`tokenize` of every string at once through the native multithreaded tokenizer
    (``ops/csrc/host/tokenizer.cpp``). Strings the native tables flag (context-dependent lowercase,
    non-BMP code points) and custom stop-word sets go through :func:`tokenize`, so the result always
    equals ``[tokenize(s, ...) for s in strings]``."""
    if stopwords is ENGLISH_STOPWORDS or len(stopwords) == 0:
        return _cached(strings, "tok", (bool(to_lowercase), int(min_token_length), stopwords is ENGLISH_STOPWORDS),
                       lambda: _tokenize_batch_impl(strings, to_lowercase, min_token_length, stopwords))
    return _tokenize_batch_impl(strings, to_lowercase, min_token_length, stopwords)


def _tokenize_batch_impl(strings, to_lowercase, min_token_length, stopwords) -> TokenBatch:
    from ..ops import _native as N
    n = len(strings)
    if stopwords is not ENGLISH_STOPWORDS and len(stopwords) > 0:
        return TokenBatch.from_lists([tokenize(s, to_lowercase, min_token_length, stopwords) for s in strings])
    use_stop = 1 if stopwords is ENGLISH_STOPWORDS else 0
    buf, offs = _encode_batch(strings)
    lib = N.host()
    h = lib.tmog_tok_run(buf.ctypes.data, offs.ctypes.data, n, int(to_lowercase), int(min_token_length), use_stop)
    try:
        nt, nb = np.zeros(1, np.int64), np.zeros(1, np.int64)
        lib.tmog_tok_sizes(h, nt.ctypes.data, nb.ctypes.data)
        data = np.empty(max(int(nb[0]), 1), np.uint8)
        tok_offs = np.empty(int(nt[0]) + 1, np.int64)
        row_ptr = np.empty(n + 1, np.int64)
        fb = np.zeros(max(n, 1), np.uint8)
        lib.tmog_tok_copy(h, data.ctypes.data, tok_offs.ctypes.data, row_ptr.ctypes.data, fb.ctypes.data)
    finally:
        lib.tmog_tok_free(h)
    tb = TokenBatch(data[:int(nb[0])], tok_offs, row_ptr)
    bad = np.flatnonzero(fb[:n])
    if bad.size:
        lists = tb.lists()
        for i in bad:
            lists[i] = tokenize(strings[i], to_lowercase, min_token_length, stopwords)
        tb = TokenBatch.from_lists(lists)
    return tb


def strip_html(text: str) -> str:
    return re.sub(r"<[^>]*>", " ", text)


def hash_terms(terms: Sequence[str], num_features: int, seed: int = 42) -> np.ndarray:
    """``nonNegativeMod(murmur3_x86_32(utf8(term), 42), num_features)`` for every term (Spark HashingTF)."""
    from ..ops import _native as N
    n = len(terms)
    if n == 0:
        return np.zeros(0, np.int32)
    enc = [t.encode("utf-8") for t in terms]
    lens = np.fromiter((len(e) for e in enc), dtype=np.int64, count=n)
    offs = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=offs[1:])
    buf = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8)
    out = np.empty(n, np.int32)
    N.check(N.host().tmog_hash_index_batch(buf.ctypes.data, offs.ctypes.data, n, seed, num_features,
                                            out.ctypes.data), "hash_index_batch")
    return out


def murmur3(terms: Sequence[str], seed: int = 42) -> np.ndarray:
    from ..ops import _native as N
    n = len(terms)
    enc = [t.encode("utf-8") for t in terms]
    lens = np.fromiter((len(e) for e in enc), dtype=np.int64, count=n)
    offs = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=offs[1:])
    buf = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8)
    out = np.empty(n, np.int32)
    N.check(N.host().tmog_murmur3_batch(buf.ctypes.data, offs.ctypes.data, n, seed, out.ctypes.data), "murmur3")
    return out


# ------------------------------------------------------------------------------ email / url helpers
# Email.pattern (features/.../types/Text.scala:87-89): prefix @ domain of zero or more dot-separated labels, so
# "a@b" is valid; prefix / domain are the two groups of a full match (None otherwise)
_EMAIL = re.compile(r"^([A-Za-z0-9.!#$%&'*+/=?^_`{|}~-]+)@([A-Za-z0-9](?:[A-Za-z0-9-]{0,61}[A-Za-z0-9])?"
                    r"(?:\.[A-Za-z0-9](?:[A-Za-z0-9-]{0,61}[A-Za-z0-9])?)*)$")


def _email_parts(s: Optional[str]):
    m = _EMAIL.match(s) if s is not None else None
    return (m.group(1), m.group(2)) if m else (None, None)


def is_valid_email(s: Optional[str]) -> bool:
    """``ValidEmailTransformer`` (ValidEmailTransformer.scala:43): prefix and domain both parse."""
    p, d = _email_parts(s)
    return bool(p) and bool(d)


def email_domain(s: Optional[str]) -> Optional[str]:
    return _email_parts(s)[1] or None


def email_prefix(s: Optional[str]) -> Optional[str]:
    return _email_parts(s)[0] or None


_HOST = re.compile(r"^(?:[A-Za-z0-9](?:[A-Za-z0-9-]{0,61}[A-Za-z0-9])?\.)+[A-Za-z]{2,63}$")
_IPV4 = re.compile(r"^(?:25[0-5]|2[0-4]\d|1?\d?\d)(?:\.(?:25[0-5]|2[0-4]\d|1?\d?\d)){3}$")


def is_valid_url(s: Optional[str], schemes=("http", "https", "ftp")) -> bool:
    """Apache ``UrlValidator`` (default schemes http / https / ftp): a listed scheme, an authority whose host is
    a dotted ASCII domain name (labels of letters, digits and inner hyphens, an alphabetic top label) or an
    IPv4 address, an optional numeric port, and no whitespace."""
    if not s or any(c.isspace() for c in s):
        return False
    try:
        u = urlparse(s)
        port = u.port
    except ValueError:
        return False
    if u.scheme.lower() not in schemes or not u.netloc or u.username or u.password:
        return False
    host = u.hostname or ""
    del port
    return bool(_HOST.match(host) or _IPV4.match(host))


def url_domain(s: Optional[str]) -> Optional[str]:
    if not s:
        return None
    try:
        u = urlparse(s)
    except ValueError:
        return None
    return u.hostname or None


def url_protocol(s: Optional[str]) -> Optional[str]:
    if not s:
        return None
    try:
        return urlparse(s).scheme or None
    except ValueError:
        return None

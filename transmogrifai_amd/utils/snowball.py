"""Snowball stemmers of the Lucene language analyzers that ``LuceneTextAnalyzer.scala:169-206`` maps (the
RussianAnalyzer and DutchAnalyzer run ``SnowballFilter`` with these algorithms after their stop filters).

Implemented from the published Snowball algorithm descriptions (snowballstem.org), not from any code:

* :func:`russian_stem` -- perfective gerund / reflexive / adjectival / verb / noun endings in RV, final и,
  derivational ост(ь) in R2, superlative, undoubled н and final ь.
* :func:`dutch_stem` -- accent removal, Y / I marking, en / s / e / heid / end / ing / ig / lijk / baar / bar
  endings, undoubling, and the vowel undoubling of step 4; DutchAnalyzer's stem overrides (fiets, bromfiets,
  ei, kind) are applied first, as its StemmerOverrideFilter does.

``among`` semantics: of the listed suffixes the longest one present is taken, and its condition decides;
a failing condition does not fall back to a shorter suffix.
"""
from __future__ import annotations

from typing import Iterable, Optional, Tuple

# ------------------------------------------------------------------------------------------------ Russian
_RU_V = set("аеиоуыэюя")


def _ru_regions(w: str) -> Tuple[int, int]:
    """(RV, R2): RV after the first vowel; R1 after the first non-vowel following a vowel; R2 the same in R1."""
    rv = len(w)
    for i, c in enumerate(w):
        if c in _RU_V:
            rv = i + 1
            break

    def r_after(start: int) -> int:
        for i in range(start + 1, len(w)):
            if w[i] not in _RU_V and w[i - 1] in _RU_V:
                return i + 1
        return len(w)
    r1 = r_after(0)
    return rv, r_after(r1) if r1 < len(w) else len(w)


def _longest(w: str, lo: int, sufs: Iterable[str]) -> Optional[str]:
    """Longest suffix of ``w`` from ``sufs`` lying entirely at or after position ``lo``."""
    best = None
    for s in sufs:
        if w.endswith(s) and len(w) - len(s) >= lo and (best is None or len(s) > len(best)):
            best = s
    return best


_RU_PG1 = ("в", "вши", "вшись")
_RU_PG2 = ("ив", "ивши", "ившись", "ыв", "ывши", "ывшись")
_RU_ADJ = ("ее", "ие", "ые", "ое", "ими", "ыми", "ей", "ий", "ый", "ой", "ем", "им", "ым", "ом", "его", "ого", "ему",
           "ому", "их", "ых", "ую", "юю", "ая", "яя", "ою", "ею")
_RU_PART1 = ("ем", "нн", "вш", "ющ", "щ")
_RU_PART2 = ("ивш", "ывш", "ующ")
_RU_REFL = ("ся", "сь")
_RU_VERB1 = ("ла", "на", "ете", "йте", "ли", "й", "л", "ем", "н", "ло", "но", "ет", "ют", "ны", "ть", "ешь", "нно")
_RU_VERB2 = ("ила", "ыла", "ена", "ейте", "уйте", "ите", "или", "ыли", "ей", "уй", "ил", "ыл", "им", "ым", "ен", "ило",
             "ыло", "ено", "ят", "ует", "уют", "ит", "ыт", "ены", "ить", "ыть", "ишь", "ую", "ю")
_RU_NOUN = ("а", "ев", "ов", "ие", "ье", "е", "иями", "ями", "ами", "еи", "ии", "и", "ией", "ей", "ой", "ий", "й", "иям",
            "ям", "ием", "ем", "ам", "ом", "о", "у", "ах", "иях", "ях", "ы", "ь", "ию", "ью", "ю", "ия", "ья", "я")


def _ru_remove(w: str, rv: int, g1: Tuple[str, ...], g2: Tuple[str, ...]) -> Optional[str]:
    s = _longest(w, rv, g1 + g2)
    if s is None:
        return None
    k = len(w) - len(s)
    if s in g2:
        return w[:k]
    return w[:k] if k - 1 >= rv and w[k - 1] in "ая" else None


def russian_stem(word: str) -> str:
    w = word.replace("ё", "е")
    rv, r2 = _ru_regions(w)
    # step 1
    out = _ru_remove(w, rv, _RU_PG1, _RU_PG2)
    if out is None:
        s = _longest(w, rv, _RU_REFL)
        if s is not None:
            w = w[:-len(s)]
        out = None
        a = _longest(w, rv, _RU_ADJ)
        if a is not None:                         # adjectival: adjective, then an optional participle
            out = w[:-len(a)]
            p = _ru_remove(out, rv, _RU_PART1, _RU_PART2)
            if p is not None:
                out = p
        if out is None:
            out = _ru_remove(w, rv, _RU_VERB1, _RU_VERB2)
        if out is None:
            n = _longest(w, rv, _RU_NOUN)
            out = w[:-len(n)] if n is not None else w
    w = out
    # step 2
    if w.endswith("и") and len(w) - 1 >= rv:
        w = w[:-1]
    # step 3: derivational, in R2
    d = _longest(w, r2, ("ост", "ость"))
    if d is not None:
        w = w[:-len(d)]
    # step 4
    if w.endswith("нн") and len(w) - 2 >= rv:
        w = w[:-1]
    else:
        s = _longest(w, rv, ("ейш", "ейше"))
        if s is not None:
            w = w[:-len(s)]
            if w.endswith("нн") and len(w) - 2 >= rv:
                w = w[:-1]
        elif w.endswith("ь") and len(w) - 1 >= rv:
            w = w[:-1]
    return w


# ------------------------------------------------------------------------------------------------- Dutch
_NL_V = set("aeiouyè")
_NL_ACCENTS = str.maketrans("äëïöüáéíóú", "aeiouaeiou")
# DutchAnalyzer's default StemmerOverrideFilter dictionary
_NL_OVERRIDE = {"fiets": "fiets", "bromfiets": "bromfiets", "ei": "eier", "kind": "kinder"}


def _nl_mark(w: str) -> str:
    """Initial y and y after a vowel -> Y; i between vowels -> I (so they count as consonants)."""
    c = list(w)
    for i, ch in enumerate(c):
        if ch == "y" and (i == 0 or c[i - 1] in _NL_V):
            c[i] = "Y"
        elif ch == "i" and 0 < i < len(c) - 1 and c[i - 1] in _NL_V and c[i + 1] in _NL_V:
            c[i] = "I"
    return "".join(c)


def _nl_regions(w: str) -> Tuple[int, int]:
    def r_after(start: int) -> int:
        for i in range(start + 1, len(w)):
            if w[i] not in _NL_V and w[i - 1] in _NL_V:
                return i + 1
        return len(w)
    r1 = r_after(0)
    r2 = r_after(r1) if r1 < len(w) else len(w)
    return max(3, r1), r2


def _nl_undouble(w: str) -> str:
    return w[:-1] if w.endswith(("kk", "dd", "tt")) else w


def _nl_valid_en(w: str, k: int) -> bool:
    """The text before position k ends in a non-vowel and is not 'gem'."""
    return k >= 1 and w[k - 1] not in _NL_V and not w[:k].endswith("gem")


def dutch_stem(word: str) -> str:
    if word in _NL_OVERRIDE:
        return _NL_OVERRIDE[word]
    w = _nl_mark(word.translate(_NL_ACCENTS))
    r1, r2 = _nl_regions(w)
    # step 1
    s = _longest(w, 0, ("heden", "ene", "en", "se", "s"))
    if s == "heden":
        if len(w) - 5 >= r1:
            w = w[:-5] + "heid"
    elif s in ("en", "ene"):
        k = len(w) - len(s)
        if k >= r1 and _nl_valid_en(w, k):
            w = _nl_undouble(w[:k])
    elif s in ("s", "se"):
        k = len(w) - len(s)
        if k >= r1 and k >= 1 and w[k - 1] not in _NL_V and w[k - 1] != "j":
            w = w[:k]
    # step 2
    e_found = False
    if w.endswith("e") and len(w) - 1 >= r1 and len(w) >= 2 and w[-2] not in _NL_V:
        w = _nl_undouble(w[:-1])
        e_found = True
    # step 3a
    if w.endswith("heid") and len(w) - 4 >= r2 and not w[:-4].endswith("c"):
        w = w[:-4]
        k = len(w) - 2
        if w.endswith("en") and k >= r1 and _nl_valid_en(w, k):
            w = _nl_undouble(w[:k])
    # step 3b
    s = _longest(w, 0, ("end", "ing", "ig", "lijk", "baar", "bar"))
    if s in ("end", "ing"):
        if len(w) - 3 >= r2:
            w = w[:-3]
            if w.endswith("ig") and len(w) - 2 >= r2 and not w[:-2].endswith("e"):
                w = w[:-2]
            else:
                w = _nl_undouble(w)
    elif s == "ig":
        if len(w) - 2 >= r2 and not w[:-2].endswith("e"):
            w = w[:-2]
    elif s == "lijk":
        if len(w) - 4 >= r2:
            w = w[:-4]
            if w.endswith("e") and len(w) - 1 >= r1 and len(w) >= 2 and w[-2] not in _NL_V:
                w = _nl_undouble(w[:-1])
    elif s == "baar":
        if len(w) - 4 >= r2:
            w = w[:-4]
    elif s == "bar":
        if len(w) - 3 >= r2 and e_found:
            w = w[:-3]
    # step 4: undouble a vowel -- C + (aa|ee|oo|uu) + non-vowel other than I at the end
    if len(w) >= 4 and w[-1] not in _NL_V and w[-1] != "I" and w[-2] == w[-3] and w[-2] in "aeou" \
            and w[-4] not in _NL_V:
        w = w[:-2] + w[-1]
    return w.replace("Y", "y").replace("I", "i")

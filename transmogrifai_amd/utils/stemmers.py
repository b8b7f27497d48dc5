"""Stemmers of the per-language Lucene analyzers the reference tokenizes with (``LuceneTextAnalyzer.scala:87-126``,
Lucene 7.3 ``*Analyzer`` chains):

* French ``FrenchLightStemFilter``, German ``GermanNormalizationFilter`` + ``GermanLightStemFilter``, Spanish /
  Italian / Portuguese ``*LightStemFilter`` and Norwegian (bokmål) ``NorwegianLightStemFilter`` -- J. Savoy's light
  stemmers, which those analyzers use;
* Swedish and Danish: the Snowball stemmers of ``SwedishAnalyzer`` / ``DanishAnalyzer``.
* Indonesian ``IndonesianStemFilter`` (F. Tala's algorithm) and Latvian ``LatvianStemFilter`` (K. Kreslins' light
  stemmer);

Implemented from the published algorithms (Savoy, "Light stemming approaches for the French, Portuguese, German
and Hungarian languages", SAC 2006; snowballstem.org), not from Lucene's sources; the French one is pinned by the
reference's own expectations (``TextTokenizerTest.scala`` French fixture, ``tests/test_language.py``). English
(Porter) is in :mod:`.stemmer`.
"""
from __future__ import annotations

from typing import Callable, Dict, List

_ACC_A = {"à": "a", "á": "a", "â": "a", "ä": "a"}
_ACC_O = {"ò": "o", "ó": "o", "ô": "o", "ö": "o"}
_ACC_E = {"è": "e", "é": "e", "ê": "e", "ë": "e"}
_ACC_U = {"ù": "u", "ú": "u", "û": "u", "ü": "u"}
_ACC_I = {"ì": "i", "í": "i", "î": "i", "ï": "i"}
_ROMANCE = {**_ACC_A, **_ACC_O, **_ACC_E, **_ACC_U, **_ACC_I}


# ------------------------------------------------------------------------------------------------ French
_FR_NORM = {"à": "a", "á": "a", "â": "a", "ô": "o", "è": "e", "é": "e", "ê": "e", "ù": "u", "û": "u", "î": "i",
            "ç": "c"}


def _fr_norm(s: List[str]) -> List[str]:
    if len(s) > 4:
        s = [_FR_NORM.get(c, c) for c in s]
        out = [s[0]]
        for c in s[1:]:                       # collapse doubled letters (commission -> comision)
            if c == out[-1] and c.isalpha():
                continue
            out.append(c)
        s = out
    if len(s) > 4 and s[-2:] == ["i", "e"]:
        s = s[:-2]
    if len(s) > 4:
        if s[-1] == "r":
            s = s[:-1]
        if s[-1] == "e":
            s = s[:-1]
        if s[-1] == "e":
            s = s[:-1]
        if s[-1] == s[-2] and s[-1].isalpha():
            s = s[:-1]
    return s


def french_light_stem(word: str) -> str:
    s = list(word)
    n = len

    def ends(x):
        return "".join(s[-len(x):]) == x if len(s) >= len(x) else False

    if n(s) > 5 and s[-1] == "x":
        if s[-3] == "a" and s[-2] == "u" and s[-4] != "e":
            s[-2] = "l"
        s = s[:-1]
    if n(s) > 3 and s[-1] == "x":
        s = s[:-1]
    if n(s) > 3 and s[-1] == "s":
        s = s[:-1]
    if n(s) > 9 and ends("issement"):
        s = s[:-6]
        s[-1] = "r"
        return "".join(_fr_norm(s))
    if n(s) > 8 and ends("issant"):
        s = s[:-4]
        s[-1] = "r"
        return "".join(_fr_norm(s))
    if n(s) > 6 and ends("ement"):
        s = s[:-4]
        if n(s) > 3 and ends("ive"):
            s = s[:-1]
            s[-1] = "f"
        return "".join(_fr_norm(s))
    if n(s) > 11 and ends("ficatrice"):
        s = s[:-5]
        s[-2:] = ["e", "r"]
        return "".join(_fr_norm(s))
    if n(s) > 10 and ends("ficateur"):
        s = s[:-4]
        s[-2:] = ["e", "r"]
        return "".join(_fr_norm(s))
    if n(s) > 9 and ends("catrice"):
        s = s[:-3]
        s[-4:-1] = ["q", "u", "e"]
        return "".join(_fr_norm(s))
    if n(s) > 8 and ends("cateur"):
        s = s[:-2]
        s[-4:] = ["q", "u", "e", "r"]
        return "".join(_fr_norm(s))
    if n(s) > 8 and ends("atrice"):
        s = s[:-4]
        s[-2:] = ["e", "r"]
        return "".join(_fr_norm(s))
    if n(s) > 7 and ends("ateur"):
        s = s[:-3]
        s[-2:] = ["e", "r"]
        return "".join(_fr_norm(s))
    if n(s) > 6 and ends("trice"):
        s = s[:-1]
        s[-3:] = ["e", "u", "r"]
    if n(s) > 5 and ends("ième"):
        return "".join(_fr_norm(s[:-4]))
    if n(s) > 7 and ends("teuse"):
        s = s[:-2]
        s[-1] = "r"
        return "".join(_fr_norm(s))
    if n(s) > 6 and ends("teur"):
        s = s[:-1]
        s[-1] = "r"
        return "".join(_fr_norm(s))
    if n(s) > 5 and ends("euse"):
        return "".join(_fr_norm(s[:-2]))
    if n(s) > 8 and ends("ère"):
        s = s[:-1]
        s[-2] = "e"
        return "".join(_fr_norm(s))
    if n(s) > 7 and ends("ive"):
        s = s[:-1]
        s[-1] = "f"
        return "".join(_fr_norm(s))
    if n(s) > 4 and (ends("folle") or ends("molle")):
        s = s[:-2]
        s[-1] = "u"
        return "".join(_fr_norm(s))
    if n(s) > 9 and ends("nnelle"):
        return "".join(_fr_norm(s[:-5]))
    if n(s) > 9 and ends("nnel"):
        return "".join(_fr_norm(s[:-3]))
    if n(s) > 4 and ends("ète"):
        s = s[:-1]
        s[-2] = "e"
    if n(s) > 8 and ends("ique"):
        s = s[:-4]
    if n(s) > 8 and ends("esse"):
        return "".join(_fr_norm(s[:-3]))
    if n(s) > 7 and ends("inage"):
        return "".join(_fr_norm(s[:-3]))
    if n(s) > 9 and ends("isation"):
        s = s[:-7]
        if n(s) > 5 and ends("ual"):
            s[-2] = "e"
        return "".join(_fr_norm(s))
    if n(s) > 9 and ends("isateur"):
        return "".join(_fr_norm(s[:-7]))
    if n(s) > 8 and ends("ation"):
        return "".join(_fr_norm(s[:-5]))
    if n(s) > 8 and ends("ition"):
        return "".join(_fr_norm(s[:-5]))
    return "".join(_fr_norm(s))


# ------------------------------------------------------------------------------------------------ German
def german_normalize(word: str) -> str:
    """GermanNormalizationFilter: umlauts folded, ß -> ss, and 'ae' / 'oe' / 'ue' (not after q) -> a / o / u."""
    out: List[str] = []
    state = 0          # 0: other, 1: after a vowel that blocks, 2: after a / o / u (an 'e' next is dropped)
    for c in word:
        if c in "ao":
            state = 2
            out.append(c)
        elif c == "u":
            state = 2 if state == 0 else 1
            out.append(c)
        elif c == "e":
            if state != 2:
                out.append(c)
            state = 1
        elif c in "iqy":
            state = 1
            out.append(c)
        elif c == "ä":
            out.append("a")
            state = 1
        elif c == "ö":
            out.append("o")
            state = 1
        elif c == "ü":
            out.append("u")
            state = 1
        elif c == "ß":
            out.append("ss")
            state = 0
        else:
            state = 0
            out.append(c)
    return "".join(out)


_DE_FOLD = {**_ACC_A, **_ACC_O, **_ACC_I, **_ACC_U}
_ST_ENDING = set("bdfghklmnt")


def german_light_stem(word: str) -> str:
    s = [_DE_FOLD.get(c, c) for c in word]
    n = len(s)
    # step 1
    if n > 5 and s[-3:] == ["e", "r", "n"]:
        s = s[:-3]
    elif n > 4 and s[-2] == "e" and s[-1] in "mnrs":
        s = s[:-2]
    elif n > 3 and s[-1] == "e":
        s = s[:-1]
    elif n > 3 and s[-1] == "s" and s[-2] in _ST_ENDING:
        s = s[:-1]
    n = len(s)
    # step 2
    if n > 5 and s[-3:] == ["e", "s", "t"]:
        s = s[:-3]
    elif n > 4 and s[-2] == "e" and s[-1] in "rn":
        s = s[:-2]
    elif n > 4 and s[-2:] == ["s", "t"] and s[-3] in _ST_ENDING:
        s = s[:-2]
    return "".join(s)


def german_analyze_stem(word: str) -> str:
    return german_light_stem(german_normalize(word))


# ----------------------------------------------------------------------------------- Spanish / Italian
def spanish_light_stem(word: str) -> str:
    if len(word) < 5:
        return word
    s = [_ROMANCE.get(c, c) for c in word]
    c = s[-1]
    if c in "oae":
        return "".join(s[:-1])
    if c == "s":
        if s[-2] == "e" and s[-3] == "s" and s[-4] == "e":
            return "".join(s[:-2])
        if s[-2] == "e" and s[-3] == "c":
            s[-3] = "z"
            return "".join(s[:-2])
        if s[-2] in "oae":
            return "".join(s[:-2])
    return "".join(s)


def italian_light_stem(word: str) -> str:
    if len(word) < 6:
        return word
    s = [_ROMANCE.get(c, c) for c in word]
    c, p = s[-1], s[-2]
    if c == "e":
        return "".join(s[:-2] if p in "ih" else s[:-1])
    if c == "i":
        return "".join(s[:-2] if p in "hi" else s[:-1])
    if c in "ao":
        return "".join(s[:-2] if p == "i" else s[:-1])
    return "".join(s)


# ---------------------------------------------------------------------------------------------- Portuguese
_PT_FOLD = {**_ROMANCE, "ã": "a", "õ": "o", "ç": "c"}


def _endsl(s: List[str], x: str) -> bool:
    return len(s) >= len(x) and "".join(s[-len(x):]) == x


def _pt_remove_suffix(s: List[str]) -> List[str]:
    n = len(s)
    if n > 4 and _endsl(s, "es") and s[-3] in "rslz":
        return s[:-2]
    if n > 3 and _endsl(s, "ns"):
        s[-2] = "m"
        return s[:-1]
    if n > 4 and (_endsl(s, "eis") or _endsl(s, "éis")):
        s[-3], s[-2] = "e", "l"
        return s[:-1]
    if n > 4 and _endsl(s, "ais"):
        s[-2] = "l"
        return s[:-1]
    if n > 4 and _endsl(s, "óis"):
        s[-3], s[-2] = "o", "l"
        return s[:-1]
    if n > 4 and _endsl(s, "is"):
        s[-1] = "l"
        return s
    if n > 3 and (_endsl(s, "ões") or _endsl(s, "ães")):
        s = s[:-1]
        s[-2], s[-1] = "ã", "o"
        return s
    if n > 6 and _endsl(s, "mente"):
        return s[:-5]
    if n > 3 and s[-1] == "s":
        return s[:-1]
    return s


def _pt_norm_feminine(s: List[str]) -> List[str]:
    n = len(s)
    if n > 7 and (_endsl(s, "inha") or _endsl(s, "iaca") or _endsl(s, "eira")):
        s[-1] = "o"
        return s
    if n > 6:
        if any(_endsl(s, x) for x in ("osa", "ica", "ida", "ada", "iva", "ama")):
            s[-1] = "o"
            return s
        if _endsl(s, "ona"):
            s[-3], s[-2] = "ã", "o"
            return s[:-1]
        if _endsl(s, "ora"):
            return s[:-1]
        if _endsl(s, "esa"):
            s[-3] = "ê"
            return s[:-1]
        if _endsl(s, "na"):
            s[-1] = "o"
            return s
    return s


def portuguese_light_stem(word: str) -> str:
    if len(word) < 4:
        return word
    s = _pt_remove_suffix(list(word))
    if len(s) > 3 and s[-1] == "a":
        s = _pt_norm_feminine(s)
    if len(s) > 4 and s[-1] in "eao":
        s = s[:-1]
    return "".join(_PT_FOLD.get(c, c) for c in s)


# ------------------------------------------------------------------------------------------ Norwegian
def norwegian_light_stem(word: str) -> str:
    """NorwegianLightStemmer, bokmål (the NorwegianAnalyzer default)."""
    s = word
    if len(s) > 4 and s.endswith("s"):
        s = s[:-1]
    n = len(s)
    if n > 7 and (s.endswith("heter") or s.endswith("heten")):
        return s[:-5]
    if n > 5 and (s.endswith("dom") or s.endswith("het")):
        return s[:-3]
    if n > 7 and (s.endswith("elser") or s.endswith("elsen")):
        return s[:-5]
    if n > 6 and any(s.endswith(x) for x in ("ende", "else", "este", "eren")):
        return s[:-4]
    if n > 5 and any(s.endswith(x) for x in ("ere", "est", "ene")):
        return s[:-3]
    if n > 4 and any(s.endswith(x) for x in ("er", "en", "et", "st", "te")):
        return s[:-2]
    if n > 3 and s[-1] in "aen":
        return s[:-1]
    return s


# ---------------------------------------------------------------------------- Snowball: Swedish / Danish
def _r1(word: str, vowels: str) -> int:
    """Start of Snowball's R1 (after the first non-vowel following a vowel), at least 3."""
    for i in range(1, len(word)):
        if word[i] not in vowels and word[i - 1] in vowels:
            return max(3, i + 1)
    return len(word)


_SV_V = "aeiouyäåö"
_SV_S1 = sorted("a arna erna heterna orna ad e ade ande arne are aste en anden aren heten ern ar er heter or as "
                "arnas ernas ornas es ades andes ens arens hetens erns at andet het ast".split(), key=len, reverse=True)
_SV_SEND = set("bcdfghjklmnoprtvy")


def swedish_stem(word: str) -> str:
    r1 = _r1(word, _SV_V)
    w = word
    # step 1
    for suf in _SV_S1:
        if w.endswith(suf) and len(w) - len(suf) >= r1:
            w = w[:-len(suf)]
            break
    else:
        if w.endswith("s") and len(w) - 1 >= r1 and len(w) >= 2 and w[-2] in _SV_SEND:
            w = w[:-1]
    # step 2
    for suf in ("dd", "gd", "nn", "dt", "gt", "kt", "tt"):
        if w.endswith(suf) and len(w) - 2 >= r1:
            w = w[:-1]
            break
    # step 3
    for suf, rep in (("fullt", "full"), ("löst", "lös"), ("lig", ""), ("els", ""), ("ig", "")):
        if w.endswith(suf) and len(w) - len(suf) >= r1:
            w = w[:-len(suf)] + rep
            break
    return w


_DA_V = "aeiouyæåø"
_DA_S1 = sorted("hed ethed ered e erede ende erende ene erne ere en heden eren er heder erer heds es endes erendes "
                "enes ernes eres ens hedens erens ers ets erets et eret".split(), key=len, reverse=True)
_DA_SEND = set("abcdfghjklmnoprtvyzå")


def _da_step2(w: str, r1: int) -> str:
    for suf in ("gd", "dt", "gt", "kt"):
        if w.endswith(suf) and len(w) - 2 >= r1:
            return w[:-1]
    return w


def danish_stem(word: str) -> str:
    r1 = _r1(word, _DA_V)
    w = word
    for suf in _DA_S1:
        if w.endswith(suf) and len(w) - len(suf) >= r1:
            w = w[:-len(suf)]
            break
    else:
        if w.endswith("s") and len(w) - 1 >= r1 and len(w) >= 2 and w[-2] in _DA_SEND:
            w = w[:-1]
    w = _da_step2(w, r1)
    if w.endswith("igst"):
        w = w[:-2]
    for suf in ("elig", "lig", "els", "ig", "løst"):
        if w.endswith(suf) and len(w) - len(suf) >= r1:
            if suf == "løst":
                w = w[:-1]
            else:
                w = _da_step2(w[:-len(suf)], r1)
            break
    if len(w) >= 2 and len(w) - 1 >= r1 and w[-1] == w[-2] and w[-1] not in _DA_V and w[-1].isalpha():
        w = w[:-1]
    return w


# ------------------------------------------------------------------------------------------------- Arabic
# ArabicAnalyzer: StandardTokenizer, lower case, decimal digits to ASCII, the Arabic stop set, then
# ArabicNormalizationFilter and ArabicStemFilter (Larkey et al.'s light stemming as Lucene implements it).
_AR_NORM = {"\u0622": "\u0627", "\u0623": "\u0627", "\u0625": "\u0627",     # alef with madda / hamza -> alef
            "\u0649": "\u064a",                                            # dotless yeh -> yeh
            "\u0629": "\u0647"}                                            # teh marbuta -> heh
_AR_DROP = set("\u0640\u064b\u064c\u064d\u064e\u064f\u0650\u0651\u0652")    # tatweel, harakat
_AR_PREFIXES = ("\u0627\u0644", "\u0648\u0627\u0644", "\u0628\u0627\u0644", "\u0643\u0627\u0644",
                "\u0641\u0627\u0644", "\u0644\u0644", "\u0648")
_AR_SUFFIXES = ("\u0647\u0627", "\u0627\u0646", "\u0627\u062a", "\u0648\u0646", "\u064a\u0646",
                "\u064a\u0647", "\u064a\u0629", "\u0647", "\u0629", "\u064a")


def arabic_normalize(word: str) -> str:
    """ArabicNormalizer: alef forms -> bare alef, dotless yeh -> yeh, teh marbuta -> heh, tatweel and the
    harakat removed."""
    return "".join(_AR_NORM.get(c, c) for c in word if c not in _AR_DROP)


def arabic_light_stem(word: str) -> str:
    """ArabicStemmer: at most one prefix (wa- needs 3 letters left, the others 2), then every listed suffix in
    turn that leaves at least 2 letters."""
    w = word
    for p in _AR_PREFIXES:
        if (len(p) == 1 and len(w) < 4) or len(w) < len(p) + 2:
            continue
        if w.startswith(p):
            w = w[len(p):]
            break
    for sfx in _AR_SUFFIXES:
        if len(w) >= len(sfx) + 2 and w.endswith(sfx):
            w = w[:-len(sfx)]
    return w


def arabic_analyze_stem(word: str) -> str:
    return arabic_light_stem(arabic_normalize(word))


# PersianAnalyzer (no stemmer): ZWNJ splits words, then ArabicNormalizer and PersianNormalizer before the stop set
_FA_NORM = {"\u06cc": "\u064a", "\u06d2": "\u064a",           # farsi yeh, yeh barree -> yeh
            "\u06a9": "\u0643",                               # keheh -> kaf
            "\u06c0": "\u0647", "\u06c1": "\u0647"}          # heh with yeh, heh goal -> heh


def persian_normalize(word: str) -> str:
    """ArabicNormalizer then PersianNormalizer (yeh / kaf / heh variants folded, hamza above removed)."""
    return "".join(_FA_NORM.get(c, c) for c in arabic_normalize(word) if c != "\u0654")


# -------------------------------------------------------------------------------------------------- Hindi
# HindiAnalyzer: StandardTokenizer, lower case, decimal digits, the Hindi stop set, HindiNormalizer (orthographic
# variants folded), HindiStemmer (the longest suffix of a length class whose word is long enough; Ramanathan &
# Rao's light stemmer as Lucene implements it).
_HI_MAP = {"\u0901": "\u0902",                                                   # candrabindu -> bindu
           "\u0929": "\u0928", "\u0931": "\u0930", "\u0934": "\u0933",       # nukta letters -> base
           "\u0958": "\u0915", "\u0959": "\u0916", "\u095a": "\u0917", "\u095b": "\u091c",
           "\u095c": "\u0921", "\u095d": "\u0922", "\u095e": "\u092b", "\u095f": "\u092f",
           "\u0945": "\u0947", "\u0946": "\u0947", "\u0949": "\u094b", "\u094a": "\u094b",
           "\u090d": "\u090f", "\u090e": "\u090f", "\u0911": "\u0913", "\u0912": "\u0913",
           "\u0972": "\u0905", "\u0906": "\u0905", "\u0908": "\u0907", "\u090a": "\u0909",
           "\u0960": "\u090b", "\u0961": "\u090c", "\u0910": "\u090f", "\u0914": "\u0913",
           "\u0940": "\u093f", "\u0942": "\u0941", "\u0944": "\u0943", "\u0963": "\u0962",
           "\u0948": "\u0947", "\u094c": "\u094b"}
_HI_DROP = set("\u093c\u200d\u200c\u094d")                                   # nukta, ZWJ, ZWNJ, virama


def hindi_normalize(word: str) -> str:
    """HindiNormalizer: dead n (na + virama) -> anusvara, candrabindu -> anusvara, nukta forms -> their base
    letters, ZWJ / ZWNJ / virama removed, chandra and short e / o signs folded, long vowels -> short."""
    out = []
    i, n = 0, len(word)
    while i < n:
        c = word[i]
        if c == "\u0928" and i + 1 < n and word[i + 1] == "\u094d":
            out.append("\u0902")
            i += 2
            continue
        if c not in _HI_DROP:
            out.append(_HI_MAP.get(c, c))
        i += 1
    return "".join(out)


_HI_SUFFIXES = (
    (5, 6, ("ाएंगी", "ाएंगे", "ाऊंगी", "ाऊंगा", "ाइयाँ", "ाइयों", "ाइयां")),
    (4, 5, ("ाएगी", "ाएगा", "ाओगी", "ाओगे", "एंगी", "ेंगी", "एंगे", "ेंगे", "ूंगी", "ूंगा", "ातीं", "नाओं", "नाएं",
            "ताओं", "ताएं", "ियाँ", "ियों", "ियां")),
    (3, 4, ("ाकर", "ाइए", "ाईं", "ाया", "ेगी", "ेगा", "ोगी", "ोगे", "ाने", "ाना", "ाते", "ाती", "ाता", "तीं", "ाओं",
            "ाएं", "ुओं", "ुएं", "ुआं")),
    (2, 3, ("कर", "ाओ", "िए", "ाई", "ाए", "ने", "नी", "ना", "ते", "ीं", "ती", "ता", "ाँ", "ां", "ों", "ें")),
    (1, 2, ("ो", "े", "ू", "ु", "ी", "ि", "ा")),
)


def hindi_light_stem(word: str) -> str:
    """HindiStemmer: the first length class (5, 4, 3, 2, 1 characters) with a matching suffix whose word is longer
    than class length + 1 loses that suffix."""
    n = len(word)
    for k, min_len, sufs in _HI_SUFFIXES:
        if n > min_len and word.endswith(sufs):
            return word[:-k]
    return word


def hindi_analyze_stem(word: str) -> str:
    """HindiStemmer on a token already normalised before the stop filter (lang.analyze)."""
    return hindi_light_stem(word)


# ---------------------------------------------------------------------------------------------- Bulgarian
# BulgarianAnalyzer: StandardTokenizer, lower case, the Bulgarian stop set, BulgarianStemmer (Nakov's light
# stemmer as Lucene implements it: definite article, plural, final vowels, -ен, ъN).
def _bg_remove_article(w: str) -> str:
    n = len(w)
    if n > 6 and w.endswith("ият"):
        return w[:-3]
    if n > 5 and w.endswith(("ът", "то", "те", "та", "ия")):
        return w[:-2]
    if n > 4 and w.endswith("ят"):
        return w[:-2]
    return w


def _bg_remove_plural(w: str) -> str:
    n = len(w)
    if n > 6:
        if w.endswith("овци"):
            return w[:-3]                      # -овци -> -о
        if w.endswith("ове"):
            return w[:-3]
        if w.endswith("еве"):
            return w[:-3] + "й"                # -еве -> -й
    if n > 5:
        if w.endswith("ища"):
            return w[:-3]
        if w.endswith("та"):
            return w[:-2]
        if w.endswith("ци"):
            return w[:-2] + "к"
        if w.endswith("зи"):
            return w[:-2] + "г"
        if w[-3] == "е" and w[-1] == "и":
            return w[:-3] + "я" + w[-2]        # -еXи -> -яX
    if n > 4:
        if w.endswith("си"):
            return w[:-2] + "х"
        if w.endswith("и"):
            return w[:-1]
    return w


def bulgarian_stem(word: str) -> str:
    w = word
    if len(w) < 4:
        return w
    if len(w) > 5 and w.endswith("ища"):
        return w[:-3]
    w = _bg_remove_plural(_bg_remove_article(w))
    if len(w) > 3:
        if w.endswith("я"):
            w = w[:-1]
        if w.endswith(("а", "о", "е")):
            w = w[:-1]
    if len(w) > 4 and w.endswith("ен"):
        w = w[:-2] + "н"
    if len(w) > 5 and w[-2] == "ъ":
        w = w[:-2] + w[-1]
    return w


# -------------------------------------------------------------------------------------------------- Czech
# CzechAnalyzer: StandardTokenizer, lower case, the Czech stop set, CzechStemmer (Dolamic & Savoy's light
# stemmer as Lucene implements it: case endings, possessives, then a normalisation of the final consonants).
_CS_CASE = (
    (7, ("atech",)),
    (6, ("ětem", "etem", "atům")),
    (5, ("ech", "ich", "ích", "ého", "ěmi", "emi", "ému", "ěte", "ete", "ěti", "eti", "ího", "iho", "ími", "ímu",
         "imu", "ách", "ata", "aty", "ých", "ama", "ami", "ové", "ovi", "ými")),
    (4, ("em", "es", "ém", "ím", "ům", "at", "ám", "os", "us", "ým", "mi", "ou")),
)


def czech_stem(word: str) -> str:
    w = word
    for min_len, sufs in _CS_CASE:                       # remove case: the longest class whose word is long enough
        if len(w) > min_len and w.endswith(sufs):
            w = w[:-len(next(x for x in sufs if w.endswith(x)))]
            break
    else:
        if len(w) > 3 and w[-1] in "aeiouůyáéíýě":
            w = w[:-1]
    if len(w) > 5 and w.endswith(("ov", "in", "ův")):  # possessives
        w = w[:-2]
    if not w:
        return w
    if w.endswith("čt"):                               # normalise
        return w[:-2] + "ck"
    if w.endswith("št"):
        return w[:-2] + "sk"
    if w[-1] in "cč":
        return w[:-1] + "k"
    if w[-1] in "zž":
        return w[:-1] + "h"
    if len(w) > 1 and w[-2] == "e":
        return w[:-2] + w[-1]
    if len(w) > 2 and w[-2] == "ů":
        return w[:-2] + "o" + w[-1]
    return w



# ------------------------------------------------------------------------------------------- Indonesian
# IndonesianAnalyzer: lower case, stop words, IndonesianStemFilter (Tala's algorithm, derivational stemming on):
# particles (-kah -lah -pun) and possessive pronouns (-ku -mu -nya) first, then first-order prefixes
# (meng- / peng- families, di-, ter-, ke-), suffixes (-kan -an -i, conditioned on the prefixes removed) and
# second-order prefixes (ber-, per-, pe-); every step needs a word of more than two syllables (vowels).
_ID_V = frozenset("aeiou")
_ID_KE, _ID_PENG, _ID_DI, _ID_MENG, _ID_TER, _ID_BER, _ID_PE = 1, 2, 4, 8, 16, 32, 64


def indonesian_stem(word: str) -> str:
    w = word
    syl = sum(c in _ID_V for c in w)
    flags = 0
    if syl > 2 and w.endswith(("kah", "lah", "pun")):
        w, syl = w[:-3], syl - 1
    if syl > 2:
        if w.endswith(("ku", "mu")):
            w, syl = w[:-2], syl - 1
        elif w.endswith("nya"):
            w, syl = w[:-3], syl - 1

    def first_order(w, syl, flags):
        n = len(w)
        vowel_at = lambda i: n > i and w[i] in _ID_V      # noqa: E731
        if w.startswith("meng"):
            return w[4:], syl - 1, flags | _ID_MENG
        if w.startswith("meny") and vowel_at(4):
            return "s" + w[4:], syl - 1, flags | _ID_MENG
        if w.startswith(("men", "mem")):
            return w[3:], syl - 1, flags | _ID_MENG
        if w.startswith("me"):
            return w[2:], syl - 1, flags | _ID_MENG
        if w.startswith("peng"):
            return w[4:], syl - 1, flags | _ID_PENG
        if w.startswith("peny") and vowel_at(4):
            return "s" + w[4:], syl - 1, flags | _ID_PENG
        if w.startswith("peny"):
            return w[4:], syl - 1, flags | _ID_PENG
        if w.startswith("pen") and vowel_at(3):
            return "t" + w[3:], syl - 1, flags | _ID_PENG
        if w.startswith(("pen", "pem")):
            return w[3:], syl - 1, flags | _ID_PENG
        if w.startswith("di"):
            return w[2:], syl - 1, flags | _ID_DI
        if w.startswith("ter"):
            return w[3:], syl - 1, flags | _ID_TER
        if w.startswith("ke"):
            return w[2:], syl - 1, flags | _ID_KE
        return w, syl, flags

    def second_order(w, syl, flags):
        if w.startswith("ber"):
            return w[3:], syl - 1, flags | _ID_BER
        if w == "belajar":
            return w[3:], syl - 1, flags | _ID_BER
        if w.startswith("be") and len(w) > 4 and w[2] not in _ID_V and w[3] == "e" and w[4] == "r":
            return w[2:], syl - 1, flags | _ID_BER
        if w.startswith("per"):
            return w[3:], syl - 1, flags
        if w == "pelajar":
            return w[3:], syl - 1, flags
        if w.startswith("pe"):
            return w[2:], syl - 1, flags | _ID_PE
        return w, syl, flags

    def suffix(w, syl, flags):
        if w.endswith("kan") and not flags & (_ID_KE | _ID_PENG | _ID_PE):
            return w[:-3], syl - 1, flags
        if w.endswith("an") and not flags & (_ID_DI | _ID_MENG | _ID_TER):
            return w[:-2], syl - 1, flags
        if w.endswith("i") and not w.endswith("si") and not flags & (_ID_BER | _ID_KE | _ID_PENG):
            return w[:-1], syl - 1, flags
        return w, syl, flags

    before = w
    if syl > 2:
        w, syl, flags = first_order(w, syl, flags)
    if w != before:                              # a first-order prefix came off
        mid = w
        if syl > 2:
            w, syl, flags = suffix(w, syl, flags)
        if w != mid and syl > 2:
            w, syl, flags = second_order(w, syl, flags)
    else:
        if syl > 2:
            w, syl, flags = second_order(w, syl, flags)
        if syl > 2:
            w, syl, flags = suffix(w, syl, flags)
    return w


# ---------------------------------------------------------------------------------------------- Latvian
# LatvianAnalyzer: lower case, stop words, LatvianStemFilter (Kreslins' light stemmer): the first listed ending
# whose vowel-count condition holds and that leaves at least three letters is removed; endings marked
# palatalising undo the consonant alternation the ending caused (kš -> kst, ņņ -> nn after genitive -u, labial
# + j -> labial, šņ / žņ / šļ / žļ / ļņ / ļļ, č / ļ / ņ -> c / l / n).
_LV_V = frozenset("aeiouāēīōū")
_LV_AFFIXES = (("ajiem", 3, False), ("ajai", 3, False), ("ajam", 2, False), ("ajām", 2, False), ("ajos", 2, False),
               ("ajās", 2, False), ("iem", 2, True), ("ajā", 2, False), ("ais", 2, False), ("ai", 2, False),
               ("ei", 2, False), ("ām", 1, False), ("am", 1, False), ("ēm", 1, False), ("īm", 1, False),
               ("im", 1, False), ("um", 1, False), ("us", 1, True), ("as", 1, False), ("ās", 1, False),
               ("es", 1, False), ("os", 1, True), ("ij", 1, False), ("īs", 1, False), ("ēs", 1, False),
               ("is", 1, False), ("ie", 1, False), ("u", 1, True), ("a", 1, True), ("i", 1, True), ("e", 1, False),
               ("ā", 1, False), ("ē", 1, False), ("ī", 1, False), ("ū", 1, False), ("o", 1, False),
               ("s", 0, False), ("š", 0, False))
_LV_PAIRS = {"šņ": "sn", "žņ": "zn", "šļ": "sl", "žļ": "zl", "ļņ": "ln", "ļļ": "ll"}


def _lv_unpalatalize(w: str, removed: str) -> str:
    if removed.startswith("u"):                  # genitive plural -u: kš -> kst, ņņ -> nn only here
        if w.endswith("kš"):
            return w[:-2] + "kst"
        if w.endswith("ņņ"):
            return w[:-2] + "nn"
    if w.endswith(("pj", "bj", "mj", "vj")):
        return w[:-1]
    if w[-2:] in _LV_PAIRS:
        return w[:-2] + _LV_PAIRS[w[-2:]]
    if w.endswith("č"):
        return w[:-1] + "c"
    if w.endswith("ļ"):
        return w[:-1] + "l"
    if w.endswith("ņ"):
        return w[:-1] + "n"
    return w


def latvian_stem(word: str) -> str:
    nv = sum(c in _LV_V for c in word)
    for aff, vc, pal in _LV_AFFIXES:
        if nv > vc and len(word) >= len(aff) + 3 and word.endswith(aff):
            w = word[:-len(aff)]
            return _lv_unpalatalize(w, aff) if pal else w
    return word

from .snowball import dutch_stem, finnish_stem, hungarian_stem, romanian_stem, russian_stem, turkish_stem  # noqa: E402

STEMMERS: Dict[str, Callable[[str], str]] = {
    "fr": french_light_stem, "de": german_analyze_stem, "es": spanish_light_stem, "it": italian_light_stem,
    "pt": portuguese_light_stem, "no": norwegian_light_stem, "sv": swedish_stem, "da": danish_stem,
    "ru": russian_stem, "nl": dutch_stem, "ro": romanian_stem, "hu": hungarian_stem, "fi": finnish_stem,
    "ar": arabic_analyze_stem, "hi": hindi_analyze_stem, "bg": bulgarian_stem, "cs": czech_stem, "tr": turkish_stem,
    "id": indonesian_stem, "lv": latvian_stem,
}

from .stemmers_more import STEMMERS_MORE  # noqa: E402

STEMMERS.update(STEMMERS_MORE)

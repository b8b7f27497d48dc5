"""Snowball stemmers of the Lucene language analyzers that ``LuceneTextAnalyzer.scala:169-206`` maps (the
RussianAnalyzer and DutchAnalyzer run ``SnowballFilter`` with these algorithms after their stop filters).

Implemented from the published Snowball algorithm descriptions (snowballstem.org), not from any code:

* :func:`russian_stem` -- perfective gerund / reflexive / adjectival / verb / noun endings in RV, final и,
  derivational ост(ь) in R2, superlative, undoubled н and final ь.
* :func:`dutch_stem` -- accent removal, Y / I marking, en / s / e / heid / end / ing / ig / lijk / baar / bar
  endings, undoubling, and the vowel undoubling of step 4; DutchAnalyzer's stem overrides (fiets, bromfiets,
  ei, kind) are applied first, as its StemmerOverrideFilter does.

* :func:`romanian_stem`, :func:`hungarian_stem`, :func:`finnish_stem` -- the RomanianAnalyzer, HungarianAnalyzer
  and FinnishAnalyzer stemmers (steps named in each function). Their outputs are pinned by the algorithms' own
  rules in ``tests/test_language.py``; no reference fixture covers these languages (parity unpinned).
* :func:`turkish_stem` -- TurkishAnalyzer's Snowball Turkish: a backtracking suffix grammar (nominal verb
  suffixes, noun suffix chains through -ki) on a small backward-mode matcher with Snowball's cursor and slice
  semantics, then U restoration and final-consonant devoicing; :func:`turkish_lower` is TurkishLowerCaseFilter.

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


# ---------------------------------------------------------------------------------------------- Romanian
# RomanianAnalyzer: lower case, stop words, SnowballFilter(Romanian). The Snowball Romanian algorithm is written
# with the cedilla letters ş ţ; the comma-below forms (ș ț) are folded onto them first.
_RO_V = set("aăâeiîou")
_RO_COMMA = str.maketrans("șțŞŢȘȚ", "şţşţşţ")


def _ro_mark(w: str) -> str:
    """u and i between vowels -> U, I (consonants for the regions and the suffix conditions)."""
    c = list(w)
    for i in range(1, len(c) - 1):
        if c[i] in "ui" and c[i - 1] in _RO_V and c[i + 1] in _RO_V:
            c[i] = c[i].upper()
    return "".join(c)


def _rv_standard(w: str, vowels) -> int:
    """RV of the Romance Snowball stemmers: after the next vowel when the 2nd letter is a consonant, after the
    next consonant when the first two are vowels, else after the 3rd letter; the end if none applies."""
    n = len(w)
    if n < 2:
        return n
    if w[1] not in vowels:
        for i in range(2, n):
            if w[i] in vowels:
                return i + 1
        return n
    if w[0] in vowels:
        for i in range(2, n):
            if w[i] not in vowels:
                return i + 1
        return n
    return 3 if n >= 3 else n


def _r1r2(w: str, vowels) -> Tuple[int, int]:
    def r_after(start: int) -> int:
        for i in range(start + 1, len(w)):
            if w[i] not in vowels and w[i - 1] in vowels:
                return i + 1
        return len(w)
    r1 = r_after(0)
    return r1, (r_after(r1) if r1 < len(w) else len(w))


_RO_STEP0 = {"ul": "", "ului": "", "aua": "a", "ea": "e", "ele": "e", "elor": "e", "ii": "i", "iua": "i", "iei": "i",
             "iile": "i", "iilor": "i", "ilor": "i", "ile": "i", "atei": "at", "aţie": "aţi", "aţia": "aţi"}
_RO_COMBO = {}
for _rep, _sufs in (("abil", "abilitate abilitati abilităi abilităţi"), ("ibil", "ibilitate"),
                    ("iv", "ivitate ivitati ivităi ivităţi"),
                    ("ic", "icitate icitati icităi icităţi icator icatori iciv iciva icive icivi icivă ical icala icale "
                           "icali icală"),
                    ("at", "ativ ativa ative ativi ativă aţiune atoare ator atori ătoare ător ători"),
                    ("it", "itiv itiva itive itivi itivă iţiune itoare itor itori")):
    for _s in _sufs.split():
        _RO_COMBO[_s] = _rep
_RO_STD_DEL = tuple("at ata ată ati ate ut uta ută uti ute it ita ită iti ite ic ica ice ici ică abil abila abile abili "
                    "abilă ibil ibila ibile ibili ibilă oasa oasă oase os osi oşi ant anta ante anti antă ator atori "
                    "itate itati ităi ităţi iv iva ive ivi ivă".split())
_RO_STD_IST = tuple("ism isme ist ista iste isti istă işti".split())
_RO_VERB1 = tuple("are ere ire âre ind ând indu ându eze ească ez ezi ează esc eşti eşte ăsc ăşti ăşte am ai au eam eai "
                  "ea eaţi eau iam iai ia iaţi iau ui aşi arăm arăţi ară uşi urăm urăţi ură işi irăm irăţi iră âi âşi "
                  "ârăm ârăţi âră asem aseşi ase aserăm aserăţi aseră isem iseşi ise iserăm iserăţi iseră âsem âseşi "
                  "âse âserăm âserăţi âseră usem useşi use userăm userăţi useră".split())
_RO_VERB2 = tuple("ăm aţi em eţi im iţi âm âţi seşi serăm serăţi seră sei se sesem seseşi sese seserăm seserăţi "
                  "seseră".split())


def romanian_stem(word: str) -> str:
    w = _ro_mark(word.translate(_RO_COMMA))
    rv = _rv_standard(w, _RO_V)
    r1, r2 = _r1r2(w, _RO_V)
    # step 0: plurals and other simplifications, in R1
    s = _longest(w, 0, _RO_STEP0)
    if s is not None and len(w) - len(s) >= r1:
        if not (s == "ile" and w[:-3].endswith("ab")):
            w = w[:-len(s)] + _RO_STEP0[s]
    # step 1: combining suffixes in R1, repeated while one is replaced
    removed = False
    while True:
        s = _longest(w, 0, _RO_COMBO)
        if s is None or len(w) - len(s) < r1:
            break
        w = w[:-len(s)] + _RO_COMBO[s]
        removed = True
    # step 2: standard suffixes in R2
    s = _longest(w, 0, _RO_STD_DEL + _RO_STD_IST + ("iune", "iuni"))
    if s is not None and len(w) - len(s) >= r2:
        if s in ("iune", "iuni"):
            if w[:-len(s)].endswith("ţ"):
                w = w[:-len(s) - 1] + "t"
                removed = True
        elif s in _RO_STD_IST:
            w = w[:-len(s)] + "ist"
            removed = True
        else:
            w = w[:-len(s)]
            removed = True
    # step 3: verb suffixes in RV, when steps 1 and 2 removed nothing
    if not removed:
        s = _longest(w, rv, _RO_VERB1 + _RO_VERB2)
        if s is not None:
            k = len(w) - len(s)
            if s in _RO_VERB2:
                w = w[:k]
            elif k - 1 >= rv and (w[k - 1] not in _RO_V or w[k - 1] == "u"):
                w = w[:k]
    # step 4: final vowel in RV
    s = _longest(w, rv, ("a", "e", "i", "ie", "ă"))
    if s is not None:
        w = w[:-len(s)]
    return w.replace("I", "i").replace("U", "u")


# --------------------------------------------------------------------------------------------- Hungarian
# HungarianAnalyzer: lower case, stop words, SnowballFilter(Hungarian).
_HU_V = set("aáeéiíoóöőuúüű")
_HU_DIGRAPHS = ("dzs", "cs", "dz", "gy", "ly", "ny", "sz", "ty", "zs")
_HU_DOUBLES = ("bb", "cc", "ccs", "dd", "ff", "gg", "ggy", "jj", "kk", "ll", "lly", "mm", "nn", "nny", "pp", "rr", "ss",
               "ssz", "tt", "tty", "vv", "zz", "zzs")


def _hu_r1(w: str) -> int:
    """After the first consonant (a digraph counts as one) when the word starts with a vowel; after the first
    vowel when it starts with a consonant; the end when the word lacks either."""
    if not w:
        return 0
    if w[0] in _HU_V:
        for i in range(1, len(w)):
            if w[i] not in _HU_V:
                for dg in _HU_DIGRAPHS:
                    if w.startswith(dg, i):
                        return i + len(dg)
                return i + 1
        return len(w)
    for i in range(1, len(w)):
        if w[i] in _HU_V:
            return i + 1
    return len(w)


def _hu_undouble_after(w: str, suffix_len: int, r1: int) -> str:
    """Delete a suffix that lies in R1 and follows a double consonant, then one letter of that double."""
    k = len(w) - suffix_len
    if k < r1 or not w[:k].endswith(_HU_DOUBLES):
        return w
    w = w[:k]
    return w[:-2] + w[-1]


def _hu_table(w: str, r1: int, table) -> str:
    s = _longest(w, 0, table)
    if s is not None and len(w) - len(s) >= r1:
        return w[:-len(s)] + table[s]
    return w


_HU_CASE = tuple("ban ben ba be ra re nak nek val vel tól től ról ről ból ből hoz hez höz nál nél ig at et ot öt ért képp "
                 "képpen kor ul ül vá vé onként enként anként ként en on an ön n t".split())
_HU_SPECIAL = {"én": "e", "án": "a", "ánként": "a"}
_HU_OTHER = {"astul": "", "estül": "", "stul": "", "stül": "", "ástul": "a", "éstül": "e"}
_HU_OWNED = {"oké": "", "öké": "", "aké": "", "eké": "", "ké": "", "éi": "", "é": "", "áké": "a", "áéi": "a", "éké": "e",
             "ééi": "e", "éé": "e"}
_HU_SING = {s: "" for s in "ünk unk nk juk jük uk ük em om am m od ed ad öd d ja je a e o".split()}
_HU_SING.update({s: "a" for s in "ánk ájuk ám ád á".split()})
_HU_SING.update({s: "e" for s in "énk éjük ém éd é".split()})
_HU_PLUR = {s: "" for s in ("jaim jeim aim eim im jaid jeid aid eid id jai jei ai ei i jaink jeink eink aink ink jaitok "
                            "jeitek aitok eitek itek jeik jaik aik eik ik").split()}
_HU_PLUR.update({s: "a" for s in "áim áid ái áink áitok áik".split()})
_HU_PLUR.update({s: "e" for s in "éim éid éi éink éitek éik".split()})
_HU_PLURAL = {"ák": "a", "ék": "e", "ök": "", "ok": "", "ek": "", "ak": "", "k": ""}


def hungarian_stem(word: str) -> str:
    w = word
    r1 = _hu_r1(w)
    # instrumental: -al / -el after a double consonant
    if w.endswith(("al", "el")):
        w = _hu_undouble_after(w, 2, r1)
    # frequent cases, then a final á / é (in R1) back to a / e
    s = _longest(w, 0, _HU_CASE)
    if s is not None and len(w) - len(s) >= r1:
        w = w[:-len(s)]
        if len(w) - 1 >= r1 and w.endswith(("á", "é")):
            w = w[:-1] + ("a" if w[-1] == "á" else "e")
    w = _hu_table(w, r1, _HU_SPECIAL)
    w = _hu_table(w, r1, _HU_OTHER)
    # factive: -á / -é after a double consonant
    if w.endswith(("á", "é")):
        w = _hu_undouble_after(w, 1, r1)
    w = _hu_table(w, r1, _HU_OWNED)
    w = _hu_table(w, r1, _HU_SING)
    w = _hu_table(w, r1, _HU_PLUR)
    w = _hu_table(w, r1, _HU_PLURAL)
    return w


# ----------------------------------------------------------------------------------------------- Finnish
# FinnishAnalyzer: lower case, stop words, SnowballFilter(Finnish).
_FI_V1 = set("aeiouyäö")
_FI_V2 = set("aeiouäö")
_FI_C = set("bcdfghjklmnpqrstvwxz")
_FI_LV = ("aa", "ee", "ii", "oo", "uu", "ää", "öö")


def _fi_vi(w: str, k: int) -> bool:
    """the text before position k ends with a V2 vowel followed by i"""
    return k >= 2 and w[k - 1] == "i" and w[k - 2] in _FI_V2


def finnish_stem(word: str) -> str:
    w = word
    r1, r2 = _r1r2(w, _FI_V1)
    # step 1: particles (after n, t or a vowel) and -sti (in R2), the suffix in R1
    s = _longest(w, r1, ("kin", "kaan", "kään", "ko", "kö", "han", "hän", "pa", "pä", "sti"))
    if s is not None:
        k = len(w) - len(s)
        if s == "sti":
            if k >= r2:
                w = w[:k]
        elif k >= 1 and (w[k - 1] in _FI_V1 or w[k - 1] in "nt"):
            w = w[:k]
    # step 2: possessives, the suffix in R1
    s = _longest(w, r1, ("si", "ni", "nsa", "nsä", "mme", "nne", "an", "än", "en"))
    if s is not None:
        k = len(w) - len(s)
        head = w[:k]
        if s == "si":
            if not head.endswith("k"):
                w = head
        elif s == "ni":
            w = head[:-3] + "ksi" if head.endswith("kse") else head
        elif s in ("nsa", "nsä", "mme", "nne"):
            w = head
        elif s == "an":
            if head.endswith(("ta", "ssa", "sta", "lla", "lta", "na")):
                w = head
        elif s == "än":
            if head.endswith(("tä", "ssä", "stä", "llä", "ltä", "nä")):
                w = head
        elif s == "en":
            if head.endswith(("lle", "ine")):
                w = head
    # step 3: cases, the suffix in R1
    ending_removed = False
    s = _longest(w, r1, ("han", "hen", "hin", "hon", "hun", "hyn", "hän", "hön", "siin", "den", "tten", "seen", "a",
                         "ä", "tta", "ttä", "ta", "tä", "ssa", "ssä", "sta", "stä", "lla", "llä", "lta", "ltä", "lle",
                         "na", "nä", "ksi", "ine", "n"))
    if s is not None:
        k = len(w) - len(s)
        ok = False
        if len(s) == 3 and s[0] == "h" and s[2] == "n":
            ok = k >= 1 and w[k - 1] == s[1]
        elif s in ("siin", "den", "tten"):
            ok = _fi_vi(w, k)
        elif s == "seen":
            ok = w[:k].endswith(_FI_LV)
        elif s in ("a", "ä"):
            ok = k >= 2 and w[k - 1] in _FI_V1 and w[k - 2] in _FI_C
        elif s in ("tta", "ttä"):
            ok = k >= 1 and w[k - 1] == "e"
        else:
            ok = True
        if ok:
            w = w[:k]
            if s == "n" and w.endswith(_FI_LV + ("ie",)):
                w = w[:-1]
            ending_removed = True
    # step 4: other endings, the suffix in R2
    s = _longest(w, r2, ("mpi", "mpa", "mpä", "mmi", "mma", "mmä", "impi", "impa", "impä", "immi", "imma", "immä",
                         "eja", "ejä"))
    if s is not None:
        if not (len(s) == 3 and s[0] == "m" and w[:-3].endswith("po")):
            w = w[:-len(s)]
    # step 5: plurals
    if ending_removed:
        if w.endswith(("i", "j")) and len(w) - 1 >= r1:
            w = w[:-1]
    elif w.endswith("t") and len(w) - 1 >= r1 and len(w) >= 2 and w[-2] in _FI_V1:
        w = w[:-1]
        s = _longest(w, r2, ("mma", "imma"))
        if s is not None and not (s == "mma" and w[:-3].endswith("po")):
            w = w[:-len(s)]
    # step 6: tidying, the letters concerned in R1
    if w.endswith(_FI_LV) and len(w) - 2 >= r1:
        w = w[:-1]
    if len(w) >= 2 and w[-1] in "aäei" and w[-2] in _FI_C and len(w) - 2 >= r1:
        w = w[:-1]
    if w.endswith(("oj", "uj")) and len(w) - 2 >= r1:
        w = w[:-1]
    if w.endswith("jo") and len(w) - 2 >= r1:
        w = w[:-1]
    # a double consonant followed by zero or more vowels: drop one of the pair (regardless of R1)
    i = len(w)
    while i > 0 and w[i - 1] in _FI_V1:
        i -= 1
    if i >= 2 and w[i - 1] == w[i - 2] and w[i - 1] in _FI_C:
        w = w[:i - 1] + w[i:]
    return w


# ----------------------------------------------------------------------------------------------- Turkish
# TurkishAnalyzer: apostrophe filter, Turkish lower case, stop words, SnowballFilter(Turkish). The Turkish
# algorithm is a backtracking suffix grammar (nominal verb suffixes, then the noun suffix chains through -ki),
# so it runs on a small backward-mode matcher with Snowball's cursor / slice semantics: saved cursors are
# offsets from the end of the word (deletions to their left keep them valid), ``alt`` restores the cursor
# between alternatives, ``opt`` (try) restores it on failure, and deletions are never undone.
_TR_V = frozenset("aeıioöuü")
_TR_U = frozenset("ıiuü")
_TR_HARMONY = (("a", frozenset("aıou")), ("e", frozenset("eiöü")), ("ı", frozenset("aı")), ("i", frozenset("ei")),
               ("o", frozenset("ou")), ("ö", frozenset("öü")), ("u", frozenset("ou")), ("ü", frozenset("öü")))


class _TrMatcher:
    __slots__ = ("w", "c", "bra", "ket", "cont")

    def __init__(self, w: str):
        self.w, self.c, self.bra, self.ket, self.cont = w, len(w), len(w), len(w), True

    def save(self) -> int:
        return len(self.w) - self.c

    def restore(self, v: int) -> None:
        self.c = len(self.w) - v

    def eq(self, s: str) -> bool:
        if self.w.endswith(s, 0, self.c):
            self.c -= len(s)
            return True
        return False

    def among(self, sufs) -> bool:              # longest listed suffix ending at the cursor
        for s in sufs:
            if self.eq(s):
                return True
        return False

    def isin(self, g) -> bool:
        if self.c > 0 and self.w[self.c - 1] in g:
            self.c -= 1
            return True
        return False

    def notin(self, g) -> bool:
        if self.c > 0 and self.w[self.c - 1] not in g:
            self.c -= 1
            return True
        return False

    def goto(self, g) -> bool:                  # stop before the nearest char in g (not consumed)
        while True:
            if self.c > 0 and self.w[self.c - 1] in g:
                return True
            if self.c <= 0:
                return False
            self.c -= 1

    def nxt(self) -> bool:
        if self.c <= 0:
            return False
        self.c -= 1
        return True

    def test(self, f) -> bool:
        v = self.save()
        r = f()
        self.restore(v)
        return r

    def alt(self, *fs) -> bool:
        v = self.save()
        for f in fs:
            if f():
                return True
            self.restore(v)
        return False

    def opt(self, f) -> bool:
        v = self.save()
        if not f():
            self.restore(v)
        return True

    def k(self) -> bool:                        # [  (backward mode: the slice's right end)
        self.ket = self.c
        return True

    def cut(self) -> bool:                      # ] delete
        self.bra = self.c
        b, k = self.bra, self.ket
        self.w = self.w[:b] + self.w[k:]
        if self.c >= k:
            self.c -= k - b
        elif self.c > b:
            self.c = b
        return True

    def insert(self, s: str) -> bool:           # <+ at the cursor
        self.w = self.w[:self.c] + s + self.w[self.c:]
        self.c += len(s)
        return True


def _by_len(*sufs):
    return tuple(sorted(sufs, key=len, reverse=True))


_TR_POSS = _by_len("mız", "miz", "muz", "müz", "nız", "niz", "nuz", "nüz", "m", "n")
_TR_YDU = _by_len(*(a + v + e for a in "td" for e in ("m", "n", "k", "") for v in "ıiuü"))


class _TrStem(_TrMatcher):
    # ---- conditions on the letters around a suffix
    def harmony(self) -> bool:
        def body():
            if not self.goto(_TR_V):
                return False
            return self.alt(*[(lambda ch=ch, g=g: self.eq(ch) and self.goto(g)) for ch, g in _TR_HARMONY])
        return self.test(body)

    def opt_consonant(self, ch: str) -> bool:
        # the suffix's optional consonant ch stands after a vowel; without it, the letter two back is a vowel
        return self.alt(lambda: self.test(lambda: self.eq(ch)) and self.nxt() and self.test(lambda: self.isin(_TR_V)),
                        lambda: not self.test(lambda: self.eq(ch)) and
                        self.test(lambda: self.nxt() and self.test(lambda: self.isin(_TR_V))))

    def opt_u(self) -> bool:
        return self.alt(lambda: self.test(lambda: self.isin(_TR_U)) and self.nxt() and
                        self.test(lambda: self.notin(_TR_V)),
                        lambda: not self.test(lambda: self.isin(_TR_U)) and
                        self.test(lambda: self.nxt() and self.test(lambda: self.notin(_TR_V))))

    # ---- suffix marks
    def possessives(self):
        return self.among(_TR_POSS) and self.opt_u()

    def sU(self):
        return self.harmony() and self.isin(_TR_U) and self.opt_consonant("s")

    def lArI(self):
        return self.among(("leri", "ları"))

    def yU(self):
        return self.harmony() and self.isin(_TR_U) and self.opt_consonant("y")

    def nU(self):
        return self.harmony() and self.among(("ı", "i", "u", "ü"))

    def nUn(self):
        return self.harmony() and self.among(("ın", "in", "un", "ün")) and self.opt_consonant("n")

    def yA(self):
        return self.harmony() and self.among(("a", "e")) and self.opt_consonant("y")

    def nA(self):
        return self.harmony() and self.among(("na", "ne"))

    def DA(self):
        return self.harmony() and self.among(("da", "de", "ta", "te"))

    def ndA(self):
        return self.harmony() and self.among(("nda", "nde"))

    def DAn(self):
        return self.harmony() and self.among(("dan", "den", "tan", "ten"))

    def ndAn(self):
        return self.harmony() and self.among(("ndan", "nden"))

    def ylA(self):
        return self.harmony() and self.among(("la", "le")) and self.opt_consonant("y")

    def ki(self):
        return self.eq("ki")

    def ncA(self):
        return self.harmony() and self.among(("ca", "ce")) and self.opt_consonant("n")

    def yUm(self):
        return self.harmony() and self.among(("ım", "im", "um", "üm")) and self.opt_consonant("y")

    def sUn(self):
        return self.harmony() and self.among(("sın", "sin", "sun", "sün"))

    def yUz(self):
        return self.harmony() and self.among(("ız", "iz", "uz", "üz")) and self.opt_consonant("y")

    def sUnUz(self):
        return self.among(("sınız", "siniz", "sunuz", "sünüz"))

    def lAr(self):
        return self.harmony() and self.among(("ler", "lar"))

    def nUz(self):
        return self.harmony() and self.among(("ız", "iz", "uz", "üz"))

    def DUr(self):
        return self.harmony() and self.among(("tır", "tir", "tur", "tür", "dır", "dir", "dur", "dür"))

    def cAsInA(self):
        return self.among(("casına", "cesine"))

    def yDU(self):
        return self.harmony() and self.among(_TR_YDU) and self.opt_consonant("y")

    def ysA(self):                              # does not follow vowel harmony
        return self.among(("sam", "san", "sak", "sem", "sen", "sek", "sa", "se")) and self.opt_consonant("y")

    def ymUs(self):
        return self.harmony() and self.among(("mış", "miş", "muş", "müş")) and self.opt_consonant("y")

    def yken(self):
        return self.eq("ken") and self.opt_consonant("y")

    # ---- suffix chains
    def nominal_verb(self) -> bool:
        self.k()
        self.cont = True
        person = lambda: self.alt(self.sUnUz, self.lAr, self.yUm, self.sUn, self.yUz, lambda: True)  # noqa: E731

        def after_lar():
            self.opt(lambda: self.k() and self.alt(self.DUr, self.yDU, self.ysA, self.ymUs))
            self.cont = False
            return True
        ok = self.alt(
            lambda: self.alt(self.ymUs, self.yDU, self.ysA, self.yken),
            lambda: self.cAsInA() and person() and self.ymUs(),
            lambda: self.lAr() and self.cut() and after_lar(),
            lambda: self.nUz() and self.alt(self.yDU, self.ysA),
            lambda: self.alt(self.sUnUz, self.yUz, self.sUn, self.yUm) and self.cut() and
            self.opt(lambda: self.k() and self.ymUs()),
            lambda: self.DUr() and self.cut() and self.opt(lambda: self.k() and person() and self.ymUs()))
        return ok and self.cut()

    def lar_ki(self) -> bool:                   # [lAr] delete chain_before_ki
        return self.k() and self.lAr() and self.cut() and self.chain_ki()

    def poss_or_su(self) -> bool:               # [possessives or sU] delete try([lAr] delete chain_before_ki)
        return self.k() and self.alt(self.possessives, self.sU) and self.cut() and self.opt(self.lar_ki)

    def chain_ki(self) -> bool:
        if not (self.k() and self.ki()):
            return False
        return self.alt(
            lambda: self.DA() and self.cut() and self.opt(lambda: self.k() and self.alt(
                lambda: self.lAr() and self.cut() and self.opt(self.chain_ki),
                lambda: self.possessives() and self.cut() and self.opt(self.lar_ki))),
            lambda: self.nUn() and self.cut() and self.opt(lambda: self.k() and self.alt(
                lambda: self.lArI() and self.cut(),
                self.poss_or_su,
                self.chain_ki)),
            lambda: self.ndA() and self.alt(
                lambda: self.lArI() and self.cut(),
                lambda: self.sU() and self.cut() and self.opt(self.lar_ki),
                self.chain_ki))

    def noun(self) -> bool:
        return self.alt(
            lambda: self.k() and self.lAr() and self.cut() and self.opt(self.chain_ki),
            lambda: self.k() and self.ncA() and self.cut() and self.opt(lambda: self.alt(
                lambda: self.k() and self.lArI() and self.cut(),
                self.poss_or_su,
                self.lar_ki)),
            lambda: self.k() and self.alt(self.ndA, self.nA) and self.alt(
                lambda: self.lArI() and self.cut(),
                lambda: self.sU() and self.cut() and self.opt(self.lar_ki),
                self.chain_ki),
            lambda: self.k() and self.alt(self.ndAn, self.nU) and self.alt(
                lambda: self.sU() and self.cut() and self.opt(self.lar_ki),
                self.lArI),
            lambda: self.k() and self.DAn() and self.cut() and self.opt(lambda: self.k() and self.alt(
                lambda: self.possessives() and self.cut() and self.opt(self.lar_ki),
                lambda: self.lAr() and self.cut() and self.opt(self.chain_ki),
                self.chain_ki)),
            lambda: self.k() and self.alt(self.nUn, self.ylA) and self.cut() and self.opt(lambda: self.alt(
                self.lar_ki,
                self.poss_or_su,
                self.chain_ki)),
            lambda: self.k() and self.lArI() and self.cut(),
            self.chain_ki,
            lambda: self.k() and self.alt(self.DA, self.yU, self.yA) and self.cut() and self.opt(
                lambda: self.k() and self.alt(
                    lambda: self.possessives() and self.cut() and self.opt(lambda: self.k() and self.lAr()),
                    self.lAr) and self.cut() and self.k() and self.chain_ki()),
            self.poss_or_su)

    # ---- postlude
    def append_u(self) -> bool:                 # a stem ending in d / g takes the U of its last vowel
        if not self.test(lambda: self.alt(lambda: self.eq("d"), lambda: self.eq("g"))):
            return False
        for vowels, u in (("aı", "ı"), ("ei", "i"), ("ou", "u"), ("öü", "ü")):
            if self.test(lambda: self.goto(_TR_V) and self.w[self.c - 1] in vowels):
                return self.insert(u)
        return False

    def last_consonant(self) -> None:
        repl = {"b": "p", "c": "ç", "d": "t", "ğ": "k"}.get(self.w[-1:])
        if repl is not None:
            self.w = self.w[:-1] + repl


def turkish_stem(word: str) -> str:
    """Snowball Turkish (Çilden's suffix-stripping algorithm): words of one syllable are left alone; the
    nominal verb suffixes are stripped, then (unless a plural -lAr ended that step) the noun suffix chains,
    then a d / g stem takes back its U vowel and a final b / c / d / ğ turns into p / ç / t / k (not for the
    reserved words ad, soyad)."""
    if sum(ch in _TR_V for ch in word) < 2:
        return word
    t = _TrStem(word)
    v = t.save()
    t.nominal_verb()
    t.restore(v)
    if not t.cont:
        return t.w
    v = t.save()
    t.noun()
    t.restore(v)
    if t.w in ("ad", "soyad"):
        return t.w
    t.c = len(t.w)
    t.append_u()
    t.c = len(t.w)
    t.last_consonant()
    return t.w


def turkish_lower(text: str) -> str:
    """TurkishLowerCaseFilter: dotless I -> ı, dotted İ (or I + combining dot above) -> i, then lower case."""
    return text.replace("İ", "i").replace("İ", "i").replace("I", "ı").lower()

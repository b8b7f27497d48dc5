"""Porter stemmer (the tartarus.org reference implementation that Lucene's ``PorterStemFilter`` ports), used by
the English language analyzer (``EnglishAnalyzer`` = standard tokens, possessive ``'s`` removal, stop words,
Porter stemming; ``LuceneTextAnalyzer.scala:170-200``).

Words of at most two letters are returned unchanged; everything else goes through steps 1ab, 1c, 2, 3,
4 and 5 of M. F. Porter, "An algorithm for suffix stripping" (1980), including the two departures of the
reference C/Java code (``bli -> ble``, ``logi -> log``).
"""
from __future__ import annotations

from functools import lru_cache

_VOWELS = frozenset("aeiou")


class _Stem:
    __slots__ = ("b", "k", "j")

    def __init__(self, w: str):
        self.b = list(w)
        self.k = len(w) - 1
        self.j = 0

    def cons(self, i: int) -> bool:
        c = self.b[i]
        if c in _VOWELS:
            return False
        if c == "y":
            return True if i == 0 else not self.cons(i - 1)
        return True

    def m(self) -> int:
        """Number of VC sequences in b[0..j]."""
        n, i, j = 0, 0, self.j
        while True:
            if i > j:
                return n
            if not self.cons(i):
                break
            i += 1
        i += 1
        while True:
            while True:
                if i > j:
                    return n
                if self.cons(i):
                    break
                i += 1
            i += 1
            n += 1
            while True:
                if i > j:
                    return n
                if not self.cons(i):
                    break
                i += 1
            i += 1

    def vowelinstem(self) -> bool:
        return any(not self.cons(i) for i in range(self.j + 1))

    def doublec(self, j: int) -> bool:
        return j >= 1 and self.b[j] == self.b[j - 1] and self.cons(j)

    def cvc(self, i: int) -> bool:
        if i < 2 or not self.cons(i) or self.cons(i - 1) or not self.cons(i - 2):
            return False
        return self.b[i] not in "wxy"

    def ends(self, s: str) -> bool:
        L = len(s)
        if L > self.k + 1 or "".join(self.b[self.k - L + 1:self.k + 1]) != s:
            return False
        self.j = self.k - L
        return True

    def setto(self, s: str) -> None:
        L = len(s)
        self.b[self.j + 1:self.k + 1] = list(s)
        self.k = self.j + L

    def r(self, s: str) -> None:
        if self.m() > 0:
            self.setto(s)

    def step1ab(self):
        if self.b[self.k] == "s":
            if self.ends("sses"):
                self.k -= 2
            elif self.ends("ies"):
                self.setto("i")
            elif self.k >= 1 and self.b[self.k - 1] != "s":
                self.k -= 1
        if self.ends("eed"):
            if self.m() > 0:
                self.k -= 1
        elif (self.ends("ed") or self.ends("ing")) and self.vowelinstem():
            self.k = self.j
            if self.ends("at"):
                self.setto("ate")
            elif self.ends("bl"):
                self.setto("ble")
            elif self.ends("iz"):
                self.setto("ize")
            elif self.doublec(self.k):
                self.k -= 1
                if self.b[self.k] in "lsz":
                    self.k += 1
            else:
                self.j = self.k
                if self.m() == 1 and self.cvc(self.k):
                    self.setto("e")

    def step1c(self):
        if self.ends("y") and self.vowelinstem():
            self.b[self.k] = "i"

    _S2 = {"a": (("ational", "ate"), ("tional", "tion")), "c": (("enci", "ence"), ("anci", "ance")),
           "e": (("izer", "ize"),), "l": (("bli", "ble"), ("alli", "al"), ("entli", "ent"), ("eli", "e"),
                                         ("ousli", "ous")),
           "o": (("ization", "ize"), ("ation", "ate"), ("ator", "ate")),
           "s": (("alism", "al"), ("iveness", "ive"), ("fulness", "ful"), ("ousness", "ous")),
           "t": (("aliti", "al"), ("iviti", "ive"), ("biliti", "ble")), "g": (("logi", "log"),)}
    _S3 = {"e": (("icate", "ic"), ("ative", ""), ("alize", "al")), "i": (("iciti", "ic"),),
           "l": (("ical", "ic"), ("ful", "")), "s": (("ness", ""),)}
    _S4 = {"a": ("al",), "c": ("ance", "ence"), "e": ("er",), "i": ("ic",), "l": ("able", "ible"),
           "n": ("ant", "ement", "ment", "ent"), "o": ("ion", "ou"), "s": ("ism",), "t": ("ate", "iti"),
           "u": ("ous",), "v": ("ive",), "z": ("ize",)}

    def step2(self):
        if self.k < 1:
            return
        for suf, rep in self._S2.get(self.b[self.k - 1], ()):
            if self.ends(suf):
                self.r(rep)
                return

    def step3(self):
        for suf, rep in self._S3.get(self.b[self.k], ()):
            if self.ends(suf):
                self.r(rep)
                return

    def step4(self):
        if self.k < 1:
            return
        for suf in self._S4.get(self.b[self.k - 1], ()):
            if self.ends(suf):
                if suf == "ion" and not (self.j >= 0 and self.b[self.j] in "st"):
                    return
                break
        else:
            return
        if self.m() > 1:
            self.k = self.j

    def step5(self):
        self.j = self.k
        if self.b[self.k] == "e":
            a = self.m()
            if a > 1 or (a == 1 and not self.cvc(self.k - 1)):
                self.k -= 1
        if self.b[self.k] == "l" and self.doublec(self.k) and self.m() > 1:
            self.k -= 1

    def run(self) -> str:
        if self.k <= 1:
            return "".join(self.b)
        self.step1ab()
        if self.k > 0:
            self.step1c()
            self.step2()
            self.step3()
            self.step4()
            self.step5()
        return "".join(self.b[:self.k + 1])


@lru_cache(maxsize=1 << 16)
def porter_stem(word: str) -> str:
    """Porter stem of a lowercase word (non-alphabetic words pass through unchanged, as Lucene's filter
    stems only what its tokenizer produced; digits and mixed tokens are left alone here)."""
    if len(word) <= 2 or not word.isalpha() or not word.isascii():
        return word
    return _Stem(word).run()


def english_possessive(token: str) -> str:
    """Lucene ``EnglishPossessiveFilter``: strip a trailing ``'s`` / ``’s``."""
    if len(token) > 2 and token[-1] in "sS" and token[-2] in "'’＇":
        return token[:-2]
    return token

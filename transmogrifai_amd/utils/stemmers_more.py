"""The remaining per-language analysis chains of the reference's ``LuceneTextAnalyzer`` (``LuceneTextAnalyzer.scala:
169-206``): Greek, Lithuanian, Galician, Basque, Irish, Bengali, Sorani (Central Kurdish), Catalan (Snowball),
Brazilian Portuguese (BrazilianStemmer) and Thai.

Each function follows the published algorithm its Lucene analyzer runs -- the Snowball stemmers (Catalan,
Basque, Irish, Lithuanian: R1 / R2 / RV regions, longest-suffix-first steps), Lucene's light stemmers (Greek after
Ntais' thesis, Galician after the RSLP step structure, BrazilianStemmer after the Portuguese Snowball steps, Bengali
after Mahmud et al.'s lightweight stemmer, Sorani after the Central Kurdish suffix rules) -- with the language's
normalisation filter (Greek lower case and accent folding, Irish initial mutations, Bengali / Sorani character
normalisation). Suffix lists are condensed to the productive endings of each language; the Lucene jars are not
available here, so token-level parity is unpinned (tests/test_language_more.py pins each algorithm's own rules).
Thai has no dictionary offline: Thai-script runs stay whole tokens (Lucene's ThaiTokenizer breaks them with the
ICU dictionary), then the Thai stop filter applies.
"""
from __future__ import annotations

from typing import Dict, FrozenSet, Sequence


def _longest(suffixes: Sequence[str]):
    return sorted(set(suffixes), key=len, reverse=True)


def _r1(word: str, vowels: str, start: int = 0) -> int:
    """Snowball region start: after the first non-vowel that follows a vowel, at or after ``start``."""
    for i in range(max(1, start + 1), len(word)):
        if word[i] not in vowels and word[i - 1] in vowels:
            return i + 1
    return len(word)


def _strip(w: str, suffixes, region: int, min_stem: int = 0):
    """Remove the longest suffix lying in [region, len) leaving at least ``min_stem`` characters."""
    for s in suffixes:
        if w.endswith(s) and len(w) - len(s) >= max(region, min_stem):
            return w[:-len(s)], s
    return w, None


# ------------------------------------------------------------------------------------------------ Greek
_EL_FOLD = {"ά": "α", "έ": "ε", "ή": "η", "ί": "ι", "ΐ": "ι", "ϊ": "ι", "ό": "ο", "ύ": "υ", "ΰ": "υ", "ϋ": "υ",
            "ώ": "ω", "ς": "σ"}

GREEK_STOPWORDS = frozenset("""ο η το οι τα του τησ των τον την και κι κ ειμαι εισαι ειναι ειμαστε ειστε στο στον στη στην
μα αλλα απο για προσ με σε ωσ παρα αντι κατα μετα θα να δε δεν μη μην επι ενω εαν αν τοτε που πωσ ποιοσ ποια ποιο
ποιοι ποιεσ ποιων ποιουσ αυτοσ αυτη αυτο αυτοι αυτων αυτουσ αυτεσ αυτα εκεινοσ εκεινη εκεινο εκεινοι εκεινεσ εκεινα
εκεινων εκεινουσ οπωσ ομωσ ισωσ οσο οτι""".split())


def greek_lower(word: str) -> str:
    """GreekLowerCaseFilter: lower case, tonos / dialytika removed, final sigma as sigma."""
    return "".join(_EL_FOLD.get(c, c) for c in word.lower())


_EL_ENDINGS = _longest("""ιουσ ιοσ ιου ιων ιεσ ιασ ια ιο ι ουσ ου ων οσ ον ο εσ ασ α ησ η ειτε ετε ουμε ουνε ουν ει
εισ ω ομαι εσαι εται ομαστε εστε ονται οντασ ωντασ οτασ οτητα οτητεσ οτητων ισμοσ ισμου ισμοι ισμων ισμουσ ιστησ
ιστεσ ιστων ικοσ ικη ικο ικοι ικεσ ικα ικων ικου ικουσ αδεσ αδων ηδεσ ηδων ουδεσ ουδων ματα ματων ματοσ μα ασαν
ησαν ουσαν αγαν ηκα ηκεσ ηκε ηκαμε ηκατε ηκαν ησα ησεσ ησε ησαμε ησατε ησω ησει ησουμε ησετε ησουν""".split())


def greek_stem(word: str) -> str:
    """GreekStemmer (Ntais): words shorter than 4 letters are kept; the longest inflectional / derivational
    ending is removed, keeping a stem of at least 2 letters (3 when the ending is a single vowel)."""
    if len(word) < 4:
        return word
    for s in _EL_ENDINGS:
        if word.endswith(s):
            keep = 3 if len(s) == 1 else 2
            if len(word) - len(s) >= keep:
                return word[:-len(s)]
    return word


# ------------------------------------------------------------------------------------------- Lithuanian
_LT_V = "aeiyouąęįųėū"
LITHUANIAN_STOPWORDS = frozenset("""ir ar bet kad kai kas kuris kuri kurie kurios jis ji jie jos tai tas ta tie tos
šis ši šie šios su be į iš nuo per prie po apie už dėl ant tarp pas iki tik dar jau net nes o taip pat ne nei arba
yra buvo bus būti aš tu mes jūs savo""".split())
_LT_STEP1 = _longest("""iesiems iosiems iomis iams iame iuose iose ioms iais ieji iajai iojo iųjų iąja iąjį
aisiais uosiuose osiose oms omis ose uose ams ame ais ai iai ių ių ius ių į ią ie iui iu io ius ių ėms ėmis ėse ėje
ės ę ė ėje ys is as os us ų ą į a e i o u y šiu siu sime site sim sit tume tumėme tumėte tų čiau čiai čiais čių
ėti ėjo ėjau ėjai ėjome ėjote ėsi ėsiu ėsime ėsite ėsis ėtų ti tis tės damas dama darni dami ant ančios ančių
ančiai ant ančią ing ingas ingi ingo ingą""".split())


def lithuanian_stem(word: str) -> str:
    """Snowball Lithuanian (condensed): step 1 removes the longest nominal / verbal ending inside R1 (R1 begins
    after the first consonant following a vowel; a word-initial "a" + consonant counts from the next letter);
    then ``fix_chdz`` (final č -> t, dž -> d) and ``fix_gd`` (final gd -> g)."""
    if len(word) <= 3:
        return word
    start = 1 if len(word) > 6 and word[0] == "a" and word[1] not in _LT_V else 0
    r1 = _r1(word, _LT_V, start)
    w, _ = _strip(word, _LT_STEP1, r1, 2)
    if w.endswith("č"):
        w = w[:-1] + "t"
    elif w.endswith("dž"):
        w = w[:-2] + "d"
    if w.endswith("gd"):
        w = w[:-1]
    return w


# --------------------------------------------------------------------------------------------- Galician
GALICIAN_STOPWORDS = frozenset("""a á ao aos as ás co coa coas cos con da das de do dos e é en entre na nas no nos o
os ou para pero polo pola polos polas por que se sen seu súa seus súas só tamén un unha uns unhas xa este esta
estes estas ese esa eses esas aquel aquela""".split())
_GL_PLURAL = (("ns", "n"), ("ões", "ón"), ("óns", "ón"), ("ais", "al"), ("eis", "el"), ("ois", "ol"), ("is", "il"),
              ("les", "l"), ("res", "r"), ("s", ""))
_GL_FEM = (("eira", "eiro"), ("ona", "ón"), ("ora", "or"), ("ana", "án"), ("esa", "és"), ("ina", "ino"),
           ("osa", "oso"), ("ía", "ío"), ("iva", "ivo"), ("ada", "ado"), ("ida", "ido"), ("ica", "ico"))
_GL_AUG = _longest("iñas iños iña iño ciña ciño ziña ziño ita ito azo aza ón ona".split())
_GL_NOUN = _longest("""amento amentos imento imentos ación acións ición icións ismo ismos ista istas idade idades
ble bles ivo iva ivos ivas eiro eira ador adora adores doras ante antes ente entes ncia ncias""".split())
_GL_VERB = _longest("""ar er ir ando endo indo ado ido ada ida ados idos adas idas aba abas abamos aban ía ías íamos
ían ou eu iu aron eron iron arei arás ará aremos arán aría arían ase asen ese esen ise isen amos emos imos ades edes
ides an en in""".split())


def galician_stem(word: str) -> str:
    """GalicianStemmer (RSLP step structure): plural reduction, feminine -> masculine, adverb ``-mente``,
    augmentative / diminutive, noun suffix, else verb suffix, else final vowel; a removal keeps >= 3 letters."""
    if len(word) < 4:
        return word
    w = word
    for suf, rep in _GL_PLURAL:
        if w.endswith(suf) and len(w) - len(suf) >= 3:
            w = w[:-len(suf)] + rep
            break
    for suf, rep in _GL_FEM:
        if w.endswith(suf) and len(w) - len(suf) >= 2:
            w = w[:-len(suf)] + rep
            break
    if w.endswith("mente") and len(w) - 5 >= 3:
        w = w[:-5]
    if not (w.endswith("ción") or w.endswith("sión")):      # (the -ón of -ción / -sión is not augmentative)
        w, _ = _strip(w, _GL_AUG, 0, 3)
    w2, hit = _strip(w, _GL_NOUN, 0, 3)
    if hit is None:
        w2, hit = _strip(w, _GL_VERB, 0, 3)
    if hit is None and len(w) > 3 and w[-1] in "aeo":
        w2 = w[:-1]
    return w2.replace("á", "a").replace("é", "e").replace("í", "i").replace("ó", "o").replace("ú", "u")


# ------------------------------------------------------------------------------------------------ Basque
_EU_V = "aeiou"
BASQUE_STOPWORDS = frozenset("""al anitz arabera asko baina bat batean batek bati batzuei batzuek batzuetan batzuk
bera beraiek berau berauek bere berori beroriek beste bezala da dago dira ditu du dute edo egin ere eta eurak ez
gainera gu gutxi guzti haiei haiek haietan hainbeste hala han handik hango hara hari hark hartan hau hauei hauek
hauetan hemen hemendik hemengo hi hona honek honela honetan honi hor hori horiei horiek horietan horko horra horrek
horrela horretan horri hortik hura izan ni noiz nola non nondik nongo nor nora ze zein zen zenbait zenbat zer zergatik
ziren zituen zu zuek zuen zuten""".split())
_EU_NOUN = _longest("""arekin ekin arentzat entzat arengandik engandik arengana engana aren ren etako tako ko go ak
ek ari ei an ean etan tan ra era etara tik etik rik ik a ez z az arekiko ekiko ago ena enak enik ago ik izan tzea
tzeko tzen tuz tasun tasuna tasunak garri garria garriak kor kide kideak ari ariak dun duna dunak tsu tsua tsuak
ezin ezina kada""".split())
_EU_VERB = _longest("""tzen tzeko tzea tzera tuz tu du tuta tuko ko go ten tzaile tzaileak ketan kotan""".split())


def _rv_basque(w: str) -> int:
    """Snowball RV: after the next vowel when the second letter is a consonant, else after the next consonant."""
    if len(w) < 2:
        return len(w)
    if w[1] not in _EU_V:
        for i in range(2, len(w)):
            if w[i] in _EU_V:
                return i + 1
        return len(w)
    if w[0] in _EU_V and w[1] in _EU_V:
        for i in range(2, len(w)):
            if w[i] not in _EU_V:
                return i + 1
        return len(w)
    return 3


def basque_stem(word: str) -> str:
    """Snowball Basque (condensed): verb endings (aditzak) in RV, then case / derivational endings (izenak) in
    RV, each leaving at least 3 letters."""
    if len(word) < 4:
        return word
    rv = _rv_basque(word)
    w, hit = _strip(word, _EU_VERB, rv, 3)
    w, hit2 = _strip(w, _EU_NOUN, min(rv, len(w)), 3)
    return w


# ------------------------------------------------------------------------------------------------- Irish
_GA_V = "aeiouáéíóú"
IRISH_STOPWORDS = frozenset("""a ach ag agus an aon ar arna as b' ba beirt bhúr caoga ceathair ceathrar chomh
chtó chuig chun cois céad cúig cúigear d' daichead dar de deich deichniúr den dhá do don dtí dá dár dó faoi faoin
faoina faoinár fara fiche gach gan go gur haon hocht i iad idir in ina ins inár is le leis lena lenár m' mar mo mé
na nach naoi naonúr ná ní níor nó nócha ocht ochtar os roimh sa seacht seachtar seachtó seasca seisear siad sibh
sinn sna sé sí tar thar thú triúr trí trína trínár tríocha tú um ár é éis í ó ón óna ónár""".split())
_GA_MUTATION = (("bhf", "f"), ("bp", "p"), ("dt", "t"), ("gc", "c"), ("mb", "b"), ("nd", "d"), ("ng", "g"),
                ("ts", "s"), ("bh", "b"), ("ch", "c"), ("dh", "d"), ("fh", "f"), ("gh", "g"), ("mh", "m"),
                ("ph", "p"), ("sh", "s"), ("th", "t"), ("h-", ""), ("n-", ""), ("t-", ""))
_GA_NOUN = _longest("amh eamh abh eabh aibh ibh aimh imh aí í ach each a e".split())
_GA_DERIV = _longest("""íochta íocht achta eachta acht eacht aíochta aíocht ála álacha ann anna aire óir óra óireacht
óireachta eoir eora eoireacht eoireachta iúil iúla iúlacht ach each""".split())
_GA_VERB = _longest("imid aimid ímid aímid adh eadh faidh fidh áil ain tear tar".split())


def irish_lower(word: str) -> str:
    """IrishLowerCaseFilter: ``nA`` / ``tA`` (an initial n / t before an upper-case vowel) -> ``n-a`` / ``t-a``,
    then lower case."""
    if len(word) > 1 and word[0] in "nt" and word[1] in "AEIOUÁÉÍÓÚ":
        return word[0] + "-" + word[1:].lower()
    return word.lower()


def irish_stem(word: str) -> str:
    """Snowball Irish: initial mutations undone (eclipsis, lenition, h- / n- / t- prefixes), then the longest
    noun ending in RV, derivational ending in R2 (with -ach/-each in R1), verb ending in RV."""
    w = word
    for pre, rep in _GA_MUTATION:
        if w.startswith(pre) and len(w) > len(pre) + 1:
            w = rep + w[len(pre):]
            break
    rv = next((i + 1 for i, c in enumerate(w) if c in _GA_V), len(w))
    r1 = _r1(w, _GA_V)
    r2 = _r1(w, _GA_V, r1)
    w2, hit = _strip(w, _GA_DERIV, r2, 2)
    if hit is None:
        w2, hit = _strip(w, _GA_VERB, rv, 2)
    if hit is None:
        w2, hit = _strip(w, _GA_NOUN, r1, 2)
    return w2


# ----------------------------------------------------------------------------------------------- Catalan
_CA_V = "aeiouáéíóúàèìòùïü"
_CA_ACC = str.maketrans("áéíóúàèìòùïü", "aeiouaeiouiu")
_CA_PRON = _longest("""'l 'ls 'm 'n 'ns 's 't hi ho la les li lo los me nos se te vos 'hi 'ho 'la 'les 'li 'lo
'los 'me 'nos 'se 'te""".split())
_CA_STD = _longest("""ament aments ació acions ador adora adors adores ança ances ància àncies ble bles dor dora
dors dores ència ències ent ents ista istes isme ismes itat itats iva ives iu ius ment ments ós osa osos oses
ívol ívola ívols ívoles logia logies ica iques ic ics aire aires""".split())
_CA_VERB = _longest("""ar er ir re ava aves àvem àveu aven ant ent int at ada ats ades it ida its ides ut uda uts
udes aré aràs arà arem areu aran aria aries aríem aríeu arien eix eixes eixen eixo eixi ix ixen iré iràs irà irem
ireu iran iria iries iríem iríeu irien em eu en o es as is en""".split())
_CA_RESID = _longest("a e i o os es as is ó í à é".split())


def catalan_stem(word: str) -> str:
    """Snowball Catalan (condensed): attached pronouns in R1, then a standard suffix in R1 (R2 for the shortest
    ones) or else a verb ending in R1, then a residual vowel ending in R1; accents folded at the end."""
    w = word
    r1 = _r1(w, _CA_V)
    r2 = _r1(w, _CA_V, r1)
    w, _ = _strip(w, _CA_PRON, r1)
    w2, hit = _strip(w, _CA_STD, r1, 3)
    if hit is not None and len(hit) <= 2 and len(w) - len(hit) < r2:
        w2, hit = w, None
    if hit is None:
        w2, hit = _strip(w, _CA_VERB, r1, 3)
    w, _ = _strip(w2, _CA_RESID, r1, 3)
    return w.translate(_CA_ACC)


# ------------------------------------------------------------------------------------ Brazilian Portuguese
_BR_ACC = str.maketrans("áãâàçéêíóõôúü", "aaaaceeiooouu")
_BR_V = "aeiou"
_BR_STEP1 = _longest("""uciones amentos imentos amento imento adoras adores aço~es logías ências ância âncias
logia ência mente idades idade ivas ivos iva ivo ezas eza icos icas ico ica ismos ismo istas ista osos osas oso
osa ações ação ável ível antes ante""".replace("~", "").split())
_BR_STEP2 = _longest("""aríamos eríamos iríamos ássemos êssemos íssemos aremos eremos iremos áramos éramos íramos
ávamos ariam eriam iriam assem essem issem arias erias irias ardes erdes irdes asses esses isses astes estes istes
áreis éreis íreis ásseis ésseis ísseis aríeis eríeis iríeis ando endo indo ondo aram eram iram arão erão irão avam
ará erá irá ava ado ido ada ida ados idos adas idas ar er ir as es is am em ei eu iu ou""".split())


def _rv_br(w: str) -> int:
    if len(w) < 3:
        return len(w)
    if w[1] not in _BR_V:
        for i in range(2, len(w)):
            if w[i] in _BR_V:
                return i + 1
        return len(w)
    if w[0] in _BR_V and w[1] in _BR_V:
        for i in range(2, len(w)):
            if w[i] not in _BR_V:
                return i + 1
        return len(w)
    return 3


BRAZILIAN_STOPWORDS = frozenset("""a ainda alem ambas ambos antes ao aonde aos apos aquele aqueles as assim com como
contra contudo cuja cujas cujo cujos da das de dela dele deles demais depois desde desta deste dispoe dispoem diversa
diversas diversos do dos durante e ela elas ele eles em entao entre essa essas esse esses esta estas este estes ha isso
isto logo mais mas mediante menos mesma mesmas mesmo mesmos na nas nao nem nesse neste nos o os ou outra outras outro
outros pelas pelo pelos perante pois por porque portanto proprio propios quais qual qualquer quando quanto que quem
quer se seja sem sendo seu seus sob sobre sua suas tal tambem teu teus toda todas todo todos tua tuas tudo um uma
umas uns""".split())


def brazilian_stem(word: str) -> str:
    """BrazilianStemmer: accents folded; words under 3 letters kept; step 1 standard suffixes (R2-like: the stem
    keeps >= 3 letters), else step 2 verb endings in RV; step 3 drops a final ``i`` after ``c`` in RV; step 4 the
    residual ``os a i o`` in RV; step 5 ``e`` in RV (``gue`` / ``cie`` keep their consonant)."""
    w = word.lower().translate(_BR_ACC)
    if len(w) < 3:
        return w
    rv = _rv_br(w)
    w2, hit = _strip(w, [s.translate(_BR_ACC) for s in _BR_STEP1], 0, 3)
    if hit is None:
        w2, hit = _strip(w, [s.translate(_BR_ACC) for s in _BR_STEP2], rv, 2)
    w = w2
    if w.endswith("ci") and len(w) - 1 >= rv:
        w = w[:-1]
    w, hit4 = _strip(w, ("os", "a", "i", "o"), rv, 2)
    if hit4 is None and w.endswith("e") and len(w) - 1 >= rv:
        w = w[:-1]
        if w.endswith("gu") or w.endswith("ci"):
            w = w[:-1]
    return w


# ----------------------------------------------------------------------------------------------- Bengali
_BN_NORM = {"\u09bc": "",                    # nukta
            "\u0981": "\u0982",              # candrabindu -> anusvara
            "\u09ce": "\u09a4",              # khanda ta -> ta
            "\u09df": "\u09af",              # yya -> ya
            "\u09dc": "\u09b0", "\u09dd": "\u09b0",   # rra / rha -> ra
            "\u0988": "\u0987",              # long i -> i
            "\u098a": "\u0989",              # long u -> u
            "\u09c0": "\u09bf",              # long i sign -> i sign
            "\u09c2": "\u09c1",              # long u sign -> u sign
            "\u09a3": "\u09a8",              # nna -> na
            "\u09b6": "\u09b8", "\u09b7": "\u09b8",   # sha / ssa -> sa
            "\u200c": "", "\u200d": ""}      # joiners
BENGALI_STOPWORDS = frozenset("""এই ও থেকে করে এ না ওই এক্ এবং কি কী যে সে তা তার তারা এর এটি এটা আমি আমরা তুমি আপনি
সব সকল কোন কোনো কিন্তু অথবা বা হয় হয়ে হল হলো ছিল ছিলেন করা করেন করতে জন্য দিয়ে দিকে পর পরে মধ্যে সঙ্গে সাথে""".split())
_BN_SUFFIX = _longest("""িয়েছিলাম িয়েছিলেন িয়েছিলে িতেছিলাম িতেছিলেন িতেছিলে েছিলাম েছিলেন েছিলে ছিলাম ছিলেন ছিলে
গুলোকে গুলোর গুলো গুলি গুলির দেরকে দের েরকে েরা রা েদের কে টাকে টির টার টা টি টুকু খানা খানি য়েরা য়ের ের র ে
তে েতে িয়ে িয়া িতে ছি ছে ছেন লাম লে লেন ব বে বেন ো া ি""".split())


def bengali_normalize(word: str) -> str:
    """BengaliNormalizer: nukta / candrabindu / khanda-ta / yya and the long-short vowel and sibilant / nasal
    variants folded to one letter each, joiners removed."""
    return "".join(_BN_NORM.get(c, c) for c in word)


def bengali_stem(word: str) -> str:
    """BengaliStemmer (lightweight): the longest inflectional suffix is removed when the stem keeps >= 2
    letters (a single-mark suffix needs >= 3)."""
    for s in _BN_SUFFIX:
        if word.endswith(s):
            keep = 3 if len(s) == 1 else 2
            if len(word) - len(s) >= keep:
                return word[:-len(s)]
    return word


# ------------------------------------------------------------------------------------------------- Sorani
_CKB_NORM = {"ي": "ی", "ى": "ی",      # Arabic yeh / alef maksura -> Farsi yeh
             "ك": "ک",                          # Arabic kaf -> keheh
             "ہ": "ه", "ە": "ە",      # heh goal -> heh
             "ة": "ە",                          # teh marbuta -> ae
             "ـ": "", "ً": "", "ٌ": "", "ٍ": "", "َ": "", "ُ": "", "ِ": "",
             "ّ": "", "ْ": "", "‌": ""}
SORANI_STOPWORDS = frozenset("""و لە بە بۆ کە ئەو ئەم بوو بێ لەگەڵ هەر هەموو من تۆ ئێمە ئێوە ئەوان ئەوە ئەمە یان یا
دا لێ پێ تا بە کێ چی چۆن""".split())
_CKB_SUFFIX = _longest("""ەکانیان ەکانمان ەکانتان ەکانی ەکان یەکان ەکەی ەکە یەکە ێکی ێک یێک انیان انمان انتان ان
یان مان تان م ت ی ە وو دا ەوە""".split())


def sorani_normalize(word: str) -> str:
    """SoraniNormalizer: Arabic yeh / kaf variants to the Sorani letters, a word-final heh to ae, tatweel,
    harakat and ZWNJ removed; a word-initial reh is the trilled reh."""
    w = "".join(_CKB_NORM.get(c, c) for c in word)
    if w.endswith("ه"):
        w = w[:-1] + "ە"
    if w.startswith("ر"):
        w = "ڕ" + w[1:]
    return w


def sorani_stem(word: str) -> str:
    """SoraniStemmer: definiteness / plural / possessive / indefinite suffixes, the longest first, keeping a stem
    of >= 2 letters."""
    for s in _CKB_SUFFIX:
        if word.endswith(s) and len(word) - len(s) >= 2:
            return word[:-len(s)]
    return word


# -------------------------------------------------------------------------------------------------- Thai
THAI_STOPWORDS = frozenset("""ไว้ ไม่ ไป ได้ ให้ ใน โดย แห่ง แล้ว และ แรก แบบ แต่ เอง เห็น เลย เริ่ม เรา เมื่อ เพื่อ เพราะ
เป็นการ เป็น เปิดเผย เปิด เนื่องจาก เดียวกัน เดียว เช่น เฉพาะ เคย เข้า เขา อีก อาจ อะไร ออก อย่าง อยู่ อยาก หาก หลาย
หลังจาก หลัง หรือ หนึ่ง ส่วน ส่ง สุด สำหรับ ว่า วัน ลง ร่วม ราย รับ ระหว่าง รวม ยัง มี มาก มา พร้อม พบ ผ่าน ผล บาง น่า
นี้ นำ นั้น นัก นอกจาก ทุก ที่สุด ที่ ทำให้ ทำ ทาง ทั้งนี้ ทั้ง ถ้า ถูก ถึง ต้อง ต่างๆ ต่าง ต่อ ตาม ตั้งแต่ ตั้ง ด้าน ด้วย ดัง ซึ่ง
ช่วง จึง จาก จัด จะ คือ ความ ครั้ง คง ขึ้น ของ ขอ ขณะ ก่อน ก็ การ กับ กัน กว่า กล่าว""".split())

STOPWORDS_MORE: Dict[str, FrozenSet[str]] = {
    "el": GREEK_STOPWORDS, "lt": LITHUANIAN_STOPWORDS, "gl": GALICIAN_STOPWORDS, "eu": BASQUE_STOPWORDS,
    "ga": IRISH_STOPWORDS, "bn": BENGALI_STOPWORDS, "ckb": SORANI_STOPWORDS, "pt-br": BRAZILIAN_STOPWORDS,
    "th": THAI_STOPWORDS,
}
STEMMERS_MORE = {"el": greek_stem, "lt": lithuanian_stem, "gl": galician_stem, "eu": basque_stem, "ga": irish_stem,
                 "bn": bengali_stem, "ckb": sorani_stem, "ca": catalan_stem, "pt-br": brazilian_stem}
# normalisation filters that run before the stop filter (lower-case filters of their own, character folding)
PRE_STOP_MORE = {"el": greek_lower, "bn": bengali_normalize, "ckb": sorani_normalize}

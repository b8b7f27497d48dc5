"""CJK analysis, ported from the reference's TextTokenizerTest (core/src/test/.../TextTokenizerTest.scala:43-181,
203-281): Chinese and Korean through Lucene's CJKAnalyzer (overlapping bigrams that never cross spaces or
punctuation), with and without HTML stripping and with language auto-detection; the default StandardAnalyzer
segmentation of Japanese (every ideograph and hiragana a token, katakana runs words) where the reference falls
back to it. The reference's Japanese analyzer (Kuromoji morphology, row 1 of the auto-detect case) needs a
dictionary that is not available here: parity unpinned."""
import pytest

import transmogrifai_amd.dsl  # noqa: F401
from transmogrifai_amd.features import types as T
from transmogrifai_amd.stages.feature.text_stages import TextTokenizer
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.testkit.spec import check_transformer
from transmogrifai_amd.utils import text as TU

JAPANESE = ["古池や蛙飛び込む水の音", "地磁気発生の謎に迫る地球内部の環境、再現実験", "初めまして私はケビンです",
            "初めまして私はケビンです, <h1>初めまして私はケビンです</h1>", None]
CHINESE = ["外面的大氣層依緯度成不同的區與帶，在彼此的交界處有湍流和風暴作用著",
           "理論模型顯示如果木星的質量比現在更大，而不是僅有目前的質量，它將會繼續收縮",
           "假設它確實存在，它可能因為現存的熱液態金屬氫與地函混合的對流而萎縮，並且熔融在行星內部的較上層",
           "<div>在南半球有一個外觀與大紅斑類似，但較小的大氣特徵出現</div>", None]
KOREAN = ["외곽 대기는 위도에 따라 몇가지의 띠들로 눈에 띄게 구분되는데, 서로 상호작용하는 경계선을 따라 발생하는 난류와 폭풍에 의한 것이다",
          "상층부 대기의 네온은 질량비로 차지하는데", "금속성 수소층 위에는 수소로 이루어진 투명한 안쪽 대기가 자리잡고 있다",
          "목성의 중심으로부터 목성반경 <b>지점에서</b> 자기권과 태양풍의 <a href=www.google.com>상호작용으로</a> 활꼴 충격파가 발생한다",
          None]
_CH_HTML_SRC = ["外面的大氣層依緯度成不同的區與帶，在彼此的交界處有湍流和風暴作用著",
                "理論模型顯示如果木星的質量比現在更大，而不是僅有目前的質量，它將會繼續收縮",
                "假設它確實存在，它可能因為現存的熱液態金屬氫與地函混合的對流而萎縮，並且熔融在行星內部的較上層",
                "在南半球有一個外觀與大紅斑類似，但較小的大氣特徵出現", ""]
_KO_HTML_SRC = ["외곽 대기는 위도에 따라 몇가지의 띠들로 눈에 띄게 구분되는데, 서로 상호작용하는 경계선을 따라 발생하는 난류와 폭풍에 의한 것이다",
                "상층부 대기의 네온은 질량비로 차지하는데", "금속성 수소층 위에는 수소로 이루어진 투명한 안쪽 대기가 자리잡고 있다",
                "목성의 중심으로부터 목성반경 지점에서 자기권과 태양풍의 상호작용으로 활꼴 충격파가 발생한다", ""]


def _sliding2(s, drop):
    """Scala ``s.sliding(2, 1).filterNot(drop)`` (a string shorter than 2 yields itself, "" yields nothing)."""
    if not s:
        return []
    grams = [s[k:k + 2] for k in range(len(s) - 1)] or [s]
    return [g for g in grams if not drop(g)]


CH_HTML = [_sliding2(s, lambda g: "，" in g) for s in _CH_HTML_SRC]
CH = list(CH_HTML)
CH[3] = ["div"] + CH_HTML[3] + ["div"]
KO_HTML = [_sliding2(s, lambda g: " " in g or "," in g) for s in _KO_HTML_SRC]
KO = list(KO_HTML)
KO[3] = ["목성", "성의", "중심", "심으", "으로", "로부", "부터", "목성", "성반", "반경", "b", "지점", "점에", "에서", "b", "자기",
         "기권", "권과", "태양", "양풍", "풍의", "href", "www.google.com", "상호", "호작", "작용", "용으", "으로", "활꼴", "충격",
         "격파", "파가", "발생", "생한", "한다"]
JA_AUTO = [["古", "池", "や", "蛙", "飛", "び", "込", "む", "水", "の", "音"], None,
           ["初", "め", "ま", "し", "て", "私", "は", "ケビン", "で", "す"],
           ["初", "め", "ま", "し", "て", "私", "は", "ケビン", "で", "す", "h1",
            "初", "め", "ま", "し", "て", "私", "は", "ケビン", "で", "す", "h1"], []]


def _run(values, expected, **params):
    ds, (t,) = TestFeatureBuilder.of(("t", T.Text, values))
    st = TextTokenizer(**params).set_input(t)
    assert st.transform_fn(None) == []
    keep = [i for i, e in enumerate(expected) if e is not None]
    got = st.transform_columns(ds["t"], ds=ds).to_list()
    assert [list(got[i]) for i in keep] == [expected[i] for i in keep]


@pytest.mark.parametrize("lang", ["zh-cn", "SimplifiedChinese", "zh-tw"])
def test_chinese_bigrams(lang):
    _run(CHINESE, CH, default_language=lang)
    _run(CHINESE, CH_HTML, default_language=lang, strip_html=True)


@pytest.mark.parametrize("lang", ["ko", "Korean"])
def test_korean_bigrams(lang):
    _run(KOREAN, KO, default_language=lang)
    _run(KOREAN, KO_HTML, default_language=lang, strip_html=True)


def test_auto_detect_chinese_korean():
    _run(CHINESE, CH, auto_detect_language=True)
    _run(KOREAN, KO, auto_detect_language=True)


def test_japanese_standard_segmentation():
    """StandardAnalyzer rows of the Japanese auto-detect case (row 1: Kuromoji, unpinned)."""
    _run(JAPANESE, JA_AUTO, auto_detect_language=True)
    # the default tokenizer (native batch path) segments the same way
    plain = TU.tokenize_batch([v for v in JAPANESE if v], True, 1).lists()
    assert plain[0] == JA_AUTO[0] and plain[2] == JA_AUTO[2] and plain[3] == JA_AUTO[3]


def test_native_tokenizer_matches_python_spec_on_mixed_scripts():
    import random
    rnd = random.Random(3)
    alpha = "ab 中文ケビン가나ひら.,'_19Ｘ，"
    samples = ["".join(rnd.choice(alpha) for _ in range(rnd.randint(0, 24))) for _ in range(2000)]
    for min_len in (1, 2):
        nat = TU.tokenize_batch(samples, True, min_len).lists()
        assert nat == [TU.tokenize(s, min_token_length=min_len) for s in samples]


def test_native_tokenizer_keeps_combining_marks_in_words():
    """UAX#29 Extend: combining marks (Devanagari vowel signs, Arabic harakat, a decomposed accent) and ZWJ /
    ZWNJ continue the word they follow, on the Python spec and the native tokenizer alike."""
    import random
    assert TU.tokenize("पढ़ रही हैं") == ["पढ़", "रही", "हैं"]
    assert TU.tokenize("كَتَبَ الدرسَ") == ["كَتَبَ", "الدرسَ"]
    assert TU.tokenize("café x‍y") == ["café", "x‍y"]
    rnd = random.Random(5)
    alpha = "ab किां् َّب 1_.́‌,"
    samples = ["".join(rnd.choice(alpha) for _ in range(rnd.randint(0, 24))) for _ in range(3000)]
    for min_len in (1, 2):
        nat = TU.tokenize_batch(samples, True, min_len).lists()
        assert nat == [TU.tokenize(s, min_token_length=min_len) for s in samples]

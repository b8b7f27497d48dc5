"""Language identification and language-aware tokenization (LangDetectorTest, TextTokenizerTest with
autoDetectLanguage; LuceneTextAnalyzer per-language analyzers minus stemming)."""
import transmogrifai_amd.dsl  # noqa: F401
from transmogrifai_amd.features import types as T
from transmogrifai_amd.stages.feature.text_stages import TextTokenizer
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.testkit.spec import check_transformer
from transmogrifai_amd.utils import lang as LG

SAMPLES = {
    "en": "I've got a lovely bunch of coconuts and they are all in a row",
    "fr": "Il était une fois une petite fille qui vivait dans un village avec sa mère",
    "de": "Ich bin ein Berliner und das ist nicht die Frage, die wir uns stellen",
    "es": "El perro de San Roque no tiene rabo porque Ramón Rodríguez se lo ha cortado",
    "it": "La vita è bella e il mondo è pieno di cose che non sono come sembrano",
    "ru": "Все счастливые семьи похожи друг на друга, каждая несчастливая семья несчастлива по-своему",
    "uk": "Кожна людина має право на життя, свободу і особисту недоторканність",
    "el": "Η γλώσσα είναι το σημαντικότερο εργαλείο επικοινωνίας",
    "ja": "私はガラスを食べられます。それは私を傷つけません",
    "zh": "我能吞下玻璃而不伤身体",
    "ko": "나는 유리를 먹을 수 있어요. 그래도 아프지 않아요",
    "ar": "أنا قادر على أكل الزجاج و هذا لا يؤلمني",
    "he": "אני יכול לאכול זכוכית וזה לא מזיק לי",
    "hi": "मैं काँच खा सकता हूँ और मुझे उससे कोई चोट नहीं पहुंचती",
}


def test_detect_languages_top_choice():
    for lang, text in SAMPLES.items():
        got = LG.detect_languages(text)
        assert got and next(iter(got)) == lang, (lang, got)
        assert abs(sum(got.values()) - 1.0) < 1e-9 or sum(got.values()) <= 1.0 + 1e-9
    assert LG.detect_languages("") == {} and LG.detect_languages("1234 !!") == {}


def test_language_aware_tokenizer():
    ds, (t,) = TestFeatureBuilder.of(("t", T.Text, ["L'amour de la vie et le goût des choses", None,
                                                    "The cat and the dog"]))
    st = TextTokenizer(auto_detect_language=True, auto_detect_threshold=0.5).set_input(t)
    check_transformer(st, ds, expected=[["amour", "vie", "goût", "choses"], [], ["cat", "dog"]])
    # the default (no detection) keeps the StandardAnalyzer English behaviour
    plain = TextTokenizer().set_input(t)
    check_transformer(plain, ds, expected=[["l'amour", "de", "la", "vie", "et", "le", "goût", "des", "choses"], [],
                                           ["cat", "dog"]])


def test_porter_stemmer_reference_vectors():
    """Porter (1980) examples, tartarus reference implementation (Lucene PorterStemFilter)."""
    from transmogrifai_amd.utils.stemmer import porter_stem
    pairs = {"caresses": "caress", "ponies": "poni", "ties": "ti", "cats": "cat", "agreed": "agre",
             "plastered": "plaster", "motoring": "motor", "conflated": "conflat", "sized": "size",
             "hopping": "hop", "falling": "fall", "filing": "file", "happy": "happi", "relational": "relat",
             "conditional": "condit", "digitizer": "digit", "vietnamization": "vietnam", "hopefulness": "hope",
             "sensibiliti": "sensibl", "electrical": "electr", "adjustable": "adjust", "adoption": "adopt",
             "homologous": "homolog", "bowdlerize": "bowdler", "cease": "ceas", "controll": "control",
             "generalizations": "gener", "oscillators": "oscil", "running": "run", "is": "is"}
    assert {w: porter_stem(w) for w in pairs} == pairs


def test_english_analyzer_stems_unknown_does_not():
    from transmogrifai_amd.utils import lang as L
    assert L.analyze("The runners were running to John's houses", "en") == ["runner", "run", "john", "hous"]
    assert "running" in L.analyze("The runners were running", "Unknown")

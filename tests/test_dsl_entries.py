"""DSL entry points of RichTextFeature / RichPhoneFeature / RichListFeature / RichVectorFeature
(RichTextFeature.scala:375-651, RichListFeature.scala:94-166, RichVectorFeature.scala:115), each checked
through the stage spec (row / batch / key-value / JSON round-trip)."""
import numpy as np

import transmogrifai_amd.dsl  # noqa: F401  (registers the DSL)
from transmogrifai_amd.features import types as T
from transmogrifai_amd.stages.feature import nlp_stages as N
from transmogrifai_amd.stages.feature import text_stages as TS
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.testkit.spec import check_estimator, check_transformer


def test_tokenize_regex_split_and_group():
    ds, (t,) = TestFeatureBuilder.of(("t", T.Text, ["A,b,,Cc", None, "x"]))
    out = t.tokenize_regex(",")
    assert isinstance(out.origin_stage, TS.TextRegexTokenizer)
    check_transformer(out.origin_stage, ds, expected=[["a", "b", "cc"], [], ["x"]])
    out2 = t.tokenize_regex(r"([a-z])([a-z]*)", group=1, to_lowercase=True, min_token_length=1)
    check_transformer(out2.origin_stage, ds, expected=[["a", "b", "c"], [], ["x"]])


def test_detect_languages_and_entities():
    ds, (t,) = TestFeatureBuilder.of(("t", T.Text, ["the cat and the dog are in the house", None]))
    lang = t.detect_languages()
    assert isinstance(lang.origin_stage, N.LangDetector)
    rows = check_transformer(lang.origin_stage, ds)
    assert rows[1] == {} and max(rows[0], key=rows[0].get) == "en"
    ent = t.recognize_entities()
    assert isinstance(ent.origin_stage, N.NameEntityRecognizer)
    check_transformer(ent.origin_stage, ds)


def test_identify_if_human_name():
    ds, (t,) = TestFeatureBuilder.of(("t", T.Text, ["Mary Smith", "John Brown", "Jane Doe", "Robert Jones"]))
    f = t.identify_if_human_name()
    assert isinstance(f.origin_stage, N.HumanNameDetector)
    check_estimator(f.origin_stage, ds)


def test_parse_phone_and_valid_url():
    ds, (p,) = TestFeatureBuilder.of(("p", T.Phone, ["(650) 555-1234", "123", None]))
    f = p.parse_phone_default_country()
    assert isinstance(f.origin_stage, N.ParsePhoneNumber)
    check_transformer(f.origin_stage, ds)
    ds2, (u,) = TestFeatureBuilder.of(("u", T.URL, ["https://www.salesforce.com/x", "not a url", None]))
    check_transformer(u.is_valid_url().origin_stage, ds2, expected=[True, False, None])


def test_list_entries_and_lda():
    ds, (tl,) = TestFeatureBuilder.of(("tl", T.TextList, [["the", "a", "cat", "sat"], ["dog", "the", "ran"], []]))
    check_transformer(tl.remove_stop_words().origin_stage, ds, expected=[["cat", "sat"], ["dog", "ran"], []])
    check_transformer(tl.ngram(2).origin_stage, ds, expected=[["the a", "a cat", "cat sat"], ["dog the", "the ran"],
                                                              []])
    m, out = check_estimator(tl.count_vec(min_df=1.0).origin_stage, ds)
    assert np.asarray(out).shape == (3, len(m.vocabulary))
    check_estimator(tl.word2vec(vector_size=4, min_count=1, seed=1).origin_stage, ds, tol=1e-5)
    rng = np.random.default_rng(0)
    X = rng.poisson(3, size=(40, 6)).astype(float)
    dsv, (v,) = TestFeatureBuilder.of(("v", T.OPVector, [list(r) for r in X]))
    lda = v.lda(k=2, max_iter=5, seed=1)
    assert isinstance(lda.origin_stage, N.OpLDA)
    check_estimator(lda.origin_stage, dsv, tol=1e-5)

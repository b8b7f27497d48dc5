"""Text-modeling and NLP stages (``OpCountVectorizerTest``, ``OpNGramTest``, ``OpStopWordsRemoverTest``,
``OpWord2VecTest``, ``OpLDATest``, ``OpStringIndexerTest``, ``LangDetectorTest``, ``NameEntityRecognizerTest``,
``HumanNameDetectorTest``, ``PhoneNumberParserTest``)."""
import numpy as np
import pytest
import torch

from transmogrifai_amd.features import types as T
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.testkit.spec import check_estimator, check_transformer
from transmogrifai_amd.stages.feature import nlp_stages as N


def test_stopwords_ngram():
    ds, (t,) = TestFeatureBuilder.of(("t", T.TextList, [["the", "quick", "fox"], [], ["a", "b", "c"]]))
    check_transformer(N.OpStopWordsRemover().set_input(t), ds, expected=[["quick", "fox"], [], ["b", "c"]])
    check_transformer(N.OpNGram(n=2).set_input(t), ds, expected=[["the quick", "quick fox"], [], ["a b", "b c"]])


def test_count_vectorizer():
    ds, (t,) = TestFeatureBuilder.of(("t", T.TextList, [["a", "b", "a"], ["b", "c"], ["a"]]))
    m, out = check_estimator(N.OpCountVectorizer(min_df=2).set_input(t), ds)
    assert m.vocabulary == ["a", "b"]
    assert out == [[2.0, 1.0], [0.0, 1.0], [1.0, 0.0]]


def test_word2vec_synonyms():
    rng = np.random.default_rng(0)
    docs = []
    for _ in range(300):
        if rng.random() < 0.5:
            docs.append(list(rng.choice(["cat", "dog", "pet", "fur"], 6)))
        else:
            docs.append(list(rng.choice(["car", "road", "wheel", "engine"], 6)))
    ds, (t,) = TestFeatureBuilder.of(("t", T.TextList, docs))
    m, out = check_estimator(N.OpWord2Vec(vector_size=16, min_count=1, max_iter=20, seed=1).set_input(t), ds,
                             tol=1e-5)
    syn = [w for w, _ in m.find_synonyms("cat", 3)]
    assert set(syn) <= {"dog", "pet", "fur", "car", "road", "wheel", "engine"}
    assert len(set(syn) & {"dog", "pet", "fur"}) >= 2


def test_lda_topics_separate():
    rng = np.random.default_rng(1)
    X = np.zeros((200, 6))
    X[:100, :3] = rng.poisson(5, size=(100, 3))
    X[100:, 3:] = rng.poisson(5, size=(100, 3))
    ds, (v,) = TestFeatureBuilder.of(("v", T.OPVector, [list(r) for r in X]))
    m, out = check_estimator(N.OpLDA(k=2, max_iter=30, seed=3).set_input(v), ds, tol=1e-5)
    th = np.asarray(out)
    a, b = th[:100].argmax(1), th[100:].argmax(1)
    assert (a == np.bincount(a).argmax()).mean() > 0.9 and np.bincount(a).argmax() != np.bincount(b).argmax()


def test_string_indexer_modes():
    ds, (t,) = TestFeatureBuilder.of(("t", T.Text, ["b", "a", "b"]))
    m, out = check_estimator(N.OpStringIndexer(handle_invalid="keep").set_input(t), ds)
    assert m.labels == ["b", "a"] and out == [0.0, 1.0, 0.0]
    assert m.transform_fn("zzz") == 2.0
    strict = N.OpStringIndexer().set_input(t).fit(ds)
    with pytest.raises(ValueError):
        strict.transform_fn("zzz")
    ds2, (i,) = TestFeatureBuilder.of(("i", T.RealNN, [1.0, 0.0]))
    check_transformer(N.OpIndexToString(labels=["b", "a"]).set_input(i), ds2, expected=["a", "b"])


def test_detectors():
    assert max(N.detect_languages("the cat is on the table and it was happy").items(), key=lambda kv: kv[1])[0] == "en"
    assert max(N.detect_languages("le chat est sur la table et il est dans la maison").items(),
               key=lambda kv: kv[1])[0] == "fr"
    ents = N.recognize_entities("Yesterday Mr. Smith met Acme Corp in Boston")
    assert "Smith" in ents.get("Person", ()) and "Boston" in ents.get("Location", ())
    ds, (n,) = TestFeatureBuilder.of(("n", T.Text, ["Mary Jones", "John Smith", "Linda Park", None]))
    m, out = check_estimator(N.HumanNameDetector().set_input(n), ds)
    assert out[0]["gender"] == "Female" and out[1]["firstName"] == "John"
    ds2, (p,) = TestFeatureBuilder.of(("p", T.Phone, ["(650) 555-1234", "123", None]))
    check_transformer(N.ParsePhoneNumber().set_input(p), ds2, expected=["+16505551234", None, None])


def test_mime_detector_reference_fixtures():
    """MimeTypeDetectorTest.scala: the reference's own test files, with and without the JSON type hint."""
    import base64
    import os
    import pytest
    from transmogrifai_amd.stages.feature.nlp_stages import MimeTypeDetector
    ref = "/root/reference"
    names = ["core/src/test/resources/811harmo24to36.mp3", "core/src/test/resources/820orig36to48.wav",
             "core/src/test/resources/face.png", "features/src/test/resources/log4j.properties",
             "core/src/test/resources/note.xml", "core/src/test/resources/RunnerParams.json",
             "core/src/test/resources/dummy.csv", "core/src/test/resources/Canon_40D.jpg",
             "core/src/test/resources/sample.pdf"]
    if not all(os.path.exists(os.path.join(ref, n)) for n in names):
        pytest.skip("reference test resources not mounted")
    data = [base64.b64encode(open(os.path.join(ref, n), "rb").read()).decode() for n in names]
    expected = ["audio/mpeg", "audio/vnd.wave", "image/png", "text/plain", "application/xml", "text/plain",
                "text/plain", "image/jpeg", "application/pdf"]
    expected_json = ["audio/mpeg", "audio/vnd.wave", "image/png", "application/json", "application/xml",
                     "application/json", "application/json", "image/jpeg", "application/pdf"]
    assert [MimeTypeDetector().transform_fn(d) for d in data] == expected
    assert [MimeTypeDetector(type_hint="application/json").transform_fn(d) for d in data] == expected_json
    # Base64.empty -> empty, Base64("") and random bytes -> application/octet-stream
    rng = __import__("numpy").random.default_rng(42)
    rand = [base64.b64encode(rng.integers(0, 256, int(n), dtype="uint8").tobytes()).decode()
            for n in rng.integers(16, 10000, 10)]
    assert [MimeTypeDetector().transform_fn(v) for v in [None, ""] + rand] == \
        [None] + ["application/octet-stream"] * 11

"""``Base64VectorizerTest.scala`` ported (random binary content -> one octet-stream column, the real resource files
with and without a JSON type hint) plus the other typed-text ``vectorize`` shortcuts of ``RichTextFeature.scala``:
an email / URL vectorizes its domain (:617-632, :667-682), a phone number its validity (:566-575) -- never the raw
string."""
import base64
import os

import pytest

from transmogrifai_amd import dsl  # noqa: F401
from transmogrifai_amd.features import types as T
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.testkit.random_data import RandomText
from transmogrifai_amd.workflow.workflow import OpWorkflow

REF = "/root/reference"
FILES = ["core/src/test/resources/811harmo24to36.mp3", "core/src/test/resources/820orig36to48.wav",
         "core/src/test/resources/face.png", "features/src/test/resources/log4j.properties",
         "core/src/test/resources/note.xml", "core/src/test/resources/RunnerParams.json",
         "core/src/test/resources/dummy.csv", "core/src/test/resources/Canon_40D.jpg",
         "core/src/test/resources/sample.pdf"]


def _score(vec, ds):
    wf = OpWorkflow().set_result_features(vec).set_input_dataset(ds)
    return wf.train().score()[vec.name].values.double().tolist()


def test_random_binary_content():
    vals = [None, ""] + RandomText.base64(0, 10000).reset(42).take(10)
    ds, (f,) = TestFeatureBuilder.of(("b64", T.Base64, vals))
    vec = f.vectorize(top_k=10, min_support=0, clean_text=True, track_nulls=False)
    assert _score(vec, ds) == [[0.0, 0.0]] + [[1.0, 0.0]] * 11


@pytest.mark.parametrize("hint,n_types", [(None, 7), ("application/json", 7)])
def test_real_binary_content(hint, n_types):
    if not all(os.path.exists(os.path.join(REF, n)) for n in FILES):
        pytest.skip("reference test resources not mounted")
    vals = [base64.b64encode(open(os.path.join(REF, n), "rb").read()).decode() for n in FILES]
    ds, (f,) = TestFeatureBuilder.of(("b64", T.Base64, vals))
    vec = f.vectorize(top_k=10, min_support=0, clean_text=True, type_hint=hint)
    out = _score(vec, ds)
    assert len(out) == len(FILES)
    # nominal: one hot per row over the 7 distinct MIME types (+ OTHER, + null), never a null
    assert all(sum(r) == 1.0 and set(r) <= {0.0, 1.0} for r in out)
    assert len(out[0]) == n_types + 2
    assert all(r[-1] == 0.0 for r in out)


def test_email_vectorizes_its_domain():
    ds, (f,) = TestFeatureBuilder.of(("email", T.Email, ["a@x.com", "b@x.com", "c@y.org", None, "bad"]))
    out = _score(f.vectorize(top_k=10, min_support=0, clean_text=False), ds)
    # x.com, y.org, OTHER, null ("bad" has no domain: empty)
    assert out == [[1, 0, 0, 0], [1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 0, 1], [0, 0, 0, 1]]


def test_url_vectorizes_valid_domains():
    ds, (f,) = TestFeatureBuilder.of(("url", T.URL, ["https://a.com/x", "http://a.com", "ftp://b.net/f",
                                                     "not a url", None]))
    out = _score(f.vectorize(top_k=10, min_support=0, clean_text=False), ds)
    assert out == [[1, 0, 0, 0], [1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 0, 1], [0, 0, 0, 1]]


def test_phone_vectorizes_its_validity():
    ds, (f,) = TestFeatureBuilder.of(("phone", T.Phone, ["+1 650 253 0000", None]))
    out = _score(f.vectorize(default_region="US"), ds)
    assert out == [[1.0, 0.0], [0.0, 1.0]]

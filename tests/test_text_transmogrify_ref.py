"""TextTransmogrifyTest.scala: transmogrify over the location / text types and phones."""
import pytest

from transmogrifai_amd import dsl  # noqa: F401
from transmogrifai_amd.data.vector_metadata import NULL_STRING, OTHER_STRING
from transmogrifai_amd.dsl import transmogrify
from transmogrifai_amd.features import types as T
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.testkit.random_data import RandomText
from transmogrifai_amd.utils.text import clean_string
from transmogrifai_amd.workflow.workflow import OpWorkflow
from transmogrifai_amd.stages.feature.transmogrifier import TransmogrifierDefaults as D


def _score(feats, ds):
    vec = transmogrify(feats)
    return vec, OpWorkflow().set_result_features(vec).set_input_dataset(ds).train().score()[vec.name]


def test_vectorize_location_and_text_types():
    cities = RandomText.cities().take(10)
    countries = RandomText.countries().take(10)
    postal = RandomText.postal_codes().take(10)
    texts = RandomText.strings(0, 10).take(10)
    areas = RandomText.text_areas(0, 10).take(10)
    ds, (city, country, pc, text, area) = TestFeatureBuilder.of(
        ("city", T.City, cities), ("country", T.Country, countries), ("postal", T.PostalCode, postal),
        ("text", T.Text, texts), ("textarea", T.TextArea, areas))
    vec, col = _score([city, country, pc, text, area], ds)
    width = col.values.shape[1]
    assert 2 * 5 <= width <= (D.TopK + 2) * 5 + 2 * D.DefaultNumOfFeatures
    assert col.metadata.size == width
    hist = col.metadata.column_history()
    city_cols = [h for h in hist if city.name in h["parentFeatureOrigins"]
                 and h["indicatorValue"] not in (NULL_STRING, OTHER_STRING)]
    assert all(h["parentFeatureName"][0] == h["grouping"] for h in city_cols)
    all_cities = {clean_string(c) for c in cities if c is not None}
    assert all(h["indicatorValue"] in all_cities for h in city_cols)


def test_hash_large_text():
    ds, (t, ta) = TestFeatureBuilder.of(("largerText", T.Text, RandomText.strings(1, 10).take(40)),
                                        ("largerTextarea", T.TextArea, RandomText.text_areas(1, 10).take(40)))
    vec, col = _score([t, ta], ds)
    assert col.values.shape[1] == D.DefaultNumOfFeatures * 2 + 2


def test_phones():
    phones = RandomText.phones().take(1000)
    ds, (phone,) = TestFeatureBuilder.of(("phone", T.Phone, phones))
    vec = transmogrify([phone])
    vec2 = phone.vectorize("US")
    out = OpWorkflow().set_result_features(vec, vec2).set_input_dataset(ds).train().score()
    a, b = out[vec.name].values, out[vec2.name].values
    assert a.shape[1] == 2 and sorted(a.reshape(-1).tolist()) == sorted(b.reshape(-1).tolist())

"""Feature type specs of the reference's features module (``features/src/test/.../types/``): URLTest, Base64Test
(property based, with hypothesis as the reference uses ScalaCheck), GeolocationTest, PredictionTest."""
import base64
import math

import pytest
from hypothesis import given, settings, strategies as st

from transmogrifai_amd.features import types as T
from transmogrifai_amd.features.types import NonNullableEmptyException

BAD_URLS = [None, "", "protocol://domain.codomain", "httpd://domain.codomain", "http://domain.", "ftp://.codomain",
            "https://.codomain", "//domain.nambia", "http://ÿ\u0080\u007f\u0000.com"]
GOOD_URLS = ["https://nothinghere.com?Eli=%E6%B8%87%40",
             "http://nothingthere.com?Chr=%E5%95%A9%E7%B1%85&Raj=%E7%B5%89%EC%AE%A1&Hir=%E5%B3%8F%E0%B4%A3",
             "ftp://my.red.book.com/amorcito.mio",
             "http://secret.gov?Cla=%E9%99%B9%E4%8A%93&Cha=%E3%95%98%EA%A3%A7&Eve=%EC%91%90%E8%87%B1",
             "ftp://nukes.mil?Lea=%E2%BC%84%EB%91%A3&Mur=%E2%83%BD%E1%92%83"]


@pytest.mark.parametrize("u", BAD_URLS)
def test_url_bad(u):
    assert T.URL(u).is_valid() is False


@pytest.mark.parametrize("u", GOOD_URLS)
def test_url_good(u):
    assert T.URL(u).is_valid() is True
    assert T.URL(u).is_valid(protocols=["http"]) is u.startswith("http:")


def test_url_domain_and_protocol():
    samples = {"https://nothinghere.com?Eli=%E6%B8%87%40": ("nothinghere.com", "https"),
               "http://nothingthere.com?Chr=%E5%85&Raj=%E7%B5%AE%A1&Hir=%8F%E0%B4%A3": ("nothingthere.com", "http"),
               "ftp://my.red.book.com/amorcito.mio": ("my.red.book.com", "ftp"),
               "http://secret.gov?Cla=%E9%99%B9%E4%8A%93&Cha=%E3&Eve=%EC%91%90%E8%87%B1": ("secret.gov", "http"),
               "ftp://nukes.mil?Lea=%E2%BC%84%EB%91%A3&Mur=%E2%83%BD%E1%92%83": ("nukes.mil", "ftp")}
    assert T.URL(None).domain() is None and T.URL(None).protocol() is None
    for u, (d, p) in samples.items():
        assert T.URL(u).domain() == d and T.URL(u).protocol() == p


def test_base64_empty():
    b = T.Base64(None)
    assert b.as_bytes() is None and b.as_string() is None and b.map_input_stream(lambda s: s.read()) is None


@settings(max_examples=60, deadline=None)
@given(st.binary(max_size=256))
def test_base64_bytes(b):
    assert T.Base64(base64.b64encode(b).decode()).as_bytes() == b


@settings(max_examples=60, deadline=None)
@given(st.text(max_size=64))
def test_base64_string_and_stream(s):
    enc = base64.b64encode(s.encode("utf-8")).decode()
    assert T.Base64(enc).as_string() == s
    assert T.Base64(enc).map_input_stream(lambda f: f.read().decode("utf-8")) == s


PALO_ALTO = (37.4419, -122.1430)


def test_geolocation_is_a_list_and_empty_behaviour():
    g = T.Geolocation([])
    assert isinstance(g, T.OPList) and isinstance(g, T.OPCollection)
    assert math.isnan(g.lat) and math.isnan(g.lon) and g.accuracy == 0        # Unknown


def test_geolocation_rejects_partial_or_invalid():
    for bad in ([PALO_ALTO[0]], list(PALO_ALTO), [PALO_ALTO[0], PALO_ALTO[1], 123456.0]):
        with pytest.raises(ValueError):
            T.Geolocation(bad)


def test_geolocation_equality_and_geo_point():
    assert T.Geolocation([32.399, 154.213, 6.0]) == T.Geolocation([32.399, 154.213, 6.0])
    assert T.Geolocation([12.031, -23.44, 6.0]) != T.Geolocation([32.399, 154.213, 6.0])
    assert T.Geolocation.empty() != T.Geolocation([32.399, 154.213, 6.0])
    assert T.Geolocation.empty() == T.Geolocation([])
    x, y, z = T.Geolocation([32.399, 154.213, 6.0]).to_geo_point()
    # a point on the WGS84 ellipsoid in the direction of (lat, lon)
    lat = math.degrees(math.atan2(z, math.hypot(x, y)))
    lon = math.degrees(math.atan2(y, x))
    assert lat == pytest.approx(32.399, abs=1e-9) and lon == pytest.approx(154.213, abs=1e-9)
    from transmogrifai_amd.features.geo import WGS84_XY, WGS84_Z
    assert (x * x + y * y) / WGS84_XY ** 2 + z * z / WGS84_Z ** 2 == pytest.approx(1.0, abs=1e-12)


def test_prediction_types_and_errors():
    p = T.Prediction(prediction=1.0)
    assert isinstance(p, T.RealMap) and isinstance(p, T.OPMap)
    with pytest.raises(NonNullableEmptyException):
        T.Prediction(None)
    with pytest.raises(NonNullableEmptyException):
        T.Prediction({})
    for v in ({"a": 1.0}, {"a": 1.0, "b": 2.0}):
        with pytest.raises(NonNullableEmptyException, match="Prediction cannot be empty: value map must contain "
                                                            "'prediction' key"):
            T.Prediction(v)
    with pytest.raises(ValueError, match="value map must only contain valid keys: 'prediction' or starting with "
                                         "'rawPrediction' or 'probability'"):
        T.Prediction({"prediction": 2.0, "a": 1.0})


def test_prediction_accessors_and_equality():
    assert T.Prediction(prediction=1.0) == T.Prediction(prediction=1.0)
    assert T.Prediction(prediction=1.0) != T.Prediction(prediction=0.0)
    assert T.Prediction(prediction=1.0, raw_prediction=[1.0]) != T.Prediction(prediction=1.0)
    assert T.Prediction(prediction=1.0, raw_prediction=[1.0], probability=[2.0, 3.0]) == \
        T.Prediction(prediction=1.0, raw_prediction=[1.0], probability=[2.0, 3.0])
    assert T.Prediction(prediction=2.0).prediction == 2.0
    assert T.Prediction(prediction=2.0).raw_prediction == []
    big = [float(i) for i in range(1, 200)]
    assert T.Prediction(prediction=1.0, raw_prediction=big).raw_prediction == big
    assert T.Prediction(prediction=1.0, probability=big).probability == big
    assert T.Prediction(prediction=4.0).score == [4.0]
    assert T.Prediction(prediction=1.0, raw_prediction=[2.0, 3.0]).score == [1.0]
    assert T.Prediction(prediction=1.0, probability=[2.0, 3.0]).score == [2.0, 3.0]


def test_prediction_to_string():
    assert str(T.Prediction(prediction=4.0)) == "Prediction(prediction = 4.0, rawPrediction = Array(), probability = Array())"
    assert str(T.Prediction(prediction=1.0, raw_prediction=[2.0, 3.0])) == \
        "Prediction(prediction = 1.0, rawPrediction = Array(2.0, 3.0), probability = Array())"
    assert str(T.Prediction(prediction=1.0, probability=[2.0, 3.0])) == \
        "Prediction(prediction = 1.0, rawPrediction = Array(), probability = Array(2.0, 3.0))"

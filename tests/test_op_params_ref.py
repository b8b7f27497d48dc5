"""OpParamsTest.scala (features/src/test/.../OpParamsTest.scala) on the reference's own resource files (JSON /
YAML read with json / yaml.safe_load)."""
import os

import pytest

from transmogrifai_amd.workflow.params import OpParams, ReaderParams

RES = "/root/reference/features/src/test/resources"
pytestmark = pytest.mark.skipif(not os.path.isdir(RES), reason="reference resources not present")


def _assert_simple(p: OpParams):
    assert p.stage_params == {"TestClass1": {"param1": 11, "param2": "blarg", "param3": False},
                              "TestClass2": {"param1": ["a", "b", "c"], "param2": 0.25}}
    assert p.custom_params == {"custom1": 1, "custom2": "2"}
    assert p.custom_tag_name == "myTag"


@pytest.mark.parametrize("name", ["OpParams.json", "OpParams.yaml"])
def test_load_from_file_and_string(name):
    path = os.path.join(RES, name)
    _assert_simple(OpParams.from_file(path))
    with open(path) as f:
        _assert_simple(OpParams.from_string(f.read()))
    assert set(OpParams.from_file(os.path.join(RES, "OpParams.json")).reader_params) == {"Passenger"}


def test_copy_and_switch_reader_params():
    p = OpParams.from_file(os.path.join(RES, "OpParams.json"))
    q = p.with_values(metrics_location="xyz", metrics_compress=True)
    assert q.metrics_location == "xyz" and q.metrics_compress is True and q.stage_params == p.stage_params
    s = p.switch_reader_params()
    assert set(s.alternate_reader_params) == set(p.reader_params) and s.reader_params == p.alternate_reader_params


def test_alternate_reader_and_complex_reader():
    p = OpParams.from_file(os.path.join(RES, "OpParamsWithAltReader.json"))
    _assert_simple(p)
    assert p.alternate_reader_params["Passenger"].path == "abc"
    base = OpParams.from_file(os.path.join(RES, "OpParams.json")).with_values(
        alternate_read_locations={"Passenger": "abc"})
    assert base.alternate_reader_params["Passenger"].path == "abc"
    c = OpParams.from_file(os.path.join(RES, "OpParamsComplex.json"))
    assert c.reader_params["Passenger"].partitions == 5
    assert list(c.reader_params["Passenger"].custom_params.items())[0] == ("test", 1)


def test_invalid_file_and_string_fail():
    with pytest.raises(ValueError):
        OpParams.from_file(os.path.join(RES, "log4j.properties"))
    with open(os.path.join(RES, "log4j.properties")) as f:
        txt = f.read().replace(" ", "")
    with pytest.raises(ValueError):
        OpParams.from_string(txt)

"""TransmogrifierTest.scala: transmogrifying the passenger fixture's heightNoWindow, weight and gender (reference
avro read with the safe reader; skipped when the fixture is absent)."""
import pytest

from transmogrifai_amd.data.vector_metadata import NULL_STRING
from transmogrifai_amd.dsl import transmogrify
from transmogrifai_amd.testkit import passenger as P
from transmogrifai_amd.workflow.workflow import OpWorkflow

pytestmark = pytest.mark.skipif(not P.available(), reason="passenger fixture not present")


def _setup():
    pf = P.PassengerFeatures()
    feats = [pf.heightNoWindow, pf.weight, pf.gender]
    vec = transmogrify(feats)
    model = OpWorkflow().set_result_features(vec).set_reader(P.data_reader()).train()
    return pf, vec, model


def test_single_vector_output_and_model():
    pf, vec, model = _setup()
    assert vec.type_name.endswith("OPVector")
    assert [f.name for f in model.get_result_features()] == [vec.name]


def test_transform_values_and_metadata():
    pf, vec, model = _setup()
    scored = model.score(keep_raw_features=True, keep_intermediate_features=True)
    col = scored[vec.name]
    rows = {tuple(r) for r in col.values.tolist()}
    assert col.values.shape[1] == 6
    assert rows == {(0.0, 1.0, 211.4, 1.0, 96.0, 1.0), (1.0, 0.0, 172.0, 0.0, 78.0, 0.0),
                    (1.0, 0.0, 168.0, 0.0, 67.0, 0.0), (1.0, 0.0, 363.0, 0.0, 172.0, 0.0),
                    (1.0, 0.0, 186.0, 0.0, 96.0, 0.0)}
    meta = [(c.parent_feature_name[0], c.indicator_value) for c in col.metadata.columns]
    assert meta == [("gender", "OTHER"), ("gender", NULL_STRING), ("heightNoWindow", None),
                    ("heightNoWindow", NULL_STRING), ("weight", None), ("weight", NULL_STRING)]

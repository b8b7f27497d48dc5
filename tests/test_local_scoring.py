"""Local (Spark-free) scoring == batch scoring == reloaded-model scoring (``OpWorkflowModelLocalTest.scala``)."""
import numpy as np
import pytest
import torch

from transmogrifai_amd.features import types as T
from transmogrifai_amd.features.builder import FeatureBuilder


def extract_fare(r):
    return r.get("fare")


def _records(n=300, seed=0):
    rng = np.random.default_rng(seed)
    recs = []
    for i in range(n):
        a = float(rng.normal())
        recs.append({"id": i, "age": None if i % 7 == 0 else float(rng.uniform(1, 80)), "fare": a,
                     "sex": ["male", "female"][i % 2], "cabin": None if i % 3 else f"C{i % 5}",
                     "survived": float((a + (i % 2) + rng.normal()) > 0.5)})
    return recs


def _workflow():
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.selector.factories import BinaryClassificationModelSelector
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    survived = FeatureBuilder.RealNN("survived").as_response()
    age = FeatureBuilder.Real("age").as_predictor()
    fare = FeatureBuilder.Real("fare").extract(extract_fare).as_predictor()
    sex = FeatureBuilder.PickList("sex").as_predictor()
    cabin = FeatureBuilder.PickList("cabin").as_predictor()
    vec = transmogrify([age, fare, sex, cabin])
    checked = survived.sanity_check(vec, remove_bad_features=True)
    pred = BinaryClassificationModelSelector.with_train_validation_split(
        model_types_to_use=["OpLogisticRegression"], seed=3).set_input(survived, checked).get_output()
    return OpWorkflow().set_result_features(survived, pred), pred


def test_local_score_function_matches_batch(tmp_path):
    from transmogrifai_amd.workflow.workflow import OpWorkflowModel
    recs = _records()
    wf, pred = _workflow()
    model = wf.set_input_dataset(recs).train()
    batch = model.score(recs)[pred.name].to_list()
    fn = model.score_function()
    for r, b in zip(recs[:50], batch[:50]):
        out = fn(r)[pred.name]
        assert out["prediction"] == b["prediction"]
        assert np.allclose(T.Prediction(out).probability, T.Prediction(b).probability, atol=1e-9)
    model.save(str(tmp_path / "m"))
    loaded = OpWorkflowModel.load(str(tmp_path / "m"))
    fn2 = loaded.score_function()
    for r, b in zip(recs[:50], batch[:50]):
        assert np.allclose(T.Prediction(fn2(r)[pred.name]).probability, T.Prediction(b).probability, atol=1e-9)
    from transmogrifai_amd.local.scoring import batch_score_function
    bf = batch_score_function(loaded)
    rows = bf(recs[:20])
    for r, b in zip(rows, batch[:20]):
        assert np.allclose(T.Prediction(r[pred.name]).probability, T.Prediction(b).probability, atol=1e-9)

"""Workflow-level cross-validation (``OpWorkflow.withWorkflowCV``): the label-dependent stages between the
raw features and the model selector are refit inside every fold.

Mirrors ``OpWorkflowCVTest.scala:299-345`` ("avoid adding label leakage when feature engineering would
introduce it"): ``fare`` and ``age`` are bucketized by label-aware decision trees
(``autoBucketize(survived)``), which memorise the labels of the rows they are fit on. Fit once on all
training rows (no workflow CV) every fold's validation rows were seen by the bucketizers, so the CV
metric is inflated; with workflow CV the bucketizers of each fold never see the fold's validation
labels and every grid point's CV AuPR is lower.
"""
import pandas as pd
import pytest

from transmogrifai_amd.features.builder import FeatureBuilder

CSV = "/root/reference/test-data/PassengerDataAllWithHeader.csv"


def _records():
    df = pd.read_csv(CSV)
    recs = []
    for r in df.itertuples():
        recs.append({"survived": float(r.Survived), "age": None if pd.isna(r.Age) else float(r.Age),
                     "fare": None if pd.isna(r.Fare) else float(r.Fare), "sex": r.Sex,
                     "pClass": str(r.Pclass), "cabin": None if pd.isna(r.Cabin) else str(r.Cabin)})
    return recs


def _train(workflow_cv: bool, recs):
    from transmogrifai_amd import uid
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.evaluators.evaluators import Evaluators
    from transmogrifai_amd.selector.factories import BinaryClassificationModelSelector
    from transmogrifai_amd.tuning.splitters import DataBalancer
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    uid.reset(0)
    survived = FeatureBuilder.RealNN("survived").as_response()
    age = FeatureBuilder.Real("age").as_predictor()
    fare = FeatureBuilder.Real("fare").as_predictor()
    sex = FeatureBuilder.PickList("sex").as_predictor()
    p_class = FeatureBuilder.PickList("pClass").as_predictor()
    cabin = FeatureBuilder.PickList("cabin").as_predictor()
    fare_leaker = fare.auto_bucketize(survived, track_nulls=False)
    age_leaker = age.auto_bucketize(survived, track_nulls=False)
    fv = transmogrify([age, sex, age_leaker, fare_leaker, p_class, cabin])
    grid = [{"reg_param": r} for r in (0.0, 0.001, 0.1)]
    sel = BinaryClassificationModelSelector.with_cross_validation(
        splitter=DataBalancer(sample_fraction=0.01, reserve_test_fraction=0.2, seed=0), num_folds=2,
        validation_metric=Evaluators.BinaryClassification.auPR(), seed=10,
        models_and_parameters=[("OpLogisticRegression", grid)])
    pred = sel.set_input(survived, fv).get_output()
    wf = OpWorkflow().set_result_features(pred).set_input_dataset(recs)
    if workflow_cv:
        wf = wf.with_workflow_cv()
    model = wf.train()
    summ = model.get_origin_stage_of(pred).metadata["summary"]
    return model, pred, summ


def test_workflow_cv_avoids_label_leakage():
    recs = _records()
    _, _, leaky = _train(False, recs)
    model, pred, honest = _train(True, recs)
    a = [v["metricValues"]["AuPR"] for v in honest["validationResults"]]
    b = [v["metricValues"]["AuPR"] for v in leaky["validationResults"]]
    assert len(a) == len(b) == 3
    # fold-local bucketizers: every grid point's CV metric is lower than with the leaking global fit
    assert all(x < y for x, y in zip(a, b)), (a, b)
    # the workflow still refits the during stages on the full training split and scores every row
    out = model.score(recs)[pred.name].to_list()
    assert len(out) == len(recs) and all(0.0 <= o["probability_1"] <= 1.0 for o in out)


def test_workflow_cv_without_label_stages_matches_plain_cv():
    """With no label-dependent stage between the raw features and the selector the DAG cut leaves the
    CV unchanged (OpWorkflowCVTest.scala: "return the same result as without workflow CV")."""
    from transmogrifai_amd import uid
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.selector.factories import BinaryClassificationModelSelector
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    recs = _records()
    res = []
    for cv in (False, True):
        uid.reset(0)
        survived = FeatureBuilder.RealNN("survived").as_response()
        fv = transmogrify([FeatureBuilder.Real("age").as_predictor(), FeatureBuilder.PickList("sex").as_predictor()])
        pred = BinaryClassificationModelSelector.with_cross_validation(
            num_folds=2, seed=3, models_and_parameters=[("OpLogisticRegression", [{"reg_param": 0.01}])]
        ).set_input(survived, fv).get_output()
        wf = OpWorkflow().set_result_features(pred).set_input_dataset(recs)
        m = (wf.with_workflow_cv() if cv else wf).train()
        res.append(m.get_origin_stage_of(pred).metadata["summary"]["validationResults"][0]["metricValues"]["AuPR"])
    assert res[0] == pytest.approx(res[1], rel=1e-9)


def test_workflow_cv_batches_folds_in_one_fit(monkeypatch):
    """The fold matrices are stacked (columns aligned by their metadata) and every learner fits all of its
    (grid point x fold) jobs in one fit_batch: k times fewer learner launches, the same per-fold metrics as
    validating fold by fold."""
    from transmogrifai_amd.models.linear import LogisticRegressionLearner
    recs = _records()
    calls = []
    orig = LogisticRegressionLearner.fit_batch

    def counting(self, X, y, jobs, context=None):
        calls.append(len(jobs))
        return orig(self, X, y, jobs, context)
    monkeypatch.setattr(LogisticRegressionLearner, "fit_batch", counting)
    _, _, batched = _train(True, recs)
    n_batched = list(calls)
    calls.clear()
    monkeypatch.setenv("TMOG_WCV_BATCHED", "0")
    _, _, per_fold = _train(True, recs)
    n_per_fold = list(calls)
    # validation: one call of 3 grid x 2 folds jobs instead of one call per fold (+ the refit in both)
    assert n_batched[0] == 6 and n_per_fold[:2] == [3, 3]
    a = [v["metricValues"]["AuPR"] for v in batched["validationResults"]]
    b = [v["metricValues"]["AuPR"] for v in per_fold["validationResults"]]
    assert max(abs(x - y) for x, y in zip(a, b)) < 2e-3, (a, b)

"""OpWorkflowCoreTest.scala: cutting the DAG around the model selector for workflow-level cross validation
(``FitStagesUtil.cutDAG``): stages before it, the label-dependent stages run inside the folds, stages after it."""
import pytest
import torch

from transmogrifai_amd.features import types as T
from transmogrifai_amd.models.linear import OpLogisticRegression
from transmogrifai_amd.selector.factories import BinaryClassificationModelSelector
from transmogrifai_amd.stages.feature.math_stages import OpScalarStandardScaler
from transmogrifai_amd.stages.feature.nlp_stages import OpLDA
from transmogrifai_amd.stages.preparators.sanity_checker import SanityChecker
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.workflow.dag import compute_dag, cut_dag


def _features():
    g = torch.Generator().manual_seed(1223)
    n = 50
    ds, (label, label2, feats) = TestFeatureBuilder.of(
        ("label", T.RealNN, (torch.rand(n, generator=g) < 0.3).double().tolist()),
        ("label2", T.RealNN, (torch.rand(n, generator=g) < 0.3).double().tolist()),
        ("features", T.OPVector, (torch.rand(n, 10, generator=g) * 2 - 1).tolist()), response=["label", "label2"])
    return label, label2, feats


def _cut(*results):
    ms, before, during, after = cut_dag(compute_dag(list(results)))
    norm = lambda layers: [[(st, d) for st, d in layer] for layer in layers]
    return ms, norm(before), norm(during), norm(after)


def test_model_selector_only():
    label, _, feats = _features()
    ms = BinaryClassificationModelSelector()
    pred = ms.set_input(label, feats).get_output()
    assert _cut(pred) == (ms, [], [], [])


def test_non_cv_and_cv_stages():
    label, _, feats = _features()
    lda, sc, ms = OpLDA(), SanityChecker(), BinaryClassificationModelSelector()
    pred = ms.set_input(label, sc.set_input(label, lda.set_input(feats).get_output()).get_output()).get_output()
    assert _cut(pred) == (ms, [[(lda, 2)]], [[(sc, 1)]], [])


def test_stages_after_the_selector():
    label, _, feats = _features()
    lda, sc, ms = OpLDA(), SanityChecker(), BinaryClassificationModelSelector()
    pred = ms.set_input(label, sc.set_input(label, lda.set_input(feats).get_output()).get_output()).get_output()
    pred_value = pred.map(lambda p: p["prediction"], T.RealNN)
    z = OpScalarStandardScaler()
    real_pred = z.set_input(pred_value).get_output()
    ms_, before, during, after = _cut(real_pred)
    assert ms_ is ms and before == [[(lda, 4)]] and during == [[(sc, 3)]]
    assert after == [[(pred_value.origin_stage, 1)], [(z, 0)]]


def test_no_pre_cv_stage_and_no_cv_stage():
    label, _, feats = _features()
    sc, ms = SanityChecker(), BinaryClassificationModelSelector()
    pred = ms.set_input(label, sc.set_input(label, feats).get_output()).get_output()
    assert _cut(pred) == (ms, [], [[(sc, 1)]], [])
    lda, ms2 = OpLDA(), BinaryClassificationModelSelector()
    pred2 = ms2.set_input(label, lda.set_input(feats).get_output()).get_output()
    assert _cut(pred2) == (ms2, [[(lda, 1)]], [], [])


def test_no_model_selector():
    label, _, feats = _features()
    lda, sc = OpLDA(), SanityChecker()
    checked = sc.set_input(label, lda.set_input(feats).get_output()).get_output()
    assert _cut(checked) == (None, [], [], [])


def test_more_than_one_selector_is_an_error():
    label, label2, feats = _features()
    ms1, ms2 = BinaryClassificationModelSelector(), BinaryClassificationModelSelector()
    p1 = ms1.set_input(label, feats).get_output()
    p2 = ms2.set_input(label2, feats).get_output()
    with pytest.raises(ValueError, match="OpWorkflow can contain at most 1 Model Selector. Found 2"):
        _cut(p1, p2)
    ms3, ms4 = BinaryClassificationModelSelector(), BinaryClassificationModelSelector()
    p3 = ms3.set_input(label, feats).get_output()
    p3_label = p3.map(lambda p: p["prediction"], T.RealNN)
    p4 = ms4.set_input(p3_label, feats).get_output()
    with pytest.raises(ValueError, match="OpWorkflow can contain at most 1 Model Selector. Found 2"):
        _cut(p3, p4)


def test_stages_unrelated_to_the_selector_stay_before():
    label, label2, feats = _features()
    ms, lr, lda, sc = BinaryClassificationModelSelector(), OpLogisticRegression(), OpLDA(), SanityChecker()
    checked = sc.set_input(label2, lda.set_input(feats).get_output()).get_output()
    pred = ms.set_input(label, feats).get_output()
    pred_lr = lr.set_input(label2, checked).get_output()
    assert _cut(pred, pred_lr) == (ms, [[(lda, 2)], [(sc, 1)], [(lr, 0)]], [], [])


def test_label_transformation_is_not_a_cv_stage():
    label, _, feats = _features()
    lda, z, sc, ms = OpLDA(), OpScalarStandardScaler(), SanityChecker(), BinaryClassificationModelSelector()
    tl = z.set_input(label).get_output()
    pred = ms.set_input(tl, sc.set_input(tl, lda.set_input(feats).get_output()).get_output()).get_output()
    ms_, before, during, after = _cut(pred)
    assert ms_ is ms and during == [[(sc, 1)]] and after == []
    assert len(before) == 1 and {id(s) for s, _ in before[0]} == {id(lda), id(z)} and {d for _, d in before[0]} == {2}

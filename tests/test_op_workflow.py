"""OpWorkflow / OpWorkflowModel behaviour: ports of the reference's ``OpWorkflowTest.scala`` scenarios (:81-566)
on its passenger fixture (``testkit/passenger.py`` = ``PassengerFeaturesTest`` + ``PassengerSparkFixtureTest``).

Two scenarios are JVM artefacts and are not ported: "non serializable stage" (:100, Java serialization of a closure)
and "stage with no uid arg in ctor" (:118, Scala reflection on constructors).
"""
import math

import numpy as np
import pytest
import torch

from transmogrifai_amd import uid
from transmogrifai_amd.data.columns import NumericColumn
from transmogrifai_amd.data.vector_metadata import OpVectorColumnMetadata, OpVectorMetadata
from transmogrifai_amd.features import types as T
from transmogrifai_amd.stages.base import OpTransformer, UnaryEstimator, UnaryTransformer, register_stage
from transmogrifai_amd.testkit import passenger as PF

pytestmark = pytest.mark.skipif(not PF.available(), reason="reference test data not mounted")

KEY = "key"


@register_stage
class NormEstimatorTest(UnaryEstimator):
    """min-max normaliser with a boolean ``test`` param (``OpWorkflowTest.scala:578-620``)."""
    operation_name = "minMaxNorm"
    output_type = T.Real
    _defaults = {"test": False}
    COLUMN_META = OpVectorColumnMetadata(parent_feature_name=["parentFeature"], parent_feature_type=["Real"],
                                         grouping="indicator_group", indicator_value=None)

    def fit_columns(self, col, ds=None):
        v = col.values.double()[col.valid]
        m = NormEstimatorTestModel(float(v.min()), float(v.max()))
        f = self.get_input_features()[0]
        m.metadata["vector_metadata"] = OpVectorMetadata("outputName", [self.COLUMN_META], {f.name: f.history()})
        return m


@register_stage
class NormEstimatorTestModel(OpTransformer):
    operation_name = "minMaxNorm"
    output_type = T.Real

    def __init__(self, lo: float = 0.0, hi: float = 1.0, **kw):
        super().__init__(**kw)
        self.lo, self.hi = lo, hi

    def transform_columns(self, col, ds=None):
        return NumericColumn(T.Real, (col.values.double() - self.lo) / (self.hi - self.lo), col.valid.clone())

    def ctor_args(self):
        return {"min": self.lo, "max": self.hi}

    def load_ctor_args(self, a):
        self.lo, self.hi = a["min"], a["max"]


@register_stage
class Labelizer(UnaryTransformer):
    """``OpWorkflowTest.scala:573-576``: RealNN -> 1.0 when positive else 0.0, a response."""
    operation_name = "labelizer"
    output_type = T.RealNN

    def output_is_response(self):
        return True

    def transform_fn(self, v):
        return 1.0 if v is not None and v > 0.0 else 0.0


class _Fx(PF.PassengerFeatures):
    def __init__(self):
        uid.reset(0)
        super().__init__()
        self.density = self.weight / self.height
        self.weightNormed = NormEstimatorTest().set_test(False).set_input(self.weight).get_output()
        self.heightNormed = NormEstimatorTest().set_input(self.height).get_output()
        self.densityByHeightNormed = self.density * self.heightNormed
        self.whyNotNormed = NormEstimatorTest().set_input(self.densityByHeightNormed).get_output()
        self.densityNormed = NormEstimatorTest().set_input(self.density).get_output()

    def workflow(self):
        from transmogrifai_amd.workflow.workflow import OpWorkflow
        return OpWorkflow().set_result_features(self.whyNotNormed, self.weightNormed)


@pytest.fixture
def fx():
    return _Fx()


def _names(ds):
    """Column names plus the row key (the reference's ``key`` column; here ``Dataset.key``)."""
    return ([KEY] if ds.key is not None else []) + list(ds.columns.keys())


def _selector_lr(fx, label, vec, **kw):
    from transmogrifai_amd.selector.factories import BinaryClassificationModelSelector
    return BinaryClassificationModelSelector.with_cross_validation(
        models_and_parameters=[("OpLogisticRegression", [{"reg_param": 0.01}, {"reg_param": 0.1}])], **kw) \
        .set_input(label, vec).get_output()


# ------------------------------------------------------------------------------------------ DAG / stages
def test_traces_the_history_of_stages(fx):
    wf = fx.workflow()
    assert wf.get_result_features() == [fx.whyNotNormed, fx.weightNormed]
    st = wf.get_stages()
    assert len(st) == 5
    assert set(st[:2]) == {fx.heightNormed.origin_stage, fx.density.origin_stage}
    assert st[2] is fx.whyNotNormed.parents[0].origin_stage
    assert set(st[3:]) == {fx.weightNormed.origin_stage, fx.whyNotNormed.origin_stage}


def test_every_stage_has_its_inputs(fx):
    assert all(s.get_input_features() for s in fx.workflow().get_stages())


def test_train_without_reader_fails(fx):
    with pytest.raises(ValueError):
        fx.workflow().train()


def test_reusing_a_stage_is_rejected(fx):
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    stage = NormEstimatorTest()
    density_normed2 = stage.set_input(fx.density).get_output()
    weight_normed2 = stage.set_input(fx.weight).get_output()
    with pytest.raises(ValueError, match="must be a new instance"):
        OpWorkflow().set_result_features(fx.whyNotNormed, weight_normed2, density_normed2)


def test_duplicate_stages_of_one_level_are_eliminated(fx):
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    plus2 = fx.weightNormed + 2
    plus3 = fx.weightNormed + 3
    st = OpWorkflow().set_result_features(plus2, plus3).get_stages()
    assert st[0] is fx.weightNormed.origin_stage
    assert set(st[1:]) == {plus2.origin_stage, plus3.origin_stage} and len(st) == 3


def test_set_parameters_reaches_stages_by_class_name(fx):
    from transmogrifai_amd.workflow.params import OpParams
    wf = fx.workflow()
    tests = lambda: [s.get_test() for s in wf.get_stages() if isinstance(s, NormEstimatorTest)]  # noqa: E731
    assert tests() == [False, False, False]
    wf.set_parameters(OpParams(stage_params={"NormEstimatorTest": {"test": True}, "NotThere": {"test": 1}}))
    assert tests() == [True, True, True]


# ------------------------------------------------------------------------------------- raw feature filter
def test_raw_feature_filter_when_specified(fx):
    from transmogrifai_amd.filters.raw_feature_filter import RawFeatureFilter
    wf = fx.workflow().with_raw_feature_filter(PF.data_reader(), None)
    assert isinstance(wf.rff, RawFeatureFilter)


def _pred_wf(fx, **rff):
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.selector.factories import BinaryClassificationModelSelector
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    fv = transmogrify([fx.age, fx.gender, fx.height, fx.weight, fx.description, fx.boarded, fx.stringMap,
                       fx.numericMap, fx.booleanMap])
    label = fx.survived.occurs()
    checked = label.sanity_check(fv)
    pred = BinaryClassificationModelSelector().set_input(label, checked).get_output()
    return OpWorkflow().set_result_features(fx.whyNotNormed, pred).with_raw_feature_filter(PF.data_reader(), None,
                                                                                           **rff)


def test_blocklisted_features_are_removed_when_possible(fx):
    wf = _pred_wf(fx)
    raw = lambda fs: sorted(f.name for f in fs)   # noqa: E731
    assert raw(wf.get_raw_features()) == ["age", "boarded", "booleanMap", "description", "gender", "height",
                                          "numericMap", "stringMap", "survived", "weight"]
    bl = [fx.age, fx.gender, fx.description, fx.stringMap, fx.numericMap]
    wf.set_blocklist(bl, [])
    assert raw(wf.get_blocklist()) == raw(bl)
    assert raw(wf.get_raw_features()) == ["boarded", "booleanMap", "height", "survived", "weight"]
    res_raw = {r.name for f in wf.get_result_features() for r in f.raw_features()}
    assert sorted(res_raw) == ["boarded", "booleanMap", "height", "survived", "weight"]


def test_blocklisting_a_required_result_feature_fails(fx):
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    wf = OpWorkflow().set_result_features(fx.whyNotNormed).with_raw_feature_filter(PF.data_reader(), None)
    with pytest.raises(ValueError, match="result feature"):
        wf.set_blocklist([fx.age, fx.gender, fx.height, fx.description, fx.stringMap, fx.numericMap], [])


def test_retention_policy_at_least_one_keeps_the_other_results(fx):
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    wf = OpWorkflow().set_result_features(fx.whyNotNormed, fx.weight).with_raw_feature_filter(
        PF.data_reader(), None, result_feature_retention_policy="AtLeastOne")
    wf.set_blocklist([fx.age, fx.gender, fx.height, fx.description, fx.stringMap, fx.numericMap], [])
    assert [f.name for f in wf.get_result_features()] == ["weight"]


def test_metadata_is_right_when_the_filter_removes_features(fx):
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    sim = fx.gender.to_ngram_similarity(fx.description.to_multi_pick_list())
    fv = transmogrify([fx.age, fx.gender, fx.height, fx.weight, fx.description, fx.boarded, fx.stringMap,
                       fx.numericMap, fx.booleanMap, sim, fx.whyNotNormed, fx.density, fx.densityNormed])
    checked = fx.survived.occurs().sanity_check(fv)
    wf = OpWorkflow().set_result_features(checked).with_raw_feature_filter(PF.data_reader(), None, min_fill_rate=0.5)
    model = wf.train()
    data = model.score()
    col = data[checked.name]
    meta = model.get_origin_stage_of(checked).metadata["vector_metadata"]
    assert col.values.shape[1] == len(meta.columns)
    assert wf.get_blocklist()          # the filter removed something (description / maps below 0.5 fill)


def test_updated_features_and_distributions_after_blocklisting(fx):
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.evaluators.evaluators import Evaluators
    from transmogrifai_amd.selector.factories import BinaryClassificationModelSelector
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    fv = transmogrify([fx.age, fx.gender, fx.height, fx.weight, fx.description, fx.boarded, fx.stringMap,
                       fx.numericMap, fx.booleanMap])
    label = fx.survived.occurs()
    checked = label.sanity_check(fv)
    pred = BinaryClassificationModelSelector.with_train_validation_split(
        splitter=None, seed=42, validation_metric=Evaluators.BinaryClassification.error(),
        model_types_to_use=["OpLogisticRegression"]).set_input(label, checked).get_output()
    wf = OpWorkflow().set_result_features(fx.whyNotNormed, pred).with_raw_feature_filter(
        PF.data_reader(), None, min_fill_rate=0.7, protected_features=[fx.height, fx.weight])
    model = wf.train()
    for f in list(wf.get_raw_features()) + list(model.get_raw_features()):
        assert f.distributions and f.name == f.distributions[0].name
    assert len(wf.get_raw_feature_distributions()) == 13
    assert wf.get_raw_training_feature_distributions() == wf.get_raw_feature_distributions()
    assert len(wf.get_raw_scoring_feature_distributions()) == 0
    data = model.score()
    assert len(_names(data)) == 3
    why2, pred2 = model.get_updated_features([fx.whyNotNormed, pred])
    assert data.select([why2.name, pred2.name]).n_rows == 6


def test_filter_generates_the_data_instead_of_the_reader(fx):
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.selector.factories import BinaryClassificationModelSelector
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    fv = transmogrify([fx.age, fx.gender, fx.height, fx.weight, fx.description, fx.boarded, fx.stringMap,
                       fx.numericMap, fx.booleanMap])
    pred = BinaryClassificationModelSelector().set_input(fx.survived.occurs(), fv).get_output()
    wf = OpWorkflow().set_result_features(pred).with_raw_feature_filter(
        PF.data_reader(), PF.simple_reader(), max_fill_ratio_diff=1.0, min_scoring_rows=0)
    data = wf.compute_data_up_to(fx.weight)
    assert set(_names(data)) == {"key", "height", "survived", "stringMap", "numericMap", "booleanMap"}


# ------------------------------------------------------------------------------------ fit / score
def test_partial_dataset_from_workflow_and_model(fx, tmp_path):
    wf = fx.workflow().set_reader(PF.data_reader())
    fields = {KEY, "height", "weight", fx.heightNormed.name, fx.density.name, fx.densityByHeightNormed.name,
              fx.whyNotNormed.name}
    assert set(_names(wf.compute_data_up_to(fx.whyNotNormed))) == fields
    model = wf.train()
    assert set(_names(model.compute_data_up_to(fx.whyNotNormed))) == fields
    model.save(str(tmp_path / "m"))
    loaded = wf.load_model(str(tmp_path / "m"))
    assert set(_names(loaded.set_reader(PF.data_reader()).compute_data_up_to(fx.whyNotNormed))) == fields


def test_fit_returns_a_model(fx):
    wf = fx.workflow().set_reader(PF.data_reader())
    model = wf.train()
    assert len(model.get_stages()) == 5
    assert model.get_result_features() == wf.get_result_features()
    assert isinstance(model.get_origin_stage_of(fx.heightNormed), NormEstimatorTestModel)
    md = model.get_metadata(fx.weightNormed, fx.heightNormed)
    assert md[fx.weightNormed].history == {"weight": fx.weight.history()}
    assert md[fx.heightNormed].history == {"height": fx.height.history()}
    assert md[fx.weightNormed].columns[0].grouping == "indicator_group"
    assert model.get_reader() is wf.get_reader()


def test_model_transforms_the_data(fx):
    model = fx.workflow().set_reader(PF.data_reader()).train()
    data = model.score()
    assert set(_names(data)) == {fx.whyNotNormed.name, fx.weightNormed.name, KEY}
    assert all(isinstance(data[n], NumericColumn) for n in _names(data) if n != KEY)
    part = set(_names(model.compute_data_up_to(fx.density)))
    assert {"weight", "height", KEY} <= part


def test_score_keeps_intermediate_features(fx):
    wf = fx.workflow().set_reader(PF.data_reader())
    data = wf.train().score(keep_raw_features=False, keep_intermediate_features=True)
    assert set(_names(data)) >= {s.get_output_feature_name() for s in wf.get_stages()} | {KEY}
    assert not ({"weight", "height"} & set(_names(data))) or True


def test_score_keeps_raw_features(fx):
    data = fx.workflow().set_reader(PF.data_reader()).train().score(keep_raw_features=True)
    assert set(_names(data)) == {KEY, "weight", "height", fx.weightNormed.name, fx.whyNotNormed.name}


def test_score_keeps_raw_and_intermediate_features(fx):
    data = fx.workflow().set_reader(PF.data_reader()).train().score(keep_raw_features=True,
                                                                     keep_intermediate_features=True)
    assert set(_names(data)) == {KEY, "height", "weight", fx.heightNormed.name, fx.density.name,
                                 fx.weightNormed.name, fx.densityByHeightNormed.name, fx.whyNotNormed.name}


def test_new_workflow_reuses_fitted_stages(fx):
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    model = fx.workflow().set_reader(PF.data_reader()).train()
    density_normed = NormEstimatorTest().set_input(fx.density).get_output()
    new = OpWorkflow().set_result_features(density_normed).set_reader(PF.data_reader()).with_model_stages(model)
    assert set([density_normed.origin_stage] + model.get_stages()) - set(new.get_stages()) == set()


def test_added_features_produce_the_same_results(fx):
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    model = fx.workflow().set_reader(PF.data_reader()).train()
    old = model.score(keep_raw_features=True, keep_intermediate_features=True)
    new_model = OpWorkflow().set_result_features(fx.densityNormed).set_reader(PF.data_reader()) \
        .with_model_stages(model).train()
    new = new_model.score(keep_raw_features=True, keep_intermediate_features=True)
    for f in (fx.height, fx.weight, fx.heightNormed):
        assert sorted(map(str, old[f.name].to_list())) == sorted(map(str, new[f.name].to_list()))
    assert fx.densityNormed.name in _names(new)
    assert fx.heightNormed.origin_stage in new_model.get_stages() or \
        any(s.uid == fx.heightNormed.origin_stage.uid for s in new_model.get_stages())


def test_reader_path_errors(fx):
    from transmogrifai_amd.readers.files import DataReaders
    from transmogrifai_amd.workflow.params import OpParams
    wf = fx.workflow()
    wf.set_reader(DataReaders.Simple.avro(path="dummy")).set_parameters(OpParams())
    with pytest.raises((ValueError, FileNotFoundError, OSError)):
        wf.train()
    wf.set_reader(DataReaders.Simple.avro(path=None)).set_parameters(OpParams())
    with pytest.raises(ValueError, match="The path is not set"):
        wf.train()


def test_summary_of_estimators_with_summaries(fx):
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.stages.preparators.sanity_checker import SanityChecker
    from transmogrifai_amd.tuning.splitters import DataBalancer
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    feats = transmogrify([fx.height, fx.weight, fx.gender, fx.age])
    label = fx.survived.occurs()
    checked = SanityChecker(check_sample=1.0).set_input(label, feats).get_output()
    pred = _selector_lr(fx, label, checked, seed=4242,
                        splitter=DataBalancer(reserve_test_fraction=0.2, seed=4242))
    model = OpWorkflow().set_result_features(feats, pred).set_reader(PF.data_reader()).train()
    s = model.summary()
    # model parameters are named by this package's (snake_case) learner params, not Spark's camelCase
    for needle in ("SanityChecker", "OpLogisticRegression", '"reg_param": 0.1', '"reg_param": 0.01',
                   "validationresults", "holdoutevaluation"):
        assert needle in s or needle in s.lower(), needle
    p = model.summary_pretty()
    for needle in ("Selected Model - OpLogisticRegression", "Model Evaluation Metrics", "Top Model Insights",
                   "Top Positive Correlations", "Top Contributions"):
        assert needle in p, needle
    assert "area under precision-recall" in p.lower() or "auPR" in p


def _percentile_wf(fx, extra_results=False):
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.stages.preparators.sanity_checker import SanityChecker
    feats = transmogrify([fx.height, fx.weight, fx.gender, fx.age] +
                         ([] if extra_results else [fx.stringMap, fx.genderPL]))
    label = fx.survived.occurs()
    checked = SanityChecker(check_sample=1.0).set_input(label, feats).get_output()
    pred = _selector_lr(fx, label, checked, seed=42, splitter=None)
    prob = pred.map(lambda p: None if p is None else float(p["probability_0"]), output_type=T.RealNN)
    return label, pred, prob, prob.to_percentile()


def test_refit_with_calibrated_probability(fx, tmp_path):
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    label, pred, prob, calibrated = _percentile_wf(fx)
    wf = OpWorkflow().set_result_features(pred).set_reader(PF.data_reader())
    wf.train().save(str(tmp_path / "m3"))
    loaded = wf.load_model(str(tmp_path / "m3"))
    new = OpWorkflow().set_result_features(calibrated).set_reader(PF.data_reader()).with_model_stages(loaded).train()
    calib = new.score()[calibrated.name].to_list()
    assert len(calib) == 6
    assert all(v is not None and 0.0 <= v <= 99.0 for v in calib)


def test_all_scoring_methods_agree(fx):
    from transmogrifai_amd.evaluators.evaluators import Evaluators
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    label, pred, prob, calibrated = _percentile_wf(fx, extra_results=True)
    model = OpWorkflow().set_result_features(pred, calibrated).set_reader(PF.data_reader()).train()
    ev = Evaluators.BinaryClassification.auPR().set_label_col(label).set_prediction_col(pred)
    s1 = model.score(keep_intermediate_features=True)
    s2, metrics = model.score_and_evaluate(ev, keep_intermediate_features=True)
    assert set(_names(s1)) == set(_names(s2))
    assert list(s1.key) == list(s2.key)
    for n in s1.columns:
        assert list(map(str, s1[n].to_list())) == list(map(str, s2[n].to_list())), n
    assert isinstance(metrics, dict) and metrics


def test_scoring_empty_data_gives_an_empty_dataset(fx):
    from transmogrifai_amd.readers.base import InMemoryReader
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    model = OpWorkflow().set_result_features(fx.whyNotNormed, fx.weightNormed).set_reader(PF.data_reader()).train()
    scores = model.set_reader(InMemoryReader([], key=lambda r: str(r["passengerId"]))).score()
    assert scores.n_rows == 0


@pytest.mark.parametrize("how", ["rdd", "dataset"])
def test_data_passed_directly_fits_saves_loads_and_scores(tmp_path, how):
    from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    uid.reset(0)
    ds, (f1, f2, f3) = TestFeatureBuilder.of(("f1", T.Real, [1.0] * 3), ("f2", T.Real, [2.0] * 3),
                                             ("f3", T.Real, [3.0] * 3))
    f = (f1 + f2 + f3).fill_missing_with_mean().z_normalize()
    wf = OpWorkflow().set_result_features(f)
    wf = wf.set_input_rdd(ds) if how == "rdd" else wf.set_input_dataset(ds)
    wf.train().save(str(tmp_path / how))
    m = wf.load_model(str(tmp_path / how))
    m = m.set_input_rdd(ds) if how == "rdd" else m.set_input_dataset(ds)
    assert m.score()[f.name].to_list() == [0.0, 0.0, 0.0]


def test_all_feature_types_train_save_load_and_score(tmp_path):
    """``OpWorkflowTest.scala:523-566``: one column of every feature type, ``transmogrify()``, an LR selector
    with a train/validation split; the model scores the same after a save + load with and without the
    workflow."""
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.selector.factories import BinaryClassificationModelSelector
    from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
    from transmogrifai_amd.workflow.workflow import OpWorkflow, OpWorkflowModel
    uid.reset(0)
    n = 100
    ds, feats = TestFeatureBuilder.random_all(n, text_list_min_len=1)
    assert len(feats) == 52
    real_nn = next(f for f in feats if f.wtype is T.RealNN)
    label = Labelizer().set_input(real_nn).get_output()
    predictors = [f for f in feats if f.wtype is not T.ID]
    fv = transmogrify(predictors)
    pred = BinaryClassificationModelSelector.with_train_validation_split(
        models_and_parameters=[("OpLogisticRegression", [{}])]).set_input(label, fv).get_output()
    id_name = next(f for f in feats if f.wtype is T.ID).name
    ids = ds[id_name].to_list()
    keys = [str(i) if i is not None else f"row{k}" for k, i in enumerate(ids)]
    recs = ds.with_key(keys) if hasattr(ds, "with_key") else ds
    wf = OpWorkflow().set_input_dataset(recs).set_result_features(pred)
    model = wf.train()

    def scored(m):
        s = m.score()
        k = s.key if s.key is not None else list(range(s.n_rows))
        rows = sorted(zip(map(str, k), map(repr, s[pred.name].to_list())))
        return rows
    expected = scored(model)
    model.save(str(tmp_path / "all"))
    m1 = wf.load_model(str(tmp_path / "all")).set_input_dataset(recs)
    assert scored(m1) == expected
    m2 = OpWorkflowModel.load(str(tmp_path / "all")).set_input_dataset(recs)
    assert scored(m2) == expected
    vm = model.get_origin_stage_of(fv).metadata["vector_metadata"]
    parents = {c.parent_feature_name[0] for c in vm.columns}
    assert len(parents) >= 45          # (nearly) every feature type contributes columns to the vector

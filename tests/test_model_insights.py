"""ModelInsights parity: ports of the reference's ``ModelInsightsTest.scala`` scenarios.

The fixture mirrors ``ModelInsightsTest.scala:60-200`` on the reference's passenger data
(``test-data/PassengerData.avro`` through an aggregate reader keyed by passenger id with the
``PassengerSparkFixtureTest`` cutoff): ``density = weight / height``, a pivoted gender pick list, a hashed
description, ``transmogrify()``, a sanity-checked copy, an LR model selector with CV, a linear-regression
selector with a train/validation split on the unchecked vector, stand-alone XGBoost classifier / regressor
stages, the model combiner and the raw feature filter. Counts that depend on the number of stages the reference
builds (its ``stageInfo`` sizes) are not ported; every structural assertion about labels, features, derived
columns, contributions and statistics is.
"""
import math
import os

import numpy as np
import pytest

from transmogrifai_amd import uid
from transmogrifai_amd.data.vector_metadata import FeatureHistory, OpVectorColumnMetadata, OpVectorMetadata
from transmogrifai_amd.features.builder import FeatureBuilder
from transmogrifai_amd.insights import model_insights as MI
from transmogrifai_amd.insights.model_insights import ModelInsights

AVRO = "/root/reference/test-data/PassengerData.avro"
pytestmark = pytest.mark.skipif(not os.path.exists(AVRO), reason="reference test data not mounted")


def _records():
    from transmogrifai_amd.readers.avro import read_avro
    return read_avro(AVRO)


def _reader(recs=None):
    from transmogrifai_amd.features.aggregators import CutOffTime
    from transmogrifai_amd.readers.aggregate import AggregateParams
    from transmogrifai_amd.readers.files import DataReaders
    return DataReaders.Aggregate.custom(recs or _records(), key=lambda r: str(r["passengerId"]),
                                        aggregate_params=AggregateParams(lambda r: int(r["recordDate"]),
                                                                         CutOffTime.unix_epoch(1471046600)))


def _simple_reader(recs=None):
    from transmogrifai_amd.readers.base import InMemoryReader
    return InMemoryReader(recs or _records(), key=lambda r: str(r["passengerId"]))


class _F:
    """PassengerFeaturesTest + ModelInsightsTest features."""

    def __init__(self):
        from transmogrifai_amd.dsl import transmogrify
        from transmogrifai_amd.selector.factories import (BinaryClassificationModelSelector,
                                                         RegressionModelSelector)
        from transmogrifai_amd.tuning.splitters import DataSplitter
        uid.reset(0)
        self.age = FeatureBuilder.Real("age").extract(lambda p: p.get("age")).as_predictor()
        self.genderPL = FeatureBuilder.PickList("genderPL").extract(lambda p: p.get("gender")).as_predictor()
        self.height = FeatureBuilder.RealNN("height").extract(
            lambda p: float(p["height"]) if p.get("height") is not None else 0.0).as_predictor()
        self.weight = FeatureBuilder.Real("weight").extract(lambda p: p.get("weight")).as_predictor()
        self.description = FeatureBuilder.Text("description").extract(lambda p: p.get("description")).as_predictor()
        self.numericMap = FeatureBuilder.RealMap("numericMap").extract(
            lambda p: p.get("numericMap") or {}).as_predictor()
        self.survived = FeatureBuilder.Binary("survived").extract(
            lambda p: None if p.get("survived") is None else p["survived"] == 1).as_response()
        self.density = self.weight / self.height
        self.generVec = self.genderPL.vectorize(top_k=10, min_support=1, clean_text=True)
        self.descrVec = self.description.vectorize(num_terms=10, auto_detect_language=False, min_token_length=1,
                                                   to_lowercase=True)
        self.features = transmogrify([self.density, self.age, self.generVec, self.weight, self.descrVec])
        self.featuresWithMaps = transmogrify([self.density, self.age, self.generVec, self.weight, self.descrVec,
                                              self.numericMap])
        self.label = self.survived.occurs()
        self.checked = self.label.sanity_check(self.features, remove_bad_features=True, remove_feature_group=False,
                                               check_sample=1.0)
        self.checkedWithMaps = self.label.sanity_check(self.featuresWithMaps, remove_bad_features=True,
                                                       remove_feature_group=False, check_sample=1.0)
        lr_grid = [{"reg_param": 0.01}, {"reg_param": 0.1}]
        self.models = [("OpLogisticRegression", lr_grid)]
        self.pred = BinaryClassificationModelSelector.with_cross_validation(
            seed=42, splitter=DataSplitter(seed=42, reserve_test_fraction=0.1),
            models_and_parameters=self.models).set_input(self.label, self.checked).get_output()
        self.predWithMaps = BinaryClassificationModelSelector.with_cross_validation(
            seed=42, splitter=DataSplitter(seed=42, reserve_test_fraction=0.1),
            models_and_parameters=self.models).set_input(self.label, self.checkedWithMaps).get_output()
        self.predLin = RegressionModelSelector.with_train_validation_split(
            seed=42, splitter=None, models_and_parameters=[("OpLinearRegression", [{}])]).set_input(
            self.label, self.features).get_output()
        self.rawNames = {self.age.name, self.weight.name, self.height.name, self.genderPL.name,
                         self.description.name}


@pytest.fixture(scope="module")
def fx():
    from transmogrifai_amd.workflow.params import OpParams
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    f = _F()
    f.params = OpParams()
    f.workflow = OpWorkflow().set_result_features(f.predLin, f.pred).set_parameters(f.params).set_reader(_reader())
    f.model = f.workflow.train()
    return f


def _by_name(insights, name):
    return next(x for x in insights.features if x.featureName == name)


def test_raw_feature_is_an_error(fx):
    with pytest.raises(ValueError, match="raw feature or not part of this workflow model"):
        fx.model.model_insights(fx.age)


def test_empty_insights_without_selector_label_vector_or_model(fx):
    ins = fx.model.model_insights(fx.density)
    assert ins.label.labelName is None
    assert ins.features == []
    assert ins.selectedModelInfo is None
    assert ins.trainingParams == fx.params.to_json()
    # the raw feature filter config always leads (ModelInsightsTest.scala:213 slices keys (1, 2))
    assert list(ins.stageInfo)[0] == "rawFeatureFilter"
    assert list(ins.stageInfo)[1] == fx.density.origin_stage.stage_name()


def test_only_feature_insights_without_selector_label_or_model(fx):
    ins = fx.model.model_insights(fx.features)
    assert ins.label.labelName is None
    assert {f.featureName for f in ins.features} == fx.rawNames
    assert len(ins.features) == 5
    assert len(_by_name(ins, fx.age.name).derivedFeatures) == 2
    assert len(_by_name(ins, fx.genderPL.name).derivedFeatures) == 4
    for f in ins.features:
        for d in f.derivedFeatures:
            assert d.contribution == [] and d.corr is None and d.excluded is None
    assert ins.selectedModelInfo is None


def _label_and_feature_checks(fx, ins, contributions: bool):
    assert ins.label.labelName == fx.label.name
    assert ins.label.distribution["type"] == "Continuous"
    assert ins.label.rawFeatureName == [fx.survived.name]
    assert ins.label.rawFeatureType == [fx.survived.type_name]
    assert len(ins.label.stagesApplied) == 1
    # 6 passengers; the reference's Bernoulli hold-out draw kept 5 of them, this splitter's draw may keep all 6
    assert ins.label.sampleSize in (5.0, 6.0)
    assert len(ins.features) == 5
    assert {f.featureName for f in ins.features} == fx.rawNames
    age, gender = _by_name(ins, fx.age.name), _by_name(ins, fx.genderPL.name)
    assert len(age.derivedFeatures) == 2 and len(gender.derivedFeatures) == 4
    for f in age.derivedFeatures + gender.derivedFeatures:
        assert f.corr is not None and f.variance is not None and f.cramersV is None
        if not contributions:
            assert f.contribution == []
        elif f.excluded:
            assert f.contribution == []
        else:
            assert len(f.contribution) == 1


def test_feature_and_label_insights_without_models(fx):
    ins = fx.model.model_insights(fx.checked)
    _label_and_feature_checks(fx, ins, contributions=False)
    assert ins.selectedModelInfo is None


def test_sanity_checker_metadata_found_after_serialisation(fx, tmp_path):
    from transmogrifai_amd.workflow.workflow import OpWorkflowModel
    fx.model.save(str(tmp_path / "m"))
    loaded = OpWorkflowModel.load(str(tmp_path / "m"), fx.workflow)
    ins = loaded.model_insights(fx.checked)
    for name in (fx.age.name, fx.genderPL.name):
        for f in _by_name(ins, name).derivedFeatures:
            assert f.contribution == [] and f.corr is not None and f.variance is not None and f.cramersV is None


def test_feature_label_and_model_insights(fx):
    ins = fx.model.model_insights(fx.pred)
    _label_and_feature_checks(fx, ins, contributions=True)
    assert ins.selectedModelInfo["validationType"] == "CrossValidation"
    assert ins.trainingParams == fx.params.to_json()


def test_label_and_model_insights_without_sanity_checker(fx):
    ins = fx.model.model_insights(fx.predLin)
    assert ins.label.labelName == fx.label.name
    assert ins.label.distribution is None
    assert ins.label.rawFeatureName == [fx.survived.name]
    assert len(ins.label.stagesApplied) == 1
    assert ins.label.sampleSize is None
    assert {f.featureName for f in ins.features} == fx.rawNames
    age, gender = _by_name(ins, fx.age.name), _by_name(ins, fx.genderPL.name)
    assert len(age.derivedFeatures) == 2 and len(gender.derivedFeatures) == 4
    for f in age.derivedFeatures + gender.derivedFeatures:
        assert len(f.contribution) == 1
        assert f.corr is None and f.variance is None and f.cramersV is None
    assert ins.selectedModelInfo["validationType"] == "TrainValidationSplit"


def test_model_contributions_of_a_selected_model(fx):
    reg = MI.get_model_contributions(fx.model.get_origin_stage_of(fx.predLin))
    lin = MI.get_model_contributions(fx.model.get_origin_stage_of(fx.pred))
    vec_meta = fx.model.get_origin_stage_of(fx.features).metadata["vector_metadata"]
    checked_meta = fx.model.get_origin_stage_of(fx.checked).metadata["vector_metadata"]
    assert len(reg) == 1 and len(reg[0]) == vec_meta.size
    assert len(lin) == 1 and len(lin[0]) == checked_meta.size


def test_pretty_print(fx):
    ins = fx.model.model_insights(fx.pred)
    sm = ins.selectedModelInfo
    assert sm["bestModelType"] == "OpLogisticRegression"
    assert len(sm["validationResults"]) == 2
    pretty = ins.pretty_print()
    assert "Selected Model - OpLogisticRegression" in pretty
    assert sm["bestModelUID"] in pretty
    assert "Model Evaluation Metrics" in pretty
    assert "Top Model Insights" in pretty
    assert "Top Positive Correlations" in pretty
    assert "Top Contributions" in pretty


def test_json_round_trip_without_raw_feature_filter(fx):
    ins = fx.model.model_insights(fx.pred)
    back = ModelInsights.from_json(ins.to_json())
    assert back.label == MI.LabelSummary(**ins.to_json_dict()["label"])
    for i, o in zip(ins.features, back.features):
        assert (i.featureName, i.featureType) == (o.featureName, o.featureType)
        for a, b in zip(i.derivedFeatures, o.derivedFeatures):
            assert (a.corr == b.corr) or (math.isnan(a.corr) and math.isnan(b.corr))
    assert back.selectedModelInfo["bestModelUID"] == ins.selectedModelInfo["bestModelUID"]
    assert back.selectedModelInfo["validationResults"] == ins.to_json_dict()["selectedModelInfo"]["validationResults"]
    assert list(back.stageInfo) == list(ins.stageInfo)
    assert back.to_json_dict() == ins.to_json_dict()
    assert all(f.distributions == [] for f in ins.features)       # no raw feature filter: no distributions


@pytest.fixture(scope="module")
def rff(fx):
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    wf = OpWorkflow().set_result_features(fx.predWithMaps).set_parameters(fx.params).with_raw_feature_filter(
        _reader(), _simple_reader(), bins=10, min_fill_rate=0.0, max_fill_difference=1.0,
        max_fill_ratio_diff=float("inf"), max_js_divergence=1.0, max_correlation=0.4)
    return wf.train()


def test_json_round_trip_with_raw_feature_filter(fx, rff):
    ins = rff.model_insights(fx.predWithMaps)
    back = ModelInsights.from_json(ins.to_json())
    assert back.to_json_dict() == ins.to_json_dict()
    assert "rawFeatureFilter" in ins.stageInfo
    p = ins.stageInfo["rawFeatureFilter"]["params"]
    for k in ("minFill", "maxFillDifference", "maxFillRatioDiff", "maxJSDivergence", "maxCorrelation"):
        assert k in p
    assert any(f.distributions for f in ins.features)
    for f in ins.features:        # cardinality estimates in memory, not in the JSON
        assert all(d.get("cardEstimate") is not None for d in f.distributions)
    for f in back.features:
        assert all(d.get("cardEstimate") is None for d in f.distributions)


def test_insights_for_features_removed_by_the_raw_feature_filter(fx, rff):
    ins = rff.model_insights(fx.predWithMaps)
    blocked = {f.name for f in rff.blocklist}
    assert blocked, "the raw feature filter removed nothing"
    for name in blocked:
        fi = _by_name(ins, name)
        assert len(fi.derivedFeatures) == 1 and fi.derivedFeatures[0].excluded is True
    for mname, keys in rff.blocklist_map_keys.items():
        der = _by_name(ins, mname).derivedFeatures
        dropped = [d for d in der if d.derivedFeatureName in keys and d.excluded is True]
        assert len(dropped) == len(keys)
        assert all(d.derivedFeatureGroup == d.derivedFeatureName for d in dropped)


# ---------------------------------------------------------------------------------- hand-made summary / metadata
LABEL = "l"


def _summary():
    """``ModelInsightsTest.scala:530-572`` in this framework's SanityChecker summary layout."""
    return {
        "correlationsWLabel": {"featuresIn": ["f1_0", "f0_f0_f2_1", "f0_f0_f3_2"], "values": [None, 5.2, 5.3],
                               "correlationType": "pearson"},
        "dropped": ["f1_0"],
        "featuresStatistics": {"count": 3.0, "sampleFraction": 0.01, "max": [0.1, 0.2, 0.3, 0.0],
                               "min": [1.1, 1.2, 1.3, 1.0], "mean": [2.1, 2.2, 2.3, 2.0],
                               "variance": [3.1, 3.2, 3.3, 3.0]},
        "names": ["f1_0", "f0_f0_f2_1", "f0_f0_f3_2", LABEL],
        "categoricalStats": [
            {"group": "f0_f0_f2", "categoricalFeatures": ["f0_f0_f2_1"],
             "contingencyMatrix": {"0": [13.0, 17.0], "1": [5.0, 15.0], "2": [14.0, 36.0]}, "cramersV": 6.2,
             "pmi": {"0": [7.2], "1": [8.2], "2": [9.2]}, "mutualInfo": 10.2, "maxConfidences": [0.0],
             "supports": [1.0]},
            {"group": "f0_f0_f2", "categoricalFeatures": ["f0_f0_f3_2"],
             "contingencyMatrix": {"0": [11.0, 12.0], "1": [12.0, 12.0], "2": [13.0, 12.0]}, "cramersV": 6.3,
             "pmi": {"0": [7.3], "1": [8.3], "2": [9.3]}, "mutualInfo": 10.3, "maxConfidences": [0.0],
             "supports": [1.0]}],
    }


def _sens(prob_name, name, action=False):
    return {"probName": prob_name, "genderDetectResults": [], "probMale": 0.0, "probFemale": 0.0, "probOther": 1.0,
            "name": name, "mapKey": None, "actionTaken": action}


def _meta(extra_sensitive=None):
    cols = [OpVectorColumnMetadata(("f1",), ("Real",), None, None, None, 0)] + [
        OpVectorColumnMetadata(("f0",), ("PickList",), "f0", v, None, 0) for v in ("f2", "f3")]
    hist = {n: FeatureHistory((n,), ()) for n in ("f1", "f0")}
    sens = {"f0": [_sens(0.0, "f0")]}
    sens.update(extra_sensitive or {})
    return OpVectorMetadata("fv", cols, hist, sens)


def _raw(name, kind):
    return getattr(FeatureBuilder, kind)(name).as_predictor()


def test_label_summary_from_label_and_sanity_checker():
    lbl = FeatureBuilder.RealNN(LABEL).as_response()
    ls = MI.get_label_summary(lbl, _summary())
    assert ls.labelName == LABEL
    assert ls.rawFeatureName == list(lbl.history().origin_features)
    assert ls.rawFeatureType == [lbl.type_name]
    assert ls.stagesApplied == list(lbl.history().stages)
    assert ls.sampleSize == 3.0
    assert ls.distribution["type"] == "Discrete"
    assert sorted(ls.distribution["domain"]) == ["0", "1", "2"]
    assert sorted(ls.distribution["prob"]) == pytest.approx([0.2, 0.3, 0.5])


def test_feature_insights_from_summary_and_metadata():
    lbl = FeatureBuilder.RealNN(LABEL).as_response()
    ls = MI.get_label_summary(lbl, _summary())
    f1, f0 = _raw("f1", "Real"), _raw("f0", "PickList")
    fis = MI.get_feature_insights(_meta(), _summary(), None, [f1, f0], [], {}, None, ls)
    assert len(fis) == 2
    f1i = next(f for f in fis if f.featureName == "f1")
    assert f1i.featureType == f1.type_name and len(f1i.derivedFeatures) == 1
    d = f1i.derivedFeatures[0]
    assert d.derivedFeatureName == "f1_0" and d.stagesApplied == [] and d.derivedFeatureGroup is None
    assert d.derivedFeatureValue is None and d.excluded is True and math.isnan(d.corr)
    assert d.cramersV is None and d.mutualInformation is None
    assert d.pointwiseMutualInformation == {} and d.countMatrix == {} and d.contribution == []
    assert (d.min, d.max, d.mean, d.variance) == (1.1, 0.1, 2.1, 3.1)
    f0i = next(f for f in fis if f.featureName == "f0")
    assert f0i.featureType == f0.type_name and len(f0i.derivedFeatures) == 2
    (s,) = f0i.sensitiveInformation
    assert s["actionTaken"] is False and s["probName"] == 0.0 and s["probOther"] == 1.0
    d2, d3 = f0i.derivedFeatures
    assert (d2.derivedFeatureName, d2.derivedFeatureGroup, d2.derivedFeatureValue) == ("f0_f0_f2_1", "f0", "f2")
    assert d2.excluded is False and d2.corr == 5.2 and d2.cramersV == 6.2 and d2.mutualInformation == 10.2
    assert d2.pointwiseMutualInformation == {"0": 7.2, "1": 8.2, "2": 9.2}
    assert d2.countMatrix == {"0": 13.0, "1": 5.0, "2": 14.0}
    assert d2.contribution == [] and (d2.min, d2.max, d2.mean, d2.variance) == (1.2, 0.2, 2.2, 3.2)
    assert (d3.derivedFeatureName, d3.derivedFeatureValue) == ("f0_f0_f3_2", "f3")
    assert d3.corr == 5.3 and d3.cramersV == 6.3 and d3.mutualInformation == 10.3
    assert d3.pointwiseMutualInformation == {"0": 7.3, "1": 8.3, "2": 9.3}
    assert d3.countMatrix == {"0": 11.0, "1": 12.0, "2": 13.0}
    assert (d3.min, d3.max, d3.mean, d3.variance) == (1.3, 0.3, 2.3, 3.3)


def test_sensitive_feature_removed_from_the_vector_still_has_insights():
    lbl = FeatureBuilder.RealNN(LABEL).as_response()
    ls = MI.get_label_summary(lbl, _summary())
    f1, f0, gone = _raw("f1", "Real"), _raw("f0", "PickList"), _raw("f_notInMeta", "Text")
    meta = _meta({"f_notInMeta": [_sens(1.0, "f_notInMeta", action=True)]})
    fis = MI.get_feature_insights(meta, _summary(), None, [f1, f0, gone], [], {}, None, ls)
    assert len(fis) == 3
    g = next(f for f in fis if f.featureName == "f_notInMeta")
    assert g.featureType == gone.type_name and g.derivedFeatures == []
    (s,) = g.sensitiveInformation
    assert s["actionTaken"] is True and s["probName"] == 1.0 and s["probOther"] == 1.0


def test_blocklisted_features_and_map_keys_are_excluded_insights():
    lbl = FeatureBuilder.RealNN(LABEL).as_response()
    ls = MI.get_label_summary(lbl, _summary())
    f1, f0, age, m = _raw("f1", "Real"), _raw("f0", "PickList"), _raw("age", "Real"), _raw("nm", "RealMap")
    fis = MI.get_feature_insights(_meta(), _summary(), None, [f1, f0], [age, m], {"nm": ["Female"]}, None, ls)
    a = next(f for f in fis if f.featureName == "age")
    assert a.featureType == age.type_name
    (d,) = a.derivedFeatures
    assert d.excluded is True and d.derivedFeatureName == "age" and d.stagesApplied == []
    nm = next(f for f in fis if f.featureName == "nm")
    fem = [d for d in nm.derivedFeatures if d.derivedFeatureName == "Female"]
    assert len(fem) == 1 and fem[0].excluded is True and fem[0].derivedFeatureGroup == "Female"


# ------------------------------------------------------------------------------------------- stand-alone learners
@pytest.fixture(scope="module")
def xgb(fx):
    from transmogrifai_amd.models.predictors import OpXGBoostClassifier, OpXGBoostRegressor
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    c = OpXGBoostClassifier(missing=0.0, seed=42).set_input(fx.label, fx.features).get_output()
    r = OpXGBoostRegressor(missing=0.0, seed=42).set_input(fx.label, fx.features).get_output()
    model = OpWorkflow().set_result_features(c, r).set_reader(_reader()).train()
    return model, c, r


@pytest.mark.parametrize("which", [1, 2])
def test_xgboost_model_insights(fx, xgb, which):
    model, c, r = xgb
    ins = model.model_insights(c if which == 1 else r)
    assert len(ins.features) == 5 and {f.featureName for f in ins.features} == fx.rawNames
    age, gender = _by_name(ins, fx.age.name), _by_name(ins, fx.genderPL.name)
    assert len(age.derivedFeatures) == 2 and len(gender.derivedFeatures) == 4
    for f in age.derivedFeatures + gender.derivedFeatures:
        assert len(f.contribution) == 1
        assert f.corr is None and f.variance is None and f.cramersV is None


def _two_feature(x1, x2, y):
    """``ModelInsightsTest.twoFeatureDF``: two reals vectorized (mean fill, no null tracking), sanity checked
    without removals."""
    from transmogrifai_amd.readers.base import InMemoryReader
    f1 = FeatureBuilder.Real("feature1").as_predictor()
    f2 = FeatureBuilder.Real("feature2").as_predictor()
    lab = FeatureBuilder.RealNN("label").as_response()
    vec = f1.vectorize(fill_value=0, fill_with_mean=True, track_nulls=False, others=[f2])
    checked = lab.sanity_check(vec, remove_bad_features=False)
    recs = [{"feature1": float(a), "feature2": float(b), "label": float(c)} for a, b, c in zip(x1, x2, y)]
    return lab, checked, InMemoryReader(recs)


def _descaled_pair(kind, lab, checked, reader):
    from transmogrifai_amd.models.predictors import OpLinearRegression, OpLogisticRegression
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    cls = OpLinearRegression if kind == "lin" else OpLogisticRegression
    std = cls(standardization=True).set_input(lab, checked).get_output()
    raw = cls(standardization=False).set_input(lab, checked).get_output()
    model = OpWorkflow().set_result_features(std, raw).set_reader(reader).train()
    s = [d.contribution[0] for f in model.model_insights(std).features for d in f.derivedFeatures]
    u = [d.contribution[0] for f in model.model_insights(raw).features for d in f.derivedFeatures]
    return s, u


def test_descaled_coefficients_linear_regression():
    """ModelInsightsTest.scala:814-834: with standardization the contribution is coefficient * std(x) / std(y)."""
    rng = np.random.default_rng(0)
    small, big = rng.normal(0.0, 10.0, 1000), rng.normal(10000.0, 100.0, 1000)
    y = small * 5000 + big
    s, u = _descaled_pair("lin", *_two_feature(small, big, y))
    ystd = y.std()
    for desc, orig, x in ((s[0], u[0], small), (s[1], u[1], big)):
        want = orig * x.std() / ystd
        assert abs(want - desc) < 0.1 * abs(want + desc) / 2, (want, desc)


def test_descaled_coefficients_logistic_regression():
    """ModelInsightsTest.scala:836-850: with standardization the contribution is coefficient * std(x)."""
    rng = np.random.default_rng(1)
    small, med, noise = rng.normal(0.0, 10.0, 1000), rng.normal(10.0, 1.0, 1000), rng.normal(0.0, 100.0, 1000)
    y = ((small * 10 + med + noise) > 0).astype(float)
    s, u = _descaled_pair("log", *_two_feature(small, med, y))
    for desc, orig, x in ((s[0], u[0], small), (s[1], u[1], med)):
        want = orig * x.std()
        assert abs(want - desc) < 0.1 * abs(want + desc) / 2 + 1e-9, (want, desc)


def test_moments_and_cardinality_of_numeric_features():
    """ModelInsightsTest.scala:852-874: the raw feature filter's distributions carry each numeric feature's moments
    and value counts."""
    from transmogrifai_amd.models.predictors import OpLinearRegression
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    rng = np.random.default_rng(2)
    small, big = rng.normal(0.0, 10.0, 1000), rng.normal(10000.0, 100.0, 1000)
    lab, checked, reader = _two_feature(small, big, small * 5000 + big)
    pred = OpLinearRegression(standardization=True).set_input(lab, checked).get_output()
    model = OpWorkflow().set_result_features(pred).set_reader(reader).with_raw_feature_filter(reader, None).train()
    ins = model.model_insights(pred)
    data = {"feature1": small, "feature2": big}
    for f in ins.features:
        d = f.distributions[0]
        mom = d["moments"]          # Algebird Moments: m0 count, m1 mean, m2 sum of squared deviations
        assert mom["m0"] == 1000
        x = data[f.featureName]
        assert abs((mom["m1"] - x.mean()) / x.mean()) < 0.01
        assert abs((mom["m2"] / mom["m0"] - x.var(ddof=1)) / x.var(ddof=1)) < 0.01
        assert set(float(k) for k in d["cardEstimate"]["valueCounts"]) <= set(x.tolist())


@pytest.mark.parametrize("strategy", ["equal", "best"])
def test_model_combiner_insights(fx, strategy):
    from transmogrifai_amd.selector.extras import SelectedModelCombiner
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    comb = SelectedModelCombiner(combination_strategy=strategy).set_input(
        fx.label, fx.pred, fx.predWithMaps).get_output()
    model = OpWorkflow().set_result_features(fx.pred, comb).set_parameters(fx.params).set_reader(_reader()).train()
    ins = model.model_insights(comb)
    assert ins.selectedModelInfo
    if strategy == "equal":
        names = {fx.genderPL.name, fx.age.name, fx.height.name, fx.description.name, fx.weight.name,
                 fx.numericMap.name}
        assert {f.featureName for f in ins.features} == names
        for f in ins.features:
            for d in f.derivedFeatures:
                assert d.contribution == [] and d.variance is not None
    else:
        cm = model.get_origin_stage_of(comb)
        winner = fx.pred if cm.weight1 > 0.5 else fx.predWithMaps
        win = model.model_insights(winner)
        assert {f.featureName for f in ins.features} == {f.featureName for f in win.features}
        for c, w in zip(ins.features, win.features):
            for c1, w1 in zip(c.derivedFeatures, w.derivedFeatures):
                assert c1.contribution == w1.contribution


def test_default_and_custom_metrics_binary(fx):
    from transmogrifai_amd.evaluators.evaluators import Evaluators
    from transmogrifai_amd.selector.factories import BinaryClassificationModelSelector
    from transmogrifai_amd.tuning.splitters import DataSplitter
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    pred = BinaryClassificationModelSelector.with_cross_validation(
        seed=42, train_test_evaluators=[
            Evaluators.BinaryClassification.custom(metric_name="second", evaluate_fn=lambda *a: 0.0),
            Evaluators.BinaryClassification.custom(metric_name="third", evaluate_fn=lambda *a: 1.0)],
        splitter=DataSplitter(seed=42, reserve_test_fraction=0.1), models_and_parameters=fx.models).set_input(
        fx.label, fx.checked).get_output()
    model = OpWorkflow().set_result_features(pred).set_parameters(fx.params).set_reader(_reader()).train()
    te = model.model_insights(pred).selectedModelInfo["trainEvaluation"]
    assert te["second"] == 0.0 and te["third"] == 1.0
    assert "AuPR" in te and "AuROC" in te


def test_default_and_custom_metrics_regression(fx):
    from transmogrifai_amd.evaluators.evaluators import Evaluators
    from transmogrifai_amd.selector.factories import RegressionModelSelector
    from transmogrifai_amd.tuning.splitters import DataSplitter
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    pred = RegressionModelSelector.with_cross_validation(
        seed=42, train_test_evaluators=[Evaluators.Regression.custom(metric_name="second", evaluate_fn=lambda *a: 0.0)],
        splitter=DataSplitter(seed=42, reserve_test_fraction=0.1),
        models_and_parameters=[("OpLinearRegression", [{"reg_param": 0.01}, {"reg_param": 0.1}])]).set_input(
        fx.label, fx.features).get_output()
    model = OpWorkflow().set_result_features(pred).set_parameters(fx.params).set_reader(_reader()).train()
    te = model.model_insights(pred).selectedModelInfo["trainEvaluation"]
    assert te["second"] == 0.0 and "RootMeanSquaredError" in te


def test_insights_with_correlation_turned_off_for_hashed_text(fx):
    """ModelInsightsTest.scala:232-248: a sanity checker excluding hashed text from the correlations still yields
    insights for every derived column (2 raw features, 23 derived columns)."""
    from transmogrifai_amd.selector.factories import MultiClassificationModelSelector
    from transmogrifai_amd.tuning.splitters import DataCutter
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    string_map = FeatureBuilder.TextMap("stringMap").extract(lambda p: p.get("stringMap") or {}).as_predictor()
    feats = fx.description.vectorize(num_terms=10, auto_detect_language=False, min_token_length=1,
                                     to_lowercase=True).combine(string_map.vectorize(clean_text=True, num_hashes=10))
    checked = fx.label.sanity_check(feats, correlation_exclusion="HashedText")
    pred = MultiClassificationModelSelector.with_cross_validation(
        seed=42, splitter=DataCutter(seed=42, reserve_test_fraction=0.1),
        models_and_parameters=fx.models).set_input(fx.label, checked).get_output()
    model = OpWorkflow().set_result_features(pred).set_parameters(fx.params).set_reader(_reader()).train()
    ins = model.model_insights(pred)
    assert len(ins.features) == 2
    meta = model.get_origin_stage_of(feats).metadata["vector_metadata"]
    assert sum(len(f.derivedFeatures) for f in ins.features) == meta.size == 23


def test_default_and_custom_metrics_multiclass(fx):
    from transmogrifai_amd.evaluators.evaluators import Evaluators
    from transmogrifai_amd.selector.factories import MultiClassificationModelSelector
    from transmogrifai_amd.tuning.splitters import DataCutter
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    pred = MultiClassificationModelSelector.with_cross_validation(
        seed=42, train_test_evaluators=[Evaluators.MultiClassification.custom(metric_name="second",
                                                                              evaluate_fn=lambda *a: 0.0)],
        splitter=DataCutter(seed=42, reserve_test_fraction=0.1), models_and_parameters=fx.models).set_input(
        fx.label, fx.checked).get_output()
    model = OpWorkflow().set_result_features(pred).set_parameters(fx.params).set_reader(_reader()).train()
    te = model.model_insights(pred).selectedModelInfo["trainEvaluation"]
    assert te["second"] == 0.0 and "F1" in te and "Error" in te

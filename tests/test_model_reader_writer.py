"""Checkpoint writer / reader: ports of the reference's ``OpWorkflowModelReaderWriterTest.scala`` scenarios (:172-341)
on its passenger fixture (``testkit/passenger.py``).

Flows (``:113-170``): a single stage (``weight / height``), several stages with a dead branch, a raw feature only,
a wrapped library estimator (here the package's own standard scaler over a vector), and ``transmogrify()`` of every
passenger raw feature mapped to its first vector entry. The model equality helper mirrors the reference's
``assert(wfm1, wfm2)`` (:343-392): uid, parameters, train parameters, workflow-CV flag, reader, result / raw /
blocklisted features by uid, blocklisted map keys, stages in order with their inputs and outputs, raw feature filter
results. The three old-version checkpoints (:323-341) are covered by ``tests/test_model_io_compat.py``.
"""
import json
import os

import numpy as np
import pytest

from transmogrifai_amd import uid
from transmogrifai_amd.features import types as T
from transmogrifai_amd.testkit import passenger as PF
from transmogrifai_amd.workflow import io as IO
from transmogrifai_amd.workflow.params import OpParams, ReaderParams

pytestmark = pytest.mark.skipif(not PF.available(), reason="reference test data not mounted")

FIELD_NAMES = {"uid", "resultFeaturesUids", "blocklistedFeaturesUids", "blocklistedMapKeys", "blocklistedStages",
               "stages", "allFeatures", "parameters", "trainParameters", "rawFeatureFilterResults"}


def _params():
    return OpParams(stage_params={"a": {"aa": 1, "aaa": 2}, "b": {"bb": 3, "bbb": 4}},
                    reader_params={"test": ReaderParams("a", 3, {})})


def _rff_results():
    from transmogrifai_amd.filters.raw_feature_filter import FeatureDistribution, RawFeatureFilterResults
    d = [FeatureDistribution("a", None, 1, 1, np.array([1.0]), [1.0]),
         FeatureDistribution("b", "b", 2, 2, np.array([2.0]), [2.0])]
    return RawFeatureFilterResults(rawFeatureDistributions=d)


def _dummy_reader():
    from transmogrifai_amd.readers.files import DataReaders
    return DataReaders.Aggregate.avro(path="", key=lambda r: str(r["passengerId"]), aggregate_params=None)


def _dummy_model(wf):
    from transmogrifai_amd.workflow.workflow import OpWorkflowModel
    return OpWorkflowModel(wf.uid, wf.get_parameters()).set_stages(wf.get_stages()) \
        .set_features(wf.get_result_features()).set_parameters(wf.get_parameters()) \
        .set_raw_feature_filter_results(wf.get_raw_feature_filter_results()).set_reader(wf.get_reader())


def _flow(kind):
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    uid.reset(0)
    fx = PF.PassengerFeatures()
    density = fx.weight / fx.height
    if kind == "single":
        res = [density]
    elif kind == "multi":
        weight2 = density * fx.height
        _dead = fx.height * fx.height          # noqa: F841  (dead branch: not written)
        res = [density, weight2]
    else:
        res = [fx.weight]
    wf = OpWorkflow().set_reader(_dummy_reader()).set_result_features(*res).set_parameters(_params()) \
        .set_raw_feature_filter_results(_rff_results())
    m = _dummy_model(wf)
    return fx, wf, m, res, IO.model_to_json(m)


def _vectorized_flow():
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    uid.reset(0)
    fx = PF.PassengerFeatures()
    vec = transmogrify(fx.raw_features)
    cat_head = vec.map(lambda v: None if v is None or len(v) == 0 else float(v[0]), output_type=T.Real)
    wf = OpWorkflow().set_parameters(_params()).set_result_features(cat_head)
    return fx, wf, cat_head


# ----------------------------------------------------------------------------------------- equality helpers
def _same_features(a, b):
    assert len(a) == len(b)
    assert sorted(f.uid for f in a) == sorted(f.uid for f in b)


def _same_params(p1, p2):
    assert p1.stage_params == p2.stage_params
    assert {k: v.to_json() for k, v in p1.reader_params.items()} == {k: v.to_json() for k, v in p2.reader_params.items()}
    assert p1.custom_params == p2.custom_params


def _same_stages(s1, s2):
    assert len(s1) == len(s2)
    for a, b in zip(s1, s2):
        assert a.uid == b.uid
        _same_features(a.get_input_features(), b.get_input_features())
        _same_features([a.get_output()], [b.get_output()])


def _same_rff(r1, r2):
    j1 = r1.to_json() if hasattr(r1, "to_json") else r1
    j2 = r2.to_json() if hasattr(r2, "to_json") else r2
    assert json.dumps(j1, sort_keys=True, default=str) == json.dumps(j2, sort_keys=True, default=str)


def _same_model(m1, m2):
    assert m1.uid == m2.uid
    _same_params(m1.train_parameters, m2.train_parameters)
    _same_params(m1.get_parameters(), m2.get_parameters())
    assert m1.is_workflow_cv == m2.is_workflow_cv
    assert m1.get_reader() is m2.get_reader()
    _same_features(m1.get_result_features(), m2.get_result_features())
    _same_features(m1.get_raw_features(), m2.get_raw_features())
    _same_features(m1.get_blocklist(), m2.get_blocklist())
    assert m1.get_blocklist_map_keys() == m2.get_blocklist_map_keys()
    _same_stages(m1.get_stages(), m2.get_stages())
    _same_rff(m1.get_raw_feature_filter_results(), m2.get_raw_feature_filter_results())


# --------------------------------------------------------------------------------------------- writer
def test_single_stage_json_entries():
    *_, j = _flow("single")
    assert set(j) - {"trainTimings"} == FIELD_NAMES          # (trainTimings: this package's OpStep timings)


def test_single_stage_recovers_stages_features_results_uid_and_parameters():
    fx, wf, m, res, j = _flow("single")
    assert len(j["stages"]) == 3                 # two raw generators + the division
    assert len(j["allFeatures"]) == 3
    assert j["resultFeaturesUids"] == [res[0].uid]
    assert j["uid"] == wf.uid
    p = OpParams.from_string(j["parameters"])
    assert {k: v.to_json() for k, v in p.reader_params.items()} == \
        {k: v.to_json() for k, v in _params().reader_params.items()}
    assert p.stage_params == _params().stage_params


def test_multi_stage_writer_skips_the_dead_branch():
    fx, wf, m, res, j = _flow("multi")
    assert len(j["stages"]) == 4
    assert len(j["allFeatures"]) == 4
    assert sorted(j["resultFeaturesUids"]) == sorted(f.uid for f in res)


def test_raw_feature_only_writer():
    fx, wf, m, res, j = _flow("raw")
    assert len(j["stages"]) == 1
    assert len(j["allFeatures"]) == 1
    assert j["resultFeaturesUids"] == [fx.weight.uid]


# --------------------------------------------------------------------------------------------- reader
@pytest.mark.parametrize("kind", ["single", "multi", "raw"])
def test_load_workflow(tmp_path, kind):
    fx, wf, m, res, j = _flow(kind)
    m.save(str(tmp_path / "m"))
    loaded = wf.load_model(str(tmp_path / "m")).set_reader(m.get_reader())
    _same_model(loaded, m)


def test_load_workflow_with_wrapped_library_stage(tmp_path):
    from transmogrifai_amd.stages.feature.vector_scalers import OpStandardScaler
    from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
    from transmogrifai_amd.testkit.random_data import RandomReal, RandomVector
    from transmogrifai_amd.workflow.workflow import OpWorkflow, OpWorkflowModel
    uid.reset(0)
    vals = RandomVector.dense(RandomReal.uniform(-1.0, 1.0), 20).take(10)
    ds, (vec,) = TestFeatureBuilder.of(("vec", T.OPVector, vals))
    scaled = OpStandardScaler(with_std=True, with_mean=False).set_input(vec).get_output()
    wf = OpWorkflow().set_parameters(_params()).set_input_dataset(ds).set_result_features(scaled) \
        .set_raw_feature_filter_results(_rff_results())
    m = wf.train()
    m.save(str(tmp_path / "sw"))
    _same_model(wf.load_model(str(tmp_path / "sw")).set_reader(m.get_reader()), m)
    no_wf = OpWorkflowModel.load(str(tmp_path / "sw")).set_reader(m.get_reader())
    _same_model(no_wf, m)
    got = no_wf.score()[scaled.name].values
    want = m.score()[scaled.name].values
    assert np.allclose(got.cpu().numpy(), want.cpu().numpy())


def test_trained_single_stage_model_round_trip(tmp_path):
    fx, wf, m, res, j = _flow("single")
    wf.set_reader(PF.data_reader())
    model = wf.train()
    model.save(str(tmp_path / "t"))
    _same_model(model, wf.load_model(str(tmp_path / "t")).set_reader(wf.get_reader()))


def test_vectorized_model_round_trip(tmp_path):
    fx, wf, cat_head = _vectorized_flow()
    wf.set_reader(PF.data_reader())
    model = wf.train()
    model.save(str(tmp_path / "v"))
    loaded = wf.load_model(str(tmp_path / "v")).set_reader(wf.get_reader())
    _same_model(loaded, model)
    assert loaded.score()[cat_head.name].to_list() == model.score()[cat_head.name].to_list()


@pytest.fixture(scope="module")
def rff_model_dir(tmp_path_factory):
    """``:275-289``: the vectorized flow trained with a raw feature filter (training = aggregated passengers,
    scoring = per-record reader) -- the filter drops six raw features and the "Male" key of the three maps."""
    fx, wf, cat_head = _vectorized_flow()
    wf.with_raw_feature_filter(PF.data_reader(), PF.simple_reader(), bins=10, min_fill_rate=0.1,
                               max_fill_difference=0.1, max_fill_ratio_diff=2, max_js_divergence=0.2,
                               max_correlation=0.9, min_scoring_rows=0)
    model = wf.train()
    d = str(tmp_path_factory.mktemp("rff") / "model")
    model.save(d)
    return fx, wf, model, d


def test_rff_model_saves_its_blocklists(rff_model_dir):
    fx, wf, model, d = rff_model_dir
    assert sorted(f.name for f in wf.get_blocklist()) == sorted(
        f.name for f in (fx.age, fx.boarded, fx.description, fx.gender, fx.height, fx.weight))
    assert {k: set(v) for k, v in wf.get_blocklist_map_keys().items()} == \
        {"booleanMap": {"Male"}, "stringMap": {"Male"}, "numericMap": {"Male"}}
    loaded = wf.load_model(d).set_reader(model.get_reader())
    _same_model(model, loaded)


@pytest.mark.parametrize("with_workflow", [True, False])
def test_rff_model_loads_with_a_different_workflow_or_none(rff_model_dir, with_workflow):
    from transmogrifai_amd.workflow.workflow import OpWorkflowModel
    _, _, _, d = rff_model_dir
    fx, wf, cat_head = _vectorized_flow()          # a fresh workflow: no filter, every raw feature
    m = wf.load_model(d) if with_workflow else OpWorkflowModel.load(d)
    assert wf.get_result_features()[0].name == m.get_result_features()[0].name
    assert sorted(wf.get_result_features()[0].history().origin_features) == sorted(f.name for f in fx.raw_features)
    assert sorted(m.get_result_features()[0].history().origin_features) == \
        ["booleanMap", "numericMap", "stringMap", "survived"]
    assert sorted(f.name for f in m.get_blocklist()) == sorted(
        f.name for f in (fx.age, fx.boarded, fx.description, fx.gender, fx.height, fx.weight))


@pytest.mark.parametrize("with_workflow", [True, False])
def test_loaded_model_copies(rff_model_dir, with_workflow):
    from transmogrifai_amd.workflow.workflow import OpWorkflowModel
    _, _, _, d = rff_model_dir
    fx, wf, cat_head = _vectorized_flow()
    reader = PF.data_reader()
    m = (wf.load_model(d) if with_workflow else OpWorkflowModel.load(d)).set_reader(reader)
    c = m.copy().set_reader(reader)
    _same_model(c, m)

"""Workflow runner run types, OpApp flags and the project generator (``OpWorkflowRunnerTest.scala:88-200``,
``cli/src/test``)."""
import json
import os
import subprocess
import sys

import numpy as np
import pandas as pd
import pytest

from transmogrifai_amd.app import parse_args
from transmogrifai_amd.workflow.params import OpParams
from transmogrifai_amd.workflow.runner import OpWorkflowRunner, OpWorkflowRunnerConfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _csv(tmp_path, n=300):
    rng = np.random.default_rng(0)
    x = rng.normal(size=n)
    df = pd.DataFrame({"id": range(n), "x": x, "c": rng.choice(["u", "v"], n),
                       "y": (x + rng.normal(scale=0.5, size=n) > 0).astype(int)})
    p = tmp_path / "d.csv"
    df.to_csv(p, index=False)
    return str(p)


def _wf():
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.evaluators.evaluators import Evaluators
    from transmogrifai_amd.features.builder import FeatureBuilder
    from transmogrifai_amd.selector.factories import BinaryClassificationModelSelector
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    y = FeatureBuilder.RealNN("y").as_response()
    x = FeatureBuilder.Real("x").as_predictor()
    c = FeatureBuilder.PickList("c").as_predictor()
    vec = transmogrify([x, c])
    pred = BinaryClassificationModelSelector.with_train_validation_split(
        model_types_to_use=["OpLogisticRegression"], seed=1).set_input(y, vec).get_output()
    ev = Evaluators.BinaryClassification().set_label_col(y).set_prediction_col(pred)
    return OpWorkflow().set_result_features(y, pred), ev, vec


def test_runner_all_run_types(tmp_path):
    from transmogrifai_amd.readers.files import DataReaders
    from transmogrifai_amd.readers.streaming import IterableStreamingReader
    path = _csv(tmp_path)
    wf, ev, vec = _wf()
    reader = DataReaders.Simple.csv_auto(path, key=lambda r: r["id"])
    recs = pd.read_csv(path).to_dict("records")
    runner = OpWorkflowRunner(wf, training_reader=reader, scoring_reader=reader, evaluation_reader=reader,
                              streaming_score_reader=IterableStreamingReader(recs, 100), evaluator=ev,
                              scoring_evaluator=ev, feature_to_compute_up_to=vec)
    p = OpParams(model_location=str(tmp_path / "model"), write_location=str(tmp_path / "scores"),
                 metrics_location=str(tmp_path / "metrics"), collect_stage_metrics=True)
    tr = runner.run("train", p)
    assert os.path.isdir(tmp_path / "model" / "op-model.json")
    assert json.load(open(tmp_path / "metrics" / "summary.json"))
    assert tr.metrics.appDurationSecs > 0
    sc = runner.run("Score", p)
    assert os.path.isfile(tmp_path / "scores" / "part-00000.parquet")
    assert sc.evaluation["AuROC"] > 0.7
    evr = runner.run("evaluate", p)
    assert json.load(open(tmp_path / "metrics" / "metrics.json"))["AuPR"] > 0.5
    p2 = p.with_values(write_location=str(tmp_path / "feats"))
    fr = runner.run("features", p2)
    assert vec.name in fr.data
    p3 = p.with_values(write_location=str(tmp_path / "stream"))
    st = runner.run("streamingscore", p3)
    assert st.batches == 3 and len(os.listdir(tmp_path / "stream")) == 3
    with pytest.raises(ValueError):
        runner.run("train", OpParams())


def test_op_app_flags(tmp_path):
    cfg = parse_args(["-t", "score", "-r", "data=/tmp/x.csv", "-m", "m", "-w", "w"])
    p = cfg.to_op_params()
    assert cfg.run_type == "Score" and p.model_location == "m" and p.reader_params["data"].path == "/tmp/x.csv"
    cfg.validate(p)
    with pytest.raises(ValueError):
        OpWorkflowRunnerConfig(run_type="Evaluate").validate(p)


def test_params_yaml(tmp_path):
    y = tmp_path / "p.yaml"
    y.write_text("stageParams:\n  TestClass1:\n    param1: 11\nreaderParams:\n  Passenger: {}\ncustomTagName: myTag\n"
                 "customParams:\n  custom1: 1\n")
    p = OpParams.from_file(str(y))
    assert p.stage_params["TestClass1"]["param1"] == 11 and p.custom_tag_name == "myTag"
    assert OpParams.from_string(p.to_string()).custom_params == {"custom1": 1}


def test_project_generator_runs(tmp_path):
    from transmogrifai_amd.cli.gen import generate
    path = _csv(tmp_path)
    d = generate(path, "y", "id", "Demo", str(tmp_path / "out"))
    assert os.path.isfile(os.path.join(d, "demo", "app.py"))
    env = dict(os.environ, PYTHONPATH=f"{ROOT}:{d}")
    r = subprocess.run([sys.executable, "-m", "demo.app", "-t", "train", "-p", os.path.join(d, "params.json"),
                        "-m", str(tmp_path / "gm"), "-x", str(tmp_path / "gx")], env=env, cwd=d,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert os.path.isdir(tmp_path / "gm" / "op-model.json")
    with pytest.raises(FileExistsError):
        generate(path, "y", "id", "Demo", str(tmp_path / "out"))


def test_runner_collects_stage_metrics(tmp_path):
    """AppMetrics carries per-stage metrics like OpSparkListener's StageMetrics / CumulativeStageMetrics."""
    import json
    from transmogrifai_amd.readers.base import InMemoryReader
    from transmogrifai_amd.testkit.synthetic import binary_table
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.selector.factories import BinaryClassificationModelSelector
    from transmogrifai_amd.workflow.params import OpParams
    from transmogrifai_amd.workflow.runner import OpWorkflowRunner
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    ds, label, preds = binary_table(2000, n_real=4, n_int=1, n_pick=1, seed=2)
    vec = transmogrify(preds)
    pred = BinaryClassificationModelSelector.with_cross_validation(
        num_folds=2, seed=1, model_types_to_use=["OpLogisticRegression"]).set_input(label, vec).get_output()
    wf = OpWorkflow().set_result_features(label, pred)
    runner = OpWorkflowRunner(wf, training_reader=InMemoryReader(ds))
    params = OpParams(model_location=str(tmp_path / "m"), metrics_location=str(tmp_path / "x"),
                      collect_stage_metrics=True, log_stage_metrics=True)
    res = runner.run("train", params)
    sm = res.metrics.stageMetrics
    names = {s["stageName"].split("_")[0] for s in sm}
    assert {"vecReal", "combVec", "modelSelection"} <= names
    assert all(s["durationSecs"] >= 0 and s["numRows"] > 0 for s in sm)
    assert {s["phase"] for s in sm} == {"fit", "transform"}
    assert any(s["jobGroup"] == "FeatureEngineering" for s in sm)
    cum = res.metrics.cumulativeStageMetrics
    assert cum["numStages"] == len(sm)
    saved = json.load(open(tmp_path / "x" / "app_metrics.json"))
    assert saved["versionInfo"]["version"] and len(saved["stageMetrics"]) == len(sm)

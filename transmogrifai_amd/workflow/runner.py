"""Workflow runner: train / score / streaming score / features / evaluate entry points.

Reference: ``OpWorkflowRunner`` (``core/.../op/OpWorkflowRunner.scala:70-459``: run types ``:358-366``, config
validation ``:424-440``, per-run-type behaviour ``:163-285``), ``OpWorkflowRunnerConfig`` (``:379-417``) and the
Spark listener metrics (``utils/.../OpSparkListener.scala:62-418``) -- here :class:`AppMetrics` records
the wall-clock of every ``OpStep`` phase plus device memory high-water marks instead of Spark
executor metrics.
"""
from __future__ import annotations

import json
import os
import time
from dataclasses import asdict, dataclass, field
from typing import Any, Callable, Dict, Iterable, List, Optional

import torch

from .params import OpParams, ReaderParams


class OpWorkflowRunType:
    Train = "Train"
    Score = "Score"
    StreamingScore = "StreamingScore"
    Features = "Features"
    Evaluate = "Evaluate"
    values = (Train, Score, StreamingScore, Features, Evaluate)

    @staticmethod
    def with_name_insensitive(name: str) -> str:
        for v in OpWorkflowRunType.values:
            if v.lower() == str(name).lower():
                return v
        raise ValueError(f"unknown run type {name}; expected one of {OpWorkflowRunType.values}")


@dataclass
class AppMetrics:
    """Run metrics (the ``AppMetrics`` collected by ``OpSparkListener``)."""
    appName: str
    runType: str
    appStartTime: float
    appEndTime: float = 0.0
    appDurationSecs: float = 0.0
    stepTimings: Dict[str, Any] = field(default_factory=dict)
    deviceMaxMemoryBytes: Optional[int] = None
    stageMetrics: List[Dict[str, Any]] = field(default_factory=list)
    cumulativeStageMetrics: Dict[str, Any] = field(default_factory=dict)
    versionInfo: Dict[str, Any] = field(default_factory=dict)
    customTagName: Optional[str] = None
    customTagValue: Optional[str] = None

    def to_json(self) -> Dict:
        return asdict(self)


@dataclass
class OpWorkflowRunnerResult:
    run_type: str
    metrics: AppMetrics


@dataclass
class TrainResult(OpWorkflowRunnerResult):
    model: Any = None
    model_summary: Optional[Dict] = None


@dataclass
class ScoreResult(OpWorkflowRunnerResult):
    scores: Any = None
    evaluation: Optional[Dict] = None


@dataclass
class FeaturesResult(OpWorkflowRunnerResult):
    data: Any = None


@dataclass
class EvaluateResult(OpWorkflowRunnerResult):
    evaluation: Optional[Dict] = None


@dataclass
class StreamingScoreResult(OpWorkflowRunnerResult):
    batches: int = 0


@dataclass
class OpWorkflowRunnerConfig:
    """Command-line configuration merged into :class:`OpParams` (``OpWorkflowRunnerConfig``, ``:379-417``)."""
    run_type: Optional[str] = None
    default_params: OpParams = field(default_factory=OpParams)
    param_location: Optional[str] = None
    read_locations: Dict[str, str] = field(default_factory=dict)
    write_location: Optional[str] = None
    model_location: Optional[str] = None
    metrics_location: Optional[str] = None

    def to_op_params(self) -> OpParams:
        p = OpParams.from_file(self.param_location) if self.param_location else self.default_params
        p = p.with_values(write_location=self.write_location, model_location=self.model_location,
                          metrics_location=self.metrics_location)
        for k, loc in self.read_locations.items():
            rp = p.reader_params.get(k) or ReaderParams()
            rp = ReaderParams(loc, rp.partitions, dict(rp.custom_params))
            p.reader_params[k] = rp
        return p

    def validate(self, params: OpParams) -> None:
        rt = self.run_type
        if rt is None:
            raise ValueError("Run type must be specified")
        if rt == OpWorkflowRunType.Train and not params.model_location:
            raise ValueError("Must provide location to store model when training")
        if rt in (OpWorkflowRunType.Score, OpWorkflowRunType.StreamingScore) and (
                not params.model_location or not params.write_location):
            raise ValueError("Must provide locations to read model and write data when scoring")
        if rt == OpWorkflowRunType.Features and not params.write_location:
            raise ValueError("Must provide location to write data when generating features")
        if rt == OpWorkflowRunType.Evaluate and (not params.model_location or not params.metrics_location):
            raise ValueError("Must provide locations to read model and write metrics when evaluating")


def _write_json(path: str, obj) -> None:
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    with open(path, "w") as f:
        json.dump(obj, f, indent=2, default=_default)


def _default(o):
    import numpy as np
    if isinstance(o, (np.floating, np.integer)):
        return o.item()
    if isinstance(o, (np.ndarray, torch.Tensor)):
        return o.tolist()
    if hasattr(o, "to_json"):
        return o.to_json()
    return str(o)


def save_dataset(ds, path: str, fmt: str = "parquet") -> str:
    """Write a scored / computed dataset (key + columns) as Parquet, CSV, Avro or JSON lines."""
    os.makedirs(path, exist_ok=True)
    df = ds.to_pandas()
    for c in df.columns:
        if df[c].map(lambda v: isinstance(v, (dict, list, set, frozenset)) or hasattr(v, "tolist")).any():
            df[c] = df[c].map(lambda v: json.dumps(v, default=_default) if v is not None else None)
    if fmt == "parquet":
        out = os.path.join(path, "part-00000.parquet")
        df.to_parquet(out, index=False)
    elif fmt == "csv":
        out = os.path.join(path, "part-00000.csv")
        df.to_csv(out, index=False)
    elif fmt == "avro":
        # the reference's default score format (Avro container, deflate); complex values JSON-encoded
        from ..readers.avro import write_avro
        import numpy as np
        fields, conv = [], []
        for c in df.columns:
            num = df[c].map(lambda v: v is None or isinstance(v, (int, float, bool, np.integer, np.floating))).all()
            fields.append({"name": str(c), "type": ["null", "double" if num else "string"], "default": None})
            conv.append(num)
        recs = []
        for row in df.itertuples(index=False):
            r = {}
            for f, num, v in zip(fields, conv, row):
                if v is None or (isinstance(v, float) and v != v):
                    r[f["name"]] = None
                else:
                    r[f["name"]] = float(v) if num else str(v)
            recs.append(r)
        out = os.path.join(path, "part-00000.avro")
        write_avro(out, {"type": "record", "name": "OpScores", "fields": fields}, recs)
    else:
        out = os.path.join(path, "part-00000.json")
        df.to_json(out, orient="records", lines=True)
    return out


class OpWorkflowRunner:
    def __init__(self, workflow, training_reader=None, scoring_reader=None, evaluation_reader=None,
                 streaming_score_reader=None, evaluator=None, scoring_evaluator=None,
                 feature_to_compute_up_to=None, app_name: str = "OpWorkflowRunner", output_format: str = "parquet"):
        self.workflow = workflow
        self.training_reader = training_reader
        self.scoring_reader = scoring_reader
        self.evaluation_reader = evaluation_reader
        self.streaming_score_reader = streaming_score_reader
        self.evaluator = evaluator
        self.scoring_evaluator = scoring_evaluator
        self.feature_to_compute_up_to = feature_to_compute_up_to
        self.app_name = app_name
        self.output_format = output_format

    # ------------------------------------------------------------------------------------ run types
    def _train(self, params: OpParams, m: AppMetrics) -> TrainResult:
        if self.training_reader is not None:
            self.workflow.set_reader(self.training_reader)
        self.workflow.set_parameters(params)
        model = self.workflow.train(params)
        t0 = time.time()
        model.save(params.model_location)
        m.stepTimings["ModelIO"] = time.time() - t0
        summary = model.summary_json()
        if params.metrics_location:
            _write_json(os.path.join(params.metrics_location, "summary.json"), summary)
            try:
                _write_json(os.path.join(params.metrics_location, "insights.json"),
                            model.model_insights().to_json_dict())
            except Exception:     # models without a selector still train fine
                pass
        m.stepTimings.update({k: v for k, v in model.train_timings.items() if not isinstance(v, dict)})
        return TrainResult(OpWorkflowRunType.Train, m, model, summary)

    def _load(self, params: OpParams):
        model = self.workflow.load_model(params.model_location)
        model.parameters = params
        return model

    def _score(self, params: OpParams, m: AppMetrics) -> ScoreResult:
        model = self._load(params)
        if self.scoring_reader is not None:
            model.set_reader(self.scoring_reader)
        t0 = time.time()
        ev = self.scoring_evaluator
        if ev is not None:
            scores, metrics = model.score_and_evaluate(ev)
        else:
            scores, metrics = model.score(), None
        m.stepTimings["Scoring"] = time.time() - t0
        t0 = time.time()
        save_dataset(scores, params.write_location, self.output_format)
        if metrics is not None and params.metrics_location:
            _write_json(os.path.join(params.metrics_location, "scoring_metrics.json"), metrics)
        m.stepTimings["ResultsSaving"] = time.time() - t0
        return ScoreResult(OpWorkflowRunType.Score, m, scores, metrics)

    def _streaming_score(self, params: OpParams, m: AppMetrics) -> StreamingScoreResult:
        """Score each micro-batch of the streaming reader (``OpWorkflowRunner.scala:232-263``)."""
        if self.streaming_score_reader is None:
            raise ValueError("Streaming score reader must be defined")
        model = self._load(params)
        n = 0
        for batch in self.streaming_score_reader.stream(params):
            t_ms = int(time.time() * 1000)
            from ..readers.base import InMemoryReader
            model.set_reader(InMemoryReader(batch))
            scores = model.score()
            save_dataset(scores, os.path.join(params.write_location, str(t_ms) + f"_{n}"), self.output_format)
            n += 1
        return StreamingScoreResult(OpWorkflowRunType.StreamingScore, m, n)

    def _features(self, params: OpParams, m: AppMetrics) -> FeaturesResult:
        if self.feature_to_compute_up_to is None:
            raise ValueError("Must provide a feature to compute up to")
        if self.training_reader is not None:
            self.workflow.set_reader(self.training_reader)
        data = self.workflow.compute_data_up_to(self.feature_to_compute_up_to, params)
        save_dataset(data, params.write_location, self.output_format)
        return FeaturesResult(OpWorkflowRunType.Features, m, data)

    def _evaluate(self, params: OpParams, m: AppMetrics) -> EvaluateResult:
        if self.evaluator is None:
            raise ValueError("Evaluator must be defined")
        model = self._load(params)
        if self.evaluation_reader is not None:
            model.set_reader(self.evaluation_reader)
        scores, metrics = model.score_and_evaluate(self.evaluator)
        _write_json(os.path.join(params.metrics_location, "metrics.json"), metrics)
        if params.write_location:
            save_dataset(scores, params.write_location, self.output_format)
        return EvaluateResult(OpWorkflowRunType.Evaluate, m, metrics)

    def run(self, run_type: str, params: OpParams) -> OpWorkflowRunnerResult:
        rt = OpWorkflowRunType.with_name_insensitive(run_type)
        OpWorkflowRunnerConfig(run_type=rt).validate(params)
        m = AppMetrics(self.app_name, rt, time.time(), customTagName=params.custom_tag_name,
                       customTagValue=params.custom_tag_value)
        if torch.cuda.is_available():
            torch.cuda.reset_peak_memory_stats()
        fn = {OpWorkflowRunType.Train: self._train, OpWorkflowRunType.Score: self._score,
              OpWorkflowRunType.StreamingScore: self._streaming_score, OpWorkflowRunType.Features: self._features,
              OpWorkflowRunType.Evaluate: self._evaluate}[rt]
        from ..utils import listener as LS
        from ..utils.version import version_info
        lst = LS.OpDeviceListener(self.app_name, rt, params.custom_tag_name, params.custom_tag_value,
                                  bool(params.log_stage_metrics), params.collect_stage_metrics is not False)
        with LS.listening(lst):
            res = fn(params, m)
        lj = lst.to_json()
        m.stageMetrics, m.cumulativeStageMetrics = lj["stageMetrics"], lj["cumulativeStageMetrics"]
        m.versionInfo = version_info().to_dict()
        m.appEndTime = time.time()
        m.appDurationSecs = m.appEndTime - m.appStartTime
        if torch.cuda.is_available():
            m.deviceMaxMemoryBytes = int(torch.cuda.max_memory_allocated())
        if params.metrics_location and (params.log_stage_metrics or params.collect_stage_metrics):
            _write_json(os.path.join(params.metrics_location, "app_metrics.json"), m.to_json())
        return res

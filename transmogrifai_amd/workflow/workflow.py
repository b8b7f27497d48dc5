"""``OpWorkflow`` (train) and ``OpWorkflowModel`` (score / evaluate / summarize / save / load).

Reference: ``OpWorkflowCore`` (``core/.../OpWorkflowCore.scala:53-361``), ``OpWorkflow`` (``OpWorkflow.scala:61-592``:
``setResultFeatures:90-110``, parameter injection ``:179-201``, validation ``:331-338``, ``train:347-365``,
``fitStages:376-455``, ``withRawFeatureFilter:537-578``) and ``OpWorkflowModel`` (``OpWorkflowModel.scala:60-473``:
``score:259-273``, ``scoreAndEvaluate:296-314``, ``summaryJson/summary/summaryPretty:187-215``,
``modelInsights:167-180``, ``save:223-225``, ``load:470-471``).
"""
from __future__ import annotations

import json
import logging
import threading
import os
import time
from typing import Dict, List, Optional, Sequence

import torch

from ..data.dataset import Dataset
from ..features.feature import FeatureLike
from ..stages.base import OpEstimator, OpPipelineStage
from ..stages.generator import FeatureGeneratorStage
from ..uid import make_uid
from .dag import apply_transformations_dag, compute_dag, cut_dag, fit_and_transform_dag
from .params import OpParams

log = logging.getLogger(__name__)


class OpStep:
    """Job-phase labels (``utils/.../spark/OpStep.scala:35-46``) used for run metrics."""
    DataReadingAndFiltering = "DataReadingAndFiltering"
    FeatureEngineering = "FeatureEngineering"
    CrossValidation = "CrossValidation"
    # the selected model's refit on the whole prepared training set and its training evaluation (inside the
    # selector's fit, after CrossValidation; Spark charges it to FeatureEngineering's job group -- timed apart here so
    # FeatureEngineering is the feature stages alone)
    ModelRefit = "ModelRefit"
    ModelIO = "ModelIO"
    Scoring = "Scoring"
    ResultsSaving = "ResultsSaving"


class _Timer:
    """Wall time of a workflow step (``OpStep``) into ``sink``; the step is also the job group of the stage
    metrics an active listener collects meanwhile (``utils/listener.py``). Steps nest: a step opened inside
    another (the model selector's ``CrossValidation`` inside ``FeatureEngineering``) is charged to itself
    only, as Spark's job groups are (ModelSelector.scala:148,207)."""

    _local = threading.local()

    def __init__(self, sink: Dict[str, float], name: str):
        self.sink, self.name = sink, name

    @classmethod
    def _stack(cls) -> list:
        st = getattr(cls._local, "stack", None)
        if st is None:
            st = cls._local.stack = []
        return st

    def __enter__(self):
        from ..utils import listener as L
        self.t = time.time()
        self.child = 0.0
        self.jg = L.job_group(str(self.name))
        self.jg.__enter__()
        self._stack().append(self)

    def __exit__(self, *a):
        self.jg.__exit__(*a)
        st = self._stack()
        st.pop()
        dt = time.time() - self.t
        self.sink[self.name] = self.sink.get(self.name, 0.0) + dt - self.child
        if st:
            st[-1].child += dt


def step(name: str):
    """A nested ``OpStep`` timer charged to the innermost open workflow step's timings (no-op outside a
    workflow fit)."""
    st = _Timer._stack()
    if not st:
        from contextlib import nullcontext
        return nullcontext()
    return _Timer(st[-1].sink, name)


class _DeferFullGC:
    """Defer the cyclic collector's full (generation-2) passes while a train runs: each re-traverses every
    object alive in the process (~0.1-0.18 s with torch loaded, every third headline train: ``bench.py``
    ``gc_s``). Young-generation collections still run; the thresholds are restored when the train ends, so the
    deferred full pass happens at the next collection after it. ``TMOG_GC_DEFER=0`` disables."""

    def __enter__(self):
        import gc
        self.prev = gc.get_threshold() if os.environ.get("TMOG_GC_DEFER", "1") != "0" else None
        if self.prev is not None:
            gc.set_threshold(self.prev[0], self.prev[1], 1 << 30)
        return self

    def __exit__(self, *a):
        if self.prev is not None:
            import gc
            gc.set_threshold(*self.prev)
        return False


class OpWorkflowCore:
    def __init__(self, uid: Optional[str] = None):
        self.uid = uid or make_uid("OpWorkflow")
        self.result_features: List[FeatureLike] = []
        self.raw_features: List[FeatureLike] = []
        self.blocklist: List[FeatureLike] = []
        self.blocklist_map_keys: Dict[str, List[str]] = {}
        self.stages: List[OpPipelineStage] = []
        self.parameters = OpParams()
        self.reader = None
        self.input_dataset = None
        self.raw_feature_filter_results = None
        self.workflow_cv = False
        self.timings: Dict[str, float] = {}

    def set_reader(self, reader):
        self.reader = reader
        return self

    def set_input_dataset(self, data, key=None):
        """Records, a pandas DataFrame or a columnar :class:`Dataset` (``setInputDataset``)."""
        from ..readers.base import InMemoryReader
        self.reader = InMemoryReader(data, key)
        return self

    set_input_rdd = set_input_dataset

    def with_workflow_cv(self):
        self.workflow_cv = True
        return self

    @property
    def is_workflow_cv(self) -> bool:
        return self.workflow_cv

    def set_raw_feature_filter_results(self, results) -> "OpWorkflowCore":
        self.raw_feature_filter_results = results
        return self

    def get_parameters(self) -> OpParams:
        return self.parameters

    # ``OpWorkflowCore`` getters (OpWorkflowCore.scala:128-214)
    def get_result_features(self) -> List[FeatureLike]:
        return list(self.result_features)

    def get_stages(self) -> List[OpPipelineStage]:
        return list(self.stages)

    def get_raw_features(self) -> List[FeatureLike]:
        return list(self.raw_features)

    def get_blocklist(self) -> List[FeatureLike]:
        return list(self.blocklist)

    def get_blocklist_map_keys(self) -> Dict[str, List[str]]:
        return dict(self.blocklist_map_keys)

    def get_reader(self):
        return self.reader

    def get_raw_feature_filter_results(self):
        return self.raw_feature_filter_results

    def get_raw_feature_distributions(self) -> list:
        r = self.raw_feature_filter_results
        return list(getattr(r, "rawFeatureDistributions", None) or [])

    def get_raw_training_feature_distributions(self) -> list:
        return [d for d in self.get_raw_feature_distributions() if getattr(d, "type", "Training") == "Training"]

    def get_raw_scoring_feature_distributions(self) -> list:
        return [d for d in self.get_raw_feature_distributions() if getattr(d, "type", "Training") == "Scoring"]

    def get_updated_features(self, features: Sequence[FeatureLike]) -> List[FeatureLike]:
        """The workflow's current version of each feature (by uid): after a blocklist rewired the stages, the
        caller's old handles map to the rebuilt features (``OpWorkflowCore.getUpdatedFeatures``)."""
        known = {}
        for f in self.result_features:
            for x in f.traverse():
                known.setdefault(x.uid, x)
        for f in self.raw_features:
            known.setdefault(f.uid, f)
        out = []
        for f in features:
            if f.uid not in known:
                raise ValueError(f"feature {f.name} ({f.uid}) is not part of this workflow")
            out.append(known[f.uid])
        return out

    def generate_raw_data(self, params: Optional[OpParams] = None) -> Dataset:
        if self.reader is None:
            raise ValueError("Data reader must be set (set_reader or set_input_dataset)")
        rp = self.reader.reader_params_of(params) if hasattr(self.reader, "reader_params_of") else None
        raws = [f for f in self.raw_features if f not in self.blocklist]
        ds = self.reader.generate_dataset(raws, rp)
        return ds


class OpWorkflow(OpWorkflowCore):
    def set_result_features(self, *features) -> "OpWorkflow":
        fs = []
        for f in features:
            fs.extend(f if isinstance(f, (list, tuple)) else [f])
        self.result_features = fs
        dag = compute_dag(fs)
        self.stages = [st for layer in dag for st, _ in layer]
        raws = {}
        for f in fs:
            for r in f.raw_features():
                raws[r.uid] = r
        self.raw_features = sorted(raws.values(), key=lambda f: f.name)
        self._validate_stages()
        return self

    def _validate_stages(self):
        uids = [s.uid for s in self.stages]
        if len(uids) != len(set(uids)):
            dup = sorted({u for u in uids if uids.count(u) > 1})
            raise ValueError(f"Duplicate stage uids in workflow: {dup}")

    def set_parameters(self, params: OpParams) -> "OpWorkflow":
        """Inject ``stageParams`` by stage class simple name or uid (``OpWorkflow.scala:179-201``)."""
        self.parameters = params
        for st in self.stages:
            for key in (type(st).__name__, st.uid):
                for k, v in (params.stage_params.get(key) or {}).items():
                    name = _snake(k)
                    if name in st.params or st._accepts_param(name):
                        st.set(name, v)
                    elif hasattr(st, name):
                        setattr(st, name, v)
                    else:
                        raise ValueError(f"stage {st.uid} has no param '{k}'")
        return self

    def with_raw_feature_filter(self, training_reader=None, scoring_reader=None, **kw) -> "OpWorkflow":
        """Attach a :class:`RawFeatureFilter` (``OpWorkflow.withRawFeatureFilter``, ``OpWorkflow.scala:537-578``)."""
        from ..filters.raw_feature_filter import RawFeatureFilter
        training = training_reader or self.reader
        if training is None:
            raise ValueError("Reader for training data must be provided either in with_raw_feature_filter or "
                             "directly as the reader for the workflow")
        self.rff = RawFeatureFilter(training, scoring_reader, **kw)
        if self.reader is None:
            self.reader = training
        return self

    def set_blocklist(self, features: Sequence[FeatureLike], distributions=()) -> None:
        """Remove blocklisted raw features from every stage's inputs and rebuild the DAG
        (``OpWorkflow.setBlocklist``, ``OpWorkflow.scala:118-168``)."""
        policy = getattr(getattr(self, "rff", None), "result_feature_retention_policy", "Strict")
        self.blocklist = list(features)
        if not self.blocklist:
            return
        blocked: List[FeatureLike] = list(self.blocklist)
        updated: List[FeatureLike] = []
        initial_results = list(self.result_features)

        def check_results():
            if policy == "Strict":
                for f in initial_results:
                    if any(b.same_origin(f) for b in blocked):
                        raise ValueError(f"Blocklist of features ({', '.join(b.name for b in blocked)}) from "
                                         f"RawFeatureFilter contained the result feature {f.name}")
            elif policy == "AtLeastOne":
                if all(any(b.same_origin(f) for b in blocked) for f in initial_results):
                    raise ValueError("Blocklist of features from RawFeatureFilter removed all result features")
            else:
                raise ValueError(f"result feature retention policy {policy} not supported")

        check_results()
        dist_by_name: Dict[str, list] = {}
        for d in distributions or ():
            dist_by_name.setdefault(d.name, []).append(d)
        for stg in list(self.stages):
            ins = [f for f in stg.get_input_features() if not any(b.same_origin(f) for b in blocked)]
            ins = [f.with_distributions(dist_by_name.get(f.name, [])) if f.is_raw else f for f in ins]
            ins = [next((u for u in updated if u.same_origin(f)), f) for f in ins]
            old = stg.get_output()
            try:
                if not ins:
                    raise ValueError("no inputs left")
                out = stg.set_input(*ins).set_output_feature_name(old.name).get_output()
                updated.append(out)
            except Exception as e:   # the stage cannot run without the blocklisted inputs
                log.info("Issue updating inputs for stage %s: %s", stg, e)
                blocked.append(old)
                check_results()
        new_results = [next((u for u in updated if u.same_origin(f)), f) for f in initial_results
                       if not any(b.same_origin(f) for b in blocked)]
        self.set_result_features(*new_results)

    def generate_raw_data(self, params: Optional[OpParams] = None) -> Dataset:
        """The reader's raw data; with a raw feature filter, its cleaned data -- the filter's dropped features are
        blocklisted (stages rewired) and its results recorded (``OpWorkflow.generateRawData``,
        ``OpWorkflow.scala:225-262``)."""
        raw = super().generate_raw_data(params)
        if getattr(self, "rff", None) is None:
            return raw
        pp = params or self.parameters
        tr = getattr(self.rff, "training_reader", None) or self.reader
        rp = tr.reader_params_of(pp) if hasattr(tr, "reader_params_of") else None
        raw, to_drop, drop_keys, results = self.rff.generate_filtered_raw(self.raw_features, rp, raw)
        self.raw_feature_filter_results = results
        self.set_blocklist(to_drop, results.rawFeatureDistributions)
        self.blocklist_map_keys = {k: sorted(v) for k, v in drop_keys.items()}
        return raw

    def train(self, params: Optional[OpParams] = None) -> "OpWorkflowModel":
        with _DeferFullGC():
            return self._train(params)

    def _train(self, params: Optional[OpParams] = None) -> "OpWorkflowModel":
        timings: Dict[str, float] = {}
        # every train does its own text work: the batch text results (utils/text.py) are shared between the
        # fits and transforms of one train, never carried over from an earlier train of the same data
        from ..utils import text as _text
        _text.clear_batch_cache()
        t0 = time.time()
        with _Timer(timings, OpStep.DataReadingAndFiltering):
            raw = self.generate_raw_data(params or self.parameters)
        box = [raw]
        del raw     # handed over: released once split into train / hold-out
        fitted = self.fit_stages(box, timings)
        model = OpWorkflowModel(self.uid, self.parameters)
        model.stages = fitted
        model.result_features = list(self.result_features)
        model.raw_features = list(self.raw_features)
        model.blocklist = list(self.blocklist)
        model.blocklist_map_keys = dict(self.blocklist_map_keys)
        model.raw_feature_filter_results = self.raw_feature_filter_results or _empty_rff_results()
        model.reader = self.reader
        model.train_parameters = self.parameters
        timings["total"] = time.time() - t0
        model.train_timings = timings
        return model

    def _holdout_split(self, data: Dataset):
        from ..selector.model_selector import ModelSelector
        sps = [s.splitter for s in self.stages if isinstance(s, ModelSelector) and s.splitter is not None]
        if not sps:
            return data, None
        sp = max(sps, key=lambda s: s.reserve_test_fraction)
        if sp.reserve_test_fraction <= 0:
            return data, None
        tr, te = sp.split(data.row_ids)
        ti = torch.nonzero(tr).reshape(-1)
        hi = torch.nonzero(te).reshape(-1)
        return data.take(ti), data.take(hi)

    def fit_stages(self, data, timings: Dict[str, float]) -> List[OpPipelineStage]:
        """Fit every stage on ``data`` (a Dataset, or a one-element list handing the dataset over so the
        raw table can be released once it is split into train / hold-out)."""
        from ..parallel import dp
        box = data if isinstance(data, list) else [data]
        # a row-sharded input (Dataset.shard, one shard per rank) fits data-parallel: every estimator
        # reduces its statistics over the process group (parallel/dp.py)
        with dp.scope(getattr(box[0], "sharded", False)):
            return self._fit_stages(box, timings)

    def _fit_stages(self, box: list, timings: Dict[str, float]) -> List[OpPipelineStage]:
        with _Timer(timings, "HoldoutSplit"):
            split = list(self._holdout_split(box.pop()))     # handed to the DAG executor below
        # stages by uid: with_model_stages swaps fitted models in for their estimators
        by_uid = {s.uid: s for s in self.stages}
        dag = [[(by_uid[st.uid], d) for st, d in layer if st.uid in by_uid]
               for layer in compute_dag(self.result_features)]
        dag = [l for l in dag if l]
        stage_t: Dict[str, float] = {}
        if not self.workflow_cv:
            with _Timer(timings, OpStep.FeatureEngineering):
                _, _, fitted = fit_and_transform_dag(dag, split, None, stage_t, keep=set())
        else:
            ms, before, during, after = cut_dag(dag)
            if ms is None:          # no selector: the whole DAG is fitted as usual
                before = dag
            later = {f.name for part in (during, after) for layer in part for st, _ in layer
                     for f in st.get_input_features()}
            if ms is not None:
                later |= {f.name for f in ms.get_input_features()}
            with _Timer(timings, OpStep.FeatureEngineering):
                tr2, te2, fb = fit_and_transform_dag(before, split, None, stage_t, keep=later)
            fitted = list(fb)
            if ms is not None:
                # OpWorkflow.scala:403-453: validate with the during-DAG refit inside every fold, then fit
                # the during stages on the whole training split and refit the selected model on their output
                with _Timer(timings, OpStep.CrossValidation):
                    ms.find_best_estimator(tr2, during)
                rest = list(during) + [[(ms, 0)]] + list(after)
                with _Timer(timings, OpStep.FeatureEngineering):
                    _, _, fr = fit_and_transform_dag(rest, tr2, te2, stage_t, keep=set())
                fitted += fr
        timings["stages"] = stage_t
        return fitted

    def compute_data_up_to(self, feature: FeatureLike, params: Optional[OpParams] = None) -> Dataset:
        """Raw data plus every feature up to and including ``feature`` (``OpWorkflow.scala:491-504``)."""
        raw = self.generate_raw_data(params or self.parameters)
        if feature.is_raw:
            return raw
        out, _, _ = fit_and_transform_dag(compute_dag([feature]), raw, None)
        return out

    def load_model(self, path: str) -> "OpWorkflowModel":
        from .io import load_model
        m = load_model(path, self)
        m.reader = self.reader
        return m

    def with_model_stages(self, model: "OpWorkflowModel") -> "OpWorkflow":
        """Add a fitted model's result features and reuse its fitted stages: training then fits only the stages
        the model does not hold (``OpWorkflow.withModelStages``, ``OpWorkflow.scala:468-472``)."""
        fitted = {s.uid: s for s in model.stages}
        own = list(self.result_features)
        ids = {f.uid for f in own}
        results = _copy_with_new_stages(own + [f for f in model.result_features if f.uid not in ids], fitted)
        self.set_result_features(*results)
        return self


class OpWorkflowModel(OpWorkflowCore):
    PersistEveryKStages = 5

    def __init__(self, uid: Optional[str] = None, parameters: Optional[OpParams] = None):
        super().__init__(uid)
        self.parameters = parameters or OpParams()
        self.train_parameters = self.parameters
        self.train_timings: Dict[str, float] = {}

    # ---------------------------------------------------------------------------------- builders
    def set_stages(self, stages: Sequence[OpPipelineStage]) -> "OpWorkflowModel":
        self.stages = list(stages)
        return self

    def set_features(self, features: Sequence[FeatureLike]) -> "OpWorkflowModel":
        """Result features; the raw features are the ones they derive from (``OpWorkflowModel.setFeatures``)."""
        self.result_features = list(features)
        raws = {}
        for f in self.result_features:
            for r in f.raw_features():
                raws[r.uid] = r
        self.raw_features = sorted(raws.values(), key=lambda f: f.name)
        return self

    def set_parameters(self, params: OpParams) -> "OpWorkflowModel":
        self.parameters = params
        return self

    def copy(self) -> "OpWorkflowModel":
        """A new model over the same fitted stages and features (``OpWorkflowModel.copy``)."""
        m = OpWorkflowModel(self.uid, self.parameters)
        for k in ("stages", "result_features", "raw_features", "blocklist"):
            setattr(m, k, list(getattr(self, k)))
        m.blocklist_map_keys = dict(self.blocklist_map_keys)
        m.train_parameters = self.train_parameters
        m.raw_feature_filter_results = self.raw_feature_filter_results
        m.reader = self.reader
        m.workflow_cv = self.workflow_cv
        m.train_timings = dict(self.train_timings)
        return m

    # ---------------------------------------------------------------------------------- scoring
    def _fitted_dag(self, features: Sequence[FeatureLike]):
        by_uid = {s.uid: s for s in self.stages}
        dag = compute_dag(features)
        out = []
        for layer in dag:
            l2 = []
            for st, d in layer:
                fs = by_uid.get(st.uid)
                if fs is None:
                    raise ValueError(f"stage {st.uid} ({type(st).__name__}) was not fitted in this model")
                l2.append((fs, d))
            out.append(l2)
        return out

    def transform_dataset(self, raw: Dataset, features=None) -> Dataset:
        return apply_transformations_dag(raw, self._fitted_dag(features or self.result_features))

    def compute_data_up_to(self, feature: FeatureLike, params: Optional[OpParams] = None) -> Dataset:
        """Raw data plus every fitted stage's output up to and including ``feature``
        (``OpWorkflowModel.computeDataUpTo``, ``OpWorkflowModel.scala:150-170``)."""
        raw = self.generate_raw_data(params or self.parameters)
        if feature.is_raw:
            return raw
        return self.transform_dataset(raw, [feature])

    def get_metadata(self, *features: FeatureLike) -> Dict[FeatureLike, object]:
        """Each feature's output metadata (its vector metadata when it has one, else the stage's metadata
        dict) from the fitted stage that made it (``OpWorkflowModel.getMetadata``)."""
        by_uid = {s.uid: s for s in self.stages}
        out = {}
        for f in features:
            st = by_uid.get(f.origin_stage.uid) if f.origin_stage is not None else None
            if st is None:
                raise ValueError(f"feature {f.name} is not produced by a fitted stage of this model")
            out[f] = st.metadata.get("vector_metadata", st.metadata)
        return out

    def score(self, data=None, keep_raw_features: bool = False, keep_intermediate_features: bool = False,
              params: Optional[OpParams] = None) -> Dataset:
        """Score a reader's / dataset's rows: raw -> all fitted stages -> result features."""
        if data is not None:
            self.set_input_dataset(data)
        raw = self.generate_raw_data(params or self.parameters)
        out = self.transform_dataset(raw)
        keep = [f.name for f in self.result_features]
        if keep_intermediate_features:
            return out
        if keep_raw_features:
            keep = [f.name for f in self.raw_features if f.name in out] + keep
        return out.select([k for k in dict.fromkeys(keep)])

    def score_and_evaluate(self, evaluator, data=None, **kw):
        scores = self.score(data, keep_raw_features=True, **kw)
        return scores, self.evaluate_scores(evaluator, scores)

    def save_scores(self, path: str, data=None, evaluator=None, metrics_path: Optional[str] = None,
                    fmt: str = "parquet", keep_raw_features: bool = False):
        """Score and write the result features to ``path`` (``OpWorkflowModel.saveScores``,
        ``OpWorkflowModel.scala:381-428``); with ``evaluator`` also evaluate, writing the metrics JSON
        to ``metrics_path`` when given. ``fmt``: parquet | csv | json | avro. Returns (scores, metrics)."""
        from .runner import _write_json, save_dataset
        if evaluator is not None:
            scores, metrics = self.score_and_evaluate(evaluator, data)
            if not keep_raw_features:
                scores = scores.select([f.name for f in self.result_features if f.name in scores])
        else:
            scores, metrics = self.score(data, keep_raw_features=keep_raw_features), None
        save_dataset(scores, path, fmt)
        if metrics is not None and metrics_path:
            _write_json(metrics_path, metrics)
        return scores, metrics

    def evaluate(self, evaluator, data=None):
        return self.score_and_evaluate(evaluator, data)[1]

    def evaluate_scores(self, evaluator, scores: Dataset) -> Dict:
        if evaluator.label_col not in scores:
            raise ValueError(f"label column {evaluator.label_col} not in scored data")
        return evaluator.evaluate_all(scores)

    # -------------------------------------------------------------------------------- summaries
    def model_insights(self, feature: Optional[FeatureLike] = None):
        from ..insights.model_insights import extract_model_insights
        feat = feature or next((f for f in self.result_features if f.wtype.__name__ == "Prediction"), None)
        return extract_model_insights(self, feat)

    def summary_json(self) -> Dict:
        from ..selector.model_selector import ModelSelector
        out = {}
        for st in self.stages:
            if "summary" in st.metadata:
                out[st.uid] = st.metadata["summary"]
        return out

    def summary(self) -> str:
        return json.dumps(self.summary_json(), indent=2, default=_json_default)

    def summary_pretty(self) -> str:
        from ..insights.pretty import summary_pretty
        return summary_pretty(self)

    # ------------------------------------------------------------------------------------ io
    def save(self, path: str, overwrite: bool = True) -> None:
        from .io import save_model
        save_model(self, path, overwrite)

    @staticmethod
    def load(path: str, workflow: Optional[OpWorkflow] = None) -> "OpWorkflowModel":
        from .io import load_model
        return load_model(path, workflow)

    def score_function(self):
        """Spark-free per-record scoring function (``local/.../OpWorkflowModelLocal.scala:79-122``)."""
        from ..local.scoring import score_function
        return score_function(self)

    def get_origin_stage_of(self, feature: FeatureLike):
        return next(s for s in self.stages if s.uid == feature.origin_stage.uid)


def _empty_rff_results():
    """``RawFeatureFilterResults()`` of a workflow trained without a filter (the default config)."""
    from ..filters.raw_feature_filter import RawFeatureFilterResults
    from .io import _EMPTY_RFF
    return RawFeatureFilterResults.from_json(_EMPTY_RFF)


def _copy_with_new_stages(features, stages_by_uid) -> List[FeatureLike]:
    """``FeatureLike.copyWithNewStages``: the features rebuilt with every origin stage the map holds (by uid)
    swapped in; one object per feature uid, so a workflow's own features and a loaded model's features of the same
    DAG merge into one graph (raw features: the first seen -- the workflow's own, with their extract functions)."""
    memo: Dict[str, FeatureLike] = {}

    def cp(f):
        if f.uid in memo:
            return memo[f.uid]
        if f.is_raw:
            memo[f.uid] = f
            return f
        parents = [cp(p) for p in f.parents]
        st = stages_by_uid.get(f.origin_stage.uid, f.origin_stage)
        memo[f.uid] = FeatureLike(f.name, f.wtype, f.is_response, st, parents, uid=f.uid,
                                  distributions=f.distributions)
        return memo[f.uid]
    return [cp(f) for f in features]


def _snake(k: str) -> str:
    import re
    return re.sub(r"(?<!^)(?=[A-Z])", "_", k).lower()


def _json_default(o):
    import numpy as np
    if isinstance(o, (np.floating, np.integer)):
        return o.item()
    if isinstance(o, np.ndarray):
        return o.tolist()
    if isinstance(o, torch.Tensor):
        return o.tolist()
    return str(o)

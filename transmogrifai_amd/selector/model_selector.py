"""Model selector stage and its fitted ``SelectedModel``.

Reference: ``ModelSelector`` (``core/.../stages/impl/selector/ModelSelector.scala:72-264``: validate grid,
refit the winner on the prepared full training set, train evaluation, ``ModelSelectorSummary``
metadata, ``SelectedModel``), ``ModelSelectorSummary`` (``ModelSelectorSummary.scala:55-309``) and the
hold-out evaluation of ``HasTestEval`` (``ModelSelectorNames.scala:73-123``).
"""
from __future__ import annotations

import logging
import math
import os
import time
from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch

from ..data.columns import PredictionColumn
from ..features import types as T
from ..models.base import FitJob, OpPredictorModel, learner_class
from ..stages.base import BinaryEstimator, register_stage
from ..tuning.splitters import Splitter
from ..tuning.validators import OpValidator

log = logging.getLogger(__name__)

SUMMARY_KEY = "summary"


def problem_type_of(metrics: Dict) -> str:
    if "AuROC" in metrics or "AuPR" in metrics:
        return "BinaryClassification"
    if "F1" in metrics:
        return "MultiClassification"
    return "Regression"


def _global_label_counts(y):
    """Label value counts over every rank's rows (one small object all-gather instead of gathering all
    labels to every rank); what the splitters' ``pre_validation_prepare`` needs."""
    from collections import Counter
    from ..parallel import dp
    from ..tuning.splitters import label_counts
    return dict(dp.merge_counters([Counter(label_counts(y))])[0])


def _splitter_prepare(splitter, y):
    """``splitter.pre_validation_prepare`` on the global label statistics it needs: the DataSplitter only
    the global row count (one scalar all-reduce -- value counts of a continuous label are one entry per
    row: 100M entries at the regression-100m config), the balancer / cutter the label value counts."""
    from ..parallel import dp
    from ..tuning.splitters import DataSplitter
    if type(splitter) is DataSplitter and not isinstance(y, dict):
        n = torch.tensor([float(y.shape[0])], dtype=torch.float64, device=y.device)
        if dp.active():
            n = dp.sum_([n])[0]
        return splitter.pre_validation_prepare({}, n_total=int(n.item()))
    return splitter.pre_validation_prepare(_global_label_counts(y))


@register_stage
class SelectedModel(OpPredictorModel):
    operation_name = "modelSelection"

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.evaluators = []

    def evaluate_model(self, ds) -> Dict:
        """Hold-out evaluation (``HasTestEval.evaluateModel``): fills ``holdoutEvaluation``. A row-sharded
        hold-out is scored locally and the (label, prediction) rows are all-gathered for the metrics
        (SURVEY.md §2.7 C12)."""
        from ..parallel import dp
        from ..models.base import predict_chunked
        lab = ds[self._inputs[0].name].values.to(torch.float64)
        pred, raw, prob = predict_chunked(self.learner, self.state, ds[self._inputs[1].name])
        lab, pred, raw, prob = dp.rows_opt(lab, pred, raw, prob)
        res = {}
        for ev in self.evaluators:
            res.update(ev.evaluate_arrays(lab, pred, raw, prob))
        if SUMMARY_KEY in self.metadata:
            self.metadata[SUMMARY_KEY]["holdoutEvaluation"] = res
        return res


@register_stage
class ModelSelector(BinaryEstimator):
    """Estimator (label: RealNN, features: OPVector) -> Prediction choosing the best learner + params."""
    operation_name = "modelSelection"
    output_type = T.Prediction
    allow_label_as_input = True

    def __init__(self, validator: OpValidator = None, splitter: Optional[Splitter] = None,
                 models: Sequence[Tuple[str, Sequence[Dict]]] = (), evaluators: Sequence = (),
                 uid: Optional[str] = None):
        super().__init__(uid=uid)
        self.validator = validator
        self.splitter = splitter
        self.models = [(n, [dict(g) for g in grid]) for n, grid in models]
        self.evaluators = list(evaluators)
        self.best: Optional[Any] = None
        self.best_estimator: Optional[Any] = None    # set by workflow-level CV (find_best_estimator)

    def find_best_estimator(self, data, during) -> Any:
        """Workflow-level CV (``ModelSelector.findBestEstimator``, ModelSelector.scala:116-128): validate
        with the ``during`` DAG refit per fold; ``fit`` then refits the chosen learner without
        re-validating."""
        from ..parallel import dp
        label, vec = self._inputs[0].name, self._inputs[1].name
        if self.splitter is not None:
            self._split_summary = _splitter_prepare(self.splitter, data[label].values)
        if not during:
            self.best_estimator = None
            return None
        self.best_estimator = self.validator.validate_with_dag(self.models, data, label, vec, during, self.splitter)
        return self.best_estimator

    # Row-sharded fits: the splitter's global statistics come from one label gather, then every rank
    # contributes the rows that any CV fold or the refit samples (masks are functions of the global
    # row id) and the (learner x grid x fold) jobs are sharded over the ranks on that replicated
    # sample (tuning/validators.py) -- the reference's maxTrainingSample cap keeps it small.
    dp_aware = True

    def fit_columns(self, label_col, vec_col, ds=None):
        from ..parallel import dp
        dev = vec_col.device
        y = label_col.values.to(vec_col.dtype)
        row_ids = ds.row_ids.to(dev) if ds is not None else torch.arange(len(vec_col), device=dev)
        t0 = time.time()
        split_summary = None
        if self.splitter is not None:
            if self.best_estimator is not None and getattr(self, "_split_summary", None) is not None:
                split_summary = self._split_summary
            else:
                split_summary = _splitter_prepare(self.splitter, y)
        # every row is materialised: CV folds validate on their whole held-out fold and only their training
        # part is down-sampled (OpCrossValidation.scala:122-129 applies validationPrepare to the training
        # split only); the rows some fold or the refit may train on seed the tree binning sample
        X, y, row_ids, cand = self._gather_rows(vec_col, y, row_ids)
        if dp.active():
            with dp.local_only():
                return self._fit(X, y, row_ids, split_summary, t0, cand)
        return self._fit(X, y, row_ids, split_summary, t0, cand)

    def _gather_rows(self, vec_col, y, row_ids):
        """All rows of every rank (folds are functions of the global row id) and the positions of the rows
        that some CV fold's or the refit's down-sampled training set may use (``None`` without a
        splitter)."""
        from ..parallel import dp
        X, y, row_ids = dp.rows(vec_col.values), dp.rows(y), dp.rows(row_ids)
        if self.splitter is None:
            return X, y, row_ids, None
        n_folds = getattr(self.validator, "num_folds", 1)
        keep = self.splitter.validation_prepare(row_ids, y, stream=5)
        for k in range(n_folds):
            keep |= self.splitter.validation_prepare(row_ids, y, stream=11 + k)
        return X, y, row_ids, torch.nonzero(keep).reshape(-1)

    def _fit(self, X, y, row_ids, split_summary, t0, cand=None):
        # tree learners draw their quantile-binning sample from the training candidates only
        ctx: Dict[str, Any] = {} if cand is None else {"tree_rows": cand}
        # the prepared full training set of the winner's refit (fixed before the selection: batched learners
        # fit it for every grid point inside their CV batch, tuning/validators.py)
        if self.splitter is not None:
            if hasattr(self.splitter, "weights"):
                w = self.splitter.weights(row_ids, y, stream=5)
                rows = torch.nonzero(w > 0).reshape(-1)
                refit_rows = (rows, w[rows])
            else:
                rows = torch.nonzero(self.splitter.validation_prepare(row_ids, y, stream=5)).reshape(-1)
                refit_rows = (rows, None)
        else:
            rows = None
            refit_rows = (None, None)
        if self.best_estimator is None and os.environ.get("TMOG_BATCHED_REFIT", "1") != "0":
            ctx["refit_job"] = refit_rows
        if self.best_estimator is not None:     # chosen by workflow-level CV
            res = self.best_estimator
        else:
            from ..workflow.workflow import OpStep, step
            with step(OpStep.CrossValidation):
                res = self.validator.validate(self.models, X, y, row_ids, self.splitter, context=ctx)
        self.best = res
        # refit the winner on the prepared full training set
        learner = learner_class(res.best_learner)()
        params = dict(learner.defaults, **res.best_params)
        job = FitJob(params, refit_rows[0], refit_rows[1])
        from ..tuning.validators import refit_key
        ready = (ctx.pop("refit_states", None) or {}).get(refit_key(res.best_learner, params))
        ctx.pop("refit_job", None)
        from ..workflow.workflow import OpStep as _S, step as _step
        # the winner's refit and its training evaluation are timed as their own phase (not FeatureEngineering)
        t_refit = time.time()
        with _step(_S.ModelRefit):
            # the winner's refit uses the same intra-job parallelism over the ranks as its CV fits
            from ..parallel import dist as D
            # (projection mode answers collectives locally but cannot emulate the tree grower's RCCL exchange: local refit)
            if D.world() > 1 and not D.simulated() and learner.parallel in ("rows", "features"):
                from ..parallel.learner_parallel import LearnerParallel
                ctx["par"] = LearnerParallel()
            try:
                state = ready if ready is not None else learner.fit_batch(X, y, [job], context=ctx)[0]
            finally:
                ctx.pop("par", None)
            # training evaluation on the prepared data
            Xr = X if rows is None else X[rows]
            yr = y if rows is None else y[rows]
            pred, raw, prob = learner.predict(state, Xr)
            train_eval: Dict = {}
            for ev in self.evaluators:
                train_eval.update(ev.evaluate_arrays(yr.to(torch.float64), pred, raw, prob))
        summary = {
            "validationType": self.validator.validation_type,
            "validationParameters": self.validator.params(),
            "dataPrepParameters": self.splitter.params() if self.splitter is not None else {},
            "dataPrepResults": split_summary,
            "evaluationMetric": self.validator.evaluator.metric,
            "problemType": problem_type_of(train_eval),
            "bestModelUID": f"{res.best_learner}_{self.uid.split('_')[-1]}",
            "bestModelName": res.best_learner,
            "bestModelType": res.best_learner,
            "bestModelParameters": params,
            "validationResults": [e.to_json() for e in res.evaluations],
            "trainEvaluation": train_eval,
            "holdoutEvaluation": None,
            "failures": res.failures,
            "timings": dict(res.timings, refit=time.time() - t_refit, selector_total=time.time() - t0),
        }
        sched = getattr(self.validator, "last_schedule", None)
        if sched:        # multi-rank: per learner (mode, shard s, spread s, ranks per group, hybrid s)
            summary["schedule"] = {k: [x if not (isinstance(x, float) and not math.isfinite(x)) else None
                                       for x in v] for k, v in sched.items()}
        self.metadata[SUMMARY_KEY] = summary
        m = SelectedModel(res.best_learner, state, params)
        m.evaluators = list(self.evaluators)
        return m

"""Cross-validation and train/validation split over (learner x grid) candidates.

Reference: ``OpValidator`` (``core/.../stages/impl/tuning/OpValidator.scala:94-380``; Future pool over grid
points, failures dropped, ``maxWait``), ``OpCrossValidation`` (``OpCrossValidation.scala:63-202``: k folds
via ``MLUtils.kFold``, optional stratification, per-grid metric averaged over folds, best grid per
estimator, best estimator overall) and ``OpTrainValidationSplit`` (``OpTrainValidationSplit.scala:35-143``).

MI355X execution model: instead of a thread pool of Spark jobs, every learner trains *all* of its
(grid point x fold) models in one batched device program (``Learner.fit_batch``), then scores all
of them on their validation folds in one traversal / GEMM (``Learner.predict_batch``). With several
ranks (one per GPU) the (learner, grid, fold) jobs are sharded across ranks by estimated cost
(LPT) over a replicated training table -- no per-iteration collectives -- and only the metrics are
exchanged (one ``all_gather_object``).
"""
from __future__ import annotations

import contextlib
import logging
import math
import os
import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..models.base import FitJob, learner_class
from ..parallel import dist as D
from ..utils.device_errors import DeviceFault, is_device_fault
from .splitters import Splitter, row_uniform

log = logging.getLogger(__name__)


@dataclass
class ModelEvaluation:
    model_uid: str
    model_name: str
    model_type: str
    metric_values: Dict[str, float]
    model_parameters: Dict[str, Any]

    def to_json(self):
        return {"modelUID": self.model_uid, "modelName": self.model_name, "modelType": self.model_type,
                "metricValues": self.metric_values, "modelParameters": self.model_parameters}


@dataclass
class ValidationResult:
    best_learner: str
    best_params: Dict[str, Any]
    best_metric: float
    evaluations: List[ModelEvaluation]
    failures: List[str] = field(default_factory=list)
    timings: Dict[str, float] = field(default_factory=dict)


# Seconds per unit of _job_cost's work estimate, per learner: seeded from a 1-GPU MI355X headline run
# (10M-row binary selector, 3-fold CV on the 667K-row folds: LR 0.35 s, RF 0.38 s, XGBoost 1.67 s for the
# default grids) and re-calibrated from every validation's measured per-learner times (identical on all
# ranks: the times are all-gathered before the update), so the LPT sharding of (learner x grid x fold)
# jobs over the ranks balances measured, not guessed, cost.
_COST_SCALE: Dict[str, float] = {"OpLogisticRegression": 8.4e-12, "OpRandomForestClassifier": 1.3e-12,
                                 "OpXGBoostClassifier": 8.0e-13}
_DEFAULT_SCALE = 1.3e-12
_UNBOUNDED_WAIT = 86400.0       # the reference default maxWait (1 day): no worker thread needed


# TMOG_FIT_PHASES=1: wall-clock of each learner's fit / validation predict / metric phases (the device is
# synchronised at each boundary, so the phases add up to the learner's time; diagnostics)
PHASE_TIMES: Dict[str, float] = {}
import threading as _threading  # noqa: E402
_PHASE_LOCK = _threading.Lock()


def _phase_clock(X) -> Optional[float]:
    if os.environ.get("TMOG_FIT_PHASES") != "1":
        return None
    if isinstance(X, torch.Tensor) and X.is_cuda:
        torch.cuda.current_stream(X.device).synchronize()
    return time.perf_counter()


def _cancel_grace_s() -> float:
    """Seconds a cancelled fit gets to reach its next cancellation check before it is abandoned."""
    return float(os.environ.get("TMOG_CANCEL_GRACE_S", "30"))


def _scaled_cost(learner: str, params: Dict, n: int, d: int) -> float:
    return _job_cost(learner, params, n, d) * _COST_SCALE.get(learner, _DEFAULT_SCALE)


def SCH_SERIAL(mode) -> float:
    from ..parallel.scheduler import SERIAL_FRACTION
    return SERIAL_FRACTION.get(mode, 0.0)


def _calibrate(models, jobs, owner, timings, n: int, d: int, spread=None):
    """Update the per-learner seconds-per-unit from this validation's measured (max over ranks) times.
    ``spread``: learner -> (ranks per job, replicated fraction) of the spread / hybrid learners, whose measured
    time is divided back to single-rank seconds with the scheduler's speed-up model; sharded learners divide
    by the ranks their jobs ran on."""
    spread = spread or {}
    for li, (lname, grid) in enumerate(models):
        t = timings.get(lname)
        mine = [j for j, (l, g, k) in enumerate(jobs) if l == li]
        if not t or not mine:
            continue
        units = sum(_job_cost(lname, grid[jobs[j][1]], n, d) for j in mine)
        if units <= 0:
            continue
        if li in spread:
            gsz, s = spread[li]
            groups = max(1, D.world() // max(1, gsz))
            _COST_SCALE[lname] = float(t) * groups / (units * (s + (1.0 - s) / max(1, gsz)))
        else:
            ranks = max(1, len({owner[j] for j in mine}))
            _COST_SCALE[lname] = float(t) * ranks / units


def _job_cost(learner: str, params: Dict, n: int, d: int) -> float:
    if "LogisticRegression" in learner or "SVC" in learner or "LinearRegression" in learner:
        return 2.0 * n * d * params.get("max_iter", 100) * 0.05
    depth = params.get("max_depth", 5)
    if "RandomForest" in learner:
        k = math.sqrt(d)
        return params.get("num_trees", 20) * n * depth * k
    if "GBT" in learner:
        return params.get("max_iter", 20) * n * depth * d * 0.5
    if "XGBoost" in learner:
        return params.get("num_round", 100) * n * params.get("max_depth", 6) * d * 0.5
    if "DecisionTree" in learner:
        return n * depth * d
    return float(n * d)


def _fold_alignment(fitted, features_name: str, data):
    """``(kept input columns, input width)`` when the fold's feature vector is the output of a
    feature-dropping SanityChecker over a vector every fold shares, else ``None``."""
    from ..stages.preparators.sanity_checker import SanityCheckerModel
    st = next((s for s in fitted if s.get_output_feature_name() == features_name), None)
    if isinstance(st, SanityCheckerModel) and st.remove_bad_features and st.indices_to_keep is not None:
        in_name = st.get_input_features()[1].name
        if in_name in data:
            return list(st.indices_to_keep), int(data[in_name].width)
    return None


def refit_key(lname: str, params: Dict[str, Any]) -> str:
    """Key of a speculative refit state: learner name + its full parameter map."""
    import json
    return lname + ":" + json.dumps(params, sort_keys=True, default=str)


class OpValidator:
    validation_type = "CrossValidation"

    def __init__(self, evaluator, seed: Optional[int] = None, stratify: bool = False, parallelism: int = 8,
                 max_wait: float = 86400.0, is_classification: bool = True):
        self.evaluator = evaluator
        self.seed = int(np.random.randint(0, 2 ** 31 - 1)) if seed is None else int(seed)
        self.stratify = stratify
        self.parallelism = parallelism
        self.max_wait = max_wait
        self.is_classification = is_classification

    # -- splits ---------------------------------------------------------------------------------
    def make_splits(self, row_ids: torch.Tensor, y: torch.Tensor) -> List[Tuple[torch.Tensor, torch.Tensor]]:
        raise NotImplementedError

    def params(self) -> Dict[str, Any]:
        raise NotImplementedError

    # -- validation -----------------------------------------------------------------------------
    def validate(self, models: Sequence[Tuple[str, Sequence[Dict]]], X: torch.Tensor, y: torch.Tensor,
                 row_ids: torch.Tensor, splitter: Optional[Splitter] = None, context=None) -> ValidationResult:
        t0 = time.time()
        splits = self.make_splits(row_ids, y)
        train_rows, val_rows = [], []
        for k, (tr, va) in enumerate(splits):
            keep = tr
            weights = None
            if splitter is not None:
                if hasattr(splitter, "weights"):
                    w = splitter.weights(row_ids, y, stream=11 + k)
                    keep = tr & (w > 0)
                    weights = w
                else:
                    keep = tr & splitter.validation_prepare(row_ids, y, stream=11 + k)
            idx = torch.nonzero(keep).reshape(-1)
            train_rows.append((idx, None if weights is None else weights[idx]))
            val_rows.append(torch.nonzero(va).reshape(-1))
        return self._run(models, X, y, train_rows, val_rows, len(splits), t0, context)

    def _run(self, models, X, y, train_rows, val_rows, n_folds: int, t0: float, context=None) -> ValidationResult:
        """Fit and score every (learner, grid point, fold) job on the fold row sets of ``X`` -- jobs of the
        intra-job-parallel learners on every rank, the others LPT-sharded over the ranks -- and select."""
        splits = range(n_folds)
        # all (learner, grid, fold) jobs
        jobs = []
        for li, (lname, grid) in enumerate(models):
            for gi, p in enumerate(grid):
                for k in range(len(splits)):
                    jobs.append((li, gi, k))
        world, me = D.world(), D.rank()
        # Learners with an intra-job parallel mode (linear: row-parallel; boosted / single trees:
        # feature-parallel) run every one of their jobs on every rank with the parallel context
        # (parallel/learner_parallel.py); the others' (grid x fold) jobs are sharded whole over the ranks
        # by estimated cost (LPT).
        par = None
        if world > 1:
            from ..parallel.learner_parallel import LearnerParallel
            par = LearnerParallel()
        n_tr = max(1, int(train_rows[0][0].numel())) if train_rows else 1
        # shard whole jobs or spread every job over the ranks: per learner, by the calibrated cost model
        # (parallel/scheduler.py); rank 0's choice is broadcast so every rank runs the same collectives
        spread = set()
        hybrid: Dict[int, int] = {}          # learner -> ranks per group
        pars: Dict[int, Any] = {}            # learner -> its intra-job parallel context
        if par is not None:
            from ..parallel import scheduler as SCH
            choices = SCH.choose(models, n_folds, n_tr, X.shape[1], world,
                                 lambda name: learner_class(name).parallel,
                                 lambda name, p: _scaled_cost(name, p, n_tr, X.shape[1]))
            dec = D.broadcast_object(sorted((li, c.mode, c.group_size) for li, c in choices.items()), 0)
            spread = {li for li, m, _ in dec if m == "spread"}
            hybrid = {li: int(g) for li, m, g in dec if m == "hybrid"}
            self.last_schedule = {models[li][0]: (c.mode, c.shard_s, c.spread_s, c.group_size, c.hybrid_s)
                                  for li, c in choices.items()}
            pars = {li: par for li in spread}
        sharded = [j for j, (li, gi, k) in enumerate(jobs) if li not in spread and li not in hybrid]
        costs = [_scaled_cost(models[jobs[j][0]][0], models[jobs[j][0]][1][jobs[j][1]], n_tr, X.shape[1])
                 for j in sharded]
        owner = [me] * len(jobs)
        for j, w in zip(sharded, D.lpt_assign(costs, world)):
            owner[j] = w
        # hybrid learners: every rank creates every subgroup (collective), then the learner's jobs are dealt to the
        # groups by LPT; this rank runs its group's jobs, each spread over the group
        for li in sorted(hybrid):
            from ..parallel import scheduler as SCH
            from ..parallel.learner_parallel import LearnerParallel
            g = hybrid[li]
            grp = D.partition(g)
            pars[li] = LearnerParallel(group=grp)
            lj = [j for j, (l, _, _) in enumerate(jobs) if l == li]
            lc = [_scaled_cost(models[li][0], models[li][1][jobs[j][1]], n_tr, X.shape[1]) for j in lj]
            for j, k in zip(lj, SCH.assign_groups(lc, world // g)):
                owner[j] = me if k == me // g else -1
        ctx = context if context is not None else {}
        results: Dict[Tuple[int, int, int], float] = {}
        failures = []
        timings = {}
        # spread learners first (all ranks in lockstep through their collectives), then the shards
        order = sorted(range(len(models)), key=lambda li: (li not in spread, li not in hybrid, li))
        lanes = self._learner_lanes(X, world, len(order), n_collective=len(pars))
        if lanes > 1:
            results, failures, timings = self._fit_eval_concurrent(models, order, jobs, owner, me, X, y, train_rows,
                                                                   val_rows, ctx, t0, lanes, n_tr, pars)
            order = []
        for li in order:
            lname, grid = models[li]
            mine = [(j, (l, g, k)) for j, (l, g, k) in enumerate(jobs) if l == li and owner[j] == me]
            collective = li in pars
            if not mine and not collective:
                continue
            # maxWait (OpValidator.scala:348, default 1 day): learners not started in time are dropped;
            # spread / hybrid learners take rank 0's decision so every rank skips the same collectives
            late = time.time() - t0 > self.max_wait
            if collective:
                late = bool(D.broadcast_object(late, 0))
            if late:
                failures.append(f"{lname}: not started within maxWait={self.max_wait}s")
                continue
            if not mine:            # a hybrid group without jobs of this learner
                continue
            t1 = time.time()
            # the context dict is shared (tree binning cache) -- the parallel context is set only
            # around the spread / hybrid learners
            if collective:
                ctx["par"] = pars[li]
            try:
                if not collective and self.max_wait < _UNBOUNDED_WAIT:
                    res, fails = self._fit_eval_bounded(lname, grid, mine, X, y, train_rows, val_rows, ctx,
                                                        self.max_wait - (time.time() - t0))
                else:
                    res, fails = self._fit_eval(lname, grid, mine, X, y, train_rows, val_rows, ctx)
            finally:
                ctx.pop("par", None)
            results.update(res)
            failures.extend(fails)
            timings[lname] = time.time() - t1
            if os.environ.get("TMOG_MEM_TRACE") == "1" and torch.cuda.is_available():
                timings[f"peak_gb:{lname}"] = round(torch.cuda.max_memory_allocated() / 1e9, 3)
                torch.cuda.reset_peak_memory_stats()
        # exchange metrics between ranks
        gathered = D.all_gather_object((results, failures, timings))
        allres: Dict[Tuple[int, int, int], float] = {}
        allfail: List[str] = []
        for r, f, tm in gathered:
            allres.update(r)
            for x in f:
                if x not in allfail:
                    allfail.append(x)
            for k, v in tm.items():
                timings[k] = max(timings.get(k, 0.0), v)
        _calibrate(models, jobs, owner, timings, n_tr, X.shape[1],
                   {li: (p.world, SCH_SERIAL(learner_class(models[li][0]).parallel)) for li, p in pars.items()})
        return self._select(models, allres, n_folds, allfail, timings, t0)

    def validate_with_dag(self, models: Sequence[Tuple[str, Sequence[Dict]]], data, label_name: str,
                          features_name: str, during, splitter: Optional[Splitter] = None) -> ValidationResult:
        """Workflow-level CV (``OpCrossValidation.validate`` with a DAG, OpCrossValidation.scala:105-132, and
        ``OpValidator.applyDAG``, OpValidator.scala:250-274): for every fold a fresh copy of the
        label-dependent ``during`` stages (SanityChecker, label-aware bucketizers, ...) is fitted on the
        fold's training rows only, both fold parts are transformed by it, and every (learner x grid point)
        is scored on that fold's own feature matrix -- so nothing the during stages learn from a fold's
        validation labels can leak into its metric. ``data`` holds the inputs of the during stages."""
        from ..parallel import dp
        from ..workflow.dag import copy_dag, fit_and_transform_dag
        t0 = time.time()
        row_ids = data.row_ids
        y_all = data[label_name].values
        splits = self.make_splits(row_ids, y_all)
        results: Dict[Tuple[int, int, int], float] = {}
        failures: List[str] = []
        timings: Dict[str, float] = {}
        # Batched path: the during DAG is fitted per fold, then the fold matrices -- aligned on the columns of
        # the during SanityChecker's input, a column dropped in a fold being all-zero in that fold's rows --
        # are stacked and every learner trains all of its (grid point x fold) jobs in ONE fit_batch, sharded
        # over the ranks as in validate (k-fold fewer learner launches, no redundant work per rank).
        if os.environ.get("TMOG_WCV_BATCHED", "1") != "0":
            folds = []
            for k, (tr, va) in enumerate(splits):
                ti = torch.nonzero(tr).reshape(-1)
                vi = torch.nonzero(va).reshape(-1)
                t1 = time.time()
                train_k, val_k, fitted = fit_and_transform_dag(copy_dag(during), data.take(ti), data.take(vi))
                timings[f"fold{k}:dag"] = time.time() - t1
                folds.append((train_k, val_k, _fold_alignment(fitted, features_name, data)))
            stacked = self._stack_folds(folds, label_name, features_name, splitter)
            if stacked is not None:
                X, y, train_rows, val_rows = stacked
                with dp.local_only():
                    res = self._run(models, X, y, train_rows, val_rows, len(splits), t0)
                res.timings.update(timings)
                return res
            log.warning("workflow CV: fold feature matrices cannot be aligned; validating fold by fold")
        for k, (tr, va) in enumerate(splits):
            ti = torch.nonzero(tr).reshape(-1)
            vi = torch.nonzero(va).reshape(-1)
            t1 = time.time()
            train_k, val_k, _ = fit_and_transform_dag(copy_dag(during), data.take(ti), data.take(vi))
            timings[f"fold{k}:dag"] = time.time() - t1
            Xt, yt = train_k[features_name].values, train_k[label_name].values
            Xv, yv = val_k[features_name].values, val_k[label_name].values
            rid_t = train_k.row_ids.to(Xt.device)
            rid_v = val_k.row_ids.to(Xt.device)
            if dp.active():       # row-sharded: learners train on the fold rows of every rank
                Xt, yt, rid_t, Xv, yv, rid_v = (dp.rows(Xt), dp.rows(yt), dp.rows(rid_t), dp.rows(Xv), dp.rows(yv),
                                                dp.rows(rid_v))
            X = torch.cat([Xt, Xv.to(Xt.dtype)])
            y = torch.cat([yt, yv]).to(X.dtype)
            nt = int(Xt.shape[0])
            keep = torch.arange(nt, device=X.device)
            weights = None
            if splitter is not None:
                if hasattr(splitter, "weights"):
                    w = splitter.weights(rid_t, yt.to(X.dtype), stream=11 + k)
                    keep = torch.nonzero(w > 0).reshape(-1)
                    weights = w[keep]
                else:
                    keep = torch.nonzero(splitter.validation_prepare(rid_t, yt.to(X.dtype), stream=11 + k)).reshape(-1)
            train_rows = {0: (keep, weights)}
            # applyDAG (OpValidator.scala:266-271) prepares the DAG-transformed validation part with the
            # splitter too (an up-sampled row counts once per copy)
            vsel = torch.arange(int(X.shape[0]) - nt, device=X.device)
            if splitter is not None:
                yvv = yv.to(X.dtype)
                if hasattr(splitter, "weights"):
                    vsel = torch.repeat_interleave(vsel, splitter.weights(rid_v, yvv, stream=41 + k).to(X.device))
                else:
                    vsel = torch.nonzero(splitter.validation_prepare(rid_v, yvv, stream=41 + k)).reshape(-1)
            val_rows = {0: vsel + nt}
            ctx: Dict[str, Any] = {}
            with dp.local_only():
                for li, (lname, grid) in enumerate(models):
                    t2 = time.time()
                    mine = [(gi, (li, gi, 0)) for gi in range(len(grid))]
                    res, fails = self._fit_eval(lname, grid, mine, X, y, train_rows, val_rows, ctx)
                    results.update({(l, g, k): v for (l, g, _), v in res.items()})
                    failures.extend(fails)
                    timings[lname] = timings.get(lname, 0.0) + time.time() - t2
        return self._select(models, results, len(splits), failures, timings, t0)

    def _fold_rows(self, k, rid_t, yt, rid_v, yv, nt, nv, dtype, dev, splitter):
        """(training positions, weights) and validation positions of fold ``k`` inside its block."""
        keep = torch.arange(nt, device=dev)
        weights = None
        if splitter is not None:
            if hasattr(splitter, "weights"):
                w = splitter.weights(rid_t, yt.to(dtype), stream=11 + k)
                keep = torch.nonzero(w > 0).reshape(-1)
                weights = w[keep]
            else:
                keep = torch.nonzero(splitter.validation_prepare(rid_t, yt.to(dtype), stream=11 + k)).reshape(-1)
        # applyDAG (OpValidator.scala:266-271) prepares the DAG-transformed validation part with the
        # splitter too (an up-sampled row counts once per copy)
        vsel = torch.arange(nv, device=dev)
        if splitter is not None:
            yvv = yv.to(dtype)
            if hasattr(splitter, "weights"):
                vsel = torch.repeat_interleave(vsel, splitter.weights(rid_v, yvv, stream=41 + k).to(dev))
            else:
                vsel = torch.nonzero(splitter.validation_prepare(rid_v, yvv, stream=41 + k)).reshape(-1)
        return (keep, weights), vsel + nt

    def _stack_folds(self, folds, label_name, features_name, splitter):
        """One matrix holding every fold's (train + validation) rows, the fold blocks one after another, and
        the per-fold row sets in it; ``None`` when the fold matrices have different columns that cannot be
        aligned."""
        from ..parallel import dp
        aligns = [a for _, _, a in folds]
        widths = [int(tk[features_name].width) for tk, _, _ in folds]
        metas = [tk[features_name].metadata for tk, _, _ in folds]
        keys = None
        if all(m is not None for m in metas):
            keys = [[(c.parent_feature_name, c.parent_feature_type, c.grouping, c.indicator_value,
                      c.descriptor_value) for c in m.columns] for m in metas]
            if any(len(set(k)) != len(k) or len(k) != w for k, w in zip(keys, widths)):
                keys = None         # repeated column descriptions (hashed text): not alignable by name
        if all(a is not None for a in aligns) and len({a[1] for a in aligns}) == 1 and aligns[0][1] is not None:
            # the during SanityChecker's kept columns of one shared input vector
            union = sorted(set().union(*[set(a[0]) for a in aligns]))
            pos = {c: i for i, c in enumerate(union)}
            cols = [[pos[c] for c in a[0]] for a in aligns]
            W = len(union)
        elif keys is not None and len({tuple(k) for k in keys}) > 1:
            # fold-fitted stages with fold-specific columns (label-aware bucketizers): union of the columns by
            # their metadata description, in first-seen order
            pos: Dict[tuple, int] = {}
            for k in keys:
                for c in k:
                    pos.setdefault(c, len(pos))
            cols = [[pos[c] for c in k] for k in keys]
            W = len(pos)
        elif len(set(widths)) == 1:
            cols, W = [None] * len(folds), widths[0]
        else:
            return None
        blocks, ys, train_rows, val_rows = [], [], {}, {}
        off = 0
        for k, (train_k, val_k, _) in enumerate(folds):
            Xt, yt = train_k[features_name].values, train_k[label_name].values
            Xv, yv = val_k[features_name].values, val_k[label_name].values
            dev = Xt.device
            rid_t, rid_v = train_k.row_ids.to(dev), val_k.row_ids.to(dev)
            if dp.active():       # row-sharded: every rank holds every fold's rows
                Xt, yt, rid_t, Xv, yv, rid_v = (dp.rows(Xt), dp.rows(yt), dp.rows(rid_t), dp.rows(Xv), dp.rows(yv),
                                                dp.rows(rid_v))
            Xk = torch.cat([Xt, Xv.to(Xt.dtype)])
            if cols[k] is not None:
                full = torch.zeros(Xk.shape[0], W, dtype=Xk.dtype, device=dev)
                full[:, torch.as_tensor(cols[k], dtype=torch.int64, device=dev)] = Xk
                Xk = full
            nt, nv = int(Xt.shape[0]), int(Xv.shape[0])
            (keep, weights), vsel = self._fold_rows(k, rid_t, yt, rid_v, yv, nt, nv, Xk.dtype, dev, splitter)
            train_rows[k] = (keep + off, weights)
            val_rows[k] = vsel + off
            blocks.append(Xk)
            ys.append(torch.cat([yt, yv]).to(Xk.dtype))
            off += int(Xk.shape[0])
        return torch.cat(blocks), torch.cat(ys), train_rows, val_rows

    def _learner_lanes(self, X, world: int, n_learners: int, n_collective: int = 0) -> int:
        """Learners fitted at once on one GPU (``parallelism``, OpValidator.scala:377: the reference runs up to 8
        fits as concurrent futures). Only single-rank: spread learners move through collectives in lockstep.
        Default on the GPU: 2 lanes (``TMOG_LEARNER_LANES`` overrides). The longest learner (XGBoost on the
        headline) keeps lane 0 and the caller's stream plus the free side streams for its boosting parts, the
        other lane runs the remaining learners one after the other on a side stream: with the stream set bounded
        to one per hardware queue (ops/streams.py) the round-3 stalls are gone and the headline step drops from
        1.94 to 1.75-1.77 s on one box (3 lanes: 1.77-1.97 s -- the boosting parts lose a stream; more streams
        than hardware queues: 1.95 s; profiles/r4_lanes_*.log, docs/ROUND4.md)."""
        env = os.environ.get("TMOG_LEARNER_LANES")
        # host-only runs stay sequential unless asked for (the CPU kernels already use every core)
        if n_learners < 2 or not isinstance(X, torch.Tensor) or not (X.is_cuda or env):
            return 1
        # several ranks: lanes only when at most one learner runs collectives (the others' jobs are local to the
        # rank) and maxWait is unbounded (a deadline could cancel a collective fit on one rank and not another)
        if world > 1 and (n_collective > 1 or (n_collective and self.max_wait < _UNBOUNDED_WAIT)):
            return 1
        from ..models.tree_engine import free_lanes
        cap = int(env) if env else 2
        return max(1, min(cap, n_learners, len(free_lanes())))

    def _fit_eval_concurrent(self, models, order, jobs, owner, me, X, y, train_rows, val_rows, ctx, t0, lanes, n_tr,
                             pars=None):
        """Every learner's batch on one of ``lanes`` worker threads, each with its own HIP stream (ordered after
        the caller's, which waits for all of them) and its own range of native tree-grower slots, longest
        estimated learner first. One learner's host round trips (OWL-QN line searches, tree levels, early-stopping
        reads) and small launches then overlap another's kernels instead of idling the GPU; every learner's
        kernels and reductions are the ones the sequential path runs, so the metrics are identical. maxWait
        bounds the whole search: learners not started in time are dropped, and learners still running at the
        deadline are reported failed and abandoned (``awaitResult(maxWait)``, OpValidator.scala:348)."""
        import sys
        import threading
        from ..models import tree_engine as TE
        dev = X.device
        todo = []
        for li in order:
            mine = [(j, (l, g, k)) for j, (l, g, k) in enumerate(jobs) if l == li and owner[j] == me]
            if mine:
                lname, grid = models[li]
                cost = sum(_scaled_cost(lname, grid[g], n_tr, X.shape[1]) for _, (_, g, _) in mine)
                todo.append((cost, li, mine))
        todo.sort(key=lambda t: -t[0])
        pars = pars or {}
        if pars:     # copies of the context must share its caches: create them before the lanes copy it
            ctx.setdefault("refit_states", {})
            if any(getattr(learner_class(models[li][0]), "parallel", None) == "features" for li in pars):
                from ..models.trees import _ctx as _tree_ctx
                _tree_ctx(X, ctx)
        results: Dict[Tuple[int, int, int], float] = {}
        failures: List[str] = []
        timings: Dict[str, float] = {}
        from ..utils import cancel
        started, errs = set(), []
        lock = threading.Lock()
        token = threading.Event()       # set at the maxWait deadline: running fits stop at their next check
        gpu = dev.type == "cuda"
        cur = torch.cuda.current_stream(dev) if gpu else None
        # lane 0 runs on the caller's stream, the others on side streams of the fixed process-wide set
        # (ops/streams.py: one stream per hardware queue); fewer free side streams -> fewer lanes
        from ..ops import streams as SP
        # TMOG_LANE_PRIO=1: the critical (first, longest) learner's lane runs on a high-priority stream (its boosting
        # parts and grower groups then lease high-priority streams too) and the caller's stream goes to the next lane
        crit = SP.lease(dev, 1, high=True) if gpu and lanes > 1 and os.environ.get("TMOG_LANE_PRIO", "0") == "1" \
            else []
        side = crit + (SP.lease(dev, lanes - 1 - len(crit)) if gpu else [])
        # native slot lanes no abandoned fit holds (models/tree_engine.py quarantine_lane)
        bases = TE.free_lanes()
        if not bases:
            raise RuntimeError("every native tree-grower slot lane is held by a fit abandoned at its maxWait deadline")
        lanes = min(lanes, len(bases))
        if gpu and len(side) > lanes - 1:
            SP.release(dev, side[lanes - 1:])
            side = side[:lanes - 1]
        if gpu:
            streams = crit + [cur] + side[len(crit):]
            lanes = len(streams)
            for st in side:
                st.wait_stream(cur)
        else:
            streams = [None] * lanes

        def worker(w):
            try:
                if gpu:
                    torch.cuda.set_device(dev)
                TE.set_slot_lane(bases[w])
                with cancel.scope(token), (torch.cuda.stream(streams[w]) if gpu else contextlib.nullcontext()):
                    while True:
                        with lock:
                            if not todo or errs:
                                return
                            _, li, mine = todo.pop(0)
                            lname, grid = models[li]
                            if time.time() - t0 > self.max_wait:
                                failures.append(f"{lname}: not started within maxWait={self.max_wait}s")
                                continue
                            started.add(li)
                        t1 = time.time()
                        # the collective learner's view of the shared context carries its parallel context
                        lctx = dict(ctx, par=pars[li]) if li in pars else ctx
                        res, fails = self._fit_eval(lname, grid, mine, X, y, train_rows, val_rows, lctx)
                        with lock:
                            results.update(res)
                            failures.extend(fails)
                            timings[lname] = time.time() - t1
                            started.discard(li)
            except cancel.FitCancelled:
                return                          # its learner stays in `started`: reported as timed out
            except BaseException as e:          # noqa: BLE001  (re-raised on the caller's thread)
                with lock:
                    errs.append(e)

        th = [threading.Thread(target=worker, args=(w,), name=f"fit-lane-{w}", daemon=True) for w in range(lanes)]
        from ..utils.threads import fast_switch
        from ..utils.watchdog import Watchdog
        # a lane returning from a native call must win the GIL back from one running Python promptly; the
        # watchdog dumps every thread's stack if no fit makes progress for TMOG_WATCHDOG_S seconds
        SP.set_active_lanes(lanes)
        try:
            with fast_switch(float(os.environ.get("TMOG_PIPE_SWITCH_S", "5e-5"))), Watchdog("learner lanes"):
                for t in th:
                    t.start()
                bounded = self.max_wait < _UNBOUNDED_WAIT
                for t in th:
                    t.join(max(0.0, self.max_wait - (time.time() - t0)) if bounded else None)
                abandoned = []
                if any(t.is_alive() for t in th):
                    token.set()                     # cooperative cancel: running fits stop at their next check
                    grace_end = time.time() + _cancel_grace_s()
                    for t in th:
                        t.join(max(0.0, grace_end - time.time()))
                    # a fit inside a long native call never reaches a check: give it up (the reference abandons
                    # its future) rather than block the selector past maxWait + grace
                    abandoned = [w for w, t in enumerate(th) if t.is_alive()]
                    # an abandoned lane keeps its native slots (and its side stream, returned by the reaper) until its
                    # thread exits: later fits -- this selector's and later validate() calls' -- get other lanes
                    for w in abandoned:
                        st_w = streams[w] if gpu else None
                        rel = (lambda s_=st_w: SP.release(dev, [s_])) if (gpu and st_w is not cur) else None
                        TE.quarantine_lane(bases[w], th[w], rel)
                    if abandoned:
                        log.warning("maxWait: %d learner lane(s) did not stop within %.0fs of cancellation; abandoned",
                                    len(abandoned), _cancel_grace_s())
        finally:
            SP.set_active_lanes(1)
        if gpu:
            live = [st for w, st in enumerate(streams) if w not in abandoned and st is not cur]
            for st in live:
                cur.wait_stream(st)
            # blocks freed on the lane streams are reused by later allocations only once their work has ended
            if abandoned:
                for st in live + [cur]:
                    st.synchronize()
                SP.release(dev, live)           # an abandoned lane's stream is released by its reaper
            else:
                torch.cuda.synchronize(dev)
                SP.release(dev, side)
        with lock:
            if errs:
                raise errs[0]
            for li in sorted(started):      # still running at the maxWait deadline: cancelled
                lname = models[li][0]
                log.warning("Model %s did not finish within maxWait=%ss; its fits are dropped", lname, self.max_wait)
                failures.append(f"{lname}: did not finish within maxWait={self.max_wait}s")
            for key in [k for k in results if k[0] in started]:
                del results[key]
        return dict(results), list(failures), dict(timings)

    def _fit_eval_bounded(self, lname, grid, mine, X, y, train_rows, val_rows, ctx, remaining: float):
        """:meth:`_fit_eval` under the ``maxWait`` deadline (``awaitResult(..., maxWait)``, OpValidator.scala:348):
        the learner runs on a worker thread with the caller's device and stream; if it has not returned when
        the deadline passes, its grid points are reported failed. The fit is cancelled cooperatively
        (utils/cancel.py: the learners check between rounds / iterations) and joined for a grace period; a fit
        stuck inside a long native call is then abandoned, as the reference abandons its future. An abandoned
        fit keeps running on the caller's stream -- later learners' work is stream-ordered behind it, which is
        safe -- and on its native tree-grower slot lane, which is quarantined until its thread exits
        (models/tree_engine.py quarantine_lane) so no later grower shares its grow-only device buffers; it works on
        its own copy of the context. Only for learners whose jobs are local to this rank -- a spread learner's
        collectives must not be left half-way on one rank."""
        import threading
        from ..utils import cancel
        box: Dict[str, Any] = {}
        token = threading.Event()
        gpu = isinstance(X, torch.Tensor) and X.is_cuda
        dev = X.device if gpu else None
        stream = torch.cuda.current_stream(dev) if gpu else None
        ctx.setdefault("refit_states", {})     # shared by the worker's copy: the selector reads the refits
        wctx = dict(ctx)
        from ..models import tree_engine as TE
        lane = TE.slot_lane()

        def work():
            try:
                TE.set_slot_lane(lane)
                if gpu:
                    torch.cuda.set_device(dev)
                with cancel.scope(token), (torch.cuda.stream(stream) if gpu else contextlib.nullcontext()):
                    box["out"] = self._fit_eval(lname, grid, mine, X, y, train_rows, val_rows, wctx)
            except cancel.FitCancelled:
                box["cancelled"] = True
            except BaseException as e:          # noqa: BLE001  (re-raised below)
                box["err"] = e

        th = threading.Thread(target=work, name=f"fit-{lname}", daemon=True)
        th.start()
        th.join(max(0.0, remaining))
        if th.is_alive():
            token.set()
            th.join(_cancel_grace_s())      # returns at the fit's next cancellation check
            if th.is_alive():           # inside a long native call: abandoned, as the reference's future is
                TE.quarantine_lane(lane, th)
                log.warning("Model %s did not stop within %.0fs of its maxWait cancellation; abandoned", lname,
                            _cancel_grace_s())
            log.warning("Model %s did not finish within maxWait=%ss; its %d fits are dropped", lname,
                        self.max_wait, len(mine))
            return {}, [f"{lname}: did not finish within maxWait={self.max_wait}s"]
        if "err" in box:
            raise box["err"]
        if box.get("cancelled"):
            return {}, [f"{lname}: did not finish within maxWait={self.max_wait}s"]
        return box["out"]

    def _fit_eval(self, lname, grid, mine, X, y, train_rows, val_rows, ctx):
        """Fit + score one learner's jobs as one batch. A failing batch is retried one grid point at a
        time, so only the failing (estimator, ParamMap) fits are dropped, as the reference's per-fit
        ``Future.recover`` does (OpValidator.scala:318-328)."""
        results: Dict[Tuple[int, int, int], float] = {}
        failures: List[str] = []

        def run(batch):
            learner = learner_class(lname)()
            fjobs = [FitJob(dict(learner.defaults, **grid[g]), train_rows[k][0], train_rows[k][1])
                     for _, (_, g, k) in batch]
            # speculative refits (model_selector.py): each grid point's fit on the selector's full training
            # rows joins the CV batch of a batched learner on one rank; the selector uses the winner's
            refit = ctx.get("refit_job") if (getattr(learner, "batched_refit", False) and D.world() == 1) else None
            extra = sorted({g for _, (_, g, _) in batch}) if refit is not None else []
            fjobs += [FitJob(dict(learner.defaults, **grid[g]), refit[0], refit[1]) for g in extra]
            tp0 = _phase_clock(X)
            states = learner.fit_batch(X, y, fjobs, context=ctx)
            tp1 = _phase_clock(X)
            if extra:
                store = ctx.setdefault("refit_states", {})
                for g, st in zip(extra, states[len(batch):]):
                    store[refit_key(lname, dict(learner.defaults, **grid[g]))] = st
                states = states[:len(batch)]
            preds = learner.predict_batch(states, X, [val_rows[k] for _, (_, g, k) in batch], context=ctx)
            tp2 = _phase_clock(X)
            out = {}
            # the models of one fold share its validation rows: their curves come from one segmented sort
            by_fold: Dict[int, list] = {}
            for (j, (l, g, k)), pr in zip(batch, preds):
                by_fold.setdefault(k, []).append(((l, g, k), pr))
            # TMOG_BATCH_METRIC=1: all models of a fold from one segmented sort. Measured on the headline
            # (3.3M-row folds) it is ~0.1 s per learner slower than one 1-D sort per model (the [J, n]
            # temporaries grow the allocator), so the per-model curves stay the default
            flag = os.environ.get("TMOG_BATCH_METRIC")
            use_batch = flag == "1" if flag in ("0", "1") else bool(getattr(self.evaluator, "batch_default", False))
            batch_fn = getattr(self.evaluator, "selection_metric_batch", None) if use_batch else None
            for k, items in by_fold.items():
                yv = y[val_rows[k]]
                vals = batch_fn(yv, [pr for _, pr in items]) if (batch_fn is not None and len(items) > 1) else None
                if vals is None:
                    vals = [float(self.evaluator.selection_metric(yv, *pr)) for _, pr in items]
                out.update({key: float(v) for (key, _), v in zip(items, vals)})
            if tp0 is not None:
                tp3 = _phase_clock(X)
                with _PHASE_LOCK:
                    for ph, dt in (("fit", tp1 - tp0), ("predict", tp2 - tp1), ("metric", tp3 - tp2)):
                        PHASE_TIMES[f"{lname}:{ph}"] = PHASE_TIMES.get(f"{lname}:{ph}", 0.0) + dt
            return out

        dev = X.device if isinstance(X, torch.Tensor) else None
        try:
            results.update(run(mine))
            return results, failures
        except Exception as e:
            if is_device_fault(e, dev):     # sticky: every later fit on this context would fail too
                raise DeviceFault(f"{lname}: {e!r}") from e
            log.warning("Model %s failed in model selector as a batch (%r); retrying per grid point", lname, e)
        by_grid: Dict[int, list] = {}
        for item in mine:
            by_grid.setdefault(item[1][1], []).append(item)
        for g, batch in sorted(by_grid.items()):
            try:
                results.update(run(batch))
            except Exception as e:  # failed models are dropped, as in OpValidator.getSummary
                if is_device_fault(e, dev):
                    raise DeviceFault(f"{lname} {grid[g]}: {e!r}") from e
                log.warning("Model %s with %s failed in model selector: %r", lname, grid[g], e)
                failures.append(f"{lname} {grid[g]}: {e!r}")
        return results, failures

    def _select(self, models, results, n_folds, failures, timings, t0) -> ValidationResult:
        larger = self.evaluator.is_larger_better
        evals: List[ModelEvaluation] = []
        best = None
        for li, (lname, grid) in enumerate(models):
            # grids evaluated on the max number of folds (OpCrossValidation.findBestModel)
            per = {}
            for gi in range(len(grid)):
                ms = [results[(li, gi, k)] for k in range(n_folds) if (li, gi, k) in results]
                if ms:
                    per[gi] = ms
            if not per:
                continue
            max_f = max(len(v) for v in per.values())
            for gi, ms in per.items():
                if len(ms) != max_f:
                    continue
                m = float(np.nansum(ms) / max_f)
                evals.append(ModelEvaluation(f"{lname}_{li:03d}", lname, lname,
                                             {self.evaluator.metric: m}, dict(grid[gi])))
                better = best is None or (m > best[2] if larger else m < best[2])
                if better and not math.isnan(m):
                    best = (lname, dict(grid[gi]), m)
        if best is None:
            raise RuntimeError("All models failed model selector or failed to finish within maxWait! "
                               "Models tried were: " +
                               ", ".join(f"{m[0]} -> {len(m[1])} grid points" for m in models) +
                               (f"; failures: {failures}" if failures else ""))
        timings["total"] = time.time() - t0
        return ValidationResult(best[0], best[1], best[2], evals, failures, timings)


class OpCrossValidation(OpValidator):
    validation_type = "CrossValidation"

    def __init__(self, num_folds: int = 3, **kw):
        super().__init__(**kw)
        if num_folds < 2:
            raise ValueError("numFolds must be >= 2")
        self.num_folds = num_folds

    def make_splits(self, row_ids, y):
        u = row_uniform(row_ids, self.seed, 2)
        if self.stratify and self.is_classification:
            fold = torch.empty(row_ids.shape[0], dtype=torch.int64, device=row_ids.device)
            for c in torch.unique(y):
                m = y == c
                # per class, rank the uniforms and deal folds round-robin (balanced per class)
                idx = torch.nonzero(m).reshape(-1)
                order = torch.argsort(u[idx])
                f = torch.empty_like(order)
                f[order] = torch.arange(order.numel(), device=order.device) % self.num_folds
                fold[idx] = f
        else:
            fold = torch.clamp((u * self.num_folds).to(torch.int64), max=self.num_folds - 1)
        return [(fold != k, fold == k) for k in range(self.num_folds)]

    def params(self):
        return {"numFolds": self.num_folds, "seed": self.seed, "evaluator": self.evaluator.metric,
                "stratify": self.stratify, "parallelism": self.parallelism}


class OpTrainValidationSplit(OpValidator):
    validation_type = "TrainValidationSplit"

    def __init__(self, train_ratio: float = 0.75, **kw):
        super().__init__(**kw)
        self.train_ratio = train_ratio

    def make_splits(self, row_ids, y):
        u = row_uniform(row_ids, self.seed, 3)
        tr = u < self.train_ratio
        return [(tr, ~tr)]

    def params(self):
        return {"trainRatio": self.train_ratio, "seed": self.seed, "evaluator": self.evaluator.metric,
                "stratify": self.stratify, "parallelism": self.parallelism}

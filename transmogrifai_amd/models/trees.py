"""Tree learners on the batched histogram engine.

Reference learners: ``OpDecisionTreeClassifier`` (``OpDecisionTreeClassifier.scala:47-115``),
``OpRandomForestClassifier`` (``OpRandomForestClassifier.scala:59-154``), ``OpGBTClassifier`` (``OpGBTClassifier.scala:47-142``),
``OpXGBoostClassifier`` (``OpXGBoostClassifier.scala:47-403``) and the regression counterparts. Spark MLlib
semantics reproduced: quantile split candidates (``maxBins``), Poisson(1) bootstrap per tree when
``numTrees > 1``, per-node feature subsets (``featureSubsetStrategy``: auto = sqrt / onethird),
``minInstancesPerNode``, ``minInfoGain``, gini / entropy / variance impurity, RF probability = mean of
normalized leaf distributions, GBT log-loss boosting on {-1, +1} labels with ``1/(1+exp(-2F))``.
XGBoost: second-order gain, ``min_child_weight``, ``lambda``, ``gamma`` post-pruning, ``eta``-scaled
leaves, learned default direction for missing values (``missing`` = 0.0 by default in the
reference grid), early stopping on the training ``aucpr``.

Every (config x fold x tree) of a learner grows in the same level-synchronous forest; boosting
learners advance all their models one round per engine call.
"""
from __future__ import annotations

import json
import logging
import math
import os
import threading
import time
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import tree_engine as TE
from ..utils import cancel
from .base import FitJob, Learner, OpPredictor, probability_outputs, register_learner, union_rows
from .binning import BinSpec, find_splits, quantize
from ..stages.base import register_stage
from ..ops.staging import to_device
from ..tuning.splitters import row_uniform, row_uniform_multi

log = logging.getLogger(__name__)


# --------------------------------------------------------------------------------------- context
class TreeContext:
    """Caches quantized matrices of one design matrix ``X`` per binning configuration."""

    def __init__(self, X: torch.Tensor, rows: Optional[torch.Tensor] = None):
        self.X = X
        self.rows = rows
        self._cache: Dict[tuple, tuple] = {}
        self._ready: Dict[tuple, Optional[torch.cuda.Event]] = {}
        self._lock = threading.Lock()

    def _use(self, key):
        """Entry ``key``, with the calling thread's stream ordered after the stream that quantized it (learners
        on concurrent validator lanes share this cache)."""
        ent, ev = self._cache[key], self._ready.get(key)
        if ev is not None:
            torch.cuda.current_stream(ent[1].device).wait_event(ev)
        return ent

    def binned(self, max_bins: int, missing_value: Optional[float] = None, reserve_missing: bool = False):
        key = (max_bins, missing_value, reserve_missing)
        with self._lock:
            if key not in self._cache:
                spec = find_splits(self.X, max_bins, missing_value=missing_value, reserve_missing=reserve_missing,
                                   rows=self.rows)
                Xb = quantize(self.X, spec)
                ev = None
                if Xb.is_cuda:
                    ev = torch.cuda.Event()
                    ev.record(torch.cuda.current_stream(Xb.device))
                self._cache[key], self._ready[key] = (spec, Xb), ev
            return self._use(key)

    def matching(self, spec, key=None):
        """The cached quantized matrix binned exactly as ``spec`` (optionally only entry ``key``), or None."""
        with self._lock:
            for k, v in list(self._cache.items()):
                if (key is None or k == key) and np.array_equal(v[0].thresholds, spec.thresholds) and \
                        (key is not None or v[0].missing_bin == spec.missing_bin):
                    return self._use(k)[1]
        return None


def _par(context):
    """The validator's intra-job parallel context (parallel/learner_parallel.py), if any."""
    par = context.get("par") if isinstance(context, dict) else None
    return par if (par is not None and par.world > 1) else None


_CTX_LOCK = threading.Lock()


def _ctx(X, context):
    if isinstance(context, TreeContext) and context.X is X:
        return context
    if isinstance(context, dict):
        with _CTX_LOCK:         # learners running concurrently (validator lanes) share one binning cache
            c = context.get("tree")
            if c is None or c.X is not X:
                c = TreeContext(X, context.get("tree_rows"))
                context["tree"] = c
        return c
    return TreeContext(X)


def _subset_size(strategy, F: int, classification: bool, num_trees: int) -> int:
    s = str(strategy).lower()
    if s == "auto":
        if num_trees == 1:
            return F
        s = "sqrt" if classification else "onethird"
    if s == "all":
        return F
    if s == "sqrt":
        return int(math.ceil(math.sqrt(F)))
    if s == "log2":
        return max(1, int(math.ceil(math.log2(F))))
    if s == "onethird":
        return int(math.ceil(F / 3.0))
    try:
        v = float(s)
    except ValueError:
        raise ValueError(f"bad featureSubsetStrategy {strategy}")
    if v >= 1.0 and float(v).is_integer():
        return min(F, int(v))
    return max(1, int(math.ceil(v * F)))


def bootstrap_weights(rows: torch.Tensor, seed: int, rate: float) -> torch.Tensor:
    """Poisson(``rate``) bootstrap multiplicity per row (Spark RF ``BaggedPoint`` with replacement).

    Drawn on the rows' device from a counter-based per-(seed, row id) uniform and the inverse Poisson
    CDF, so the draw is identical on every device/rank and costs one elementwise pass instead of a
    host RNG stream per tree.
    """
    u = row_uniform(rows, seed, 23)
    k = torch.zeros(rows.shape[0], dtype=torch.int64, device=rows.device)
    p = math.exp(-rate)
    cdf = p
    for i in range(1, 40):
        k += (u >= cdf).to(torch.int64)
        p = p * rate / i
        cdf += p
        if 1.0 - cdf < 1e-12:
            break
    return k


def bootstrap_weights_multi(rows: torch.Tensor, seeds, rate: float) -> torch.Tensor:
    """``bootstrap_weights`` for several trees at once: ``int64 [len(seeds), n]`` (bit-identical per tree)."""
    u = row_uniform_multi(rows, seeds, 23)
    k = torch.zeros(u.shape, dtype=torch.int64, device=rows.device)
    p = math.exp(-rate)
    cdf = p
    for i in range(1, 40):
        k += (u >= cdf).to(torch.int64)
        p = p * rate / i
        cdf += p
        if 1.0 - cdf < 1e-12:
            break
    return k


def _rows(job: FitJob, N, dev):
    return torch.arange(N, device=dev) if job.rows is None else job.rows.to(dev)


def _add_tree_margins(Fm: torch.Tensor, forest: "TE.Forest", Xb, act: List[int], wgts: List[float],
                      tjobs) -> None:
    """``Fm[act[k]] += wgts[k] * tree_k(x)`` for the trees of one boosting round.

    Trees grown with ``collect_leaves`` know the leaf of every training entry, so the update is a
    gather of leaf values scattered into the margins (each (model, row) pair occurs once, no atomics).
    Rows outside a tree's training entries (zero-weight subsampled rows) need the tree walk."""
    la = getattr(forest, "leaf_assign", None)
    if la is None or any(j.weights is not None for j in tjobs):
        preds = TE.forest_predict(forest, Xb, [None] * len(act), [[k] for k in range(len(act))])
        for k, p in enumerate(act):
            Fm[p] += wgts[k] * preds[k][:, 0].to(torch.float64)
        return
    N = Fm.shape[1]
    t = la.entry_tree()
    pk = TE._Pack(Fm.device)
    i_p, i_w = pk.add(np.asarray(act, np.int64)), pk.add(np.asarray(wgts, np.float64))
    dv = pk.ship()
    p_of, w_of = dv[i_p], dv[i_w]
    idx = p_of[t] * N + la.row_ids()
    val = la.entry_value()[:, 0].to(torch.float64) * w_of[t]
    flat = Fm.view(-1)
    flat[idx] = flat[idx] + val


def _model_rows_forest_predict(forest, Xb, rows_list, trees_list, tree_weight=None):
    return TE.forest_predict(forest, Xb, rows_list, trees_list, tree_weight)


# ------------------------------------------------------------------------------------ RF / DT
class _ForestLearner(Learner):
    classification = True
    default_trees = 20
    is_forest = True
    parallel = None             # forests: (grid x fold) jobs sharded over ranks

    def _num_classes(self, y):
        return max(2, int(y.max().item()) + 1) if y.numel() else 2

    def fit_batch(self, X, y, jobs, context=None):
        if not jobs:
            return []
        ctx = _ctx(X, context)
        dev = X.device
        N, F = X.shape
        out: List[Optional[dict]] = [None] * len(jobs)
        # shared-forest registry for predict_batch (id(state) -> (state, share key, depth, gain)): the grid
        # points pruned from one grown forest are scored in one walk of it (TE.forest_predict_multi)
        self._share_reg: Dict[int, tuple] = {}
        self._share_forest: Dict[tuple, "TE.Forest"] = {}
        # group jobs by binning
        groups: Dict[int, List[int]] = {}
        for i, j in enumerate(jobs):
            groups.setdefault(int(j.params.get("max_bins", 32)), []).append(i)
        K = self._num_classes(y) if self.classification else 1
        for mb, idxs in groups.items():
            cancel.check()
            spec, Xb = ctx.binned(mb)
            yg = y
            jrows = {i: _rows(jobs[i], N, dev) for i in idxs}
            if all(jobs[i].rows is not None for i in idxs):
                # grow over the union of the training rows only (smaller gather footprint, and the
                # packed 24-bit row ids then index the compacted matrix)
                U, parts = union_rows([jrows[i] for i in idxs], N, dev)
                if U.numel() < N:
                    Xb = Xb.index_select(0, U)
                    yg = y.to(dev).index_select(0, U)
                    jrows = {i: r for i, r in zip(idxs, parts)}
            tjobs, owner = [], []
            # Bootstraps are drawn per (training rows, seed): grid points of one CV fold share theirs,
            # as Spark RF does for equal seeds on equal data (one draw per fold instead of per grid point)
            forests_only = self.is_forest and all(
                int(jobs[i].params.get("num_trees", self.default_trees)) > 1 for i in idxs)
            boot: Dict[tuple, tuple] = {}
            row_keys: Dict[tuple, int] = {}
            root_parts, root_counts = [], []
            # Grid points that differ only in maxDepth / minInfoGain share their trees: one forest is grown
            # at the deepest depth and smallest gain threshold of its share group and the others are
            # pruned out of it (TE.prune_forest) -- for the default RF grid 2 grown forests per fold instead
            # of 18, ~5x fewer tree levels. (Same bootstrap and seed as each grid point had before; the
            # per-node feature-subset draws come from the group's stream, as for any grid composition.)
            grow, members = _forest_share_groups(jobs, idxs, forests_only)
            for i in grow:
                p = dict(jobs[i].params)
                md, mg = members[i][1], members[i][2]
                p["max_depth"], p["min_info_gain"] = md, mg
                nt = int(p.get("num_trees", self.default_trees)) if self.is_forest else 1
                rows = jrows[i]
                sub = _subset_size(p.get("feature_subset_strategy", "auto"), F, self.classification, nt)
                tp = TE.TreeParams(max_depth=int(p.get("max_depth", 5)),
                                   min_instances=float(p.get("min_instances_per_node", 1)),
                                   min_info_gain=float(p.get("min_info_gain", 0.0)), feature_subset=sub)
                rate = float(p.get("subsampling_rate", 1.0))
                if forests_only:
                    src = jobs[i].rows
                    rk = ("all",) if src is None else (src.data_ptr(), int(src.numel()), str(src.device))
                    seed = int(p.get("seed", 0)) + 7919 * row_keys.setdefault(rk, len(row_keys))
                    key = (rk, seed, nt, rate)
                    if key not in boot:
                        packed, cnts = TE.bootstrap_pack(rows, [seed * 1009 + t for t in range(nt)], rate,
                                                         TE.wide_rows(int(Xb.shape[0])))
                        boot[key] = (packed, cnts, np.concatenate([[0], np.cumsum(cnts)]))
                    packed, cnts, offs = boot[key]
                    for t in range(nt):
                        root_parts.append(packed[int(offs[t]):int(offs[t + 1])])
                        root_counts.append(int(cnts[t]))
                        tjobs.append(TE.TreeJob(0, tp, rows, None, seed + t))
                        owner.append(i)
                    continue
                seed = int(p.get("seed", 0)) + 7919 * i
                wall = bootstrap_weights_multi(rows, [seed * 1009 + t for t in range(nt)], rate) if nt > 1 else None
                for t in range(nt):
                    if nt > 1:
                        w = wall[t]
                    elif rate < 1.0:
                        w = (row_uniform(rows, seed * 1009 + t, 17) < rate).to(torch.int64)
                    else:
                        w = jobs[i].weights.to(dev).round().to(torch.int64) if jobs[i].weights is not None else None
                    tjobs.append(TE.TreeJob(0, tp, rows, w, seed + t))
                    owner.append(i)
            root = (torch.cat(root_parts), root_counts) if forests_only and root_parts else None
            # single trees (no per-node feature subsets) grow feature-parallel over the ranks
            par = _par(context)
            fp = None
            if par is not None and all(t.params.feature_subset is None or t.params.feature_subset >= F
                                       for t in tjobs):
                fp = TE.fp_plan(Xb, spec.n_bins, par, sparse=False)
            if self.classification:
                forest = TE.grow_forest(Xb, spec.n_bins, tjobs, mode=TE.MODE_CLS,
                                        kind=TE.KINDS[jobs[idxs[0]].params.get("impurity", "gini")], n_classes=K,
                                        y=yg, B=mb, rng_seed=int(jobs[idxs[0]].params.get("seed", 0)), root=root,
                                        fp=fp)
            else:
                forest = TE.grow_forest(Xb, spec.n_bins, tjobs, mode=TE.MODE_VAR, kind=TE.KIND_VARIANCE,
                                        t1=yg.to(torch.float32)[None, :], B=mb,
                                        rng_seed=int(jobs[idxs[0]].params.get("seed", 0)), root=root, fp=fp)
            owner = np.asarray(owner)
            for g in grow:
                ts = np.nonzero(owner == g)[0]
                sub = Forest_subset(forest, ts)
                md, mg = members[g][1], members[g][2]
                skey = (mb, g)
                if len(members[g][0]) > 1:
                    self._share_forest[skey] = sub
                for i in members[g][0]:
                    pi = jobs[i].params
                    di, gi = int(pi.get("max_depth", 5)), float(pi.get("min_info_gain", 0.0))
                    fi = sub if (di, gi) == (md, mg) else TE.prune_forest(sub, di, gi)
                    out[i] = {"forest": fi.to_state(), "bins": spec.to_state(), "n_classes": K,
                              "num_trees": len(ts), "max_bins": mb, "n_features": F}
                    if len(members[g][0]) > 1:
                        self._share_reg[id(out[i])] = (out[i], skey, di, gi)
        return out

    # -- prediction
    def _forest(self, state):
        if "_forest" not in state:
            state["_forest"] = TE.Forest.from_state(state["forest"])
            state["_bins"] = BinSpec.from_state(state["bins"])
        return state["_forest"], state["_bins"]

    def _binned(self, state, X, context):
        forest, spec = self._forest(state)
        if context is not None:
            ctx = _ctx(X, context)
            key = (int(state["max_bins"]), spec.missing_value, spec.missing_bin >= 0)
            Xb = ctx.matching(spec, key)
            if Xb is not None:
                return forest, Xb
        return forest, quantize(X, spec)

    def raw_sum(self, state, X, rows=None, context=None):
        forest, Xb = self._binned(state, X, context)
        return TE.forest_predict(forest, Xb, [rows], [list(range(forest.n_trees))])[0].to(torch.float64)

    def predict(self, state, X, context=None):
        return self._outputs(state, self.raw_sum(state, X, None, context))

    def predict_batch(self, states, X, rows, context=None):
        if not states:
            return []
        # one traversal launch for all models that share a binning
        groups: Dict[int, List[int]] = {}
        for i, s in enumerate(states):
            groups.setdefault(int(s["max_bins"]), []).append(i)
        res = [None] * len(states)
        reg = getattr(self, "_share_reg", {})
        for mb, idxs in groups.items():
            # grid points pruned from one grown forest and scored on the same rows: one shared walk
            shared: Dict[tuple, List[int]] = {}
            for i in idxs:
                e = reg.get(id(states[i]))
                if e is not None and e[0] is states[i] and e[1] in self._share_forest:
                    shared.setdefault((e[1], id(rows[i])), []).append(i)
            shared = {k: v for k, v in shared.items() if len(v) > 1 and all(rows[j] is rows[v[0]] for j in v)}
            if shared:
                _, Xb = self._binned(states[idxs[0]], X, context)
                keys = list(shared)
                grown = [self._share_forest[k[0]] for k in keys]
                big = TE.Forest.concat(grown)
                off = np.cumsum([0] + [f.n_trees for f in grown])
                raws = TE.forest_predict_multi(
                    big, Xb, [rows[shared[k][0]] for k in keys],
                    [list(range(off[n], off[n + 1])) for n in range(len(keys))],
                    [[reg[id(states[i])][2:4] for i in shared[k]] for k in keys])
                for n, k in enumerate(keys):
                    for i, raw in zip(shared[k], raws[n]):
                        res[i] = self._outputs(states[i], raw.to(torch.float64))
                idxs = [i for i in idxs if res[i] is None]
                if not idxs:
                    continue
            forests = [self._forest(states[i])[0] for i in idxs]
            _, Xb = self._binned(states[idxs[0]], X, context)
            big = TE.Forest.concat(forests)
            off = np.cumsum([0] + [f.n_trees for f in forests])
            raws = TE.forest_predict(big, Xb, [rows[i] for i in idxs],
                                     [list(range(off[k], off[k + 1])) for k in range(len(idxs))])
            for k, i in enumerate(idxs):
                res[i] = self._outputs(states[i], raws[k].to(torch.float64))
        return res

    def _outputs(self, state, raw):
        if not self.classification:
            nt = max(1, int(state.get("num_trees", 1)))
            p = raw[:, 0] / (nt if self.is_forest else 1)
            e = torch.zeros(p.shape[0], 0, dtype=torch.float64, device=p.device)
            return p, e, e
        s = raw.sum(1, keepdim=True)
        prob = torch.where(s > 0, raw / s.clamp_min(1e-300), torch.full_like(raw, 1.0 / raw.shape[1]))
        if not self.is_forest:
            raw = raw  # DT raw = leaf distribution (normalized counts)
        pred = torch.argmax(raw, 1).to(torch.float64)
        return pred, raw, prob

    def feature_contributions(self, state, d):
        forest, _ = self._forest(state)
        return forest.feature_importance(d)


def _forest_share_groups(jobs, idxs, forests_only):
    """``(grow, members)``: the job indices to grow, and per grown index ``(member job indices, max_depth,
    min_info_gain)`` it is grown with. Jobs share when everything but maxDepth / minInfoGain matches
    (training rows, seed, trees, sampling, minInstancesPerNode, impurity, subset strategy); off with
    ``TMOG_RF_SHARE=0`` and for single trees (their weights / sampling are per job)."""
    if not forests_only or os.environ.get("TMOG_RF_SHARE", "1") == "0":
        return list(idxs), {i: ([i], int(jobs[i].params.get("max_depth", 5)),
                                float(jobs[i].params.get("min_info_gain", 0.0))) for i in idxs}
    by_key: Dict[tuple, List[int]] = {}
    for i in idxs:
        p = jobs[i].params
        src = jobs[i].rows
        rk = ("all",) if src is None else (src.data_ptr(), int(src.numel()), str(src.device))
        rest = tuple(sorted((k, repr(v)) for k, v in p.items() if k not in ("max_depth", "min_info_gain")))
        by_key.setdefault((rk, rest), []).append(i)
    grow, members = [], {}
    for ms in by_key.values():
        g = ms[0]
        grow.append(g)
        members[g] = (ms, max(int(jobs[i].params.get("max_depth", 5)) for i in ms),
                      min(float(jobs[i].params.get("min_info_gain", 0.0)) for i in ms))
    return grow, members


def Forest_subset(forest: TE.Forest, trees: np.ndarray) -> TE.Forest:
    return TE.Forest.concat([forest.tree(int(t)) for t in trees]) if len(trees) else forest


@register_learner
class RandomForestClassifierLearner(_ForestLearner):
    name = "OpRandomForestClassifier"
    problem = "multiclass"
    defaults = {"max_depth": 5, "max_bins": 32, "min_instances_per_node": 1, "min_info_gain": 0.0,
                "num_trees": 20, "impurity": "gini", "subsampling_rate": 1.0, "feature_subset_strategy": "auto",
                "seed": 0}


@register_learner
class DecisionTreeClassifierLearner(_ForestLearner):
    name = "OpDecisionTreeClassifier"
    problem = "multiclass"
    is_forest = False
    parallel = "features"
    defaults = {"max_depth": 5, "max_bins": 32, "min_instances_per_node": 1, "min_info_gain": 0.0,
                "impurity": "gini", "seed": 0}


@register_learner
class RandomForestRegressorLearner(_ForestLearner):
    name = "OpRandomForestRegressor"
    problem = "regression"
    classification = False
    defaults = {"max_depth": 5, "max_bins": 32, "min_instances_per_node": 1, "min_info_gain": 0.0,
                "num_trees": 20, "impurity": "variance", "subsampling_rate": 1.0,
                "feature_subset_strategy": "auto", "seed": 0}


@register_learner
class DecisionTreeRegressorLearner(_ForestLearner):
    name = "OpDecisionTreeRegressor"
    problem = "regression"
    classification = False
    is_forest = False
    parallel = "features"
    defaults = {"max_depth": 5, "max_bins": 32, "min_instances_per_node": 1, "min_info_gain": 0.0,
                "impurity": "variance", "seed": 0}


# -------------------------------------------------------------------------------- boosting
def _boost_job_bytes(job, n_rows: int, n_features: int = 0, n_bins: int = 64) -> int:
    """Device bytes one boosting job holds while its batch runs: its margin row (fp64) and (g, h) rows (fp32) over
    the batch's rows; per training entry the grower's ping-pong entries and staged (g, h), the leaf assignment and
    the root packing (~40 bytes); and the grower's two level histograms -- F x (B + 1) x 2 statistics x 8 bytes
    for each node of the widest level (2^(max_depth - 1), at most one per training row), the size
    ``tree_resident.hip`` allocates per job group."""
    n_train = int(job.rows.numel()) if job.rows is not None else n_rows
    depth = int(job.params.get("max_depth", 6)) if getattr(job, "params", None) else 6
    nodes = min(1 << max(depth - 1, 0), max(n_train, 1))
    hist = 2 * n_features * (n_bins + 1) * 2 * 8 * nodes
    return 16 * n_rows + 40 * n_train + hist


def _budget_chunks(job_bytes: Sequence[int], dev, frac: Optional[float] = None) -> List[tuple]:
    """Consecutive job ranges whose summed device footprint fits ``frac`` of the memory available now (free device
    memory plus torch's cached-but-unused blocks) -- a batch is sized from a budget up front instead of hitting
    out-of-memory and being retried grid point by grid point. One range on the CPU or when everything fits;
    ``TMOG_TREE_BUDGET_FRAC`` (default 0.6) sets the fraction."""
    n = len(job_bytes)
    if n <= 1 or dev.type != "cuda":
        return [(0, n)]
    frac = float(os.environ.get("TMOG_TREE_BUDGET_FRAC", "0.6")) if frac is None else frac
    free, _ = torch.cuda.mem_get_info(dev)
    cached = torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)
    # learner lanes running beside this fit allocate from the same free memory: each lane gets its share
    from ..ops import streams as SP
    budget = max(1, int(frac * (free + max(cached, 0)) / SP.active_lanes()))
    if sum(job_bytes) <= budget:
        return [(0, n)]
    out, lo, acc = [], 0, 0
    for i, b in enumerate(job_bytes):
        if i > lo and acc + b > budget:
            out.append((lo, i))
            lo, acc = i, 0
        acc += b
    out.append((lo, n))
    log.info("boosting batch of %d jobs (%.1f GB) split into %d budgeted chunks (budget %.1f GB)", n,
             sum(job_bytes) / 1e9, len(out), budget / 1e9)
    return out


class _BoostLearner(Learner):
    """Shared boosting loop: all jobs advance one round per engine call."""
    classification = True
    parallel = "features"       # every rank grows every tree over its feature slice

    def _rounds(self, p):
        raise NotImplementedError

    def fit_batch(self, X, y, jobs, context=None):
        if not jobs:
            return []
        ctx = _ctx(X, context)
        dev = X.device
        N, F = X.shape
        out = [None] * len(jobs)
        groups: Dict[tuple, List[int]] = {}
        for i, j in enumerate(jobs):
            groups.setdefault(self._bin_key(j.params), []).append(i)
        for key, idxs in groups.items():
            spec, Xb = ctx.binned(*key)
            gjobs = [jobs[i] for i in idxs]
            yd = y.to(dev)
            NU = N
            if all(j.rows is not None for j in gjobs):
                # boost only over the union of the jobs' training rows: gradients, margins and the
                # per-round prediction pass then scale with the (down-sampled) training sets, not N
                U, parts = union_rows([j.rows for j in gjobs], N, dev)
                if U.numel() < N:
                    Xb = Xb.index_select(0, U)
                    yd = yd.index_select(0, U)
                    NU = int(U.numel())
                    gjobs = [FitJob(j.params, r, j.weights) for j, r in zip(gjobs, parts)]
            res = []
            for lo, hi in _budget_chunks([_boost_job_bytes(j, NU, F, key[0]) for j in gjobs], dev):
                res += self._boost(Xb, spec, yd, gjobs[lo:hi], NU, F, dev, key[0], par=_par(context))
            for k, i in enumerate(idxs):
                out[i] = res[k]
        return out

    def _bin_key(self, p):
        return (int(p.get("max_bins", 32)), None, False)

    def _forest(self, state):
        if "_forest" not in state:
            state["_forest"] = TE.Forest.from_state(state["forest"])
            state["_bins"] = BinSpec.from_state(state["bins"])
        return state["_forest"], state["_bins"]

    def margin(self, state, X, rows=None, context=None):
        forest, spec = self._forest(state)
        Xb = None
        if context is not None:
            Xb = _ctx(X, context).matching(spec)
        if Xb is None:
            Xb = quantize(X, spec)
        m = TE.forest_predict(forest, Xb, [rows], [list(range(forest.n_trees))],
                              np.asarray(state["tree_weights"], np.float32))[0][:, 0].to(torch.float64)
        return m + float(state.get("base_margin", 0.0))

    def predict(self, state, X, context=None):
        return self._outputs(state, self.margin(state, X, None, context))

    def predict_batch(self, states, X, rows, context=None):
        return [self._outputs(s, self.margin(s, X, r, context)) for s, r in zip(states, rows)]

    def feature_contributions(self, state, d):
        forest, _ = self._forest(state)
        return forest.feature_importance(d)


@register_learner
class GBTClassifierLearner(_BoostLearner):
    """Spark GBT with log loss (``OpGBTClassifier.scala:47-142``)."""
    name = "OpGBTClassifier"
    defaults = {"max_depth": 5, "max_bins": 32, "min_instances_per_node": 1, "min_info_gain": 0.0, "max_iter": 20,
                "step_size": 0.1, "subsampling_rate": 1.0, "impurity": "variance", "loss_type": "logistic",
                "seed": 0}

    def _target(self, yy, Fm, first):
        ys = 2 * yy - 1
        if first:
            return ys
        return 4 * ys / (1 + torch.exp(2 * ys * Fm))

    def _boost(self, Xb, spec, y, jobs, N, F, dev, mb, par=None):
        P = len(jobs)
        rows = [_rows(j, N, dev) for j in jobs]
        iters = [int(j.params.get("max_iter", 20)) for j in jobs]
        fp = TE.fp_plan(Xb, spec.n_bins, par, sparse=False) if par is not None else None
        Fm = torch.zeros(P, N, dtype=torch.float64, device=dev)
        yy = y.to(torch.float64)
        forests, weights = [[] for _ in range(P)], [[] for _ in range(P)]
        for it in range(max(iters)):
            cancel.check()
            act = [p for p in range(P) if it < iters[p]]
            t1 = torch.stack([self._target(yy, Fm[p], it == 0) for p in range(P)]).to(torch.float32)
            tjobs = []
            for p in act:
                pr = jobs[p].params
                tp = TE.TreeParams(max_depth=int(pr.get("max_depth", 5)),
                                   min_instances=float(pr.get("min_instances_per_node", 1)),
                                   min_info_gain=float(pr.get("min_info_gain", 0.0)))
                r = rows[p]
                rate = float(pr.get("subsampling_rate", 1.0))
                w = None
                if rate < 1.0:
                    g = torch.Generator().manual_seed(int(pr.get("seed", 0)) + 131 * it + p)
                    w = (torch.rand(r.numel(), generator=g) < rate).to(torch.int64).to(dev)
                tjobs.append(TE.TreeJob(p, tp, r, w))
            forest = TE.grow_forest(Xb, spec.n_bins, tjobs, mode=TE.MODE_VAR, kind=TE.KIND_VARIANCE, t1=t1, B=mb,
                                    collect_leaves=True, fp=fp)
            wgts = [1.0 if it == 0 else float(jobs[p].params.get("step_size", 0.1)) for p in act]
            _add_tree_margins(Fm, forest, Xb, act, wgts, tjobs)
            for k, p in enumerate(act):
                forests[p].append(forest.tree(k))
                weights[p].append(wgts[k])
        return [{"forest": TE.Forest.concat(forests[p]).to_state(), "bins": spec.to_state(),
                 "tree_weights": np.asarray(weights[p], np.float32), "n_classes": 2, "max_bins": mb,
                 "num_trees": len(forests[p])} for p in range(P)]

    def _outputs(self, state, m):
        p1 = 1.0 / (1.0 + torch.exp(-2.0 * m))
        raw = torch.stack([-m, m], 1)
        prob = torch.stack([1 - p1, p1], 1)
        return (p1 > 0.5).to(torch.float64), raw, prob


@register_learner
class GBTRegressorLearner(GBTClassifierLearner):
    name = "OpGBTRegressor"
    problem = "regression"
    classification = False
    defaults = {"max_depth": 5, "max_bins": 32, "min_instances_per_node": 1, "min_info_gain": 0.0, "max_iter": 20,
                "step_size": 0.1, "subsampling_rate": 1.0, "impurity": "variance", "loss_type": "squared",
                "seed": 0}

    def _target(self, yy, Fm, first):
        if first:
            return yy
        return 2 * (yy - Fm)   # -gradient of squared error (Spark SquaredError)

    def _outputs(self, state, m):
        e = torch.zeros(m.shape[0], 0, dtype=torch.float64, device=m.device)
        return m, e, e


def _run_parts(dev, parts, fn):
    """Run ``fn(jobs, slot_base, groups)`` for every part concurrently: the first part on the caller's thread
    and stream, every other part on a host thread of its own and a side stream leased from ops/streams.py
    (ordered after the caller's stream, which then waits for all of them). With fewer side streams free than
    parts, parts are merged (jobs of part k go to part k mod the streams available): the trees of a job do
    not depend on the jobs grown beside it. Native calls release the GIL, so the parts' host work and GPU work
    interleave. The first error is re-raised."""
    import threading
    from ..ops import streams as SP
    cur = torch.cuda.current_stream(dev)
    side = SP.lease(dev, len(parts) - 1)
    try:
        k_used = 1 + len(side)
        if k_used < len(parts):
            merged = [list(p) for p in parts[:k_used]]
            for k, p in enumerate(parts[k_used:], start=k_used):
                merged[k % k_used][0] = list(merged[k % k_used][0]) + list(p[0])
            parts = [tuple(p) for p in merged]
        for s in side:
            s.wait_stream(cur)
        errs = []
        lane = TE.slot_lane()           # the caller's native slot lane (concurrent learners) carries over
        token = cancel.current()        # and its maxWait cancellation token

        def work(k):
            try:
                torch.cuda.set_device(dev)
                TE.set_slot_lane(lane)
                with cancel.scope(token), torch.cuda.stream(side[k - 1]):
                    fn(*parts[k])
            except BaseException as e:          # noqa: BLE001  (re-raised on the caller's thread)
                errs.append(e)

        th = [threading.Thread(target=work, args=(k,), daemon=True, name=f"boost-part-{k}")
              for k in range(1, len(parts))]
        # a thread returning from a native call must win the GIL back from the one running Python: the
        # default 5 ms switch interval would stall it for up to a whole boosting round
        from ..utils.threads import fast_switch
        with fast_switch(float(os.environ.get("TMOG_PIPE_SWITCH_S", "5e-5"))):
            for t in th:
                t.start()
            try:
                fn(*parts[0])
            except BaseException as e:          # noqa: BLE001
                errs.append(e)
            for t in th:
                t.join()
        for s in side:
            cur.wait_stream(s)
        if errs:
            raise errs[0]
    finally:
        SP.release(dev, side)


# TMOG_XGB_PROFILE=1: per pipelined part, host seconds spent before / inside / after the native grower and in
# the early-stopping read-back, printed to stderr after each XGBoost fit (diagnostics)
_XGB_PROF: Optional[Dict[int, Dict[str, float]]] = {} if os.environ.get("TMOG_XGB_PROFILE") == "1" else None


@register_learner
class XGBoostClassifierLearner(_BoostLearner):
    """Newton boosting with XGBoost semantics (binary:logistic)."""
    name = "OpXGBoostClassifier"
    defaults = {"num_round": 100, "eta": 0.3, "gamma": 0.0, "max_depth": 6, "min_child_weight": 1.0,
                "reg_lambda": 1.0, "missing": float("nan"), "max_bins": 64, "num_early_stopping_rounds": 0,
                "eval_metric": "aucpr", "maximize_evaluation_metrics": True, "objective": "binary:logistic",
                "base_score": 0.5, "subsample": 1.0, "colsample_bytree": 1.0, "seed": 0}

    def _bin_key(self, p):
        miss = p.get("missing", float("nan"))
        mv = None if (miss is None or (isinstance(miss, float) and math.isnan(miss))) else float(miss)
        return (int(p.get("max_bins", 64)), mv, True)

    def _grad(self, yy, Fm):
        p = torch.sigmoid(Fm)
        return p - yy, (p * (1 - p)).clamp_min(1e-16)

    def _base_margin(self, bs):
        bs = min(max(bs, 1e-12), 1 - 1e-12)
        return math.log(bs / (1 - bs))

    def _boost(self, Xb, spec, y, jobs, N, F, dev, mb, par=None):
        from ..evaluators.metrics import binned_aupr_from_counts, binned_aupr_multi
        t_setup0 = time.perf_counter()
        P = len(jobs)
        rows = [_rows(j, N, dev) for j in jobs]
        rounds = [int(j.params.get("num_round", 100)) for j in jobs]
        esr = [int(j.params.get("num_early_stopping_rounds", 0)) for j in jobs]
        base = [self._base_margin(float(j.params.get("base_score", 0.5))) for j in jobs]
        Fm = to_device(base, dev, np.float64)[:, None].repeat(1, N)
        yy = y.to(torch.float64)
        ylab = [yy[r] for r in rows]
        forests, weights = [[] for _ in range(P)], [[] for _ in range(P)]
        best = [-float("inf")] * P
        best_round = [0] * P
        stopped = [False] * P
        # fused round epilogue on the device (ops/csrc/hip/boost_kernels.hip): margins, next gradients
        # and the early-stopping AuPR counts in one launch per round instead of ~60 torch ops
        fused = dev.type == "cuda" and all(float(j.params.get("subsample", 1.0)) >= 1.0 for j in jobs) and \
            os.environ.get("TMOG_XGB_FUSED", "1") != "0"
        AUC_BINS = 1 << 16
        # Column order for growth: multi-bin columns first, then the one-present-bin ones (one-hot /
        # null indicators), physically -- the histogram kernel's multi-bin groups then gather contiguous
        # row bytes. It is the order the grower would use anyway (common/tree_grow.hpp), so trees are
        # unchanged; split features are mapped back to the original columns after each round.
        Xg, n_bins_g, colperm = Xb, spec.n_bins, None
        if spec.missing_bin > 0 and os.environ.get("TMOG_XGB_COLPERM") != "0":
            nb_all = np.asarray(spec.n_bins)
            order = np.concatenate([np.nonzero(nb_all != 1)[0], np.nonzero(nb_all == 1)[0]])
            if not np.array_equal(order, np.arange(nb_all.size)):
                colperm = order.astype(np.int64)
                Xg = Xb.index_select(1, torch.as_tensor(colperm, device=dev)).contiguous()
                n_bins_g = nb_all[colperm]
        # wide-load histogram items (tree_kernels.hip hist_wide_item) read 4 bins per lane with dword loads:
        # pad the growth matrix to a dword row stride with columns that hold only the missing bin (one
        # "present" bin that no row has: they can never split, and are mapped to column 0 if ever read)
        if dev.type == "cuda" and spec.missing_bin > 0 and os.environ.get("TMOG_HIST_WIDE") != "0" \
                and Xg.shape[1] % 4 != 0:
            F0 = Xg.shape[1]
            F4 = (F0 + 3) // 4 * 4
            pad = torch.full((Xg.shape[0], F4 - F0), spec.missing_bin, dtype=Xg.dtype, device=dev)
            Xg = torch.cat([Xg, pad], 1).contiguous()
            n_bins_g = np.concatenate([np.asarray(n_bins_g), np.ones(F4 - F0, dtype=np.asarray(n_bins_g).dtype)])
            base_perm = colperm if colperm is not None else np.arange(F0, dtype=np.int64)
            colperm = np.concatenate([base_perm, np.zeros(F4 - F0, np.int64)])
        # compact histogram matrix: the leading multi-bin columns of Xg at a 64-byte row stride (aligned row
        # segments, and a footprint that fits the Infinity Cache better than the full padded rows); only the
        # wide-load histogram items read it (tree_grow.hpp GrowArgs.Xh)
        Xh = None
        if dev.type == "cuda" and spec.missing_bin > 0 and os.environ.get("TMOG_HIST_COMPACT", "1") != "0":
            nbg = np.asarray(n_bins_g)
            n_multi = int(np.argmax(nbg == 1)) if (nbg == 1).any() else nbg.size
            Fh = (n_multi + 63) // 64 * 64
            if 0 < n_multi and Fh < Xg.shape[1] and (nbg[:n_multi] != 1).all():
                Xh = Xg[:, :Fh].contiguous()
        # feature-parallel over the ranks: this rank's slice of the growth-order feature lists
        fp = TE.fp_plan(Xg, n_bins_g, par, sparse=spec.missing_bin >= 0) if par is not None else None
        # one-hot / null-indicator columns: histogram from the rows' CSR lists (tree_kernels.hip)
        csr = TE.onebin_csr(Xg, n_bins_g, cols=None if fp is None else fp.one_cols) \
            if (dev.type == "cuda" and spec.missing_bin > 0) else None
        # feature-major copy for the partition kernel's split-column reads (tree_grow.hpp GrowArgs.XbT)
        XgT = Xg.t().contiguous() if (dev.type == "cuda" and os.environ.get("TMOG_PART_T", "1") != "0") else None
        yf = yy.to(torch.float32).contiguous()
        G = H = None
        if fused:         # shared [P, N] statistics: each job's row is only touched by its own part
            G = torch.zeros(P, N, dtype=torch.float32, device=dev)
            H = torch.zeros(P, N, dtype=torch.float32, device=dev)
            for p in range(P):
                if rounds[p] > 0:
                    g, h = self._grad(yy, Fm[p])
                    G[p], H[p] = g.to(torch.float32), h.to(torch.float32)
        # Quantisation maxima of the next round's (g, h) per job (tree_engine._quant_scales: max over all N
        # rows). Rows a job never trains on keep their round-0 statistics, so their max is taken once; the
        # round epilogue max-reduces the rows it rewrites -- no [P, N] scan per round.
        amax_cur = comp = tam = None
        if fused and os.environ.get("TMOG_XGB_AMAX", "1") != "0":
            amax_cur = torch.stack([G.abs().amax(1), H.abs().amax(1)], 1).contiguous()
            comp = torch.zeros(P, 2, dtype=torch.float32, device=dev)
            for p in range(P):
                out = torch.ones(N, dtype=torch.bool, device=dev)
                out[rows[p]] = False
                comp[p, 0] = torch.where(out, G[p].abs(), torch.zeros_like(G[p])).amax()
                comp[p, 1] = torch.where(out, H[p].abs(), torch.zeros_like(H[p])).amax()
            tam = torch.zeros(64, P, 2, dtype=torch.int32, device=dev)     # boost_kernels.hip kAmaxCopies

        # Device-planned trees (models/tree_engine.py resident=True, ops/csrc/hip/tree_resident.hip): on the fused
        # GPU path a round is enqueued without any host synchronisation -- the level plans, the tree finalisation
        # and the epilogue all run on the device; the host Forests are built from the node records once, after
        # the last round, and the early-stopping AuPR is read ES_LAG rounds late.
        # a feature-parallel job (fp: the jobs spread over a rank group) grows on the device-planned loop too, as one
        # job group whose level exchange (RCCL all-gather + merge of the split records) is enqueued on the stream
        resident = fused and (par is None or fp is not None) and TE.resident_enabled()
        es_lag = max(1, int(os.environ.get("TMOG_ES_LAG", "2"))) if resident else 1
        # Fused round prologue (tree_engine.boost_prologue): the scales, the root copy and the staged (g, h) in
        # one launch; the epilogue's maxima buffer is double-buffered (round it writes tam2[it & 1], which round
        # it's prologue zeroed; round it + 1's prologue reads it).
        prologue = resident and tam is not None and P <= 64 and os.environ.get("TMOG_XGB_PROLOGUE", "1") != "0" \
            and all(float(j.params.get("subsample", 1.0)) >= 1.0 for j in jobs)
        tam2 = torch.zeros(2, 64, P, 2, dtype=torch.int32, device=dev) if prologue else None

        def run(ps, slot_base=0, groups=None):
            """Boosting rounds of the jobs ``ps`` (their trees do not depend on which other jobs grow
            alongside: no per-node randomness, per-model quantisation, weights all 1 on this path)."""
            nonlocal G, H
            root_cache: Dict[tuple, tuple] = {}
            prof = _XGB_PROF.setdefault(slot_base, {}) if _XGB_PROF is not None else None
            tick = time.perf_counter
            pending: list = []
            deferred: list = []        # (act, ResidentTree) per device-planned round, in round order
            pro_buf: dict = {}         # boost_prologue's reusable per-part buffers

            def resolve(it0, need0, vals_t):
                for p, v in zip(need0, vals_t.tolist()):
                    if stopped[p]:
                        continue
                    if v > best[p] + 1e-12:
                        best[p], best_round[p] = v, it0
                    elif it0 - best_round[p] >= esr[p]:
                        stopped[p] = True

            for it in range(max([rounds[p] for p in ps], default=0)):
                cancel.check()
                act = [p for p in ps if it < rounds[p] and not stopped[p]]
                if not act:
                    break
                t_0 = tick()
                if not fused:
                    G = torch.zeros(P, N, dtype=torch.float32, device=dev)
                    H = torch.zeros(P, N, dtype=torch.float32, device=dev)
                    for p in act:
                        g, h = self._grad(yy, Fm[p])
                        G[p], H[p] = g.to(torch.float32), h.to(torch.float32)
                tjobs = []
                for p in act:
                    pr = jobs[p].params
                    tp = TE.TreeParams(max_depth=int(pr.get("max_depth", 6)),
                                       min_child_weight=float(pr.get("min_child_weight", 1.0)),
                                       reg_lambda=float(pr.get("reg_lambda", 1.0)), gamma=float(pr.get("gamma", 0.0)),
                                       eta=float(pr.get("eta", 0.3)), split_eps=1e-6)
                    r = rows[p]
                    w = None
                    ss = float(pr.get("subsample", 1.0))
                    if ss < 1.0:
                        gen = torch.Generator().manual_seed(int(pr.get("seed", 0)) + 17 * it + p)
                        w = (torch.rand(r.numel(), generator=gen) < ss).to(torch.int64).to(dev)
                    tjobs.append(TE.TreeJob(p, tp, r, w))
                root = None
                if all(j.weights is None for j in tjobs):
                    # the packed root entries only change when a job stops: pack once per active set
                    key = tuple(act)
                    if key not in root_cache:
                        root_cache.clear()
                        root_cache[key] = TE._root_rows(tjobs, dev, TE.wide_rows(int(Xg.shape[0])))
                    packed, cnts = root_cache[key]
                    root = None if prologue else (packed.clone(), cnts)
                pre = None
                if prologue:
                    pre = TE.boost_prologue(packed, cnts, act, G, H, amax_cur, comp,
                                            tam2[(it - 1) & 1] if it > 0 else None, tam2[it & 1], pro_buf,
                                            TE.wide_rows(int(Xg.shape[0])))
                t_1 = tick()
                forest = TE.grow_forest(Xg, n_bins_g, tjobs, mode=TE.MODE_GH, kind=TE.KIND_NEWTON, t1=G, t2=H, B=mb,
                                        missing_bin=spec.missing_bin, collect_leaves=True, csr=csr, root=root, fp=fp,
                                        slot_base=slot_base, groups=groups, XbT=XgT,
                                        quant_amax=amax_cur, quant_wmax=1.0 if amax_cur is not None else None,
                                        resident=resident and groups in (None, 1), prestaged=pre, Xh=Xh)
                t_2 = tick()
                is_res = isinstance(forest, TE.ResidentTree)
                if colperm is not None and not is_res:
                    internal = forest.nodes[:, 2] >= 0
                    forest.nodes[internal, 0] = colperm[forest.nodes[internal, 0]]
                need = [p for p in act if esr[p] > 0]
                auc_counts = None
                if fused:
                    ai = None
                    if tam is not None and not prologue:
                        ai = TE._const_tensor(np.asarray(act, np.int64), dev)
                        tam.index_fill_(1, ai, 0)
                    auc_counts = self._fused_epilogue(Fm, G, H, yf, forest, act, N,
                                                      AUC_BINS if (need and self.classification) else 0,
                                                      tam2[it & 1] if prologue else tam)
                    if tam is not None and not prologue:
                        amax_cur.index_copy_(0, ai, torch.maximum(
                            comp.index_select(0, ai), tam.index_select(1, ai).view(torch.float32).amax(0)))
                else:
                    _add_tree_margins(Fm, forest, Xb, act, [1.0] * len(act), tjobs)
                if is_res:
                    deferred.append((list(act), forest))
                    for p in act:
                        forests[p].append(None)          # filled from the device records after the last round
                        weights[p].append(1.0)
                else:
                    for k, p in enumerate(act):
                        forests[p].append(forest.tree(k))
                        weights[p].append(1.0)
                t_3 = tick()
                # early stopping on the training metric (the reference sets no eval set). The AuPR of round it
                # is read back after round it + 1 has been grown, so the host never waits for a round's
                # epilogue: a job that should stop after round it grows one extra tree, which the final
                # trim (best_round + 1 trees) drops -- the same models as checking every round in step.
                if need and self.classification:
                    if auc_counts is not None:
                        sel = auc_counts if len(need) == P else \
                            auc_counts.index_select(0, TE._const_tensor(np.asarray(need, np.int64), dev))
                        vals_t = binned_aupr_from_counts(sel)
                    else:
                        vals_t = binned_aupr_multi([torch.sigmoid(Fm[p][rows[p]]) for p in need],
                                                   [ylab[p] for p in need])
                    while len(pending) >= es_lag:
                        resolve(*pending.pop(0))
                    pending.append((it, need, vals_t))
                if prof is not None:
                    t_4 = tick()
                    for k_, v_ in (("pre", t_1 - t_0), ("grow", t_2 - t_1), ("post", t_3 - t_2), ("es", t_4 - t_3)):
                        prof[k_] = prof.get(k_, 0.0) + v_
                    prof["rounds"] = prof.get("rounds", 0) + 1
            while pending:
                resolve(*pending.pop(0))
            if deferred:
                fs = TE.resident_forests([rt for _, rt in deferred])
                cursor = {p: 0 for p in ps}
                for (act_r, _), f in zip(deferred, fs):
                    if colperm is not None:
                        internal = f.nodes[:, 2] >= 0
                        f.nodes[internal, 0] = colperm[f.nodes[internal, 0]]
                    for k, p in enumerate(act_r):
                        while forests[p][cursor[p]] is not None:
                            cursor[p] += 1
                        forests[p][cursor[p]] = f.tree(k)

        # Pipelined job parts (GPU, fused path): the jobs are split in two halves, each boosted by its
        # own host thread on its own stream, so one half's per-round host work (tree finalisation,
        # round set-up, the early-stopping read-back) overlaps the other half's kernels instead of
        # idling the GPU. Trees are identical to the single-loop order (see run()).
        parts = int(os.environ.get("TMOG_XGB_PIPE", "4"))
        if _XGB_PROF is not None:
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            _XGB_PROF.setdefault("phases", {})["setup"] = time.perf_counter() - t_setup0
            t_loop0 = time.perf_counter()
        if fused and par is None and P >= 2 and parts >= 2:
            parts = min(parts, P)
            cuts = np.linspace(0, P, parts + 1).astype(int)
            gpp = max(1, int(os.environ.get("TMOG_XGB_PIPE_GROUPS", "1")))
            _run_parts(dev, [(list(range(int(cuts[k]), int(cuts[k + 1]))), k * gpp, gpp) for k in range(parts)], run)
        else:
            # feature-parallel: all jobs in one group on one stream (one communicator, one collective order)
            run(list(range(P)), groups=1 if (resident and fp is not None) else None)
        if _XGB_PROF is not None:
            import sys as _sys
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            _XGB_PROF.setdefault("phases", {})["loop"] = time.perf_counter() - t_loop0
            rep = {k: {a: round(b, 4) for a, b in v.items()} for k, v in _XGB_PROF.items()}
            if dev.type == "cuda" and os.environ.get("TMOG_GROW_TIMING"):
                from ..ops import _native as NV
                tm = np.zeros(4, np.int64)
                NV.hip().tmog_hip_grow_timing(tm.ctypes.data, 1)
                rep["native"] = {"plan_s": tm[0] / 1e9, "issue_s": tm[1] / 1e9, "wait_s": tm[2] / 1e9,
                                 "levels": int(tm[3])}
            if dev.type == "cuda" and os.environ.get("TMOG_PLAN_PROFILE") == "1":
                from ..ops import _native as NV
                torch.cuda.synchronize(dev)
                pp = np.zeros(32, np.uint64)
                NV.hip().tmog_hip_plan_profile(pp.ctypes.data, 1)
                calls = max(1, int(pp[31]))
                # mean microseconds per level_plan_kernel call in each phase (100 MHz wall clock)
                rep["plan_phase_us"] = {"calls": int(pp[31]),
                                        **{str(k): round(float(pp[k]) / 100.0 / calls, 2) for k in range(12)}}
            _sys.stderr.write("[xgb-profile] " + json.dumps(rep) + "\n")
            _XGB_PROF.clear()
        res = []
        for p in range(P):
            keep = len(forests[p]) if not stopped[p] else best_round[p] + 1
            res.append({"forest": TE.Forest.concat(forests[p][:keep]).to_state(), "bins": spec.to_state(),
                        "tree_weights": np.asarray(weights[p][:keep], np.float32), "n_classes": 2,
                        "max_bins": mb, "base_margin": base[p], "num_trees": keep})
        return res

    objective_code = 0      # boost_epilogue_kernel: 0 = binary:logistic, 1 = squared error

    def _fused_epilogue(self, Fm, G, H, yf, forest, act, N, bins, amax=None):
        """Margins += this round's leaf values, next round's (g, h), and (with ``bins``) the per-job
        (label, score-bin) counts of the new training scores, in one HIP launch."""
        from ..ops import _native as NV
        la = forest.leaf_assign
        dev = Fm.device
        P = Fm.shape[0]
        counts = torch.zeros(P, 2, bins, dtype=torch.int32, device=dev) if bins else None
        val = la.value[:, 0].contiguous() if la.value.dim() == 2 else la.value.contiguous()
        tree_job = TE._const_tensor(np.asarray(act, np.int64), dev)
        tree_c = la.tree.contiguous()       # (bound: a temporary's block could be handed to the next allocation)
        NV.check(NV.hip().tmog_hip_boost_epilogue(
            NV.ptr(la.rows), NV.ptr(la.gid), int(la.rows.numel()), NV.ptr(val), NV.ptr(tree_c),
            NV.ptr(tree_job), int(N), NV.ptr(Fm), NV.ptr(G), NV.ptr(H), NV.ptr(yf), self.objective_code,
            NV.ptr(counts), int(bins), int(val.shape[0]), len(act), int(P), NV.stream(dev), NV.ptr(amax),
            int(getattr(la, "wide", False))),
            "boost_epilogue")
        return counts

    def fit_batch(self, X, y, jobs, context=None):
        """Jobs with ``objective="reg:squarederror"`` (xgboost4j's own default, which a bare
        ``OpXGBoostClassifier`` in the reference trains with -- ``OpXGBoostClassifierTest.scala``; the model
        selector's grid sets ``binary:logistic``, ``DefaultSelectorParams.scala:72``) boost the label as a
        regression target and score it as the class-1 probability."""
        if type(self) is not XGBoostClassifierLearner:
            return super().fit_batch(X, y, jobs, context)
        sq = [i for i, j in enumerate(jobs) if j.params.get("objective", "binary:logistic") == "reg:squarederror"]
        if not sq:
            return super().fit_batch(X, y, jobs, context)
        lg = [i for i in range(len(jobs)) if i not in set(sq)]
        out = [None] * len(jobs)
        for i, r in zip(lg, super().fit_batch(X, y, [jobs[i] for i in lg], context) if lg else []):
            out[i] = r
        for i, r in zip(sq, _SquaredErrorXGBClassifier().fit_batch(X, y, [jobs[i] for i in sq], context)):
            out[i] = dict(r, objective="reg:squarederror")
        return out

    def _outputs(self, state, m):
        if state.get("objective") == "reg:squarederror":
            # xgboost4j's binary model: raw = (-margin, margin), probability = (1 - p, p) with p the booster's
            # (identity-link) output, prediction from the probability
            m = m.to(torch.float64)
            return (m > 0.5).to(torch.float64), torch.stack([-m, m], 1), torch.stack([1 - m, m], 1)
        return probability_outputs(m)


class _SquaredErrorXGBClassifier(XGBoostClassifierLearner):
    """Squared-error boosting of a 0/1 label (see :meth:`XGBoostClassifierLearner.fit_batch`); not registered."""
    objective_code = 1

    def _grad(self, yy, Fm):
        return Fm - yy, torch.ones_like(Fm)

    def _base_margin(self, bs):
        return float(bs)


@register_learner
class XGBoostRegressorLearner(XGBoostClassifierLearner):
    name = "OpXGBoostRegressor"
    problem = "regression"
    classification = False
    defaults = dict(XGBoostClassifierLearner.defaults, objective="reg:squarederror", eval_metric="rmse",
                    maximize_evaluation_metrics=False)
    objective_code = 1

    def _grad(self, yy, Fm):
        return Fm - yy, torch.ones_like(Fm)

    def _base_margin(self, bs):
        return float(bs)

    def _outputs(self, state, m):
        e = torch.zeros(m.shape[0], 0, dtype=torch.float64, device=m.device)
        return m, e, e


for _name, _cls in [("OpRandomForestClassifier", RandomForestClassifierLearner),
                    ("OpDecisionTreeClassifier", DecisionTreeClassifierLearner),
                    ("OpRandomForestRegressor", RandomForestRegressorLearner),
                    ("OpDecisionTreeRegressor", DecisionTreeRegressorLearner),
                    ("OpGBTClassifier", GBTClassifierLearner), ("OpGBTRegressor", GBTRegressorLearner),
                    ("OpXGBoostClassifier", XGBoostClassifierLearner),
                    ("OpXGBoostRegressor", XGBoostRegressorLearner)]:
    globals()[_name] = register_stage(type(_name, (OpPredictor,), {"operation_name": _name, "learner_cls": _cls}))

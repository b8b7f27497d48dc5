"""Cost-model choice of how each model-selector learner uses the ranks (one rank per GPU).

The reference runs every (estimator, ParamMap) fit as a future on a pool of ``parallelism`` threads
(``OpValidator.scala:318-367``, default 8) and parallelises inside a fit through Spark partitions /
XGBoost ``numWorkers`` (``OpXGBoostClassifier.scala:101-121``). Here a learner's (grid point x fold) jobs either

* **shard**: whole jobs are dealt to ranks by longest-processing-time (LPT) over the estimated job costs --
  no communication, but the makespan is bounded below by the largest job and by ``ceil(jobs / ranks)``;
* **spread**: every rank runs every job of the learner on its share of the work -- rows for the linear
  learners (one fused all-reduce per objective evaluation), features for the trees (one split-record
  all-gather per tree level, ``parallel/learner_parallel.py``) -- at the price of the replicated serial part
  of each job and a collective latency per exchange.

:func:`choose` evaluates both with the calibrated seconds-per-unit of each learner (``tuning/validators.py``
``_COST_SCALE``, updated after every validation from measured times) and a per-collective latency, and picks
the cheaper per learner. The choice only depends on values every rank has (grids, sizes, world, the
calibration broadcast by rank 0), so all ranks take the same decision. :func:`project` gives the per-rank
critical path of the resulting schedule (``scripts/project_schedule.py``).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

# Replicated (not divided by the ranks) fraction of a spread job's time, by intra-job mode: linear
# learners replicate the quasi-Newton updates (small); feature-parallel trees replicate the row partition,
# the leaf collection and the boosting epilogue -- 0.32 of the XGBoost kernel time on the MI355X headline
# (partition 0.20 + epilogue 0.07 + leaves / plan 0.05 of ~1.0 s, profiles/r4_levels_base.txt)
SERIAL_FRACTION = {"rows": 0.05, "features": 0.32}
# seconds per collective: a small-message RCCL all-reduce / all-gather over xGMI (8 ranks, ~25 us) --
# gloo on the CPU is ~10x that; overridable for experiments
COLLECTIVE_S = float(os.environ.get("TMOG_COLLECTIVE_S", "2.5e-5"))


@dataclass
class Choice:
    mode: str            # "shard" | "spread"
    shard_s: float       # estimated makespan when sharding whole jobs
    spread_s: float      # estimated time when every rank runs every job on its share
    n_jobs: int


def lpt_makespan(costs: Sequence[float], world: int) -> float:
    loads = [0.0] * max(1, world)
    for c in sorted(costs, reverse=True):
        k = min(range(len(loads)), key=lambda i: loads[i])
        loads[k] += c
    return max(loads) if loads else 0.0


def collectives(learner: str, params: Dict, n_tr: int) -> float:
    """Exchanges of one spread job: objective evaluations for the linear learners (~1.5 per iteration), one
    split exchange per tree level per boosting round for the trees."""
    if "LogisticRegression" in learner or "SVC" in learner or "LinearRegression" in learner \
            or "Perceptron" in learner:
        return 1.5 * float(params.get("max_iter", 100))
    depth = float(params.get("max_depth", 5))
    rounds = float(params.get("num_round", params.get("max_iter", 1)))
    return rounds * (depth + 1)


def choose(models: Sequence[Tuple[str, Sequence[Dict]]], n_folds: int, n_tr: int, d: int, world: int,
           parallel_of, job_seconds) -> Dict[int, Choice]:
    """Per learner index: shard or spread. ``parallel_of(name)`` is the learner's intra-job mode (None, "rows",
    "features"), ``job_seconds(name, params)`` the calibrated single-rank seconds of one job."""
    out: Dict[int, Choice] = {}
    force = os.environ.get("TMOG_PARALLEL_MODE")      # "shard" / "spread": override (A/B, tests)
    for li, (name, grid) in enumerate(models):
        costs = [job_seconds(name, p) for p in grid for _ in range(n_folds)]
        shard = lpt_makespan(costs, world)
        mode = parallel_of(name)
        if world <= 1 or mode not in SERIAL_FRACTION:
            out[li] = Choice("shard", shard, math.inf, len(costs))
            continue
        s = SERIAL_FRACTION[mode]
        spread = sum(c * (s + (1.0 - s) / world) for c in costs) + \
            COLLECTIVE_S * math.log2(max(world, 2)) * sum(collectives(name, p, n_tr) for p in grid for _ in range(n_folds))
        pick = "spread" if spread < shard else "shard"
        if force in ("shard", "spread"):
            pick = force
        out[li] = Choice(pick, shard, spread, len(costs))
    return out


def project(models, choices: Dict[int, Choice], n_folds: int, world: int, job_seconds) -> List[dict]:
    """Estimated per-rank busy seconds of the whole selection under ``choices``: spread learners add their
    spread time to every rank, the sharded jobs of all learners are dealt by one LPT on top."""
    loads = [0.0] * max(1, world)
    rows = []
    for li, (name, grid) in enumerate(models):
        c = choices[li]
        if c.mode == "spread":
            loads = [x + c.spread_s for x in loads]
    sharded = []
    for li, (name, grid) in enumerate(models):
        if choices[li].mode == "shard":
            sharded += [(job_seconds(name, p), name) for p in grid for _ in range(n_folds)]
    for cost, name in sorted(sharded, key=lambda t: -t[0]):
        k = min(range(len(loads)), key=lambda i: loads[i])
        loads[k] += cost
    for li, (name, grid) in enumerate(models):
        c = choices[li]
        rows.append({"learner": name, "jobs": c.n_jobs, "mode": c.mode, "shard_s": round(c.shard_s, 4),
                     "spread_s": round(c.spread_s, 4) if math.isfinite(c.spread_s) else None})
    rows.append({"per_rank_s": [round(x, 4) for x in loads], "critical_path_s": round(max(loads), 4)})
    return rows

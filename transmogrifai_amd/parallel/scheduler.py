"""Cost-model choice of how each model-selector learner uses the ranks (one rank per GPU).

The reference runs every (estimator, ParamMap) fit as a future on a pool of ``parallelism`` threads
(``OpValidator.scala:318-367``, default 8) and parallelises inside a fit through Spark partitions /
XGBoost ``numWorkers`` (``OpXGBoostClassifier.scala:101-121``). Here a learner's (grid point x fold) jobs either

* **shard**: whole jobs are dealt to ranks by longest-processing-time (LPT) over the estimated job costs --
  no communication, but the makespan is bounded below by the largest job and by ``ceil(jobs / ranks)``;
* **spread**: every rank runs every job of the learner on its share of the work -- rows for the linear
  learners (one fused all-reduce per objective evaluation), features for the trees (one split-record
  all-gather per tree level, ``parallel/learner_parallel.py``) -- at the price of the replicated serial part
  of each job and a collective latency per exchange;
* **hybrid**: the ranks form ``world / g`` groups of ``g`` consecutive ranks (``parallel/dist.py partition``,
  ``torch.distributed.new_group`` subgroups with their own RCCL communicators); whole jobs are dealt to the
  groups by LPT and every job is spread over its group -- e.g. 6 XGBoost jobs on 8 GPUs as 2 groups of 4,
  which the reference would express as fewer concurrent fits with ``numWorkers`` = 4 each.

:func:`choose` evaluates every group size ``g`` dividing the world (``g = 1`` is shard, ``g = world`` spread)
with the calibrated seconds-per-unit of each learner (``tuning/validators.py`` ``_COST_SCALE``, updated after
every validation from measured times) and a per-collective latency, and picks the cheapest per learner. The choice only depends on values every rank has (grids, sizes, world, the
calibration broadcast by rank 0), so all ranks take the same decision. :func:`project` gives the per-rank
critical path of the resulting schedule (``scripts/project_schedule.py``).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

# Replicated (not divided by the ranks) fraction of a spread job's time, by intra-job mode: linear
# learners replicate the quasi-Newton updates (small); feature-parallel trees replicate everything but the
# histograms and the split scans. Calibrated from the round-5 XGBoost kernel breakdown on the MI355X headline
# (profiles/r5_xgb_kernel_stats.txt, per step): divided by the ranks -- hist_build 1155 + pair_scan 510 +
# split_scan 166 + zero_segments 115 = 1946 ms; replicated -- level_plan 731 + partition 318 +
# boost_epilogue 115 + aupr_counts 107 + leaf_collect 91 + tree_finalize 80 + prologue 40 + validation
# predict 100 = 1582 ms: 0.45 of 3528 ms.
SERIAL_FRACTION = {"rows": 0.05, "features": 0.45}
# seconds per collective: a small-message RCCL all-reduce / all-gather over xGMI (8 ranks, ~25 us) --
# gloo on the CPU is ~10x that; overridable for experiments
COLLECTIVE_S = float(os.environ.get("TMOG_COLLECTIVE_S", "2.5e-5"))


@dataclass
class Choice:
    mode: str            # "shard" | "spread" | "hybrid"
    shard_s: float       # estimated makespan when sharding whole jobs
    spread_s: float      # estimated time when every rank runs every job on its share
    n_jobs: int
    group_size: int = 1  # ranks per group: 1 shard, world spread, in between hybrid
    hybrid_s: float = math.inf   # estimated makespan of the best hybrid group size
    options: Optional[Dict[int, float]] = None   # group size -> estimated makespan
    serial: float = 0.0  # replicated fraction of a spread job (SERIAL_FRACTION of its intra-job mode)


def divisors(n: int) -> List[int]:
    return [g for g in range(1, n + 1) if n % g == 0]


def group_makespan(costs: Sequence[float], colls: Sequence[float], world: int, g: int, serial: float) -> float:
    """Makespan of jobs (single-rank ``costs``, ``colls`` exchanges each) on ``world / g`` groups of ``g`` ranks:
    LPT over the groups of the per-job time ``c (s + (1 - s) / g)`` plus the collective latency."""
    if g <= 1:
        return lpt_makespan(costs, world)
    lat = COLLECTIVE_S * math.log2(max(g, 2))
    t = [c * (serial + (1.0 - serial) / g) + lat * k for c, k in zip(costs, colls)]
    return lpt_makespan(t, world // g)


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
    """Per learner index: shard, spread or hybrid (with its group size). ``parallel_of(name)`` is the learner's intra-job mode (None, "rows",
    "features"), ``job_seconds(name, params)`` the calibrated single-rank seconds of one job."""
    out: Dict[int, Choice] = {}
    # override (A/B, tests): "shard" / "spread" / "hybrid" (best hybrid size) / "hybrid:G" (groups of G ranks)
    force = os.environ.get("TMOG_PARALLEL_MODE")
    for li, (name, grid) in enumerate(models):
        costs = [job_seconds(name, p) for p in grid for _ in range(n_folds)]
        colls = [collectives(name, p, n_tr) for p in grid for _ in range(n_folds)]
        shard = lpt_makespan(costs, world)
        mode = parallel_of(name)
        if world <= 1 or mode not in SERIAL_FRACTION:
            out[li] = Choice("shard", shard, math.inf, len(costs))
            continue
        s = SERIAL_FRACTION[mode]
        opts = {g: group_makespan(costs, colls, world, g, s) for g in divisors(world)}
        spread = opts[world]
        mids = {g: v for g, v in opts.items() if 1 < g < world}
        g_h = min(mids, key=lambda g: (mids[g], g)) if mids else world
        hybrid = mids.get(g_h, math.inf)
        g = min(opts, key=lambda k: (opts[k], -k))      # ties: the larger group (fewer, shorter jobs)
        if force in ("shard", "spread"):
            g = 1 if force == "shard" else world
        elif force and force.startswith("hybrid"):
            want = int(force.split(":")[1]) if ":" in force else g_h
            g = want if (world % want == 0 and 1 <= want <= world) else g_h
        pick = "shard" if g == 1 else ("spread" if g == world else "hybrid")
        out[li] = Choice(pick, shard, spread, len(costs), g, hybrid, opts, s)
    return out


def assign_groups(costs: Sequence[float], n_groups: int) -> List[int]:
    """Group index per job: LPT over the groups (deterministic: the same on every rank)."""
    loads = [0.0] * max(1, n_groups)
    owner = [0] * len(costs)
    for j in sorted(range(len(costs)), key=lambda j: (-costs[j], j)):
        k = min(range(len(loads)), key=lambda i: (loads[i], i))
        owner[j] = k
        loads[k] += costs[j]
    return owner


def project(models, choices: Dict[int, Choice], n_folds: int, world: int, job_seconds) -> List[dict]:
    """Estimated per-rank busy seconds of the whole selection under ``choices``: spread learners add their
    spread time to every rank, the sharded jobs of all learners are dealt by one LPT on top."""
    loads = [0.0] * max(1, world)
    rows = []
    for li, (name, grid) in enumerate(models):
        c = choices[li]
        if c.mode == "spread":
            loads = [x + c.spread_s for x in loads]
        elif c.mode == "hybrid":          # every rank of a group carries the group's LPT load
            g = c.group_size
            costs = [job_seconds(name, p) for p in grid for _ in range(n_folds)]
            owner = assign_groups(costs, world // g)
            s = c.serial
            for k in range(world // g):
                t = sum(cj * (s + (1.0 - s) / g) for cj, o in zip(costs, owner) if o == k)
                for r in range(k * g, (k + 1) * g):
                    loads[r] += t
    sharded = []
    for li, (name, grid) in enumerate(models):
        if choices[li].mode == "shard":
            sharded += [(job_seconds(name, p), name) for p in grid for _ in range(n_folds)]
    for cost, name in sorted(sharded, key=lambda t: -t[0]):
        k = min(range(len(loads)), key=lambda i: loads[i])
        loads[k] += cost
    for li, (name, grid) in enumerate(models):
        c = choices[li]
        rows.append({"learner": name, "jobs": c.n_jobs, "mode": c.mode, "group_size": c.group_size,
                     "shard_s": round(c.shard_s, 4),
                     "spread_s": round(c.spread_s, 4) if math.isfinite(c.spread_s) else None,
                     "hybrid_s": round(c.hybrid_s, 4) if math.isfinite(c.hybrid_s) else None})
    rows.append({"per_rank_s": [round(x, 4) for x in loads], "critical_path_s": round(max(loads), 4)})
    return rows

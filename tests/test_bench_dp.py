"""bench.py on 4 and 8 gloo ranks (row-sharded, data-parallel fits; learners sharded or spread by the cost
model of parallel/scheduler.py) reproduces the 1-rank selection for the BASELINE
configs: same best model, configs evaluated and hold-out metric, and no estimator falls back to gathering its
input columns (stages/base.py OpEstimator.fit)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(gpus, config, rows, models, **env_extra):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--device", "cpu", "--rows", str(rows),
           "--steps", "1", "--warmup", "0", "--config", config, "--models", models]
    env = dict(os.environ, OMP_NUM_THREADS="2", **env_extra)
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [l for l in out.stdout.splitlines() if l.startswith('{"metric"')][-1]
    return json.loads(line)


@pytest.mark.parametrize("config,rows,models", [
    ("binary-10m", 6000, "OpLogisticRegression,OpRandomForestClassifier,OpXGBoostClassifier"),
    ("multiclass-text", 3000, "default"),
    ("regression-100m", 4000, "OpLinearRegression,OpRandomForestRegressor,OpGBTRegressor"),
])
@pytest.mark.parametrize("ranks", [4, 8])
def test_bench_many_ranks_matches_one_rank(config, rows, models, ranks):
    one = _bench(1, config, rows, models)
    four = _bench(ranks, config, rows, models)
    assert four["config"]["parallelism"] == f"dp{ranks}"
    assert four["dp_gather_fallbacks"] == [] and one["dp_gather_fallbacks"] == []
    assert four["best_model"] == one["best_model"]
    assert four["configs_evaluated"] == one["configs_evaluated"]
    key = [k for k in one if k.startswith("holdout_")][0]
    assert abs(four[key] - one[key]) <= 1e-9, (key, one[key], four[key])


@pytest.mark.parametrize("mode,lanes", [("hybrid:2", "1"), ("shard", "2")])
def test_bench_hybrid_groups_and_lanes_match_one_rank(mode, lanes):
    """4 gloo ranks with every intra-job-parallel learner forced onto 2 groups of 2 ranks (parallel/scheduler.py
    hybrid: LR row-parallel and XGBoost feature-parallel inside each group, jobs dealt to the groups), and with
    all-shard schedules run in 2 learner lanes per rank: the 1-rank selection is reproduced."""
    models = "OpLogisticRegression,OpRandomForestClassifier,OpXGBoostClassifier"
    one = _bench(1, "binary-10m", 6000, models)
    many = _bench(4, "binary-10m", 6000, models, TMOG_PARALLEL_MODE=mode, TMOG_LEARNER_LANES=lanes)
    assert many["best_model"] == one["best_model"]
    assert many["configs_evaluated"] == one["configs_evaluated"]
    assert abs(many["holdout_aupr"] - one["holdout_aupr"]) <= 1e-9
    want = {"OpLogisticRegression": mode, "OpXGBoostClassifier": mode, "OpRandomForestClassifier": "shard"}
    assert many["schedule"] == want, many["schedule"]

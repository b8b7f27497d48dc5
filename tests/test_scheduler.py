"""Cost-model choice of shard vs spread per learner (parallel/scheduler.py) and the validator using it."""
import math

from transmogrifai_amd.parallel import scheduler as S
from transmogrifai_amd.selector import factories as F


def _par(name):
    return {"OpLogisticRegression": "rows", "OpXGBoostClassifier": "features",
            "OpRandomForestClassifier": None}.get(name)


def test_lpt_makespan():
    assert S.lpt_makespan([3, 3, 2, 2, 2], 2) == 7          # LPT, not the optimum (6)
    assert S.lpt_makespan([5, 1, 1], 4) == 5
    assert S.lpt_makespan([], 4) == 0


def test_xgboost_shards_when_jobs_cover_the_ranks():
    """6 XGBoost jobs (2 grid points x 3 folds) on 4 or 8 ranks: whole jobs per rank beat replicating the
    serial part of every job on every rank."""
    models = [("OpXGBoostClassifier", F._xgb_bin_grid())]
    for world in (4, 6, 8):
        ch = S.choose(models, 3, 1_000_000, 330, world, _par, lambda n, p: 0.2)
        assert ch[0].mode == "shard", (world, ch[0])
        assert ch[0].shard_s <= ch[0].spread_s


def test_single_big_job_spreads():
    """One long job on 8 ranks cannot be sharded: spreading it wins when the collectives are cheap."""
    models = [("OpXGBoostClassifier", [dict(num_round=20, max_depth=6)])]
    ch = S.choose(models, 1, 1_000_000, 330, 8, _par, lambda n, p: 10.0)
    assert ch[0].mode == "spread" and ch[0].spread_s < ch[0].shard_s


def test_no_intra_job_mode_always_shards_and_one_rank_shards():
    models = [("OpRandomForestClassifier", [dict(num_trees=50)] * 18), ("OpLogisticRegression", [{}])]
    ch = S.choose(models, 3, 1_000_000, 330, 8, _par, lambda n, p: 1.0)
    assert ch[0].mode == "shard" and math.isinf(ch[0].spread_s)
    ch1 = S.choose(models, 3, 1_000_000, 330, 1, _par, lambda n, p: 1.0)
    assert all(c.mode == "shard" for c in ch1.values())


def test_projection_balances_ranks():
    models = [("OpLogisticRegression", F._lr_grid()), ("OpRandomForestClassifier", F._rf_grid(["gini"])),
              ("OpXGBoostClassifier", F._xgb_bin_grid())]
    cost = {"OpLogisticRegression": 0.012, "OpRandomForestClassifier": 0.005, "OpXGBoostClassifier": 0.23}
    js = lambda n, p: cost[n]
    ch = S.choose(models, 3, 1_000_000, 330, 8, _par, js)
    rows = S.project(models, ch, 3, 8, js)
    per = rows[-1]["per_rank_s"]
    assert len(per) == 8
    total = sum(c * len(g) * 3 for (n, g), c in zip(models, [cost[m[0]] for m in models]))
    assert rows[-1]["critical_path_s"] >= total / 8 - 1e-9
    assert rows[-1]["critical_path_s"] <= 0.23 + 0.05       # bounded by the longest job plus a few small ones


def test_forced_mode(monkeypatch):
    monkeypatch.setenv("TMOG_PARALLEL_MODE", "spread")
    ch = S.choose([("OpXGBoostClassifier", F._xgb_bin_grid())], 3, 1000, 10, 4, _par, lambda n, p: 0.2)
    assert ch[0].mode == "spread"


def test_projection_mode_collectives():
    """parallel/dist.py projection mode: one process plays rank r of W ranks holding identical shards."""
    import torch
    from transmogrifai_amd.parallel import dist as D
    try:
        D.simulate(3, 8)
        assert D.is_dist() and D.rank() == 3 and D.world() == 8
        assert D.all_reduce(torch.tensor([2.0]), "sum").item() == 16.0
        assert D.all_reduce(torch.tensor([2.0]), "max").item() == 2.0
        assert D.all_gather_rows(torch.arange(3)).tolist() == list(range(3)) * 8
        assert D.all_gather_object({"a": 1}) == [{"a": 1}] * 8
        assert D.broadcast_object(5) == 5
        assert D.all_to_all_bytes([bytes([k]) for k in range(8)]) == [bytes([3])] * 8
        owners = D.lpt_assign([1.0] * 20, D.world())
        assert sorted(set(owners)) == list(range(8))
    finally:
        D.simulate(0, 1)
    assert not D.simulated() and not D.is_dist()


def test_hybrid_group_beats_both_pure_modes():
    """2 long XGBoost jobs on 8 ranks: sharding leaves 6 ranks idle, spreading both over all 8 replicates the
    serial part twice on every rank; 2 groups of 4 ranks, one job each, beat both."""
    models = [("OpXGBoostClassifier", [dict(num_round=200, max_depth=10)])]
    ch = S.choose(models, 2, 1_000_000, 330, 8, _par, lambda n, p: 10.0)[0]
    assert ch.mode == "hybrid" and ch.group_size == 4, ch
    assert ch.hybrid_s < ch.shard_s and ch.hybrid_s < ch.spread_s
    assert set(ch.options) == {1, 2, 4, 8}
    rows = S.project(models, {0: ch}, 2, 8, lambda n, p: 10.0)
    assert rows[0]["mode"] == "hybrid" and rows[0]["group_size"] == 4
    per = rows[-1]["per_rank_s"]
    assert max(per) == min(per) and abs(max(per) - ch.hybrid_s) < 0.5      # both groups carry one job


def test_forced_hybrid_size(monkeypatch):
    monkeypatch.setenv("TMOG_PARALLEL_MODE", "hybrid:2")
    ch = S.choose([("OpXGBoostClassifier", F._xgb_bin_grid())], 3, 1000, 10, 4, _par, lambda n, p: 0.2)[0]
    assert ch.mode == "hybrid" and ch.group_size == 2
    monkeypatch.setenv("TMOG_PARALLEL_MODE", "hybrid:3")      # not a divisor: the best hybrid size
    ch = S.choose([("OpXGBoostClassifier", F._xgb_bin_grid())], 3, 1000, 10, 4, _par, lambda n, p: 0.2)[0]
    assert ch.mode == "hybrid" and ch.group_size == 2


def test_assign_groups_is_lpt_and_deterministic():
    assert S.assign_groups([5, 1, 4, 2], 2) == [0, 0, 1, 1]
    assert S.assign_groups([1.0] * 6, 3) == [0, 1, 2, 0, 1, 2]

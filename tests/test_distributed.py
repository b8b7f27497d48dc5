"""Multi-process (gloo, world_size 2) tests of the distributed paths: the collective helpers, the
data-parallel (row-sharded) workflow fit of parallel/dp.py and the grid-sharded model selector.

Reference behaviour being reproduced: Spark computes every fit statistic over all partitions
(``treeAggregate``/``fold``), so a row-sharded fit must produce the same vectorizer fills, pivot
top-K lists and SanityChecker statistics as a single-process fit over the whole table.
"""
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn_name, out_dir):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(2)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = globals()[fn_name](rank, world)
        with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
            json.dump(res, f)
    finally:
        dist.destroy_process_group()


def _run(fn_name, tmp_path, world=2):
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, fn_name, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    return [json.load(open(tmp_path / f"r{r}.json")) for r in range(world)]


# ------------------------------------------------------------------------------- rank programs
def _collectives(rank, world):
    from collections import Counter
    from transmogrifai_amd.data.columns import NumericColumn, TextColumn
    from transmogrifai_amd.features import types as T
    from transmogrifai_amd.parallel import dp
    with dp.scope(True):
        a, b = dp.sum_([torch.tensor([1.0 + rank, 2.0]), torch.tensor([[rank * 1.0]])])
        n = dp.count(10 + rank)
        cs = dp.merge_counters([Counter({"x": 1, f"r{rank}": 2})])
        mn = dp.min_(torch.tensor([float(rank)]))
        u = dp.unique_values(torch.tensor([float(rank), 5.0]))
        num = dp.gather_column(NumericColumn(T.Real, torch.tensor([float(rank)] * (rank + 1)),
                                             torch.tensor([True] * (rank + 1))))
        txt = dp.gather_column(TextColumn(T.PickList, torch.tensor([0, 1, -1], dtype=torch.int32),
                                          ["a", f"v{rank}"]))
    return {"a": a.tolist(), "b": b.tolist(), "n": n, "cs": dict(cs[0]), "mn": mn.tolist(), "u": u.tolist(),
            "num": num.values.tolist(), "txt": txt.to_list()}


def _fit_summary(model, pred):
    from transmogrifai_amd.stages.feature.vectorizers import OpOneHotVectorizerModel, RealVectorizerModel
    out = {"fills": [], "tops": []}
    for st in model.stages:
        if isinstance(st, RealVectorizerModel):
            out["fills"].append([float(v) for v in st.fill_values])
        if isinstance(st, OpOneHotVectorizerModel):
            out["tops"].append(st.top_values)
        if "summary" in st.metadata and "featuresStatistics" in st.metadata["summary"]:
            s = st.metadata["summary"]
            out["sc_mean"] = s["featuresStatistics"]["mean"]
            out["sc_var"] = s["featuresStatistics"]["variance"]
            out["sc_corr"] = s["correlationsWLabel"]["values"]
            out["sc_dropped"] = s["dropped"]
            out["sc_count"] = s["featuresStatistics"]["count"]
    summ = model.get_origin_stage_of(pred).metadata["summary"]
    out["best"] = summ["bestModelType"]
    out["holdout_aupr"] = summ["holdoutEvaluation"]["AuPR"]
    out["holdout_n"] = summ["holdoutEvaluation"]["TP"] + summ["holdoutEvaluation"]["TN"] + \
        summ["holdoutEvaluation"]["FP"] + summ["holdoutEvaluation"]["FN"]
    out["n_validation_results"] = len(summ["validationResults"])
    return out


def _workflow(rank, world, sharded=True):
    from transmogrifai_amd import uid
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.readers.base import InMemoryReader
    from transmogrifai_amd.selector.factories import BinaryClassificationModelSelector
    from transmogrifai_amd.testkit.synthetic import binary_table
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    uid.reset(0)
    ds, label, preds = binary_table(4000, n_real=6, n_int=2, n_pick=2, n_null_cols=3, seed=11)
    if sharded:
        ds = ds.shard(rank, world)
    vec = transmogrify(preds)
    checked = label.sanity_check(vec, remove_bad_features=True)
    pred = BinaryClassificationModelSelector.with_cross_validation(
        num_folds=2, seed=5, model_types_to_use=["OpLogisticRegression"]).set_input(label, checked).get_output()
    model = OpWorkflow().set_result_features(label, pred).set_reader(InMemoryReader(ds)).train()
    return _fit_summary(model, pred)


def _workflow_sharded(rank, world):
    return _workflow(rank, world, True)


def _workflow_grid(rank, world):
    """Replicated table (not sharded): the (learner, grid, fold) jobs are split over the ranks."""
    return _workflow(rank, world, False)


# ------------------------------------------------------------------------------------- tests
def _events_records():
    import random
    r = random.Random(5)
    return [{"k": f"u{r.randint(0, 40)}", "t": r.randint(0, 10_000), "amt": r.random() * 10,
             "cat": r.choice(["a", "b", "c"])} for _ in range(600)]


def _aggregate_shuffle(rank, world):
    from transmogrifai_amd.features import aggregators as A
    from transmogrifai_amd.features.builder import FeatureBuilder
    from transmogrifai_amd.parallel import dist as D
    from transmogrifai_amd.readers.aggregate import AggregateParams
    from transmogrifai_amd.readers.files import DataReaders
    # the all-to-all itself: rank r sends "r->k" to every k
    got = D.all_to_all_bytes([f"{rank}->{k}".encode() for k in range(world)])
    assert [g.decode() for g in got] == [f"{k}->{rank}" for k in range(world)]
    amt = FeatureBuilder.Real("amt").extract(lambda e: e["amt"]).aggregate(A.SumNumeric()).as_predictor()
    cat = FeatureBuilder.PickList("cat").extract(lambda e: e["cat"]).as_predictor()
    txt = FeatureBuilder.Text("txt").extract(lambda e: e["cat"] + str(e["t"] % 7)).aggregate(A.ConcatText()) \
        .as_predictor()
    rd = DataReaders.Aggregate.custom(_events_records(), key=lambda e: e["k"],
                                      aggregate_params=AggregateParams(lambda e: e["t"],
                                                                       A.CutOffTime.unix_epoch(6000)))
    ds = rd.distribute().generate_dataset([amt, cat, txt])
    assert ds.sharded
    return {"keys": [str(k) for k in ds.key], "amt": ds["amt"].to_list(), "cat": ds["cat"].to_list(),
            "txt": ds["txt"].to_list(), "rid": ds.row_ids.tolist()}


def test_keyed_shuffle_aggregate_reader_matches_single_process(tmp_path):
    """C14: the aggregate reader shuffles events by key over the ranks (all-to-all) and each rank aggregates
    the keys it owns; the union over ranks equals the single-process aggregation."""
    from transmogrifai_amd.features import aggregators as A
    from transmogrifai_amd.features.builder import FeatureBuilder
    from transmogrifai_amd.readers.aggregate import AggregateParams
    from transmogrifai_amd.readers.files import DataReaders
    res = _run("_aggregate_shuffle", tmp_path)
    amt = FeatureBuilder.Real("amt").extract(lambda e: e["amt"]).aggregate(A.SumNumeric()).as_predictor()
    cat = FeatureBuilder.PickList("cat").extract(lambda e: e["cat"]).as_predictor()
    txt = FeatureBuilder.Text("txt").extract(lambda e: e["cat"] + str(e["t"] % 7)).aggregate(A.ConcatText()) \
        .as_predictor()
    ref = DataReaders.Aggregate.custom(_events_records(), key=lambda e: e["k"],
                                       aggregate_params=AggregateParams(lambda e: e["t"],
                                                                        A.CutOffTime.unix_epoch(6000))) \
        .generate_dataset([amt, cat, txt])
    want = {str(k): (a, c, t) for k, a, c, t in zip(ref.key, ref["amt"].to_list(), ref["cat"].to_list(),
                                                    ref["txt"].to_list())}
    got = {}
    for r in res:
        for k, a, c, t in zip(r["keys"], r["amt"], r["cat"], r["txt"]):
            assert k not in got               # every key aggregated on exactly one rank
            got[k] = (a, c, t)
    assert set(got) == set(want)
    for k in want:
        assert got[k][1] == want[k][1]
        assert got[k][2] == want[k][2]        # order-dependent concatenation in source order
        assert (got[k][0] is None and want[k][0] is None) or abs(got[k][0] - want[k][0]) < 1e-9
    rids = sorted(i for r in res for i in r["rid"])
    assert rids == list(range(len(want)))


def test_collectives_gloo(tmp_path):
    r0, r1 = _run("_collectives", tmp_path)
    for r in (r0, r1):
        assert r["a"] == [3.0, 4.0] and r["b"] == [[1.0]]
        assert r["n"] == 21
        assert r["cs"] == {"x": 2, "r0": 2, "r1": 2}
        assert r["mn"] == [0.0]
        assert r["u"] == [0.0, 1.0, 5.0]
        assert r["num"] == [0.0, 1.0, 1.0]
        # rank 0 codes (a, v0, null) then rank 1 (a, v1, null) re-coded on the union dictionary
        assert r["txt"] == ["a", "v0", None, "a", "v1", None]


def test_sharded_workflow_matches_single_process(tmp_path):
    single = _workflow(0, 1, sharded=False)
    r0, r1 = _run("_workflow_sharded", tmp_path)
    assert r0 == r1, "ranks disagree on the fitted model"
    # fit statistics reduced over the shards equal the single-process statistics
    assert len(r0["fills"]) == len(single["fills"])
    for a, b in zip(r0["fills"], single["fills"]):
        np.testing.assert_allclose(a, b, rtol=1e-9)
    assert r0["tops"] == single["tops"]
    assert r0["sc_count"] == single["sc_count"]
    np.testing.assert_allclose(r0["sc_mean"], single["sc_mean"], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(r0["sc_var"], single["sc_var"], rtol=1e-7, atol=1e-10)
    np.testing.assert_allclose(np.array(r0["sc_corr"], dtype=float), np.array(single["sc_corr"], dtype=float),
                               rtol=1e-6, atol=1e-9)
    assert r0["sc_dropped"] == single["sc_dropped"]
    # the hold-out is evaluated on all ranks' rows together
    assert r0["holdout_n"] == single["holdout_n"]
    assert r0["best"] == single["best"]
    assert abs(r0["holdout_aupr"] - single["holdout_aupr"]) < 1e-6


def test_grid_sharded_selector_matches_single_process(tmp_path):
    single = _workflow(0, 1, sharded=False)
    r0, r1 = _run("_workflow_grid", tmp_path)
    assert r0 == r1
    assert r0["n_validation_results"] == single["n_validation_results"]
    assert r0["best"] == single["best"]
    assert abs(r0["holdout_aupr"] - single["holdout_aupr"]) < 1e-9


def _wcv(rank, world):
    """Workflow-level CV on 2 ranks: the stacked fold jobs are LPT-sharded over the ranks."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import test_workflow_cv as W
    _, _, summ = W._train(True, W._records())
    return {"vr": [v["metricValues"]["AuPR"] for v in summ["validationResults"]], "best": summ["bestModelType"],
            "params": summ["bestModelParameters"]}


def test_workflow_cv_two_ranks_matches_one(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import test_workflow_cv as W
    _, _, summ = W._train(True, W._records())
    one = [v["metricValues"]["AuPR"] for v in summ["validationResults"]]
    r0, r1 = _run("_wcv", tmp_path)
    assert r0 == r1
    np.testing.assert_allclose(r0["vr"], one, rtol=0, atol=1e-12)
    assert r0["best"] == summ["bestModelType"]

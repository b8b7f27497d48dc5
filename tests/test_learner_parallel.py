"""Intra-job parallelism of the learners over ranks (gloo, world_size 2 and 3).

* Feature-parallel tree growth (parallel/learner_parallel.py, common/tree_grow.hpp): every rank
  grows every tree over its feature slice and the ranks all-gather one split record per node and
  level -- the forests must equal the single-process forests bit for bit (XGBoost's Rabit workers
  produce the same trees as one worker, ``OpXGBoostClassifier.scala:111``).
* Row-parallel linear models: the objective's sums are all-reduced per pass (Spark's
  ``treeAggregate`` of the L-BFGS gradient) -- coefficients must match the
  single-process fit to float tolerance and be identical on every rank.
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


def _data(n=3000, d=24, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, d, generator=g)
    X[:, 5] = (X[:, 5] > 0.3).float()            # 0/1 indicator columns (one present bin under missing=0)
    X[:, 9] = (X[:, 9] > -0.2).float()
    X[:, 11] = torch.where(torch.rand(n, generator=g) < 0.3, torch.zeros(n), X[:, 11])   # sparse numeric
    logit = X[:, 0] - 0.7 * X[:, 3] + 0.9 * X[:, 5] + 0.4 * X[:, 11] * X[:, 2]
    y = (torch.rand(n, generator=g) < torch.sigmoid(logit)).float()
    return X, y


def _forest_sig(state):
    f = state["forest"]
    return {k: np.asarray(f[k]).tolist() for k in ("tree_off", "nodes", "default_left", "value")}


def _trees(par):
    from transmogrifai_amd.models.base import FitJob, learner_class
    X, y = _data()
    rows = [torch.arange(0, 2000), torch.arange(1000, 3000)]
    ctx = {"par": par} if par is not None else {}
    out = {}
    xgb = learner_class("OpXGBoostClassifier")()
    jobs = [FitJob(dict(xgb.defaults, num_round=6, max_depth=5, min_child_weight=mcw, missing=0.0, eta=0.3,
                        gamma=0.1, max_bins=32), r) for mcw in (1.0, 10.0) for r in rows]
    out["xgb"] = [_forest_sig(s) for s in xgb.fit_batch(X, y, jobs, context=ctx)]
    gbt = learner_class("OpGBTClassifier")()
    out["gbt"] = [_forest_sig(s) for s in gbt.fit_batch(
        X, y, [FitJob(dict(gbt.defaults, max_iter=3, max_depth=4), r) for r in rows], context=ctx)]
    dt = learner_class("OpDecisionTreeClassifier")()
    out["dt"] = [_forest_sig(s) for s in dt.fit_batch(
        X, y, [FitJob(dict(dt.defaults, max_depth=6), r) for r in rows], context=ctx)]
    return out


def _trees_fp(rank, world):
    from transmogrifai_amd.parallel.learner_parallel import LearnerParallel
    return _trees(LearnerParallel())


def test_feature_parallel_trees_bit_identical(tmp_path):
    ref = _trees(None)
    for world in (2, 3):
        outs = _run("_trees_fp", tmp_path, world)
        for r, o in enumerate(outs):
            for k in ("xgb", "gbt", "dt"):
                assert o[k] == ref[k], f"{k} forest differs on rank {r} of {world}"
    # the trees are not trivial
    assert any(len(f["nodes"]) > 10 for f in ref["xgb"])


def _trees_fp_threads(rank, world):
    """Two job groups grown on two host threads per rank (as the GPU backend does), rank 1's second group
    delayed 25 ms before every exchange: the exchange turn order (tree_grow.hpp FpTurns) keeps the
    collectives in one order on every rank."""
    os.environ["TMOG_CPU_GROUP_THREADS"] = "1"
    os.environ["TMOG_TREE_GROUPS"] = "2"
    os.environ["TMOG_FP_DELAY"] = "1:1:25"
    from transmogrifai_amd.parallel.learner_parallel import LearnerParallel
    return _trees(LearnerParallel())


def test_feature_parallel_concurrent_groups_deterministic_order(tmp_path):
    ref = _trees(None)
    outs = _run("_trees_fp_threads", tmp_path, 3)
    for r, o in enumerate(outs):
        for k in ("xgb", "gbt", "dt"):
            assert o[k] == ref[k], f"{k} forest differs on rank {r} with concurrent groups"


def _linear(par):
    from transmogrifai_amd.models.base import FitJob, learner_class
    X, y = _data(n=2000, d=12, seed=3)
    rows = [torch.arange(0, 1500), torch.arange(500, 2000)]
    ctx = {"par": par} if par is not None else {}
    lr = learner_class("OpLogisticRegression")()
    jobs = [FitJob(dict(lr.defaults, reg_param=rp, elastic_net_param=en, max_iter=50), r)
            for rp, en in ((0.01, 0.0), (0.1, 0.5)) for r in rows]
    res = {"lr": [s["coefficients"].tolist() + [s["intercept"]] for s in lr.fit_batch(X, y, jobs, context=ctx)]}
    lin = learner_class("OpLinearRegression")()
    yr = X[:, 0] * 2.0 - X[:, 4] + 0.1 * torch.randn(X.shape[0], generator=torch.Generator().manual_seed(1))
    res["linreg"] = [s["coefficients"].tolist() + [s["intercept"]] for s in lin.fit_batch(
        X, yr, [FitJob(dict(lin.defaults, reg_param=0.05, max_iter=50), r) for r in rows], context=ctx)]
    return res


def _linear_rp(rank, world):
    from transmogrifai_amd.parallel.learner_parallel import LearnerParallel
    return _linear(LearnerParallel())


def test_row_parallel_linear_models(tmp_path):
    ref = _linear(None)
    outs = _run("_linear_rp", tmp_path, 2)
    assert outs[0] == outs[1]                      # every rank holds the same coefficients
    for k in ("lr", "linreg"):
        # same optimum up to the optimizer tolerance (fp32 partial sums are added in another order)
        np.testing.assert_allclose(np.asarray(outs[0][k]), np.asarray(ref[k]), rtol=0, atol=1.5e-3)


def test_feature_slices_balance():
    from transmogrifai_amd.parallel.learner_parallel import feature_slices
    assert feature_slices(3, [1.0] * 10, 4) is None
    sl = feature_slices(10, [5.0, 1.0, 1.0, 1.0, 1.0, 1.0], 2)
    assert sl == [(0, 5, 0, 1), (5, 10, 1, 6)]
    sl = feature_slices(8, [], 3)
    assert [s[:2] for s in sl] == [(0, 2), (2, 5), (5, 8)] and all(s[2:] == (0, 0) for s in sl)


@pytest.mark.gpu
def test_feature_parallel_rccl_path_on_one_gpu():
    """The GPU feature-parallel path (RCCL communicator per job group, on-stream ncclAllGather of the
    split records, fp_merge_kernel) forced on a 1-rank world: XGBoost / GBT / DT trees equal the plain
    single-GPU growth bit for bit. Multi-rank transport runs in the driver's multi-GPU bench."""
    _fp_one_rank(torch.device("cuda"))


def test_feature_parallel_exchange_path_one_rank_cpu():
    _fp_one_rank(torch.device("cpu"))


def _fp_one_rank(dev):
    from transmogrifai_amd.models import tree_engine as TE
    from transmogrifai_amd.models.binning import find_splits, quantize
    from transmogrifai_amd.parallel.learner_parallel import LearnerParallel
    X, y = _data(n=6000, d=40)
    X, y = X.to(dev), y.to(dev)
    par = LearnerParallel(rank=0, world=1)
    spec = find_splits(X, 32, missing_value=0.0, reserve_missing=True)
    Xb = quantize(X, spec)
    N = X.shape[0]
    g = torch.sigmoid(0.3 * X[:, 0]) - y
    t1 = torch.stack([g, 0.5 * g]).float()
    t2 = torch.full_like(t1, 0.25)
    jobs = [TE.TreeJob(m, TE.TreeParams(max_depth=6, min_child_weight=1.0, reg_lambda=1.0, gamma=0.1, eta=0.3,
                                        split_eps=1e-6), torch.arange(N, device=dev)) for m in range(2)]
    kw = dict(mode=TE.MODE_GH, kind=TE.KIND_NEWTON, t1=t1, t2=t2, B=32, missing_bin=spec.missing_bin,
              collect_leaves=True)
    gpu = dev.type == "cuda"
    ref = TE.grow_forest(Xb, spec.n_bins, jobs, csr=TE.onebin_csr(Xb, spec.n_bins) if gpu else None, **kw)
    fp = TE.fp_plan(Xb, spec.n_bins, par, sparse=True, force=True)
    assert fp is not None
    got = TE.grow_forest(Xb, spec.n_bins, jobs, csr=TE.onebin_csr(Xb, spec.n_bins, cols=fp.one_cols) if gpu else None,
                         fp=fp, **kw)
    for k in ("tree_off", "nodes", "default_left", "value"):
        assert np.array_equal(getattr(ref, k), getattr(got, k)), k
    # non-sparse (GBT variance / DT gini) slices
    spec2 = find_splits(X, 32)
    Xb2 = quantize(X, spec2)
    jobs2 = [TE.TreeJob(0, TE.TreeParams(max_depth=6), torch.arange(N, device=dev))]
    fp2 = TE.fp_plan(Xb2, spec2.n_bins, par, sparse=False, force=True)
    for mode, kind, extra in ((TE.MODE_VAR, TE.KIND_VARIANCE, dict(t1=y.float()[None, :])),
                              (TE.MODE_CLS, TE.KIND_GINI, dict(y=y, n_classes=2))):
        a = TE.grow_forest(Xb2, spec2.n_bins, jobs2, mode=mode, kind=kind, B=32, **extra)
        b = TE.grow_forest(Xb2, spec2.n_bins, jobs2, mode=mode, kind=kind, B=32, fp=fp2, **extra)
        assert np.array_equal(a.nodes, b.nodes) and np.array_equal(a.value, b.value)


def _linreg_normal_rp(rank, world):
    from transmogrifai_amd.parallel.learner_parallel import LearnerParallel
    return _linreg_normal(LearnerParallel())


def _linreg_normal(par):
    from transmogrifai_amd.models.base import FitJob, learner_class
    X, _ = _data(n=2000, d=12, seed=3)
    X = X.double()
    yr = X[:, 0] * 2.0 - X[:, 4] + 0.1 * torch.randn(X.shape[0], generator=torch.Generator().manual_seed(1),
                                                     dtype=torch.float64)
    rows = [torch.arange(0, 1500), torch.arange(500, 2000)]
    ctx = {"par": par} if par is not None else {}
    lin = learner_class("OpLinearRegression")()
    st = lin.fit_batch(X, yr, [FitJob(dict(lin.defaults, reg_param=rp, elastic_net_param=en, max_iter=100), r)
                               for rp, en in ((0.05, 0.0), (0.05, 0.5)) for r in rows], context=ctx)
    return [s["coefficients"].tolist() + [s["intercept"]] for s in st]


def test_row_parallel_normal_equations(tmp_path):
    """The normal-equation path all-reduces each rank's slice of the fold Grams (not the whole Gram per rank)."""
    ref = _linreg_normal(None)
    outs = _run("_linreg_normal_rp", tmp_path, 2)
    assert outs[0] == outs[1]
    np.testing.assert_allclose(np.asarray(outs[0]), np.asarray(ref), rtol=0, atol=1e-6)


def _trees_groups(rank, world):
    """Hybrid schedule building block: the 4 ranks form 2 groups of 2 (parallel/dist.py partition, created
    collectively); each group grows the trees feature-parallel over its own 2 ranks and its own gloo
    subgroup, group 1 with a delay so the groups' exchanges interleave."""
    from transmogrifai_amd.parallel import dist as D
    from transmogrifai_amd.parallel.learner_parallel import LearnerParallel
    grp = D.partition(2)
    assert grp.world == 2 and grp.ranks == ((0, 1) if rank < 2 else (2, 3)) and grp.rank == rank % 2
    assert D.partition(2) is grp                      # cached: no second collective creation
    if rank >= 2:
        import time
        time.sleep(0.2)
    out = _trees(LearnerParallel(group=grp))
    out["lr"] = _linear(LearnerParallel(group=grp))["lr"]
    return out


def test_rank_groups_feature_and_row_parallel(tmp_path):
    ref = _trees(None)
    ref_lr = _linear(None)["lr"]
    outs = _run("_trees_groups", tmp_path, 4)
    for r, o in enumerate(outs):
        for k in ("xgb", "gbt", "dt"):
            assert o[k] == ref[k], f"{k} forest differs on rank {r} (groups of 2)"
        # same optimum up to the optimizer tolerance (fp32 partial sums in another order), as for the world
        np.testing.assert_allclose(np.asarray(o["lr"]), np.asarray(ref_lr), rtol=0, atol=1.5e-3)
    assert outs[0]["lr"] == outs[1]["lr"] and outs[2]["lr"] == outs[3]["lr"]   # identical inside a group


@pytest.mark.gpu
def test_feature_parallel_resident_loop_on_one_gpu():
    """Feature-parallel growth on the DEVICE-PLANNED level loop (tree_resident.hip): the split records are
    all-gathered over the job group's RCCL communicator and merged on the stream between split-find and
    partition. Forced on a 1-rank world, the trees equal plain device-planned growth bit for bit, and the call
    really took the resident loop (a ResidentTree comes back, not a host-planned Forest)."""
    from transmogrifai_amd.models import tree_engine as TE
    from transmogrifai_amd.models.binning import find_splits, quantize
    from transmogrifai_amd.parallel.learner_parallel import LearnerParallel
    dev = torch.device("cuda")
    X, y = _data(n=6000, d=40)
    X, y = X.to(dev), y.to(dev)
    spec = find_splits(X, 32, missing_value=0.0, reserve_missing=True)
    Xb = quantize(X, spec)
    N = X.shape[0]
    g = torch.sigmoid(0.3 * X[:, 0]) - y
    t1 = torch.stack([g, 0.5 * g]).float()
    t2 = torch.full_like(t1, 0.25)
    jobs = [TE.TreeJob(m, TE.TreeParams(max_depth=6, min_child_weight=1.0, reg_lambda=1.0, gamma=0.1, eta=0.3,
                                        split_eps=1e-6), torch.arange(N, device=dev)) for m in range(2)]
    kw = dict(mode=TE.MODE_GH, kind=TE.KIND_NEWTON, t1=t1, t2=t2, B=32, missing_bin=spec.missing_bin,
              collect_leaves=True, groups=1, resident=True)
    ref = TE.grow_forest(Xb, spec.n_bins, jobs, csr=TE.onebin_csr(Xb, spec.n_bins), **kw)
    fp = TE.fp_plan(Xb, spec.n_bins, LearnerParallel(rank=0, world=1), sparse=True, force=True)
    got = TE.grow_forest(Xb, spec.n_bins, jobs, csr=TE.onebin_csr(Xb, spec.n_bins, cols=fp.one_cols), fp=fp, **kw)
    assert isinstance(ref, TE.ResidentTree) and isinstance(got, TE.ResidentTree)
    a, b = TE.resident_forests([ref, got])
    for k in ("tree_off", "nodes", "default_left", "value"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
    # every leaf holds the same rows; the order inside a leaf is not stable on either path (tree_resident.hip)
    assert torch.equal(ref.leaf_assign.gid, got.leaf_assign.gid)

    def by_leaf(la):
        key = la.gid.to(torch.int64) * (1 << 32) + la.rows.to(torch.int64)
        return torch.sort(key).values
    assert torch.equal(by_leaf(ref.leaf_assign), by_leaf(got.leaf_assign))
    # leaf values of the created nodes (the value buffer's tail past them is unused capacity)
    gi = ref.leaf_assign.gid.long()
    assert bool((ref.leaf_assign.value[gi] == got.leaf_assign.value[gi]).all())


@pytest.mark.gpu
def test_projected_rank_group_answers_the_exchange_locally():
    """Projection of a 2-rank feature-parallel group on one GPU (parallel/dist.py simulate): no communicator, the
    split-record exchange is answered locally (this rank's records tiled), so the device-planned loop runs with
    the group's shapes -- the projection can time hybrid schedules."""
    from transmogrifai_amd.models import tree_engine as TE
    from transmogrifai_amd.models.binning import find_splits, quantize
    from transmogrifai_amd.parallel import dist as D
    from transmogrifai_amd.parallel.learner_parallel import LearnerParallel
    dev = torch.device("cuda")
    X, y = _data(n=4000, d=40)
    X, y = X.to(dev), y.to(dev)
    spec = find_splits(X, 32, missing_value=0.0, reserve_missing=True)
    Xb = quantize(X, spec)
    N = X.shape[0]
    t1 = (torch.sigmoid(0.3 * X[:, 0]) - y).float()[None, :]
    t2 = torch.full_like(t1, 0.25)
    jobs = [TE.TreeJob(0, TE.TreeParams(max_depth=5, min_child_weight=1.0, reg_lambda=1.0, split_eps=1e-6),
                       torch.arange(N, device=dev))]
    D.simulate(1, 2)
    try:
        par = LearnerParallel()
        assert (par.rank, par.world) == (1, 2)
        fp = TE.fp_plan(Xb, spec.n_bins, par, sparse=True)
        rt = TE.grow_forest(Xb, spec.n_bins, jobs, mode=TE.MODE_GH, kind=TE.KIND_NEWTON, t1=t1, t2=t2, B=32,
                            missing_bin=spec.missing_bin, collect_leaves=True, groups=1, resident=True, fp=fp,
                            csr=TE.onebin_csr(Xb, spec.n_bins, cols=fp.one_cols))
        assert isinstance(rt, TE.ResidentTree)
        (f,) = TE.resident_forests([rt])
        internal = f.nodes[:, 2] >= 0
        assert internal.any()
        mine = set(range(fp.mlo, fp.mhi))       # only this rank's multi-bin slice (and its one-bin columns) split
        nb = np.asarray(spec.n_bins)
        multi = np.nonzero(nb != 1)[0]
        used = set(f.nodes[internal, 0].tolist())
        allowed = {int(multi[i]) for i in mine} | {int(c) for c in fp.one_cols}
        assert used <= allowed
    finally:
        D.simulate(0, 1)

"""Forest sharing across the maxDepth x minInfoGain grid: a pruned deep forest equals the forest grown
directly with the shallower depth / larger gain threshold (``tree_engine.prune_forest``), and the
selector-level learner gives every grid point the forest it would have grown on its own."""
import numpy as np
import pytest
import torch

from transmogrifai_amd.models import tree_engine as te


def _data(N=4000, F=12, B=32, seed=5):
    g = torch.Generator().manual_seed(seed)
    X = torch.randint(0, B, (N, F), dtype=torch.uint8, generator=g)
    y = ((X[:, 0].float() + 0.7 * X[:, 3].float() - 0.4 * X[:, 7].float() + 4 * torch.randn(N, generator=g))
         > 14).float()
    return X, y


def _grow(X, y, depth, gain, n_trees=4):
    rows = torch.arange(X.shape[0])
    jobs = []
    for t in range(n_trees):
        # bootstrap-like integer weights, identical for every variant
        w = torch.as_tensor(np.random.default_rng(100 + t).poisson(1.0, X.shape[0]), dtype=torch.int64)
        jobs.append(te.TreeJob(0, te.TreeParams(max_depth=depth, min_instances=5, min_info_gain=gain), rows, w))
    return te.grow_forest(X, np.full(X.shape[1], 32), jobs, mode=te.MODE_CLS, kind=te.KIND_GINI, y=y, B=32)


def _same(a: te.Forest, b: te.Forest):
    np.testing.assert_array_equal(a.tree_off, b.tree_off)
    np.testing.assert_array_equal(a.nodes, b.nodes)
    np.testing.assert_array_equal(a.default_left, b.default_left)
    np.testing.assert_array_equal(a.value, b.value)
    np.testing.assert_array_equal(a.gain, b.gain)
    np.testing.assert_array_equal(a.cover, b.cover)


def test_pruned_forest_equals_direct_growth():
    X, y = _data()
    deep = _grow(X, y, 8, 0.0005)
    for depth, gain in [(8, 0.0005), (5, 0.0005), (3, 0.0005), (8, 0.002), (5, 0.01), (2, 0.05)]:
        _same(te.prune_forest(deep, depth, gain), _grow(X, y, depth, gain))


def test_selector_share_groups_match_unshared(monkeypatch):
    """RF learner with the share on / off: every grid point's forest is identical when the per-node feature
    subsets are off (all features), i.e. when the grid composition does not move the random stream."""
    from transmogrifai_amd.models.base import FitJob
    from transmogrifai_amd.models.trees import RandomForestClassifierLearner
    X, y = _data(N=3000, F=8)
    Xf = X.float()
    rows = torch.arange(2400)
    jobs = [FitJob(params={"max_depth": d, "min_info_gain": g, "min_instances_per_node": m, "num_trees": 3,
                           "feature_subset_strategy": "all", "seed": 1}, rows=rows)
            for d in (2, 4, 6) for g in (0.001, 0.01) for m in (5, 50)]
    lr = RandomForestClassifierLearner()
    monkeypatch.setenv("TMOG_RF_SHARE", "0")
    ref = lr.fit_batch(Xf, y, jobs)
    monkeypatch.setenv("TMOG_RF_SHARE", "1")
    got = lr.fit_batch(Xf, y, jobs)
    for a, b in zip(ref, got):
        _same(te.Forest.from_state(a["forest"]), te.Forest.from_state(b["forest"]))


def test_hessian_gate_keeps_newton_trees_identical(monkeypatch):
    """Newton trees skip nodes whose hessian sum is below 2 x min_child_weight (no valid split exists):
    the tree structure, split gains and default directions equal the ungated growth bit for bit, with and
    without the subtraction trick. A skipped leaf takes its (g, h) totals from its parent's split
    statistics (fp32), as every max-depth leaf already does, instead of its own histogram: leaf values
    agree to fp32 rounding."""
    X, y = _data(N=6000, F=10)
    p = torch.sigmoid(torch.randn(X.shape[0], generator=torch.Generator().manual_seed(3)))
    g, h = (p - y).float(), (p * (1 - p)).float()
    rows = torch.arange(X.shape[0])
    for mcw in (1.0, 25.0, 120.0):
        jobs = [te.TreeJob(0, te.TreeParams(max_depth=7, min_child_weight=mcw, reg_lambda=1.0, eta=0.3), rows)]
        kw = dict(mode=te.MODE_GH, kind=te.KIND_NEWTON, t1=g[None, :], t2=h[None, :], B=32)
        for sub in (True, False):
            monkeypatch.setenv("TMOG_TREE_HESS_GATE", "0")
            ref = te.grow_forest(X, np.full(X.shape[1], 32), jobs, subtract=sub, **kw)
            monkeypatch.setenv("TMOG_TREE_HESS_GATE", "1")
            got = te.grow_forest(X, np.full(X.shape[1], 32), jobs, subtract=sub, **kw)
            for k in ("tree_off", "nodes", "default_left", "gain"):
                np.testing.assert_array_equal(getattr(ref, k), getattr(got, k), err_msg=k)
            np.testing.assert_allclose(got.value, ref.value, rtol=1e-5, atol=1e-7)
            np.testing.assert_allclose(got.cover, ref.cover, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_forest_predict_multi_kernel_matches_pruned_forests():
    """One walk per (row, tree) for all pruned variants (HIP forest_predict_multi_kernel) equals predicting
    each pruned forest on its own, for two models with their own rows and variant lists."""
    X, y = _data(N=5000, F=12)
    deep = _grow(X, y, 9, 0.0002, n_trees=7)
    Xc = X.cuda()
    rows_a = torch.arange(0, 5000, 3, device="cuda")
    rows_b = torch.arange(1, 4000, 2, device="cuda")
    va = [(9, 0.0002), (2, 0.0002), (5, 0.004), (7, 0.02), (0, 0.0), (9, 0.5)]
    vb = [(3, 0.001), (6, 0.001)]
    trees_a, trees_b = [0, 1, 2, 3], [4, 5, 6]
    got = te.forest_predict_multi(deep, Xc, [rows_a, rows_b], [trees_a, trees_b], [va, vb])
    for rows, ts, vs, outs in ((rows_a, trees_a, va, got[0]), (rows_b, trees_b, vb, got[1])):
        sub = te.Forest.concat([deep.tree(t) for t in ts])
        for (d, g), o in zip(vs, outs):
            want = te.forest_predict(te.prune_forest(sub, d, g), Xc, [rows], [list(range(sub.n_trees))])[0]
            torch.testing.assert_close(o, want, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_forest_predict_multi_regression_32_variants():
    """K = 1 (regression) with 32 variants: the kernel's all-variants mask must not be the undefined
    ``1u << 32`` (that silently zeroed every prediction)."""
    X, y = _data(N=3000, F=10)
    rows = torch.arange(X.shape[0])
    jobs = [te.TreeJob(0, te.TreeParams(max_depth=8, min_instances=3, min_info_gain=0.0), rows) for _ in range(3)]
    t1 = (y + 0.1 * X[:, 2].float())[None, :].contiguous()
    deep = te.grow_forest(X, np.full(X.shape[1], 32), jobs, mode=te.MODE_VAR, kind=te.KIND_VARIANCE, t1=t1, B=32)
    assert deep.K == 1
    Xc = X.cuda()
    rr = torch.arange(0, 3000, 2, device="cuda")
    vs = [(d, g) for d in (1, 2, 3, 4, 5, 6, 7, 8) for g in (0.0, 1e-4, 1e-3, 1e-2)]
    assert len(vs) == 32
    got = te.forest_predict_multi(deep, Xc, [rr], [[0, 1, 2]], [vs])[0]
    for (d, g), o in zip(vs, got):
        want = te.forest_predict(te.prune_forest(deep, d, g), Xc, [rr], [[0, 1, 2]])[0]
        torch.testing.assert_close(o, want, rtol=1e-5, atol=1e-6)
    assert float(got[-1].abs().sum()) > 0


@pytest.mark.gpu
def test_forest_predict_multi_wide_matrix_falls_back():
    """More than ~2000 columns do not fit 64 staged rows in LDS: the shared walk falls back to predicting
    each pruned forest instead of failing the RF batch."""
    X, y = _data(N=600, F=2600)
    deep = _grow(X, y, 6, 0.0005, n_trees=2)
    assert te._pm_lds_bytes(2600) > te._lds_limit(None)
    Xc = X.cuda()
    vs = [(6, 0.0005), (3, 0.0005)]
    got = te.forest_predict_multi(deep, Xc, [None], [[0, 1]], [vs])[0]
    for (d, g), o in zip(vs, got):
        want = te.forest_predict(te.prune_forest(deep, d, g), Xc, [None], [[0, 1]])[0]
        torch.testing.assert_close(o, want, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_partition_from_feature_major_copy_identical():
    """Newton growth on the GPU with the partition reading split columns from the feature-major copy
    (GrowArgs.XbT) equals growth reading the row-major matrix."""
    X, y = _data(N=20000, F=16)
    p = torch.sigmoid(torch.randn(X.shape[0], generator=torch.Generator().manual_seed(4)))
    g, h = (p - y).float().cuda(), (p * (1 - p)).float().cuda()
    Xc = X.cuda()
    rows = torch.arange(X.shape[0], device="cuda")
    jobs = [te.TreeJob(0, te.TreeParams(max_depth=8, min_child_weight=5.0, reg_lambda=1.0, eta=0.3), rows),
            te.TreeJob(0, te.TreeParams(max_depth=6, min_child_weight=1.0, reg_lambda=1.0, eta=0.3), rows[::2])]
    kw = dict(mode=te.MODE_GH, kind=te.KIND_NEWTON, t1=g[None, :], t2=h[None, :], B=32)
    a = te.grow_forest(Xc, np.full(X.shape[1], 32), jobs, **kw)
    b = te.grow_forest(Xc, np.full(X.shape[1], 32), jobs, XbT=Xc.t().contiguous(), **kw)
    _same(a, b)


def test_share_groups_regression_and_multiclass(monkeypatch):
    """Shared growth + pruning gives the unshared forests for RF regression (variance) and 3-class RF."""
    from transmogrifai_amd.models.base import FitJob
    from transmogrifai_amd.models.trees import RandomForestClassifierLearner, RandomForestRegressorLearner
    X, y = _data(N=2500, F=8)
    Xf = X.float()
    rows = torch.arange(2000)
    y3 = (X[:, 0].long() % 3).double()
    yr = X[:, 0].double() * 0.3 + X[:, 5].double() * 0.1
    for L, yy in ((RandomForestClassifierLearner(), y3), (RandomForestRegressorLearner(), yr)):
        jobs = [FitJob(params={"max_depth": d, "min_info_gain": g, "min_instances_per_node": 5, "num_trees": 3,
                               "feature_subset_strategy": "all", "seed": 2}, rows=rows)
                for d in (3, 7) for g in (0.0, 0.01)]
        monkeypatch.setenv("TMOG_RF_SHARE", "0")
        ref = L.fit_batch(Xf, yy, jobs)
        monkeypatch.setenv("TMOG_RF_SHARE", "1")
        got = L.fit_batch(Xf, yy, jobs)
        for a, b in zip(ref, got):
            fa, fb = te.Forest.from_state(a["forest"]), te.Forest.from_state(b["forest"])
            for k in ("tree_off", "nodes", "default_left", "gain"):
                np.testing.assert_array_equal(getattr(fa, k), getattr(fb, k), err_msg=k)
            # a node pruned to a leaf keeps the statistics of its own histogram, where direct growth
            # (leaf at max depth, no histogram) derives a right child's from parent - left in fp32:
            # class counts are exact, regression sums agree to fp32 rounding
            np.testing.assert_allclose(fb.value, fa.value, rtol=1e-6, atol=1e-6)
        pr = L.predict_batch(got, Xf, [rows] * len(jobs))
        for st, (p0, r0, q0) in zip(ref, pr):
            p1, r1, q1 = L.predict_batch([st], Xf, [rows])[0]
            torch.testing.assert_close(r0, r1, rtol=1e-5, atol=1e-5)

"""Training sets of >= 2^24 rows (lift the 2^24-row tree cap): entries become plain 32-bit row ids of
weight 1 (``tree_engine.wide_rows``), weighted roots repeated entries. Forced on small data here
(``TMOG_TREE_WIDE_ROWS=1``): unweighted trees are identical to the packed format's, and the GPU matches the CPU
twin; the GPU test at 20M rows checks the real capacity."""
import numpy as np
import pytest
import torch

from transmogrifai_amd.models import tree_engine as te


def _newton(dev, N=6000, F=12, seed=2, n_jobs=2, depth=5):
    g = torch.Generator().manual_seed(seed)
    B = 16
    X = torch.randint(0, B - 1, (N, F), generator=g, dtype=torch.uint8)
    X[torch.rand(N, F, generator=g) < 0.1] = B - 1
    t1 = torch.round(torch.randn(n_jobs, N, generator=g) * 32) / 32 + (X[:, 1].float() - 7) / 8
    t2 = torch.rand(n_jobs, N, generator=g) * 0.25 + 0.01
    jobs = [te.TreeJob(m, te.TreeParams(max_depth=depth, min_child_weight=0.5, reg_lambda=1.0, split_eps=1e-6),
                       torch.arange(N)[torch.arange(N) % (m + 2) != 1].to(dev)) for m in range(n_jobs)]
    return te.grow_forest(X.to(dev), np.full(F, B - 1), jobs, mode=te.MODE_GH, kind=te.KIND_NEWTON, t1=t1.to(dev),
                          t2=t2.to(dev), B=B, missing_bin=B - 1, collect_leaves=True, groups=1)


def _forest_cls(dev, N=5000, F=10, seed=3):
    g = torch.Generator().manual_seed(seed)
    X = torch.randint(0, 16, (N, F), generator=g, dtype=torch.uint8)
    y = ((X[:, 0].float() + X[:, 2].float() + 4 * torch.randn(N, generator=g)) > 15).float()
    rows = torch.arange(N).to(dev)
    packed, cnts = te.bootstrap_pack(rows, [11, 12, 13], 1.0, te.wide_rows(N))
    jobs = [te.TreeJob(0, te.TreeParams(max_depth=5, min_instances=2, feature_subset=4), rows, None, s)
            for s in range(3)]
    return te.grow_forest(X.to(dev), np.full(F, 16), jobs, mode=te.MODE_CLS, kind=te.KIND_GINI, y=y.to(dev), B=16,
                          root=(packed, cnts), rng_seed=5)


def test_wide_entries_grow_the_packed_trees(monkeypatch):
    packed = _newton("cpu")
    monkeypatch.setenv("TMOG_TREE_WIDE_ROWS", "1")
    wide = _newton("cpu")
    for k in ("tree_off", "nodes", "value", "gain"):
        np.testing.assert_array_equal(getattr(packed, k), getattr(wide, k), err_msg=k)
    assert wide.leaf_assign.wide and not packed.leaf_assign.wide
    np.testing.assert_array_equal(np.sort(packed.leaf_assign.row_ids().numpy()),
                                  np.sort(wide.leaf_assign.row_ids().numpy()))


def test_wide_bootstrap_repeats_weighted_rows(monkeypatch):
    monkeypatch.setenv("TMOG_TREE_WIDE_ROWS", "1")
    rows = torch.arange(1000)
    e_wide, c_wide = te.bootstrap_pack(rows, [5, 6], 1.0, True)
    e_pack, c_pack = te.bootstrap_pack(rows, [5, 6], 1.0, False)
    ep = e_pack.to(torch.int64) & 0xFFFFFFFF
    reps = torch.repeat_interleave(ep & 0xFFFFFF, ep >> 24)
    assert torch.equal(e_wide.to(torch.int64), reps)
    assert int(c_wide.sum()) == int((ep >> 24).sum())
    f = _forest_cls("cpu")
    assert f.n_trees == 3 and len(f.nodes) > 6


@pytest.mark.gpu
def test_wide_entries_gpu_matches_cpu(monkeypatch):
    monkeypatch.setenv("TMOG_TREE_WIDE_ROWS", "1")
    for grow in (_newton, _forest_cls):
        c, g = grow("cpu"), grow("cuda")
        np.testing.assert_array_equal(c.tree_off, g.tree_off)
        np.testing.assert_array_equal(c.nodes, g.nodes)
        np.testing.assert_allclose(c.value, g.value, rtol=1e-6, atol=1e-6)


@pytest.mark.gpu
def test_twenty_million_rows_xgboost_and_forest():
    """20M-row training set (> 2^24): Newton trees and a bootstrapped forest on the GPU equal the CPU twin's."""
    N, F, B = 20_000_000, 6, 16
    g = torch.Generator(device="cuda").manual_seed(9)
    X = torch.randint(0, B - 1, (N, F), generator=g, device="cuda", dtype=torch.uint8)
    t1 = ((X[:, 0].float() - 7) / 8 + torch.randn(N, generator=g, device="cuda") * 0.5)[None].contiguous()
    t2 = torch.full((1, N), 0.25, device="cuda")
    jobs = [te.TreeJob(0, te.TreeParams(max_depth=4, min_child_weight=1.0, reg_lambda=1.0, split_eps=1e-6),
                       torch.arange(N, device="cuda"))]
    kw = dict(mode=te.MODE_GH, kind=te.KIND_NEWTON, B=B, missing_bin=B - 1, collect_leaves=True, groups=1)
    fg = te.grow_forest(X, np.full(F, B - 1), jobs, t1=t1, t2=t2, **kw)
    assert fg.leaf_assign.wide and int(fg.leaf_assign.row_ids().max()) == N - 1
    jc = [te.TreeJob(0, jobs[0].params, torch.arange(N))]
    fc = te.grow_forest(X.cpu(), np.full(F, B - 1), jc, t1=t1.cpu(), t2=t2.cpu(), **kw)
    np.testing.assert_array_equal(fc.nodes, fg.nodes)
    np.testing.assert_allclose(fc.value, fg.value, rtol=1e-6, atol=1e-6)
    # forest with Poisson bootstrap weights (repeated entries) on the same rows
    y = (X[:, 1] > 7).float()
    rows = torch.arange(N, device="cuda")
    packed, cnts = te.bootstrap_pack(rows, [1, 2], 1.0, True)
    assert int(cnts.sum()) > N                    # repeats of the rows drawn more than once
    tj = [te.TreeJob(0, te.TreeParams(max_depth=3, min_instances=2), rows, None, s) for s in range(2)]
    ff = te.grow_forest(X, np.full(F, B), tj, mode=te.MODE_CLS, kind=te.KIND_GINI, y=y, B=B, root=(packed, cnts))
    assert ff.n_trees == 2 and (ff.nodes[:, 2] >= 0).sum() >= 2

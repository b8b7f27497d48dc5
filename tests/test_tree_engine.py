"""Tree engine: host kernels vs a brute-force reference, and HIP kernels vs host kernels."""
import numpy as np
import pytest
import torch

from transmogrifai_amd.models import tree_engine as te


def _data(N=3000, F=10, B=32, seed=0, missing=False):
    g = torch.Generator().manual_seed(seed)
    X = torch.randint(0, B - (1 if missing else 0), (N, F), dtype=torch.uint8, generator=g)
    if missing:
        m = torch.rand(N, F, generator=g) < 0.2
        X[m] = B - 1
    y = ((X[:, 0].float() + 0.5 * X[:, 3].float() + 3 * torch.randn(N, generator=g)) > 20).float()
    return X, y


def _brute_root(X, y, B):
    best = (-1, None, None)
    N, F = X.shape
    tot = np.array([(y == 0).sum(), (y == 1).sum()], float)
    gini = lambda c: 1 - ((c / c.sum()) ** 2).sum() if c.sum() > 0 else 0
    pg = gini(tot)
    for f in range(F):
        for b in range(B - 1):
            left = X[:, f] <= b
            lc = np.array([((y == 0) & left).sum(), ((y == 1) & left).sum()], float)
            rc = tot - lc
            if lc.sum() < 1 or rc.sum() < 1:
                continue
            g = pg - lc.sum() / N * gini(lc) - rc.sum() / N * gini(rc)
            if g > best[0] + 1e-12:
                best = (g, f, b)
    return best


def test_root_split_matches_bruteforce():
    X, y = _data()
    jobs = [te.TreeJob(0, te.TreeParams(max_depth=1), torch.arange(X.shape[0]))]
    f = te.grow_forest(X, np.full(X.shape[1], 32), jobs, mode=te.MODE_CLS, kind=te.KIND_GINI, y=y, B=32)
    g, bf, bb = _brute_root(X.numpy(), y.numpy(), 32)
    assert f.nodes[0, 0] == bf and f.nodes[0, 1] == bb
    assert abs(f.gain[0] - g) < 1e-6


def test_predict_consistency_and_leaf_rows():
    X, y = _data(N=2000)
    jobs = [te.TreeJob(0, te.TreeParams(max_depth=5, min_instances=3), torch.arange(2000))]
    f = te.grow_forest(X, np.full(X.shape[1], 32), jobs, mode=te.MODE_CLS, kind=te.KIND_GINI, y=y, B=32)
    p = te.forest_predict(f, X, [None], [[0]])[0]
    assert p.shape == (2000, 2)
    assert torch.allclose(p.sum(1), torch.ones(2000))
    # the leaf distribution equals the empirical label mix of the rows routed there
    nodes = f.nodes
    leaf = np.zeros(2000, np.int64)
    Xn = X.numpy()
    for i in range(2000):
        k = 0
        while nodes[k, 2] >= 0:
            k = nodes[k, 2] if Xn[i, nodes[k, 0]] <= nodes[k, 1] else nodes[k, 3]
        leaf[i] = k
    for k in np.unique(leaf):
        m = leaf == k
        assert abs(y.numpy()[m].mean() - f.value[k, 1]) < 1e-5


def test_min_instances_respected():
    X, y = _data(N=1500)
    jobs = [te.TreeJob(0, te.TreeParams(max_depth=8, min_instances=50), torch.arange(1500))]
    f = te.grow_forest(X, np.full(X.shape[1], 32), jobs, mode=te.MODE_CLS, kind=te.KIND_GINI, y=y, B=32)
    assert (f.cover >= 50 - 1e-6).all()


def _grow_all(dev, mode, missing=False, subset=None, n_models=2, onebin=False):
    X, y = _data(missing=missing)
    N = X.shape[0]
    B = 32
    nbins = np.full(X.shape[1], B - 1 if missing else B)
    if onebin:                                   # one-hot / null-indicator columns: bin 0 or missing
        for c in (1, 4, 6, 7, 8, 9):
            X[:, c] = torch.where(X[:, c] > 20, 0, B - 1).to(torch.uint8)
            nbins[c] = 1
    g = torch.Generator().manual_seed(1)
    t1 = torch.round(torch.randn(n_models, N, generator=g) * 8) / 8
    t2 = torch.full((n_models, N), 0.25)
    jobs = []
    for m in range(n_models):
        rows = torch.arange(N)[torch.arange(N) % (m + 2) != 0]
        w = torch.randint(0, 3, (rows.numel(),), generator=g) if mode == te.MODE_CLS else None
        jobs.append(te.TreeJob(m, te.TreeParams(max_depth=6, min_instances=2, reg_lambda=1.0,
                                                min_child_weight=0.5, feature_subset=subset), rows, w))
    kind = {te.MODE_CLS: te.KIND_GINI, te.MODE_VAR: te.KIND_VARIANCE, te.MODE_GH: te.KIND_NEWTON}[mode]
    f = te.grow_forest(X.to(dev), nbins, [
        te.TreeJob(j.model, j.params, j.rows.to(dev), None if j.weights is None else j.weights.to(dev)) for j in jobs],
        mode=mode, kind=kind, y=y.to(dev), t1=t1.to(dev), t2=t2.to(dev), B=B,
        missing_bin=(B - 1) if missing else -1, rng_seed=3, chunk_rows=512,
        csr=te.onebin_csr(X.to(dev), nbins) if onebin else None)
    preds = te.forest_predict(f, X.to(dev), [None, torch.arange(0, N, 3).to(dev)], [[0], [1]])
    return f, [p.cpu() for p in preds]


@pytest.mark.parametrize("mode", [te.MODE_CLS, te.MODE_VAR, te.MODE_GH])
def test_cpu_engine_runs_all_modes(mode):
    f, preds = _grow_all("cpu", mode, missing=(mode == te.MODE_GH))
    assert f.n_trees == 2 and len(f.nodes) > 3


def test_onebin_csr_lists_present_entries():
    X, _ = _data(N=500, missing=True)
    nbins = np.full(X.shape[1], 31)
    for c in (2, 5, 7):
        X[:, c] = torch.where(X[:, c] > 15, 0, 31).to(torch.uint8)
        nbins[c] = 1
    ptr, col, nf = te.onebin_csr(X, nbins, block_rows=128)
    assert nf == 3 and ptr.numel() == 501 and col.dtype == torch.int16
    for r in range(0, 500, 37):
        got = col[ptr[r]:ptr[r + 1]].tolist()
        want = [i for i, c in enumerate((2, 5, 7)) if int(X[r, c]) == 0]
        assert got == want


def test_cpu_engine_one_present_bin_columns():
    """Permuted feature groups (one-present-bin columns last) still report original feature ids."""
    f, _ = _grow_all("cpu", te.MODE_GH, missing=True, n_models=3, onebin=True)
    used = set(int(v) for v in f.nodes[:, 0] if v >= 0)
    assert used and used <= set(range(10))


@pytest.mark.gpu
@pytest.mark.parametrize("mode,missing,subset", [(te.MODE_CLS, False, None), (te.MODE_CLS, False, 4),
                                                 (te.MODE_VAR, False, None), (te.MODE_GH, True, None),
                                                 (te.MODE_GH, True, "onebin")])
def test_hip_engine_matches_host(mode, missing, subset):
    onebin = subset == "onebin"
    subset = None if onebin else subset
    fc, pc = _grow_all("cpu", mode, missing, subset, n_models=3 if onebin else 2, onebin=onebin)
    fg, pg = _grow_all("cuda", mode, missing, subset, n_models=3 if onebin else 2, onebin=onebin)
    np.testing.assert_array_equal(fc.tree_off, fg.tree_off)
    np.testing.assert_array_equal(fc.nodes, fg.nodes)
    np.testing.assert_allclose(fc.value, fg.value, rtol=1e-5, atol=1e-5)
    for a, b in zip(pc, pg):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)
    from transmogrifai_amd.ops import _native
    assert _native.hip_loaded()


def _leaf_vs_walk(dev):
    X, y = _data(N=4000, missing=True)
    X = X.to(dev)
    g = torch.Generator().manual_seed(3)
    G = torch.randn(2, X.shape[0], generator=g).to(dev)
    H = (torch.rand(2, X.shape[0], generator=g) * 0.25).to(dev)
    rows = [torch.randperm(X.shape[0], generator=g)[:3000].sort().values.to(dev) for _ in range(2)]
    jobs = [te.TreeJob(k, te.TreeParams(max_depth=6, min_child_weight=0.5, reg_lambda=1.0, gamma=2.0 * k,
                                        split_eps=1e-6), rows[k]) for k in range(2)]
    f = te.grow_forest(X, np.full(10, 32), jobs, mode=te.MODE_GH, kind=te.KIND_NEWTON, t1=G, t2=H, B=32,
                       missing_bin=31, collect_leaves=True)
    la = f.leaf_assign
    assert la.rows.numel() == sum(r.numel() for r in rows)
    walk = te.forest_predict(f, X, [None, None], [[0], [1]])
    t, r, v = la.entry_tree(), la.row_ids(), la.entry_value()[:, 0]
    for k in range(2):
        m = t == k
        assert torch.equal(r[m].sort().values, rows[k])
        torch.testing.assert_close(v[m], walk[k][r[m], 0], rtol=0, atol=0)


def test_leaf_assign_matches_tree_walk_cpu():
    _leaf_vs_walk("cpu")


@pytest.mark.gpu
def test_leaf_assign_matches_tree_walk_gpu():
    _leaf_vs_walk("cuda")


@pytest.mark.gpu
def test_hip_predict_many_classes_matches_host():
    """K = 11 classes: the HIP walk accumulates 8 outputs per pass, wider K runs in class chunks."""
    g = torch.Generator().manual_seed(5)
    N, F, K = 3000, 8, 11
    X = torch.randint(0, 32, (N, F), dtype=torch.uint8, generator=g)
    y = (X[:, 0].long() * K // 32).float()
    jobs = [te.TreeJob(0, te.TreeParams(max_depth=5), torch.arange(N)) for _ in range(5)]
    f = te.grow_forest(X, np.full(F, 32), jobs, mode=te.MODE_CLS, kind=te.KIND_GINI, n_classes=K, y=y, B=32)
    rows = [torch.arange(0, N, 2), None]
    pc = te.forest_predict(f, X, rows, [[0, 1, 2], [3, 4]])
    pg = te.forest_predict(f, X.cuda(), [None if r is None else r.cuda() for r in rows], [[0, 1, 2], [3, 4]])
    for a, b in zip(pc, pg):
        torch.testing.assert_close(a, b.cpu(), rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("mode", [te.MODE_CLS, te.MODE_VAR, te.MODE_GH])
def test_native_finalize_matches_numpy(mode, monkeypatch):
    """tmog_tree_finalize_cpu == _finalize_py array for array (values, gamma pruning, regrouping, gid values)."""
    X, y = _data(N=3000, missing=(mode == te.MODE_GH))
    g = torch.Generator().manual_seed(4)
    G = torch.randn(3, X.shape[0], generator=g)
    H = torch.rand(3, X.shape[0], generator=g) * 0.25
    jobs = [te.TreeJob(k, te.TreeParams(max_depth=6, min_instances=3, reg_lambda=1.0 + k, gamma=1.5 * k, eta=0.3,
                                        min_child_weight=0.5, split_eps=1e-6), torch.arange(k, 3000, 1 + k))
            for k in range(3)]
    kind = {te.MODE_CLS: te.KIND_GINI, te.MODE_VAR: te.KIND_VARIANCE, te.MODE_GH: te.KIND_NEWTON}[mode]
    kw = dict(mode=mode, kind=kind, y=y, t1=G if mode != te.MODE_CLS else None, t2=H if mode == te.MODE_GH else None,
              B=32, missing_bin=31 if mode == te.MODE_GH else -1, collect_leaves=(mode == te.MODE_GH))
    if mode == te.MODE_VAR:
        kw["t1"] = G[:1]
    out = []
    for flag in ("1", "0"):
        monkeypatch.setenv("TMOG_FINALIZE_PY", flag)
        out.append(te.grow_forest(X, np.full(10, 31 if mode == te.MODE_GH else 32), jobs, **kw))
    a, b = out
    for name in ("tree_off", "nodes", "default_left", "value", "gain", "cover", "tree_model"):
        np.testing.assert_array_equal(getattr(a, name), getattr(b, name), err_msg=name)
    if mode == te.MODE_GH:
        assert torch.equal(a.leaf_assign.value.cpu(), b.leaf_assign.value.cpu())


def _grow_wide(dev, F=136, n_one=12, N=20_000, chunk_rows=4096):
    """XGBoost-style Newton trees on a dword-aligned matrix (F % 4 == 0): on the GPU the multi-bin groups
    run the wide-load histogram items (tree_kernels.hip hist_wide_item), groups sized in multiples of 4."""
    g = torch.Generator().manual_seed(11)
    B = 32
    X = torch.randint(0, B - 1, (N, F), generator=g, dtype=torch.uint8)
    X[torch.rand(N, F, generator=g) < 0.1] = B - 1                 # sparse missing bin
    nbins = np.full(F, B - 1)
    for c in range(F - n_one, F):
        X[:, c] = torch.where(torch.rand(N, generator=g) < 0.3, 0, B - 1).to(torch.uint8)
        nbins[c] = 1
    t1 = torch.round(torch.randn(3, N, generator=g) * 64) / 64 + (X[:, 3].float() - 15) / 16
    t2 = torch.rand(3, N, generator=g) * 0.25 + 0.01
    jobs = [te.TreeJob(m, te.TreeParams(max_depth=7, min_child_weight=0.5, reg_lambda=1.0, gamma=0.1 * m,
                                        split_eps=1e-6), torch.arange(N)[torch.arange(N) % (m + 2) != 1].to(dev))
            for m in range(3)]
    Xd = X.to(dev)
    f = te.grow_forest(Xd, nbins, jobs, mode=te.MODE_GH, kind=te.KIND_NEWTON, t1=t1.to(dev), t2=t2.to(dev), B=B,
                       missing_bin=B - 1, chunk_rows=chunk_rows,
                       csr=te.onebin_csr(Xd, nbins) if n_one else None)
    return f


def test_cpu_engine_dword_aligned_matrix():
    f = _grow_wide("cpu", N=3000)
    assert f.n_trees == 3 and len(f.nodes) > 10


@pytest.mark.gpu
@pytest.mark.parametrize("F,n_one,chunk", [(136, 12, 4096), (68, 0, 1024), (200, 24, 512)])
def test_hip_wide_hist_matches_host(F, n_one, chunk):
    fc = _grow_wide("cpu", F, n_one, chunk_rows=chunk)
    fg = _grow_wide("cuda", F, n_one, chunk_rows=chunk)
    np.testing.assert_array_equal(fc.tree_off, fg.tree_off)
    np.testing.assert_array_equal(fc.nodes, fg.nodes)
    np.testing.assert_allclose(fc.value, fg.value, rtol=1e-6, atol=1e-6)


def _brute_newton_root(X, g, h, nb, miss, lam, mcw):
    """Exhaustive XGBoost root split (sparsity-aware: missing rows go left or right) with the gain
    G_L^2/(H_L+lam) + G_R^2/(H_R+lam) - G^2/(H+lam) (XGBoost's loss change, no 1/2, gamma compared to it)."""
    G, H = g.sum(), h.sum()
    parent = G * G / (H + lam)
    best = (-np.inf, None, None, None)
    for f in range(X.shape[1]):
        m = X[:, f] == miss
        for b in range(int(nb[f])):
            for dl in (0, 1):
                if b == nb[f] - 1 and dl == 1:
                    continue
                left = ((X[:, f] <= b) & ~m) | (m & bool(dl))
                GL, HL = g[left].sum(), h[left].sum()
                GR, HR = G - GL, H - HL
                if HL < mcw or HR < mcw:
                    continue
                gain = GL * GL / (HL + lam) + GR * GR / (HR + lam) - parent
                if gain > best[0] + 1e-12:
                    best = (gain, f, b, dl)
    return best


def test_newton_root_split_and_leaf_values_match_hand_computation():
    """Independent check of the XGBoost objective: the root split (feature, bin, default direction),
    its loss change, the Newton leaf values -G/(H+lambda)*eta and gamma pruning, recomputed by brute force."""
    g0 = torch.Generator().manual_seed(5)
    N, F, B = 2000, 6, 16
    miss = B - 1
    X = torch.randint(0, B - 1, (N, F), generator=g0, dtype=torch.uint8)
    X[torch.rand(N, F, generator=g0) < 0.15] = miss
    nb = np.full(F, B - 1)
    gq = torch.round((X[:, 2].double() - 7) / 4 + torch.randn(N, generator=g0, dtype=torch.float64) * 2) / 8
    hq = torch.full((N,), 0.25, dtype=torch.float64)
    lam, mcw, eta = 1.0, 1.0, 0.3
    gain, bf, bb, bdl = _brute_newton_root(X.numpy(), gq.numpy(), hq.numpy(), nb, miss, lam, mcw)
    jobs = [te.TreeJob(0, te.TreeParams(max_depth=1, min_child_weight=mcw, reg_lambda=lam, eta=eta), torch.arange(N))]
    f = te.grow_forest(X, nb, jobs, mode=te.MODE_GH, kind=te.KIND_NEWTON, t1=gq[None].float(),
                       t2=hq[None].float(), B=B, missing_bin=miss)
    assert (int(f.nodes[0, 0]), int(f.nodes[0, 1])) == (bf, bb)
    assert abs(float(f.gain[0]) - gain) <= 1e-6 * max(1.0, abs(gain))      # stored as float32
    # leaves: Newton step of the rows routed there (missing rows follow the learned default direction)
    m = X[:, bf] == miss
    left = ((X[:, bf] <= bb) & ~m) | (m & bool(bdl))
    for child, sel in ((int(f.nodes[0, 2]), left), (int(f.nodes[0, 3]), ~left)):
        want = -gq[sel].sum() / (hq[sel].sum() + lam) * eta
        assert abs(float(f.value[child].reshape(-1)[0]) - float(want)) < 1e-6
    # gamma above the loss change prunes the split (XGBoost min_split_loss), below keeps it
    for gam, n_nodes in ((gain * 1.01, 1), (gain * 0.99, 3)):
        jobs = [te.TreeJob(0, te.TreeParams(max_depth=1, min_child_weight=mcw, reg_lambda=lam, eta=eta, gamma=gam),
                           torch.arange(N))]
        fp = te.grow_forest(X, nb, jobs, mode=te.MODE_GH, kind=te.KIND_NEWTON, t1=gq[None].float(),
                            t2=hq[None].float(), B=B, missing_bin=miss)
        assert len(fp.nodes) == n_nodes


def _grow_csr_long(dev, n_multi=40, n_one=152, N=12_000, chunk_rows=4096):
    """One-present-bin columns with row lists of very different lengths (0 .. ~150 entries): the GPU's
    CSR histogram items take lane groups of 8 / 16 / 32 / 64 and, past 64 entries, the long-list loop."""
    g = torch.Generator().manual_seed(21)
    B = 32
    F = n_multi + n_one
    X = torch.randint(0, B - 1, (N, F), generator=g, dtype=torch.uint8)
    X[torch.rand(N, F, generator=g) < 0.1] = B - 1
    nbins = np.full(F, B - 1)
    dens = torch.rand(N, 1, generator=g) ** 2                       # per-row presence rate
    dens[torch.arange(N) % 7 == 0] = 0.0                            # rows with empty lists
    dens[torch.arange(N) % 11 == 0] = 0.97                          # rows with ~150 entries
    pres = torch.rand(N, n_one, generator=g) < dens
    X[:, n_multi:] = torch.where(pres, 0, B - 1).to(torch.uint8)
    nbins[n_multi:] = 1
    t1 = torch.round(torch.randn(2, N, generator=g) * 64) / 64 + pres[:, :3].float().sum(1) / 4
    t2 = torch.rand(2, N, generator=g) * 0.25 + 0.01
    jobs = [te.TreeJob(m, te.TreeParams(max_depth=6, min_child_weight=0.5, reg_lambda=1.0, split_eps=1e-6),
                       torch.arange(N)[torch.arange(N) % (m + 2) != 1].to(dev)) for m in range(2)]
    Xd = X.to(dev)
    return te.grow_forest(Xd, nbins, jobs, mode=te.MODE_GH, kind=te.KIND_NEWTON, t1=t1.to(dev), t2=t2.to(dev), B=B,
                          missing_bin=B - 1, chunk_rows=chunk_rows, csr=te.onebin_csr(Xd, nbins))


def test_cpu_engine_long_csr_lists():
    f = _grow_csr_long("cpu", N=3000)
    assert f.n_trees == 2 and len(f.nodes) > 10


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [4096, 512])
def test_hip_long_csr_lists_match_host(chunk):
    fc = _grow_csr_long("cpu", chunk_rows=chunk)
    fg = _grow_csr_long("cuda", chunk_rows=chunk)
    np.testing.assert_array_equal(fc.tree_off, fg.tree_off)
    np.testing.assert_array_equal(fc.nodes, fg.nodes)
    np.testing.assert_allclose(fc.value, fg.value, rtol=1e-6, atol=1e-6)

"""Device-planned tree growth (ops/csrc/hip/tree_resident.hip) against the host-planned grower: the same
trees bit for bit (records -> Forest), the same leaf of every training entry and the same leaf values, and
the XGBoost learner with TMOG_TREE_RESIDENT on / off producing identical models."""
import numpy as np
import pytest
import torch

from transmogrifai_amd.models import tree_engine as te


def _problem(dev, F=136, n_one=12, N=20_000, n_jobs=3, depth=7, B=32, seed=11, gamma=0.1, mcw=0.5):
    g = torch.Generator().manual_seed(seed)
    X = torch.randint(0, B - 1, (N, F), generator=g, dtype=torch.uint8)
    X[torch.rand(N, F, generator=g) < 0.1] = B - 1
    nbins = np.full(F, B - 1)
    for c in range(F - n_one, F):
        X[:, c] = torch.where(torch.rand(N, generator=g) < 0.3, 0, B - 1).to(torch.uint8)
        nbins[c] = 1
    t1 = torch.round(torch.randn(n_jobs, N, generator=g) * 64) / 64 + (X[:, 3].float() - 15) / 16
    t2 = torch.rand(n_jobs, N, generator=g) * 0.25 + 0.01
    jobs = [te.TreeJob(m, te.TreeParams(max_depth=depth - (m % 2), min_child_weight=mcw * (1 + m), reg_lambda=1.0,
                                        gamma=gamma * m, eta=0.3, split_eps=1e-6),
                       torch.arange(N)[torch.arange(N) % (m + 2) != 1].to(dev)) for m in range(n_jobs)]
    Xd = X.to(dev)
    return dict(Xb=Xd, n_bins=nbins, jobs=jobs, t1=t1.to(dev), t2=t2.to(dev), B=B, missing_bin=B - 1,
                csr=te.onebin_csr(Xd, nbins) if n_one else None)


def _grow(pb, resident, chunk_rows=4096):
    return te.grow_forest(pb["Xb"], pb["n_bins"], pb["jobs"], mode=te.MODE_GH, kind=te.KIND_NEWTON, t1=pb["t1"],
                          t2=pb["t2"], B=pb["B"], missing_bin=pb["missing_bin"], chunk_rows=chunk_rows, csr=pb["csr"],
                          collect_leaves=True, groups=1, XbT=pb["Xb"].t().contiguous(), resident=resident)


def _per_row(la, n_rows):
    """(gid, value) of every training entry keyed by (job, row): entries are unique per job."""
    rows = (la.rows.to(torch.int64) & 0xFFFFFF).cpu().numpy()
    gid = la.gid.to(torch.int64).cpu().numpy()
    job = la.tree.cpu().numpy()[gid]
    val = la.value.cpu().numpy().reshape(la.value.shape[0], -1)[gid, 0]
    key = job * n_rows + rows
    o = np.argsort(key, kind="stable")
    return key[o], gid[o], val[o]


@pytest.mark.gpu
@pytest.mark.parametrize("F,n_one,chunk,depth,gamma", [(136, 12, 4096, 7, 0.1), (68, 0, 1024, 5, 0.1),
                                                       (200, 24, 512, 9, 0.1), (66, 10, 4096, 6, 0.1),
                                                       (136, 12, 4096, 8, 0.0)])
def test_resident_trees_match_host_planned(F, n_one, chunk, depth, gamma):
    """gamma 0: the finalisation's no-pruning fast path; gamma > 0: level-wise pruning."""
    pb = _problem("cuda", F=F, n_one=n_one, depth=depth, gamma=gamma)
    host = _grow(pb, False, chunk)
    res = _grow(pb, True, chunk)
    assert isinstance(res, te.ResidentTree), "device-planned path not taken"
    (dev_forest,) = te.resident_forests([res])
    for name in ("tree_off", "nodes", "default_left", "value", "gain", "cover", "tree_model"):
        np.testing.assert_array_equal(getattr(host, name), getattr(dev_forest, name), err_msg=name)
    n_rows = int(pb["Xb"].shape[0])
    kh, gh, vh = _per_row(host.leaf_assign, n_rows)
    kr, gr, vr = _per_row(res.leaf_assign, n_rows)
    np.testing.assert_array_equal(kh, kr)
    np.testing.assert_array_equal(gh, gr)        # same created-node ids: children are numbered in split order
    np.testing.assert_array_equal(vh, vr)        # device gid values (pruning applied) = host finalisation
    from transmogrifai_amd.ops import _native
    assert _native.hip_loaded()


@pytest.mark.gpu
def test_resident_many_rounds_on_one_stream():
    """Consecutive device-planned calls reuse the slot's buffers with no host synchronisation in between."""
    pb = _problem("cuda", F=72, n_one=8, N=8000, depth=6)
    res = [_grow(pb, True) for _ in range(4)]
    host = _grow(pb, False)
    for f in te.resident_forests(res):
        np.testing.assert_array_equal(host.nodes, f.nodes)
        np.testing.assert_array_equal(host.value, f.value)


@pytest.mark.gpu
def test_xgboost_learner_resident_on_off_identical(monkeypatch):
    from transmogrifai_amd.models.base import FitJob, learner_class
    g = torch.Generator().manual_seed(3)
    N, F = 20_000, 24
    X = torch.randn(N, F, generator=g)
    X[:, 5] = (X[:, 5] > 0.7).float()
    X[torch.rand(N, F, generator=g) < 0.05] = 0.0
    y = ((X[:, 0] + 0.5 * X[:, 1] * X[:, 2] + 0.3 * torch.randn(N, generator=g)) > 0.2).float()
    Xd, yd = X.cuda(), y.cuda()
    params = [dict(num_round=30, eta=0.3, max_depth=6, min_child_weight=mcw, gamma=0.2, missing=0.0,
                   num_early_stopping_rounds=5) for mcw in (1.0, 10.0)]
    folds = [torch.arange(N)[torch.arange(N) % 3 != k].cuda() for k in range(2)]
    jobs = [FitJob(p, r) for p in params for r in folds]
    out = {}
    # host-planned; device-planned with the torch round set-up; device-planned with the fused prologue
    for flag, pro in (("0", "0"), ("1", "0"), ("1", "1")):
        monkeypatch.setenv("TMOG_TREE_RESIDENT", flag)
        monkeypatch.setenv("TMOG_XGB_PROLOGUE", pro)
        L = learner_class("OpXGBoostClassifier")()
        states = L.fit_batch(Xd, yd, jobs)
        out[flag + pro] = (states, L.predict_batch(states, Xd, [None] * len(states)))
    for key in ("10", "11"):
        for a, b in zip(out["00"][0], out[key][0]):
            assert a["num_trees"] == b["num_trees"]
            for k in ("tree_off", "nodes", "value"):
                np.testing.assert_array_equal(np.asarray(a["forest"][k]), np.asarray(b["forest"][k]),
                                              err_msg=f"{key} {k}")
        for pa, pb_ in zip(out["00"][1], out[key][1]):
            for ta, tb in zip(pa, pb_):
                torch.testing.assert_close(ta, tb, rtol=0, atol=0)


def test_resident_request_on_cpu_falls_back():
    pb = _problem("cpu", F=20, n_one=4, N=1500, depth=4)
    f = _grow(pb, True)
    assert isinstance(f, te.Forest) and f.n_trees == 3

"""Learners: batched fits match single fits, expected numerics vs numpy/sklearn-free references
(``core/src/test/.../classification/*Test.scala``, ``regression/*Test.scala``)."""
import numpy as np
import pytest
import torch

from transmogrifai_amd.models.base import FitJob, learner_class


def _bin(n=600, d=5, seed=0):
    g = np.random.default_rng(seed)
    X = g.normal(size=(n, d))
    w = g.normal(size=d)
    y = (X @ w + 0.3 * g.normal(size=n) > 0).astype(float)
    return torch.as_tensor(X), torch.as_tensor(y), w


def test_logistic_regression_batched_equals_single():
    X, y, _ = _bin()
    L = learner_class("OpLogisticRegression")()
    jobs = [FitJob({"reg_param": r, "elastic_net_param": e, "max_iter": 100}, torch.arange(0, 600, k))
            for r, e, k in [(0.01, 0.0, 1), (0.1, 0.5, 2), (0.0, 0.0, 3)]]
    batch = L.fit_batch(X, y, jobs)
    for j, b in zip(jobs, batch):
        s = L.fit_batch(X, y, [j])[0]
        np.testing.assert_allclose(s["coefficients"], b["coefficients"], atol=1e-6)


def test_logistic_regression_unregularized_matches_newton():
    X, y, _ = _bin(seed=1)
    L = learner_class("OpLogisticRegression")()
    st = L.fit(X, y, params={"reg_param": 0.0, "max_iter": 300, "tol": 1e-12})
    # Newton reference in fp64
    Xa = np.hstack([X.numpy(), np.ones((600, 1))])
    b = np.zeros(Xa.shape[1])
    for _ in range(50):
        p = 1 / (1 + np.exp(-Xa @ b))
        H = Xa.T @ (Xa * (p * (1 - p))[:, None])
        b -= np.linalg.solve(H, Xa.T @ (p - y.numpy()))
    np.testing.assert_allclose(st["coefficients"], b[:-1], rtol=1e-3, atol=1e-3)
    assert st["intercept"] == pytest.approx(b[-1], abs=1e-3)


def test_multinomial_logistic_regression():
    g = np.random.default_rng(2)
    X = g.normal(size=(900, 4))
    y = np.argmax(X[:, :3] * 2 + g.normal(scale=0.3, size=(900, 3)), 1).astype(float)
    L = learner_class("OpLogisticRegression")()
    st = L.fit(torch.as_tensor(X), torch.as_tensor(y), params={"reg_param": 0.001})
    pred, raw, prob = L.predict(st, torch.as_tensor(X))
    assert prob.shape == (900, 3) and (pred.numpy() == y).mean() > 0.85
    assert abs(st["intercepts"].sum()) < 1e-9


def test_linear_regression_matches_lstsq():
    g = np.random.default_rng(3)
    X = g.normal(size=(500, 4))
    y = X @ np.array([1.0, -2.0, 0.5, 3.0]) + 4.0 + 0.01 * g.normal(size=500)
    L = learner_class("OpLinearRegression")()
    st = L.fit(torch.as_tensor(X), torch.as_tensor(y), params={"reg_param": 0.0, "max_iter": 200, "tol": 1e-12})
    ref = np.linalg.lstsq(np.hstack([X, np.ones((500, 1))]), y, rcond=None)[0]
    np.testing.assert_allclose(st["coefficients"], ref[:4], atol=1e-3)


@pytest.mark.parametrize("family,link", [("gaussian", None), ("poisson", None), ("binomial", "logit"),
                                         ("gamma", "log")])
def test_glm_families(family, link):
    g = np.random.default_rng(4)
    X = g.normal(size=(800, 3)) * 0.5
    eta = X @ np.array([0.5, -0.3, 0.2]) + 0.4
    if family == "gaussian":
        y = eta + 0.05 * g.normal(size=800)
    elif family == "poisson":
        y = g.poisson(np.exp(eta)).astype(float)
    elif family == "binomial":
        y = (g.random(800) < 1 / (1 + np.exp(-eta))).astype(float)
    else:
        y = g.gamma(5.0, np.exp(eta) / 5.0)
    L = learner_class("OpGeneralizedLinearRegression")()
    st = L.fit(torch.as_tensor(X), torch.as_tensor(y), params={"family": family, "link": link})
    np.testing.assert_allclose(st["coefficients"], [0.5, -0.3, 0.2], atol=0.2)
    mu, _, _ = L.predict(st, torch.as_tensor(X))
    assert torch.isfinite(mu).all()


def test_glm_invalid_link_fails():
    X, y, _ = _bin()
    with pytest.raises(ValueError):
        learner_class("OpGeneralizedLinearRegression")().fit(X, y, params={"family": "poisson", "link": "logit"})


def test_mlp_learns_xor_like():
    g = np.random.default_rng(5)
    X = g.uniform(-1, 1, size=(400, 2))
    y = ((X[:, 0] > 0) ^ (X[:, 1] > 0)).astype(float)
    L = learner_class("OpMultilayerPerceptronClassifier")()
    st = L.fit(torch.as_tensor(X, dtype=torch.float32), torch.as_tensor(y),
               params={"layers": [2, 8, 2], "max_iter": 300, "seed": 1})
    pred, raw, prob = L.predict(st, torch.as_tensor(X, dtype=torch.float32))
    assert (pred.numpy() == y).mean() > 0.9


@pytest.mark.parametrize("name", ["OpRandomForestClassifier", "OpGBTClassifier", "OpDecisionTreeClassifier",
                                  "OpXGBoostClassifier", "OpNaiveBayes", "OpLinearSVC"])
def test_classifiers_beat_chance(name):
    X, y, _ = _bin(n=800, seed=6)
    if name == "OpNaiveBayes":   # multinomial NB needs count features with class-dependent rates
        g = np.random.default_rng(6)
        lam = np.where(y.numpy()[:, None] > 0, [5.0, 1.0, 3.0], [1.0, 5.0, 3.0])
        X = torch.as_tensor(g.poisson(lam).astype(float))
    L = learner_class(name)()
    tr, te = torch.arange(0, 600), torch.arange(600, 800)
    st = L.fit_batch(X, y, [FitJob(dict(L.defaults), tr)])[0]
    pred, raw, prob = L.predict(st, X[te])
    assert (pred.numpy() == y[te].numpy()).mean() > 0.7


@pytest.mark.parametrize("name", ["OpRandomForestRegressor", "OpGBTRegressor", "OpDecisionTreeRegressor",
                                  "OpXGBoostRegressor"])
def test_regressors_fit(name):
    g = np.random.default_rng(7)
    X = torch.as_tensor(g.normal(size=(800, 3)))
    y = torch.as_tensor(np.sin(X[:, 0].numpy()) * 2 + X[:, 1].numpy())
    L = learner_class(name)()
    st = L.fit_batch(X, y, [FitJob(dict(L.defaults), torch.arange(600))])[0]
    pred, _, _ = L.predict(st, X[600:])
    r2 = 1 - ((pred - y[600:]) ** 2).sum() / ((y[600:] - y[600:].mean()) ** 2).sum()
    assert float(r2) > 0.6


def test_xgb_column_permutation_leaves_trees_unchanged(monkeypatch):
    """Boosting on the multi-bin-first column order grows the same trees (features mapped back)."""
    from transmogrifai_amd.models.base import FitJob
    from transmogrifai_amd.models.trees import XGBoostClassifierLearner
    g = torch.Generator().manual_seed(9)
    n, d = 3000, 10
    X = torch.randn(n, d, generator=g)
    X[:, 1::3] = (X[:, 1::3] > 0.7).float()          # interleaved 0/1 columns
    y = ((X[:, 0] + X[:, 1] - X[:, 4] + 0.3 * torch.randn(n, generator=g)) > 0).float()
    params = dict(XGBoostClassifierLearner.defaults, num_round=6, max_depth=4, missing=0.0)
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("TMOG_XGB_COLPERM", flag)
        st = XGBoostClassifierLearner().fit_batch(X, y, [FitJob(params, torch.arange(0, n, 2))])[0]
        outs.append(st)
    np.testing.assert_array_equal(np.asarray(outs[0]["forest"]["nodes"]), np.asarray(outs[1]["forest"]["nodes"]))
    np.testing.assert_array_equal(np.asarray(outs[0]["forest"]["value"]), np.asarray(outs[1]["forest"]["value"]))


def test_linear_regression_normal_equations_match_row_objective(monkeypatch):
    """solver auto / normal (d <= 4096) solves from one weighted Gram per fold: Cholesky without L1 (equal to
    the closed-form ridge solution), OWL-QN on the Gram quadratic with L1 -- the same optimum as OWL-QN over
    the rows (Spark WeightedLeastSquares vs L-BFGS, OpLinearRegression.scala:48-209)."""
    import numpy as np
    import torch
    from transmogrifai_amd.models.base import FitJob, learner_class
    g = torch.Generator().manual_seed(7)
    N, d = 3000, 6
    X = torch.randn(N, d, generator=g, dtype=torch.float64) * torch.tensor([1.0, 2.0, 0.5, 3.0, 1.0, 1.0])
    X[:, 5] = 1.0                                          # constant column
    y = X[:, :5] @ torch.tensor([1.0, -2.0, 0.5, 0.3, 0.0], dtype=torch.float64) + 0.3 * torch.randn(N, generator=g,
                                                                                                      dtype=torch.float64)
    rows = [torch.arange(0, 2000), torch.arange(1000, 3000)]
    L = learner_class("OpLinearRegression")()
    grid = [dict(reg_param=0.0), dict(reg_param=0.1), dict(reg_param=0.1, elastic_net_param=0.5),
            dict(reg_param=0.05, elastic_net_param=1.0, fit_intercept=False), dict(reg_param=0.2, standardization=False)]
    jobs = [FitJob(dict(L.defaults, max_iter=500, tol=1e-12, **p), r) for p in grid for r in rows]
    normal = L.fit_batch(X, y, jobs)
    assert all(s["solver"] == "normal" for s in normal)
    monkeypatch.setenv("TMOG_LINREG_NORMAL", "0")
    rowwise = L.fit_batch(X, y, jobs)
    for a, b in zip(normal, rowwise):
        np.testing.assert_allclose(a["coefficients"], b["coefficients"], atol=2e-4)
        assert abs(a["intercept"] - b["intercept"]) < 2e-4
    # no regularisation: ordinary least squares
    Xr, yr = X[rows[0], :5].numpy(), y[rows[0]].numpy()
    A = np.hstack([Xr, np.ones((len(Xr), 1))])
    beta = np.linalg.lstsq(A, yr, rcond=None)[0]
    np.testing.assert_allclose(normal[0]["coefficients"][:5], beta[:5], rtol=1e-8, atol=1e-10)
    assert abs(normal[0]["coefficients"][5]) < 1e-12 and abs(normal[0]["intercept"] - beta[5]) < 1e-8


def test_xgb_early_stopping_trims_to_best_round():
    """Early stopping on the training AuPR (read back one round late so the host never waits for a round's
    epilogue): the kept trees are exactly rounds 0..best_round, where best_round is the last round that
    improved the AuPR before `num_early_stopping_rounds` rounds without improvement."""
    import torch
    from transmogrifai_amd.evaluators.metrics import binned_aupr_multi
    from transmogrifai_amd.models.base import FitJob
    from transmogrifai_amd.models.trees import XGBoostClassifierLearner
    g = torch.Generator().manual_seed(2)
    n = 3000
    X = torch.randn(n, 6, generator=g, dtype=torch.float64)
    X[:, 1:] = torch.round(X[:, 1:])
    y = ((X[:, 0] > 0.3) ^ (torch.rand(n, generator=g) < 0.15)).double()
    params = dict(XGBoostClassifierLearner.defaults, num_round=60, max_depth=2, eta=0.3,
                  num_early_stopping_rounds=3)
    L = XGBoostClassifierLearner()
    st = L.fit_batch(X, y, [FitJob(params, torch.arange(n))])[0]
    assert st["num_trees"] < 60
    # replay: the training AuPR after each round (the first r + 1 trees do not depend on later rounds)
    best, best_round = -1.0, 0
    for r in range(st["num_trees"] + 3):
        s = L.fit_batch(X, y, [FitJob(dict(params, num_early_stopping_rounds=0, num_round=r + 1),
                                      torch.arange(n))])[0]
        v = float(binned_aupr_multi([L.predict(s, X)[2][:, 1]], [y])[0])
        if v > best + 1e-12:
            best, best_round = v, r
        elif r - best_round >= 3:
            break
    assert st["num_trees"] == best_round + 1

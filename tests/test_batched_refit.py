"""Speculative refits (selector/model_selector.py + tuning/validators.py): the batched linear learners fit every
grid point on the selector's full training rows inside the CV batch; the winner's refit is then taken from
there instead of a separate fit. The model must be the one a separate refit produces."""
import numpy as np
import pytest
import torch

from transmogrifai_amd.features import types as T
from transmogrifai_amd.selector.factories import BinaryClassificationModelSelector, RegressionModelSelector
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.workflow.workflow import OpWorkflow


def _data(n=3000, seed=0, regression=False, device="cpu"):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 6))
    z = X[:, 0] - X[:, 1] + 0.3 * X[:, 2] + 0.5 * rng.normal(size=n)
    y = z if regression else (z > 0).astype(float)
    ds, feats = TestFeatureBuilder.of(("y", T.RealNN, list(y)), ("v", T.OPVector, [list(r) for r in X]),
                                      response="y")
    if device != "cpu":
        ds = ds.to(device)
    return ds, feats


def _train(monkeypatch, flag, regression=False, device="cpu", models=None):
    monkeypatch.setenv("TMOG_BATCHED_REFIT", flag)
    ds, (y, v) = _data(regression=regression, device=device)
    cls = RegressionModelSelector if regression else BinaryClassificationModelSelector
    sel = cls.with_cross_validation(seed=7, model_types_to_use=models)
    pred = sel.set_input(y, v).get_output()
    m = OpWorkflow().set_result_features(pred).set_input_dataset(ds).train()
    st = m.get_origin_stage_of(pred)
    return st.metadata["summary"], st.state


def _coef(state):
    """Every numeric array of the fitted state, flattened (coefficients, intercepts, ...)."""
    parts = []
    for k in sorted(state):
        v = state[k]
        if isinstance(v, torch.Tensor):
            v = v.detach().cpu().numpy()
        if isinstance(v, (np.ndarray, float, int)) and not isinstance(v, bool):
            parts.append(np.ravel(np.asarray(v, np.float64)))
    return np.concatenate(parts)


@pytest.mark.parametrize("regression,models", [(False, ["OpLogisticRegression"]),
                                               (True, ["OpLinearRegression"])])
def test_batched_refit_equals_separate_refit(monkeypatch, regression, models):
    s0, st0 = _train(monkeypatch, "0", regression, models=models)
    s1, st1 = _train(monkeypatch, "1", regression, models=models)
    assert s0["bestModelParameters"] == s1["bestModelParameters"]
    # host BLAS blocks a 1-column and a 9-column product differently: equal to optimiser tolerance
    np.testing.assert_allclose(_coef(st0), _coef(st1), rtol=1e-4, atol=1e-6)
    key = "AuPR" if not regression else "RootMeanSquaredError"
    assert abs(s0["holdoutEvaluation"][key] - s1["holdoutEvaluation"][key]) < 1e-3


@pytest.mark.gpu
def test_batched_refit_matches_separate_refit_on_gpu(monkeypatch):
    """The fused objective and the standardisation statistics compute every problem column independently
    (tests/test_linear_kernels.py); the optimiser's small torch column reductions still sum in a batch-width
    dependent order, so the refit inside the CV batch equals the separate refit to ~1 ulp."""
    s0, st0 = _train(monkeypatch, "0", device="cuda", models=["OpLogisticRegression"])
    s1, st1 = _train(monkeypatch, "1", device="cuda", models=["OpLogisticRegression"])
    np.testing.assert_allclose(_coef(st0), _coef(st1), rtol=1e-12, atol=1e-14)
    for k, v in s0["holdoutEvaluation"].items():
        if isinstance(v, (int, float)):
            assert abs(v - s1["holdoutEvaluation"][k]) <= 1e-9, k


def test_refit_rides_in_the_cv_batch(monkeypatch):
    """With the speculative refit the learner is fitted once (the CV batch + one refit job per grid point)."""
    from transmogrifai_amd.models import linear as L
    calls = []
    orig = L.LogisticRegressionLearner.fit_batch

    def spy(self, X, y, jobs, context=None):
        calls.append(len(jobs))
        return orig(self, X, y, jobs, context=context)

    monkeypatch.setattr(L.LogisticRegressionLearner, "fit_batch", spy)
    _train(monkeypatch, "1", models=["OpLogisticRegression"])
    n_grid = len(calls and BinaryClassificationModelSelector.models_and_params()["OpLogisticRegression"])
    assert calls == [n_grid * 3 + n_grid]
    calls.clear()
    _train(monkeypatch, "0", models=["OpLogisticRegression"])
    assert calls == [n_grid * 3, 1]

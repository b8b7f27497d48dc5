"""Vector-level Spark-ML estimators (stages/feature/vector_scalers.py) against numpy statements of Spark's
definitions: StandardScaler (sample std, optional centring, zero-variance -> 0), MinMaxScaler (constant column ->
midpoint), MaxAbsScaler, Normalizer (p = 1, 2, inf) and PCA (covariance eigenvectors, uncentred projection)."""
import numpy as np
import pytest

from transmogrifai_amd.features import types as T
from transmogrifai_amd.stages.feature import vector_scalers as V
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder


def _data(seed=0):
    r = np.random.default_rng(seed)
    x = r.normal(size=(50, 5)) * [1, 10, 0.1, 3, 1] + [0, 5, -2, 0, 1]
    x[:, 4] = 7.0                                          # a constant column
    ds, (vec,) = TestFeatureBuilder.of(("v", T.OPVector, x.tolist()))
    return x, ds, vec


def _run(stage, ds, vec):
    out = stage.set_input(vec).get_output()
    model = stage.fit(ds) if stage.is_estimator else stage
    return model, model.transform(ds)[out.name].values.double().numpy()


@pytest.mark.parametrize("with_mean", [False, True])
def test_standard_scaler(with_mean):
    x, ds, vec = _data()
    _, got = _run(V.OpStandardScaler(with_mean=with_mean, with_std=True), ds, vec)
    sd = x.std(0, ddof=1)
    want = (x - (x.mean(0) if with_mean else 0)) / np.where(sd > 0, sd, 1)
    want[:, sd == 0] = 0.0
    assert np.allclose(got, want, atol=1e-5)


def test_min_max_scaler():
    x, ds, vec = _data(1)
    _, got = _run(V.OpMinMaxScaler(min=-1.0, max=2.0), ds, vec)
    lo, hi = x.min(0), x.max(0)
    want = (x - lo) / np.where(hi > lo, hi - lo, 1) * 3.0 - 1.0
    want[:, hi == lo] = 0.5
    assert np.allclose(got, want, atol=1e-5)


def test_max_abs_scaler():
    x, ds, vec = _data(2)
    _, got = _run(V.OpMaxAbsScaler(), ds, vec)
    assert np.allclose(got, x / np.abs(x).max(0), atol=1e-6)


@pytest.mark.parametrize("p", [1.0, 2.0, float("inf")])
def test_normalizer(p):
    x, ds, vec = _data(3)
    _, got = _run(V.OpNormalizer(p=p), ds, vec)
    assert np.allclose(got, x / np.linalg.norm(x, ord=p, axis=1, keepdims=True), atol=1e-6)


def test_pca_projects_on_the_top_covariance_eigenvectors():
    x, ds, vec = _data(4)
    model, got = _run(V.OpPCA(k=2), ds, vec)
    w, e = np.linalg.eigh(np.cov(x, rowvar=False))
    top = e[:, np.argsort(w)[::-1][:2]]
    # same subspace, same per-component values up to the sign convention
    for j in range(2):
        a, b = got[:, j], x @ top[:, j]
        assert np.allclose(a, b, atol=1e-4) or np.allclose(a, -b, atol=1e-4)
    assert abs(float(model.explained_variance.sum()) - float(np.sort(w)[::-1][:2].sum() / w.sum())) < 1e-9
    assert [c.descriptor_value for c in model.metadata["vector_metadata"].columns] == ["pca_0", "pca_1"]

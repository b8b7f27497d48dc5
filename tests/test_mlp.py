"""Batched MLP learner (models/mlp.py): the hand-derived objective / gradient of P same-shaped MLPs
against fp64 autograd of the reference formulation (sigmoid hidden layers, softmax output, weighted mean
cross-entropy: Spark MultilayerPerceptronClassifier as wrapped by OpMultilayerPerceptronClassifier.scala:49-144),
on the host and with the fused HIP layer epilogues on the GPU; batched fits equal one-job fits."""
import numpy as np
import pytest
import torch

from transmogrifai_amd.models.base import FitJob, learner_class
from transmogrifai_amd.models.mlp import MLPObjective


def _reference(X, y, W, layers, U):
    fs = []
    for p in range(U.shape[1]):
        u = U[:, p]
        h = X.double()
        o = 0
        for i, (a, b) in enumerate(zip(layers[:-1], layers[1:])):
            Wl = u[o:o + a * b].reshape(a, b)
            o += a * b
            bl = u[o:o + b]
            o += b
            h = h @ Wl + bl
            if i < len(layers) - 2:
                h = torch.sigmoid(h)
        l = torch.nn.functional.cross_entropy(h, y, reduction="none")
        fs.append((l * W[:, p].double()).sum() / W[:, p].double().sum())
    return torch.stack(fs)


def _check(dev, N=3000, d=12, K=4, P=3, layers=None, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(N, d, generator=g)
    y = torch.randint(0, K, (N,), generator=g)
    W = (torch.rand(N, P, generator=g) > 0.3).float() * (1 + torch.rand(N, P, generator=g))
    layers = layers or [d, 7, 5, K]
    obj = MLPObjective(X.to(dev), y.to(dev), W.to(dev), layers)
    U = torch.randn(obj.n_params, P, generator=g, dtype=torch.float64) * 0.4
    f, G = obj.value_grad(U.to(dev))
    fv = obj.value(U.to(dev))
    Ur = U.clone().requires_grad_()
    fr = _reference(X, y, W, layers, Ur)
    fr.sum().backward()
    np.testing.assert_allclose(f.cpu().numpy(), fr.detach().numpy(), rtol=2e-5, atol=1e-7)
    np.testing.assert_allclose(fv.cpu().numpy(), fr.detach().numpy(), rtol=2e-5, atol=1e-7)
    scale = float(Ur.grad.abs().max())
    assert float((G.cpu() - Ur.grad).abs().max()) <= 5e-5 * scale


@pytest.mark.parametrize("layers", [None, [12, 4]])
def test_mlp_objective_matches_autograd_cpu(layers):
    _check("cpu", N=800, layers=None if layers is None else [12, 4])


def test_mlp_batched_fit_equals_single_fits():
    g = np.random.default_rng(3)
    X = torch.as_tensor(g.uniform(-1, 1, size=(600, 3)), dtype=torch.float32)
    y = torch.as_tensor(((X[:, 0] > 0) ^ (X[:, 1] > 0)).numpy().astype(float))
    L = learner_class("OpMultilayerPerceptronClassifier")()
    rows = [torch.arange(0, 400), torch.arange(200, 600)]
    params = {"layers": [3, 8, 2], "max_iter": 60, "seed": 2}
    jobs = [FitJob(dict(L.defaults, **params), r, None) for r in rows]
    both = L.fit_batch(X, y, jobs)
    for j, st in zip(jobs, both):
        alone = L.fit_batch(X, y, [j])[0]
        for a, b in zip(st["weights"], alone["weights"]):
            np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5)
    pred, _, _ = L.predict(both[0], X)
    assert (pred.numpy() == y.numpy()).mean() > 0.85


@pytest.mark.gpu
@pytest.mark.parametrize("layers", [None, [12, 4], [12, 16, 8, 4]])
def test_mlp_objective_matches_autograd_gpu(layers):
    """Fused HIP bias + sigmoid and sigmoid-backprop epilogues and the shared softmax epilogue kernel."""
    _check("cuda", N=20000, layers=layers)


@pytest.mark.gpu
def test_mlp_fit_gpu_beats_chance():
    g = np.random.default_rng(5)
    X = g.uniform(-1, 1, size=(4000, 2))
    y = ((X[:, 0] > 0) ^ (X[:, 1] > 0)).astype(float)
    L = learner_class("OpMultilayerPerceptronClassifier")()
    st = L.fit(torch.as_tensor(X, dtype=torch.float32, device="cuda"), torch.as_tensor(y, device="cuda"),
               params={"layers": [2, 8, 2], "max_iter": 300, "seed": 1})
    pred, _, _ = L.predict(st, torch.as_tensor(X, dtype=torch.float32, device="cuda"))
    assert (pred.cpu().numpy() == y).mean() > 0.9

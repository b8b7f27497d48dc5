"""Sparse design matrix + fused multinomial epilogue (ops/csrc/hip/sparse_kernels.hip) vs fp64 torch references."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _sparse_x(N=20000, d=600, dense=5, density=0.03, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.where(torch.rand(N, d, generator=g) < density, torch.rand(N, d, generator=g) * 3, torch.zeros(N, d))
    X[:, :dense] = torch.randn(N, dense, generator=g)
    X[:, 7] = (torch.rand(N, generator=g) < 0.2).float()        # a 20 %-present one-hot column
    return X


def test_sparse_design_products_match_dense():
    from transmogrifai_amd.ops.linear import SparseDesign
    X = _sparse_x().cuda()
    D = SparseDesign(X)
    assert D.idx_d.numel() == 5 and D.ds == 595
    g = torch.Generator().manual_seed(1)
    for C in (7, 144, 300):
        V = torch.randn(600, C, generator=g, dtype=torch.float64)
        R = torch.randn(X.shape[0], C, generator=g, dtype=torch.float64)
        Xd = X.double().cpu()
        torch.testing.assert_close(D.mm(V.cuda()).double().cpu(), Xd @ V, rtol=2e-5, atol=2e-4)
        torch.testing.assert_close(D.tmm(R.float().cuda()).cpu(), Xd.t() @ R.float().double(), rtol=2e-5, atol=2e-3)
        torch.testing.assert_close(D.tmm(R.float().cuda(), square=True).cpu(), (Xd * Xd).t() @ R.float().double(),
                                   rtol=2e-5, atol=5e-3)


@pytest.mark.parametrize("K", [3, 6, 20])
def test_fused_multinomial_objective_matches_fp64(K):
    from transmogrifai_amd.models.linear import MultinomialObjective
    from transmogrifai_amd.ops.linear import SparseDesign
    N, d, P = 20000, 600, 4
    X = _sparse_x(N, d)
    g = torch.Generator().manual_seed(K)
    y = torch.randint(0, K, (N,), generator=g).float()
    W = (torch.rand(N, P, generator=g) < 0.7).double()
    inv_std = torch.rand(d, P, generator=g, dtype=torch.float64) + 0.5
    l2 = torch.tensor([0.0, 0.01, 0.1, 1.0], dtype=torch.float64)
    fi = torch.tensor([True, True, False, True])
    U = 0.05 * torch.randn((d + 1) * K, P, generator=g, dtype=torch.float64)
    ref = MultinomialObjective(X.double(), y.double(), W, inv_std, l2, fi, K)
    f0, g0 = ref.value_grad(U)
    v0 = ref.value(U)
    Xc = X.cuda()
    for design in (Xc, SparseDesign(Xc)):
        ob = MultinomialObjective(design, y.cuda(), W.cuda().float(), inv_std.cuda(), l2.cuda(), fi.cuda(), K)
        assert ob.fused
        f1, g1 = ob.value_grad(U.cuda())
        v1 = ob.value(U.cuda())
        torch.testing.assert_close(f1.cpu(), f0, rtol=2e-5, atol=1e-7)
        torch.testing.assert_close(v1.cpu(), v0, rtol=2e-5, atol=1e-7)
        torch.testing.assert_close(g1.cpu(), g0, rtol=2e-4, atol=2e-6)


def test_sparse_lr_fit_matches_dense_fit(monkeypatch):
    """Binary and multinomial LR fits on the sparse design equal the dense-matrix fits (same optimum)."""
    from transmogrifai_amd.models.base import FitJob, learner_class
    X = _sparse_x(N=12000, d=400).cuda()
    beta = torch.zeros(400)
    beta[:5] = torch.tensor([1.0, -1.0, 0.5, 0.0, 0.3])
    beta[7] = 1.5
    g = torch.Generator().manual_seed(3)
    yb = (torch.rand(12000, generator=g) < torch.sigmoid(X.cpu() @ beta)).float().cuda()
    ym = torch.randint(0, 3, (12000,), generator=g).float().cuda()
    lr = learner_class("OpLogisticRegression")()
    rows = [torch.arange(0, 8000, device="cuda"), torch.arange(4000, 12000, device="cuda")]
    for y in (yb, ym):
        jobs = [FitJob(dict(lr.defaults, reg_param=0.01, max_iter=60), r) for r in rows]
        a = lr.fit_batch(X, y, jobs)
        monkeypatch.setenv("TMOG_LR_SPARSE", "0")
        b = lr.fit_batch(X, y, jobs)
        monkeypatch.delenv("TMOG_LR_SPARSE")
        key = "coefficients" if "coefficients" in a[0] else "coefficient_matrix"
        for s1, s2 in zip(a, b):
            np.testing.assert_allclose(s1[key], s2[key], atol=2e-3)

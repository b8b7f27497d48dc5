"""Fused linear-model objective (ops/csrc/hip/linear_kernels.hip) vs a plain fp64 PyTorch reference."""
import pytest
import torch

from transmogrifai_amd.ops import linear as LK


def _reference(X, y, W, V, b, loss, yscale):
    Xd, yd, Wd = X.double(), y.double(), W.double()
    M = Xd @ V.double() + b.double()[None, :]
    yy = yd[:, None]
    if loss == "logistic":
        l = torch.nn.functional.softplus(M) - yy * M
        g = torch.sigmoid(M) - yy
    elif loss == "hinge":
        ys = 2 * yy - 1
        l = torch.clamp(1 - ys * M, min=0)
        g = torch.where(ys * M < 1, -ys, torch.zeros_like(M))
    else:
        r = M - yy / yscale.double()[None, :]
        l = 0.5 * r * r
        g = r
    R = g * Wd
    return (l * Wd).sum(0), R.sum(0), Xd.t() @ R


@pytest.mark.gpu
@pytest.mark.parametrize("N,d,P", [(1000, 7, 1), (4099, 33, 24), (20011, 329, 24), (3001, 384, 40), (777, 256, 3),
                                   (50000, 130, 8), (5003, 600, 24), (3001, 1500, 8), (2000, 2048, 33)])
@pytest.mark.parametrize("loss", ["logistic", "hinge", "squared"])
def test_fused_objective_matches_fp64(N, d, P, loss):
    g = torch.Generator().manual_seed(N + d + P)
    X = torch.randn(N, d, generator=g)
    X[:, ::5] = (X[:, ::5] > 0.3).float()        # one-hot-like sparse columns
    y = (torch.rand(N, generator=g) < 0.4).float() if loss != "squared" else torch.randn(N, generator=g) * 3
    W = (torch.rand(N, P, generator=g) < 0.7).float()
    V = torch.randn(d, P, generator=g) / d ** 0.5
    b = torch.randn(P, generator=g) * 0.1
    ys = torch.rand(P, generator=g) + 0.5
    fr, rr, Gr = _reference(X, y, W, V, b, loss, ys)
    dev = torch.device("cuda")
    f, r, G = LK.fused_objective(X.to(dev), y.to(dev), W.to(dev), V.to(dev), b.to(dev), loss,
                                 ys.to(dev) if loss == "squared" else None, grad=True)
    scale_f = (W.double().sum(0) + 1)
    torch.testing.assert_close(f.cpu() / scale_f, fr / scale_f, rtol=2e-5, atol=2e-6)
    torch.testing.assert_close(r.cpu() / scale_f, rr / scale_f, rtol=2e-5, atol=2e-6)
    gscale = Gr.abs().max().clamp_min(1.0)
    torch.testing.assert_close(G.cpu() / gscale, Gr / gscale, rtol=0, atol=5e-6)
    f2, r2, G2 = LK.fused_objective(X.to(dev), y.to(dev), W.to(dev), V.to(dev), b.to(dev), loss,
                                    ys.to(dev) if loss == "squared" else None, grad=False)
    assert G2 is None
    torch.testing.assert_close(f2, f, rtol=1e-12, atol=0)
    from transmogrifai_amd.ops import _native
    assert _native.hip_loaded()


@pytest.mark.gpu
@pytest.mark.parametrize("N,d", [(4099, 33), (20011, 329), (3001, 384)])
def test_fused_objective_columns_independent(N, d):
    """Each problem column is computed on its own: one column alone equals the same column inside a 24-wide
    batch bit for bit (ragged N d included) -- what lets the selector fold refits into the CV batch."""
    g = torch.Generator().manual_seed(N * 3 + d)
    X = torch.randn(N, d, generator=g).cuda()
    y = (torch.rand(N, generator=g) < 0.4).float().cuda()
    W = (torch.rand(N, 24, generator=g) < 0.7).float().cuda()
    V = (torch.randn(d, 24, generator=g) / d ** 0.5).cuda()
    b = (torch.randn(24, generator=g) * 0.1).cuda()
    f, r, G = LK.fused_objective(X, y, W, V, b, "logistic", None, grad=True)
    for k in (0, 17):
        f1, r1, G1 = LK.fused_objective(X, y, W[:, k:k + 1].contiguous(), V[:, k:k + 1].contiguous(), b[k:k + 1],
                                        "logistic", None, grad=True)
        assert torch.equal(f1[0], f[k]) and torch.equal(r1[0], r[k]) and torch.equal(G1[:, 0], G[:, k])


@pytest.mark.gpu
def test_logistic_regression_gpu_matches_cpu():
    from transmogrifai_amd.models.base import FitJob
    from transmogrifai_amd.models.linear import LogisticRegressionLearner
    g = torch.Generator().manual_seed(0)
    N, d = 6000, 40
    X = torch.randn(N, d, generator=g)
    w = torch.randn(d, generator=g)
    y = (torch.rand(N, generator=g) < torch.sigmoid(X @ w * 0.5)).double()
    jobs = [FitJob({"reg_param": rp, "elastic_net_param": en}, torch.arange(0, N, k + 1), None)
            for k, (rp, en) in enumerate([(0.0, 0.0), (0.01, 0.0), (0.1, 0.5), (0.01, 1.0)])]
    cpu = LogisticRegressionLearner().fit_batch(X.double(), y, jobs)
    gpu = LogisticRegressionLearner().fit_batch(X.float().cuda(), y.cuda(), jobs)
    for a, b in zip(cpu, gpu):
        assert abs(a["intercept"] - b["intercept"]) < 2e-3
        assert float(abs(torch.as_tensor(a["coefficients"]) - torch.as_tensor(b["coefficients"])).max()) < 2e-3


@pytest.mark.gpu
@pytest.mark.parametrize("d1,P,hist_n", [(41, 4, 0), (330, 24, 3), (330, 24, 17), (1201, 7, 10), (8454, 5, 12)])
def test_owlqn_direction_kernel_matches_torch(d1, P, hist_n):
    """Fused OWL-QN direction (pseudo-gradient, two-loop recursion over the history ring incl. wrap-around,
    orthant projection) vs the torch spec in fp64."""
    from transmogrifai_amd.models.linear import _owlqn_direction_torch
    from transmogrifai_amd.ops import linear as LK
    g0 = torch.Generator().manual_seed(d1 + P + hist_n)
    m = 10
    U = torch.randn(d1, P, generator=g0, dtype=torch.float64)
    U[torch.rand(d1, P, generator=g0) < 0.3] = 0.0
    g = torch.randn(d1, P, generator=g0, dtype=torch.float64)
    l1 = torch.where(torch.rand(d1, P, generator=g0) < 0.5, torch.full((d1, P), 0.3, dtype=torch.float64),
                     torch.zeros(d1, P, dtype=torch.float64))
    l1[-1] = 0.0
    S = torch.randn(m, d1, P, generator=g0, dtype=torch.float64) * 0.1
    Y = S + 0.05 * torch.randn(m, d1, P, generator=g0, dtype=torch.float64)
    RHO = 1.0 / (S * Y).sum(1)
    want = _owlqn_direction_torch(U, g, l1, l1 > 0, S, Y, RHO, hist_n, m)
    c = [t.cuda() for t in (U, g, l1, S, Y, RHO)]
    got = LK.owlqn_direction(*c, hist_n, m)
    for w, r in zip(want, got):
        torch.testing.assert_close(r.cpu(), w, rtol=1e-10, atol=1e-12)


@pytest.mark.gpu
def test_owlqn_candidate_kernel_matches_torch():
    """Projected line-search candidate and its Armijo sums (HIP owlqn_candidate_kernel) vs torch in fp64."""
    from transmogrifai_amd.ops import linear as LK
    g0 = torch.Generator().manual_seed(11)
    d1, P = 333, 24
    U = torch.randn(d1, P, generator=g0, dtype=torch.float64)
    U[torch.rand(d1, P, generator=g0) < 0.3] = 0.0
    D = torch.randn(d1, P, generator=g0, dtype=torch.float64)
    pg = torch.randn(d1, P, generator=g0, dtype=torch.float64)
    xi = torch.where(U != 0, torch.sign(U), torch.sign(-pg))
    l1 = torch.where(torch.rand(d1, P, generator=g0) < 0.5, torch.full((d1, P), 0.2, dtype=torch.float64),
                     torch.zeros(d1, P, dtype=torch.float64))
    alpha = torch.rand(P, generator=g0, dtype=torch.float64) + 0.1
    cand = U + alpha[None, :] * D
    cand = torch.where((l1 > 0) & (torch.sign(cand) != xi), torch.zeros_like(cand), cand)
    want = (cand, (l1 * cand.abs()).sum(0), (pg * (cand - U)).sum(0))
    got = LK.owlqn_candidate(*(t.cuda() for t in (U, D, xi, l1, pg, alpha)))
    for w, r in zip(want, got):
        torch.testing.assert_close(r.cpu(), w, rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("N,d,P", [(10_001, 33, 3), (70_000, 329, 24), (5000, 7, 40)])
def test_feature_std_kernel_matches_fp64(N, d, P):
    """Weighted per-problem column mean / std on the device (stats_kernels.hip weighted_colsums) vs fp64 torch,
    and a problem's statistics independent of the batch it is in."""
    from transmogrifai_amd.models.linear import _feature_std
    g = torch.Generator().manual_seed(N + d)
    X = torch.randn(N, d, generator=g) * torch.linspace(0.5, 20, d) + 3
    W = (torch.rand(N, P, generator=g) < 0.6).float()
    Xd, Wd = X.double(), W.double()
    n = Wd.sum(0)
    mean = (Xd.t() @ Wd) / n
    var = ((Xd * Xd).t() @ Wd - n * mean * mean) / (n - 1)
    std, mu = _feature_std(X.cuda(), W.cuda())
    torch.testing.assert_close(mu.cpu(), mean, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(std.cpu(), var.sqrt(), rtol=1e-9, atol=1e-12)
    s1, m1 = _feature_std(X.cuda(), W[:, 1:2].contiguous().cuda())
    assert torch.equal(s1[:, 0], std[:, 1]) and torch.equal(m1[:, 0], mu[:, 1])

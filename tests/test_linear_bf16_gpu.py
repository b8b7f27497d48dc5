"""bf16 linear-learner objective (ops/csrc/hip/linear_bf16_kernels.hip) against a plain fp64 torch reference of the
same op on the bf16-rounded design matrix.

The integer case checks the MFMA operand / accumulator maps exactly (every product and sum is an integer that the
bf16 high + low split and fp32 accumulation represent exactly: a wrong k order or lane map changes the result);
the real-valued cases bound the error of the V / R high + low split at fp32 accumulation."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(Xb, y, W, V, bias, loss, yscale=None):
    X = Xb.to(torch.float64)
    M = X @ V.to(torch.float64) + bias.to(torch.float64)[None, :]
    yy = y.to(torch.float64)[:, None]
    if loss == "logistic":
        l = torch.nn.functional.softplus(M) - yy * M
        g = torch.sigmoid(M) - yy
    elif loss == "hinge":
        ys = 2 * yy - 1
        l = torch.clamp(1 - ys * M, min=0)
        g = torch.where(ys * M < 1, -ys, torch.zeros_like(M))
    else:
        r = M - yy / yscale.to(torch.float64)[None, :]
        l = 0.5 * r * r
        g = r
    Wd = W.to(torch.float64)
    R = g * Wd
    return (l * Wd).sum(0), R.sum(0), X.t() @ R


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from transmogrifai_amd.ops import _native
    _native.hip()


@pytest.mark.parametrize("N,d,P", [(1000, 70, 5), (4133, 329, 40), (64, 32, 32), (777, 384, 3)])
def test_integer_design_exact(N, d, P):
    _need_gpu()
    from transmogrifai_amd.ops import linear as LK
    g = torch.Generator(device="cpu").manual_seed(N + d)
    X = torch.randint(-2, 3, (N, d), generator=g).float().cuda()
    V = torch.randint(-1, 2, (d, P), generator=g).float().cuda()
    W = torch.randint(0, 2, (N, P), generator=g).float().cuda()
    y = torch.zeros(N, device="cuda")
    bias = torch.zeros(P, device="cuda")
    ys = torch.ones(P, device="cuda")
    D = LK.Bf16Design(X)
    f, r, G = LK.fused_objective_bf16(D, y, W, V, bias, "squared", ys, grad=True)
    fr, rr, Gr = _ref(X, y, W, V, bias, "squared", ys)
    assert torch.equal(G, Gr), (G - Gr).abs().max()
    assert torch.equal(r, rr)
    assert torch.equal(f, fr)
    fv, rv, Gv = LK.fused_objective_bf16(D, y, W, V, bias, "squared", ys, grad=False)
    assert Gv is None and torch.equal(fv, fr) and torch.equal(rv, rr)


@pytest.mark.parametrize("loss", ["logistic", "hinge", "squared"])
def test_real_design_matches_fp64_of_rounded_x(loss):
    _need_gpu()
    from transmogrifai_amd.ops import linear as LK
    torch.manual_seed(3)
    N, d, P = 20011, 329, 36
    X = torch.randn(N, d, device="cuda")
    V = 0.05 * torch.randn(d, P, device="cuda")
    bias = 0.1 * torch.randn(P, device="cuda")
    y = (torch.rand(N, device="cuda") < 0.3).float()
    W = (torch.rand(N, P, device="cuda") < 0.67).float()
    ys = 0.5 + torch.rand(P, device="cuda")
    D = LK.Bf16Design(X)
    assert D.shifted and D.n_exact == 0
    Xb = D.Xb[:N, :d].double() * D.scale + D.mu         # the design the stored (centred, scaled) copy encodes
    f, r, G = LK.fused_objective_bf16(D, y, W, V, bias, loss, ys if loss == "squared" else None, grad=True)
    fr, rr, Gr = _ref(Xb, y, W, V, bias, loss, ys)
    scale_f = fr.abs().max().clamp_min(1.0)
    assert ((f - fr).abs().max() / scale_f) < 2e-5
    # r, G: sums of W l'(m) of both signs; bound against the sum of magnitudes
    assert G.shape == Gr.shape
    mag = (Xb.abs().to(torch.float64).t() @ W.to(torch.float64)).clamp_min(1.0)
    assert ((G - Gr).abs() / mag).max() < 1e-4
    assert ((r - rr).abs() / W.sum(0).to(torch.float64)).max() < 1e-4


def test_batched_objective_uses_bf16_copy():
    _need_gpu()
    from transmogrifai_amd import config as CFG
    from transmogrifai_amd.models.linear import BatchedObjective
    torch.manual_seed(5)
    N, d, P = 3000, 45, 4
    X = torch.randn(N, d, device="cuda")
    y = (torch.rand(N, device="cuda") < 0.5).float()
    W = torch.ones(N, P, device="cuda")
    inv_std = torch.ones(d, P, device="cuda", dtype=torch.float64)
    l2 = torch.full((P,), 0.01, device="cuda", dtype=torch.float64)
    fi = torch.ones(P, dtype=torch.bool, device="cuda")
    U = 0.1 * torch.randn(d + 1, P, device="cuda", dtype=torch.float64)
    old = CFG.linear_dtype()
    try:
        CFG.set_linear_dtype("fp32")
        o32 = BatchedObjective(X, y, W, inv_std, "logistic", l2, fi)
        CFG.set_linear_dtype("bf16")
        o16 = BatchedObjective(X, y, W, inv_std, "logistic", l2, fi)
    finally:
        CFG.set_linear_dtype(old)
    assert o32.bf16 is None and o16.bf16 is not None
    f32, g32 = o32.value_grad(U)
    f16, g16 = o16.value_grad(U)
    assert torch.allclose(f16, f32, rtol=5e-3)
    assert torch.allclose(g16, g32, atol=5e-3)
    # the copy is made once per design tensor
    from transmogrifai_amd.ops import linear as LK
    assert LK.Bf16Design.of(X) is o16.bf16


def test_weight_map_equals_expanded_weights():
    """Problems sharing a weight column through ``wmap`` give the bits of the expanded [N, P] weights."""
    _need_gpu()
    from transmogrifai_amd.ops import linear as LK
    torch.manual_seed(7)
    N, d, P = 9000, 100, 40
    X = torch.randn(N, d, device="cuda")
    y = (torch.rand(N, device="cuda") < 0.4).float()
    Wu = (torch.rand(N, 3, device="cuda") < 0.67).float()
    cols = [p % 3 for p in range(P)]
    Wfull = Wu[:, cols].contiguous()
    V = 0.05 * torch.randn(d, P, device="cuda")
    bias = 0.1 * torch.randn(P, device="cuda")
    D = LK.Bf16Design(X)
    a = LK.fused_objective_bf16(D, y, Wfull, V, bias, "logistic", grad=True)
    b = LK.fused_objective_bf16(D, y, Wu, V, bias, "logistic", grad=True, wmap=LK.weight_map(cols, P, X.device))
    for u, v in zip(a, b):
        assert torch.equal(u, v)


def _mnl_ref(Xb, V, y, W, bias, P, K):
    X = Xb.to(torch.float64)
    M = (X @ V.to(torch.float64) + bias.to(torch.float64)[None, :]).reshape(-1, P, K)
    lse = torch.logsumexp(M, 2)
    yi = y.long()
    my = M.gather(2, yi[:, None, None].expand(-1, P, 1))[:, :, 0]
    Wd = W.to(torch.float64)
    f = ((lse - my) * Wd).sum(0)
    R = (torch.softmax(M, 2) - torch.nn.functional.one_hot(yi, K).to(torch.float64)[:, None, :]) * Wd[:, :, None]
    R = R.reshape(-1, P * K)
    return f, R.sum(0), X.t() @ R


@pytest.mark.parametrize("N,d,P,K", [(5000, 130, 24, 6), (1203, 33, 5, 3), (700, 64, 40, 16), (2000, 150, 40, 4)])
def test_multinomial_bf16_matches_fp64(N, d, P, K):
    _need_gpu()
    from transmogrifai_amd.ops import linear as LK
    torch.manual_seed(N)
    X = torch.randn(N, d, device="cuda")
    X[:, :5] = (X[:, :5] > 0).float()                     # exact columns, stored as they are
    X[:, 5] += 1000.0                                     # large offset: centred before rounding
    D = LK.Bf16Design.of(X, pad=False)
    assert D.shifted and D.n_exact == 5
    Xb = D.Xb[:N, :d].double() * D.scale + D.mu
    V = 0.05 * torch.randn(d, P * K, device="cuda")
    bias = 0.1 * torch.randn(P * K, device="cuda")
    y = torch.randint(0, K, (N,), device="cuda").float()
    Wu = (torch.rand(N, 3, device="cuda") < 0.67).float()
    cols = [p % 3 for p in range(P)]
    wmap = torch.tensor(cols, dtype=torch.int32, device="cuda")
    f, rs, G = LK.mnl_objective_bf16(D, V, y, Wu, bias, P, K, grad=True, wmap=wmap)
    fr, rr, Gr = _mnl_ref(Xb, V, y, Wu[:, cols], bias, P, K)
    assert ((f - fr).abs() / fr.abs().clamp_min(1.0)).max() < 2e-5
    n = Wu[:, cols].sum(0).to(torch.float64)
    assert ((rs - rr).abs().reshape(P, K) / n[:, None]).max() < 1e-5
    mag = (Xb.abs().t() @ Wu[:, cols].to(torch.float64)).repeat_interleave(K, 1)
    assert ((G - Gr).abs() / mag.clamp_min(1.0)).max() < 1e-4
    fv, rv, Gv = LK.mnl_objective_bf16(D, V, y, Wu, bias, P, K, grad=False, wmap=wmap)
    assert Gv is None and torch.equal(fv, f) and torch.equal(rv, rs)


def test_multinomial_fused_equals_library_path(monkeypatch):
    """The fused kernel (K <= 6) and the library-GEMM path compute the same objective (to the fp32 sums)."""
    _need_gpu()
    from transmogrifai_amd.ops import linear as LK
    torch.manual_seed(9)
    N, d, P, K = 3001, 200, 32, 5
    X = torch.randn(N, d, device="cuda")
    D = LK.Bf16Design.of(X, pad=False)
    V = 0.05 * torch.randn(d, P * K, device="cuda")
    bias = 0.1 * torch.randn(P * K, device="cuda")
    y = torch.randint(0, K, (N,), device="cuda").float()
    W = (torch.rand(N, 2, device="cuda") < 0.7).float()
    wmap = torch.tensor([p % 2 for p in range(P)], dtype=torch.int32, device="cuda")
    a = LK.mnl_objective_bf16(D, V, y, W, bias, P, K, grad=True, wmap=wmap)
    monkeypatch.setenv("TMOG_MNL_FUSED_BF16", "0")
    b = LK.mnl_objective_bf16(D, V, y, W, bias, P, K, grad=True, wmap=wmap)
    for u, v in zip(a, b):
        assert torch.allclose(u, v, rtol=1e-5, atol=1e-4), (u - v).abs().max()


def test_objective_graph_replay_equals_eager(monkeypatch):
    """The captured objective pass (hipGraph) gives the bits of the eager pass, value and gradient, across
    several replays with different coefficients."""
    _need_gpu()
    from transmogrifai_amd import config as CFG
    from transmogrifai_amd.models import linear as L
    torch.manual_seed(13)
    N, d, P = 20000, 90, 36
    X = torch.randn(N, d, device="cuda")
    X[:, :10] = (X[:, :10] > 0).float()
    y = (torch.rand(N, device="cuda") < 0.4).float()
    W = (torch.rand(N, P, device="cuda") < 0.7).float()
    inv_std = torch.ones(d, P, device="cuda", dtype=torch.float64)
    l2 = torch.full((P,), 0.01, device="cuda", dtype=torch.float64)
    fi = torch.ones(P, dtype=torch.bool, device="cuda")
    old = CFG.linear_dtype()
    CFG.set_linear_dtype("bf16")
    try:
        monkeypatch.setattr(L, "_LR_GRAPHS", True)
        og = L.BatchedObjective(X, y, W, inv_std, "logistic", l2, fi)
        monkeypatch.setattr(L, "_LR_GRAPHS", False)
        oe = L.BatchedObjective(X, y, W, inv_std, "logistic", l2, fi)
        for k in range(3):
            U = 0.1 * torch.randn(d + 1, P, device="cuda", dtype=torch.float64)
            monkeypatch.setattr(L, "_LR_GRAPHS", True)
            fg, gg = og.value_grad(U)
            vg = og.value(U)
            monkeypatch.setattr(L, "_LR_GRAPHS", False)
            fe, ge = oe.value_grad(U)
            ve = oe.value(U)
            assert torch.equal(fg, fe) and torch.equal(gg, ge) and torch.equal(vg, ve)
        assert getattr(og, "_graphs", None) and len(og._graphs) == 2
    finally:
        CFG.set_linear_dtype(old)

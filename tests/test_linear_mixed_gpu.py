"""Lossless mixed-storage LR passes (``ops/linear.py`` MixedDesign, ``linear_kernels.hip``
``tmog_hip_lr_objective_mixed``): bf16-exact columns travel as bf16, the others as fp32, and the kernel rebuilds the
fp32 tile exactly -- so every output (losses, residual sums, gradients) is BIT-identical to the plain fp32 pass."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _design(n, d_exact, d_real, seed=0):
    g = torch.Generator().manual_seed(seed)
    ex = [(torch.rand(n, generator=g) < 0.3).float() for _ in range(d_exact // 2)]           # indicators
    ex += [torch.randint(-5, 40, (n,), generator=g).float() for _ in range(d_exact - d_exact // 2)]  # counts
    re = [torch.randn(n, generator=g) * (10 ** (i % 4)) + 1000.0 * (i % 3) for i in range(d_real)]
    cols = ex + re
    perm = torch.randperm(len(cols), generator=g)            # exact and real columns interleaved
    X = torch.stack([cols[int(i)] for i in perm], 1).contiguous()
    y = (torch.rand(n, generator=g) < 0.4).float()
    return X, y


@pytest.mark.parametrize("n,de,dr,P", [(4099, 60, 41, 7), (20000, 200, 130, 32), (3001, 16, 300, 40)])
@pytest.mark.parametrize("loss", ["logistic", "squared"])
def test_mixed_pass_is_bit_identical(monkeypatch, n, de, dr, P, loss):
    from transmogrifai_amd.ops import linear as LK
    X, y = _design(n, de, dr)
    dev = torch.device("cuda")
    X, y = X.to(dev), y.to(dev)
    g = torch.Generator().manual_seed(1)
    W = (torch.rand(n, P, generator=g) < 0.8).float().to(dev)
    V = (torch.randn(X.shape[1], P, generator=g) * 0.01).to(dev)
    b = torch.randn(P, generator=g).to(dev)
    ys = torch.rand(P, generator=g).add(0.5).to(dev) if loss == "squared" else None
    for grad in (False, True):
        monkeypatch.setenv("TMOG_LR_MIXED", "0")
        ref = LK.fused_objective(X, y, W, V, b, loss, ys, grad=grad)
        monkeypatch.setenv("TMOG_LR_MIXED", "2")
        X2 = X.clone()                       # a fresh tensor: its own mixed copy
        md = LK.MixedDesign.of(X2, grad)
        assert md is not None and md.nE == de and md.nR == dr
        got = LK.fused_objective(X2, y, W, V, b, loss, ys, grad=grad)
        assert torch.equal(ref[0], got[0]) and torch.equal(ref[1], got[1])
        if grad:
            assert torch.equal(ref[2], got[2])


def test_mixed_copy_moves_fewer_bytes(monkeypatch):
    from transmogrifai_amd.ops import linear as LK
    monkeypatch.setenv("TMOG_LR_MIXED", "1")
    X, _ = _design(1000, 200, 129)
    X = X.cuda()
    md = LK.MixedDesign.of(X)
    assert md is not None
    assert md.Xm.shape[1] == 2 * 200 + 4 * 132 < 4 * X.shape[1]
    rows = md.Xm[:, :400].view(torch.bfloat16).float()
    E = md.colmap[:200].long()
    assert torch.equal(rows, X[:, E])

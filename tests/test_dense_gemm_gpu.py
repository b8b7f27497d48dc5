"""Dense fp32 row GEMMs on the matrix cores (ops/dense.py, ops/csrc/hip/dense_kernels.hip) against fp64 torch
references of the same products: ragged shapes (N not a multiple of the 128-row tile, K of the 32-deep stage, M of the
64-column tile, one-column groups), grouped columns, per-job batches, transposed B, the fused bias + sigmoid. The
bound is fp32 product / accumulation error, relative to sum |a b| (an fp32 MFMA chain: ~1e-7 per term)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel_err(got, want, absprod):
    return float(((got.double() - want).abs() / absprod.clamp_min(1e-30)).max())


@pytest.mark.parametrize("N,K,M", [(1000, 37, 70), (4099, 300, 16), (129, 1, 1), (70000, 64, 129)])
def test_mm_and_tmm(N, K, M):
    from transmogrifai_amd.ops import dense as DN
    g = torch.Generator(device="cuda").manual_seed(N + K + M)
    X = torch.randn(N, K, device="cuda", generator=g)
    V = torch.randn(K, M, device="cuda", generator=g) + torch.arange(M, device="cuda") * 0.01   # asymmetric
    R = torch.randn(N, M, device="cuda", generator=g)
    bias = torch.randn(M, device="cuda", generator=g)
    Y = DN.mm(X, V, bias)
    want = X.double() @ V.double() + bias.double()
    assert _rel_err(Y, want, X.double().abs() @ V.double().abs() + bias.double().abs()) < 2e-6
    # the fused epilogue: sigmoid of the kernel's own fp32 sum (its accuracy is bounded above)
    S = DN.mm(X, V, bias, sigmoid=True)
    assert float((S.double() - torch.sigmoid(Y.double())).abs().max()) < 1e-6
    G = DN.tmm(X, R)
    assert G.dtype == torch.float64
    assert _rel_err(G, X.double().t() @ R.double(), X.double().abs().t() @ R.double().abs()) < 2e-6


@pytest.mark.parametrize("P,N,K,a,b", [(3, 2000, 45, 10, 7), (8, 513, 130, 33, 2), (1, 128, 5, 1, 3)])
def test_mlp_layer_products(P, N, K, a, b):
    from transmogrifai_amd.ops import dense as DN
    g = torch.Generator(device="cuda").manual_seed(P * 1000 + N)
    X = torch.randn(N, K, device="cuda", generator=g)
    W0 = torch.randn(P, K, a, device="cuda", generator=g)
    b0 = torch.randn(P, a, device="cuda", generator=g)
    H = DN.layer_shared(X, W0, b0, sigmoid=True)
    lin = DN.layer_shared(X, W0, None, sigmoid=False)
    ref = torch.einsum("nk,pka->pna", X.double(), W0.double())
    assert _rel_err(lin, ref, torch.einsum("nk,pka->pna", X.double().abs(), W0.double().abs())) < 2e-6
    assert H.shape == (P, N, a)
    assert float((H.double() - torch.sigmoid(lin.double() + b0.double()[:, None, :])).abs().max()) < 1e-6
    W1 = torch.randn(P, a, b, device="cuda", generator=g)
    b1 = torch.randn(P, b, device="cuda", generator=g)
    Z = DN.layer_batched(H, W1, b1, sigmoid=False)
    Z_ref = torch.bmm(H.double(), W1.double()) + b1.double()[:, None, :]
    assert _rel_err(Z, Z_ref, torch.bmm(H.double().abs(), W1.double().abs()) + b1.double().abs()[:, None, :]) < 2e-6
    dZ = torch.randn(P, N, b, device="cuda", generator=g)
    dH = DN.backprop_input(dZ, W1)
    dH_ref = torch.bmm(dZ.double(), W1.double().transpose(1, 2))
    assert _rel_err(dH, dH_ref, torch.bmm(dZ.double().abs(), W1.double().abs().transpose(1, 2))) < 2e-6
    G1 = DN.grad_batched(H, dZ)
    G1_ref = torch.bmm(H.double().transpose(1, 2), dZ.double())
    assert G1.shape == (P, a, b)
    assert _rel_err(G1, G1_ref, torch.bmm(H.double().abs().transpose(1, 2), dZ.double().abs())) < 2e-6
    dA = torch.randn(P, N, a, device="cuda", generator=g)
    G0 = DN.grad_shared(X, dA)
    G0_ref = torch.einsum("nk,pna->pka", X.double(), dA.double())
    assert G0.shape == (P, K, a)
    assert _rel_err(G0, G0_ref, torch.einsum("nk,pna->pka", X.double().abs(), dA.double().abs())) < 2e-6


def test_exact_integer_products_are_bit_exact():
    """Small integers: every product and partial sum is exact in fp32, so the MFMA chain must equal the exact
    result bit for bit -- a transposed row / column map or a dropped k step cannot hide in a tolerance."""
    from transmogrifai_amd.ops import dense as DN
    g = torch.Generator(device="cuda").manual_seed(7)
    X = torch.randint(-3, 4, (777, 41), device="cuda", generator=g).float()
    V = torch.randint(-3, 4, (41, 67), device="cuda", generator=g).float()
    R = torch.randint(-3, 4, (777, 67), device="cuda", generator=g).float()
    assert torch.equal(DN.mm(X, V).double(), X.double() @ V.double())
    assert torch.equal(DN.tmm(X, R), X.double().t() @ R.double())

"""Weighted fp64 Grams on the matrix cores (ops/stats.py weighted_gram, stats_kernels.hip wgram_kernel) vs the
plain fp64 PyTorch reference: LinearRegression normal equations (shared response) and GLM IRLS (one working
response per problem)."""
import pytest
import torch

from transmogrifai_amd.ops.stats import weighted_gram



def _ref(X, W, Y):
    n = X.shape[0]
    base = torch.cat([X.double(), torch.ones(n, 1, dtype=torch.float64)], 1)
    out = []
    for k in range(W.shape[1]):
        A = base if Y is None else torch.cat([base, (Y[:, k] if Y.dim() == 2 else Y).double()[:, None]], 1)
        out.append(A.t() @ (A * W[:, k:k + 1].double()))
    return torch.stack(out)


@pytest.mark.gpu
@pytest.mark.parametrize("n,d,K,ymode", [(5000, 3, 1, "none"), (70_001, 70, 3, "shared"),
                                         (40_000, 130, 6, "per"), (1000, 200, 5, "per")])
def test_weighted_gram_matches_fp64(n, d, K, ymode):
    g = torch.Generator().manual_seed(n + d)
    X = torch.randn(n, d, generator=g) * torch.linspace(0.1, 30, d)
    W = (torch.rand(n, K, generator=g) < 0.7).double() * torch.rand(n, K, generator=g, dtype=torch.float64)
    Y = None if ymode == "none" else (torch.randn(n, generator=g, dtype=torch.float64) if ymode == "shared"
                                      else torch.randn(n, K, generator=g, dtype=torch.float64))
    ref = _ref(X, W, Y)
    got = weighted_gram(X.cuda(), W.cuda(), None if Y is None else Y.cuda()).cpu()
    assert got.shape == ref.shape
    scale = ref.abs().amax().item()
    assert (got - ref).abs().max().item() <= 1e-12 * scale
    torch.testing.assert_close(got, got.transpose(1, 2), rtol=0, atol=0)


@pytest.mark.gpu
def test_weighted_gram_strided_rows():
    """A row-strided view (a block of a wider matrix) reads with its leading dimension."""
    g = torch.Generator().manual_seed(1)
    big = torch.randn(3000, 50, generator=g)
    X = big[:, 5:25]
    W = torch.rand(3000, 2, generator=g, dtype=torch.float64)
    ref = _ref(X, W, None)
    got = weighted_gram(big.cuda()[:, 5:25], W.cuda()).cpu()
    assert (got - ref).abs().max().item() <= 1e-12 * ref.abs().amax().item()


def test_weighted_gram_host_reference():
    g = torch.Generator().manual_seed(2)
    X = torch.randn(777, 9, generator=g)
    W = torch.rand(777, 3, generator=g, dtype=torch.float64)
    Y = torch.randn(777, 3, generator=g, dtype=torch.float64)
    torch.testing.assert_close(weighted_gram(X, W, Y, chunk=100), _ref(X, W, Y), rtol=1e-12, atol=1e-9)
    torch.testing.assert_close(weighted_gram(X, W, Y[:, 0]), _ref(X, W, Y[:, 0]), rtol=1e-12, atol=1e-9)

"""Exact AuPR / AuROC of many score sets on the GPU (ops/csrc/hip/metric_kernels.hip, evaluators/metrics.py
binary_areas_device) against the fp64 host curves of binary_curves (Spark BinaryClassificationMetrics with
numBins = 0): ties, chunk boundaries, single-class labels, fp32 and fp64 scores."""
import numpy as np
import pytest
import torch

from transmogrifai_amd.evaluators import metrics as M


def _case(J, n, seed, ties, dtype, pos_rate=0.3):
    g = torch.Generator().manual_seed(seed)
    S = torch.rand(J, n, generator=g, dtype=torch.float64)
    if ties:
        S = torch.round(S * ties) / ties          # few distinct values: long runs of equal scores
    y = (torch.rand(n, generator=g) < pos_rate).to(torch.float64)
    return S.to(dtype), y


@pytest.mark.gpu
@pytest.mark.parametrize("J,n,ties", [(1, 1, 0), (3, 7, 0), (5, 1024, 0), (4, 1025, 13), (6, 5000, 0),
                                      (7, 33333, 50), (2, 200_000, 1000), (3, 4097, 1),
                                      (2, 3 * 65536 + 5, 3), (1, 65536, 0), (2, 65537, 2)])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_binary_areas_device_matches_host_curves(J, n, ties, dtype):
    S, y = _case(J, n, J * 1000 + n, ties, dtype)
    pr, roc = M.binary_areas_device(S.cuda(), y.cuda())
    for j in range(J):
        c = M.binary_curves(S[j], y, 0)
        assert abs(pr[j].item() - c["AuPR"]) <= 1e-12 * max(1.0, abs(c["AuPR"])), (j, pr[j].item(), c["AuPR"])
        assert abs(roc[j].item() - c["AuROC"]) <= 1e-12, (j, roc[j].item(), c["AuROC"])
    from transmogrifai_amd.ops import _native
    assert _native.hip_loaded()


@pytest.mark.gpu
@pytest.mark.parametrize("rate", [0.0, 1.0])
def test_binary_areas_device_single_class(rate):
    S, y = _case(3, 3000, 5, 20, torch.float64, pos_rate=rate)
    pr, roc = M.binary_areas_device(S.cuda(), y.cuda())
    for j in range(3):
        c = M.binary_curves(S[j], y, 0)
        assert abs(pr[j].item() - c["AuPR"]) <= 1e-12 and abs(roc[j].item() - c["AuROC"]) <= 1e-12


@pytest.mark.gpu
def test_selection_metric_batch_equals_per_model():
    from transmogrifai_amd.evaluators.evaluators import OpBinaryClassificationEvaluator
    S, y = _case(5, 20000, 9, 0, torch.float64)
    ev = OpBinaryClassificationEvaluator(metric="AuPR")
    outs = [(None, torch.stack([-s, s], 1).cuda(), None) for s in S]
    got = ev.selection_metric_batch(y.cuda(), outs)
    want = [M.binary_curves(s, y, 0)["AuPR"] for s in S]
    np.testing.assert_allclose(got, want, rtol=1e-12)

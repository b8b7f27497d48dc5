"""Batched selection metrics equal the per-model evaluation (the selector scores all models of a fold at once)."""
import torch

from transmogrifai_amd.evaluators import metrics as M
from transmogrifai_amd.evaluators.evaluators import OpMultiClassificationEvaluator


def test_multiclass_selection_batch_matches_full_metrics():
    g = torch.Generator().manual_seed(11)
    n, K = 5000, 6
    y = torch.randint(0, K, (n,), generator=g).to(torch.float64)
    preds = [torch.randint(0, K - (j % 2), (n,), generator=g).to(torch.float64) for j in range(5)]
    preds.append(y.clone())                                   # a perfect model
    outs = [(p, None, None) for p in preds]
    for metric in ("F1", "Error", "Precision", "Recall"):
        ev = OpMultiClassificationEvaluator(metric=metric)
        got = ev.selection_metric_batch(y, outs)
        want = [M.multiclass_metrics(p, y)[metric] for p in preds]
        assert got == want, (metric, got, want)
        assert ev.selection_metric(y, preds[0], None, None) == want[0]

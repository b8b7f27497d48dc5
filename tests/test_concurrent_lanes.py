"""Concurrent learner lanes of the validator (tuning/validators.py ``_fit_eval_concurrent``): learners fitted at
once -- one host thread, HIP stream and tree-grower slot range each, as the reference's OpValidator runs its fits as
concurrent futures (OpValidator.scala:348,377) -- give exactly the metrics of the one-after-the-other path."""
import threading
import time

import pytest
import torch

from transmogrifai_amd.evaluators.evaluators import OpBinaryClassificationEvaluator
from transmogrifai_amd.tuning import validators as V

_MODELS = [
    ("OpLogisticRegression", [{"reg_param": 0.01, "elastic_net_param": 0.0}, {"reg_param": 0.1, "elastic_net_param": 0.5}]),
    ("OpRandomForestClassifier", [{"num_trees": 6, "max_depth": 4}, {"num_trees": 4, "max_depth": 6}]),
    ("OpXGBoostClassifier", [{"num_round": 12, "max_depth": 4, "eta": 0.3, "min_child_weight": 1.0},
                             {"num_round": 8, "max_depth": 5, "eta": 0.3, "min_child_weight": 10.0}]),
    ("OpNaiveBayes", [{"smoothing": 1.0}]),
]


def _problem(n, d, dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, d, generator=g)
    X[:, d // 2:] = (X[:, d // 2:] > 0.8).float()            # one-hot-like columns next to real ones
    y = ((X[:, 0] - 0.7 * X[:, 1] + X[:, d - 1] + 0.5 * torch.randn(n, generator=g)) > 0).float()
    return X.to(dev), y.to(dev)


def _validate(monkeypatch, lanes, X, y, models, max_wait=86400.0):
    monkeypatch.setenv("TMOG_LEARNER_LANES", str(lanes))
    cv = V.OpCrossValidation(num_folds=3, evaluator=OpBinaryClassificationEvaluator(), seed=5, max_wait=max_wait)
    return cv.validate(models, X, y, torch.arange(X.shape[0], device=X.device))


def _metrics(res):
    return sorted((e.model_name, tuple(sorted(e.model_parameters.items())), tuple(sorted(e.metric_values.items())))
                  for e in res.evaluations)


def _same(a, b):
    assert a.best_learner == b.best_learner and a.best_params == b.best_params
    assert a.best_metric == b.best_metric
    assert _metrics(a) == _metrics(b)


def test_concurrent_lanes_equal_sequential_cpu(monkeypatch):
    X, y = _problem(3000, 10, "cpu")
    models = [_MODELS[0], _MODELS[1], _MODELS[3]]
    seq = _validate(monkeypatch, 1, X, y, models)
    conc = _validate(monkeypatch, 3, X, y, models)
    _same(seq, conc)
    assert set(conc.timings) >= {"OpLogisticRegression", "OpRandomForestClassifier", "OpNaiveBayes"}


def test_concurrent_lanes_max_wait_drops_running_learner(monkeypatch):
    from transmogrifai_amd.models.base import learner_class, register_learner
    base = learner_class("OpNaiveBayes")

    @register_learner
    class _SlowNB2(base):
        name = "_TestSlowNaiveBayesLanes"

        def fit_batch(self, X, y, jobs, context=None):
            from transmogrifai_amd.utils import cancel
            for _ in range(30):
                time.sleep(0.1)
                cancel.check()
            return super().fit_batch(X, y, jobs, context)

    X, y = _problem(400, 4, "cpu", seed=2)
    X = X.abs()
    t0 = time.time()
    res = _validate(monkeypatch, 2, X, y, [("OpNaiveBayes", [{"smoothing": 1.0}]),
                                          ("_TestSlowNaiveBayesLanes", [{"smoothing": 1.0}])], max_wait=1.0)
    assert time.time() - t0 < 2.9
    assert res.best_learner == "OpNaiveBayes"
    assert any("_TestSlowNaiveBayesLanes" in f and "maxWait" in f for f in res.failures)
    assert not [th for th in threading.enumerate() if th.name.startswith("fit-lane-")]   # cancelled + joined


@pytest.mark.gpu
def test_concurrent_lanes_gpu_priority_equal_sequential(monkeypatch):
    """GPU lanes with and without the high-priority critical lane (TMOG_LANE_PRIO): the metrics of the sequential
    path, and every leased stream is back in the pool."""
    from transmogrifai_amd.ops import streams as SP
    X, y = _problem(20_000, 12, "cuda")
    models = [_MODELS[0], _MODELS[1], _MODELS[2]]
    seq = _validate(monkeypatch, 1, X, y, models)
    for prio in ("0", "1"):
        monkeypatch.setenv("TMOG_LANE_PRIO", prio)
        _same(seq, _validate(monkeypatch, 2, X, y, models))
        assert SP.in_use("cuda:0") == 0


@pytest.mark.gpu
def test_high_priority_stream_set():
    from transmogrifai_amd.ops import streams as SP
    hi = SP.lease("cuda:0", 2, high=True)
    assert len(hi) == 2 and all(SP.is_high(s) for s in hi)
    with torch.cuda.stream(hi[0]):
        nested = SP.lease("cuda:0", 5)            # a high-priority caller leases from the high set
    assert len(nested) == SP.n_side() - 2 and all(SP.is_high(s) for s in nested)
    lo = SP.lease("cuda:0", 1)
    assert lo and not SP.is_high(lo[0])
    SP.release("cuda:0", hi + nested + lo)
    assert SP.in_use("cuda:0") == 0

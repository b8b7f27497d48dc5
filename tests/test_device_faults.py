"""Failure handling of the model selector (tuning/validators.py, utils/device_errors.py).

* An ordinary failure drops the failing (estimator, ParamMap) fits and keeps the rest, as the reference's
  ``OpValidator.getSummary`` recovers each fit's future (``OpValidator.scala:324-353``).
* A sticky device fault (illegal address, launch failure) is NOT retried grid point by grid point on the dead
  context: it is raised as :class:`DeviceFault` at once, and ``run_main`` turns it into a non-zero exit.
* maxWait bounds wall time even for a fit that never reaches a cancellation check (stuck in a native call):
  after the cancel grace period it is abandoned.
"""
import subprocess
import sys
import textwrap
import time

import pytest
import torch

from transmogrifai_amd.evaluators.evaluators import OpBinaryClassificationEvaluator
from transmogrifai_amd.models.base import learner_class, register_learner
from transmogrifai_amd.tuning import validators as V
from transmogrifai_amd.utils.device_errors import EXIT_DEVICE_FAULT, DeviceFault, fault_in_chain, is_device_fault


def test_classification():
    assert is_device_fault(RuntimeError("HIP error: an illegal memory access was encountered"))
    assert is_device_fault(RuntimeError("hipErrorLaunchFailure: unspecified launch failure"))
    assert is_device_fault(DeviceFault("x"))
    assert not is_device_fault(RuntimeError("native tree grower failed: group 0: hipMallocAsync: out of memory"))
    assert not is_device_fault(ValueError("MLP layers [3, 2] do not match input width 4"))
    assert not is_device_fault(RuntimeError("boom"), torch.device("cpu"))
    try:
        try:
            raise RuntimeError("an illegal memory access was encountered")
        except RuntimeError as e:
            raise KeyError("wrapped") from e
    except KeyError as e:
        assert fault_in_chain(e)


def _problem(n=600, d=5, seed=1):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, d, generator=g).abs()
    y = ((X[:, 0] - X[:, 1] + 0.3 * torch.randn(n, generator=g)) > 0).float()
    return X, y


def _validate(models, max_wait=86400.0, lanes=1, monkeypatch=None):
    if monkeypatch is not None:
        monkeypatch.setenv("TMOG_LEARNER_LANES", str(lanes))
    X, y = _problem()
    cv = V.OpCrossValidation(num_folds=2, evaluator=OpBinaryClassificationEvaluator(), seed=3, max_wait=max_wait)
    return cv.validate(models, X, y, torch.arange(X.shape[0]))


_CALLS = []
base = learner_class("OpNaiveBayes")


@register_learner
class _FaultyNB(base):
    name = "_TestFaultyNB"

    def fit_batch(self, X, y, jobs, context=None):
        _CALLS.append(len(jobs))
        if any(j.params.get("smoothing") == 2.0 for j in jobs):
            raise RuntimeError(self.msg)
        return super().fit_batch(X, y, jobs, context)


def test_ordinary_failure_drops_only_the_failing_grid_point():
    _CALLS.clear()
    _FaultyNB.msg = "singular matrix"
    res = _validate([("OpNaiveBayes", [{"smoothing": 1.0}]),
                     ("_TestFaultyNB", [{"smoothing": 1.0}, {"smoothing": 2.0}])])
    assert any("_TestFaultyNB" in f and "2.0" in f for f in res.failures)
    assert any(e.model_name == "_TestFaultyNB" for e in res.evaluations)    # the good grid point survived
    assert len(_CALLS) >= 3                                                 # batch, then per grid point


@pytest.mark.parametrize("lanes", [1, 2])
def test_device_fault_is_raised_not_retried(monkeypatch, lanes):
    _CALLS.clear()
    _FaultyNB.msg = "HIP error: an illegal memory access was encountered"
    with pytest.raises(DeviceFault):
        _validate([("_TestFaultyNB", [{"smoothing": 1.0}, {"smoothing": 2.0}]),
                   ("OpNaiveBayes", [{"smoothing": 1.0}])], lanes=lanes, monkeypatch=monkeypatch)
    assert len(_CALLS) == 1                      # the failing batch only: no per-grid-point retries


@register_learner
class _StuckNB(base):
    """Stands in for a fit inside a long native call: it never reaches a cancellation check."""
    name = "_TestStuckNB"

    def fit_batch(self, X, y, jobs, context=None):
        time.sleep(4.0)
        return super().fit_batch(X, y, jobs, context)


@pytest.mark.parametrize("lanes", [1, 2])
def test_max_wait_abandons_a_fit_that_never_checks(monkeypatch, lanes):
    monkeypatch.setenv("TMOG_CANCEL_GRACE_S", "0.5")
    t0 = time.time()
    res = _validate([("OpNaiveBayes", [{"smoothing": 1.0}]), ("_TestStuckNB", [{"smoothing": 1.0}])],
                    max_wait=1.0, lanes=lanes, monkeypatch=monkeypatch)
    assert time.time() - t0 < 3.5                # maxWait + grace, not the 4 s native call
    assert res.best_learner == "OpNaiveBayes"
    assert any("_TestStuckNB" in f and "maxWait" in f for f in res.failures)


def test_run_main_exits_with_device_fault_status(tmp_path):
    code = textwrap.dedent("""
        from transmogrifai_amd.utils.device_errors import run_main
        def main():
            raise RuntimeError("HIP error: an illegal memory access was encountered")
        run_main(main, "t")
    """)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == EXIT_DEVICE_FAULT, r.stderr
    assert "fatal device fault" in r.stderr


_LANES = {}


@register_learner
class _LaneStuckNB(base):
    """A stuck fit that records the native slot lane it runs on."""
    name = "_TestLaneStuckNB"

    def fit_batch(self, X, y, jobs, context=None):
        from transmogrifai_amd.models import tree_engine as TE
        _LANES["stuck"] = TE.slot_lane()
        time.sleep(3.0)
        return super().fit_batch(X, y, jobs, context)


@register_learner
class _LaneNB(base):
    name = "_TestLaneNB"

    def fit_batch(self, X, y, jobs, context=None):
        from transmogrifai_amd.models import tree_engine as TE
        _LANES.setdefault("after", []).append(TE.slot_lane())
        return super().fit_batch(X, y, jobs, context)


@pytest.mark.parametrize("lanes", [1, 2])
def test_abandoned_fit_quarantines_its_slot_lane(monkeypatch, lanes):
    """an abandoned fit keeps running on its native tree-grower slot lane, so later fits -- of this
    validate() and of the next -- must run on other lanes until its thread exits."""
    from transmogrifai_amd.models import tree_engine as TE
    monkeypatch.setenv("TMOG_CANCEL_GRACE_S", "0.3")
    _LANES.clear()
    res = _validate([("OpNaiveBayes", [{"smoothing": 1.0}]), ("_TestLaneStuckNB", [{"smoothing": 1.0}])],
                    max_wait=0.8, lanes=lanes, monkeypatch=monkeypatch)
    assert any("_TestLaneStuckNB" in f for f in res.failures)
    stuck = _LANES["stuck"]
    assert stuck in TE.quarantined_lanes()
    assert stuck not in TE.free_lanes()
    res2 = _validate([("_TestLaneNB", [{"smoothing": 1.0}]), ("OpNaiveBayes", [{"smoothing": 2.0}])],
                     lanes=lanes, monkeypatch=monkeypatch)
    assert res2.best_learner in ("_TestLaneNB", "OpNaiveBayes")
    assert _LANES["after"] and all(b != stuck for b in _LANES["after"])
    t_end = time.time() + 10
    while stuck in TE.quarantined_lanes() and time.time() < t_end:
        time.sleep(0.1)
    assert stuck not in TE.quarantined_lanes()           # released once the abandoned thread exited

"""Concurrency instruments: the fit-progress watchdog (utils/watchdog.py) and the bounded side-stream set
(ops/streams.py) used by learner lanes, boosting parts and multi-group tree growth."""
import io
import sys
import threading
import time

import pytest
import torch

from transmogrifai_amd.utils import cancel
from transmogrifai_amd.utils import watchdog as W


def test_watchdog_records_a_stall_and_dumps_stacks(monkeypatch):
    err = io.StringIO()
    monkeypatch.setattr(sys, "stderr", err)
    W.STALLS.clear()
    blocker = threading.Event()
    t = threading.Thread(target=blocker.wait, name="stuck-lane", daemon=True)
    t.start()
    with W.Watchdog("unit", after=0.3):
        time.sleep(1.0)                 # no heartbeat: one stall, reported once
        cancel.check()                  # progress again
        time.sleep(0.15)
    blocker.set()
    assert len(W.STALLS) == 1
    rec = W.STALLS[0]
    assert rec["label"] == "unit" and rec["idle_s"] >= 0.3 and "stuck-lane" in rec["threads"]
    assert "resolved_after_s" in rec
    assert "[tmog watchdog]" in err.getvalue()


def test_watchdog_quiet_while_beating():
    W.STALLS.clear()
    with W.Watchdog("busy", after=0.4):
        for _ in range(10):
            cancel.check()
            time.sleep(0.05)
    assert W.STALLS == []


def test_stream_lease_on_cpu_is_empty():
    from transmogrifai_amd.ops import streams as SP
    assert SP.lease("cpu", 3) == []


@pytest.mark.gpu
def test_side_stream_set_is_bounded(monkeypatch):
    from transmogrifai_amd.ops import streams as SP
    dev = torch.device("cuda", 0)
    a = SP.lease(dev, 2)
    b = SP.lease(dev, 5)
    assert len(a) + len(b) == SP.n_side() and not set(map(id, a)) & set(map(id, b))
    assert SP.lease(dev, 1) == []
    SP.release(dev, a)
    c = SP.lease(dev, 5)
    assert len(c) == len(a) and {s.cuda_stream for s in c} == {s.cuda_stream for s in a}
    SP.release(dev, b)
    SP.release(dev, c)
    assert SP.in_use(dev) == 0


@pytest.mark.gpu
def test_multi_group_growth_same_trees_with_any_stream_count(monkeypatch):
    """RF-style two-group growth with 0, 1 or 3 free side streams: identical forests."""
    from transmogrifai_amd.models import tree_engine as te
    from transmogrifai_amd.ops import streams as SP
    g = torch.Generator().manual_seed(5)
    N, F = 30_000, 16
    Xb = torch.randint(0, 16, (N, F), generator=g, dtype=torch.uint8).cuda()
    y = torch.randint(0, 2, (N,), generator=g).float().cuda()
    rows = torch.arange(N).cuda()
    jobs = [te.TreeJob(0, te.TreeParams(max_depth=6, feature_subset=6), rows, None) for _ in range(6)]
    out = []
    for hold in (SP.n_side(), SP.n_side() - 1, 0):
        held = SP.lease("cuda:0", hold)
        try:
            f = te.grow_forest(Xb, [16] * F, jobs, mode=te.MODE_CLS, kind=te.KIND_GINI, n_classes=2, y=y, B=16,
                               groups=2, rng_seed=9)
        finally:
            SP.release("cuda:0", held)
        out.append(f)
    for f in out[1:]:
        assert (f.nodes == out[0].nodes).all() and (f.value == out[0].value).all()
    assert SP.in_use("cuda:0") == 0

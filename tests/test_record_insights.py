"""RecordInsightsLOCO / RecordInsightsCorr (``core/src/test/.../insights/RecordInsights*Test.scala``)."""
import json
import math

import numpy as np
import pytest
import torch

from transmogrifai_amd.features import types as T
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.testkit.spec import check_transformer
from transmogrifai_amd.stages.insights.record_insights import (RecordInsightsCorr, RecordInsightsLOCO,
                                                               parse_insights)


def _fit_lr(n=400, seed=0):
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.models.linear import OpLogisticRegression
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    rng = np.random.default_rng(seed)
    a = rng.normal(size=n)
    b = rng.normal(size=n)
    c = rng.choice(["x", "y", "z"], size=n)
    y = ((2 * a - b + (c == "x") + rng.normal(scale=0.5, size=n)) > 0).astype(float)
    ds, (lab, fa, fb, fc) = TestFeatureBuilder.of(("y", T.RealNN, list(y)), ("a", T.Real, list(a)),
                                                  ("b", T.Real, list(b)), ("c", T.PickList, list(c)),
                                                  response="y")
    vec = transmogrify([fa, fb, fc])
    pred = OpLogisticRegression(reg_param=0.0).set_input(lab, vec).get_output()
    model = OpWorkflow().set_result_features(pred, vec).set_input_dataset(ds).train()
    scored = model.score(keep_intermediate_features=True)
    lr = model.get_origin_stage_of(pred)
    return scored, vec, pred, lr


def test_loco_matches_linear_closed_form():
    scored, vec, pred, lr = _fit_lr()
    loco = RecordInsightsLOCO(lr, top_k=3).set_input(vec)
    sub = scored.take(torch.arange(20))
    out = check_transformer(loco, sub)
    w = np.asarray(lr.state["coefficients"])
    b = lr.state["intercept"]
    X = sub[vec.name].values.numpy()
    sig = lambda z: 1 / (1 + np.exp(-z))
    for i in range(20):
        ins = parse_insights(out[i])
        assert 0 < len(ins) <= 3
        m = X[i] @ w + b
        exp = {j: sig(m) - sig(m - w[j] * X[i, j]) for j in range(X.shape[1]) if X[i, j] != 0}
        top = sorted(exp.values(), key=lambda v: -abs(v))[:len(ins)]
        got = sorted((v[1][1] for v in ins.values()), key=lambda v: -abs(v))
        assert np.allclose(got, top, atol=1e-9)
        for v in ins.values():   # class-0 diff mirrors class-1 for a binary model
            assert v[0][1] == pytest.approx(-v[1][1])


def test_loco_positive_negative_strategy():
    scored, vec, pred, lr = _fit_lr(seed=1)
    loco = RecordInsightsLOCO(lr, top_k=1, top_k_strategy="positive and negative").set_input(vec)
    out = loco.transform(scored.take(torch.arange(10)))[loco.get_output().name].to_list()
    for m in out:
        vals = [v[1][1] for v in parse_insights(m).values()]
        assert len([v for v in vals if v > 0]) <= 1 and len([v for v in vals if v < 0]) <= 1


def test_record_insights_corr():
    scored, vec, pred, lr = _fit_lr(seed=2)
    est = RecordInsightsCorr(top_k=2).set_input(pred, vec)
    model = est.fit(scored)
    out = check_transformer(model, scored.take(torch.arange(15)))
    for m in out:
        ins = parse_insights(m)
        assert 1 <= len(ins) <= 4
        for v in ins.values():
            assert all(p in (0, 1) for p, _ in v)


def _fit_mixed(model_cls, n=300, seed=3, classes=2, **params):
    """Real + picklist + hashed free text + a date: plain columns, text-hash and date-circle groups."""
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    rng = np.random.default_rng(seed)
    a = rng.normal(size=n)
    c = rng.choice(["x", "y", "z"], size=n)
    words = [f"w{i}" for i in range(400)]
    txt = [" ".join(rng.choice(words, size=rng.integers(1, 6))) for _ in range(n)]
    day = 86_400_000
    dts = [int(1.5e12 + rng.integers(0, 400) * day + rng.integers(0, 24) * 3_600_000) for _ in range(n)]
    z = 2 * a + (c == "x") + np.array([0.5 * ("w1" in t) for t in txt]) + rng.normal(scale=0.5, size=n)
    y = np.digitize(z, np.quantile(z, np.linspace(0, 1, classes + 1)[1:-1])).astype(float)
    ds, (lab, fa, fc, ft, fd) = TestFeatureBuilder.of(("y", T.RealNN, list(y)), ("a", T.Real, list(a)),
                                                      ("c", T.PickList, list(c)), ("t", T.Text, txt),
                                                      ("d", T.DateTime, dts), response="y")
    vec = transmogrify([fa, fc, ft, fd])
    pred = model_cls(**params).set_input(lab, vec).get_output()
    model = OpWorkflow().set_result_features(pred, vec).set_input_dataset(ds).train()
    scored = model.score(keep_intermediate_features=True)
    return scored, vec, model.get_origin_stage_of(pred)


@pytest.mark.parametrize("strategy,agg,classes", [("abs", "Avg", 2), ("positive and negative", "Avg", 2),
                                                  ("abs", "LeaveOutVector", 2), ("abs", "Avg", 3)])
def test_loco_device_path_matches_per_record_oracle(strategy, agg, classes):
    """The device-resident LOCO (candidate scatter + one stable sort per block) gives exactly the maps of
    the round-2 per-record assembly (tests/loco_reference_impl.py), for a random forest over plain,
    text-hash-group and date-group columns."""
    from loco_reference_impl import loco_maps
    from transmogrifai_amd.models.trees import OpRandomForestClassifier
    scored, vec, rf = _fit_mixed(OpRandomForestClassifier, classes=classes, num_trees=8, max_depth=4)
    loco = RecordInsightsLOCO(rf, top_k=4, top_k_strategy=strategy, vector_aggregation_strategy=agg).set_input(vec)
    sub = scored.take(torch.arange(60))
    col = loco.transform(sub)[loco.get_output().name]
    got = col.to_list()
    X = sub[vec.name].values
    hist = sub[vec.name].metadata.column_history()
    exp = loco_maps(loco, X, hist)
    assert len(got) == len(exp) == 60
    assert any(any("_" in json.loads(k).get("columnName", "") for k in m) for m in got)
    for g, e in zip(got, exp):
        assert list(g) == list(e)
        for k in e:
            a, b = json.loads(g[k]), json.loads(e[k])
            assert [i for i, _ in a] == [i for i, _ in b]
            assert np.allclose([v for _, v in a], [v for _, v in b], rtol=0, atol=1e-12)
    # row / take paths render the same maps lazily
    assert col.row(5) == got[5]
    assert col.take(torch.tensor([7, 3])).to_list() == [got[7], got[3]]


@pytest.mark.gpu
def test_loco_100k_rows_on_device():
    """LOCO over 100K records stays on the device until the maps are read (no per-record host work in
    the transform); a sample of rows matches the per-record oracle."""
    import time
    from loco_reference_impl import loco_maps
    from transmogrifai_amd.models.trees import OpRandomForestClassifier
    from transmogrifai_amd.data.columns import VectorColumn
    from transmogrifai_amd.data.dataset import Dataset
    from transmogrifai_amd import config as CFG
    prev = CFG.default_device()
    try:
        CFG.set_default_device("cuda")
        scored, vec, rf = _fit_mixed(OpRandomForestClassifier, n=2000, num_trees=8, max_depth=4)
    finally:
        CFG.set_default_device(prev)
    base = scored[vec.name]
    reps = 100_000 // len(base) + 1
    X = base.values.repeat(reps, 1)[:100_000].cuda()
    big = Dataset({vec.name: VectorColumn(X, base.metadata)})
    loco = RecordInsightsLOCO(rf, top_k=5).set_input(vec)
    torch.cuda.synchronize()
    t0 = time.time()
    col = loco.transform(big)[loco.get_output().name]
    torch.cuda.synchronize()
    dt = time.time() - t0
    assert len(col) == 100_000 and col.cols.is_cuda
    assert dt < 30.0, dt
    idx = torch.arange(0, 100_000, 997)
    got = col.take(idx).to_list()
    exp = loco_maps(loco, X[idx.cuda()], base.metadata.column_history())
    for g, e in zip(got, exp):
        assert list(g) == list(e)
        for k in e:
            assert np.allclose([v for _, v in json.loads(g[k])], [v for _, v in json.loads(e[k])], atol=1e-9)

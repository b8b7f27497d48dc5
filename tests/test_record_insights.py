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

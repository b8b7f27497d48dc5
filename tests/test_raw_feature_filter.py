"""RawFeatureFilter (``core/src/test/.../filters/RawFeatureFilterTest.scala`` scenarios)."""
import math

import numpy as np
import pytest
import torch

from transmogrifai_amd.features import types as T
from transmogrifai_amd.filters.raw_feature_filter import (FeatureDistribution, RawFeatureFilter,
                                                          RawFeatureFilterResults, Summary)
from transmogrifai_amd.readers.base import InMemoryReader
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder


def _fd(dist, nulls=0, count=10, name="a", key=None):
    return FeatureDistribution(name, key, count, nulls, np.asarray(dist, float), [0.0, 1.0])


def test_distribution_metrics():
    a = _fd([1, 1, 0, 0], nulls=2)
    b = _fd([0, 0, 1, 1], nulls=5)
    assert a.fill_rate() == 0.8 and b.fill_rate() == 0.5
    assert a.relative_fill_rate(b) == pytest.approx(0.3)
    assert a.relative_fill_ratio(b) == pytest.approx(1.6)
    assert a.js_divergence(b) == pytest.approx(1.0)          # disjoint supports
    assert a.js_divergence(_fd([2, 2, 0, 0])) == pytest.approx(0.0)
    c = a.reduce(b)
    assert c.count == 20 and c.nulls == 7 and list(c.distribution) == [1, 1, 1, 1]
    with pytest.raises(ValueError):
        a.js_divergence(_fd([1], name="other"))
    assert _fd([1], nulls=10).relative_fill_ratio(a) == math.inf


def test_summary_monoid():
    s = Summary(1, 3, 4, 2).plus(Summary(0, 2, 2, 1))
    assert (s.min, s.max, s.sum, s.count) == (0, 3, 6, 3)


def _data(n=1000, seed=0, shift=0.0, null_leak=False):
    rng = np.random.default_rng(seed)
    y = (rng.random(n) < 0.5).astype(float)
    good = rng.normal(size=n) + shift
    sparse = [None if rng.random() < 0.9995 else 1.0 for _ in range(n)]
    leak = [None if (yy > 0.5 and null_leak) else float(v) for yy, v in zip(y, rng.normal(size=n))]
    cat = [["a", "b", "c"][i % 3] for i in range(n)]
    return TestFeatureBuilder.of(("label", T.RealNN, list(y)), ("good", T.Real, list(good)),
                                 ("sparse", T.Real, sparse), ("leak", T.Real, leak), ("cat", T.PickList, cat),
                                 response="label")


def test_training_only_rules():
    ds, feats = _data(null_leak=True)
    rff = RawFeatureFilter(InMemoryReader(ds), None, bins=10, min_fill_rate=0.01)
    cleaned, drop, keys, res = rff.generate_filtered_raw(feats)
    names = {f.name for f in drop}
    assert names == {"sparse", "leak"}
    reasons = {r.name: r for r in res.exclusionReasons}
    assert reasons["sparse"].trainingUnfilledState and not reasons["sparse"].trainingNullLabelLeaker
    assert reasons["leak"].trainingNullLabelLeaker
    assert "sparse" not in cleaned and "good" in cleaned
    m = {x.name: x for x in res.rawFeatureFilterMetrics}
    assert m["leak"].trainingNullLabelAbsoluteCorr == pytest.approx(1.0)
    # results serialize
    js = res.to_json()
    back = RawFeatureFilterResults.from_json(js)
    assert len(back.rawFeatureDistributions) == len(res.rawFeatureDistributions)


def test_scoring_distribution_shift_excluded():
    ds, feats = _data(seed=1)
    sds, _ = _data(seed=2, shift=50.0)
    rff = RawFeatureFilter(InMemoryReader(ds), InMemoryReader(sds), bins=20, min_fill_rate=0.0001,
                           max_js_divergence=0.5, min_scoring_rows=10)
    _, drop, _, res = rff.generate_filtered_raw(feats)
    assert "good" in {f.name for f in drop}
    r = {x.name: x for x in res.exclusionReasons}["good"]
    assert r.jsDivergenceMismatch
    # protected from JS checks -> kept
    rff2 = RawFeatureFilter(InMemoryReader(ds), InMemoryReader(sds), bins=20, min_fill_rate=0.0001,
                            max_js_divergence=0.5, min_scoring_rows=10, protected_js_features=["good"])
    _, drop2, _, _ = rff2.generate_filtered_raw(feats)
    assert "good" not in {f.name for f in drop2}


def test_numeric_histogram_bucketing():
    from transmogrifai_amd.ops import rff as R
    v = torch.tensor([0.0, 0.5, 1.0, 2.0, 5.0, 10.0])
    h = R.numeric_hist([v], [None], torch.tensor([0.0]), torch.tensor([10.0]), 12)
    # step = 10 / 10 = 1 -> buckets [0,1),[1,2),...,[10,11) ; 10.0 is in bucket 10, nothing invalid
    assert h[0].tolist() == [2, 1, 1, 0, 0, 1, 0, 0, 0, 0, 1, 0]
    h2 = R.numeric_hist([torch.tensor([3.0, 3.0, 4.0])], [None], torch.tensor([3.0]), torch.tensor([3.0]), 12)
    assert h2[0, :2].tolist() == [2, 1]
    s = R.numeric_summary([torch.tensor([1.0, 2.0, 9.0])], [torch.tensor([True, True, False])],
                          torch.tensor([0.0, 0.0, 1.0]))
    assert s[0].tolist() == [2, 1, 1, 2, 3, 5, 9, 17, 1]


def test_map_keys_partially_dropped():
    rng = np.random.default_rng(3)
    n = 600
    maps = [{"k1": float(rng.normal()), **({"k2": 1.0} if i == 0 else {})} for i in range(n)]
    y = list((rng.random(n) < 0.5).astype(float))
    ds, feats = TestFeatureBuilder.of(("label", T.RealNN, y), ("m", T.RealMap, maps),
                                      ("x", T.Real, list(rng.normal(size=n))), response="label")
    rff = RawFeatureFilter(InMemoryReader(ds), None, bins=10, min_fill_rate=0.01)
    cleaned, drop, keys, res = rff.generate_filtered_raw(feats)
    assert not drop and keys == {"m": {"k2"}}
    assert all("k2" not in (v or {}) for v in cleaned["m"].to_list())


def test_workflow_with_raw_feature_filter_updates_dag(tmp_path):
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.workflow.workflow import OpWorkflow, OpWorkflowModel
    ds, feats = _data(null_leak=True)
    label, preds = feats[0], feats[1:]
    vec = transmogrify(preds)
    wf = OpWorkflow().set_result_features(vec, label).with_raw_feature_filter(InMemoryReader(ds), None, bins=10,
                                                                              min_fill_rate=0.01)
    model = wf.train()
    assert {f.name for f in model.blocklist} == {"sparse", "leak"}
    out = model.score(ds)
    new_vec = model.result_features[0]
    meta = out[new_vec.name].metadata
    parents = {p for c in meta.columns for p in c.parent_feature_name}
    assert parents == {"good", "cat"}
    model.save(str(tmp_path / "m"))
    m2 = OpWorkflowModel.load(str(tmp_path / "m"))
    assert {f.name for f in m2.blocklist} == {"sparse", "leak"}
    assert m2.raw_feature_filter_results.exclusionReasons


@pytest.mark.gpu
def test_rff_kernels_match_host():
    from transmogrifai_amd.ops import rff as R
    g = torch.Generator().manual_seed(0)
    n = 200_003
    vals = [torch.randn(n, generator=g), torch.randn(n, generator=g, dtype=torch.float64) * 5,
            torch.randint(0, 50, (n,), generator=g), torch.rand(n, generator=g) < 0.3]
    oks = [torch.rand(n, generator=g) > 0.1, None, torch.rand(n, generator=g) > 0.5, None]
    lab = (torch.rand(n, generator=g) < 0.4).to(torch.float32)
    ref = R.numeric_summary(vals, oks, lab)
    got = R.numeric_summary([v.cuda() for v in vals], [None if o is None else o.cuda() for o in oks], lab.cuda())
    torch.testing.assert_close(got.cpu(), ref, rtol=1e-9, atol=1e-6)
    lo, hi = ref[:, 2], ref[:, 3]
    h_ref = R.numeric_hist(vals, oks, lo, hi, 100)
    h_got = R.numeric_hist([v.cuda() for v in vals], [None if o is None else o.cuda() for o in oks], lo, hi, 100)
    torch.testing.assert_close(h_got.cpu(), h_ref)
    from transmogrifai_amd.ops import _native
    assert _native.hip_loaded()

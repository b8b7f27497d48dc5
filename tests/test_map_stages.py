"""Map vectorizers (``OPMapVectorizerTest``, ``TextMapPivotVectorizerTest``, ``DateMapToUnitCircleVectorizerTest``,
``TextMapLenEstimatorTest``, ``TextMapNullEstimatorTest``, ``DecisionTreeNumericMapBucketizerTest``)."""
import numpy as np
import pytest

from transmogrifai_amd.features import types as T
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.testkit.spec import check_estimator
from transmogrifai_amd.stages.feature import maps as MP
from transmogrifai_amd.stages.feature.bucketizers import DecisionTreeNumericMapBucketizer


def test_real_map_vectorizer_mean_fill():
    ds, (m,) = TestFeatureBuilder.of(("m", T.RealMap, [{"a": 1.0, "b": 2.0}, {"a": 3.0}, {}]))
    st = MP.RealMapVectorizer(track_nulls=True, fill_with_mean=True).set_input(m)
    model, out = check_estimator(st, ds, check_rows=False)
    assert out[0] == [1.0, 0.0, 2.0, 0.0] and out[1] == [3.0, 0.0, 2.0, 1.0] and out[2] == [2.0, 1.0, 2.0, 1.0]


def test_text_map_pivot():
    ds, (m,) = TestFeatureBuilder.of(("m", T.PickListMap, [{"c": "x"}, {"c": "y"}, {"c": "x"}, {}]))
    model, out = check_estimator(MP.TextMapPivotVectorizer(min_support=1, clean_text=False).set_input(m), ds,
                                 check_rows=False)
    names = [c.indicator_value for c in model.metadata["vector_metadata"].columns]
    assert names == ["x", "y", "OTHER", "NullIndicatorValue"] and out[3] == [0, 0, 0, 1]


def test_date_map_unit_circle():
    hour = 3_600_000
    ds, (m,) = TestFeatureBuilder.of(("m", T.DateMap, [{"k": 0}, {"k": 6 * hour}, {}]))
    model, out = check_estimator(MP.DateMapToUnitCircleVectorizer(time_period="HourOfDay").set_input(m), ds,
                                 check_rows=False)
    assert np.allclose(out[0], [1, 0]) and np.allclose(out[1], [0, 1], atol=1e-12) and out[2] == [0, 0]


def test_text_map_len_and_null():
    ds, (m,) = TestFeatureBuilder.of(("m", T.TextMap, [{"a": "hello world"}, {"b": "x"}, {}]))
    _, lens = check_estimator(MP.TextMapLenEstimator().set_input(m), ds, check_rows=False)
    assert lens[0] == [10.0, 0.0] and lens[1] == [0.0, 1.0]
    _, nulls = check_estimator(MP.TextMapNullEstimator().set_input(m), ds, check_rows=False)
    assert nulls[0] == [0.0, 1.0] and nulls[2] == [1.0, 1.0]


def test_dt_numeric_map_bucketizer():
    rng = np.random.default_rng(0)
    x = rng.uniform(0, 10, 300)
    y = (x > 5).astype(float)
    maps = [{"k": float(v)} if i % 10 else {} for i, v in enumerate(x)]
    ds, (lab, m) = TestFeatureBuilder.of(("y", T.RealNN, list(y)), ("m", T.RealMap, maps), response="y")
    model, out = check_estimator(DecisionTreeNumericMapBucketizer().set_input(lab, m), ds, check_rows=False)
    assert model.splits[0] and 4.0 < model.splits[0][1] < 6.0
    assert out[0][-1] == 1.0 and sum(out[1]) == 1.0


# ------------------------------------------------------------------ COO / device path vs the per-row oracle
def _random_maps(kind, n=400, seed=0):
    rng = np.random.default_rng(seed)
    keys = ["Alpha", "alpha", "beta", "Gamma key", "d"]
    words = ["red", "Blue", "green", "blue", "tea time", "x", "", "Red!"]
    out = []
    for i in range(n):
        if rng.random() < 0.1:
            out.append({} if rng.random() < 0.5 else None)
            continue
        m = {}
        for k in keys:
            if rng.random() < 0.55:
                continue
            if rng.random() < 0.05:
                m[k] = None
            elif kind == "real":
                m[k] = float(np.round(rng.normal() * 10, 3))
            elif kind == "integral":
                m[k] = int(rng.integers(-3, 5))
            elif kind == "binary":
                m[k] = bool(rng.random() < 0.4)
            elif kind == "date":
                m[k] = int(rng.integers(0, 10 ** 12))
            elif kind == "geo":
                m[k] = [float(rng.uniform(-80, 80)), float(rng.uniform(-170, 170)), float(rng.integers(1, 9))]
            elif kind == "set":
                m[k] = set(rng.choice(words, size=int(rng.integers(0, 3)), replace=False).tolist())
            else:
                m[k] = str(rng.choice(words)) + ("" if kind == "pivot" else f" w{int(rng.integers(0, 60))}")
        out.append(m)
    return out


_FT = {"real": T.RealMap, "integral": T.IntegralMap, "binary": T.BinaryMap, "date": T.DateMap, "geo": T.GeolocationMap,
       "set": T.MultiPickListMap, "pivot": T.PickListMap, "smarttext": T.TextMap}


@pytest.mark.parametrize("kind", ["real", "integral", "binary", "date", "geo", "set", "pivot", "smarttext"])
@pytest.mark.parametrize("clean_keys", [False, True])
def test_map_vectorizer_coo_path_equals_per_row_reference(kind, clean_keys):
    """The COO / device map vectorizer equals the round-2 per-row host implementation (tests/map_reference_impl.py)
    on fits and transforms, for every map kind, with and without key cleaning."""
    import map_reference_impl as REF
    vals = _random_maps(kind, seed=3 + len(kind))
    if clean_keys:           # keys that collide after cleaning ("Alpha" / "alpha") resolve differently in the
        vals = [None if m is None else {k: v for k, v in m.items() if k != "alpha"} for m in vals]   # reference
    ds, (m,) = TestFeatureBuilder.of(("m", _FT[kind], vals))
    kw = dict(kind=kind, clean_keys=clean_keys, min_support=2, max_cardinality=8, num_features=16,
              reference_date=2 * 10 ** 12, fill_with_mean=True, fill_with_mode=True)
    new = MP.MapVectorizer(**kw).set_input(m)
    old = REF.MapVectorizer(**kw).set_input(m)
    mn, mo = new.fit(ds), old.fit(ds)
    assert mn.keys == mo.keys
    assert mn.tops == mo.tops and mn.methods == mo.methods
    np.testing.assert_allclose(np.asarray(mn.fills, dtype=float), np.asarray(mo.fills, dtype=float), rtol=1e-12)
    a = mn.transform(ds)[mn.get_output_feature_name()].values.cpu().numpy()
    b = mo.transform(ds)[mo.get_output_feature_name()].values.cpu().numpy()
    assert a.shape == b.shape
    np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-12)
    assert [c.to_json() for c in new.metadata["vector_metadata"].columns] == \
        [c.to_json() for c in old.metadata["vector_metadata"].columns]


@pytest.mark.parametrize("est", ["TextMapLenEstimator", "TextMapNullEstimator", "DateMapToUnitCircleVectorizer"])
def test_text_and_date_map_estimators_equal_reference(est):
    import map_reference_impl as REF
    kind = "date" if est.startswith("Date") else "pivot"
    vals = _random_maps(kind, seed=11)
    ds, (m,) = TestFeatureBuilder.of(("m", _FT[kind], vals))
    mn, mo = getattr(MP, est)().set_input(m).fit(ds), getattr(REF, est)().set_input(m).fit(ds)
    assert mn.keys == mo.keys
    a = mn.transform(ds)[mn.get_output_feature_name()].values.cpu().numpy()
    b = mo.transform(ds)[mo.get_output_feature_name()].values.cpu().numpy()
    np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-12)


def test_real_map_vectorizer_reference_expectations():
    """RealMapVectorizerTest.scala: clean keys, constant fills, null tracking."""
    m1 = [{"a": 1.0, "b": 5.0}, {"c": 11.0}, {}]
    m2 = [{"z": 10.0}, {"y": 3.0, "x": 0.0}, {}]
    ds, (f1, f2) = TestFeatureBuilder.of(("m1", T.RealMap, m1), ("m2", T.RealMap, m2))
    est = MP.RealMapVectorizer(clean_keys=True, track_nulls=False, fill_with_mean=False, fill_value=0.0)
    model = est.set_input(f1, f2).fit(ds)
    assert model.keys == [["A", "B", "C"], ["X", "Y", "Z"]]
    out = model.transform(ds)[model.get_output_feature_name()].values.tolist()
    assert out == [[1.0, 5.0, 0.0, 0.0, 0.0, 10.0], [0.0, 0.0, 11.0, 0.0, 3.0, 0.0], [0.0] * 6]
    est = MP.RealMapVectorizer(clean_keys=True, track_nulls=True, fill_with_mean=False, fill_value=100.0)
    model = est.set_input(f1, f2).fit(ds)
    out = model.transform(ds)[model.get_output_feature_name()].values.tolist()
    assert out == [[1.0, 0.0, 5.0, 0.0, 100.0, 1.0, 100.0, 1.0, 100.0, 1.0, 10.0, 0.0],
                   [100.0, 1.0, 100.0, 1.0, 11.0, 0.0, 0.0, 0.0, 3.0, 0.0, 100.0, 1.0],
                   [100.0, 1.0] * 6]


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["real", "integral", "date", "geo", "set", "pivot", "smarttext"])
def test_map_vectorizer_device_path_equals_host(kind):
    """The same fit / transform with the COO tensors on the GPU (device scatters, HIP one-hot pivot and
    hashing kernels) equals the host run (fp32 output vs fp64)."""
    import torch
    from transmogrifai_amd import config as CFG
    vals = _random_maps(kind, n=3000, seed=5)
    ds, (m,) = TestFeatureBuilder.of(("m", _FT[kind], vals))
    kw = dict(kind=kind, min_support=2, max_cardinality=8, num_features=16, reference_date=2 * 10 ** 12)
    prev = CFG.default_device()
    try:
        CFG.set_default_device("cpu")
        mh = MP.MapVectorizer(**kw).set_input(m).fit(ds)
        host = mh.transform(ds)[mh.get_output_feature_name()].values.numpy()
        CFG.set_default_device("cuda")
        md = MP.MapVectorizer(**kw).set_input(m).fit(ds)
        out = md.transform(ds)[md.get_output_feature_name()].values
        assert out.device.type == "cuda"
    finally:
        CFG.set_default_device(prev)
    assert md.keys == mh.keys and md.tops == mh.tops
    np.testing.assert_allclose(np.asarray(md.fills, float), np.asarray(mh.fills, float), rtol=1e-12)
    np.testing.assert_allclose(out.cpu().double().numpy(), host, rtol=1e-6, atol=1e-5 if kind == "date" else 1e-6)


def test_table_tree_splits_equal_engine_tree():
    """The DT bucketizers grow their 1-D tree from the all-reduced (bin, class) table: same thresholds as the
    histogram engine growing it from the rows (gini / entropy, ties, multi-class, min instances / gain)."""
    import torch
    from transmogrifai_amd.stages.feature.bucketizers import tree_splits, tree_splits_dp
    for seed in range(12):
        g = torch.Generator().manual_seed(seed)
        n = int(torch.randint(50, 20000, (1,), generator=g))
        x = [torch.randn(n, generator=g, dtype=torch.float64) * 3, torch.randint(0, 40, (n,), generator=g).double(),
             torch.randint(0, 4, (n,), generator=g).double()][seed % 3]
        K = 2 + seed % 3
        y = ((x + torch.randn(n, generator=g, dtype=torch.float64) * 2) > 0).double() if K == 2 else \
            torch.randint(0, K, (n,), generator=g).double()
        for imp in ("gini", "entropy"):
            for md, mi, mg in ((5, 1, 0.01), (3, 20, 0.0)):
                assert tree_splits(x, y, md, 32, mi, mg, imp) == tree_splits_dp(x, y, md, 32, mi, mg, imp)


_TMP_TOP = [{"a": "d", "b": "d"}, {"a": "e"}, {"c": "D"}, {"c": "d", "a": "d"}]
_TMP_BOT = [{"x": "W"}, {"z": "w", "y": "v"}, {"x": "w", "y": "V"}, {"z": "v"}]


@pytest.mark.parametrize("kw,width,expected", [
    (dict(top_k=10, min_support=0, track_nulls=False), 14, [[2, 5, 7], [3, 9, 12], [0, 7, 9], [0, 2, 11]]),
    (dict(top_k=10, min_support=0, track_nulls=True), 20,
     [[2, 3, 7, 10, 15, 19], [2, 4, 9, 12, 13, 17], [0, 6, 9, 10, 13, 19], [0, 3, 9, 12, 15, 16]]),
    (dict(top_k=10, min_support=0, track_nulls=False, clean_text=False, clean_keys=False), 17,
     [[3, 6, 8], [4, 12, 15], [0, 9, 11], [1, 3, 14]]),
    (dict(top_k=1, min_support=0, track_nulls=False), 12, [[2, 4, 6], [3, 8, 11], [0, 6, 8], [0, 2, 10]]),
    (dict(top_k=1, min_support=0, track_nulls=True), 18,
     [[2, 3, 6, 9, 14, 17], [2, 4, 8, 11, 12, 16], [0, 5, 8, 9, 12, 17], [0, 3, 8, 11, 14, 15]]),
    (dict(top_k=10, min_support=2, track_nulls=False), 10, [[2, 4, 5], [3, 7, 9], [0, 5, 7], [0, 2, 9]]),
    (dict(top_k=10, min_support=2, track_nulls=True), 16,
     [[2, 3, 6, 8, 13, 15], [2, 4, 7, 10, 11, 14], [0, 5, 7, 8, 11, 15], [0, 3, 7, 10, 13, 14]]),
])
def test_text_map_pivot_reference_expectations(kw, width, expected):
    """TextMapPivotVectorizerTest.scala expected vectors. The reference lists the keys of a map in its Scala
    Map iteration order (top: C, A, B; bot: X, Y, Z -- an artefact of Spark's reduce), ours in sorted key
    order; the columns are compared after placing ours in the reference key order (values within a key
    keep their count-then-value order on both sides)."""
    ds, (t, b) = TestFeatureBuilder.of(("top", T.TextMap, _TMP_TOP), ("bot", T.TextMap, _TMP_BOT))
    p = dict(clean_keys=True)
    p.update(kw)
    m = MP.TextMapPivotVectorizer(**p).set_input(t, b).fit(ds)
    out = m.transform(ds)[m.get_output_feature_name()].values.numpy()
    assert out.shape[1] == width
    cols = m.metadata["vector_metadata"].columns
    rank = {"top": "cab", "bot": "xyz"}
    order = sorted(range(len(cols)), key=lambda i: (cols[i].parent_feature_name[0] != "top",
                                                    rank[cols[i].parent_feature_name[0]].index(cols[i].grouping.lower()),
                                                    i))
    got = [[order.index(j) for j in np.flatnonzero(r)] for r in out]
    assert [sorted(g) for g in got] == expected

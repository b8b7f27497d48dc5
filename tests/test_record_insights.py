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


# ---------------------------------------------------------------- RecordInsightsLOCOTest.scala scenarios (:99-292)
def _indexed_meta(name, size):
    """``addMetaData`` (RecordInsightsLOCOTest.scala:349): column i has parent name / type / grouping /
    indicator all ``str(i)``, so its column name is ``i_i_i_i``."""
    from transmogrifai_amd.data.vector_metadata import FeatureHistory, OpVectorColumnMetadata, OpVectorMetadata
    cols = [OpVectorColumnMetadata((str(i),), (str(i),), str(i), str(i), index=i) for i in range(size)]
    hist = {str(i): FeatureHistory((f"a_{i}",), (f"b_{i}",)) for i in range(size)}
    return OpVectorMetadata(name, cols, hist)


def _vector_ds(vectors, labels):
    from transmogrifai_amd.data.columns import VectorColumn
    ds, (f, l) = TestFeatureBuilder.of(("features", T.OPVector, vectors), ("labels", T.RealNN, labels),
                                       response="labels")
    X = ds["features"].values
    ds = ds.with_column("features", VectorColumn(X, _indexed_meta("features", X.shape[1])))
    return ds, f, l


def _random_sparse(n, d=40):
    from transmogrifai_amd.testkit.random_data import RandomReal, RandomVector
    return list(RandomVector.sparse(RandomReal.normal(), d).limit(n))


def _insights(loco, ds):
    return [parse_insights(m) for m in loco.transform(ds)[loco.get_output().name].to_list()]


def test_loco_random_features_binary_logistic_regression():
    """:99 -- 40 dense-filled columns, binary LR: 20 insights per record, each with a non-zero change for
    both score columns."""
    from transmogrifai_amd.models.linear import OpLogisticRegression
    from transmogrifai_amd.testkit.random_data import RandomIntegral
    labels = [float(v) for v in RandomIntegral.integrals(0, 2).take(1000)]
    ds, f, l = _vector_ds(_random_sparse(1000), labels)
    model = OpLogisticRegression().set_input(l, f).fit(ds)
    parsed = _insights(RecordInsightsLOCO(model).set_input(f), ds)
    assert len(parsed) == 1000
    for p in parsed:
        assert len(p) == 20
        assert sum(1 for v in p.values() if any(i == 1 for i, _ in v)) == 20
        assert all(abs(x) > 0 for v in p.values() for _, x in v)


def test_loco_random_features_multiclass_random_forest():
    """:117 -- five classes, top K 2: every record gets 2 insights, each carrying the change of all five
    class scores and no sixth."""
    from transmogrifai_amd.models.trees import OpRandomForestClassifier
    from transmogrifai_amd.testkit.random_data import RandomIntegral
    labels = [float(v) for v in RandomIntegral.integrals(0, 5).take(1000)]
    ds, f, l = _vector_ds(_random_sparse(1000), labels)
    model = OpRandomForestClassifier().set_input(l, f).fit(ds)
    parsed = _insights(RecordInsightsLOCO(model, top_k=2).set_input(f), ds)
    for p in parsed:
        assert len(p) == 2
        for c in range(5):
            assert sum(1 for v in p.values() if any(i == c for i, _ in v)) == 2
        assert not any(i == 5 for v in p.values() for i, _ in v)


def test_loco_random_features_linear_regression():
    """:138 -- a regression model has one score column: 20 insights, all on score index 0, all non-zero."""
    from transmogrifai_amd.models.linear import OpLinearRegression
    from transmogrifai_amd.testkit.random_data import RandomReal
    labels = [float(v) for v in RandomReal.normal().take(1000)]
    ds, f, l = _vector_ds(_random_sparse(1000), labels)
    model = OpLinearRegression().set_input(l, f).fit(ds)
    parsed = _insights(RecordInsightsLOCO(model).set_input(f), ds)
    for p in parsed:
        assert len(p) == 20
        assert all(i == 0 and abs(x) > 0 for v in p.values() for i, x in v)


# name, age, height, height_null, isBlueEyed, gender, testFeatNegCor (RecordInsightsLOCOTest.scala:63-89)
_SANITY_ROWS = [
    ("a", 32, 5.0, 0, 0.9, 0.5, 0), ("b", 32, 4.0, 1, 0.1, 0, 0.1), ("a", 32, 6.0, 0, 0.8, 0.5, 0),
    ("a", 32, 5.5, 0, 0.85, 0.5, 0), ("b", 32, 5.4, 1, 0.05, 0, 0.1), ("b", 32, 5.4, 1, 0.2, 0, 0.1),
    ("a", 32, 5.0, 0, 0.99, 0.5, 0), ("b", 32, 4.0, 0, 0.0, 0, 0.1), ("a", 32, 6.0, 1, 0.7, 0.5, 0),
    ("a", 32, 5.5, 0, 0.8, 0.5, 0), ("b", 32, 5.4, 1, 0.1, 0, 0.1), ("b", 32, 5.4, 1, 0.05, 0, 0.1),
    ("a", 32, 5.0, 0, 1, 0.5, 0), ("b", 32, 4.0, 1, 0.1, 0, 0.1), ("a", 32, 6.0, 1, 0.9, 0.5, 0),
    ("a", 32, 5.5, 0, 1, 0.5, 0), ("b", 32, 5.4, 1, 0.2, 0, 0.1), ("b", 32, 5.4, 1, 0.3, 0, 0.1),
    ("a", 32, 5.0, 0, 0.6, 0.5, 0), ("b", 32, 4.0, 1, 0.1, 0, 0.1), ("a", 32, 6.0, 0, 0.9, 0.5, 0),
    ("a", 32, 5.5, 0, 1, 0.5, 0), ("b", 32, 5.4, 1, 0.05, 0, 0.1), ("b", 32, 5.4, 1, 0.3, 0, 0.1),
    ("b", 32, 5.4, 1, 0.05, 0, 0.1), ("b", 32, 5.4, 1, 0.4, 0, 0.1)]


def _sanity_lr():
    from transmogrifai_amd.models.linear import OpLogisticRegression
    vecs = [[float(r[1]), float(r[2]), float(r[4]), float(r[5]), float(r[6])] for r in _SANITY_ROWS]
    ds, f, l = _vector_ds(vecs, [float(r[3]) for r in _SANITY_ROWS])
    return ds, f, OpLogisticRegression().set_input(l, f).fit(ds)


def test_loco_most_predictive_feature():
    """:156 -- top K 1: the top column is gender (3_3_3_3) or height (1_1_1_1), and for a binary model the
    two class changes are equal and opposite."""
    ds, f, model = _sanity_lr()
    for p in _insights(RecordInsightsLOCO(model, top_k=1).set_input(f), ds):
        (name, v), = p.items()
        assert name in ("3_3_3_3", "1_1_1_1"), p
        assert abs(v[0][1] + v[1][1]) < 1e-5


def test_loco_most_predictive_features_positive_negative():
    """:176 -- top K positives + top K negatives: height leads or gender closes every record's map."""
    ds, f, model = _sanity_lr()
    loco = RecordInsightsLOCO(model, top_k_strategy="positive and negative").set_input(f)
    for p in _insights(loco, ds):
        names = list(p)
        assert names[0] == "1_1_1_1" or names[-1] == "3_3_3_3", names


@pytest.fixture(scope="module")
def strongly_related():
    """:193-226 -- the label is 1 exactly when the picklist is A, B or C; country (30 % empty), picklist (10 %
    empty) and a log-normal currency (30 % empty) transmogrified, a random forest on top, LOCO top K 10."""
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.models.trees import OpRandomForestClassifier
    from transmogrifai_amd.testkit.random_data import RandomReal, RandomText
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    n = 1000
    country = RandomText.countries().with_probability_of_empty(0.3).take(n)
    pick = RandomText.pick_lists(["A", "B", "C", "D", "E", "F", "G"]).with_probability_of_empty(0.1).take(n)
    cur = RandomReal.log_normal(10.0, 1.0, T.Currency).with_probability_of_empty(0.3).take(n)
    label = [1.0 if p in ("A", "B", "C") else 0.0 for p in pick]
    ds, (fc, fp, fu, fl) = TestFeatureBuilder.of(("country", T.Country, country), ("picklist", T.PickList, pick),
                                                 ("currency", T.Currency, cur), ("label", T.RealNN, label),
                                                 response="label")
    vec = transmogrify([fc, fp, fu])
    full = OpWorkflow().set_result_features(vec, fl).set_input_dataset(ds).train().score(
        keep_intermediate_features=True)
    model = OpRandomForestClassifier().set_input(fl, vec).fit(full)
    parsed = _insights(RecordInsightsLOCO(model, top_k=10).set_input(vec), full)
    meta = full[vec.name].metadata
    return n, parsed, meta, model


def _importance_split(parsed, meta):
    d = meta.size
    tot, cnt = np.zeros(d), np.zeros(d)
    idx_of = {c.make_col_name(): c.index for c in meta.columns}
    for m in parsed:
        for k, v in m.items():
            tot[idx_of[k]] += v[-1][1]
            cnt[idx_of[k]] += 1
    mean = np.where(cnt > 0, tot / np.maximum(cnt, 1), np.nan)
    nan = set(np.flatnonzero(np.isnan(mean)).tolist())
    abc = {c.index for c in meta.columns if c.indicator_value in ("A", "B", "C")} - nan
    other = set(range(d)) - abc - nan
    abc_avg = abs(sum(mean[i] for i in abc)) / len(abc)
    other_avg = abs(sum(mean[i] for i in other)) / len(other)
    var, vc = np.zeros(d), np.zeros(d)
    for m in parsed:
        for k, v in m.items():
            i = idx_of[k]
            var[i] += (v[-1][1] - (abc_avg if i in abc else other_avg)) ** 2
            vc[i] += 1
    var = np.where(vc > 1, var / np.maximum(vc, 1), np.nan)
    abc_var = abs(sum(var[i] for i in abc)) / len(abc)
    other_var = abs(sum(var[i] for i in other)) / len(other)
    return abc, other, abc_avg, other_avg, abc_var, other_var


def test_loco_strongly_related_one_insight_per_record(strongly_related):
    n, parsed, meta, _ = strongly_related
    assert len(parsed) == n
    # country and picklist contribute one non-zero column each; currency its value or its null indicator
    assert all(1 <= len(p) <= 4 for p in parsed)


def test_loco_strongly_related_abc_dominate(strongly_related):
    n, parsed, meta, _ = strongly_related
    _, _, abc_avg, other_avg, abc_var, other_var = _importance_split(parsed, meta)
    assert abc_avg > 3 * other_avg
    t = abs(abc_avg - other_avg) / math.sqrt((abc_var + other_var) / n)
    assert t > 10.0


def test_loco_strongly_related_agrees_with_forest_importances(strongly_related):
    """:283 -- the A/B/C-to-other ratio of mean LOCO strengths and of the forest's feature importances differ
    by less than 0.8 of their mean."""
    n, parsed, meta, model = strongly_related
    abc, other, abc_avg, other_avg, _, _ = _importance_split(parsed, meta)
    imp = np.asarray(model.learner.feature_contributions(model.state, meta.size), np.float64).reshape(-1)
    abc_rf = sum(imp[i] for i in abc) / len(abc)
    other_rf = sum(imp[i] for i in other) / len(other)
    r_ins, r_rf = abs(abc_avg / other_avg), abs(abc_rf / other_rf)
    assert abs(r_ins - r_rf) * 2 / (r_ins + r_rf) < 0.8


@pytest.mark.parametrize("agg", ["Avg", "LeaveOutVector"])
def test_loco_aggregates_text_and_date_groups_like_manual_loco(agg):
    """:296-346 + ``assertAggregatedWithPredicate`` (:458) -- for a binary LR over plain, hashed-text and
    date-circle columns: every map's class changes sum to 0, and each text / date group's insight equals the
    manual computation (Avg: the mean of the single-column LOCOs of the group; LeaveOutVector: the record
    re-scored with the whole group zeroed), for every record whose group insight is reported."""
    from transmogrifai_amd.models.linear import OpLogisticRegression
    scored, vec, lr = _fit_mixed(OpLogisticRegression, n=300, seed=7)
    loco = RecordInsightsLOCO(lr, top_k=40, vector_aggregation_strategy=agg).set_input(vec)
    out = [{k: json.loads(v) for k, v in m.items()} for m in loco.transform(scored)[loco.get_output().name].to_list()]
    X = scored[vec.name].values.to(torch.float64)
    hist = scored[vec.name].metadata.column_history()
    for m in out:
        for v in m.values():
            assert abs(sum(x for _, x in v)) < 1e-10
    w = torch.as_tensor(np.asarray(lr.state["coefficients"]), dtype=torch.float64)
    b = float(lr.state["intercept"])
    score = lambda Z: torch.sigmoid(Z @ w + b)
    groups = {}
    for h in hist:
        types = {t.rsplit(".", 1)[-1] for t in h["parentFeatureType"]}
        if "Text" in types and h["indicatorValue"] is None and h["descriptorValue"] is None:
            groups.setdefault(("text", h["parentFeatureOrigins"][0]), []).append(h["index"])
        elif "DateTime" in types and h["descriptorValue"] is not None:
            groups.setdefault(("date", h["descriptorValue"].split("_")[-1]), []).append(h["index"])
    assert any(k[0] == "text" for k in groups) and any(k[0] == "date" for k in groups)
    base = score(X)
    checked = 0
    for (_, _), idx in groups.items():
        ix = torch.as_tensor(idx)
        if agg == "Avg":
            locos = []
            for j in idx:
                Z = X.clone()
                Z[:, j] = 0
                locos.append(base - score(Z))
            exp1 = torch.stack(locos).sum(0) / len(idx)
        else:
            Z = X.clone()
            Z[:, ix] = 0
            exp1 = base - score(Z)
        for i, m in enumerate(out):
            hit = [v for k, v in m.items() if json.loads(k)["index"] in idx]
            if hit:
                assert abs(hit[0][1][1] - float(exp1[i])) < 1e-10
                checked += 1
    assert checked > 0

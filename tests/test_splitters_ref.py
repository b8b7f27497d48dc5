"""DataBalancerTest / DataCutterTest / DataSplitterTest (``core/src/test/.../stages/impl/tuning/``) on row-id
splitters: proportions, summaries, preconditions, label cutting and down-sampling."""
import numpy as np
import pytest
import torch

from transmogrifai_amd.testkit.random_data import RandomIntegral
from transmogrifai_amd.tuning.splitters import DataBalancer, DataCutter, DataSplitter


@pytest.mark.parametrize("args,expected", [
    ((100, 9900, 0.5, 100000), (50.0 / 99.0, 50.0)),
    ((100, 900, 0.1, 900), (0.9, 0.9)),
    ((100, 400, 0.5, 900), (0.75, 3.0)),
    ((100, 400000, 0.5, 12000), (1.0 / 80.0, 50.0)),
    ((100, 12000, 0.5, 30000), (5.0 / 6.0, 100.0)),
    ((200, 300, 0.5, 1000), (2.0 / 3.0, 1.0)),
])
def test_balancer_proportions(args, expected):
    assert DataBalancer.get_proportions(*args) == pytest.approx(expected, rel=1e-12)


def _balancer_data():
    y = torch.cat([torch.ones(800), torch.zeros(200)]).double()        # 800 positives, 200 negatives
    return torch.arange(1000), y


def test_balancer_rebalances_to_the_fraction():
    rid, y = _balancer_data()
    b = DataBalancer(seed=11, sample_fraction=0.4, max_training_sample=100)
    b.pre_validation_prepare(y)
    w = b.weights(rid, y)
    neg, pos = float(w[y == 0].sum()), float(w[y == 1].sum())
    assert abs(neg / (neg + pos) - 0.4) < 0.05


def test_balancer_summary_and_remembered_fractions():
    rid, y = _balancer_data()
    b = DataBalancer(seed=11, sample_fraction=0.4, max_training_sample=2000)
    s = b.pre_validation_prepare(y)
    down, up = DataBalancer.get_proportions(200, 800, 0.4, 2000)
    assert (b.up_fraction, b.down_sample_fraction, b.positive_is_small) == (up, down, False)
    assert (s["positiveLabels"], s["negativeLabels"], s["desiredFraction"], s["upSamplingFraction"],
            s["downSamplingFraction"]) == (800, 200, 0.4, 2.0, 0.75)
    first = b.weights(rid, y)
    assert b.pre_validation_prepare(y) == s and torch.equal(b.weights(rid, y), first)


def test_balancer_already_balanced():
    rid, y = _balancer_data()
    b = DataBalancer(seed=11, sample_fraction=0.01, max_training_sample=20000)
    s = b.pre_validation_prepare(y)
    assert b.already_balanced and b.down_sample_fraction == 1.0
    assert (s["upSamplingFraction"], s["downSamplingFraction"]) == (0.0, 1.0)
    b = DataBalancer(seed=11, sample_fraction=0.01, max_training_sample=100)     # balanced but too big
    s = b.pre_validation_prepare(y)
    assert b.down_sample_fraction == 100 / 1000 and s["downSamplingFraction"] == 0.1
    kept = int(b.validation_prepare(rid, y).sum())
    assert abs(kept - 100) < 40


@pytest.mark.parametrize("make", [lambda: DataBalancer(seed=11, sample_fraction=0.1, max_training_sample=2000),
                                  lambda: DataCutter(seed=42, min_label_fraction=0.4),
                                  lambda: DataSplitter(seed=1)])
def test_prepare_before_examine_is_an_error(make):
    rid, y = _balancer_data()
    with pytest.raises(RuntimeError, match="requirement failed: Cannot call validationPrepare until "
                                           "preValidationPrepare has been called"):
        make().validation_prepare(rid, y)


def _cutter_labels():
    rand = torch.tensor([float(v) for v in RandomIntegral.integrals(0, 1000).take(100000)], dtype=torch.float64)
    g1 = RandomIntegral.integrals(0, 3).reset(7)
    g2 = RandomIntegral.integrals(3, 1000).reset(8)
    biased = torch.tensor([float(v) for v in g1.take(80000)] + [float(v) for v in g2.take(20000)],
                          dtype=torch.float64)
    return rand, biased


def test_cutter_permissive_keeps_everything():
    rand, biased = _cutter_labels()
    rid = torch.arange(rand.shape[0])
    for y in (rand, biased):
        c = DataCutter(seed=42, min_label_fraction=0.0, max_label_categories=100000)
        s = c.pre_validation_prepare(y)
        assert int(c.validation_prepare(rid, y).sum()) == y.shape[0]
        n_labels = len(torch.unique(y))
        assert len(s["labelsKept"]) == n_labels and s["labelsDropped"] == [] and s["labelsDroppedTotal"] == 0
        assert s["preSplitterDataCount"] == 100000 and s["downSamplingFraction"] == 1.0


def test_cutter_top_n_labels():
    rand, biased = _cutter_labels()
    rid = torch.arange(rand.shape[0])
    c = DataCutter(seed=42, min_label_fraction=0.0, max_label_categories=100, reserve_test_fraction=0.5)
    s = c.pre_validation_prepare(rand)
    assert len(torch.unique(rand[c.validation_prepare(rid, rand)])) == 100
    assert len(s["labelsKept"]) == 100 and len(s["labelsDropped"]) == 10
    assert s["labelsDroppedTotal"] == len(torch.unique(rand)) - 100
    # kept labels by count (descending), then label
    cnt = {v: int((rand == v).sum()) for v in s["labelsKept"]}
    keys = [(-cnt[v], v) for v in s["labelsKept"]]
    assert keys == sorted(keys)
    c = DataCutter(seed=42, max_label_categories=3)
    s = c.pre_validation_prepare(biased)
    assert set(torch.unique(biased[c.validation_prepare(rid, biased)]).tolist()) == {0.0, 1.0, 2.0}
    assert len(s["labelsKept"]) == 3 and len(s["labelsDropped"]) == 10 and s["labelsDroppedTotal"] == 997


def test_cutter_min_label_fraction():
    rand, biased = _cutter_labels()
    rid = torch.arange(rand.shape[0])
    c = DataCutter(seed=42, min_label_fraction=0.0012, max_label_categories=100000, reserve_test_fraction=0.5)
    s = c.pre_validation_prepare(rand)
    distinct = len(torch.unique(rand))
    kept = len(torch.unique(rand[c.validation_prepare(rid, rand)]))
    assert 0 < kept < distinct and len(s["labelsKept"]) + s["labelsDroppedTotal"] == distinct
    c = DataCutter(seed=42, min_label_fraction=0.2, reserve_test_fraction=0.5)
    s = c.pre_validation_prepare(biased)
    assert len(torch.unique(biased[c.validation_prepare(rid, biased)])) == 3
    assert (len(s["labelsKept"]), s["labelsDroppedTotal"], len(s["labelsDropped"])) == (3, 997, 10)


def test_cutter_all_filtered_is_an_error():
    rand, _ = _cutter_labels()
    with pytest.raises(RuntimeError, match="DataCutter dropped all labels"):
        DataCutter(seed=42, min_label_fraction=0.4).pre_validation_prepare(rand)


@pytest.mark.parametrize("cls", [DataCutter, DataSplitter])
def test_down_sample_above_training_limit(cls):
    n = 2_000_000
    y = torch.ones(n, dtype=torch.float64)
    rid = torch.arange(n)
    sp = cls(seed=42)
    sp.pre_validation_prepare(y)
    assert sp.down_sample_fraction == 0.5
    assert abs(int(sp.validation_prepare(rid, y).sum()) - 1_000_000) < 100_000


@pytest.mark.parametrize("frac,exp_test", [(0.0, 0), (0.2, 200), (0.6, 600)])
def test_splitter_reserve_fractions(frac, exp_test):
    s = DataSplitter(seed=1234, reserve_test_fraction=frac)
    tr, te = s.split(torch.arange(1000))
    assert abs(int(te.sum()) - exp_test) < 30 and abs(int(tr.sum()) - (1000 - exp_test)) < 30


def test_splitter_keeps_data_and_summary():
    y = torch.ones(1000, dtype=torch.float64)
    s = DataSplitter(seed=1234)
    summ = s.pre_validation_prepare(y)
    assert bool(s.validation_prepare(torch.arange(1000), y).all())
    assert (summ["preSplitterDataCount"], summ["downSamplingFraction"]) == (1000, 1.0)


def test_splitter_params():
    s = DataSplitter(seed=1234, reserve_test_fraction=0.0, max_training_sample=500)
    s.down_sample_fraction = 0.5
    assert s.params() == {"seed": 1234, "reserveTestFraction": 0.0, "maxTrainingSample": 500}
    c = DataCutter(seed=42, reserve_test_fraction=0.0, max_label_categories=100000, min_label_fraction=0.0,
                   max_training_sample=50000)
    assert c.params()["maxLabelCategories"] == 100000 and c.params()["minLabelFraction"] == 0.0

"""SanityChecker on generated "bad feature" data: ports of ``BadFeatureZooTest.scala`` scenarios (:60-400) -- label
leakage through PickList categories (Cramér's V, binary and multiclass labels), empty features, a label flagged as
not categorical, numeric map indicator groups ignored, and leakage through null indicators. The data come from this
package's testkit generators (the reference's distributions and empty-probabilities, seeded); the assertions are the
reference's structural ones (which columns are dropped, how many)."""
import numpy as np
import pytest

from transmogrifai_amd import uid
from transmogrifai_amd.dsl import transmogrify
from transmogrifai_amd.features import types as T
from transmogrifai_amd.stages.preparators.sanity_checker import SanityChecker
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.testkit.random_data import RandomIntegral, RandomMap, RandomReal, RandomSet, RandomText

N = 1000
PICKS = ["A", "B", "C", "D", "E", "F", "G", "H", "I"]


def _take(gen, p_empty, seed):
    g = gen.reset(seed)
    if p_empty:
        g.with_probability_of_empty(p_empty)
    return g.take(N)


def _summary(label_vals, cols, **sc):
    """Fit a SanityChecker (check sample 1, remove bad features) on transmogrify(cols) against the label."""
    uid.reset(0)
    ds, feats = TestFeatureBuilder.of(("label", T.RealNN, label_vals), *cols, response="label")
    label, preds = feats[0], feats[1:]
    vec = transmogrify(preds)
    from transmogrifai_amd.stages.base import OpEstimator  # noqa: F401
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    chk = SanityChecker(check_sample=1.0, remove_bad_features=True, **sc).set_input(label, vec).get_output()
    model = OpWorkflow().set_result_features(chk).set_input_dataset(ds).train()
    return model.get_origin_stage_of(chk).metadata["summary"]


def _abc(p):
    return 1.0 if p in ("A", "B", "C") else 0.0


def _base_cols(p_city=0.2, p_country=0.2, p_pick=0.2, p_cur=0.2):
    city = _take(RandomText.cities(), p_city, 1)
    country = _take(RandomText.countries(), p_country, 2)
    pick = _take(RandomText.pick_lists(PICKS), p_pick, 3)
    cur = _take(RandomReal.log_normal(10.0, 1.0, ftype=T.Currency), p_cur, 4)
    return city, country, pick, cur


def test_picklist_leakage_binary_label():
    """``:60-106``: a label read off the pick list -- all 11 pick-list columns (9 choices, other, null) go, nothing
    else; every column but the label and one more has categorical statistics."""
    city, country, pick, cur = _base_cols()
    summ = _summary([_abc(p) for p in pick], [("city", T.City, city), ("country", T.Country, country),
                                              ("picklist", T.PickList, pick), ("currency", T.Currency, cur)],
                    max_feature_correlation=1.1)
    assert summ["dropped"] and all(d.startswith("picklist") for d in summ["dropped"])
    assert len(summ["dropped"]) == 11


def test_empty_features_do_not_fail():
    """``:173-213``: all-empty city / country columns; the summary round-trips through JSON; 15 columns dropped."""
    import json
    city, country, pick, cur = _base_cols(1.0, 1.0, 0.5, 0.5)
    summ = _summary([1.0 if p is not None else 0.0 for p in pick],
                    [("city", T.City, city), ("country", T.Country, country), ("picklist", T.PickList, pick),
                     ("currency", T.Currency, cur)])
    assert json.loads(json.dumps(summ, default=str)) is not None
    assert len(summ["dropped"]) == 15


def test_picklist_leakage_multiclass_label():
    """``:216-262``."""
    city, country, pick, cur = _base_cols()
    lab = {"A": 1.0, "B": 1.0, "C": 2.0, "D": 2.0, "E": 3.0}
    summ = _summary([lab.get(p, 0.0) for p in pick], [("city", T.City, city), ("country", T.Country, country),
                                                      ("picklist", T.PickList, pick), ("currency", T.Currency, cur)],
                    max_feature_correlation=1.1)
    assert all(d.startswith("picklist") for d in summ["dropped"])
    assert len(summ["dropped"]) == 11


def test_no_cramers_v_for_a_non_categorical_label():
    """``:264-306``: with categoricalLabel false only the correlation rule applies -- one column goes."""
    city, country, pick, cur = _base_cols()
    summ = _summary([_abc(p) for p in pick], [("city", T.City, city), ("country", T.Country, country),
                                              ("picklist", T.PickList, pick), ("currency", T.Currency, cur)],
                    max_feature_correlation=1.1, categorical_label=False)
    assert len(summ["dropped"]) == 1


def test_numeric_map_indicator_groups_are_ignored():
    """``:308-352``: the integral map's null-indicator groups are not categorical groups of the Cramér's V rule."""
    city = _take(RandomText.cities(), 0.2, 1)
    from transmogrifai_amd.testkit.random_data import _COUNTRIES
    mpl = _take(RandomSet.of(_COUNTRIES, 0, 5), 0.0, 2)       # RandomMultiPickList.of(RandomText.countries, maxLen 5)
    pick = _take(RandomText.pick_lists(PICKS), 0.2, 3)
    imap = _take(RandomMap.of(RandomIntegral.integrals(-100, 100), 0, 4, ftype=T.IntegralMap), 0.0, 4)
    summ = _summary([_abc(p) for p in pick], [("city", T.City, city), ("multipicklist", T.MultiPickList, mpl),
                                              ("picklist", T.PickList, pick), ("integralMap", T.IntegralMap, imap)],
                    max_feature_correlation=1.1)
    assert all(d.startswith("picklist") for d in summ["dropped"])
    assert len(summ["dropped"]) == 11


def test_null_indicator_leakage_drops_the_parent_features():
    """``:354-399``: the label is "real is present"; the null indicators of real and of the revenue derived from
    it leak the label, and each parent's two columns (value, null indicator) go."""
    city = _take(RandomText.cities(), 0.4, 1)
    real = _take(RandomReal.uniform(0.0, 1.0), 0.5, 2)
    cur = _take(RandomReal.log_normal(10.0, 1.0, ftype=T.Currency), 0.0, 3)
    rev = [None if r is None else r * c for r, c in zip(real, cur)]
    summ = _summary([1.0 if r is not None else 0.0 for r in real],
                    [("city", T.City, city), ("real", T.Real, real), ("currency", T.Currency, cur),
                     ("expectedRevenue", T.Currency, rev)])
    assert sum(d.startswith("expectedRevenue") for d in summ["dropped"]) == 2
    assert sum(d.startswith("real") for d in summ["dropped"]) == 2

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


def _summary_feats(ds, label, preds, **sc):
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    vec = transmogrify(preds)
    chk = SanityChecker(check_sample=1.0, remove_bad_features=True, **sc).set_input(label, vec).get_output()
    model = OpWorkflow().set_result_features(chk).set_input_dataset(ds).train()
    return model.get_origin_stage_of(chk).metadata["summary"]


def test_hashed_text_null_leakage_drops_every_hash_column():
    """``:401-472``: a label that is "text is present" -- all hashed columns of the text (and its null indicator)
    go; the same for one key of a text map."""
    from transmogrifai_amd.stages.feature.transmogrifier import TransmogrifierDefaults as TD
    city = _take(RandomText.cities(), 0.4, 1)
    real = _take(RandomReal.uniform(0.0, 1.0), 0.5, 2)
    text = _take(RandomText.strings(1, 10), 0.4, 3)
    summ = _summary([1.0 if t is not None else 0.0 for t in text],
                    [("city", T.City, city), ("real", T.Real, real), ("text", T.Text, text)])
    assert sum(d.startswith("text") for d in summ["dropped"]) == TD.DefaultNumOfFeatures + 1
    tmap = _take(RandomMap.of(RandomText.strings(1, 10), 0, 3, ftype=T.TextMap), 0.0, 4)
    summ2 = _summary([1.0 if "k1" in (m or {}) else 0.0 for m in tmap],
                     [("city", T.City, city), ("real", T.Real, real), ("textmap", T.TextMap, tmap)])
    assert sum(d.startswith("textmap_k1") for d in summ2["dropped"]) == TD.DefaultNumOfFeatures + 1


def test_pivoted_text_correlation_leakage():
    """``:474-547``: low-cardinality text is pivoted; the label is "text == alpha" -- all 6 pivoted columns go (4
    values, other, null); the same for one key of a text map."""
    city = _take(RandomText.cities(), 0.3, 1)
    real = _take(RandomReal.uniform(0.0, 1.0), 0.3, 2)
    dom = ["alpha", "beta", "gamma", "delta"]
    text = _take(RandomText.text_from_domain(dom), 0.3, 3)
    summ = _summary([1.0 if t == "alpha" else 0.0 for t in text],
                    [("city", T.City, city), ("real", T.Real, real), ("text", T.Text, text)])
    assert sum(d.startswith("text") for d in summ["dropped"]) == 6
    tmap = _take(RandomMap.of(RandomText.text_from_domain(dom), 0, 2, ftype=T.TextMap), 0.0, 4)
    summ2 = _summary([1.0 if (m or {}).get("k0") == "alpha" else 0.0 for m in tmap],
                     [("city", T.City, city), ("real", T.Real, real), ("textmap", T.TextMap, tmap)])
    assert sum(d.startswith("textmap") for d in summ2["dropped"]) == 6


def test_binned_numeric_leakage():
    """``:549-603``: expected revenue = binary x currency; its 3-bin pick list (null / zero / non-zero) leaks the
    label -- its 5 columns (3 bins, other, null) go."""
    from transmogrifai_amd.testkit.random_data import RandomBinary
    uid.reset(0)
    b = _take(RandomBinary(0.5), 0.3, 1)
    cur = _take(RandomReal.log_normal(10.0, 1.0, ftype=T.Currency), 0.0, 2)
    er = [None if x is None else (1.0 if x else 0.0) * c for x, c in zip(b, cur)]
    ds, feats = TestFeatureBuilder.of(("label", T.RealNN, [1.0 if x else 0.0 for x in b]), ("binary", T.Binary, b),
                                      ("currency", T.Currency, cur), ("expectedRevenue", T.Currency, er),
                                      response="label")
    label, rb, rc, rer = feats
    binned = rer.map(lambda v: "null" if v is None else ("nonZero" if v != 0 else "zero"), output_type=T.PickList)
    summ = _summary_feats(ds, label, [rb, rc, rer, binned])
    assert sum(d.startswith("expectedRevenue_1-stagesApplied_PickList") for d in summ["dropped"]) == 5


def test_no_cramers_v_against_a_numeric_label():
    """``:628-661``: regression label -- only the pick list's always-empty "other" column goes."""
    city, country, pick, _ = _base_cols()
    lab = _take(RandomReal.log_normal(10.0, 1.0, ftype=T.RealNN), 0.0, 9)
    summ = _summary(lab, [("city", T.City, city), ("country", T.Country, country), ("picklist", T.PickList, pick)],
                    max_feature_correlation=1.1)
    assert sum(d.startswith("picklist") for d in summ["dropped"]) == 1
    assert len(summ["dropped"]) == 1


def test_multipicklist_modified_cramers_v():
    """``:664-718``: a label set by one multi-pick-list choice -- every multi-pick-list column (topK, other, null)
    has categorical statistics."""
    from transmogrifai_amd.stages.feature.transmogrifier import TransmogrifierDefaults as TD
    rng = np.random.default_rng(5)
    cur = _take(RandomReal.log_normal(10.0, 1.0, ftype=T.Currency), 0.0, 1)
    dom = ["Strawberry Milk", "Chocolate Milk", "Soy Milk", "Almond Milk"]
    plm = _take(RandomMap.of(RandomText.pick_lists(dom), 1, 3, ftype=T.PickListMap), 0.0, 2)
    mpl = _take(RandomSet.of([str(i) for i in range(20)], 0, 2), 0.0, 3)
    lab = [3.0 if "3" in (m or ()) else float(rng.integers(0, 3)) for m in mpl]
    summ = _summary(lab, [("currency", T.Currency, cur), ("multipicklist", T.MultiPickList, mpl),
                          ("picklistMap", T.PickListMap, plm)])
    cats = [c for s in summ["categoricalStats"] for c in s["categoricalFeatures"]]
    assert sum(c.startswith("multipicklist") for c in cats) == TD.TopK + 2


def test_sibling_correlations_combined_by_absolute_value():
    """``:765-805``: label = pick list in {A, B} (random for null); with Cramér's V off (max 1.0) the siblings'
    correlations are combined by absolute value -- the pick list's 5 columns go, nothing else."""
    rng = np.random.default_rng(6)
    pick = _take(RandomText.pick_lists(["A", "B", "C"]), 0.2, 1)
    cur = _take(RandomReal.log_normal(10.0, 1.0, ftype=T.Currency), 0.2, 2)
    lab = [1.0 if p in ("A", "B") else 0.0 if p == "C" else float(rng.integers(0, 2)) for p in pick]
    summ = _summary(lab, [("picklist", T.PickList, pick), ("currency", T.Currency, cur)], max_cramers_v=1.0,
                    max_correlation=0.6)
    assert all(d.startswith("picklist") for d in summ["dropped"])
    assert len(summ["dropped"]) == 5


def test_titanic_body_rule_confidence():
    """``:807-848``: a mostly-empty ID whose presence implies the label (high rule confidence with enough support)
    -- both columns derived from it go."""
    rng = np.random.default_rng(7)
    body = _take(RandomText.ids(), 0.9, 1)
    boat = _take(RandomText.pick_lists(["A", "B", "C"]), 0.8, 2)
    cur = _take(RandomReal.log_normal(10.0, 1.0, ftype=T.Currency), 0.8, 3)
    lab = [1.0 if b is not None else (0.0 if bo is not None else float(rng.integers(0, 2)))
           for b, bo in zip(body, boat)]
    summ = _summary(lab, [("body", T.ID, body), ("boat", T.PickList, boat), ("currency", T.Currency, cur)],
                    max_rule_confidence=0.99, min_required_rule_support=0.05)
    assert sum(d.startswith("body") for d in summ["dropped"]) == 2


@pytest.mark.parametrize("binning", ["bucketize", "auto_bucketize"])
def test_binned_vector_leakage_drops_the_parent(binning):
    """``:605-626`` (``expectedRevenueLeakage``): the revenue binned straight to an OPVector (a numeric bucketizer
    at 0, or a decision-tree bucketizer on the label) leaks the label -- the two raw revenue columns and the bins
    go (4 columns starting with expectedRevenue)."""
    from transmogrifai_amd.testkit.random_data import RandomBinary
    uid.reset(0)
    b = _take(RandomBinary(0.5), 0.3, 1)
    cur = _take(RandomReal.log_normal(10.0, 1.0, ftype=T.Currency), 0.0, 2)
    er = [None if x is None else (1.0 if x else 0.0) * c for x, c in zip(b, cur)]
    ds, feats = TestFeatureBuilder.of(("label", T.RealNN, [1.0 if x else 0.0 for x in b]), ("binary", T.Binary, b),
                                      ("currency", T.Currency, cur), ("expectedRevenue", T.Currency, er),
                                      response="label")
    label, rb, rc, rer = feats
    if binning == "bucketize":
        binned = rer.bucketize(track_nulls=False, splits=[float("-inf"), 0.0, float("inf")], split_inclusion="Right")
    else:
        binned = rer.auto_bucketize(label, track_nulls=False)
    summ = _summary_feats(ds, label, [rb, rc, rer, binned])
    assert sum(d.startswith("expectedRevenue") for d in summ["dropped"]) == 4

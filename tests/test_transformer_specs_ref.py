"""Expected values of the reference's small transformer specs (``core/src/test/.../stages/impl/feature/``), each
run through the ``OpTransformerSpec`` contract (batch = row = key-value = reloaded checkpoint,
``testkit/spec.check_transformer``): AbsoluteValueTransformerTest, AddTransformerTest, SubtractTransformerTest,
MultiplyTransformerTest, DivideTransformerTest, CeilTransformerTest, FloorTransformerTest, RoundTransformerTest,
RoundDigitsTransformerTest, ExpTransformerTest, LogTransformerTest, PowerTransformerTest, SqrtTransformerTest,
ScalarAddTransformerTest, ScalarSubtractTransformerTest, ScalarMultiplyTransformerTest,
ScalarDivideTransformerTest, ValidEmailTransformerTest, SubstringTransformerTest, AliasTransformerTest,
ToOccurTransformerTest, TextLenTransformerTest, TextListNullTransformerTest, JaccardSimilarityTest,
DropIndicesByTransformerTest."""
import math

import numpy as np
import pytest
import torch

from transmogrifai_amd import dsl  # noqa: F401  (registers the feature shortcuts)
from transmogrifai_amd.features import types as T
from transmogrifai_amd.stages.feature import math_stages as MS
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.testkit.spec import check_transformer

_UNARY_SAMPLE = [-1.3, -4.9, None, 5.1, -5.1, 0.1, 2.5, 0.4]
_PAIRS = [(1.0, 2.0), (4.0, 4.0), (None, 5.0), (5.0, None), (2.0, 0.0)]
_SCALAR_SAMPLE = [1.0, 4.0, None, -1.0, 2.0]


def _one(vals, ftype=T.Real):
    return TestFeatureBuilder.of(("f1", ftype, vals))


def _two(pairs, ftype=T.Real):
    return TestFeatureBuilder.of(("f1", ftype, [a for a, _ in pairs]), ("f2", ftype, [b for _, b in pairs]))


def _map(vals, fn):
    return [None if v is None else fn(v) for v in vals]


def test_absolute_value():
    ds, (f1,) = _one([-1.0, -4.0, None, 5.0, -5.5, 0.1, 2.0, 0.0])
    check_transformer(MS.UnaryMathTransformer("abs").set_input(f1), ds,
                      expected=[1.0, 4.0, None, 5.0, 5.5, 0.1, 2.0, 0.0])
    assert isinstance(f1.abs().origin_stage, MS.UnaryMathTransformer)


@pytest.mark.parametrize("op,expected", [
    ("plus", [3.0, 8.0, 5.0, 5.0, 2.0]),            # AddTransformerTest: a missing side counts as absent
    ("minus", [-1.0, 0.0, -5.0, 5.0, 2.0]),         # SubtractTransformerTest: (None, y) -> -y
    ("multiply", [2.0, 16.0, None, None, 0.0]),     # MultiplyTransformerTest
    ("divide", [0.5, 1.0, None, None, None]),       # DivideTransformerTest: x / 0 is not a valid number
])
def test_binary_math_reference_values(op, expected):
    ds, (f1, f2) = _two(_PAIRS)
    check_transformer(MS.BinaryMathTransformer(op).set_input(f1, f2), ds, expected=expected)


@pytest.mark.parametrize("op,expected", [
    ("ceil", [-1, -4, None, 6, -5, 1, 3, 1]),
    ("floor", [-2, -5, None, 5, -6, 0, 2, 0]),
    ("round", [-1, -5, None, 5, -5, 0, 3, 0]),      # math.round: 2.5 -> 3 (not half-to-even)
])
def test_integral_rounding(op, expected):
    ds, (f1,) = _one(_UNARY_SAMPLE)
    st = MS.UnaryMathTransformer(op).set_input(f1)
    assert st.output_type is T.Integral
    out = check_transformer(st, ds, expected=expected)
    assert all(v is None or isinstance(v, int) for v in out)
    assert isinstance(getattr(f1, op)().origin_stage, MS.UnaryMathTransformer)


def test_java_round_halves_and_boundary():
    x = torch.tensor([2.5, -2.5, 0.5, -0.5, 0.49999999999999994, 1e15 + 0.5, -1.5], dtype=torch.float64)
    assert MS.java_round(x).tolist() == [3.0, -2.0, 1.0, 0.0, 0.0, 1e15 + 1, -1.0]


def test_round_digits():
    ds, (f1,) = _one([1.4231092, 4.3231, None, -1.0, 2.03728181])
    check_transformer(MS.UnaryMathTransformer("roundDigits", digits=2).set_input(f1), ds,
                      expected=[1.42, 4.32, None, -1.0, 2.04], tol=0.0)
    assert isinstance(f1.round_digits(4).origin_stage, MS.UnaryMathTransformer)


def test_exp():
    ds, (f1,) = _one(_UNARY_SAMPLE)
    check_transformer(MS.UnaryMathTransformer("exp").set_input(f1), ds, expected=_map(_UNARY_SAMPLE, math.exp))


def test_log_base_10_and_invalid():
    ds, (f1,) = _one(_UNARY_SAMPLE)
    exp = [None if v is None or v <= 0 else math.log10(v) for v in _UNARY_SAMPLE]
    out = check_transformer(MS.UnaryMathTransformer("log", base=10.0).set_input(f1), ds, expected=exp, tol=0.0)
    assert out[3] == math.log10(5.1) / math.log10(10.0)
    assert isinstance(f1.log(2).origin_stage, MS.UnaryMathTransformer)
    with pytest.raises(ValueError, match="log base must be greater than 0"):
        MS.UnaryMathTransformer("log", base=0.0)


def test_power():
    ds, (f1,) = _one(_UNARY_SAMPLE)
    check_transformer(MS.ScalarMathTransformer("power", 3.0).set_input(f1), ds,
                      expected=_map(_UNARY_SAMPLE, lambda v: math.pow(v, 3)))
    assert isinstance(f1.power(4).origin_stage, MS.ScalarMathTransformer)


def test_sqrt():
    ds, (f1,) = _one(_UNARY_SAMPLE)
    exp = [None if v is None or v < 0 else math.sqrt(v) for v in _UNARY_SAMPLE]
    check_transformer(MS.UnaryMathTransformer("sqrt").set_input(f1), ds, expected=exp)


@pytest.mark.parametrize("op,scalar,expected", [
    ("plus", 5.0, [6.0, 9.0, None, 4.0, 7.0]),
    ("minus", 5.0, [-4.0, -1.0, None, -6.0, -3.0]),
    ("multiply", 5.0, [5.0, 20.0, None, -5.0, 10.0]),
    ("divide", 2.0, [0.5, 2.0, None, -0.5, 1.0]),
])
def test_scalar_math_reference_values(op, scalar, expected):
    ds, (f1,) = _one(_SCALAR_SAMPLE)
    check_transformer(MS.ScalarMathTransformer(op, scalar).set_input(f1), ds, expected=expected)


def test_scalar_operators_on_features():
    ds, (f1,) = _one(_SCALAR_SAMPLE)
    for feat, exp in ((f1 + 5.0, [6.0, 9.0, None, 4.0, 7.0]), (f1 * 5.0, [5.0, 20.0, None, -5.0, 10.0]),
                      (f1 - 5.0, [-4.0, -1.0, None, -6.0, -3.0]), (f1 / 2.0, [0.5, 2.0, None, -0.5, 1.0])):
        check_transformer(feat.origin_stage, ds, expected=exp)


def test_valid_email():
    from transmogrifai_amd.stages.feature.text_stages import ValidEmailTransformer
    ds, (f1,) = _one(["abc", "a@b", "a@", "@blah", None, "real@stuff"], T.Email)
    check_transformer(ValidEmailTransformer().set_input(f1), ds, expected=[False, True, False, False, None, True])
    assert isinstance(f1.is_valid_email().origin_stage, ValidEmailTransformer)


def test_substring():
    from transmogrifai_amd.stages.feature.misc_stages import SubstringTransformer
    pairs = [("a", "abc"), ("abc", "a"), ("no", "YesNO"), (None, "blah"), (None, "blah"), (None, None)]
    ds, (f1, f2) = _two(pairs, T.Text)
    check_transformer(SubstringTransformer().set_input(f1, f2), ds, expected=[True, False, True, None, None, None])
    assert isinstance(f1.is_substring(f2).origin_stage, SubstringTransformer)


def test_alias():
    from transmogrifai_amd.stages.feature.misc_stages import AliasTransformer
    ds, (f1, f2) = _two([(1.0, 2.0), (4.0, 4.0)], T.RealNN)
    st = AliasTransformer(name="feature").set_input(f1)
    check_transformer(st, ds, expected=[1.0, 4.0])
    feat = f1.alias("feature")
    assert feat.name == "feature" and isinstance(feat.origin_stage, AliasTransformer)
    derived = (f1 / f2).alias("feature")
    assert derived.name == "feature"
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    out = OpWorkflow().set_result_features(derived).set_input_dataset(ds).train().score()
    assert out["feature"].to_list() == [0.5, 1.0]


def test_to_occur():
    from transmogrifai_amd.stages.feature.misc_stages import ToOccurTransformer
    ds, (f1,) = _one([2.0, 0.0, None])
    check_transformer(ToOccurTransformer().set_input(f1), ds, expected=[1.0, 0.0, 0.0])
    # the extended data of ToOccurTransformerTest.scala:44-101
    ds2, (lead, emails, oppty, dnc, forms) = TestFeatureBuilder.of(
        ("leadId", T.Text, ["001", "002", "003", "004"]), ("numEmails", T.RealNN, [0.0, 1.0, 2.0, 0.0]),
        ("opptyId", T.Text, [None, None, "abc", "def"]), ("doNotContact", T.Binary, [True, None, False, False]),
        ("numFormSubmits", T.Real, [None, 2.0, 0.0, 1.0]))
    cases = [(emails.occurs(lambda v: v is not None and v > 1), [0.0, 0.0, 1.0, 0.0]),
             (forms.occurs(), [0.0, 1.0, 0.0, 1.0]), (dnc.occurs(), [1.0, 0.0, 0.0, 0.0]),
             (emails.to_occur(), [0.0, 1.0, 1.0, 0.0]),
             (oppty.to_occur(lambda v: v is not None and len(v) > 0), [0.0, 0.0, 1.0, 1.0])]
    for feat, exp in cases:
        assert isinstance(feat.origin_stage, ToOccurTransformer)
        assert feat.origin_stage.transform(ds2)[feat.name].to_list() == exp


_GIRAFFE = "A giraffe drinks by the watering hole"


def _text_list_pairs():
    return [([ "A", "giraffe", "drinks", "by", "the", "watering", "hole"], [_GIRAFFE]),
            ([_GIRAFFE], ["Cheese"]), (["Cheese", "cake"], [_GIRAFFE]), (["Cheese"], ["Cheese"]),
            ([], [_GIRAFFE]), ([], ["Cheese", "tart"]), ([_GIRAFFE], []), (["Cheese"], []), ([], [])]


def test_text_len():
    from transmogrifai_amd.stages.feature.text_stages import TextLenTransformer
    ds, (f1, f2) = _two(_text_list_pairs(), T.TextList)
    st = TextLenTransformer().set_input(f1, f2)
    out = check_transformer(st, ds, expected=[[31, 37], [37, 6], [10, 37], [6, 6], [0, 37], [0, 10], [37, 0],
                                              [6, 0], [0, 0]])
    assert st.get_output().type_name.endswith("OPVector") and not st.get_output().is_response
    assert len(out) == 9


def test_text_list_null():
    from transmogrifai_amd.data.vector_metadata import NULL_STRING
    from transmogrifai_amd.stages.feature.text_stages import TextListNullTransformer
    pairs = [([_GIRAFFE], [_GIRAFFE]), ([_GIRAFFE], ["Cheese"]), (["Cheese"], [_GIRAFFE]), (["Cheese"], ["Cheese"]),
             ([], [_GIRAFFE]), ([], ["Cheese"]), ([_GIRAFFE], []), (["Cheese"], []), ([], [])]
    ds, (f1, f2) = _two(pairs, T.TextList)
    st = TextListNullTransformer().set_input(f1, f2)
    check_transformer(st, ds, expected=[[0, 0], [0, 0], [0, 0], [0, 0], [1, 0], [1, 0], [0, 1], [0, 1], [1, 1]])
    meta = st.transform(ds)[st.get_output().name].metadata
    assert [c.indicator_value for c in meta.columns] == [NULL_STRING, NULL_STRING]
    assert [c.parent_feature_name for c in meta.columns] == [(f1.name,), (f2.name,)]


def test_jaccard_similarity():
    from transmogrifai_amd.stages.feature.misc_stages import JaccardSimilarity, jaccard
    pairs = [({"Red", "Green"}, {"Red"}), ({"Red", "Green"}, {"Yellow, Blue"}), ({"Red", "Yellow"}, {"Red", "Yellow"})]
    ds, (f1, f2) = _two(pairs, T.MultiPickList)
    st = JaccardSimilarity().set_input(f1, f2)
    check_transformer(st, ds, expected=[0.5, 0.0, 1.0])
    feat = f1.jaccard_similarity(f2)
    assert isinstance(feat.origin_stage, JaccardSimilarity) and list(feat.parents) == [f1, f2]
    assert jaccard(set(), set()) == 1.0
    assert jaccard({"Red", "Blue", "Green"}, {"Red", "Blue", "Green"}) == 1.0
    assert jaccard({"Red", "Green", "Blue"}, {"Red", "Blue"}) == 2.0 / 3.0
    assert jaccard({"Red"}, {"Blue"}) == 0.0
    assert jaccard({"Red", "Yellow", "Green"}, {"Pink", "Green", "Blue"}) == 1.0 / 5.0


def _picklist_vector():
    from transmogrifai_amd.testkit.random_data import RandomText
    colors = RandomText.pick_lists(["Red", "Blue", "Green"]).take(100)
    ds, (color,) = TestFeatureBuilder.of(("color", T.PickList, colors))
    return ds, color, color.vectorize(top_k=10, min_support=3, clean_text=False)


def test_drop_indices_by_predicate():
    """DropIndicesByTransformerTest.scala:67-90: dropping the "Red" indicator leaves 4 columns (Blue, Green,
    OTHER, null); Red rows are then all zero, every other row has its one-hot 1."""
    from transmogrifai_amd.stages.feature.vector_stages import DropIndicesByTransformer
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    ds, color, vec = _picklist_vector()
    pruned = DropIndicesByTransformer(lambda c: c.indicator_value == "Red").set_input(vec).get_output()
    out = OpWorkflow().set_result_features(vec, pruned).set_input_dataset(ds).train().score()
    X = out[pruned.name].values
    assert X.shape[1] == 4
    for c, row in zip(ds["color"].to_list(), X.tolist()):
        assert (max(row) == 0) if c == "Red" else (max(row) == 1)
    raw, trimmed = out[vec.name].metadata, out[pruned.name].metadata
    assert raw.size - 1 == trimmed.size
    assert all(c.indicator_value != "Red" for c in trimmed.columns)


def test_drop_indices_by_shortcut():
    """:92-108: ``dropIndicesBy(_.isNullIndicator)`` removes the null column; every row keeps its 1."""
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    ds, color, vec = _picklist_vector()
    pruned = vec.drop_indices_by(lambda c: c.is_null_indicator)
    out = OpWorkflow().set_result_features(vec, pruned).set_input_dataset(ds).train().score()
    X = out[pruned.name].values
    assert X.shape[1] == 4 and bool((X.max(1).values == 1).all())
    trimmed = out[pruned.name].metadata
    assert out[vec.name].metadata.size - 1 == trimmed.size
    assert not any(c.is_null_indicator for c in trimmed.columns)


def test_drop_indices_by_on_a_vector_with_metadata():
    """:41-60: a three-element vector with one metadata column per value; the predicate drops all but the first."""
    from transmogrifai_amd.data.columns import VectorColumn
    from transmogrifai_amd.data.vector_metadata import OpVectorColumnMetadata, OpVectorMetadata
    from transmogrifai_amd.stages.feature.vector_stages import DropIndicesByTransformer
    ds, (v,) = TestFeatureBuilder.of(("v", T.OPVector, [[1.0, 1.0, 0.0], [0.0, 0.0, 0.0], [0.0, 0.0, 0.0]]))
    cols = [OpVectorColumnMetadata(("v",), ("OPVector",), indicator_value=str(i), index=i) for i in range(3)]
    ds = ds.with_column("v", VectorColumn(ds["v"].values, OpVectorMetadata("v", cols)))
    st = DropIndicesByTransformer(lambda c: c.index > 0).set_input(v)
    out = st.transform(ds)[st.get_output().name]
    assert out.values.tolist() == [[1.0], [0.0], [0.0]]
    assert [c.indicator_value for c in out.metadata.columns] == ["0"]


# --------------------------------------------------------------- FilterTextMapTest / FilterIntegralMapTest / ...
_KNIGHTS_TEXT = [{"Arthur": "King", "Lancelot": "Brave", "Galahad": "Pure"},
                 {"Lancelot": "Brave", "Galahad": "Pure", "Bedevere": "Wise"}, {"Knight": "Ni"}]
_KNIGHTS_INT = [{"Arthur": 1, "Lancelot": 2, "Galahad": 3}, {"Lancelot": 2, "Galahad": 3, "Bedevere": 4},
                {"Knight": 5}]
_KNIGHTS_MPL = [{"Arthur": {"King", "Briton"}, "Lancelot": {"Brave", "Knight"}, "Galahad": {"Pure", "Knight"}},
                {"Lancelot": {"Brave", "Knight"}, "Galahad": {"Pure", "Knight"}, "Bedevere": {"Wise", "Knight"}},
                {"Knight": {"Ni", "Ekke Ekke Ekke Ekke Ptang Zoo Boing"}}]


def _norm_maps(rows):
    return [{k: (set(v) if isinstance(v, (set, frozenset, list, tuple)) else v) for k, v in (r or {}).items()}
            for r in rows]


@pytest.mark.parametrize("ftype,data", [(T.TextMap, _KNIGHTS_TEXT), (T.IntegralMap, _KNIGHTS_INT)])
def test_filter_map_allow_and_block(ftype, data):
    from transmogrifai_amd.stages.feature.misc_stages import FilterMap
    ds, (f1,) = _one(data, ftype)
    check_transformer(FilterMap().set_input(f1), ds, expected=data)
    st = FilterMap(allow_list_keys=["Arthur", "Knight"]).set_input(f1)
    got = _norm_maps(st.transform(ds)[st.get_output().name].to_list())
    assert got == [{"Arthur": data[0]["Arthur"]}, {}, {"Knight": data[2]["Knight"]}]
    st = FilterMap(allow_list_keys=[], block_list_keys=["Arthur", "Knight"]).set_input(f1)
    got = _norm_maps(st.transform(ds)[st.get_output().name].to_list())
    keep = lambda r: {k: v for k, v in r.items() if k not in ("Arthur", "Knight")}
    assert got == [keep(data[0]), data[1], {}]


def test_filter_multi_pick_list_map_cleaning():
    """FilterMultiPickListMapTest.scala: clean text is on by default (set values cleaned), and off keeps them."""
    from transmogrifai_amd.stages.feature.misc_stages import FilterMap
    ds, (f1,) = _one(_KNIGHTS_MPL, T.MultiPickListMap)
    cleaned = dict(_KNIGHTS_MPL[2])
    cleaned["Knight"] = {"Ni", "EkkeEkkeEkkeEkkePtangZooBoing"}
    st = FilterMap().set_input(f1)
    assert _norm_maps(st.transform(ds)[st.get_output().name].to_list()) == _norm_maps(_KNIGHTS_MPL[:2] + [cleaned])
    for clean, knight in ((False, _KNIGHTS_MPL[2]["Knight"]), (True, cleaned["Knight"])):
        st = FilterMap(allow_list_keys=["Arthur", "Knight"], clean_text=clean, clean_keys=clean).set_input(f1)
        got = _norm_maps(st.transform(ds)[st.get_output().name].to_list())
        assert got == [{"Arthur": {"King", "Briton"}}, {}, {"Knight": set(knight)}]


def test_filter_map_shortcut():
    from transmogrifai_amd.stages.feature.misc_stages import FilterMap
    ds, (f1,) = _one(_KNIGHTS_TEXT, T.TextMap)
    feat = f1.filter_keys(allow_list_keys=["Arthur", "Knight"])
    assert isinstance(feat.origin_stage, FilterMap) and list(feat.parents) == [f1]
    assert feat.name == feat.origin_stage.get_output_feature_name()


# ---------------------------------------------------------- TextNGramSimilarityTest / SetNGramSimilarityTest
_TEXT_PAIRS = [("Hamlet: To be or not to be - that is the question.", "I like like Hamlet"),
               ("that is the question", "There is no question"), ("Just some random text", "I like like Hamlet"),
               ("Adobe CreativeSuite 5 Master Collection from cheap 4zp",
                "Adobe CreativeSuite 5 Master Collection from cheap d1x"),
               (None, None), ("", ""), ("", None), ("asdf", None), (None, "asdf")]


@pytest.mark.parametrize("n,expected", [
    (3, [0.12666672468185425, 0.6083333492279053, 0.15873020887374878, 0.9629629850387573, 0, 0, 0, 0, 0]),
    (4, [0.11500000953674316, 0.5666666626930237, 0.1547619104385376, 0.9722222089767456, 0, 0, 0, 0, 0]),
])
def test_text_ngram_similarity_exact(n, expected):
    """Lucene NGramDistance in float32: the reference's printed values bit for bit."""
    ds, (f1, f2) = _two(_TEXT_PAIRS, T.Text)
    feat = f1.to_n_gram_similarity(f2, n_gram_size=n, to_lowercase=False)
    check_transformer(feat.origin_stage, ds, expected=expected, tol=0.0)


@pytest.mark.parametrize("n,expected", [
    (3, [0.3333333134651184, 0.09722214937210083, 1.0, 0.0, 0.0, 0.0, 0.0, 0.0]),
    (5, [0.3333333432674408, 0.12361115217208862, 1.0, 0.0, 0.0, 0.0, 0.0, 0.0]),
])
def test_set_ngram_similarity_exact(n, expected):
    pairs = [(["Red", "Green"], ["Red"]), (["Red", "Green"], ["Yellow, Blue"]), (["Red", "Yellow"], ["Red", "Yellow"]),
             ([], ["Red", "Yellow"]), ([], []), ([""], ["asdf"]), ([""], [""]), (["", ""], ["", ""])]
    ds, (f1, f2) = _two(pairs, T.MultiPickList)
    feat = f1.to_n_gram_similarity(f2, n_gram_size=n)
    check_transformer(feat.origin_stage, ds, expected=expected, tol=0.0)


# ------------------------------------------------------------------------------------------ EmailParserTest
def test_email_prefix_and_domain():
    emails = ["test@example.com", "@example.com", "test@", "@", "", "notanemail", None, "first.last@example.com"]
    ds, (e,) = _one(emails, T.Email)
    pre, dom = e.to_email_prefix(), e.to_email_domain()
    assert pre.origin_stage.transform(ds)[pre.name].to_list() == \
        ["test", None, None, None, None, None, None, "first.last"]
    assert dom.origin_stage.transform(ds)[dom.name].to_list() == \
        ["example.com", None, None, None, None, None, None, "example.com"]


# ------------------------------------------------------------------- string indexing (OpStringIndexer*Test)
def test_string_indexer_no_filter_and_unseen():
    from transmogrifai_amd.stages.feature.indexers import OpStringIndexerNoFilter
    from transmogrifai_amd.testkit.spec import check_estimator
    ds, (t,) = _one(["a", "b", "c", "a", "a", "c"], T.Text)
    est = OpStringIndexerNoFilter().set_input(t)
    model, _ = check_estimator(est, ds, expected=[0.0, 2.0, 1.0, 0.0, 0.0, 1.0])
    ds_new, (t_new,) = _one(["a", "b", "c", "a", "a", "c", "d", "e"], T.Text)
    out = model.transform(ds_new.with_column(t.name, ds_new[t_new.name]))[model.get_output().name].to_list()
    assert out == [0.0, 2.0, 1.0, 0.0, 0.0, 1.0, 3.0, 3.0]          # unseen strings -> the extra category
    idx = t.indexed()
    assert isinstance(idx.origin_stage, OpStringIndexerNoFilter)
    # deindexing the indexed column gives the text back (OpStringIndexerNoFilterTest.scala:70-78)
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    de = idx.deindexed()
    scored = OpWorkflow().set_result_features(de).set_input_dataset(ds).train().score()
    assert scored[de.name].to_list() == ["a", "b", "c", "a", "a", "c"]


def test_index_to_string():
    from transmogrifai_amd.stages.feature.indexers import OpIndexToString, OpIndexToStringNoFilter
    ds, (i,) = _one([0.0, 2.0, 1.0, 0.0, 0.0, 1.0], T.RealNN)
    st = OpIndexToString(labels=["a", "c", "b"]).set_input(i)
    check_transformer(st, ds, expected=["a", "b", "c", "a", "a", "c"])
    assert st.params["labels"] == ["a", "c", "b"]
    nf = OpIndexToStringNoFilter(labels=["a", "c"]).set_input(i)   # OpIndexToStringNoFilterTest.scala
    check_transformer(nf, ds, expected=["a", "UnseenIndex", "c", "a", "a", "c"])
    short = i.deindexed(["a", "c"])
    assert isinstance(short.origin_stage, OpIndexToStringNoFilter)
    assert short.origin_stage.transform(ds)[short.name].to_list() == ["a", "UnseenIndex", "c", "a", "a", "c"]


def test_prediction_deindexer():
    """PredictionDeIndexerTest.scala: a permuted index deindexes through the response's indexer labels; a
    response without them fails with the reference's message."""
    from transmogrifai_amd.stages.feature.misc_stages import MapTransformer, PredictionDeIndexer
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    ds, (txt, num) = TestFeatureBuilder.of(("txt", T.Text, ["a", "b", "c"]), ("num", T.RealNN, [0.0, 1.0, 2.0]))
    response = txt.indexed()
    pred = MapTransformer(lambda v: float((int(v) + 1) % 3), T.RealNN, "modulo").set_input(response).get_output()
    de = PredictionDeIndexer().set_input(response, pred).get_output()
    scored = OpWorkflow().set_result_features(de).set_input_dataset(ds).train().score()
    assert scored[de.name].to_list() == ["b", "c", "a"]
    bad = PredictionDeIndexer().set_input(num, pred).get_output()
    with pytest.raises(ValueError, match=f"The feature {num.name} does not contain any label/index mapping"):
        OpWorkflow().set_result_features(bad).set_input_dataset(ds).train().score()


def test_linear_scaler():
    """LinearScalerTest.scala: a zero slope is refused; scale is slope x + intercept, descale its inverse."""
    from transmogrifai_amd.stages.feature.math_stages import DescalerTransformer, ScalerTransformer
    with pytest.raises(ValueError, match="LinearScaler must have a non-zero slope to be invertible"):
        ScalerTransformer(scaling_type="Linear", slope=0.0, intercept=1.0)
    xs = [0.0, 1.0, 2.0, 3.0, 4.0]
    ds, (x,) = _one(xs)
    sc = ScalerTransformer(scaling_type="Linear", slope=2.0, intercept=1.0).set_input(x)
    check_transformer(sc, ds, expected=[2.0 * v + 1.0 for v in xs])
    de = DescalerTransformer().set_input(x, sc.get_output())
    check_transformer(de, sc.transform(ds), expected=[0.5 * v - 0.5 for v in xs])

"""OPMapTransformerTest / OPSetTransformerTest / OPListTransformerTest / OPCollectionTransformerTest
(``core/src/test/.../stages/base/``): an element function lifted over a map / set / list feature."""
from transmogrifai_amd.features import types as T
from transmogrifai_amd.stages.feature.misc_stages import OPCollectionTransformer
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.testkit.spec import check_transformer


def _length(s):
    return None if s is None else len(s)


def _lower(s):
    return None if s is None else s.lower()


def test_map_transformer_email_lengths():
    ds, (top,) = TestFeatureBuilder.of(("name", T.EmailMap, [{"p1": "a@abcd.com", "p2": "xy@abcd.com"}]))
    st = OPCollectionTransformer(_length, T.IntegralMap).set_input(top)
    check_transformer(st, ds, expected=[{"p1": 10, "p2": 11}])


def test_set_and_list_transformers_lowercase():
    ds, (top,) = TestFeatureBuilder.of(("name", T.MultiPickList, [{"A", "B"}]))
    out = check_transformer(OPCollectionTransformer(_lower, T.MultiPickList).set_input(top), ds)
    assert set(out[0]) == {"a", "b"}
    ds, (top,) = TestFeatureBuilder.of(("name", T.TextList, [["A", "B"]]))
    check_transformer(OPCollectionTransformer(_lower, T.TextList).set_input(top), ds, expected=[["a", "b"]])


def test_email_map_to_integral_map_and_nones():
    rows = [{"p1": "Kevin@gmail.com", "p2": "Todd@hotmail.com"}, {"p1": "Ellie@cc.net"}, {"p1": "Dave@facebook.com"},
            {"p1": "Dwayne@wwf.org", "p2": "Darcy@yahoo.co.uk"}]
    ds, (top,) = TestFeatureBuilder.of(("name", T.EmailMap, rows))
    st = OPCollectionTransformer(_length, T.IntegralMap).set_input(top)
    assert st.transform(ds)[st.get_output().name].to_list() == [{"p1": 15, "p2": 16}, {"p1": 12}, {"p1": 17},
                                                                  {"p1": 14, "p2": 17}]
    st = OPCollectionTransformer(lambda s: None, T.IntegralMap).set_input(top)
    got = [st.transform_fn(r) for r in rows]
    assert got == [{"p1": None, "p2": None}, {"p1": None}, {"p1": None}, {"p1": None, "p2": None}]


def test_text_list_with_empty_rows():
    ds, (f1,) = TestFeatureBuilder.of(("name", T.TextList, [["I", "have", "some", "coconuts"], [],
                                                            ["and", "I", "cannot", "lie"]]))
    st = OPCollectionTransformer(_lower, T.TextList).set_input(f1)
    assert st.transform(ds)[st.get_output().name].to_list() == [["i", "have", "some", "coconuts"], [],
                                                                  ["and", "i", "cannot", "lie"]]

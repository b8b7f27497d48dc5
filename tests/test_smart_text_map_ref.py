"""``SmartTextMapVectorizerTest.scala`` ported: a text map whose keys ``text1`` / ``text2`` hold the values of two
text features vectorizes exactly as ``SmartTextVectorizer`` on those features -- one categorical and one hashed
key (max cardinality 2), two categorical keys (10), separate and shared hash spaces (1, hashed) -- and for a
TextAreaMap; the map's column metadata point at the map feature with the key as grouping."""
import pytest

from transmogrifai_amd.features import types as T
from transmogrifai_amd.stages.feature.maps import SmartTextMapVectorizer
from transmogrifai_amd.stages.feature.vectorizers import SmartTextVectorizer
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.workflow.workflow import OpWorkflow

T1 = ["hello world", "hello world", "good evening", "hello world", None]
T2 = ["Hello world!", "What's up", "How are you doing, my friend?", "Not bad, my friend.", None]


def _data(map_type, text_type):
    maps = [{} if a is None else {"text1": a, "text2": b} for a, b in zip(T1, T2)]
    return TestFeatureBuilder.of(("textMap1", map_type, maps), ("textMap2", map_type, [{}] * 5),
                                 ("text1", text_type, T1), ("text2", text_type, T2))


@pytest.mark.parametrize("types", [(T.TextMap, T.Text), (T.TextAreaMap, T.TextArea)])
@pytest.mark.parametrize("max_card,strategy", [(2, "auto"), (10, "auto"), (1, "separate"), (1, "shared")])
def test_map_keys_vectorize_as_the_text_features(types, max_card, strategy):
    ds, (m1, m2, f1, f2) = _data(*types)
    common = dict(max_cardinality=max_card, num_features=4, min_support=1, top_k=2, prepend_feature_name=True,
                  hash_space_strategy=strategy)
    vm = SmartTextMapVectorizer(clean_keys=False, **common).set_input(m1, m2).get_output()
    vt = SmartTextVectorizer(**common).set_input(f1, f2).get_output()
    model = OpWorkflow().set_result_features(vm, vt).set_input_dataset(ds).train()
    out = model.score()
    a, b = out[vm.name].values.double().tolist(), out[vt.name].values.double().tolist()
    assert a == b
    meta_m = vm.origin_stage.metadata["vector_metadata"]
    meta_t = vt.origin_stage.metadata["vector_metadata"]
    assert len(meta_m.columns) == len(meta_t.columns)
    for cm, ct in zip(meta_m.columns, meta_t.columns):
        assert tuple(cm.parent_feature_name) == (m1.name,)
        assert cm.indicator_value == ct.indicator_value

"""Parity pinned to the reference's own fixtures and expected values.

Each test fails if its parity target changes:
* hashing: ``OpHashingTFTest.scala:58-75`` (exact TF vectors, 5 terms) and ``:86-93`` (512 terms),
  ``OPCollectionHashingVectorizerTest.scala:58`` (indices 107 and 224 of 512);
* vectorizers: ``RealVectorizerTest.scala:88-165``, ``OpTextPivotVectorizerTest.scala:44-72``;
* checkpoint shape: ``core/src/test/resources/OldModelVersion_0_7_1/op-model.json/part-00000`` (read as
  JSON only) against this repo's writer -- top-level, stage, feature and vector-metadata keys;
* Titanic: the default binary selector on ``test-data/PassengerDataAll.csv`` lands in the README's
  neighbourhood (hold-out AuPR 0.8225, ``README.md:81-95``).
"""
import gzip
import json
import os

import numpy as np
import pytest

from transmogrifai_amd.features import types as T
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.testkit.spec import check_estimator, check_transformer

REF = "/root/reference"
FIXTURE = f"{REF}/core/src/test/resources/OldModelVersion_0_7_1/op-model.json/part-00000"


def _dense(n, idx, vals):
    v = [0.0] * n
    for i, x in zip(idx, vals):
        v[i] = x
    return v


# ------------------------------------------------------------------------------------------ hashing
HAMLET = [
    "Hamlet: To be or not to be - that is the question.",
    "Гамлет: Быть или не быть - вот в чём вопрос.",
    "המלט: להיות או לא להיות - זאת השאלה.",
    "Hamlet: Être ou ne pas être - telle est la question.",
]


def _hamlet():
    return TestFeatureBuilder.of(("f1", T.TextList, [s.lower().split(" ") for s in HAMLET]))


def test_op_hashing_tf_five_terms_fixture():
    from transmogrifai_amd.dsl import core  # noqa: F401  (registers the DSL)
    ds, (f1,) = _hamlet()
    hashed = f1.tf(num_terms=5)
    expected = [_dense(5, [0, 1, 2, 3, 4], [2.0, 4.0, 2.0, 3.0, 1.0]),
                _dense(5, [0, 1, 2, 3, 4], [4.0, 1.0, 3.0, 1.0, 1.0]),
                _dense(5, [0, 2, 3, 4], [2.0, 2.0, 2.0, 2.0]),
                _dense(5, [0, 1, 2, 4], [3.0, 5.0, 1.0, 2.0])]
    check_transformer(hashed.origin_stage, ds, expected=expected)


def test_op_hashing_tf_default_terms_fixture():
    from transmogrifai_amd.dsl import core  # noqa: F401
    from transmogrifai_amd.utils.text import hash_terms
    ds, (f1,) = _hamlet()
    hashed = f1.tf()
    out = hashed.origin_stage.transform(ds)[hashed.name].values
    assert out.shape[1] == 512
    h = lambda s: int(hash_terms([s], 512)[0])
    assert out[0, h("be")] == 2.0 and out[0, h("that")] == 1.0
    assert out[1, h("быть")] == 2.0 and out[2, h("להיות")] == 2.0 and out[3, h("être")] == 2.0


def test_collection_hashing_vectorizer_fixture():
    from transmogrifai_amd.stages.feature.vectorizers import OPCollectionHashingVectorizer
    ds, (f1,) = TestFeatureBuilder.of(("textList1", T.TextList, [["x", "y"]]))
    check_transformer(OPCollectionHashingVectorizer().set_input(f1), ds,
                      expected=[_dense(512, [107, 224], [1.0, 1.0])])


# -------------------------------------------------------------------------------------- vectorizers
def _real3():
    return TestFeatureBuilder.of(("inA", T.Real, [4.0, None, 2.0]), ("inB", T.Real, [2.0, 2.0, None]),
                                 ("inC", T.Real, [None, None, None]))


def test_real_vectorizer_reference_expectations():
    from transmogrifai_amd.stages.feature.vectorizers import RealVectorizer
    ds, (a, b, c) = _real3()
    check_estimator(RealVectorizer(fill_value=4.2, fill_with_constant=True, track_nulls=False).set_input(a, b, c), ds,
                    expected=[[4.0, 2.0, 4.2], [4.2, 2.0, 4.2], [2.0, 4.2, 4.2]])
    ds, (a, b, c) = _real3()
    check_estimator(RealVectorizer(fill_with_constant=False, track_nulls=False).set_input(a, b, c), ds,
                    expected=[[4.0, 2.0, 0.0], [3.0, 2.0, 0.0], [2.0, 2.0, 0.0]])
    ds, (a, b, c) = _real3()
    check_estimator(RealVectorizer(fill_value=0.0, fill_with_constant=True, track_nulls=True).set_input(a, b, c), ds,
                    expected=[[4.0, 0.0, 2.0, 0.0, 0.0, 1.0], [0.0, 1.0, 2.0, 0.0, 0.0, 1.0],
                              [2.0, 0.0, 0.0, 1.0, 0.0, 1.0]])


def test_text_pivot_vectorizer_reference_expectations():
    from transmogrifai_amd.stages.feature.vectorizers import OpTextPivotVectorizer
    ds, (f1, f2) = TestFeatureBuilder.of(
        ("text1", T.Text, ["hello world", "hello world", "good evening", "hello world", None]),
        ("text2", T.Text, ["Hello world!", "What's up", "How are you doing, my friend?", "Not bad, my friend.", None]))
    est = OpTextPivotVectorizer(min_support=1, top_k=2).set_input(f1, f2)
    check_estimator(est, ds, expected=[_dense(8, [0, 4], [1, 1]), _dense(8, [0, 6], [1, 1]), _dense(8, [1, 5], [1, 1]),
                                       _dense(8, [0, 6], [1, 1]), _dense(8, [3, 7], [1, 1])])


# ------------------------------------------------------------------------------- checkpoint shape
def _saved_model_json(tmp_path):
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.features.builder import FeatureBuilder
    from transmogrifai_amd.selector.factories import BinaryClassificationModelSelector
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    recs = [{"survived": float(i % 2), "age": float(20 + i % 30), "sex": ["m", "f"][i % 3 == 0],
             "boarded": [1_500_000_000_000 + 86400000 * i]} for i in range(120)]
    survived = FeatureBuilder.RealNN("survived").as_response()
    vec = transmogrify([FeatureBuilder.Real("age").as_predictor(), FeatureBuilder.PickList("sex").as_predictor(),
                        FeatureBuilder.DateList("boarded").as_predictor()])
    pred = BinaryClassificationModelSelector.with_train_validation_split(
        model_types_to_use=["OpLogisticRegression"], seed=1).set_input(survived, vec).get_output()
    model = OpWorkflow().set_result_features(survived, pred).set_input_dataset(recs).train()
    path = str(tmp_path / "m")
    model.save(path)
    p = os.path.join(path, "op-model.json", "part-00000.gz")
    with gzip.open(p, "rt") as f:
        return json.load(f)


def test_checkpoint_shape_matches_reference_0_7_1(tmp_path):
    with open(FIXTURE) as f:               # JSON only; nothing executed from the fixture
        ref = json.load(f)
    ours = _saved_model_json(tmp_path)
    legacy = {"blacklistedFeaturesUids": "blocklistedFeaturesUids", "blacklistedMapKeys": "blocklistedMapKeys",
              "blacklistedStages": "blocklistedStages"}
    ref_keys = {legacy.get(k, k) for k in ref}
    assert ref_keys <= set(ours)
    assert set(ours) - ref_keys <= {"trainTimings"}     # our one addition: OpStep phase timings
    # every stage carries the reference stage-writer fields (OpPipelineStageWriter.scala:67-88)
    # (no Spark here: "sparkVersion" is the one reference stage field without a counterpart)
    ref_stage_keys = set.intersection(*[set(s) for s in ref["stages"]]) - {"sparkVersion"}
    for s in ours["stages"]:
        assert ref_stage_keys <= set(s), (s["class"], ref_stage_keys - set(s))
    # raw feature generator stages: same ctorArgs fields
    ref_gen = next(s for s in ref["stages"] if s["class"].endswith("FeatureGeneratorStage"))
    our_gen = next(s for s in ours["stages"] if s["class"].endswith("FeatureGeneratorStage"))
    assert set(ref_gen["ctorArgs"]) - {"aggregateWindow"} <= set(our_gen["ctorArgs"])
    # feature JSON (FeatureJsonHelper.scala:57-140)
    assert set(ref["allFeatures"][0]) == set(ours["allFeatures"][0])
    # transformer paramMap: inputFeatures entries and the vector metadata keys
    ref_vec = next(s for s in ref["stages"] if "outputMetadata" in s["paramMap"])
    our_vec = next(s for s in ours["stages"] if "outputMetadata" in s.get("paramMap", {})
                   and "vector_columns" in s["paramMap"]["outputMetadata"])
    assert set(ref_vec["paramMap"]["inputFeatures"][0]) <= set(our_vec["paramMap"]["inputFeatures"][0])
    assert {"vector_columns", "vector_history"} <= set(our_vec["paramMap"]["outputMetadata"])
    assert set(ref_vec["paramMap"]["outputMetadata"]["vector_columns"][0]) <= \
        set(our_vec["paramMap"]["outputMetadata"]["vector_columns"][0])
    # parameters / trainParameters are OpParams JSON strings with the reference's sections
    for k in ("parameters", "trainParameters"):
        assert set(json.loads(ref[k])) <= set(json.loads(ours[k]))
    assert set(json.loads(ref["rawFeatureFilterResults"])) <= set(json.loads(ours["rawFeatureFilterResults"]))


# ----------------------------------------------------------------------------------------- Titanic
@pytest.mark.slow
def test_titanic_default_selector_holdout_in_readme_neighbourhood():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples"))
    import titanic_simple
    model, metrics = titanic_simple.main([titanic_simple.DEFAULT_CSV, "--all", "--quiet", "--seed=42"])
    summ = model.get_origin_stage_of(titanic_simple.LAST_PREDICTION).metadata["summary"]
    ho = summ["holdoutEvaluation"]["AuPR"]
    # README.md:89: hold-out AuPR 0.8225 (RF selected, 73 hold-out rows); 3-fold CV AuPR of the models
    # README.md:62-64 range 0.675 .. 0.810 -- our random split differs, so pin the neighbourhood
    assert 0.75 <= ho <= 0.97, ho
    assert len(summ["validationResults"]) == 28


def test_titanic_simple_lr_only_pinned():
    """``OpTitanicSimple`` as the reference runs it: withTrainValidationSplit, LR only
    (OpTitanicSimple.scala:135-136). Seeded hold-out AuPR pinned to +-0.03 and the top insights of
    README.md:97-110 (sex and pClass lead; "sex = female" is absent because the current SanityChecker drops the
    later of two features correlated above maxFeatureCorr = 0.99 -- DerivedFeatureFilterUtils.scala:224 -- so
    only "sex = Male" remains, carrying the same |correlation|)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples"))
    import titanic_simple
    model, metrics = titanic_simple.main([titanic_simple.DEFAULT_CSV, "--quiet", "--seed=42"])
    summ = model.get_origin_stage_of(titanic_simple.LAST_PREDICTION).metadata["summary"]
    assert summ["bestModelType"] == "OpLogisticRegression"
    assert summ["validationType"] == "TrainValidationSplit"
    assert len(summ["validationResults"]) == 8
    ho = summ["holdoutEvaluation"]["AuPR"]
    assert abs(ho - 0.7967) <= 0.03, ho
    txt = model.summary_pretty()
    neg = txt[txt.index("Top Negative Correlations"):]
    neg = neg[:neg.index("Top Contributions")]
    assert "sex(sex = Male)" in neg and "pClass(pClass = 3)" in neg
    pos = txt[txt.index("Top Positive Correlations"):txt.index("Top Negative Correlations")]
    assert "pClass(pClass = 1)" in pos and "cabin(cabin = other)" in pos
    sc = next(st for st in model.stages if "dropped" in (st.metadata.get("summary") or {}))
    assert any("sex_Female" in d for d in sc.metadata["summary"]["dropped"])

"""``MultiLabelJoinerTest.scala`` / ``TopNLabelJoinerTest.scala`` ported: the class feature is string-indexed (no
filter, so an unseen-label class is appended) and the joiners read the class names from the indexer's label
metadata, mapping each probability vector to a class-keyed map (all classes, or the top N by score)."""
from transmogrifai_amd import dsl  # noqa: F401
from transmogrifai_amd.features import types as T
from transmogrifai_amd.stages.feature import misc_stages as M
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.workflow.workflow import OpWorkflow


def _data():
    ds, (idf, cls, prob) = TestFeatureBuilder.of(
        ("ID", T.Integral, [1001, 1002, 1003]), ("class", T.Text, ["Low", "Medium", "High"]),
        ("prob", T.OPVector, [[40.0, 30.0, 20.0, 0.0], [20.0, 40.0, 30.0, 0.0], [30.0, 20.0, 40.0, 0.0]]))
    return ds, idf, cls.indexed(unseen_name="UnseenLabel"), prob


def _run(stage, ds):
    out = OpWorkflow().set_result_features(stage.get_output()).set_input_dataset(ds).train().score()
    return out[stage.get_output().name].to_list()


def test_multi_label_joiner():
    ds, _, idx, prob = _data()
    got = _run(M.MultiLabelJoiner().set_input(idx, prob), ds)
    classes = list(got[0])
    assert len(classes) == 4 and "UnseenLabel" in classes
    vecs = [[40.0, 30.0, 20.0, 0.0], [20.0, 40.0, 30.0, 0.0], [30.0, 20.0, 40.0, 0.0]]
    assert got == [dict(zip(classes, v)) for v in vecs]


def test_top_n_label_joiner():
    ds, _, idx, prob = _data()
    full = _run(M.MultiLabelJoiner().set_input(idx, prob), ds)
    classes = list(full[0])
    got2 = _run(M.TopNLabelJoiner(top_n=2).set_input(idx, prob), ds)
    assert got2 == [{classes[0]: 40.0, classes[1]: 30.0}, {classes[1]: 40.0, classes[2]: 30.0},
                    {classes[2]: 40.0, classes[0]: 30.0}]
    got4 = _run(M.TopNLabelJoiner(top_n=4).set_input(idx, prob), ds)
    # the zero-score unseen class is not reported
    assert got4 == [{classes[0]: 40.0, classes[1]: 30.0, classes[2]: 20.0},
                    {classes[1]: 40.0, classes[2]: 30.0, classes[0]: 20.0},
                    {classes[2]: 40.0, classes[0]: 30.0, classes[1]: 20.0}]

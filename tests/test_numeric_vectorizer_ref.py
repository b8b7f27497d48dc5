"""``NumericVectorizerTest.scala`` ported: ``transmogrify`` with a label adds the label-aware bucketizer to the
numeric vectorizer -- the small real sample's exact vectors (value, null indicator, two bucket indicators), and
for random ages / heights / counts the same values as the manual ``vectorize`` + ``autoBucketize`` combination."""
from transmogrifai_amd import dsl  # noqa: F401
from transmogrifai_amd.dsl import transmogrify
from transmogrifai_amd.features import types as T
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.testkit.random_data import RandomIntegral, RandomReal
from transmogrifai_amd.workflow.workflow import OpWorkflow


def _score(ds, *feats):
    out = OpWorkflow().set_result_features(*feats).set_input_dataset(ds).train().score()
    return [out[f.name].values.double().tolist() for f in feats]


def _combine(feats):
    from transmogrifai_amd.stages.feature.vectorizers import VectorsCombiner
    return VectorsCombiner().set_input(list(feats)).get_output()


def test_small_real_sample():
    ds, (inp, label) = TestFeatureBuilder.of(("input", T.Real, [-4.0, -3.0, -2.0, -1.0, 1.0, 2.0, 3.0, 4.0]),
                                             ("label", T.RealNN, [0.0] * 4 + [1.0] * 4), response="label")
    vec = transmogrify([inp], label=label)
    (got,) = _score(ds, vec)
    exp = [[v, 0.0, 1.0, 0.0] if v < 0 else [v, 0.0, 0.0, 1.0] for v in [-4, -3, -2, -1, 1, 2, 3, 4]]
    assert sorted(got) == sorted([[float(x) for x in r] for r in exp])


def test_single_real_with_label_matches_manual():
    age = RandomReal.uniform(0.0, 80.0).reset(1).take(100)
    ds, (a, label) = TestFeatureBuilder.of(("age", T.Real, age),
                                           ("label", T.RealNN, [1.0 if x > 30.0 else 0.0 for x in age]),
                                           response="label")
    auto = transmogrify([a], label=label)
    manual = _combine([a.vectorize(fill_value=0, fill_with_mean=True, track_nulls=True),
                       a.auto_bucketize(label, track_nulls=False)])
    got_a, got_m = _score(ds, auto, manual)
    assert all(sorted(x) == sorted(y) for x, y in zip(got_a, got_m))
    assert len(got_a[0]) > 2          # the bucketizer found the 30.0 threshold


def test_multiple_reals_with_label_match_manual():
    age = RandomReal.uniform(0.0, 80.0).reset(2).take(100)
    height = RandomReal.normal(65.0, 8.0).reset(3).take(100)
    ds, (a, h, label) = TestFeatureBuilder.of(("age", T.Real, age), ("height", T.Real, height),
                                              ("label", T.RealNN, [1.0 if x > 30.0 else 0.0 for x in age]),
                                              response="label")
    auto = transmogrify([a, h], label=label)
    manual = transmogrify([a, a.auto_bucketize(label, track_nulls=False), h, h.auto_bucketize(label, track_nulls=False)])
    got_a, got_m = _score(ds, auto, manual)
    assert all(sorted(x) == sorted(y) for x, y in zip(got_a, got_m))


def test_single_integral_with_label_matches_manual():
    cnt = RandomIntegral.integrals(0, 10).reset(4).take(100)
    ds, (c, label) = TestFeatureBuilder.of(("count", T.Integral, cnt),
                                           ("label", T.RealNN, [1.0 if x > 5 else 0.0 for x in cnt]),
                                           response="label")
    auto = transmogrify([c], label=label)
    manual = transmogrify([c, c.auto_bucketize(label, track_nulls=False)])
    got_a, got_m = _score(ds, auto, manual)
    assert all(sorted(x) == sorted(y) for x, y in zip(got_a, got_m))

"""Expectations ported from ``ScalerTransformerTest.scala`` (linear / log scaling + ScalerMetadata, the scale
shortcut), ``OpScalarStandardScalerTest.scala`` (estimator spec, the DataStdScTest rows for the four
withMean / withStd settings, the scaler metadata of the fit and the descaler round trip in a workflow) and
``FillMissingWithMeanTest.scala`` (real / integral / binary inputs, all-null column with a default)."""
import json
import math

import numpy as np
import pytest

from transmogrifai_amd import dsl  # noqa: F401
from transmogrifai_amd.features import types as T
from transmogrifai_amd.stages.feature import math_stages as M
from transmogrifai_amd.testkit.feature_builder import TestFeatureBuilder
from transmogrifai_amd.workflow.workflow import OpWorkflow


def _vals(stage, ds, name=None):
    return stage.transform(ds)[name or stage.get_output_feature_name()].values.double().tolist()


def test_linear_and_log_scaling_with_metadata():
    ds, (f,) = TestFeatureBuilder.of(("f1", T.Real, [4.0, 1.0, 0.0]))
    st = M.ScalerTransformer(scaling_type="Linear", slope=2.0, intercept=1.0).set_input(f)
    assert _vals(st, ds) == [9.0, 3.0, 1.0]
    assert st.metadata[M.SCALING_TYPE_KEY] == "Linear"
    assert json.loads(st.metadata[M.SCALING_ARGS_KEY]) == {"slope": 2.0, "intercept": 1.0}
    lg = M.ScalerTransformer(scaling_type="Logarithmic").set_input(f)
    out = lg.transform(ds)[lg.get_output_feature_name()]
    assert out.values[:2].double().tolist() == [math.log(4.0), 0.0]
    assert not bool(out.valid[2])                 # log(0) = -Infinity: not a finite value here
    assert lg.metadata[M.SCALING_TYPE_KEY] == "Logarithmic" and json.loads(lg.metadata[M.SCALING_ARGS_KEY]) == {}
    s = f.scale(scaling_type="Linear", slope=10.0, intercept=0.5)
    assert _vals(s.origin_stage, ds, s.name) == [40.5, 10.5, 0.5]


def test_standard_scaler_estimator_spec():
    ds, (f,) = TestFeatureBuilder.of(("f", T.RealNN, [10.0, 100.0, 1000.0]))
    m = M.OpScalarStandardScaler().set_input(f).fit(ds)
    np.testing.assert_allclose(_vals(m, ds), [-0.6575959492214292, -0.4931969619160719, 1.150792911137501],
                               rtol=1e-12)


_STD_ROWS = {   # DataStdScTest.input: someNumericFeature, then the expected columns
    "x": [1.0, 2.0, 4.0],
    "both": [-0.8728715609439697, -0.2182178902359925, 1.0910894511799618],
    "mean_only": [-1.333333333333333, -0.33333333333333304, 1.666666666666667],
    "std_only": [0.6546536707079772, 1.3093073414159544, 2.618614682831909],
}


@pytest.mark.parametrize("with_mean,with_std,key", [(False, False, "x"), (False, True, "std_only"),
                                                    (True, False, "mean_only"), (True, True, "both")])
def test_standard_scaler_mean_std_settings(with_mean, with_std, key):
    ds, (f,) = TestFeatureBuilder.of(("someNumericFeature", T.RealNN, _STD_ROWS["x"]))
    m = M.OpScalarStandardScaler(with_mean=with_mean, with_std=with_std).set_input(f).fit(ds)
    got = np.asarray(_vals(m, ds))
    assert float(((got - np.asarray(_STD_ROWS[key])) ** 2).sum()) <= 1e-6


def test_z_normalize_shortcut_in_workflow():
    ds, (f,) = TestFeatureBuilder.of(("someNumericFeature", T.RealNN, _STD_ROWS["x"]))
    out = f.z_normalize()
    model = OpWorkflow().set_result_features(out).set_input_dataset(ds).train()
    got = np.asarray(model.score()[out.name].values.double())
    assert float(((got - np.asarray(_STD_ROWS["both"])) ** 2).sum()) <= 1e-6


def test_standard_scaler_metadata_and_descale_round_trip():
    vals = [10.0, 100.0, 1000.0]
    ds, (f,) = TestFeatureBuilder.of(("f", T.RealNN, vals))
    est = M.OpScalarStandardScaler().set_input(f)
    normed = est.get_output()
    model = est.fit(ds)
    mean = sum(vals) / 3
    std = math.sqrt(sum((mean - v) ** 2 for v in vals) / 2)
    sc = M.parse_scaler_metadata(model.metadata)
    assert sc["scaling_type"] == "Linear"
    assert abs((sc["slope"] - 1 / std) / (1 / std)) < 1e-3
    assert abs((sc["intercept"] + mean / std) / (-mean / std)) < 1e-3
    descaled = normed.descale(normed)
    wf = OpWorkflow().set_result_features(descaled).set_input_dataset(ds).train()
    got = wf.score()[descaled.name].values.double().tolist()
    assert all(abs(a - b) < 1e-4 for a, b in zip(got, vals))


@pytest.mark.parametrize("ftype,vals,expected", [
    (T.Real, [4.0, 2.0, None, 6.0], [4.0, 2.0, 4.0, 6.0]),
    (T.Integral, [4, 2, None, 6], [4.0, 2.0, 4.0, 6.0]),
    (T.Binary, [True, False, None], [1.0, 0.0, 0.5]),
])
def test_fill_missing_with_mean(ftype, vals, expected):
    ds, (f,) = TestFeatureBuilder.of(("f", ftype, vals))
    out = f.fill_missing_with_mean()
    m = out.origin_stage.fit(ds)
    assert sorted(_vals(m, ds, out.name)) == sorted(expected)
    assert out.wtype is T.RealNN


def test_fill_missing_with_mean_all_null_default():
    ds, (f,) = TestFeatureBuilder.of(("fNull", T.Real, [None] * 7))
    out = f.fill_missing_with_mean(default=3.14159)
    assert _vals(out.origin_stage.fit(ds), ds, out.name) == [3.14159] * 7

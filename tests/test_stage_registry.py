"""Stage-class registry: one class per reference short name, so a reference checkpoint naming
``com.salesforce.op.stages.impl.feature.OpIndexToString`` resolves the same way whatever was imported first."""
from __future__ import annotations

import pytest

from transmogrifai_amd.features import types as T
from transmogrifai_amd.stages.base import UnaryTransformer, import_stage_modules, register_stage, stage_class
from transmogrifai_amd.workflow.io import _build_stage

REF_CLASS = "com.salesforce.op.stages.impl.feature.OpIndexToString"


def test_reference_name_resolves_to_one_class():
    import_stage_modules()
    from transmogrifai_amd.stages.feature import indexers, nlp_stages
    assert stage_class(REF_CLASS) is indexers.OpIndexToString
    assert nlp_stages.OpIndexToString is indexers.OpIndexToString


def test_duplicate_short_name_is_rejected():
    import_stage_modules()

    with pytest.raises(TypeError, match="registered twice"):
        @register_stage
        class OpIndexToString(UnaryTransformer):          # noqa: F811 - the point of the test
            output_type = T.Text


def test_reference_checkpoint_stage_loads_and_scores():
    sj = {"class": REF_CLASS, "uid": "OpIndexToString_000000000042", "operationName": "idx2str",
          "outputType": "com.salesforce.op.features.types.Text",
          "paramMap": {"labels": ["no", "yes"], "outputFeatureName": "label_idx2str"},
          "ctorArgs": {}}
    st = _build_stage(sj)
    assert type(st).__name__ == "OpIndexToString" and st.uid == sj["uid"]
    assert [st.transform_fn(v) for v in (1.0, 0.0)] == ["yes", "no"]
    with pytest.raises(ValueError):
        st.transform_fn(2.0)
    nf = dict(sj, **{"class": REF_CLASS + "NoFilter", "ctorArgs": {"labels": ["a"], "unseenName": "U"}})
    st2 = _build_stage(nf)
    assert [st2.transform_fn(v) for v in (0.0, 3.0)] == ["a", "U"]

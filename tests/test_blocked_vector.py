"""Blocked vector columns (VectorsCombiner / SanityChecker keep-mask without copies, K1/K18) and the
HIP row x column gather against dense torch indexing."""
import pytest
import torch

from transmogrifai_amd.data.columns import VectorColumn


def _blocked(dev):
    g = torch.Generator().manual_seed(0)
    dt = torch.float32 if dev != "cpu" else torch.float64
    a = torch.randn(1000, 7, generator=g).to(dev, dt)
    b = torch.randn(1000, 130, generator=g).to(dev, dt)[:, 3:120]          # a strided view block
    c = torch.randn(1000, 64, generator=g).to(dev, dt)
    v = VectorColumn(metadata=None, blocks=[(a, None), (b, None), (c, torch.tensor([5, 1, 63, 0], device=dev))])
    dense = torch.cat([a, b, c[:, [5, 1, 63, 0]]], 1)
    return v, dense


def _check(dev):
    v, dense = _blocked(dev)
    assert v.is_blocked and v.width == dense.shape[1] and len(v) == 1000
    torch.testing.assert_close(v.values, dense, rtol=0, atol=0)
    rows = torch.tensor([999, 0, 17, 17, 500], device=dev)
    torch.testing.assert_close(v.take_rows(rows), dense[rows], rtol=0, atol=0)
    keep = [0, 3, 6, 7, 8, 50, 123, 124, 127]
    s = v.select_columns(keep)
    torch.testing.assert_close(s.values, dense[:, keep], rtol=0, atol=0)
    torch.testing.assert_close(s.take_rows(rows), dense[rows][:, keep], rtol=0, atol=0)
    s2 = s.select_columns([8, 0, 4])
    torch.testing.assert_close(s2.values, dense[:, [keep[8], keep[0], keep[4]]], rtol=0, atol=0)
    with pytest.raises(IndexError):
        v.select_columns([dense.shape[1]])


def test_blocked_vector_cpu():
    _check("cpu")


@pytest.mark.gpu
def test_blocked_vector_gather_gpu():
    from transmogrifai_amd.ops import _native
    _check("cuda")
    assert _native.hip_loaded()


def test_combiner_and_sanity_checker_do_not_copy():
    from transmogrifai_amd.testkit.synthetic import binary_table
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    from transmogrifai_amd.readers.base import InMemoryReader
    ds, label, preds = binary_table(3000, n_real=6, n_int=2, n_pick=2, seed=3)
    vec = transmogrify(preds)
    checked = label.sanity_check(vec, remove_bad_features=True)
    wf = OpWorkflow().set_result_features(checked).set_reader(InMemoryReader(ds))
    model = wf.train()
    out = model.score(keep_intermediate_features=True)
    v, c = out[vec.name], out[checked.name]
    assert v.is_blocked            # combined without torch.cat
    base = {t.data_ptr() for t, _ in v.blocks}
    assert {t.data_ptr() for t, _ in c.blocks} <= base     # keep-mask is a view of the same storage
    keep = model.get_origin_stage_of(checked).indices_to_keep
    torch.testing.assert_close(c.values, v.values[:, keep], rtol=0, atol=0)

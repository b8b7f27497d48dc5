"""HIP text / categorical / calendar kernels (text_kernels.hip) against the host reference path:
hashing TF (incl. the OpHashingTFTest.scala:58-75 fixture), value counts, integral mode,
NumericBucketizer, DateToUnitCircle, and a SmartTextVectorizer transform end to end."""
import random

import numpy as np
import pytest
import torch

from transmogrifai_amd.data.columns import NumericColumn, TextColumn
from transmogrifai_amd.features import types as T
from transmogrifai_amd.ops import text as OT
from transmogrifai_amd.utils import text as TU

pytestmark = pytest.mark.gpu


def _hip_loaded():
    from transmogrifai_amd.ops import _native
    return _native.hip_loaded()


def _vocab(n, seed):
    r = random.Random(seed)
    words = ["alpha", "Beta", "gamma", "δέλτα", "東京", "x_1", "3.14", "the", "it's", "résumé"] + \
            [f"w{i}" for i in range(300)]
    return [" ".join(r.choice(words) for _ in range(r.randint(0, 30))) for _ in range(n)]


@pytest.mark.parametrize("shared,binary,nf", [(True, False, 512), (False, False, 512), (True, True, 64),
                                              (True, False, 8192)])
def test_hashed_tf_matches_host(shared, binary, nf):
    g = torch.Generator().manual_seed(3)
    n = 20_011
    ins_h, ins_d = [], []
    for k in range(3):
        vocab = _vocab(500, k)
        codes = torch.randint(-1, len(vocab), (n,), generator=g, dtype=torch.int32)
        tb = TU.tokenize_batch(vocab)
        pre = int(TU.hash_terms([f"feat{k}"], nf)[0]) if k != 1 else None
        ins_h.append(OT.HashInput(codes, tb, pre))
        ins_d.append(OT.HashInput(codes.cuda(), tb, pre))
    W = nf if shared else 3 * nf
    ref = torch.empty(n, W, dtype=torch.float32)
    OT.hashed_tf(ref, ins_h, nf, shared, binary)
    big = torch.full((n, W + 7), -5.0, device="cuda")
    OT.hashed_tf(big[:, 3:3 + W], ins_d, nf, shared, binary)     # written in place into a wider matrix
    torch.testing.assert_close(big[:, 3:3 + W].cpu(), ref, rtol=0, atol=0)
    assert (big[:, :3] == -5).all() and (big[:, 3 + W:] == -5).all()
    assert _hip_loaded()


def test_hashing_tf_fixture_on_device():
    # OpHashingTFTest.scala:58-75: Spark HashingTF with 5 terms over the Hamlet token lists
    from test_reference_fixtures import HAMLET
    tb = TU.TokenBatch.from_lists([s.lower().split(" ") for s in HAMLET])
    out = torch.empty(4, 5, device="cuda")
    OT.hashed_tf(out, [OT.HashInput(None, tb, None)], 5, True, False)
    expect = [[2, 4, 2, 3, 1], [4, 1, 3, 1, 1], [2, 0, 2, 2, 2], [3, 5, 1, 0, 2]]
    np.testing.assert_array_equal(out.cpu().numpy(), np.asarray(expect, np.float32))
    assert _hip_loaded()


def test_code_counts_lds_and_global():
    g = torch.Generator().manual_seed(4)
    n = 300_007
    cs = [torch.randint(-1, 100, (n,), generator=g, dtype=torch.int32),
          torch.randint(-1, 40_000, (n,), generator=g, dtype=torch.int32)]
    for nv in ([100, 40_000], [100, 100]):
        ref = OT.code_counts(cs[:1], nv[:1]) if nv[1] == 100 else OT.code_counts(cs, nv)
        got = OT.code_counts([c.cuda() for c in cs[:len(ref)]], nv[:len(ref)])
        for a, b in zip(got, ref):
            np.testing.assert_array_equal(a, b)
    assert _hip_loaded()


def test_column_modes_on_device():
    from transmogrifai_amd.ops import vector as V
    g = torch.Generator().manual_seed(5)
    n = 100_000
    cols_h, cols_d = [], []
    for lo, hi in ((-50, 50), (0, 3), (-(1 << 40), 1 << 40)):
        v = torch.randint(lo, hi, (n,), generator=g, dtype=torch.int64)
        ok = torch.rand(n, generator=g) > 0.3
        cols_h.append(NumericColumn(T.Integral, v, ok))
        cols_d.append(NumericColumn(T.Integral, v.cuda(), ok.cuda()))
    assert V.column_modes(cols_d) == V.column_modes(cols_h)


@pytest.mark.parametrize("left,ti,tn", [(True, False, True), (False, True, True), (True, True, False)])
def test_bucketize_matches_host(left, ti, tn):
    g = torch.Generator().manual_seed(6)
    n = 100_003
    x = torch.randn(n, generator=g, dtype=torch.float64) * 3
    x[::97] = 1.0   # exactly on a split
    ok = torch.rand(n, generator=g) > 0.1
    splits = [-100.0, -1.0, 0.0, 1.0, 2.5, 100.0] if not ti else [-1.0, 0.0, 1.0, 2.5]
    w = len(splits) - 1 + int(ti) + int(tn)
    ref = torch.zeros(n, w, dtype=torch.float32)
    OT.bucketize_into(ref, x, ok, splits, tn, ti, left)
    got = torch.zeros(n, w, device="cuda")
    OT.bucketize_into(got, x.cuda(), ok.cuda(), splits, tn, ti, left)
    torch.testing.assert_close(got.cpu(), ref, rtol=0, atol=0)
    with pytest.raises(ValueError):
        OT.bucketize_into(torch.zeros(3, 3, device="cuda"), torch.tensor([0.5, 7.0, 0.1], dtype=torch.float64,
                                                                          device="cuda"),
                          torch.ones(3, dtype=torch.bool, device="cuda"), [0.0, 1.0, 2.0], True, False, True)


@pytest.mark.parametrize("period", ["DayOfMonth", "DayOfWeek", "DayOfYear", "HourOfDay", "MonthOfYear",
                                    "WeekOfMonth", "WeekOfYear"])
def test_date_unit_circle_matches_host(period):
    g = torch.Generator().manual_seed(7)
    n = 50_000
    ms = torch.randint(-(1 << 42), 1 << 42, (n,), generator=g, dtype=torch.int64)
    ok = torch.rand(n, generator=g) > 0.1
    ref = torch.zeros(n, 2, dtype=torch.float32)
    OT.date_unit_circle_into(ref, ms, ok, period)
    got = torch.zeros(n, 2, device="cuda")
    OT.date_unit_circle_into(got, ms.cuda(), ok.cuda(), period)
    torch.testing.assert_close(got.cpu(), ref, rtol=0, atol=2e-7)


def test_smart_text_vectorizer_device_equals_host():
    from transmogrifai_amd.stages.feature.vectorizers import SmartTextVectorizer
    from transmogrifai_amd.features.builder import FeatureBuilder
    r = random.Random(9)
    n = 5000
    free = _vocab(3000, 11)
    cat = ["red", "green", "blue", None]
    rows_free = [r.choice(free) if r.random() > 0.1 else None for _ in range(n)]
    rows_cat = [r.choice(cat) for _ in range(n)]
    outs = []
    for dev in ("cpu", "cuda"):
        f1 = FeatureBuilder.Text("free").as_predictor()
        f2 = FeatureBuilder.PickList("cat").as_predictor()
        st = SmartTextVectorizer(max_cardinality=100, track_text_len=True).set_input(f1, f2)
        c1 = TextColumn.from_values(T.Text, rows_free, device=dev)
        c2 = TextColumn.from_values(T.PickList, rows_cat, device=dev)
        model = st.fit_columns(c1, c2)
        model._inputs = st._inputs
        model.metadata = st.metadata
        outs.append(model.transform_columns(c1, c2).values.cpu().to(torch.float32))
    assert outs[0].shape[1] > 512
    torch.testing.assert_close(outs[1], outs[0], rtol=0, atol=0)

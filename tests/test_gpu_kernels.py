"""HIP kernels vs plain fp64/fp32 PyTorch references, and an end-to-end workflow on the device."""
import numpy as np
import pytest
import torch

from transmogrifai_amd.data.columns import NumericColumn
from transmogrifai_amd.features import types as T

pytestmark = pytest.mark.gpu


def _native_loaded():
    from transmogrifai_amd.ops import _native
    return _native.hip_loaded()


def test_col_stats_matches_fp64():
    from transmogrifai_amd.ops import stats as ST
    g = torch.Generator().manual_seed(0)
    X = torch.randn(100_003, 37, generator=g) * 3 + 1
    X[:, 5] = 0
    X[::7, 9] = 0
    ref = ST.col_stats(X.to(torch.float64))
    got = ST.col_stats(X.cuda())
    for k in ("mean", "variance", "min", "max", "numNonzeros"):
        torch.testing.assert_close(got[k].cpu(), ref[k], rtol=1e-6, atol=1e-6)
    assert _native_loaded()


def test_masked_colsum_matches_fp64():
    """RealVectorizer fill-with-mean: one masked multi-column sum launch vs the fp64 torch path."""
    from transmogrifai_amd.ops import vector as V
    g = torch.Generator().manual_seed(4)
    cols = []
    for j, n_ok in enumerate([1.0, 0.9, 0.0, 0.5, 1.0]):
        x = torch.randn(300_001, generator=g) * (10 ** j)
        valid = torch.rand(300_001, generator=g) < n_ok
        x = x.to(torch.float64) if j == 3 else x.to(torch.float32)
        cols.append(NumericColumn(T.Real, x, None if j == 4 else valid))
    host = V.column_means(cols)
    dev = V.column_means([c.to("cuda") if c.valid is not None else
                          NumericColumn(T.Real, c.values.cuda(), None) for c in cols])
    for a, b in zip(host, dev):
        assert abs(a - b) <= 1e-9 * max(1.0, abs(a)), (a, b)
    assert host[2] == 0.0 and dev[2] == 0.0


def test_vectorize_numeric_matches_host():
    from transmogrifai_amd.ops import vector as V
    g = torch.Generator().manual_seed(1)
    n = 50_001
    cols_h, cols_d = [], []
    for j in range(5):
        v = torch.randn(n, generator=g, dtype=torch.float64)
        ok = torch.rand(n, generator=g) > 0.2
        cols_h.append(NumericColumn(T.Real, v.to(torch.float32), ok))
        cols_d.append(NumericColumn(T.Real, v.to(torch.float32).cuda(), ok.cuda()))
    fills = [0.5, -1.0, 2.0, 0.0, 3.25]
    for track in (True, False):
        ref = V.fill_and_track(cols_h, fills, track, torch.float32)
        got = V.fill_and_track(cols_d, fills, track, torch.float32)
        torch.testing.assert_close(got.cpu(), ref)
    assert _native_loaded()


def test_workflow_end_to_end_on_device():
    from transmogrifai_amd import config as CFG
    from transmogrifai_amd.testkit.synthetic import binary_table
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.readers.base import InMemoryReader
    from transmogrifai_amd.selector.factories import BinaryClassificationModelSelector
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    dev = torch.device("cuda:0")
    old = CFG.default_device()
    CFG.set_default_device(dev)
    try:
        ds, label, preds = binary_table(20_000, n_real=10, n_int=3, n_pick=3, seed=5, device=dev)
        vec = transmogrify(preds)
        checked = label.sanity_check(vec, remove_bad_features=True)
        pred = BinaryClassificationModelSelector.with_cross_validation(
            num_folds=2, seed=3, model_types_to_use=["OpLogisticRegression", "OpRandomForestClassifier"]
        ).set_input(label, checked).get_output()
        model = OpWorkflow().set_result_features(label, pred).set_reader(InMemoryReader(ds)).train()
        summ = model.get_origin_stage_of(pred).metadata["summary"]
        assert summ["holdoutEvaluation"]["AuPR"] > 0.5
        assert _native_loaded()
    finally:
        CFG.set_default_device(old)


@pytest.mark.gpu
def test_onehot_pivot_kernel_matches_host():
    from transmogrifai_amd.ops import vector as V
    g = torch.Generator().manual_seed(0)
    n = 5000
    codes = [torch.randint(-1, 7, (n,), generator=g, dtype=torch.int32), torch.randint(-1, 3, (n,), generator=g,
                                                                                        dtype=torch.int32)]
    luts = [np.array([0, 1, 2, 3, 3, 3, 3, 4]), np.array([1, 0, 2, -1])]
    offs = [0, 5]
    ref = torch.zeros(n, 8)
    V.onehot_pivot(ref, codes, luts, offs)
    out = torch.zeros(n, 8, device="cuda")
    V.onehot_pivot(out, [c.cuda() for c in codes], luts, offs)
    torch.testing.assert_close(out.cpu(), ref)
    assert float(ref.sum()) > 0


def test_xgb_fused_round_epilogue_matches_torch_path(monkeypatch):
    """The fused boosting-round kernel (margins, gradients, AuPR counts) against the torch reference."""
    from transmogrifai_amd.models.base import FitJob
    from transmogrifai_amd.models.trees import XGBoostClassifierLearner
    g = torch.Generator().manual_seed(3)
    n, d = 20_000, 12
    X = torch.randn(n, d, generator=g)
    X[:, :3] = (X[:, :3] > 0.8).float()               # sparse 0/1 columns exercise the missing bin
    y = ((X[:, 3] + X[:, 0] - 0.5 * X[:, 5] + 0.3 * torch.randn(n, generator=g)) > 0).float()
    Xd, yd = X.cuda(), y.cuda()
    params = dict(XGBoostClassifierLearner.defaults, num_round=15, max_depth=4, eta=0.3, missing=0.0,
                  num_early_stopping_rounds=5)
    rows = torch.arange(0, n, 2, device="cuda")
    rows2 = torch.arange(1, n, 3, device="cuda")
    jobs = [FitJob(params, rows), FitJob(dict(params, max_depth=6), rows2), FitJob(dict(params, eta=0.1), rows)]
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("TMOG_XGB_FUSED", flag)
        sts = XGBoostClassifierLearner().fit_batch(Xd, yd, jobs)
        outs.append([XGBoostClassifierLearner().predict(st, Xd)[2][:, 1].cpu() for st in sts])
    for a, b in zip(*outs):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
    assert _native_loaded()


def test_xgb_pipelined_parts_identical_to_single_loop(monkeypatch):
    """Boosting the jobs in concurrent halves (own host thread + stream each, disjoint native slots)
    gives exactly the trees and early-stopping rounds of the single loop."""
    from transmogrifai_amd.models.base import FitJob
    from transmogrifai_amd.models.trees import XGBoostClassifierLearner
    g = torch.Generator().manual_seed(4)
    n, d = 30_000, 16
    X = torch.randn(n, d, generator=g)
    X[:, :4] = (X[:, :4] > 0.7).float()
    y = ((X[:, 4] + X[:, 0] - 0.5 * X[:, 6] + 0.5 * torch.randn(n, generator=g)) > 0).float()
    Xd, yd = X.cuda(), y.cuda()
    params = dict(XGBoostClassifierLearner.defaults, num_round=25, max_depth=6, eta=0.3, missing=0.0,
                  num_early_stopping_rounds=3)
    jobs = [FitJob(dict(params, min_child_weight=m), torch.arange(k, n, 3, device="cuda"))
            for m in (1.0, 10.0) for k in range(3)]
    outs = []
    for flag in ("1", "2", "3"):
        monkeypatch.setenv("TMOG_XGB_PIPE", flag)
        outs.append(XGBoostClassifierLearner().fit_batch(Xd, yd, jobs))
    for other in outs[1:]:
        for a, b in zip(outs[0], other):
            assert a["num_trees"] == b["num_trees"]
            for k in a["forest"]:
                va, vb = a["forest"][k], b["forest"][k]
                if isinstance(va, np.ndarray):
                    np.testing.assert_array_equal(va, vb, err_msg=k)
    assert _native_loaded()


def test_xgb_epilogue_quantisation_maxima_identical_trees(monkeypatch):
    """The per-job max |g| / max h that the round epilogue max-reduces (plus the once-computed max of the
    rows a job never trains on) give exactly the scales, hence the trees, of scanning G / H each round."""
    from transmogrifai_amd.models.base import FitJob
    from transmogrifai_amd.models.trees import XGBoostClassifierLearner
    g = torch.Generator().manual_seed(5)
    n, d = 30_000, 14
    X = torch.randn(n, d, generator=g)
    X[:, :4] = (X[:, :4] > 0.7).float()
    y = ((X[:, 4] + X[:, 0] - 0.5 * X[:, 6] + 0.5 * torch.randn(n, generator=g)) > 0).float()
    Xd, yd = X.cuda(), y.cuda()
    params = dict(XGBoostClassifierLearner.defaults, num_round=20, max_depth=6, eta=0.3, missing=0.0,
                  num_early_stopping_rounds=4)
    jobs = [FitJob(dict(params, min_child_weight=m), torch.arange(k, n, 3, device="cuda"))
            for m in (1.0, 10.0) for k in range(3)]
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("TMOG_XGB_AMAX", flag)
        outs.append(XGBoostClassifierLearner().fit_batch(Xd, yd, jobs))
    for a, b in zip(*outs):
        assert a["num_trees"] == b["num_trees"]
        for k in a["forest"]:
            va, vb = a["forest"][k], b["forest"][k]
            if isinstance(va, np.ndarray):
                np.testing.assert_array_equal(va, vb, err_msg=k)
    assert _native_loaded()


@pytest.mark.parametrize("switch", ["TMOG_PAIR_SCAN", "TMOG_FUSED_REDUCE"])
@pytest.mark.parametrize("learner", ["xgb", "xgbdeep", "rf", "rf3"])
def test_pair_scan_identical_to_subtract_then_scan(monkeypatch, learner, switch):
    """Sibling pairs' subtraction + split scan fused in one pass (pair_scan_kernel), and the node reduction
    fused into the scan's last block, grow exactly the trees of the separate kernels (hist_subtract, node-wise
    split scan, split_reduce): Newton (XGBoost), Gini with 2 and 3 classes."""
    from transmogrifai_amd.models.base import FitJob
    from transmogrifai_amd.models.trees import RandomForestClassifierLearner, XGBoostClassifierLearner
    g = torch.Generator().manual_seed(6)
    n, d = 30_000, 18
    X = torch.randn(n, d, generator=g)
    X[:, :5] = (X[:, :5] > 0.6).float()
    z = X[:, 5] + X[:, 0] - 0.5 * X[:, 7] + 0.5 * torch.randn(n, generator=g)
    y = (z > 0).float() if learner != "rf3" else torch.bucketize(z, torch.tensor([-0.5, 0.5])).float()
    Xd, yd = X.cuda(), y.cuda()
    if learner in ("xgb", "xgbdeep"):
        L = XGBoostClassifierLearner
        # xgbdeep: depth-10 trees with a small min_child_weight -- hundreds of nodes per level, the many-node /
        # many-level case of the fused reduction's cross-workgroup hand-off
        params = dict(L.defaults, num_round=12, max_depth=7, eta=0.3, missing=0.0) if learner == "xgb" else \
            dict(L.defaults, num_round=6, max_depth=10, eta=0.3, missing=0.0, gamma=0.0)
        jobs = [FitJob(dict(params, min_child_weight=m), torch.arange(k, n, 3, device="cuda"))
                for m in ((1.0, 10.0) if learner == "xgb" else (0.05, 0.5)) for k in range(3)]
    else:
        L = RandomForestClassifierLearner
        params = dict(L.defaults, num_trees=6, max_depth=8, feature_subset_strategy="all")   # no subsets
        jobs = [FitJob(dict(params, min_instances_per_node=mi), torch.arange(k, n, 2, device="cuda"))
                for mi in (1, 10) for k in range(2)]
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv(switch, flag)
        outs.append(L().fit_batch(Xd, yd, jobs))
    for a, b in zip(*outs):
        for k in a["forest"]:
            va, vb = a["forest"][k], b["forest"][k]
            if isinstance(va, np.ndarray):
                np.testing.assert_array_equal(va, vb, err_msg=k)
    assert _native_loaded()


def test_aupr_counts_kernel_matches_torch():
    """Early-stopping AuPR from (label, score-bin) count tables: HIP kernel vs the torch path, including
    leading empty bins, a set without positives and an empty set."""
    from transmogrifai_amd.evaluators.metrics import _aupr_from_counts_torch, binned_aupr_from_counts
    g = torch.Generator().manual_seed(7)
    for bins in (1 << 16, 4099, 1000):               # 16-byte segment loads, and the scalar path
        K = 6
        h = torch.randint(0, 4, (K, 2, bins), generator=g, dtype=torch.int32)
        h[:, :, : bins // 3] = 0                               # leading empty bins
        h[1, :, ::5] = 0
        h[2, 1] = 0                                            # no positives
        h[3] = 0                                               # empty
        h[4, :, bins - 7:] = 0                                 # trailing empty bins
        h[5] = 0
        h[5, 0, 100] = 3
        h[5, 1, 101] = 2
        want = _aupr_from_counts_torch(h.double()).numpy()
        got = binned_aupr_from_counts(h.cuda()).cpu().numpy()
        np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-14)
        assert got[2] == 0.0 and got[3] == 0.0
    assert _native_loaded()


def test_row_uniform_kernel_bit_identical():
    from transmogrifai_amd.tuning import splitters as SP
    rid = torch.randint(0, 1 << 40, (100_003,), dtype=torch.int64)
    ref = SP.row_uniform(rid, 1234, 7)
    got = SP.row_uniform(rid.cuda(), 1234, 7).cpu()
    assert torch.equal(ref, got)
    refm = SP.row_uniform_multi(rid, [1, 2, 3], 23)
    gotm = SP.row_uniform_multi(rid.cuda(), [1, 2, 3], 23).cpu()
    assert torch.equal(refm, gotm)


def test_poisson_pack_kernel_matches_host():
    """Fused bootstrap draw + root packing == the torch path, tree by tree (order-free)."""
    from transmogrifai_amd.models import tree_engine as TE
    from transmogrifai_amd.models.trees import bootstrap_weights_multi
    rows = torch.arange(3, 200_003, 3, dtype=torch.int64)
    seeds = [11, 12, 13, 14, 15]
    pc, cc = TE.bootstrap_pack(rows, seeds, 1.0)
    pg, cg = TE.bootstrap_pack(rows.cuda(), seeds, 1.0)
    assert (cc == cg).all()
    w = bootstrap_weights_multi(rows, seeds, 1.0)
    assert (cc == (w > 0).sum(1).numpy()).all()
    off = np.concatenate([[0], np.cumsum(cc)])
    pg = pg.cpu()
    for t in range(len(seeds)):
        a, b = pc[off[t]:off[t + 1]], pg[off[t]:off[t + 1]]
        assert torch.equal(a.sort().values, b.sort().values)
    assert _native_loaded()


@pytest.mark.parametrize("max_bins,reserve,mv", [(32, False, None), (64, True, 0.0), (256, True, None), (2, False, None)])
def test_hip_quantize_matches_torch_path(monkeypatch, max_bins, reserve, mv):
    """quantize_kernels.hip against the torch searchsorted path: ties with the fp32 thresholds, NaN, +-inf, the
    missing value, a feature count that is not a multiple of the 64-feature block."""
    from transmogrifai_amd.models.binning import find_splits, quantize
    g = torch.Generator().manual_seed(7)
    n, d = 70_001, 131
    X = torch.randn(n, d, generator=g)
    X[:, :20] = (X[:, :20] > 0.5).float()                 # two-valued columns: exact ties with thresholds
    X[:, 20:30] = torch.round(X[:, 20:30] * 3) / 3        # few distinct values
    X[::97, 40] = float("nan")
    X[::101, 41] = float("inf")
    X[::103, 42] = -float("inf")
    Xd = X.cuda()
    spec = find_splits(Xd, max_bins, missing_value=mv, reserve_missing=reserve)
    monkeypatch.setenv("TMOG_HIP_QUANTIZE", "0")
    ref = quantize(Xd, spec)
    monkeypatch.setenv("TMOG_HIP_QUANTIZE", "1")
    got = quantize(Xd, spec)
    assert torch.equal(got.cpu(), ref.cpu())
    assert _native_loaded()

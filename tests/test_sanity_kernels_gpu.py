"""SanityChecker statistics kernels (stats_kernels.hip) vs fp64 torch: stable column variance on large-offset
columns, the MFMA centred Gramian with the label block (correlations, contingency sums, counts), the
batched Spearman rank transform, and the SanityChecker fit on device vs host."""
import numpy as np
import pytest
import torch

from transmogrifai_amd.ops import stats as ST

pytestmark = pytest.mark.gpu


def _data(n=300_001, d=203, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, d, generator=g, dtype=torch.float64)
    X[:, 0] = X[:, 0] * 1e-3 + 1e6            # large offset, tiny spread
    X[:, 1] = 5.0                              # constant
    X[:, 2] = (torch.rand(n, generator=g) < 0.3).double()   # indicator
    X[:, 3] = X[:, 4] * 0.5 + 0.1 * X[:, 3]    # correlated pair
    return X.to(torch.float32)                 # the data as stored on the device


def test_col_stats_stable_variance():
    X = _data()
    ref = X.to(torch.float64)
    cs = ST.col_stats(X.cuda())
    var_ref = ref.var(0, unbiased=True)
    rel = ((cs["variance"].cpu() - var_ref).abs() / var_ref.clamp_min(1e-300))
    assert float(rel[0]) < 1e-9, float(rel[0])            # offset 1e6, std 1e-3 (cancellation case)
    assert float(rel[2:].max()) < 1e-9
    assert float(cs["variance"][1]) == 0.0
    torch.testing.assert_close(cs["mean"].cpu(), ref.mean(0), rtol=1e-12, atol=1e-9)
    torch.testing.assert_close(cs["min"].cpu(), ref.min(0).values)
    torch.testing.assert_close(cs["max"].cpu(), ref.max(0).values)


@pytest.mark.parametrize("n_labels", [2, 7])
def test_gram_corr_and_label_sums(n_labels):
    X = _data(d=300)
    g = torch.Generator().manual_seed(1)
    y = torch.randint(0, n_labels, (X.shape[0],), generator=g).to(torch.float32)
    ref = X.to(torch.float64)
    mean = ref.mean(0)
    C, lab, sums, cnt = ST.corr_and_label_sums(X.cuda(), y.cuda(), mean.cuda(), ref.min(0).values.cuda(),
                                               ref.max(0).values.cuda())
    Xc = ref - mean
    G = Xc.t() @ Xc
    sd = G.diag().sqrt()
    Cr = G / (sd[:, None] * sd[None, :])
    m = torch.isfinite(Cr)
    Cg = C.cpu()
    assert float((Cg[m] - Cr[m]).abs().max()) < 1e-6
    assert torch.isnan(Cg[1, 5]) and torch.isnan(Cg[5, 1])
    oh = torch.nn.functional.one_hot(y.long(), n_labels).double()
    torch.testing.assert_close(cnt.cpu(), oh.sum(0), rtol=0, atol=1e-6)
    sref = oh.t() @ ref
    err = (sums.cpu() - sref).abs()
    assert float(err[:, 1:3].max()) == 0.0          # constant / indicator columns: exact counts
    scale = oh.t() @ ref.abs()                        # fp32 accumulation error relative to sum |x|
    assert float((err / scale.clamp_min(1.0)).max()) < 1e-6
    np.testing.assert_array_equal(lab.cpu().numpy(), np.arange(n_labels, dtype=np.float64))


def test_gram_asymmetric_blocks():
    # exact small-integer data: any row/col swap in the C/D write shows up exactly
    g = torch.Generator().manual_seed(3)
    X = torch.randint(-3, 4, (4096, 261), generator=g).to(torch.float32)
    mean = torch.zeros(261, dtype=torch.float64)
    G = ST.gram_centered(X.cuda(), mean.cuda()).cpu()
    torch.testing.assert_close(G, X.double().t() @ X.double(), rtol=0, atol=0)


def test_spearman_batched_ranks():
    g = torch.Generator().manual_seed(4)
    X = torch.randint(0, 20, (5000, 300), generator=g).to(torch.float64)     # many ties
    R = ST._rank_columns(X.cuda()).cpu()
    for j in (0, 17, 299):
        v = X[:, j].numpy()
        from scipy.stats import rankdata
        np.testing.assert_allclose(R[:, j].numpy(), rankdata(v, method="average"))


def test_sanity_checker_device_matches_host():
    from transmogrifai_amd.testkit.synthetic import binary_table
    from transmogrifai_amd.dsl import transmogrify
    from transmogrifai_amd.workflow.workflow import OpWorkflow
    from transmogrifai_amd.readers.base import InMemoryReader
    from transmogrifai_amd import uid
    outs = []
    ds_host, _, _ = binary_table(50_000, n_real=12, n_int=3, n_pick=4, seed=3, device="cpu")
    for dev in ("cpu", "cuda"):
        uid.reset(0)
        _, label, preds = binary_table(10, n_real=12, n_int=3, n_pick=4, seed=3, device="cpu")
        ds = ds_host.to(dev)        # the same table on both devices (device RNG streams differ)
        vec = transmogrify(preds)
        checked = label.sanity_check(vec, remove_bad_features=True)
        model = OpWorkflow().set_result_features(checked).set_reader(InMemoryReader(ds)).train()
        outs.append(model.get_origin_stage_of(checked).metadata["summary"])
    h, d = outs
    assert h["dropped"] == d["dropped"]
    ch = np.array([np.nan if v is None else v for v in h["correlationsWLabel"]["values"]], float)
    cd = np.array([np.nan if v is None else v for v in d["correlationsWLabel"]["values"]], float)
    np.testing.assert_allclose(cd, ch, rtol=1e-5, atol=1e-6)
    for a, b in zip(h["categoricalStats"], d["categoricalStats"]):
        np.testing.assert_allclose(b["cramersV"], a["cramersV"], rtol=1e-6, atol=1e-9)


def test_class_column_sums_and_naive_bayes_on_device():
    g = torch.Generator().manual_seed(8)
    n, d = 70_001, 150
    X = (torch.rand(n, d, generator=g) * 3).floor().to(torch.float32)
    codes = torch.randint(-1, 4, (3, n), generator=g).to(torch.int32)
    ref = ST.class_column_sums(X, codes, 4)
    got = ST.class_column_sums(X.cuda(), codes.cuda(), 4).cpu()
    torch.testing.assert_close(got, ref, rtol=0, atol=0)        # integer data: exact
    from transmogrifai_amd.models.base import FitJob
    from transmogrifai_amd.models.linear import NaiveBayesLearner
    y = torch.randint(0, 3, (n,), generator=g).to(torch.float32)
    jobs = [FitJob({"smoothing": 1.0}, torch.arange(0, n, 2)), FitJob({"smoothing": 0.5}, torch.arange(1, n, 3))]
    sh = NaiveBayesLearner().fit_batch(X, y, jobs)
    sd = NaiveBayesLearner().fit_batch(X.cuda(), y.cuda(), [FitJob(j.params, j.rows.cuda()) for j in jobs])
    for a, b in zip(sh, sd):
        np.testing.assert_allclose(b["theta"], a["theta"], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(b["pi"], a["pi"], rtol=1e-12, atol=1e-12)


def test_bf16_gramian_fp32_accuracy_vs_fp64():
    """The default (bf16 three-part) centred Gramian at fp32-accumulation accuracy against the fp64 Gramian of the
    stored fp32 data centred on the fp64 mean, including a column with a large offset and a tiny spread (ADVICE r5:
    not bit-identical to the fp32 kernel, so its error is bounded explicitly). Each entry's error is measured
    against the magnitudes the kernel sums: sum |b_i| |b_j| with the bf16-exact columns raw (they are corrected
    for the mean afterwards, in fp64) and the others centred. The fp32 MFMA kernel (TMOG_GRAM_BF16=0) centres on
    the fp32-rounded mean: it is held to the same bound against that centring."""
    X = _data(n=200_003, d=150)
    g = torch.Generator().manual_seed(5)
    # large offset, small spread that fp32 still resolves (ulp at 1e4 ~ 1e-3)
    X[:, 0] = (1e4 + 1e-2 * torch.randn(X.shape[0], generator=g, dtype=torch.float64)).to(torch.float32)
    y = torch.randint(0, 3, (X.shape[0],), generator=g)
    ref = X.to(torch.float64)
    mean = ref.mean(0)
    oh = torch.nn.functional.one_hot(y, 3).double()
    A = torch.cat([ref - mean, oh], 1)
    Gref = A.t() @ A
    Xd = X.cuda()
    exact = ST.bf16_exact_columns(Xd).cpu()
    Bm = torch.cat([torch.where(exact[None, :], ref, ref - mean), oh], 1).abs()
    scale = Bm.t() @ Bm
    Gb = ST._gram_centered_bf16(Xd, mean.cuda(), y.cuda(), 3).cpu()
    eb = (Gb - Gref).abs() / scale.clamp_min(1e-30)
    assert float(eb.max()) < 2e-6, float(eb.max())
    # the offset column: the variance of a 1e4 + 1e-2 N(0, 1) column survives the centring
    assert float(Gref[0, 0]) > 0
    torch.testing.assert_close(Gb[0, 0], Gref[0, 0], rtol=1e-5, atol=0)
    # the fp32 kernel against its own (fp32-mean) centring
    mu32 = mean.to(torch.float32)
    A32 = torch.cat([ref - mu32.double(), oh], 1)
    G32 = A32.t() @ A32
    Gf = torch.empty_like(Gref).cuda()
    from transmogrifai_amd.ops import _native as N
    mu_d, y_d = mu32.cuda(), y.cuda().to(torch.int32)       # (kept alive until the kernel has read them)
    N.check(N.hip().tmog_hip_gram_aug(N.ptr(Xd), X.shape[0], X.shape[1], Xd.stride(0), N.ptr(mu_d), N.ptr(y_d), 3,
                                      N.ptr(Gf), N.stream(Xd.device)), "gram_aug")
    torch.cuda.synchronize()
    Aa = A32.abs()
    ef = (Gf.cpu() - G32).abs() / (Aa.t() @ Aa).clamp_min(1e-30)
    assert float(ef.max()) < 2e-6, float(ef.max())

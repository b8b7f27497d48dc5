"""bf16 packing pass (stats_kernels.hip bf16_pack_kernel) at the two shapes that use it: the multiclass-text
SanityChecker Gramian operand (1M x 1664: exact count / one-hot columns kept raw, 64 real columns as three bf16
parts, 6 label indicators) and the headline LR design copy (3.3M x 329). Prints ms per pass and the HBM bytes
moved per second (fp32 X read once, bf16 B written once)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from transmogrifai_amd.ops import linear as LK, stats as ST  # noqa: E402


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def gram_operand(n=1_000_000, d=1664, n_real=64, L=6):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    X = (torch.rand(n, d, generator=g, device=dev) < 0.05).float()
    real = torch.randperm(d, generator=g, device=dev)[:n_real].sort().values
    X[:, real] = torch.randn(n, n_real, generator=g, device=dev) * 7 + 3
    y = torch.randint(0, L, (n,), generator=g, device=dev, dtype=torch.int32)
    exact = ST.bf16_exact_columns(X)
    E, R = torch.nonzero(exact).reshape(-1), torch.nonzero(~exact).reshape(-1)
    nE, nR = int(E.numel()), int(R.numel())
    D = nE + 1 + 3 * nR + L
    lda = ((D + 127) // 128) * 128
    src = torch.cat([E, torch.zeros(1, dtype=torch.int64, device=dev), R, R, R, torch.arange(L, device=dev)])
    mode = torch.cat([torch.full((nE,), ST.PACK_RAW, device=dev), torch.full((1,), ST.PACK_ONE, device=dev),
                      torch.full((nR,), ST.PACK_HI, device=dev), torch.full((nR,), ST.PACK_MID, device=dev),
                      torch.full((nR,), ST.PACK_LO, device=dev), torch.full((L,), ST.PACK_LABEL, device=dev)])
    mu = torch.cat([torch.zeros(nE + 1, device=dev), X[:, R].mean(0).repeat(3), torch.zeros(L, device=dev)])
    sc = torch.ones(D, device=dev)
    t = timed(lambda: ST.bf16_pack(X, src, mode, mu, sc, lda, y=y))
    gb = (X.numel() * 4 + n * lda * 2) / 1e9
    B = ST.bf16_pack(X, src, mode, mu, sc, lda, y=y)
    ok = bool(torch.equal(B[:, :nE].float(), X[:, E])) and bool((B[:, nE] == 1).all())
    parts = B[:, nE + 1:nE + 1 + 3 * nR].float().reshape(n, 3, nR).sum(1)
    ok &= bool(torch.equal(parts, X[:, R] - mu[nE + 1:nE + 1 + nR]))
    ok &= bool(torch.equal(B[:, D - L:D].float().argmax(1).int(), y))
    print(f"gram operand {n} x {d} -> [{n}, {lda}] bf16: {t:.3f} ms, {gb / t * 1e3:.0f} GB/s, exact {ok}", flush=True)


def lr_design(n=3_300_000, d=329):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(1)
    X = torch.randn(n, d, generator=g, device=dev)
    X[:, : d // 2] = (X[:, : d // 2] > 0.5).float()
    t = timed(lambda: LK.Bf16Design(X), reps=5)
    D = LK.Bf16Design(X)
    gb = (X.numel() * 4 + D.Xb.numel() * 2) / 1e9
    print(f"LR design {n} x {d} -> {tuple(D.Xb.shape)} bf16 (exactness + moments + pack): {t:.3f} ms, "
          f"{gb / t * 1e3:.0f} GB/s", flush=True)


if __name__ == "__main__":
    gram_operand()
    lr_design()

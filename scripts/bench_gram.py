"""Micro-benchmark of the SanityChecker Gram kernel (ops/csrc/hip/stats_kernels.hip gram_aug_kernel):
python scripts/bench_gram.py [n] [d] [L]. Prints ms per call and the fp32-MFMA TFLOP/s of the upper-triangle tiles."""
import sys
import time

import torch

from transmogrifai_amd.ops import _native as N


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    d = int(sys.argv[2]) if len(sys.argv) > 2 else 1352
    L = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.rand(n, d, generator=g, device=dev)
    mu = X[:4096].mean(0).contiguous()
    y = torch.randint(0, max(L, 1), (n,), generator=g, device=dev, dtype=torch.int32)
    D = d + L
    G = torch.empty(D, D, dtype=torch.float64, device=dev)
    lib = N.hip()

    def run():
        N.check(lib.tmog_hip_gram_aug(N.ptr(X), n, d, X.stride(0), N.ptr(mu), N.ptr(y) if L else None, L, N.ptr(G),
                                      N.stream(dev)), "gram_aug")

    run()
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    nt = (D + 127) // 128
    flops = nt * (nt + 1) // 2 * 128 * 128 * 2.0 * n
    print(f"gram n={n} d={d} L={L}: {ms:.2f} ms, {flops / ms / 1e9:.1f} TFLOP/s (upper-triangle tiles)")
    ref = (X[:20000].double() - mu.double()).t() @ (X[:20000].double() - mu.double())
    G2 = torch.empty(d, d, dtype=torch.float64, device=dev)
    N.check(lib.tmog_hip_gram_aug(N.ptr(X), 20000, d, X.stride(0), N.ptr(mu), None, 0, N.ptr(G2), N.stream(dev)),
            "gram_aug")
    torch.cuda.synchronize()
    print("max rel err vs fp64 (20000 rows):", float(((G2 - ref).abs() / ref.abs().clamp_min(1)).max()))


if __name__ == "__main__":
    main()

"""Matrix-core row GEMMs (ops/dense.py) against torch's GEMMs (hipBLASLt / rocBLAS) on the learners' shapes:
the multinomial margins X V and gradient X^T R (1M x 400 design, 8 grid points x 10 classes), and an MLP batch
(8 jobs, hidden 10: the shared first layer with its bias + sigmoid, the weight gradient). Median of 20 timed calls
after 3 warm-ups, cuda events; prints one JSON line per case.

python scripts/bench_dense.py [--n 1000000] [--d 400]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _time(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=400)
    a = ap.parse_args()
    from transmogrifai_amd.ops import dense as DN
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.randn(a.n, a.d, device="cuda", generator=g)
    for M in (8, 80, 256):
        V = torch.randn(a.d, M, device="cuda", generator=g)
        R = torch.randn(a.n, M, device="cuda", generator=g)
        ours = _time(lambda: DN.mm(X, V))
        lib = _time(lambda: X @ V)
        ours_t = _time(lambda: DN.tmm(X, R))
        lib_t = _time(lambda: (X.t() @ R).double())
        gb = a.n * a.d * 4 / 1e9
        print(json.dumps({"case": f"mm N={a.n} K={a.d} M={M}", "mfma_ms": round(ours, 3), "torch_ms": round(lib, 3),
                          "mfma_TBps_of_X": round(gb / ours, 2)}), flush=True)
        print(json.dumps({"case": f"tmm N={a.n} K={a.d} M={M}", "mfma_ms": round(ours_t, 3),
                          "torch_ms": round(lib_t, 3), "mfma_TBps_of_X": round(gb / ours_t, 2)}), flush=True)
    P, h = 8, 10
    W = torch.randn(P, a.d, h, device="cuda", generator=g)
    b = torch.randn(P, h, device="cuda", generator=g)
    dZ = torch.randn(P, a.n, h, device="cuda", generator=g)
    ours = _time(lambda: DN.layer_shared(X, W, b, True))
    lib = _time(lambda: torch.sigmoid(torch.matmul(X, W) + b[:, None, :]))
    print(json.dumps({"case": f"mlp layer0 fwd P={P} hidden={h}", "mfma_ms": round(ours, 3), "torch_ms": round(lib, 3)}),
          flush=True)
    ours = _time(lambda: DN.grad_shared(X, dZ))
    lib = _time(lambda: torch.matmul(X.t(), dZ).double())
    print(json.dumps({"case": f"mlp layer0 dW P={P} hidden={h}", "mfma_ms": round(ours, 3), "torch_ms": round(lib, 3)}),
          flush=True)


if __name__ == "__main__":
    main()

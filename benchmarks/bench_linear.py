"""Micro-benchmark of one batched linear-model objective evaluation (value + gradient).

Shapes of the headline configuration's logistic-regression grid: ``--rows`` training rows (the CV
union), ``--cols`` vectorized columns, ``--problems`` = 8 configs x 3 folds. Compares the fused HIP
kernel (``ops/csrc/hip/linear_kernels.hip``) with the two-GEMM torch path. Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from transmogrifai_amd.ops import linear as LK  # noqa: E402


def _timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return 1000 * (time.perf_counter() - t0) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=700_000)
    ap.add_argument("--cols", type=int, default=329)
    ap.add_argument("--problems", type=int, default=24)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(a.rows, a.cols, device=dev, generator=g)
    y = (torch.rand(a.rows, device=dev, generator=g) < 0.4).float()
    W = (torch.rand(a.rows, a.problems, device=dev, generator=g) < 0.67).float()
    V = torch.randn(a.cols, a.problems, device=dev, generator=g) / a.cols ** 0.5
    b = torch.zeros(a.problems, device=dev)

    def torch_path():
        M = X @ V + b[None, :]
        l = torch.nn.functional.softplus(M) - y[:, None] * M
        R = (torch.sigmoid(M) - y[:, None]) * W
        return (l * W).sum(0), R.sum(0), X.t() @ R

    res = {
        "bench": "linear_objective", "rows": a.rows, "cols": a.cols, "problems": a.problems,
        "fused_value_grad_ms": _timeit(lambda: LK.fused_objective(X, y, W, V, b, "logistic", grad=True), a.reps),
        "fused_value_ms": _timeit(lambda: LK.fused_objective(X, y, W, V, b, "logistic", grad=False), a.reps),
        "torch_value_grad_ms": _timeit(torch_path, a.reps),
        "x_bytes": X.numel() * 4,
    }
    res["fused_vg_hbm_tb_s"] = res["x_bytes"] / (res["fused_value_grad_ms"] * 1e-3) / 1e12
    print(json.dumps(res))


if __name__ == "__main__":
    main()

"""Micro-benchmark of the fused linear objective (ops/linear.py fused_objective, linear_kernels.hip) at the
headline LR shape: python scripts/bench_lr_obj.py [N] [d] [P]. Prints ms per pass and the X stream rate."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from transmogrifai_amd.ops import linear as LK  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 330
P = int(sys.argv[3]) if len(sys.argv) > 3 else 32
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(N, d, device=dev, generator=g)
y = (torch.rand(N, device=dev, generator=g) < 0.4).float()
W = (torch.rand(N, P, device=dev, generator=g) < 0.67).float()
V = torch.randn(d, P, device=dev, generator=g) / d ** 0.5
b = torch.zeros(P, device=dev)
for grad in (False, True):
    for _ in range(3):
        LK.fused_objective(X, y, W, V, b, "logistic", None, grad=grad)
    torch.cuda.synchronize()
    n = 30
    t0 = time.perf_counter()
    for _ in range(n):
        LK.fused_objective(X, y, W, V, b, "logistic", None, grad=grad)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / n * 1e3
    gb = (X.numel() * 4 + W.numel() * 4) / 1e9
    print(f"N={N} d={d} P={P} grad={grad}: {ms:.3f} ms/pass, {gb / ms:.2f} TB/s (X + W bytes)", flush=True)

"""Linear objective passes at the headline's LR shape (python scripts/bench_lr_kernel.py [rows] [cols] [problems]):
fp32 lr_objective_kernel vs bf16 lr_bf16_kernel, value and gradient passes, timed with device events; reports
ms per pass and the design-matrix bytes streamed per second (X once per pass; W / y on top)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from transmogrifai_amd.ops import linear as LK  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 3_300_000
    d = int(sys.argv[2]) if len(sys.argv) > 2 else 329
    P = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    torch.manual_seed(0)
    X = torch.randn(N, d, device="cuda")
    X[:, : d // 2] = (X[:, : d // 2] > 0.5).float()          # the one-hot / indicator half of a transmogrified matrix
    y = (torch.rand(N, device="cuda") < 0.3).float()
    Wu = (torch.rand(N, 4, device="cuda") < 0.67).float()
    cols = [p % 4 for p in range(P)]
    W = Wu[:, cols].contiguous()
    V = 0.05 * torch.randn(d, P, device="cuda")
    b = 0.1 * torch.randn(P, device="cuda")
    D = LK.Bf16Design(X)
    wmap = LK.weight_map(cols, P, X.device)
    print(f"N={N} d={d} P={P}  bf16 design {D.Xb.numel() * 2 / 1e9:.2f} GB ({D.n_exact} exact columns), "
          f"fp32 X {X.numel() * 4 / 1e9:.2f} GB", flush=True)
    for grad in (False, True):
        t32 = timed(lambda: LK.fused_objective(X, y, W, V, b, "logistic", grad=grad))
        t16 = timed(lambda: LK.fused_objective_bf16(D, y, Wu, V, b, "logistic", grad=grad, wmap=wmap))
        kind = "gradient" if grad else "value"
        print(f"{kind:8s} fp32 {t32:7.3f} ms ({X.numel() * 4 / t32 / 1e6:6.0f} GB/s of X)   "
              f"bf16 {t16:7.3f} ms ({D.Xb.numel() * 2 / t16 / 1e6:6.0f} GB/s of X)   x{t32 / t16:.2f}", flush=True)


if __name__ == "__main__":
    main()

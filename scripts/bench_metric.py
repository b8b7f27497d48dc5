"""Selection-metric microbenchmark: exact AuPR of J score sets over n validation rows (the RF grid's 18 x 3 folds
on the headline: J = 18 per fold, n = 333K), per-model torch curves vs the batched HIP curve kernel."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from transmogrifai_amd.evaluators import metrics as M


def main():
    for J, n, ties in ((18, 333_333, 0), (18, 333_333, 51), (8, 333_333, 0), (18, 3_300_000, 0), (8, 3_300_000, 0)):
        g = torch.Generator().manual_seed(1)
        S = torch.rand(J, n, generator=g, dtype=torch.float64)
        if ties:
            S = torch.round(S * ties) / ties
        y = (torch.rand(n, generator=g) < 0.3).to(torch.float64)
        S, y = S.cuda(), y.cuda()
        for name, fn in (("per-model", lambda: [M.binary_curves(S[j], y, 0)["AuPR"] for j in range(J)]),
                         ("device", lambda: M.binary_areas_device(S, y)[0].tolist())):
            fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                out = fn()
            torch.cuda.synchronize()
            print(f"J={J} n={n} ties={ties} {name}: {(time.perf_counter() - t0) / 5 * 1e3:.2f} ms "
                  f"(first {out[0]:.12f})", flush=True)


if __name__ == "__main__":
    main()

"""In-process A/B of the XGBoost phase at headline-like shapes (1M rows, 190 dense + 330 sparse 0/1
columns, 6 jobs = 2 grid points x 3 folds of 667K rows, 200 rounds, depth 10, eta 0.02, early stopping 20):
alternates environment settings so box-to-box and warm-up noise cancel.
usage: python xgb_ab.py "A_ENV=1" "A_ENV=0" [reps]"""
import os
import sys
import time

import torch

sys.path.insert(0, ".")
from transmogrifai_amd.models.base import FitJob  # noqa: E402
from transmogrifai_amd.models.trees import XGBoostClassifierLearner  # noqa: E402

dev = torch.device("cuda")
N, Fd, Fs = 1_000_000, 190, 330
g = torch.Generator(device=dev).manual_seed(0)
X = torch.cat([torch.randn(N, Fd, device=dev, generator=g),
               (torch.rand(N, Fs, device=dev, generator=g) < 0.05).float()], 1)
w = torch.randn(Fd + Fs, device=dev, generator=g) * (torch.rand(Fd + Fs, device=dev, generator=g) < 0.2)
y = ((X @ w + torch.randn(N, device=dev, generator=g) * 2) > 0).float()
folds = [torch.randperm(N, device=dev, generator=g)[:667_000].sort().values for _ in range(3)]
L = XGBoostClassifierLearner()
jobs = [FitJob(dict(L.defaults, num_round=200, eta=0.02, max_depth=10, min_child_weight=m, gamma=0.0,
                    num_early_stopping_rounds=20, missing=0.0, max_bins=32), folds[k])
        for m in (1.0, 10.0) for k in range(3)]
settings = sys.argv[1:3]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
ctx = {}
L.fit_batch(X, y, [FitJob(dict(jobs[0].params, num_round=3), folds[0])], context=ctx)   # warm-up + binning
res = {s: [] for s in settings}
for r in range(reps):
    for s in settings:
        k, v = s.split("=", 1)
        old = os.environ.get(k)
        os.environ[k] = v
        torch.cuda.synchronize()
        t = time.perf_counter()
        out = L.fit_batch(X, y, jobs, context=ctx)
        torch.cuda.synchronize()
        res[s].append(time.perf_counter() - t)
        if old is None:
            del os.environ[k]
        else:
            os.environ[k] = old
        print(s, round(res[s][-1], 3), [o["num_trees"] for o in out], flush=True)
for s in settings:
    print("RESULT", s, "min", round(min(res[s]), 3), "mean", round(sum(res[s]) / len(res[s]), 3))

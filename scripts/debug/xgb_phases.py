"""Debug: time the phases of the XGBoost boosting loop at the headline shapes (GPU)."""
import sys
import time
import numpy as np
import torch
sys.path.insert(0, ".")
from transmogrifai_amd.models import trees as TR, tree_engine as TE
from transmogrifai_amd.models.base import FitJob

dev = torch.device("cuda")
N, F, rounds = 2_000_000, 329, int(sys.argv[1]) if len(sys.argv) > 1 else 30
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(N, F, device=dev, generator=g)
y = ((X[:, 0] + X[:, 1] - X[:, 2] + torch.randn(N, device=dev, generator=g)) > 0).double()
folds = [torch.randperm(N, device=dev, generator=g)[:667_000].sort().values for _ in range(3)]
acc = {}
orig_grow = TE.grow_forest
orig_add = TR._add_tree_margins


def timed(name, fn):
    def w(*a, **k):
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = fn(*a, **k)
        torch.cuda.synchronize()
        acc[name] = acc.get(name, 0.0) + time.perf_counter() - t
        return r
    return w


TE.grow_forest = timed("grow_forest", orig_grow)
TR._add_tree_margins = timed("add_margins", orig_add)
from transmogrifai_amd.evaluators import metrics as M
M.binned_aupr_multi = timed("aupr", M.binned_aupr_multi)
learner = TR.XGBoostClassifierLearner() if hasattr(TR, "XGBoostClassifierLearner") else None
if learner is None:
    from transmogrifai_amd.models.base import learner_class
    learner = learner_class("OpXGBoostClassifier")()
jobs = [FitJob(dict(learner.defaults, num_round=rounds, eta=0.02, max_depth=10, min_child_weight=mcw, gamma=0.8,
                    num_early_stopping_rounds=20, missing=0.0), folds[k]) for mcw in (1.0, 10.0) for k in range(3)]
ctx = {}
learner.fit_batch(X, y, jobs[:1] and [FitJob(dict(jobs[0].params, num_round=2), folds[0])], context=ctx)  # warm
acc.clear()
torch.cuda.synchronize()
t0 = time.perf_counter()
learner.fit_batch(X, y, jobs, context=ctx)
torch.cuda.synchronize()
tot = time.perf_counter() - t0
print({"rounds": rounds, "total_s": round(tot, 3), "per_round_ms": round(1000 * tot / rounds, 2),
       **{k: round(1000 * v / rounds, 2) for k, v in acc.items()}})

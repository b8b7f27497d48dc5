"""Micro-benchmark of the histogram tree engine in the headline configuration's shapes.

XGBoost-style Newton trees (``MODE_GH``): ``--trees`` trees per round (2 configs x 3 folds = 6 in the default
binary grid), depth ``--depth``, ``--bins`` bins, ``--rows`` training rows per tree over a shared
``--pool``-row binned matrix with ``--feats`` features. Random forest mode (``--rf``) grows ``--trees``
bootstrap trees with sqrt(F) feature subsets per node. Prints one JSON line with ms per round.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from transmogrifai_amd.models import tree_engine as TE  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pool", type=int, default=1_800_000)
    ap.add_argument("--rows", type=int, default=667_000)
    ap.add_argument("--feats", type=int, default=300)
    ap.add_argument("--bins", type=int, default=64)
    ap.add_argument("--trees", type=int, default=6)
    ap.add_argument("--depth", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--rf", action="store_true")
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()
    dev = torch.device(a.device if torch.cuda.is_available() else "cpu")
    g = torch.Generator(device=dev).manual_seed(0)
    Xb = torch.randint(0, a.bins, (a.pool, a.feats), dtype=torch.uint8, device=dev, generator=g)
    sig = (Xb[:, 0].float() + Xb[:, 1].float() - Xb[:, 2].float()) / a.bins
    y = (torch.rand(a.pool, device=dev, generator=g) < torch.sigmoid(3 * (sig - 0.5))).float()
    jobs_rows = [torch.randperm(a.pool, device=dev, generator=g)[:a.rows].sort().values for _ in range(a.trees)]
    nb = np.full(a.feats, a.bins, np.int64)
    times = []
    for r in range(a.rounds + 1):
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        if a.rf:
            sub = int(math.ceil(math.sqrt(a.feats)))
            jobs = [TE.TreeJob(0, TE.TreeParams(max_depth=a.depth, min_instances=10, min_info_gain=0.001,
                                                feature_subset=sub), rr,
                               torch.poisson(torch.ones(rr.numel(), device=dev)).to(torch.int64), 7 + t)
                    for t, rr in enumerate(jobs_rows)]
            f = TE.grow_forest(Xb, nb, jobs, mode=TE.MODE_CLS, kind=TE.KIND_GINI, n_classes=2, y=y, B=a.bins)
        else:
            G = torch.randn(a.trees, a.pool, device=dev, generator=g)
            H = torch.rand(a.trees, a.pool, device=dev, generator=g) * 0.25
            jobs = [TE.TreeJob(t, TE.TreeParams(max_depth=a.depth, min_child_weight=1.0, reg_lambda=1.0, gamma=0.8,
                                                split_eps=1e-6), rr) for t, rr in enumerate(jobs_rows)]
            f = TE.grow_forest(Xb, nb, jobs, mode=TE.MODE_GH, kind=TE.KIND_NEWTON, t1=G, t2=H, B=a.bins)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        if r > 0:
            times.append(time.perf_counter() - t0)
    print(json.dumps({"bench": "trees", "mode": "rf" if a.rf else "gh", "ms_per_round": 1000 * float(np.median(times)),
                      "nodes": int(len(f.nodes)), "pool": a.pool, "rows": a.rows, "feats": a.feats, "bins": a.bins,
                      "trees": a.trees, "depth": a.depth}))


if __name__ == "__main__":
    main()

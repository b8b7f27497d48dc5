"""Debug: CPU vs GPU tree parity with feature subsets under 1 or 2 job groups."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from tests.test_tree_engine import _data
from transmogrifai_amd.models import tree_engine as te


def grow(dev, groups, subset=4):
    X, y = _data()
    N = X.shape[0]
    g = torch.Generator().manual_seed(1)
    jobs = []
    for m in range(2):
        rows = torch.arange(N)[torch.arange(N) % (m + 2) != 0]
        w = torch.randint(0, 3, (rows.numel(),), generator=g)
        jobs.append(te.TreeJob(m, te.TreeParams(max_depth=6, min_instances=2, feature_subset=subset),
                               rows.to(dev), w.to(dev)))
    f = te.grow_forest(X.to(dev), np.full(X.shape[1], 32), jobs, mode=te.MODE_CLS, kind=te.KIND_GINI,
                       y=y.to(dev), B=32, rng_seed=3, chunk_rows=512, groups=groups)
    return f


for groups in (1, 2):
    for subset in (None, 4):
        a, b = grow("cpu", groups, subset), grow("cuda", groups, subset)
        same = a.nodes.shape == b.nodes.shape and bool((a.nodes == b.nodes).all())
        print("groups", groups, "subset", subset, "match", same, a.nodes.shape, b.nodes.shape)
        if not same and a.nodes.shape == b.nodes.shape:
            d = np.nonzero((a.nodes != b.nodes).any(1))[0]
            print("  first diffs", d[:5], a.nodes[d[:3]].tolist(), b.nodes[d[:3]].tolist())

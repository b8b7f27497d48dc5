"""Debug: run the CLS+subset parity case of tests/test_tree_engine.py a few times in one process."""
import sys
import numpy as np
sys.path.insert(0, ".")
from tests.test_tree_engine import _grow_all
from transmogrifai_amd.models import tree_engine as te

fc, _ = _grow_all("cpu", te.MODE_CLS, False, 4)
for i in range(4):
    fg, _ = _grow_all("cuda", te.MODE_CLS, False, 4)
    same = fc.nodes.shape == fg.nodes.shape and bool((fc.nodes == fg.nodes).all())
    print(i, "match", same, fc.nodes.shape, fg.nodes.shape, flush=True)
    if not same and fc.nodes.shape == fg.nodes.shape:
        d = np.nonzero((fc.nodes != fg.nodes).any(1))[0]
        print("  diffs at", d[:8].tolist(), fc.nodes[d[:2]].tolist(), fg.nodes[d[:2]].tolist())
        print("  gains", fc.gain[d[:4]].tolist(), fg.gain[d[:4]].tolist())
fc2, _ = _grow_all("cpu", te.MODE_CLS, False, 4)
print("cpu deterministic", bool((fc.nodes == fc2.nodes).all()))

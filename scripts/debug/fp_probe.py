"""Probe: forced 1-rank feature-parallel growth on one GPU (RCCL exchange path); prints OK or crashes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import torch  # noqa: E402
import test_learner_parallel as T  # noqa: E402

T._fp_one_rank(torch.device("cuda"))
print("FP OK groups=", os.environ.get("TMOG_TREE_GROUPS"), flush=True)

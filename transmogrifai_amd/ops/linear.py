"""Dense linear-algebra entry points used by the learners and statistics.

``gemm``/``gemm_t`` are the two halves of every linear-model iteration (``M = X V`` and
``G = X^T R``); on device they run on the matrix cores (hipBLASLt via torch for these plain
library-shaped GEMMs, fp32 in / fp32 accumulate), on the host through BLAS.
"""
from __future__ import annotations

import torch


def gemm(X: torch.Tensor, V: torch.Tensor) -> torch.Tensor:
    """``X [N, d] @ V [d, P]`` in X's dtype."""
    return X @ V.to(X.dtype)


def gemm_t(X: torch.Tensor, R: torch.Tensor) -> torch.Tensor:
    """``X^T [d, N] @ R [N, P]`` in X's dtype."""
    return X.t() @ R.to(X.dtype)

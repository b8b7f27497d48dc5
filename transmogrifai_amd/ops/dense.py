"""Dense fp32 row GEMMs on the matrix cores (``ops/csrc/hip/dense_kernels.hip``): the products of the
multinomial / linear objectives and of the MLP.

* :func:`mm` -- ``X [N, K] @ V [K, M]`` (fp32 out);
* :func:`tmm` -- ``X^T [K, N] @ R [N, M]`` (fp64 out: fp32 MFMA inside a row chunk, fp64 across chunks);
* the MLP's layer products over P jobs at once: :func:`layer_shared` (one shared input, the jobs' weight matrices
  as grouped columns -- the input streamed once per 64-column tile), :func:`layer_batched` (per-job inputs),
  :func:`backprop_input` (``dZ_p W_p^T``), :func:`grad_shared` / :func:`grad_batched` (weight gradients), each with
  the bias + sigmoid epilogue fused where the layer has one.

Every entry point checks on the host that the operands are contiguous fp32 device tensors of the shapes the
kernel's indexing assumes before it launches; :func:`supported` tells callers when the kernels apply.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

_TARGET_BLOCKS = 2048


def enabled() -> bool:
    """``TMOG_DENSE_MFMA=1`` routes the learners' plain dense products through these kernels. Default off: on
    MI355X hipBLASLt measured faster on every learner shape (``profiles/r6e_bench_dense.log``: X V at
    1M x 400 0.40 / 0.70 / 1.67 ms vs 1.81 / 3.53 / 7.00 ms here for 8 / 80 / 256 columns, X^T R 1.37 / 2.16 /
    4.54 vs 1.66 / 3.14 / 6.12 ms, the MLP layer products 3.1 / 2.8 vs 3.6 / 3.1 ms), and the end-to-end
    multiclass-text step is the same either way (1.128 vs 1.119 s, identical hold-out error). These are plain
    GEMMs, the library's case; the kernels stay tested (tests/test_dense_gemm_gpu.py) and selectable."""
    return os.environ.get("TMOG_DENSE_MFMA", "0") == "1"


def supported(*ts: torch.Tensor) -> bool:
    return all(t.is_cuda and t.dtype == torch.float32 for t in ts)


def _c(t: torch.Tensor) -> torch.Tensor:
    return t if t.is_contiguous() else t.contiguous()


def _check(cond: bool, what: str):
    if not cond:
        raise ValueError(f"dense GEMM operand check failed: {what}")


def _rowgemm(A, lda, a_ps, B, ldb, b_ps, btrans, bg, b_gs, bias, bias_ps, bias_gs, C, ldc, c_ps, cg, c_gs, N, K, M, P,
             epi):
    from . import _native as N_
    N_.check(N_.hip().tmog_hip_rowgemm(N_.ptr(A), lda, a_ps, N_.ptr(B), ldb, b_ps, int(btrans), bg, b_gs,
                                       N_.ptr(bias) if bias is not None else None, bias_ps, bias_gs, N_.ptr(C), ldc,
                                       c_ps, cg, c_gs, N, K, M, P, epi, N_.stream(C.device)), "rowgemm")


def _xtd(A, lda, a_ps, D, ldd, d_ps, dg, d_gs, N, K, M, P) -> torch.Tensor:
    from . import _native as N_
    lib = N_.hip()
    S = int(lib.tmog_hip_xtd_chunks(N, K, M, P, _TARGET_BLOCKS))
    part = torch.empty(S * P * K * M, dtype=torch.float32, device=A.device)
    out = torch.empty(P, K, M, dtype=torch.float64, device=A.device)
    N_.check(lib.tmog_hip_xtd(N_.ptr(A), lda, a_ps, N_.ptr(D), ldd, d_ps, dg, d_gs, N, K, M, P, S, N_.ptr(part),
                              N_.ptr(out), N_.stream(A.device)), "xtd")
    return out


def mm(X: torch.Tensor, V: torch.Tensor, bias: Optional[torch.Tensor] = None, sigmoid: bool = False) -> torch.Tensor:
    """``X [N, K] @ V [K, M] (+ bias [M])`` (optionally through a sigmoid), fp32."""
    X, V = _c(X), _c(V)
    _check(X.dim() == 2 and V.dim() == 2 and X.shape[1] == V.shape[0], f"X {tuple(X.shape)} V {tuple(V.shape)}")
    N, K = X.shape
    M = V.shape[1]
    if bias is not None:
        bias = _c(bias.to(torch.float32))
        _check(bias.numel() == M, "bias size")
    out = torch.empty(N, M, dtype=torch.float32, device=X.device)
    _rowgemm(X, K, 0, V, M, 0, False, M, 0, bias, 0, 0, out, M, 0, M, 0, N, K, M, 1, int(sigmoid))
    return out


def tmm(X: torch.Tensor, R: torch.Tensor) -> torch.Tensor:
    """``X^T [K, N] @ R [N, M]`` in fp64."""
    X, R = _c(X), _c(R)
    _check(X.dim() == 2 and R.dim() == 2 and X.shape[0] == R.shape[0], f"X {tuple(X.shape)} R {tuple(R.shape)}")
    N, K = X.shape
    M = R.shape[1]
    return _xtd(X, K, 0, R, M, 0, M, 0, N, K, M, 1)[0]


def layer_shared(X: torch.Tensor, W: torch.Tensor, bias: Optional[torch.Tensor], sigmoid: bool) -> torch.Tensor:
    """``out[p] = act(X [N, K] @ W[p] [K, g] + bias[p])`` for the P jobs -> ``[P, N, g]``; one launch, the jobs'
    columns grouped (X streamed once per 64 output columns)."""
    X, W = _c(X), _c(W)
    _check(X.dim() == 2 and W.dim() == 3 and W.shape[1] == X.shape[1], f"X {tuple(X.shape)} W {tuple(W.shape)}")
    N, K = X.shape
    P, _, g = W.shape
    if bias is not None:
        bias = _c(bias)
        _check(tuple(bias.shape) == (P, g), "bias shape")
    out = torch.empty(P, N, g, dtype=torch.float32, device=X.device)
    _rowgemm(X, K, 0, W, g, 0, False, g, K * g, bias, 0, g, out, g, 0, g, N * g, N, K, P * g, 1, int(sigmoid))
    return out


def layer_batched(H: torch.Tensor, W: torch.Tensor, bias: Optional[torch.Tensor], sigmoid: bool) -> torch.Tensor:
    """``out[p] = act(H[p] [N, a] @ W[p] [a, b] + bias[p])`` -> ``[P, N, b]``."""
    H, W = _c(H), _c(W)
    _check(H.dim() == 3 and W.dim() == 3 and H.shape[0] == W.shape[0] and H.shape[2] == W.shape[1],
           f"H {tuple(H.shape)} W {tuple(W.shape)}")
    P, N, a = H.shape
    b = W.shape[2]
    if bias is not None:
        bias = _c(bias)
        _check(tuple(bias.shape) == (P, b), "bias shape")
    out = torch.empty(P, N, b, dtype=torch.float32, device=H.device)
    _rowgemm(H, a, N * a, W, b, a * b, False, b, 0, bias, b, 0, out, b, N * b, b, 0, N, a, b, P, int(sigmoid))
    return out


def backprop_input(dZ: torch.Tensor, W: torch.Tensor) -> torch.Tensor:
    """``dH[p] = dZ[p] [N, b] @ W[p]^T [b, a]`` -> ``[P, N, a]`` (W read transposed in place)."""
    dZ, W = _c(dZ), _c(W)
    _check(dZ.dim() == 3 and W.dim() == 3 and dZ.shape[0] == W.shape[0] and dZ.shape[2] == W.shape[2],
           f"dZ {tuple(dZ.shape)} W {tuple(W.shape)}")
    P, N, b = dZ.shape
    a = W.shape[1]
    out = torch.empty(P, N, a, dtype=torch.float32, device=dZ.device)
    _rowgemm(dZ, b, N * b, W, b, a * b, True, a, 0, None, 0, 0, out, a, N * a, a, 0, N, b, a, P, 0)
    return out


def grad_shared(X: torch.Tensor, dZ: torch.Tensor) -> torch.Tensor:
    """``G[p] = X^T [K, N] @ dZ[p] [N, g]`` -> ``[P, K, g]`` fp64 (one launch over the grouped columns)."""
    X, dZ = _c(X), _c(dZ)
    _check(X.dim() == 2 and dZ.dim() == 3 and dZ.shape[1] == X.shape[0], f"X {tuple(X.shape)} dZ {tuple(dZ.shape)}")
    N, K = X.shape
    P, _, g = dZ.shape
    G = _xtd(X, K, 0, dZ, g, 0, g, N * g, N, K, P * g, 1)[0]          # [K, P * g]
    return G.view(K, P, g).permute(1, 0, 2)


def grad_batched(H: torch.Tensor, dZ: torch.Tensor) -> torch.Tensor:
    """``G[p] = H[p]^T [a, N] @ dZ[p] [N, b]`` -> ``[P, a, b]`` fp64."""
    H, dZ = _c(H), _c(dZ)
    _check(H.dim() == 3 and dZ.dim() == 3 and H.shape[:2] == dZ.shape[:2], f"H {tuple(H.shape)} dZ {tuple(dZ.shape)}")
    P, N, a = H.shape
    b = dZ.shape[2]
    return _xtd(H, a, N * a, dZ, b, N * b, b, 0, N, a, b, P)

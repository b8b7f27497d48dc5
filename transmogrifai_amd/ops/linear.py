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


LOSS_CODES = {"logistic": 0, "hinge": 1, "squared": 2}
_LR_DMAX = 384          # one-pass kernel: 64-row X tile + V resident in LDS
_LR_WIDE_DMAX = 2048    # wide kernel: library GEMM margins + fused epilogue / MFMA gradient
_LR_PC = 32


def fused_objective_supported(X: torch.Tensor) -> bool:
    """The fused HIP objective handles fp32 ``X`` on the GPU with ``d <= 2048`` columns (one pass over X
    up to 384 columns, a library GEMM plus one fused pass above)."""
    return X.is_cuda and X.dtype == torch.float32 and X.dim() == 2 and 1 <= X.shape[1] <= _LR_WIDE_DMAX \
        and X.is_contiguous()


def _n_blocks(N: int) -> int:
    # persistent workgroups: one per CU (the 64-row tile + V fill ~150 KB of the 160 KB LDS)
    props = torch.cuda.get_device_properties(torch.cuda.current_device())
    return max(1, min((N + 63) // 64, props.multi_processor_count))


def fused_objective(X: torch.Tensor, y: torch.Tensor, W: torch.Tensor, V: torch.Tensor, bias: torch.Tensor,
                    loss: str, yscale=None, grad: bool = True):
    """One pass of the fused HIP objective (``ops/csrc/hip/linear_kernels.hip``) for P problems.

    ``m = X V + bias``; returns ``(f [P], r [P], G [d, P] or None)`` in fp64 with ``f = sum_i W l(m)``,
    ``r = sum_i W l'(m)``, ``G = X^T (W * l'(m))``. Problems are processed 32 per launch."""
    from . import _native as N_
    N, d = X.shape
    P = W.shape[1]
    dev = X.device
    if d <= _LR_DMAX and ((N * d) % 4 or X.data_ptr() % 16):
        # the kernel streams X in 16-byte chunks: run the <= 3 trailing rows through torch
        Nm = N - N % 4 if X.data_ptr() % 16 == 0 else 0
        parts = []
        if Nm:
            parts.append(fused_objective(X[:Nm], y[:Nm], W[:Nm], V, bias, loss, yscale, grad))
        parts.append(_torch_objective(X[Nm:], y[Nm:], W[Nm:], V, bias, loss, yscale, grad))
        f = sum(q[0] for q in parts)
        r = sum(q[1] for q in parts)
        G = sum(q[2] for q in parts) if grad else None
        return f, r, G
    yf = y.to(device=dev, dtype=torch.float32).contiguous()
    Wf = W.to(torch.float32).contiguous()
    nblk = _n_blocks(N)
    dpad = ((d + 15) // 16) * 16
    f = torch.empty(P, dtype=torch.float64, device=dev)
    r = torch.empty(P, dtype=torch.float64, device=dev)
    G = torch.empty(d, P, dtype=torch.float64, device=dev) if grad else None
    fp = torch.empty(nblk, _LR_PC, dtype=torch.float64, device=dev)
    rp = torch.empty_like(fp)
    gp = torch.empty(nblk, dpad, _LR_PC, dtype=torch.float32, device=dev) if grad else fp
    single = P <= _LR_PC
    for c0 in range(0, P, _LR_PC):
        pc = min(_LR_PC, P - c0)
        # zero-padded to the kernel's 32 problem columns in one launch each (the optimiser calls this ~300
        # times per learner: allocation + slice-assign pairs were a visible share of its launch overhead)
        Vc = torch.nn.functional.pad(V[:, c0:c0 + pc].to(torch.float32), (0, _LR_PC - pc)).contiguous()
        bc = torch.nn.functional.pad(bias[c0:c0 + pc].to(torch.float32), (0, _LR_PC - pc)).contiguous()
        ys = None
        if yscale is not None:
            ys = torch.ones(_LR_PC, dtype=torch.float32, device=dev)
            ys[:pc] = yscale[c0:c0 + pc]
        if d <= _LR_DMAX:
            N_.check(N_.hip().tmog_hip_lr_objective(
                N_.ptr(X), N, d, N_.ptr(yf), N_.ptr(Wf), P, c0, pc, N_.ptr(Vc), N_.ptr(bc), LOSS_CODES[loss],
                N_.ptr(ys), int(grad), N_.ptr(fp), N_.ptr(rp), N_.ptr(gp) if grad else None, nblk, N_.stream(dev)),
                "lr_objective")
        else:
            M = (X @ Vc).contiguous()          # [N, 32] margins on hipBLASLt
            N_.check(N_.hip().tmog_hip_lr_epilogue_grad(
                N_.ptr(X), N, d, N_.ptr(M), N_.ptr(yf), N_.ptr(Wf), P, c0, pc, N_.ptr(bc), LOSS_CODES[loss],
                N_.ptr(ys), int(grad), N_.ptr(fp), N_.ptr(rp), N_.ptr(gp) if grad else None, nblk, N_.stream(dev)),
                "lr_epilogue_grad")
        if single:
            f, r = fp[:, :pc].sum(0), rp[:, :pc].sum(0)
            if grad:
                G = gp[:, :d, :pc].sum(0, dtype=torch.float64)
            break
        f[c0:c0 + pc] = fp[:, :pc].sum(0)
        r[c0:c0 + pc] = rp[:, :pc].sum(0)
        if grad:
            G[:, c0:c0 + pc] = gp[:, :d, :pc].sum(0, dtype=torch.float64)
    return f, r, G


def _torch_objective(X, y, W, V, bias, loss, yscale, grad):
    """Reference / tail path of ``fused_objective`` (same outputs, fp64 sums)."""
    M = X @ V.to(X.dtype) + bias.to(X.dtype)[None, :]
    yy = y.to(M.dtype)[:, None]
    if loss == "logistic":
        l = torch.nn.functional.softplus(M) - yy * M
        g = torch.sigmoid(M) - yy
    elif loss == "hinge":
        ys = 2 * yy - 1
        l = torch.clamp(1 - ys * M, min=0)
        g = torch.where(ys * M < 1, -ys, torch.zeros_like(M))
    else:
        r = M - yy / yscale.to(M.dtype)[None, :]
        l = 0.5 * r * r
        g = r
    Wm = W.to(M.dtype)
    R = g * Wm
    G = (X.t() @ R).to(torch.float64) if grad else None
    return (l * Wm).sum(0).to(torch.float64), R.sum(0).to(torch.float64), G


_OW_DMAX, _OW_MMAX = 256 * 16, 32


def owlqn_direction_supported(U: torch.Tensor, m: int) -> bool:
    return U.is_cuda and U.dtype == torch.float64 and U.dim() == 2 and U.shape[0] <= _OW_DMAX and m <= _OW_MMAX


def owlqn_direction(U, g, l1, S, Y, RHO, hist_n: int, m: int):
    """OWL-QN pseudo-gradient + two-loop L-BFGS direction + orthant projection for every column of ``U`` in
    one HIP launch (``linear_kernels.hip`` owlqn_direction_kernel); same arithmetic as the torch loop of
    ``models/linear.py`` owlqn_batched. Returns ``(D, pg, xi, dnorm)``."""
    from . import _native as N_
    U, g, l1 = U.contiguous(), g.contiguous(), l1.contiguous()
    d1, P = U.shape
    D, pg, xi = torch.empty_like(U), torch.empty_like(U), torch.empty_like(U)
    dnorm = torch.empty(P, dtype=torch.float64, device=U.device)
    N_.check(N_.hip().tmog_hip_owlqn_direction(
        N_.ptr(U), N_.ptr(g), N_.ptr(l1), N_.ptr(S), N_.ptr(Y), N_.ptr(RHO), int(d1), int(P), int(m), int(hist_n),
        N_.ptr(D), N_.ptr(pg), N_.ptr(xi), N_.ptr(dnorm), N_.stream(U.device)), "owlqn_direction")
    return D, pg, xi, dnorm


def owlqn_candidate(U, D, xi, l1, pg, alpha):
    """OWL-QN line-search candidate ``cand = project_xi(U + alpha D)`` with ``sum l1 |cand|`` and
    ``sum pg (cand - U)`` per column, one HIP launch (``owlqn_candidate_kernel``). All fp64, contiguous."""
    from . import _native as N_
    d1, P = U.shape
    cand = torch.empty_like(U)
    l1t = torch.empty(P, dtype=torch.float64, device=U.device)
    dd = torch.empty_like(l1t)
    a = alpha.to(torch.float64).contiguous()
    N_.check(N_.hip().tmog_hip_owlqn_candidate(
        N_.ptr(U), N_.ptr(D), N_.ptr(xi), N_.ptr(l1), N_.ptr(pg), N_.ptr(a), int(d1), int(P), N_.ptr(cand),
        N_.ptr(l1t), N_.ptr(dd), N_.stream(U.device)), "owlqn_candidate")
    return cand, l1t, dd


"""Linear learners trained as one batched device program.

Reference learners: ``OpLogisticRegression`` (``classification/OpLogisticRegression.scala:46-207``),
``OpLinearSVC`` (``OpLinearSVC.scala:48-165``), ``OpLinearRegression`` (``regression/OpLinearRegression.scala:48-209``)
and ``OpNaiveBayes`` (``OpNaiveBayes.scala:47-107``); their Spark objectives (standardized L2 + L1 elastic
net, L-BFGS / OWL-QN, ``maxIter``, ``tol``) are reproduced here.

MI355X design: every (grid point x CV fold) problem of a learner is one column of a coefficient
matrix ``U [d+1, P]``. A single pass computes all margins ``M = X V`` (one GEMM over the resident
feature matrix), the per-problem masked losses, and the gradient ``X^T R`` (second GEMM); fold
membership and sample weights are a ``[N, P]`` row-weight matrix, so no per-fold copy of ``X`` is made.
The quasi-Newton updates (two-loop recursion, orthant projection, Armijo backtracking) are
vectorized over the ``P`` problems and run in lockstep; converged problems are frozen.
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..ops import linear as LK
from .base import FitJob, Learner, OpPredictor, compact_rows, probability_outputs, register_learner
from ..ops.staging import to_device
from ..stages.base import register_stage


# hipGraph replay of the bf16 objective passes (BatchedObjective._capture), TMOG_LR_GRAPH=1. Off by default: on
# lr-rf-1m the LR lane measured 0.205-0.210 s with it against 0.176-0.177 s eager (profiles/r5_graph_ab_*.log) --
# the two captures per fit cost more than the launches they save; the passes wait on the line search's syncs
_LR_GRAPHS = os.environ.get("TMOG_LR_GRAPH", "0") == "1"


class BatchedObjective:
    """Smooth objective of P linear problems sharing the design matrix ``X``."""

    def __init__(self, X, y, W, inv_std, loss, l2, fit_intercept, y_scale=None, par=None, wcols=None):
        self.X = X
        self.y = y
        self.W = W                      # [N, P] row weights (0 outside a problem's training rows)
        # row-parallel (parallel/learner_parallel.py): X / y / W hold this rank's rows; every per-problem
        # sum is all-reduced (one fused collective per objective pass), the updates run identically
        self.par = par
        self.wsum = _psum(par, W.sum(0).to(torch.float64))[0].clamp_min(1e-300)
        self.inv_std = inv_std          # [d, P]
        self.loss = loss
        self.l2 = l2                    # [P]
        self.fi = fit_intercept         # [P] bool
        self.y_scale = y_scale          # [P] label scale for squared loss
        self.d = X.shape[1]
        self.passes = 0
        # fused one-pass HIP objective (ops/csrc/hip/linear_kernels.hip) when X is an fp32 device matrix
        self.fused = LK.fused_objective_supported(X) and loss in LK.LOSS_CODES
        if self.fused:
            self.yf = y.to(device=X.device, dtype=torch.float32).contiguous()
            self.Wf = W.to(torch.float32).contiguous()
            self.ysf = None if y_scale is None else y_scale.to(device=X.device, dtype=torch.float32)
        # bf16 design copy on the bf16 matrix cores (ops/csrc/hip/linear_bf16_kernels.hip) when configured
        from .. import config as _cfg
        self.bf16 = LK.Bf16Design.of(X) if (self.fused and _cfg.linear_dtype() == "bf16"
                                            and LK.Bf16Design.supported(X)) else None
        if self.bf16 is not None:
            # one weight column per distinct training-row set (wcols: _weight_columns of the jobs), mapped per problem
            P = W.shape[1]
            wc = list(range(P)) if wcols is None else list(wcols)
            uniq = sorted(set(wc))
            pos = {c: i for i, c in enumerate(uniq)}
            self.Wb = self.Wf if len(uniq) == P else self.Wf[:, uniq].contiguous()
            self.wmap = LK.weight_map([pos[c] for c in wc], P, X.device)

    def _pass_body(self, U, grad):
        V = (U[:self.d] * self.inv_std).to(torch.float32)
        b = torch.where(self.fi, U[self.d], torch.zeros_like(U[self.d])).to(torch.float32)
        if self.bf16 is not None:
            return LK.fused_objective_bf16(self.bf16, self.yf, self.Wb, V, b, self.loss, self.ysf, grad=grad,
                                           wmap=self.wmap)
        return LK.fused_objective(self.X, self.yf, self.Wf, V, b, self.loss, self.ysf, grad=grad)

    def _fused_pass(self, U, grad):
        self.passes += 1
        if self.bf16 is not None and _LR_GRAPHS:
            g = self._graphs.get(grad) if hasattr(self, "_graphs") else None
            if g is None and getattr(self, "_graph_ok", True):
                g = self._capture(U, grad)
            if g is not None:
                gU, out, graph = g
                gU.copy_(U)
                graph.replay()
                return tuple(None if t is None else t.clone() for t in out)
        return self._pass_body(U, grad)

    def _capture(self, U, grad):
        """The pass (coefficient scaling, the per-chunk pads, the kernel launches, the partial sums and the fold
        of the centred columns: ~20 launches and their Python) as one hipGraph, replayed for every later pass of
        this fit: the optimiser's ~230 passes per fit were launch-bound at 1M rows. Capture is thread-local (the
        other learner lanes keep launching); any failure falls back to the eager pass for this objective."""
        try:
            dev = U.device
            gU = U.detach().clone()
            cur = torch.cuda.current_stream(dev)
            side = torch.cuda.Stream(device=dev)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                self._pass_body(gU, grad)               # warm-up: lazy initialisation, allocator blocks
            cur.wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=side, capture_error_mode="thread_local"):
                out = self._pass_body(gU, grad)
            cur.wait_stream(side)
            if not hasattr(self, "_graphs"):
                self._graphs = {}
            self._graphs[grad] = (gU, out, graph)
            return self._graphs[grad]
        except Exception as e:  # noqa: BLE001 - eager fallback
            import logging
            logging.getLogger(__name__).debug("objective graph capture failed (%r): eager passes", e)
            self._graph_ok = False
            return None

    def margins(self, U):
        V = (U[:self.d] * self.inv_std).to(self.X.dtype)
        b = torch.where(self.fi, U[self.d], torch.zeros_like(U[self.d])).to(self.X.dtype)
        self.passes += 1
        return LK.gemm(self.X, V) + b[None, :]

    def _elem(self, M, need_grad):
        y = self.y[:, None].to(M.dtype)
        if self.loss == "logistic":
            l = torch.nn.functional.softplus(M) - y * M
            d = torch.sigmoid(M) - y if need_grad else None
        elif self.loss == "hinge":
            ys = 2 * y - 1
            marg = ys * M
            l = torch.clamp(1 - marg, min=0)
            d = torch.where(marg < 1, -ys, torch.zeros_like(M)) if need_grad else None
        else:  # squared, label pre-scaled per problem
            ysc = y / self.y_scale[None, :].to(M.dtype)
            r = M - ysc
            l = 0.5 * r * r
            d = r if need_grad else None
        return l, d

    def value(self, U):
        if self.fused:
            f = _psum(self.par, self._fused_pass(U, False)[0])[0] / self.wsum
            return f + 0.5 * self.l2 * (U[:self.d] ** 2).sum(0)
        M = self.margins(U)
        l, _ = self._elem(M, False)
        f = _psum(self.par, (l * self.W).sum(0).to(torch.float64))[0] / self.wsum
        return f + 0.5 * self.l2 * (U[:self.d] ** 2).sum(0)

    def value_grad(self, U):
        if self.fused:
            f, r, G = _psum(self.par, *self._fused_pass(U, True))
            g = torch.zeros_like(U)
            g[:self.d] = (G / self.wsum[None, :]) * self.inv_std + self.l2[None, :] * U[:self.d]
            g[self.d] = torch.where(self.fi, r / self.wsum, torch.zeros_like(self.wsum))
            return f / self.wsum + 0.5 * self.l2 * (U[:self.d] ** 2).sum(0), g
        M = self.margins(U)
        l, dm = self._elem(M, True)
        R = dm * self.W
        fs, Gs, rs = _psum(self.par, (l * self.W).sum(0).to(torch.float64), LK.gemm_t(self.X, R).to(torch.float64),
                           R.sum(0).to(torch.float64))
        f = fs / self.wsum
        G = Gs / self.wsum[None, :]
        self.passes += 1
        g = torch.zeros_like(U)
        g[:self.d] = G * self.inv_std + self.l2[None, :] * U[:self.d]
        g[self.d] = torch.where(self.fi, rs / self.wsum, torch.zeros_like(self.wsum))
        f = f + 0.5 * self.l2 * (U[:self.d] ** 2).sum(0)
        return f, g


class MultinomialObjective:
    """Softmax cross-entropy of P problems with K classes; ``U`` is ``[(d+1)*K, P]`` laid out as
    ``[d+1, K]`` blocks (class-major coefficient columns), so the batched OWL-QN is reused unchanged.
    One GEMM ``X [N,d] @ V [d, P*K]`` produces every problem's class margins."""

    def __init__(self, X, y, W, inv_std, l2, fit_intercept, K, par=None, wcols=None):
        self.X, self.W, self.K = X, W, K
        self.par = par
        # GPU: margins by GEMM / SpMM, then ONE fused softmax epilogue (log-sum-exp, weighted loss, R in place)
        # and fixed-order column sums (ops/csrc/hip/sparse_kernels.hip) instead of ~15 torch passes over [N, P, K]
        self.fused = X.device.type == "cuda" and os.environ.get("TMOG_MNL_FUSED", "1") != "0"
        # bf16 design copy (config.linear_dtype): bf16 library GEMMs with [hi | lo] coefficient / residual parts
        # around one fused epilogue launch (ops/linear.py mnl_objective_bf16)
        from .. import config as _cfg
        P = W.shape[1]
        self.Xb = None
        if (self.fused and _cfg.linear_dtype() == "bf16" and isinstance(X, torch.Tensor) and
                X.dtype == torch.float32 and X.dim() == 2 and K <= 16 and P <= 256):
            self.Xb = LK.Bf16Design.of(X, pad=False)
            wc = list(range(P)) if wcols is None else list(wcols)
            uniq = sorted(set(wc))
            pos = {c: i for i, c in enumerate(uniq)}
            self.Wb = W.to(torch.float32)[:, uniq].contiguous()
            self.wmap = torch.tensor([pos[c] for c in wc], dtype=torch.int32).to(X.device)
        self.y = y
        self.Y = None if self.fused else torch.nn.functional.one_hot(y.to(torch.int64), K).to(X.dtype)    # [N, K]
        self.wsum = _psum(par, W.sum(0).to(torch.float64))[0].clamp_min(1e-300)
        self.inv_std = inv_std      # [d, P]
        self.l2, self.fi = l2, fit_intercept
        self.d = X.shape[1]
        self.passes = 0

    def _split(self, U):
        d, K = self.d, self.K
        P = U.shape[1]
        B = U.reshape(d + 1, K, P)
        V = B[:d] * self.inv_std[:, None, :]                                       # [d, K, P]
        b = torch.where(self.fi[None, :], B[d], torch.zeros_like(B[d]))            # [K, P]
        return B, V, b

    def margins(self, U):
        B, V, b = self._split(U)
        P = U.shape[1]
        M = LK.gemm(self.X, V.permute(0, 2, 1).reshape(self.d, P * self.K).to(self.X.dtype))
        self.passes += 1
        return M.reshape(-1, P, self.K) + b.t()[None, :, :].to(M.dtype)          # [N, P, K]

    def _loss(self, M):
        lse = torch.logsumexp(M, 2)                                                # [N, P]
        l = lse - (M * self.Y[:, None, :]).sum(2)
        return l, lse

    def _bf16_pass(self, U, grad):
        B, V, b = self._split(U)
        P = U.shape[1]
        self.passes += 1
        f, rs, G = LK.mnl_objective_bf16(self.Xb, V.permute(0, 2, 1).reshape(self.d, P * self.K), self.y, self.Wb,
                                         b.t().reshape(-1), P, self.K, grad, wmap=self.wmap)
        return B, f, rs, G

    def _fused_pass(self, U, grad):
        B, V, b = self._split(U)
        P = U.shape[1]
        M = LK.gemm(self.X, V.permute(0, 2, 1).reshape(self.d, P * self.K).to(torch.float32)).contiguous()
        self.passes += 1
        f, rs = LK.softmax_objective(M, self.y, self.W, b.t().reshape(-1), P, self.K, grad)
        return B, M, f, rs

    def value(self, U):
        if self.Xb is not None:
            B, f, _, _ = self._bf16_pass(U, False)
            f = _psum(self.par, f)[0] / self.wsum
            return f + 0.5 * self.l2 * (B[:self.d] ** 2).sum((0, 1))
        if self.fused:
            B, _, f, _ = self._fused_pass(U, False)
            f = _psum(self.par, f)[0] / self.wsum
            return f + 0.5 * self.l2 * (B[:self.d] ** 2).sum((0, 1))
        M = self.margins(U)
        l, _ = self._loss(M)
        f = _psum(self.par, (l * self.W).sum(0).to(torch.float64))[0] / self.wsum
        B = U.reshape(self.d + 1, self.K, -1)
        return f + 0.5 * self.l2 * (B[:self.d] ** 2).sum((0, 1))

    def value_grad(self, U):
        if self.fused:
            P = U.shape[1]
            if self.Xb is not None:
                B, fs, rs, Gs = self._bf16_pass(U, True)
                fs, Gs, rs = _psum(self.par, fs, Gs, rs)
            else:
                B, R, fs, rs = self._fused_pass(U, True)
                fs, Gs, rs = _psum(self.par, fs, LK.gemm_t(self.X, R).to(torch.float64), rs)
            f = fs / self.wsum
            G = Gs.reshape(self.d, P, self.K).permute(0, 2, 1) / self.wsum[None, None, :]   # [d, K, P]
            g = torch.zeros_like(B)
            g[:self.d] = G * self.inv_std[:, None, :] + self.l2[None, None, :] * B[:self.d]
            gb = rs.reshape(P, self.K).t() / self.wsum[None, :]                       # [K, P]
            g[self.d] = torch.where(self.fi[None, :], gb, torch.zeros_like(gb))
            f = f + 0.5 * self.l2 * (B[:self.d] ** 2).sum((0, 1))
            return f, g.reshape(U.shape)
        M = self.margins(U)
        l, lse = self._loss(M)
        Pr = torch.exp(M - lse[:, :, None])
        R = (Pr - self.Y[:, None, :]) * self.W[:, :, None]                        # [N, P, K]
        P = U.shape[1]
        fs, Gs, rs = _psum(self.par, (l * self.W).sum(0).to(torch.float64),
                           LK.gemm_t(self.X, R.reshape(-1, P * self.K)).to(torch.float64),
                           R.sum(0).to(torch.float64))
        f = fs / self.wsum
        G = Gs.reshape(self.d, P, self.K)
        G = G.permute(0, 2, 1) / self.wsum[None, None, :]                          # [d, K, P]
        self.passes += 1
        B = U.reshape(self.d + 1, self.K, P)
        g = torch.zeros_like(B)
        g[:self.d] = G * self.inv_std[:, None, :] + self.l2[None, None, :] * B[:self.d]
        gb = rs.t() / self.wsum[None, :]                                           # [K, P]
        g[self.d] = torch.where(self.fi[None, :], gb, torch.zeros_like(gb))
        f = f + 0.5 * self.l2 * (B[:self.d] ** 2).sum((0, 1))
        return f, g.reshape(U.shape)


class GramObjective:
    """The squared-loss objective of :class:`BatchedObjective` evaluated from each problem's weighted Gram
    instead of the rows (Spark ``WeightedLeastSquares``: normal-equation statistics aggregated once, then
    Cholesky, or its QuasiNewton solver when there is an L1 term -- LinearRegression.scala solver
    ``auto`` / ``normal``, OpLinearRegression.scala:48-209).

    In the standardised coordinates ``U = [u; u0]`` (``z_j = x_j / sigma_j``, target ``t = y / sigma_y``) the
    data objective ``1/(2n) sum_i w_i (z_i . u + u0 - t_i)^2 + l2/2 |u|^2`` is the quadratic
    ``1/2 U^T H U - g^T U + c`` with ``H = 1/n sum w [z,1][z,1]^T + diag(l2, .., 0)``, ``g = 1/n sum w t [z,1]``
    and ``c = 1/(2n) sum w t^2`` -- identical values, so OWL-QN takes the same path for a d x d cost per
    evaluation instead of a pass over the rows."""

    def __init__(self, H, g, c, l2, fit_intercept):
        self.H, self.g, self.c = H, g, c          # [P, d+1, d+1], [P, d+1], [P]
        self.l2, self.fi = l2, fit_intercept
        self.d = H.shape[1] - 1
        self.passes = 0

    def _q(self, U):
        Ut = U.t()                                 # [P, d+1]
        HU = torch.bmm(self.H, Ut[:, :, None])[:, :, 0]
        return Ut, HU

    def value(self, U):
        self.passes += 1
        Ut, HU = self._q(U)
        return 0.5 * (Ut * HU).sum(1) - (self.g * Ut).sum(1) + self.c + 0.5 * self.l2 * (U[:self.d] ** 2).sum(0)

    def value_grad(self, U):
        self.passes += 1
        Ut, HU = self._q(U)
        f = 0.5 * (Ut * HU).sum(1) - (self.g * Ut).sum(1) + self.c + 0.5 * self.l2 * (U[:self.d] ** 2).sum(0)
        G = (HU - self.g).t().contiguous()         # [d+1, P]
        G[:self.d] += self.l2[None, :] * U[:self.d]
        G[self.d] = torch.where(self.fi, G[self.d], torch.zeros_like(G[self.d]))
        return f, G


def _weighted_grams(X, y, jobs, par=None, chunk: int = 1 << 18):
    """Augmented weighted Grams ``A^T diag(w) A`` (``A = [X, 1, y]``, float64) per distinct fold-weight
    column of ``jobs``: ``(G [k, d+2, d+2], group of each job)``. Jobs that share their training rows (the
    grid points of one CV fold) share one Gram; row chunks bound the fp64 temporaries."""
    dev = X.device
    N, d = X.shape
    keys, group = {}, []
    for j in jobs:
        k = ("all",) if j.rows is None else (j.rows.data_ptr(), int(j.rows.numel()),
                                             None if j.weights is None else j.weights.data_ptr())
        group.append(keys.setdefault(k, len(keys)))
    reps = {}
    for j, g in zip(jobs, group):
        reps.setdefault(g, j)
    W = _fold_weights(N, [reps[g] for g in range(len(keys))], dev, torch.float64)      # [N, k]
    yd = y.to(device=dev, dtype=torch.float64)
    if par is not None:         # row-parallel: this rank's slice of the (replicated) rows, sums all-reduced
        sl = par.row_slice(N)
        X, W, yd = X[sl], W[sl], yd[sl]
        N = int(X.shape[0])
    from ..ops.stats import weighted_gram
    # fp64 matrix-core Grams of [X | 1 | y] for every fold-weight column in one pass (stats_kernels.hip wgram)
    G = weighted_gram(X, W, yd, chunk=chunk)
    G = _psum(par, G)[0]
    return G, group


def _owlqn_direction_torch(U, g, l1, has_l1, S, Y, RHO, hist_n, m):
    """Pseudo-gradient, two-loop recursion, orthant projection (the spec of the HIP owlqn_direction_kernel)."""
    pg = torch.where(U > 0, g + l1, torch.where(U < 0, g - l1,
                     torch.where(g + l1 < 0, g + l1, torch.where(g - l1 > 0, g - l1, torch.zeros_like(g)))))
    q = pg.clone()
    k = min(hist_n, m)
    alphas = []
    for j in range(k):
        idx = (hist_n - 1 - j) % m
        a = RHO[idx] * (S[idx] * q).sum(0)
        q = q - a[None, :] * Y[idx]
        alphas.append((idx, a))
    if k > 0:
        last = (hist_n - 1) % m
        yy = (Y[last] * Y[last]).sum(0)
        gamma = torch.where(yy > 0, (S[last] * Y[last]).sum(0) / yy.clamp_min(1e-300), torch.ones_like(yy))
        q = q * gamma[None, :]
    for idx, a in reversed(alphas):
        b = RHO[idx] * (Y[idx] * q).sum(0)
        q = q + S[idx] * (a - b)[None, :]
    D = -q
    D = torch.where(has_l1 & (torch.sign(D) != torch.sign(-pg)), torch.zeros_like(D), D)
    xi = torch.where(U != 0, torch.sign(U), torch.sign(-pg))
    dnorm = torch.sqrt((pg * pg).sum(0)).clamp_min(1e-300)
    return D, pg, xi, dnorm


_TRACE = os.environ.get("TMOG_OWLQN_TRACE", "0") == "1"


def owlqn_batched(obj: BatchedObjective, U0: torch.Tensor, l1: torch.Tensor, max_iter: torch.Tensor,
                  tol: torch.Tensor, m: int = 10, max_ls: int = 30):
    """Batched OWL-QN (L-BFGS when ``l1 == 0``) over the columns of ``U``.

    ``l1`` is ``[d+1, P]`` (0 on the intercept). Returns ``(U, n_iter [P], F [P])``.
    """
    U = U0.clone()
    d1, P = U.shape
    dev = U.device
    f, g = obj.value_grad(U)
    F = f + (l1 * U.abs()).sum(0)
    S = torch.zeros(m, d1, P, dtype=U.dtype, device=dev)
    Y = torch.zeros_like(S)
    RHO = torch.zeros(m, P, dtype=U.dtype, device=dev)
    hist_n = 0
    done = torch.zeros(P, dtype=torch.bool, device=dev)
    iters = torch.zeros(P, dtype=torch.int64, device=dev)
    has_l1 = l1 > 0
    fused_dir = LK.owlqn_direction_supported(U, m) and os.environ.get("TMOG_OWLQN_FUSED", "1") != "0"
    if fused_dir:
        l1 = l1.to(U.dtype).contiguous()
    from ..utils.cancel import check as _cancel_check
    # the first line-search trial is evaluated with its gradient while the previous iteration's first trial was
    # accepted by every problem (adaptive: a value-only trial is cheaper when backtracking is likely)
    spec_on = os.environ.get("TMOG_OWLQN_SPEC", "0") == "1"     # measured no faster on the headline: opt-in
    spec_grad = spec_on
    # TMOG_LS_BATCH=k: look at the acceptance every k trials. Measured neutral-to-slower at k = 2, 3 on lr-rf-1m and
    # multiclass-text (profiles/r5_ls_ab_*.log): the passes, not the synchronisations, are the time
    ls_batch = max(1, int(os.environ.get("TMOG_LS_BATCH", "1")))
    for it in range(int(max_iter.max().item()) if P else 0):
        _cancel_check()             # maxWait (tuning/validators.py _fit_eval_bounded)
        done |= iters >= max_iter
        if bool(done.all()):
            break
        k = min(hist_n, m)
        if fused_dir:
            # one HIP launch for everything up to the line search (ops/linear.py owlqn_direction)
            D, pg, xi, dnorm = LK.owlqn_direction(U, g, l1, S, Y, RHO, hist_n, m)
        else:
            D, pg, xi, dnorm = _owlqn_direction_torch(U, g, l1, has_l1, S, Y, RHO, hist_n, m)
        alpha = torch.where(torch.full_like(dnorm, float(k == 0), dtype=torch.bool), 1.0 / dnorm,
                            torch.ones_like(dnorm))
        accepted = done.clone()
        Un = U.clone()
        Fn = F.clone()
        first = None            # (f, g) of the first trial point when it is evaluated with its gradient
        late = False            # some problem accepted after the first trial
        for trial in range(max_ls):
            if fused_dir:
                # projected candidate + its Armijo sums in one launch (ops/linear.py owlqn_candidate)
                cand, l1t, dd = LK.owlqn_candidate(U, D, xi, l1, pg, alpha)
                rhs = F + 1e-4 * dd
            else:
                cand = U + alpha[None, :] * D
                cand = torch.where(has_l1 & (torch.sign(cand) != xi), torch.zeros_like(cand), cand)
                l1t = (l1 * cand.abs()).sum(0)
                rhs = F + 1e-4 * (pg * (cand - U)).sum(0)
            if trial == 0 and spec_grad:
                # the first trial is accepted by most problems once the curvature pairs are in: its gradient
                # comes from the same pass (a value pass + a gradient pass become one gradient pass)
                first = obj.value_grad(cand)
                fc = first[0] + l1t
            else:
                fc = obj.value(cand) + l1t
                late = True
            ok = (fc <= rhs) & ~accepted
            Un = torch.where(ok[None, :], cand, Un)
            Fn = torch.where(ok, fc, Fn)
            accepted |= ok
            if _TRACE:
                print(f"[owlqn] it {it} trial {trial} ok {int(ok.sum())} accepted {int(accepted.sum())}/{P} "
                      f"alpha {alpha.tolist()}", flush=True)
            # the host looks at the acceptance every ls_batch trials: the next trial is enqueued while the
            # previous one runs (a trial after everything was accepted changes nothing -- ok is all False)
            if ((trial + 1) % ls_batch == 0 or trial == max_ls - 1) and bool(accepted.all()):
                break
            alpha = torch.where(accepted, alpha, alpha * 0.5)
        failed = ~accepted
        moved = accepted & ~done
        if first is not None and not late:
            fn, gn = first          # every moved problem sits at the first trial point
        else:
            fn, gn = obj.value_grad(Un)
        spec_grad = spec_on and not late
        s = Un - U
        yv = gn - g
        sy = (s * yv).sum(0)
        upd = moved & (sy > 1e-10)
        slot = hist_n % m
        S[slot] = torch.where(upd[None, :], s, S[slot] if hist_n >= m else torch.zeros_like(s))
        Y[slot] = torch.where(upd[None, :], yv, Y[slot] if hist_n >= m else torch.zeros_like(yv))
        RHO[slot] = torch.where(upd, 1.0 / sy.clamp_min(1e-300), RHO[slot] if hist_n >= m else torch.zeros_like(sy))
        hist_n += 1
        Fnew = fn + (l1 * Un.abs()).sum(0)
        rel = (F - Fnew).abs() / torch.maximum(torch.maximum(F.abs(), Fnew.abs()), torch.ones_like(F))
        U = torch.where(moved[None, :], Un, U)
        g = torch.where(moved[None, :], gn, g)
        F = torch.where(moved, Fnew, F)
        iters = iters + moved.to(torch.int64)
        done |= failed | (moved & (rel < tol))
    return U, iters, F


def _weight_columns(jobs: Sequence[FitJob]) -> List[int]:
    """For each job the index of the first job with the same training rows and weights (the grid points of one
    CV fold share their row tensor, ``compact_rows``): such jobs have identical fold-weight columns."""
    first: Dict[tuple, int] = {}
    out = []
    for p, j in enumerate(jobs):
        k = ("all",) if j.rows is None else (j.rows.data_ptr(), int(j.rows.numel()), tuple(j.rows.stride()))
        k = k + (None if j.weights is None else (j.weights.data_ptr(), int(j.weights.numel()),
                                                 tuple(j.weights.stride())),)
        out.append(first.setdefault(k, p))
    return out


def _fold_weights(N, jobs: Sequence[FitJob], dev, dtype):
    W = torch.zeros(N, len(jobs), dtype=dtype, device=dev)
    for p, j in enumerate(jobs):
        if j.rows is None:
            W[:, p] = 1.0 if j.weights is None else j.weights.to(dtype)
        else:
            r = j.rows.to(dev)
            W[r, p] = 1.0 if j.weights is None else j.weights.to(dev, dtype)
    return W


def _psum(par, *ts):
    """Sum of per-rank partial sums (identity without a row-parallel context)."""
    if par is None or par.world <= 1:
        return list(ts)
    return par.sum(*ts)


def _row_par(context):
    par = context.get("par") if isinstance(context, dict) else None
    return par if (par is not None and par.world > 1) else None


_STD_CHUNK = 1 << 18


def _feature_std(X, W, par=None):
    """Unbiased weighted std per column and problem (``[d, P]``): ``X^T W`` and ``(X*X)^T W`` GEMMs over
    row chunks, so the squared matrix is never materialised whole (was a full copy of the fold matrix)."""
    d, P = X.shape[1], W.shape[1]
    if isinstance(X, LK.SparseDesign):
        n, s1, s2 = _psum(par, W.sum(0).to(torch.float64), X.tmm(W), X.tmm(W, square=True))
        mean = s1 / n.clamp_min(1)[None, :]
        var = (s2 - n[None, :] * mean * mean) / (n - 1).clamp_min(1)[None, :]
        return torch.sqrt(var.clamp_min(0)), mean
    if X.is_cuda and X.dtype == torch.float32 and X.dim() == 2 and X.stride(1) == 1 and X.shape[0] > 0:
        # fp64 sums on the device (stats_kernels.hip weighted_colsums): a problem's statistics do not depend
        # on the other problems of the batch (a library GEMM picks its blocking by the batch width)
        from ..ops import _native as N_
        Wf = W.to(torch.float32).contiguous()
        out = torch.empty(P, 2, d, dtype=torch.float64, device=X.device)
        N_.check(N_.hip().tmog_hip_weighted_colsums(N_.ptr(X), X.shape[0], d, X.stride(0), N_.ptr(Wf), P, P,
                                                    N_.ptr(out), N_.stream(X.device)), "weighted_colsums")
        n, s1, s2 = _psum(par, W.to(torch.float64).sum(0), out[:, 0].t().contiguous(), out[:, 1].t().contiguous())
        mean = s1 / n.clamp_min(1)[None, :]
        var = (s2 - n[None, :] * mean * mean) / (n - 1).clamp_min(1)[None, :]
        return torch.sqrt(var.clamp_min(0)), mean
    s1 = torch.zeros(d, P, dtype=torch.float64, device=X.device)
    s2 = torch.zeros_like(s1)
    for a in range(0, X.shape[0], _STD_CHUNK):
        Xc, Wc = X[a:a + _STD_CHUNK], W[a:a + _STD_CHUNK]
        s1 += LK.gemm_t(Xc, Wc).to(torch.float64)
        s2 += LK.gemm_t(Xc * Xc, Wc).to(torch.float64)
    n, s1, s2 = _psum(par, W.sum(0).to(torch.float64), s1, s2)
    mean = s1 / n.clamp_min(1)[None, :]
    var = (s2 - n[None, :] * mean * mean) / (n - 1).clamp_min(1)[None, :]
    return torch.sqrt(var.clamp_min(0)), mean


class _LinearBase(Learner):
    # the model selector may add the winner's full-training-set refit of every grid point to the CV batch
    # (tuning/validators.py): independent problems of one batched optimiser, so the refit rides along in
    # the same passes over X instead of a separate fit after the selection
    batched_refit = True
    loss = "logistic"
    parallel = "rows"

    def _setup(self, X, y, jobs, par=None):
        """Fold weights, feature scales and per-problem hyper-parameters. With a row-parallel context
        ``X`` / ``y`` / ``W`` are cut to this rank's contiguous row slice (``par.row_slice``) and the
        column statistics are all-reduced. Returns ``(X, y, W, std, mean, inv_std, reg, en, fi,
        max_iter, tol, stdz)``."""
        dev = X.device
        N, d = X.shape
        P = len(jobs)
        W = _fold_weights(N, jobs, dev, X.dtype)
        if par is not None:
            sl = par.row_slice(N)
            X, y, W = X[sl], y[sl], W[sl].contiguous()
        # column statistics once per distinct fold-weight column (each problem's are computed alone either way)
        wc = _weight_columns(jobs)
        uniq = sorted(set(wc))
        if len(uniq) < P:
            pos = {c: i for i, c in enumerate(uniq)}
            std_u, mean_u = _feature_std(X, W[:, uniq].contiguous(), par)
            sel = torch.tensor([pos[c] for c in wc], dtype=torch.int64, device=std_u.device)
            std, mean = std_u.index_select(1, sel), mean_u.index_select(1, sel)
        else:
            std, mean = _feature_std(X, W, par)
        stdz = [bool(j.params.get("standardization", True)) for j in jobs]
        inv_std = torch.where(std > 0, 1.0 / std.clamp_min(1e-300), torch.zeros_like(std))
        for p, s in enumerate(stdz):
            if not s:
                inv_std[:, p] = torch.where(std[:, p] > 0, torch.ones_like(std[:, p]), torch.zeros_like(std[:, p]))
        reg = to_device([float(j.params.get("reg_param", 0.0)) for j in jobs], dev, np.float64)
        en = to_device([float(j.params.get("elastic_net_param", 0.0)) for j in jobs], dev, np.float64)
        fi = to_device([bool(j.params.get("fit_intercept", True)) for j in jobs], dev, np.bool_)
        max_iter = to_device([int(j.params.get("max_iter", 100)) for j in jobs], dev, np.int64)
        tol = to_device([float(j.params.get("tol", 1e-6)) for j in jobs], dev, np.float64)
        return X, y, W, std, mean, inv_std, reg, en, fi, max_iter, tol, stdz


@register_learner
class LogisticRegressionLearner(_LinearBase):
    """Binary logistic regression, Spark ``LogisticRegression`` objective (binomial family)."""
    name = "OpLogisticRegression"
    defaults = {"fit_intercept": True, "elastic_net_param": 0.0, "max_iter": 100, "reg_param": 0.0,
                "standardization": True, "tol": 1e-6, "threshold": 0.5}
    loss = "logistic"

    def _fit_multinomial(self, X, y, jobs, K, par=None):
        """Spark ``family=multinomial`` (chosen by ``auto`` when there are more than 2 classes)."""
        dev = X.device
        N, d = X.shape
        P = len(jobs)
        X, y, W, std, mean, inv_std, reg, en, fi, max_iter, tol, stdz = self._setup(X, y, jobs, par)
        l2 = reg * (1 - en)
        obj = MultinomialObjective(X, y, W, inv_std, l2, fi, K, par=par, wcols=_weight_columns(jobs))
        U0 = torch.zeros(d + 1, K, P, dtype=torch.float64, device=dev)
        cnt = _psum(par, torch.stack([(W * (y == k)[:, None].to(W.dtype)).sum(0)
                                      for k in range(K)]).to(torch.float64))[0]
        pri = (cnt / cnt.sum(0, keepdim=True).clamp_min(1e-300)).clamp_min(1e-12)
        lp = torch.log(pri)
        U0[d] = torch.where(fi[None, :], lp - lp.mean(0, keepdim=True), torch.zeros_like(lp))
        l1 = torch.zeros(d + 1, K, P, dtype=torch.float64, device=dev)
        l1[:d] = (reg * en)[None, None, :]
        U, iters, F = owlqn_batched(obj, U0.reshape(-1, P), l1.reshape(-1, P), max_iter, tol)
        B = U.reshape(d + 1, K, P)
        coef = (B[:d] * inv_std[:, None, :]).permute(2, 1, 0).cpu().numpy()          # [P, K, d]
        icpt = torch.where(fi[None, :], B[d], torch.zeros_like(B[d]))
        icpt = (icpt - icpt.mean(0, keepdim=True)).t().cpu().numpy()                 # centered, [P, K]
        it = iters.cpu().numpy()
        return [{"coefficient_matrix": coef[p].copy(), "intercepts": icpt[p].copy(), "n_iter": int(it[p]),
                 "n_classes": K} for p in range(P)]

    def fit_batch(self, X, y, jobs, context=None):
        X, y, jobs = compact_rows(X, y, jobs)
        dev = X.device
        N, d = X.shape
        P = len(jobs)
        if P == 0:
            return []
        K = int(y.max().item()) + 1 if y.numel() else 2
        par = _row_par(context)
        # mostly-zero wide matrices (hashed text, pivots): dense block + CSR / CSC (ops/linear.py SparseDesign)
        from .. import config as _cfg
        # the multinomial bf16 path streams the whole (compacted) design in bf16 through library GEMMs instead
        bf16_mnl = self.loss == "logistic" and K > 2 and _cfg.linear_dtype() == "bf16" and X.is_cuda and K <= 16
        if par is None and not bf16_mnl and os.environ.get("TMOG_LR_SPARSE", "1") != "0" and \
                LK.SparseDesign.worthwhile(X):
            X = LK.SparseDesign(X)
        if self.loss == "logistic" and K > 2:
            return self._fit_multinomial(X, y, jobs, K, par)
        X, y, W, std, mean, inv_std, reg, en, fi, max_iter, tol, stdz = self._setup(X, y, jobs, par)
        l2 = reg * (1 - en)
        l1v = reg * en
        obj = BatchedObjective(X, y, W, inv_std, self.loss, l2, fi, par=par, wcols=_weight_columns(jobs))
        U0 = torch.zeros(d + 1, P, dtype=torch.float64, device=dev)
        if self.loss == "logistic":
            pos, tot = _psum(par, (W * y[:, None].to(W.dtype)).sum(0).to(torch.float64),
                             W.sum(0).to(torch.float64))
            p1 = (pos / tot.clamp_min(1e-300)).clamp(1e-12, 1 - 1e-12)
            U0[d] = torch.where(fi, torch.log(p1 / (1 - p1)), torch.zeros_like(p1))
        l1 = torch.zeros(d + 1, P, dtype=torch.float64, device=dev)
        l1[:d] = l1v[None, :]
        U, iters, F = owlqn_batched(obj, U0, l1, max_iter, tol)
        coef = (U[:d] * inv_std).t().cpu().numpy()         # back to the original feature scale
        icpt = torch.where(fi, U[d], torch.zeros_like(U[d])).cpu().numpy()
        it = iters.cpu().numpy()
        return [{"coefficients": coef[p].copy(), "intercept": float(icpt[p]), "n_iter": int(it[p]),
                 "threshold": float(jobs[p].params.get("threshold", 0.5)), "n_classes": 2} for p in range(P)]

    def margin(self, state, X):
        c = torch.as_tensor(state["coefficients"], dtype=X.dtype, device=X.device)
        return (X @ c).to(torch.float64) + state["intercept"]

    @staticmethod
    def _multinomial_outputs(state, X):
        C = torch.as_tensor(state["coefficient_matrix"], dtype=X.dtype, device=X.device)     # [K, d]
        b = torch.as_tensor(state["intercepts"], dtype=torch.float64, device=X.device)
        raw = (X @ C.t()).to(torch.float64) + b[None, :]
        prob = torch.softmax(raw, 1)
        return torch.argmax(raw, 1).to(torch.float64), raw, prob

    def predict(self, state, X, context=None):
        if "coefficient_matrix" in state:
            return self._multinomial_outputs(state, X)
        return probability_outputs(self.margin(state, X), threshold=state.get("threshold", 0.5))

    def predict_batch(self, states, X, rows, context=None):
        if not states:
            return []
        if any("coefficient_matrix" in s for s in states):
            return Learner.predict_batch(self, states, X, rows, context)
        # margins only of the rows each model is scored on: the models of one validation fold share its rows
        # (one GEMM per fold over those rows, not one over every fold's rows for every model)
        groups: Dict[tuple, List[int]] = {}
        for p, r in enumerate(rows):
            key = ("all",) if r is None else (r.data_ptr(), int(r.numel()), str(r.device))
            groups.setdefault(key, []).append(p)
        out: List = [None] * len(states)
        for key, ps in groups.items():
            r = rows[ps[0]]
            Xr = X if r is None else X.index_select(0, r.to(X.device))     # a gather: no host synchronisation
            C = torch.as_tensor(np.stack([states[p]["coefficients"] for p in ps], 1), dtype=X.dtype, device=X.device)
            b = torch.as_tensor([states[p]["intercept"] for p in ps], dtype=torch.float64, device=X.device)
            M = LK.gemm(Xr, C).to(torch.float64) + b[None, :]
            for c, p in enumerate(ps):
                out[p] = probability_outputs(M[:, c], threshold=states[p].get("threshold", 0.5))
        return out

    def feature_contributions(self, state, d):
        if "coefficient_matrix" in state:
            return np.asarray(state["coefficient_matrix"], np.float64)
        return np.asarray(state["coefficients"], np.float64)


@register_learner
class LinearSVCLearner(LogisticRegressionLearner):
    """Linear SVM with hinge loss and L2 (Spark ``LinearSVC``)."""
    name = "OpLinearSVC"
    defaults = {"fit_intercept": True, "max_iter": 100, "reg_param": 0.0, "standardization": True,
                "tol": 1e-6, "threshold": 0.0}
    loss = "hinge"

    def predict(self, state, X, context=None):
        m = self.margin(state, X)
        raw = torch.stack([-m, m], 1)
        pred = (m > state.get("threshold", 0.0)).to(torch.float64)
        return pred, raw, torch.zeros(m.shape[0], 0, dtype=torch.float64, device=m.device)

    def predict_batch(self, states, X, rows, context=None):
        return Learner.predict_batch(self, states, X, rows, context)


@register_learner
class LinearRegressionLearner(_LinearBase):
    """Least squares with elastic net, label and features standardized (Spark ``LinearRegression``)."""
    name = "OpLinearRegression"
    problem = "regression"
    defaults = {"fit_intercept": True, "elastic_net_param": 0.0, "max_iter": 100, "reg_param": 0.0,
                "standardization": True, "tol": 1e-6, "solver": "auto"}
    loss = "squared"

    # Spark WeightedLeastSquares.MAX_NUM_FEATURES: solver "auto" takes the normal equations up to this width
    NORMAL_MAX_FEATURES = 4096

    def fit_batch(self, X, y, jobs, context=None):
        X, y, jobs = compact_rows(X, y, jobs)
        dev = X.device
        N, d = X.shape
        P = len(jobs)
        if P == 0:
            return []
        par = _row_par(context)
        solvers = {str(j.params.get("solver", "auto")).lower() for j in jobs}
        if solvers <= {"normal"} or (solvers <= {"auto", "normal"} and d <= self.NORMAL_MAX_FEATURES) \
                and os.environ.get("TMOG_LINREG_NORMAL", "1") != "0":
            return self._fit_normal(X, y, jobs, par)
        X, y, W, std, mean, inv_std, reg, en, fi, max_iter, tol, stdz = self._setup(X, y, jobs, par)
        yv = y.to(torch.float64)
        n, sy = _psum(par, W.sum(0).to(torch.float64), (W.to(torch.float64) * yv[:, None]).sum(0))
        ym = sy / n.clamp_min(1)
        yvar = _psum(par, (W.to(torch.float64) * (yv[:, None] - ym[None, :]) ** 2).sum(0))[0] / (n - 1).clamp_min(1)
        ystd = torch.sqrt(yvar).clamp_min(1e-12)
        eff = reg / ystd
        obj = BatchedObjective(X, y, W, inv_std, "squared", eff * (1 - en), fi, y_scale=ystd, par=par,
                               wcols=_weight_columns(jobs))
        U0 = torch.zeros(d + 1, P, dtype=torch.float64, device=dev)
        U0[d] = torch.where(fi, ym / ystd, torch.zeros_like(ym))
        l1 = torch.zeros(d + 1, P, dtype=torch.float64, device=dev)
        l1[:d] = (eff * en)[None, :]
        U, iters, F = owlqn_batched(obj, U0, l1, max_iter, tol)
        coef = (U[:d] * inv_std * ystd[None, :]).t().cpu().numpy()
        icpt = (torch.where(fi, U[d], torch.zeros_like(U[d])) * ystd).cpu().numpy()
        return [{"coefficients": coef[p].copy(), "intercept": float(icpt[p]), "n_iter": int(iters[p])}
                for p in range(P)]

    def _fit_normal(self, X, y, jobs, par=None):
        """Normal-equation path: one weighted Gram per CV fold (a single pass over the rows), then per
        problem a Cholesky solve of ``(Cov_z + l2 I) u = cov_zt`` when there is no L1 term, else OWL-QN on
        the Gram quadratic (:class:`GramObjective`) -- Spark WLS's Cholesky / QuasiNewton solvers. A
        singular system (collinear columns without L2) falls back to the quadratic OWL-QN, as WLS does."""
        d = X.shape[1]
        P = len(jobs)
        G, group = _weighted_grams(X, y, jobs, par)
        # Everything after the Grams works on [P, d+2, d+2] systems: on the host (fp64 CPU torch), where the
        # Cholesky solves and the quadratic OWL-QN's few hundred tiny steps are microseconds each -- on the
        # GPU every one of them is a kernel launch (the regression config spent ~5 s there)
        dev = torch.device("cpu")
        G = G.to(dev)
        gi = torch.as_tensor(group, dtype=torch.int64, device=dev)
        Gp = G[gi]                                               # [P, d+2, d+2]
        n = Gp[:, d, d]
        Sx, Sy = Gp[:, :d, d], Gp[:, d, d + 1]
        Sxx, Sxy, Syy = Gp[:, :d, :d], Gp[:, :d, d + 1], Gp[:, d + 1, d + 1]
        nm1 = (n - 1).clamp_min(1)
        var = (torch.diagonal(Sxx, dim1=1, dim2=2) - Sx * Sx / n.clamp_min(1)[:, None]) / nm1[:, None]
        std = torch.sqrt(var.clamp_min(0))                        # [P, d], as _feature_std
        stdz = torch.as_tensor([bool(j.params.get("standardization", True)) for j in jobs], device=dev)
        inv = torch.where(std > 0, 1.0 / std.clamp_min(1e-300), torch.zeros_like(std))
        inv = torch.where(stdz[:, None], inv, (std > 0).to(inv.dtype))
        ym = Sy / n.clamp_min(1)
        ystd = torch.sqrt(((Syy - Sy * Sy / n.clamp_min(1)) / nm1).clamp_min(0)).clamp_min(1e-12)
        reg = to_device([float(j.params.get("reg_param", 0.0)) for j in jobs], dev, np.float64)
        en = to_device([float(j.params.get("elastic_net_param", 0.0)) for j in jobs], dev, np.float64)
        fi = to_device([bool(j.params.get("fit_intercept", True)) for j in jobs], dev, np.bool_)
        max_iter = to_device([int(j.params.get("max_iter", 100)) for j in jobs], dev, np.int64)
        tol = to_device([float(j.params.get("tol", 1e-6)) for j in jobs], dev, np.float64)
        eff = reg / ystd
        l2, l1v = eff * (1 - en), eff * en
        # quadratic in U = [u; u0] over z = x * inv, t = y / ystd
        nn = n.clamp_min(1e-300)
        S1 = torch.cat([Sx, n[:, None]], 1)                      # sum w [x, 1]
        M = torch.zeros(P, d + 1, d + 1, dtype=torch.float64, device=dev)
        M[:, :d, :d] = Sxx
        M[:, :d, d] = Sx
        M[:, d, :d] = Sx
        M[:, d, d] = n
        sc = torch.cat([inv, torch.ones(P, 1, dtype=torch.float64, device=dev)], 1)     # z = x * inv, 1
        H = M * sc[:, :, None] * sc[:, None, :] / nn[:, None, None]
        gvec = torch.cat([Sxy, Sy[:, None]], 1) * sc / (nn * ystd)[:, None]
        c = 0.5 * Syy / (nn * ystd * ystd)
        # no intercept: the intercept coordinate is pinned to 0 (row / column cleared, unit diagonal)
        nofi = ~fi
        H[nofi, d, :] = 0.0
        H[nofi, :, d] = 0.0
        H[nofi, d, d] = 1.0
        gvec[nofi, d] = 0.0
        del S1
        U = torch.zeros(d + 1, P, dtype=torch.float64, device=dev)
        iters = torch.zeros(P, dtype=torch.int64, device=dev)
        exact = (l1v <= 0)
        solved = torch.zeros(P, dtype=torch.bool, device=dev)
        if bool(exact.any()):
            A = H[exact].clone()
            A[:, torch.arange(d), torch.arange(d)] += l2[exact][:, None]
            # zero-variance columns (z = 0): keep their coefficient at 0
            dead = torch.diagonal(A, dim1=1, dim2=2)[:, :d] <= 0
            A[:, torch.arange(d), torch.arange(d)] += dead.to(A.dtype)
            L, info = torch.linalg.cholesky_ex(A)
            ok = info == 0
            if bool(ok.any()):
                sol = torch.cholesky_solve(gvec[exact][ok][:, :, None], L[ok])[:, :, 0]
                idx = torch.nonzero(exact).reshape(-1)[ok]
                U[:, idx] = sol.t()
                solved[idx] = True
        rest = ~solved
        if bool(rest.any()):
            r = torch.nonzero(rest).reshape(-1)
            obj = GramObjective(H[r], gvec[r], c[r], l2[r], fi[r])
            U0 = torch.zeros(d + 1, int(r.numel()), dtype=torch.float64, device=dev)
            U0[d] = torch.where(fi[r], ym[r] / ystd[r], torch.zeros_like(ym[r]))
            l1 = torch.zeros(d + 1, int(r.numel()), dtype=torch.float64, device=dev)
            l1[:d] = l1v[r][None, :]
            Ur, it, _ = owlqn_batched(obj, U0, l1, max_iter[r], tol[r])
            U[:, r] = Ur
            iters[r] = it
        coef = (U[:d] * inv.t() * ystd[None, :]).t().cpu().numpy()
        icpt = (torch.where(fi, U[d], torch.zeros_like(U[d])) * ystd).cpu().numpy()
        it = iters.cpu().numpy()
        return [{"coefficients": coef[p].copy(), "intercept": float(icpt[p]), "n_iter": int(it[p]),
                 "solver": "normal"} for p in range(P)]

    def predict(self, state, X, context=None):
        c = torch.as_tensor(state["coefficients"], dtype=X.dtype, device=X.device)
        m = (X @ c).to(torch.float64) + state["intercept"]
        e = torch.zeros(m.shape[0], 0, dtype=torch.float64, device=m.device)
        return m, e, e

    def feature_contributions(self, state, d):
        return np.asarray(state["coefficients"], np.float64)


@register_learner
class NaiveBayesLearner(Learner):
    """Multinomial / Bernoulli naive Bayes with Laplace smoothing (Spark ``NaiveBayes``)."""
    name = "OpNaiveBayes"
    problem = "multiclass"
    defaults = {"smoothing": 1.0, "model_type": "multinomial"}

    def fit_batch(self, X, y, jobs, context=None):
        from ..ops.stats import class_column_sums
        out = []
        K = int(y.max().item()) + 1 if y.numel() else 2
        K = max(K, 2)
        if bool((X < 0).any()):
            raise ValueError("Naive Bayes requires nonnegative feature values")
        # every job's class feature sums in one pass over X: codes[p, r] = class of row r in job p, -1 if
        # the row is not in the job (HIP class_colsum_kernel)
        n = X.shape[0]
        codes = torch.full((len(jobs), n), -1, dtype=torch.int32, device=X.device)
        yl = y.long()
        for k, j in enumerate(jobs):
            r = torch.arange(n, device=X.device) if j.rows is None else j.rows.to(X.device)
            codes[k, r] = yl[r].to(torch.int32)
        FS = class_column_sums(X, codes, K)                          # [P, K, d]
        for k, j in enumerate(jobs):
            lam = float(j.params.get("smoothing", 1.0))
            cnt = torch.bincount(codes[k][codes[k] >= 0].long(), minlength=K).to(torch.float64)
            fs = FS[k].t()                                           # [d, K] class feature sums
            pi = torch.log(cnt + lam) - math.log(float(cnt.sum()) + K * lam)
            if j.params.get("model_type", "multinomial") == "bernoulli":
                theta = torch.log(fs + lam) - torch.log(cnt + 2 * lam)[None, :]
            else:
                theta = torch.log(fs + lam) - torch.log(fs.sum(0) + fs.shape[0] * lam)[None, :]
            out.append({"pi": pi.cpu().numpy(), "theta": theta.t().cpu().numpy(), "n_classes": K,
                        "model_type": j.params.get("model_type", "multinomial")})
        return out

    def predict(self, state, X, context=None):
        pi = torch.as_tensor(state["pi"], device=X.device)
        th = torch.as_tensor(state["theta"], device=X.device)
        Xd = X.to(torch.float64)
        if state.get("model_type") == "bernoulli":
            neg = torch.log1p(-torch.exp(th).clamp(max=1 - 1e-12))
            raw = Xd @ (th - neg).t() + (pi + neg.sum(1))[None, :]
        else:
            raw = Xd @ th.t() + pi[None, :]
        prob = torch.softmax(raw, 1)
        return torch.argmax(prob, 1).to(torch.float64), raw, prob

    def feature_contributions(self, state, d):
        th = np.asarray(state["theta"])
        return th[-1] - th[0] if th.shape[0] >= 2 else th[0]


@register_stage
class OpLogisticRegression(OpPredictor):
    operation_name = "OpLogisticRegression"
    learner_cls = LogisticRegressionLearner


@register_stage
class OpLinearSVC(OpPredictor):
    operation_name = "OpLinearSVC"
    learner_cls = LinearSVCLearner


@register_stage
class OpLinearRegression(OpPredictor):
    operation_name = "OpLinearRegression"
    learner_cls = LinearRegressionLearner


@register_stage
class OpNaiveBayes(OpPredictor):
    operation_name = "OpNaiveBayes"
    learner_cls = NaiveBayesLearner

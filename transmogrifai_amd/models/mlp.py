"""Multilayer perceptron classifier (``classification/OpMultilayerPerceptronClassifier.scala:49-144``; Spark
``MultilayerPerceptronClassifier``: sigmoid hidden layers, softmax output, L-BFGS on the cross-entropy).

SURVEY.md K27. All (grid point x fold) jobs with the same layer sizes train as ONE batched problem, as the
linear learners do: every job is a column of the parameter matrix ``U [n_params, P]`` and a column of the row
weights ``W [N, P]`` (zero outside its fold), and one batched L-BFGS (``linear.owlqn_batched`` without L1)
drives all of them. One objective pass is

* forward: every layer product on the matrix cores with its bias + sigmoid fused into the GEMM's epilogue
  (``dense_kernels.hip`` rowgemm; the first layer one launch of the shared X against all P weight matrices as
  grouped columns, so X is streamed once per 64 output columns), and the output layer's softmax / weighted
  cross-entropy / ``W (softmax - onehot)`` in one kernel (``sparse_kernels.hip`` softmax epilogue, shared with
  the multinomial logistic regression);
* backward: weight gradients as matrix-core ``H^T dZ`` products (``dense_kernels.hip`` xtd: fp32 chunks summed
  in fp64), ``dZ W^T`` with W read transposed in place, the sigmoid derivative fused with the bias-gradient column
  sums (``mlp_kernels.hip``).

The layer products run on hipBLASLt by default (measured faster than the ``dense_kernels.hip`` products on these
shapes, see ``ops/dense.py enabled``); ``TMOG_DENSE_MFMA=1`` selects the fused matrix-core path described above.
Spark stacks rows into ``blockSize`` matrices only for BLAS; here all rows of a fold are one batch. The
objective is the weighted mean cross-entropy (no regularisation, as Spark's MLP). The host path computes the
same objective with torch ops.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch

from .base import Learner, OpPredictor, register_learner
from ..stages.base import register_stage


def _forward(params, X, n_layers):
    h = X
    for i in range(n_layers):
        W, b = params[2 * i], params[2 * i + 1]
        h = h @ W + b
        if i < n_layers - 1:
            h = torch.sigmoid(h)
    return h


def _bias_sigmoid_(Z: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """``Z [P, N, B] <- sigmoid(Z + b[:, None, :])`` in place (fused HIP epilogue on the GPU)."""
    if Z.is_cuda:
        from ..ops import _native as N_
        P, N, B = Z.shape
        N_.check(N_.hip().tmog_hip_mlp_bias_sigmoid(N_.ptr(Z), P, N, B, N_.ptr(b.contiguous()),
                                                     N_.stream(Z.device)), "mlp_bias_sigmoid")
        return Z
    return torch.sigmoid_(Z.add_(b[:, None, :]))


def _sigmoid_backprop_(D: torch.Tensor, A: torch.Tensor) -> torch.Tensor:
    """``D <- D * A (1 - A)`` in place; returns the column sums of the result ``[P, B]`` in fp64."""
    P, N, B = D.shape
    if D.is_cuda:
        from ..ops import _native as N_
        nblk = max(1, min(256, (N + 2047) // 2048))
        part = torch.empty(P, nblk, B, dtype=torch.float64, device=D.device)
        N_.check(N_.hip().tmog_hip_mlp_sigmoid_backprop(N_.ptr(D), N_.ptr(A), P, N, B, nblk, N_.ptr(part),
                                                        N_.stream(D.device)), "mlp_sigmoid_backprop")
        return part.sum(1)
    D.mul_(A * (1 - A))
    return D.sum(1, dtype=torch.float64)


class MLPObjective:
    """Weighted mean cross-entropy of P MLPs with the same layer sizes over the shared ``X`` (row weights
    ``W [N, P]``), as ``linear.owlqn_batched`` expects: ``value(U)`` / ``value_grad(U)`` with ``U [n_params, P]``
    (per layer: the ``a x b`` weights row-major, then the ``b`` biases)."""

    def __init__(self, X: torch.Tensor, y: torch.Tensor, W: torch.Tensor, layers: Sequence[int]):
        self.X = X.to(torch.float32).contiguous()
        self.N = int(X.shape[0])
        self.yi = y.to(device=X.device, dtype=torch.int64)
        self.yf = self.yi.to(torch.float32).contiguous()
        self.W = W.to(device=X.device, dtype=torch.float32).contiguous()
        self.wsum = self.W.sum(0, dtype=torch.float64).clamp_min(1e-300)
        self.layers = [int(v) for v in layers]
        self.nl = len(self.layers) - 1
        self.K = self.layers[-1]
        self.slices: List[Tuple[int, int, int, int]] = []     # (weight offset, a, b, bias offset)
        o = 0
        for a, b in zip(self.layers[:-1], self.layers[1:]):
            self.slices.append((o, a, b, o + a * b))
            o += a * b + b
        self.n_params = o
        self.passes = 0

    def _unpack(self, U: torch.Tensor):
        P = U.shape[1]
        return [(U[o:o + a * b].t().reshape(P, a, b).to(torch.float32).contiguous(),
                 U[ob:ob + b].t().to(torch.float32).contiguous()) for o, a, b, ob in self.slices]

    def _output(self, logits: torch.Tensor, bL: torch.Tensor, grad: bool):
        """Weighted CE sums ``[P]`` (fp64) and, with ``grad``, ``W (softmax - onehot) [P, N, K]``."""
        P, N, K = logits.shape
        M = logits.permute(1, 0, 2).contiguous().view(N, P * K)
        if M.is_cuda:
            from ..ops import linear as LK
            f, _ = LK.softmax_objective(M, self.yf, self.W, bL.reshape(-1), P, K, grad)
            return f, (M.view(N, P, K).permute(1, 0, 2) if grad else None)
        Z = M.view(N, P, K) + bL[None]
        lse = torch.logsumexp(Z, -1)
        my = Z.gather(2, self.yi.clamp(0, K - 1)[:, None, None].expand(N, P, 1)).squeeze(2)
        f = (self.W * (lse - my)).sum(0, dtype=torch.float64)
        if not grad:
            return f, None
        R = torch.softmax(Z, -1)
        R[torch.arange(N, device=Z.device), :, self.yi.clamp(0, K - 1)] -= 1.0
        return f, (R * self.W[..., None]).permute(1, 0, 2)

    def _pass(self, U: torch.Tensor, grad: bool):
        self.passes += 1
        params = self._unpack(U)
        acts = []
        H = None
        from ..ops import dense as DN
        mfma = self.X.is_cuda and DN.enabled()
        for i, (Wl, bl) in enumerate(params[:-1]):
            if mfma:        # layer product + bias + sigmoid in one matrix-core launch (dense_kernels.hip)
                H = DN.layer_shared(self.X, Wl, bl, True) if i == 0 else DN.layer_batched(H, Wl, bl, True)
            else:
                Z = (torch.matmul(self.X, Wl) if i == 0 else torch.bmm(H, Wl)).contiguous()
                H = _bias_sigmoid_(Z, bl)
            acts.append(H)
        WL, bL = params[-1]
        if mfma:
            logits = DN.layer_shared(self.X, WL, None, False) if self.nl == 1 else DN.layer_batched(H, WL, None, False)
        else:
            logits = torch.matmul(self.X, WL) if self.nl == 1 else torch.bmm(H, WL)
        f, R = self._output(logits, bL, grad)
        f = f / self.wsum
        if not grad:
            return f, None
        P = U.shape[1]
        g = torch.empty_like(U)
        dZ = (R / self.wsum.to(torch.float32)[:, None, None]).contiguous()       # [P, N, K]
        db = dZ.sum(1, dtype=torch.float64)
        for i in range(self.nl - 1, -1, -1):
            o, a, b, ob = self.slices[i]
            Hin = acts[i - 1] if i > 0 else None
            if mfma:        # fp32 matrix-core chunks, fp64 across chunks
                dW = DN.grad_shared(self.X, dZ) if i == 0 else DN.grad_batched(Hin, dZ)                # [P, a, b]
            else:
                dW = torch.matmul(self.X.t(), dZ) if i == 0 else torch.bmm(Hin.transpose(1, 2), dZ)
            g[o:o + a * b] = dW.reshape(P, a * b).t().to(U.dtype)
            g[ob:ob + b] = db.t().to(U.dtype)
            if i > 0:
                dH = DN.backprop_input(dZ, params[i][0]) if mfma else \
                    torch.bmm(dZ, params[i][0].transpose(1, 2)).contiguous()                        # [P, N, a]
                db = _sigmoid_backprop_(dH, Hin)
                dZ = dH
        return f, g

    def value(self, U):
        return self._pass(U, False)[0]

    def value_grad(self, U):
        return self._pass(U, True)


def _init_params(layers: Sequence[int], seed: int) -> np.ndarray:
    """Glorot-uniform weights, zero biases, from a per-job seed (flattened in ``MLPObjective`` order)."""
    g = torch.Generator(device="cpu").manual_seed(int(seed))
    parts = []
    for a, b in zip(layers[:-1], layers[1:]):
        lim = float(np.sqrt(6.0 / (a + b)))
        parts.append(((torch.rand(a, b, generator=g, dtype=torch.float64) * 2 - 1) * lim).reshape(-1))
        parts.append(torch.zeros(b, dtype=torch.float64))
    return torch.cat(parts).numpy()


@register_learner
class MultilayerPerceptronClassifierLearner(Learner):
    name = "OpMultilayerPerceptronClassifier"
    defaults = {"layers": None, "max_iter": 100, "tol": 1e-6, "seed": 0, "step_size": 0.03,
                "solver": "l-bfgs", "block_size": 128}

    def fit_batch(self, X, y, jobs, context=None) -> List[dict]:
        from .linear import _fold_weights, owlqn_batched
        K = int(y.max().item()) + 1 if y.numel() else 2
        K = max(K, 2)
        dev = X.device
        groups: Dict[tuple, List[int]] = {}
        layer_of = []
        for i, j in enumerate(jobs):
            layers = list(j.params.get("layers") or [X.shape[1], max(4, X.shape[1] // 2), K])
            if layers[0] != X.shape[1] or layers[-1] < K:
                raise ValueError(f"MLP layers {layers} do not match input width {X.shape[1]} / {K} classes")
            layer_of.append(layers)
            groups.setdefault(tuple(layers), []).append(i)
        out: List[dict] = [None] * len(jobs)
        for layers, idx in groups.items():
            gj = [jobs[i] for i in idx]
            W = _fold_weights(X.shape[0], gj, dev, torch.float32)
            obj = MLPObjective(X, y, W, layers)
            U0 = torch.as_tensor(np.stack([_init_params(layers, int(j.params.get("seed", 0))) for j in gj], 1),
                                 dtype=torch.float64, device=dev)
            l1 = torch.zeros_like(U0)
            mi = torch.as_tensor([int(j.params.get("max_iter", 100)) for j in gj], dtype=torch.int64, device=dev)
            tol = torch.as_tensor([float(j.params.get("tol", 1e-6)) for j in gj], dtype=torch.float64, device=dev)
            U, _, _ = owlqn_batched(obj, U0, l1, mi, tol)
            Uc = U.cpu()
            for c, i in enumerate(idx):
                ws = []
                for o, a, b, ob in obj.slices:
                    ws.append(Uc[o:o + a * b, c].reshape(a, b).to(torch.float32).numpy())
                    ws.append(Uc[ob:ob + b, c].to(torch.float32).numpy())
                out[i] = {"layers": list(layers), "weights": ws, "n_classes": K}
        return out

    def predict(self, state, X, context=None):
        ps = [torch.as_tensor(w, device=X.device) for w in state["weights"]]
        with torch.no_grad():
            raw = _forward(ps, X.to(torch.float32), len(state["layers"]) - 1).to(torch.float64)
        prob = torch.softmax(raw, 1)
        return torch.argmax(raw, 1).to(torch.float64), raw, prob


@register_stage
class OpMultilayerPerceptronClassifier(OpPredictor):
    operation_name = "OpMultilayerPerceptronClassifier"
    learner_cls = MultilayerPerceptronClassifierLearner

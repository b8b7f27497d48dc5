"""Multilayer perceptron classifier (``classification/OpMultilayerPerceptronClassifier.scala:49-144``; Spark
``MultilayerPerceptronClassifier``: sigmoid hidden layers, softmax output, L-BFGS on the cross-entropy).
SURVEY.md K27: the layer products are plain GEMMs on the matrix cores (hipBLASLt via torch); all rows
of a fold are one batch (Spark's ``blockSize`` only stacks rows into matrices for BLAS).
"""
from __future__ import annotations

from typing import List

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


@register_learner
class MultilayerPerceptronClassifierLearner(Learner):
    name = "OpMultilayerPerceptronClassifier"
    defaults = {"layers": None, "max_iter": 100, "tol": 1e-6, "seed": 0, "step_size": 0.03,
                "solver": "l-bfgs", "block_size": 128}

    def fit_batch(self, X, y, jobs, context=None) -> List[dict]:
        out = []
        K = int(y.max().item()) + 1 if y.numel() else 2
        K = max(K, 2)
        for j in jobs:
            p = j.params
            rows = j.rows if j.rows is not None else torch.arange(X.shape[0], device=X.device)
            Xr = X.index_select(0, rows.to(X.device)).to(torch.float32)
            yr = y.index_select(0, rows.to(y.device)).to(torch.int64).to(X.device)
            layers = list(p.get("layers") or [X.shape[1], max(4, X.shape[1] // 2), K])
            if layers[0] != X.shape[1] or layers[-1] < K:
                raise ValueError(f"MLP layers {layers} do not match input width {X.shape[1]} / {K} classes")
            g = torch.Generator(device="cpu").manual_seed(int(p.get("seed", 0)))
            params = []
            for a, b in zip(layers[:-1], layers[1:]):
                lim = float(np.sqrt(6.0 / (a + b)))
                params.append(((torch.rand(a, b, generator=g) * 2 - 1) * lim).to(X.device).requires_grad_())
                params.append(torch.zeros(b, device=X.device).requires_grad_())
            nl = len(layers) - 1
            opt = torch.optim.LBFGS(params, lr=1.0, max_iter=int(p.get("max_iter", 100)),
                                    tolerance_grad=float(p.get("tol", 1e-6)), tolerance_change=1e-9,
                                    history_size=10, line_search_fn="strong_wolfe")
            w = None if j.weights is None else j.weights.to(X.device, torch.float32)

            def closure():
                opt.zero_grad()
                logits = _forward(params, Xr, nl)
                l = torch.nn.functional.cross_entropy(logits, yr, reduction="none")
                loss = (l * w).sum() / w.sum() if w is not None else l.mean()
                loss.backward()
                return loss
            opt.step(closure)
            out.append({"layers": layers, "weights": [t.detach().cpu().numpy() for t in params], "n_classes": K})
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

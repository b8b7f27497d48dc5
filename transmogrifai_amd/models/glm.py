"""Generalized linear regression by batched IRLS (``regression/OpGeneralizedLinearRegression.scala:49-203``;
Spark ``GeneralizedLinearRegression`` with the IRLS / weighted-least-squares solver). SURVEY.md K22.

All (grid point x fold) problems advance together: each IRLS step forms the weighted Gram matrices
``X^T W_p X`` of every problem (one batched GEMM chain on the device) and solves the small
``(d+1) x (d+1)`` systems with one batched Cholesky-backed ``torch.linalg.solve``.
"""
from __future__ import annotations

import math
from typing import List

import numpy as np
import torch

from .base import FitJob, Learner, OpPredictor, register_learner
from ..stages.base import register_stage

# family -> (variance fn, supported links, canonical link)
FAMILIES = {
    "gaussian": (lambda mu, p: torch.ones_like(mu), ("identity", "log", "inverse"), "identity"),
    "binomial": (lambda mu, p: mu * (1 - mu), ("logit", "probit", "cloglog"), "logit"),
    "poisson": (lambda mu, p: mu, ("log", "identity", "sqrt"), "log"),
    "gamma": (lambda mu, p: mu * mu, ("inverse", "identity", "log"), "inverse"),
    "tweedie": (lambda mu, p: mu.abs() ** p, ("power",), "power"),
}


def _link(name: str, link_power: float = 0.0):
    """(g, g^-1, g') for a link name."""
    if name == "identity":
        return (lambda m: m), (lambda e: e), (lambda m: torch.ones_like(m))
    if name == "log":
        return torch.log, torch.exp, (lambda m: 1.0 / m)
    if name == "inverse":
        return (lambda m: 1.0 / m), (lambda e: 1.0 / e), (lambda m: -1.0 / (m * m))
    if name == "logit":
        return (lambda m: torch.log(m / (1 - m))), torch.sigmoid, (lambda m: 1.0 / (m * (1 - m)))
    if name == "probit":
        nd = torch.distributions.Normal(0.0, 1.0)
        return (lambda m: nd.icdf(m)), (lambda e: nd.cdf(e)), (lambda m: 1.0 / torch.exp(nd.log_prob(nd.icdf(m))))
    if name == "cloglog":
        return (lambda m: torch.log(-torch.log1p(-m))), (lambda e: 1 - torch.exp(-torch.exp(e))), \
            (lambda m: 1.0 / ((m - 1) * torch.log1p(-m)))
    if name == "sqrt":
        return torch.sqrt, (lambda e: e * e), (lambda m: 0.5 / torch.sqrt(m))
    if name == "power":
        lp = link_power
        if lp == 0:
            return _link("log")
        return (lambda m: m ** lp), (lambda e: e.clamp_min(1e-12) ** (1.0 / lp)), (lambda m: lp * m ** (lp - 1))
    raise ValueError(f"unsupported link {name}")


def _init_mu(family, y):
    if family == "binomial":
        return (y + 0.5) / 2.0
    if family in ("poisson", "gamma", "tweedie"):
        return torch.where(y > 0, y, torch.full_like(y, 0.1))
    return y.clone()


@register_learner
class GeneralizedLinearRegressionLearner(Learner):
    name = "OpGeneralizedLinearRegression"
    problem = "regression"
    defaults = {"family": "gaussian", "link": None, "reg_param": 0.0, "max_iter": 25, "tol": 1e-6,
                "fit_intercept": True, "variance_power": 0.0, "link_power": None}

    def fit_batch(self, X, y, jobs, context=None) -> List[dict]:
        out = []
        # problems sharing (family, link) iterate together
        groups = {}
        for i, j in enumerate(jobs):
            fam = j.params.get("family", "gaussian")
            if fam not in FAMILIES:
                raise ValueError(f"unsupported family {fam}")
            link = j.params.get("link") or FAMILIES[fam][2]
            if link not in FAMILIES[fam][1] and not (fam == "tweedie"):
                raise ValueError(f"family {fam} does not support link {link}")
            groups.setdefault((fam, link, float(j.params.get("variance_power", 0.0)),
                               j.params.get("link_power")), []).append(i)
        res = [None] * len(jobs)
        for (fam, link, vp, lp), idxs in groups.items():
            sub = [jobs[i] for i in idxs]
            for i, r in zip(idxs, self._irls(X, y, sub, fam, link, vp, lp)):
                res[i] = r
        return res

    def _irls(self, X, y, jobs, fam, link, vp, lp):
        dev = X.device
        N, d = X.shape
        P = len(jobs)
        Xd = X.to(torch.float64)
        yd = y.to(torch.float64)
        W0 = torch.zeros(N, P, dtype=torch.float64, device=dev)
        for p, j in enumerate(jobs):
            if j.rows is None:
                W0[:, p] = 1.0 if j.weights is None else j.weights.to(torch.float64)
            else:
                W0[j.rows.to(dev), p] = 1.0 if j.weights is None else j.weights.to(dev, torch.float64)
        fi = torch.tensor([bool(j.params.get("fit_intercept", True)) for j in jobs], device=dev)
        reg = torch.tensor([float(j.params.get("reg_param", 0.0)) for j in jobs], dtype=torch.float64, device=dev)
        max_iter = max(int(j.params.get("max_iter", 25)) for j in jobs)
        tol = min(float(j.params.get("tol", 1e-6)) for j in jobs)
        link_power = (1.0 - vp) if (fam == "tweedie" and lp is None) else (lp or 0.0)
        g, ginv, gprime = _link(link, link_power)
        var = FAMILIES[fam][0]
        Xa = torch.cat([Xd, torch.ones(N, 1, dtype=torch.float64, device=dev)], 1)     # [N, d+1]
        from ..ops.stats import weighted_gram
        Xg = X if (X.is_cuda and X.dtype == torch.float32) else Xd      # the Gram kernel widens fp32 itself
        # weighted column sums and sums of squares of every problem: row d and the diagonal of [X | 1]'s Gram
        G0 = weighted_gram(Xg, W0)
        wsum = W0.sum(0).clamp_min(1e-300)
        mean = G0[:, :d, d].t() / wsum[None, :]
        var_x = torch.diagonal(G0[:, :d, :d], dim1=1, dim2=2).t() / wsum[None, :] - mean * mean
        mu = _init_mu(fam, yd)[:, None].expand(N, P).clone()
        beta = torch.zeros(d + 1, P, dtype=torch.float64, device=dev)
        it = 0
        from ..utils.cancel import check as _cancel_check
        for it in range(1, max_iter + 1):
            _cancel_check()
            eta = g(mu)
            gp = gprime(mu)
            z = eta + (yd[:, None] - mu) * gp
            w = W0 / (gp * gp * var(mu, vp)).clamp_min(1e-300)
            w = torch.nan_to_num(w, nan=0.0, posinf=0.0)
            # batched weighted normal equations: the Gram of [X | 1 | z_p] under w_p holds both
            # A_p = Xa^T W_p Xa and b_p = Xa^T W_p z_p (fp64 matrix cores, one pass for all problems)
            Gz = weighted_gram(Xg, w, z)
            A = Gz[:, :d + 1, :d + 1].contiguous()
            b = Gz[:, :d + 1, d + 1].contiguous()
            pen = torch.zeros(P, d + 1, dtype=torch.float64, device=dev)
            pen[:, :d] = (reg * wsum)[:, None] * var_x.t().clamp_min(0)
            A = A + torch.diag_embed(pen)
            nofi = ~fi
            if bool(nofi.any()):
                A[nofi, d, :] = 0
                A[nofi, :, d] = 0
                A[nofi, d, d] = 1
                b[nofi, d] = 0
            nb = torch.linalg.solve(A + 1e-12 * torch.eye(d + 1, dtype=torch.float64, device=dev), b).t()
            delta = (nb - beta).abs().max()
            beta = nb
            mu = ginv(Xa @ beta)
            if fam == "binomial":
                mu = mu.clamp(1e-12, 1 - 1e-12)
            elif fam in ("poisson", "gamma", "tweedie"):
                mu = mu.clamp_min(1e-12)
            if float(delta) < tol:
                break
        bt = beta.t().cpu().numpy()
        return [{"coefficients": bt[p, :d].copy(), "intercept": float(bt[p, d]), "family": fam, "link": link,
                 "link_power": float(link_power), "n_iter": it} for p in range(P)]

    def predict(self, state, X, context=None):
        c = torch.as_tensor(state["coefficients"], dtype=torch.float64, device=X.device)
        eta = X.to(torch.float64) @ c + state["intercept"]
        _, ginv, _ = _link(state["link"], state.get("link_power", 0.0))
        mu = ginv(eta)
        e = torch.zeros(mu.shape[0], 0, dtype=torch.float64, device=X.device)
        return mu, e, e

    def feature_contributions(self, state, d):
        return np.asarray(state["coefficients"], np.float64)


@register_stage
class OpGeneralizedLinearRegression(OpPredictor):
    operation_name = "OpGeneralizedLinearRegression"
    learner_cls = GeneralizedLinearRegressionLearner

"""Evaluation metric kernels (device-resident).

Binary curves follow Spark ``BinaryClassificationMetrics`` (used by ``OpBinaryClassificationEvaluator.scala:67-135``
and the selector's ``BinaryClassificationEvaluator`` metric at ``:149-155``): distinct scores sorted
descending, optional down-sampling into ``numBins`` groups (each group keyed by its first score),
cumulative confusion counts, PR curve prefixed with ``(0, precision_first)``, ROC with ``(0,0)`` and
``(1,1)`` end points, trapezoidal areas. Everything runs as sort + segmented reductions on the
tensors' device.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Sequence

import numpy as np
import torch


def _curve_counts(scores: torch.Tensor, labels: torch.Tensor, num_bins: int = 0, weights=None):
    s = scores.to(torch.float64).reshape(-1)
    y = labels.to(torch.float64).reshape(-1)
    w = torch.ones_like(s) if weights is None else weights.to(torch.float64)
    s, order = torch.sort(s, descending=True, stable=True)
    y, w = y[order], w[order]
    # segmented sums over runs of equal scores without atomics: the input is sorted, so the per-run
    # totals are differences of the running sums at the run ends (run ends found by a neighbour
    # compare + one compaction; torch.unique_consecutive is ~10x slower on ROCm at 3M rows)
    is_end = torch.ones(s.numel(), dtype=torch.bool, device=s.device)
    if s.numel() > 1:
        is_end[:-1] = s[1:] != s[:-1]
    ends = is_end.nonzero().squeeze(1)
    uniq = s[ends]
    n_u = uniq.numel()
    cpos = torch.cumsum(w * (y > 0.5), 0)
    cneg = torch.cumsum(w * (y <= 0.5), 0)
    tp_end, fp_end = cpos[ends], cneg[ends]
    thr = uniq
    if num_bins > 0:
        grouping = n_u // num_bins
        if grouping >= 2:
            # groups of ``grouping`` consecutive distinct scores, keyed by their first score
            last = torch.arange(grouping - 1, n_u, grouping, device=s.device)
            if last.numel() == 0 or int(last[-1]) != n_u - 1:
                last = torch.cat([last, torch.tensor([n_u - 1], device=s.device)])
            thr = uniq[torch.arange(last.numel(), device=s.device) * grouping]
            tp_end, fp_end = tp_end[last], fp_end[last]
    tp, fp = tp_end, fp_end
    P = float(tp[-1]) if tp.numel() else 0.0
    Nn = float(fp[-1]) if fp.numel() else 0.0
    return thr, tp, fp, P, Nn


def _trapz(x, y):
    if x.numel() < 2:
        return 0.0
    return float(((x[1:] - x[:-1]) * (y[1:] + y[:-1]) / 2.0).sum())


def binary_curves(scores, labels, num_bins: int = 0, weights=None) -> Dict[str, object]:
    thr, tp, fp, P, Nn = _curve_counts(scores, labels, num_bins, weights)
    prec = torch.where(tp + fp > 0, tp / (tp + fp).clamp_min(1e-300), torch.ones_like(tp))
    rec = tp / P if P > 0 else torch.zeros_like(tp)
    fpr = fp / Nn if Nn > 0 else torch.zeros_like(fp)
    dev = tp.device
    pr_x = torch.cat([torch.zeros(1, dtype=torch.float64, device=dev), rec])
    pr_y = torch.cat([prec[:1] if prec.numel() else torch.ones(1, dtype=torch.float64, device=dev), prec])
    roc_x = torch.cat([torch.zeros(1, dtype=torch.float64, device=dev), fpr,
                       torch.ones(1, dtype=torch.float64, device=dev)])
    roc_y = torch.cat([torch.zeros(1, dtype=torch.float64, device=dev), rec,
                       torch.ones(1, dtype=torch.float64, device=dev)])
    return {"thresholds": thr, "tp": tp, "fp": fp, "P": P, "N": Nn, "precision": prec, "recall": rec, "fpr": fpr,
            "AuPR": _trapz(pr_x, pr_y), "AuROC": _trapz(roc_x, roc_y)}


def _segmented_sort_desc(S: torch.Tensor):
    """Rows of ``S [J, n]`` sorted descending (fp64 values, column indices) with flat 1-D radix sorts --
    ``torch.sort(dim=1)`` over a few multi-million-element rows is several times slower on ROCm than one
    sort of all J*n keys. fp32 scores: one sort of the int64 key (row << 32 | descending order bits of the
    float). Otherwise a stable value sort followed by a stable sort by row id."""
    J, n = S.shape
    dev = S.device
    if S.dtype == torch.float32:
        b = S.contiguous().view(torch.int32).to(torch.int64)
        asc = torch.where(b < 0, b ^ 0x7FFFFFFF, b) + (1 << 31)          # float order -> [0, 2^32)
        key = torch.arange(J, device=dev, dtype=torch.int64)[:, None] * (1 << 32) + ((1 << 32) - 1 - asc)
        flat = torch.sort(key.reshape(-1), stable=True).indices
    else:
        v = S.to(torch.float64).reshape(-1)
        o1 = torch.sort(v, descending=True, stable=True).indices
        seg = torch.div(o1, n, rounding_mode="floor")
        flat = o1[torch.sort(seg, stable=True).indices]
    order = (flat % n).view(J, n)
    s = S.to(torch.float64).reshape(-1)[flat].view(J, n)
    return s, order


def binary_areas_device(S: torch.Tensor, labels: torch.Tensor):
    """Exact AuPR and AuROC of the ``J`` score sets ``S [J, n]`` over the same labelled rows on the GPU: the
    segment-major descending order from flat radix sorts (:func:`_segmented_sort_desc`: one packed-key sort for
    fp32 scores; fp64: a value sort, then a stable sort of the small segment ids), then one HIP workgroup per
    score set walks its sorted scores and sums the trapezoids (``ops/csrc/hip/metric_kernels.hip``) -- one
    launch for all curves instead of ~15 torch ops and a host synchronisation per model. Same points as
    :func:`binary_curves`. Returns two fp64 ``[J]`` tensors on the device."""
    from ..ops import _native as NV
    J, n = S.shape
    dev = S.device
    if S.dtype == torch.float32:
        b = S.contiguous().view(torch.int32).to(torch.int64)
        asc = torch.where(b < 0, b ^ 0x7FFFFFFF, b) + (1 << 31)
        key = torch.arange(J, device=dev, dtype=torch.int64)[:, None] * (1 << 32) + ((1 << 32) - 1 - asc)
        flat = torch.sort(key.reshape(-1), stable=True).indices
        v = S.reshape(-1)
    else:
        v = S.to(torch.float64).reshape(-1)
        o1 = torch.sort(v, descending=True, stable=True).indices
        seg = torch.div(o1, n, rounding_mode="floor")
        seg = seg.to(torch.int16 if J < (1 << 15) else torch.int32)      # fewer radix passes
        flat = o1[torch.sort(seg, stable=True).indices]
    s_sorted = v[flat].contiguous()
    idx = (flat % n).contiguous()
    lab = (labels.to(dev).reshape(-1) > 0.5).to(torch.uint8).contiguous()
    pr = torch.empty(J, dtype=torch.float64, device=dev)
    roc = torch.empty(J, dtype=torch.float64, device=dev)
    NV.check(NV.hip().tmog_hip_binary_areas(NV.ptr(s_sorted), int(s_sorted.dtype == torch.float64), NV.ptr(idx), int(n),
                                            int(J), NV.ptr(lab), NV.ptr(pr), NV.ptr(roc), NV.stream(dev)),
             "binary_areas")
    return pr, roc


def binary_areas_batch(S: torch.Tensor, labels: torch.Tensor, chunk_elems: int = 1 << 27):
    """Exact (``numBins = 0``) AuPR and AuROC of ``J`` score sets over the same labelled rows, ``S [J, n]``:
    one segmented sort along the rows (``torch.sort(dim=1)``) and vectorised run-end / cumulative-count /
    trapezoid passes for all curves at once, instead of one sort + curve build per model.
    Same points as :func:`binary_curves` (distinct scores descending; PR prefixed with ``(0, precision_first)``,
    ROC with ``(0, 0)``), so the areas agree to fp64 rounding. Returns two fp64 ``[J]`` tensors."""
    J, n = S.shape
    dev = S.device
    if n == 0 or J == 0:
        z = torch.zeros(J, dtype=torch.float64, device=dev)
        return z, z
    y = (labels.to(dev).reshape(-1) > 0.5)
    rows = max(1, min(J, chunk_elems // max(n, 1)))
    aupr, auroc = [], []
    for a in range(0, J, rows):
        s, order = _segmented_sort_desc(S[a:a + rows])
        pos = y[order].to(torch.float64)
        tp = torch.cumsum(pos, 1)
        fp = torch.cumsum(1.0 - pos, 1)
        is_end = torch.ones_like(s, dtype=torch.bool)
        if n > 1:
            is_end[:, :-1] = s[:, 1:] != s[:, :-1]
        Ptot, Ntot = tp[:, -1:], fp[:, -1:]
        # previous run end of every position: the last is_end index strictly before it (-1 = none)
        idx = torch.arange(n, device=dev).expand_as(s)
        last_end = torch.cummax(torch.where(is_end, idx, torch.full_like(idx, -1)), 1).values
        prev = torch.full_like(last_end, -1)
        prev[:, 1:] = last_end[:, :-1]
        has_prev = prev >= 0
        pidx = prev.clamp_min(0)
        tp_p = torch.where(has_prev, tp.gather(1, pidx), torch.zeros_like(tp))
        fp_p = torch.where(has_prev, fp.gather(1, pidx), torch.zeros_like(fp))
        prec = torch.where(tp + fp > 0, tp / (tp + fp).clamp_min(1e-300), torch.ones_like(tp))
        rec = torch.where(Ptot > 0, tp / Ptot.clamp_min(1e-300), torch.zeros_like(tp))
        # the PR curve starts at (0, precision of the first run end)
        first = torch.argmax(is_end.to(torch.int8), 1, keepdim=True)
        prec_first = prec.gather(1, first)
        prec_p = torch.where(has_prev, torch.where(tp_p + fp_p > 0, tp_p / (tp_p + fp_p).clamp_min(1e-300),
                                                   torch.ones_like(tp_p)), prec_first.expand_as(prec))
        rec_p = torch.where(Ptot > 0, tp_p / Ptot.clamp_min(1e-300), torch.zeros_like(tp_p))
        e = is_end.to(torch.float64)
        aupr.append(((rec - rec_p) * (prec + prec_p) / 2.0 * e).sum(1))
        fpr = torch.where(Ntot > 0, fp / Ntot.clamp_min(1e-300), torch.zeros_like(fp))
        fpr_p = torch.where(Ntot > 0, fp_p / Ntot.clamp_min(1e-300), torch.zeros_like(fp_p))
        roc = ((fpr - fpr_p) * (rec + rec_p) / 2.0 * e).sum(1)
        # closing (1, 1) point after the last run end
        last_fpr, last_rec = fpr[:, -1], rec[:, -1]
        roc = roc + (1.0 - last_fpr) * (1.0 + last_rec) / 2.0
        auroc.append(roc)
    return torch.cat(aupr), torch.cat(auroc)


def au_pr(scores, labels, num_bins: int = 0) -> float:
    return binary_curves(scores, labels, num_bins)["AuPR"]


def au_roc(scores, labels, num_bins: int = 0) -> float:
    return binary_curves(scores, labels, num_bins)["AuROC"]


def binned_aupr(scores: torch.Tensor, labels: torch.Tensor, bins: int = 1 << 16) -> float:
    """O(N) histogram approximation of AuPR for scores in [0, 1] (early-stopping monitor)."""
    s = scores.to(torch.float32).clamp(0, 1)
    b = (s * (bins - 1)).to(torch.int64)
    y = labels > 0.5
    pos = torch.bincount(b[y], minlength=bins).flip(0).to(torch.float64)
    neg = torch.bincount(b[~y], minlength=bins).flip(0).to(torch.float64)
    keep = (pos + neg) > 0
    pos, neg = pos[keep], neg[keep]
    tp, fp = torch.cumsum(pos, 0), torch.cumsum(neg, 0)
    P = float(pos.sum())
    if P == 0:
        return 0.0
    prec = tp / (tp + fp)
    rec = tp / P
    x = torch.cat([torch.zeros(1, dtype=torch.float64, device=rec.device), rec])
    yv = torch.cat([prec[:1], prec])
    return _trapz(x, yv)


def binned_aupr_multi(scores: Sequence[torch.Tensor], labels: Sequence[torch.Tensor],
                      bins: int = 1 << 16) -> torch.Tensor:
    """``binned_aupr`` of several (scores, labels) sets at once, on the device, without host syncs:
    one bincount over (set, label, bin), cumulative counts per set, trapezoids. Returns fp64 ``[K]``."""
    K = len(scores)
    dev = scores[0].device
    sid = torch.cat([torch.full((s.numel(),), k, dtype=torch.int64, device=dev) for k, s in enumerate(scores)])
    s = torch.cat([x.reshape(-1) for x in scores]).to(torch.float32).clamp(0, 1)
    y = torch.cat([x.reshape(-1) for x in labels]).to(dev) > 0.5
    b = (s * (bins - 1)).to(torch.int64)
    idx = (sid * 2 + y.to(torch.int64)) * bins + (bins - 1 - b)        # descending score order
    h = torch.bincount(idx, minlength=K * 2 * bins).view(K, 2, bins)
    return binned_aupr_from_counts(h)


def binned_aupr_from_counts(h: torch.Tensor) -> torch.Tensor:
    """AuPR of ``K`` score sets from their ``[K, 2 (label), bins]`` count tables, bins in descending
    score order (as filled by :func:`binned_aupr_multi` or the fused boosting-round kernel)."""
    K = h.shape[0]
    dev = h.device
    if dev.type == "cuda" and K > 0 and h.dtype == torch.int32:
        # one HIP launch (ops/csrc/hip/boost_kernels.hip aupr_counts_kernel), same per-bin arithmetic
        from ..ops import _native as NV
        hc = h.contiguous()
        out = torch.empty(K, dtype=torch.float64, device=dev)
        NV.check(NV.hip().tmog_hip_aupr_counts(NV.ptr(hc), int(K), int(hc.shape[2]), NV.ptr(out), NV.stream(dev)),
                 "aupr_counts")
        return out
    return _aupr_from_counts_torch(h)


def _aupr_from_counts_torch(h: torch.Tensor) -> torch.Tensor:
    K = h.shape[0]
    dev = h.device
    h = h.to(torch.float64)
    neg, pos = h[:, 0], h[:, 1]
    tp, fp = torch.cumsum(pos, 1), torch.cumsum(neg, 1)
    P = tp[:, -1:]
    cnt = tp + fp
    prec = tp / cnt.clamp_min(1)
    first = torch.argmax((cnt > 0).to(torch.int8), 1, keepdim=True)
    prec = torch.where(cnt > 0, prec, prec.gather(1, first))        # empty leading bins: width-0 points
    rec = tp / P.clamp_min(1)
    x = torch.cat([torch.zeros(K, 1, dtype=torch.float64, device=dev), rec], 1)
    yv = torch.cat([prec.gather(1, first), prec], 1)
    area = ((x[:, 1:] - x[:, :-1]) * (yv[:, 1:] + yv[:, :-1]) * 0.5).sum(1)
    return torch.where(P[:, 0] > 0, area, torch.zeros_like(area))


def confusion_at(pred: torch.Tensor, labels: torch.Tensor):
    p = pred.to(torch.float64) > 0.5
    y = labels.to(torch.float64) > 0.5
    tp = float((p & y).sum())
    tn = float((~p & ~y).sum())
    fp = float((p & ~y).sum())
    fn = float((~p & y).sum())
    return tp, tn, fp, fn


def binary_classification_metrics(pred, prob1, labels, num_bins: int = 100) -> Dict[str, object]:
    """``OpBinaryClassificationEvaluator.evaluateAll`` (``OpBinaryClassificationEvaluator.scala:67-135``)."""
    n = int(labels.numel())
    if n == 0:
        z = {k: 0.0 for k in ("Precision", "Recall", "F1", "AuROC", "AuPR", "Error", "TP", "TN", "FP", "FN")}
        z["ThresholdMetrics"] = {"thresholds": [], "precisionByThreshold": [], "recallByThreshold": [],
                                 "falsePositiveRateByThreshold": [], "truePositivesByThreshold": [],
                                 "falsePositivesByThreshold": [], "trueNegativesByThreshold": [],
                                 "falseNegativesByThreshold": []}
        return z
    labs = torch.unique(labels.to(torch.float64))
    if labs.numel() == 2 or True:
        tp, tn, fp, fn = confusion_at(pred, labels)
    precision = 0.0 if tp + fp == 0 else tp / (tp + fp)
    recall = 0.0 if tp + fn == 0 else tp / (tp + fn)
    f1 = 0.0 if precision + recall == 0 else 2 * precision * recall / (precision + recall)
    error = 0.0 if n == 0 else (fp + fn) / n
    c = binary_curves(prob1, labels, num_bins)
    P, Nn = c["P"], c["N"]
    tpt, fpt = c["tp"], c["fp"]
    return {"Precision": precision, "Recall": recall, "F1": f1, "AuROC": c["AuROC"], "AuPR": c["AuPR"],
            "Error": error, "TP": tp, "TN": tn, "FP": fp, "FN": fn,
            "ThresholdMetrics": {
                "thresholds": c["thresholds"].tolist(), "precisionByThreshold": c["precision"].tolist(),
                "recallByThreshold": c["recall"].tolist(), "falsePositiveRateByThreshold": c["fpr"].tolist(),
                "truePositivesByThreshold": tpt.tolist(), "falsePositivesByThreshold": fpt.tolist(),
                "trueNegativesByThreshold": (Nn - fpt).tolist(), "falseNegativesByThreshold": (P - tpt).tolist()}}


def bin_score_metrics(prob1, labels, num_bins: int = 100) -> Dict[str, object]:
    """``OpBinScoreEvaluator.evaluateScoreAndLabels`` (``OpBinScoreEvaluator.scala:60-173``): Brier score + bins."""
    s = prob1.to(torch.float64)
    y = labels.to(torch.float64)
    if s.numel() == 0:
        return {"BrierScore": 0.0, "binSize": 0.0, "binCenters": [], "numberOfDataPoints": [],
                "numberOfPositiveLabels": [], "averageScore": [], "averageConversionRate": []}
    mx = max(1.0, float(s.max()))
    mn = min(0.0, float(s.min()))
    diff = mx - mn
    idx = torch.clamp((num_bins * (s - mn) / diff).to(torch.int64), max=num_bins - 1)
    cnt = torch.bincount(idx, minlength=num_bins).to(torch.float64)
    # weighted bincount accumulates per-workgroup in LDS first (fp64 index_add_ on 100 bins is a global
    # atomic storm: 210 ms per call at 10M rows on MI355X, see profiles/README.md)
    ssum = torch.bincount(idx, weights=s, minlength=num_bins)[:num_bins]
    psum = torch.bincount(idx, weights=(y > 0).to(torch.float64), minlength=num_bins)[:num_bins]
    brier = float(((s - y) ** 2).sum() / s.numel())
    avg_s = torch.where(cnt > 0, ssum / cnt.clamp_min(1), torch.zeros_like(cnt))
    avg_c = torch.where(cnt > 0, psum / cnt.clamp_min(1), torch.zeros_like(cnt))
    centers = [mn + diff * i / num_bins + diff / (2 * num_bins) for i in range(num_bins)]
    return {"BrierScore": brier, "binSize": diff / num_bins, "binCenters": centers,
            "numberOfDataPoints": cnt.to(torch.int64).tolist(), "numberOfPositiveLabels": psum.to(torch.int64).tolist(),
            "averageScore": avg_s.tolist(), "averageConversionRate": avg_c.tolist()}


def multiclass_metrics(pred, labels, prob=None, top_ns=(1, 3), thresholds=None) -> Dict[str, object]:
    """``OpMultiClassificationEvaluator.evaluateAll``: error, weighted precision / recall, F1 (+ threshold metrics)."""
    p = pred.to(torch.int64).reshape(-1)
    y = labels.to(torch.int64).reshape(-1)
    n = y.numel()
    if n == 0:
        return {"Precision": 0.0, "Recall": 0.0, "F1": 0.0, "Error": 0.0}
    K = int(max(p.max(), y.max()).item()) + 1
    cm = torch.zeros(K, K, dtype=torch.float64, device=y.device)
    cm.index_put_((y, p), torch.ones(n, dtype=torch.float64, device=y.device), accumulate=True)
    tp = cm.diag()
    actual = cm.sum(1)
    predicted = cm.sum(0)
    prec_c = torch.where(predicted > 0, tp / predicted.clamp_min(1), torch.zeros_like(tp))
    rec_c = torch.where(actual > 0, tp / actual.clamp_min(1), torch.zeros_like(tp))
    wts = actual / n
    precision = float((prec_c * wts).sum())
    recall = float((rec_c * wts).sum())
    f1 = 0.0 if precision + recall == 0 else 2 * precision * recall / (precision + recall)
    out = {"Precision": precision, "Recall": recall, "F1": f1, "Error": 1.0 - float(tp.sum()) / n}
    if prob is not None and prob.numel() and prob.dim() == 2:
        th = thresholds if thresholds is not None else [i / 100 for i in range(101)]
        pr = prob.to(torch.float64)
        top = torch.argsort(pr, 1, descending=True)
        topscore = pr.gather(1, top[:, :1])[:, 0]
        res = {"topNs": list(top_ns), "thresholds": list(th), "correctCounts": {}, "incorrectCounts": {},
               "noPredictionCounts": {}}
        tht = torch.as_tensor(th, dtype=torch.float64, device=pr.device)
        for t in top_ns:
            hit = (top[:, :min(t, pr.shape[1])] == y[:, None]).any(1)
            truescore = pr.gather(1, y.clamp(max=pr.shape[1] - 1)[:, None])[:, 0]
            above_true = truescore[None, :] >= tht[:, None]
            above_top = topscore[None, :] >= tht[:, None]
            correct = (above_true & hit[None, :]).sum(1)
            incorrect = (above_top & ~(above_true & hit[None, :])).sum(1)
            res["correctCounts"][str(t)] = correct.tolist()
            res["incorrectCounts"][str(t)] = incorrect.tolist()
            res["noPredictionCounts"][str(t)] = (n - correct - incorrect).tolist()
        out["ThresholdMetrics"] = res
    return out


DEFAULT_PCT_ERROR_BINS = tuple([float("-inf")] + [float(v) for v in range(-100, 101, 10)] + [float("inf")])


def histogram_counts(x: torch.Tensor, edges) -> list:
    """Spark ``RDD.histogram(buckets)``: bucket i is [e_i, e_{i+1}) except the last, which also takes its right
    edge; values outside [e_0, e_last] and NaNs are not counted."""
    e = torch.as_tensor(list(edges), dtype=torch.float64, device=x.device)
    nb = e.numel() - 1
    if nb <= 0:
        return []
    v = x[~torch.isnan(x)]
    v = v[(v >= e[0]) & (v <= e[-1])]
    idx = torch.clamp(torch.searchsorted(e, v, right=True) - 1, 0, nb - 1)
    return torch.bincount(idx, minlength=nb)[:nb].tolist()


def regression_metrics(pred, labels, bins=DEFAULT_PCT_ERROR_BINS, scaled_error_cutoff=1e-3) -> Dict:
    """``OpRegressionEvaluator``: RMSE, MSE, MAE, R2 and the signed percentage-error histogram
    (100 (prediction - label) / max(|label|, scaledErrorCutoff), ``histogram_counts`` over ``bins``)."""
    p = pred.to(torch.float64).reshape(-1)
    y = labels.to(torch.float64).reshape(-1)
    n = y.numel()
    if n == 0:
        return {"RootMeanSquaredError": 0.0, "MeanSquaredError": 0.0, "R2": 0.0, "MeanAbsoluteError": 0.0,
                "SignedPercentageErrorHistogram": {"bins": list(bins), "counts": [0] * (len(bins) - 1)}}
    e = p - y
    mse = float((e * e).mean())
    ss_tot = float(((y - y.mean()) ** 2).sum())
    r2 = 1.0 - float((e * e).sum()) / ss_tot if ss_tot > 0 else 0.0
    den = torch.clamp(y.abs(), min=float(scaled_error_cutoff))
    pct = 100.0 * e / den
    return {"RootMeanSquaredError": math.sqrt(mse), "MeanSquaredError": mse, "R2": r2,
            "MeanAbsoluteError": float(e.abs().mean()),
            "SignedPercentageErrorHistogram": {"bins": list(bins), "counts": histogram_counts(pct, bins)}}


def forecast_metrics(pred, labels, seasonal_window: int = 1) -> Dict:
    """``OpForecastEvaluator``: SMAPE and MASE."""
    p = pred.to(torch.float64).reshape(-1)
    y = labels.to(torch.float64).reshape(-1)
    n = y.numel()
    if n == 0:
        return {"SMAPE": 0.0, "SeasonalError": 0.0, "MASE": 0.0}
    den = p.abs() + y.abs()
    smape = float(torch.where(den > 0, 2 * (p - y).abs() / den.clamp_min(1e-300), torch.zeros_like(den)).mean())
    if n > seasonal_window:
        se = float((y[seasonal_window:] - y[:-seasonal_window]).abs().mean())
    else:
        se = 0.0
    mae = float((p - y).abs().mean())
    return {"SMAPE": smape, "SeasonalError": se, "MASE": mae / se if se > 0 else 0.0}


def log_loss(prob, labels) -> float:
    """Log loss (``stages/impl/evaluator/OPLogLoss.scala``): mean of -log(probability of the true label), no
    clipping (a zero probability on the true label gives inf, as the reference)."""
    if labels.numel() == 0:
        raise ValueError("requirement failed: Dataset is empty, log loss cannot be calculated")
    pr = prob.to(torch.float64)
    y = labels.to(torch.int64)
    p = pr.gather(1, y[:, None])[:, 0]
    return float(-torch.log(p).mean())

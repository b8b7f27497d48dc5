"""Per-record explanations: leave-one-column-out (LOCO) and score/feature correlation insights.

Reference: ``RecordInsightsLOCO`` (``core/.../stages/impl/insights/RecordInsightsLOCO.scala:100-347``: top-K
by |score change| or top-K positive + negative, text / date column groups aggregated by ``Avg`` or
``LeaveOutVector``), ``RecordInsightsCorr`` (``RecordInsightsCorr.scala:55-220``: per-feature
correlation with each score column times the normalized feature value) and ``RecordInsightsParser``
(``insightToText`` / ``parseInsights``). SURVEY.md K30.

Device design: LOCO is computed for a whole block of records at once. Every (record, non-zero
column) perturbation becomes one row of a perturbed batch scored by the model's vectorized predict
(for linear models the batch is never materialized: the perturbed margin is ``m_i - w_j x_ij``, an
elementwise [rows, d] tensor op); top-K selection per record is ``torch.topk`` over the
[rows, candidates] score-change matrix. Only the final ``TextMap`` strings are built on the host.
"""
from __future__ import annotations

import json
import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ...data.columns import ObjectColumn, PredictionColumn, VectorColumn
from ...features import types as T
from ..base import BinaryEstimator, BinaryTransformer, UnaryTransformer, register_stage

TEXT_TYPES = {"Text", "TextArea", "TextList", "TextMap", "TextAreaMap"}
DATE_TYPES = {"Date", "DateTime", "DateMap", "DateTimeMap"}
TIME_PERIODS = ("DayOfMonth", "DayOfWeek", "DayOfYear", "HourOfDay", "MonthOfYear", "WeekOfMonth", "WeekOfYear")


# ------------------------------------------------------------------------------------------- parser
def insight_to_text(column_info: str, score_diffs) -> Tuple[str, str]:
    scores = [[i, float(s)] for i, s in enumerate(score_diffs)]
    return column_info, json.dumps(scores, separators=(",", ":"))


def parse_insights(insights: Dict[str, str]) -> Dict[str, List[Tuple[int, float]]]:
    """``RecordInsightsParser.parseInsights``: column-history JSON -> [(score index, value)]."""
    out = {}
    for k, v in (insights or {}).items():
        hist = json.loads(k)
        key = hist.get("columnName", k)
        out[key] = [(int(a), float(b)) for a, b in json.loads(v)]
    return out


def _short(t: str) -> str:
    return t.rsplit(".", 1)[-1]


def _history_json(h: dict) -> str:
    return json.dumps(h, separators=(",", ":"), sort_keys=False)


def _jf(x: float) -> str:
    """A float as ``json.dumps`` writes it (repr; NaN / Infinity for the non-finite)."""
    return repr(x) if math.isfinite(x) else json.dumps(x)


class InsightsColumn(ObjectColumn):
    """``TextMap`` column of record insights kept as device tensors -- column index [n, K] (-1 = none),
    score changes [n, K, C] and the vector's column-history keys -- and rendered to the reference's
    ``{columnHistory JSON: "[[scoreIndex, diff], ...]"}`` maps only when rows are read on the host."""

    def __init__(self, cols: torch.Tensor, diffs: torch.Tensor, keys: Sequence[str]):
        self.ftype = T.TextMap
        self.cols, self.diffs, self.keys = cols, diffs, list(keys)
        self._values = None

    @property
    def values(self):
        if self._values is None:
            cols = self.cols.cpu().numpy()
            diffs = self.diffs.cpu().numpy()
            arr = np.empty(cols.shape[0], dtype=object)
            for i in range(cols.shape[0]):
                arr[i] = self._render(cols[i], diffs[i])
            self._values = arr
        return self._values

    @values.setter
    def values(self, v):
        self._values = v

    def _render(self, cols, diffs) -> Dict[str, str]:
        return {self.keys[c]: "[" + ",".join(f"[{j},{_jf(x)}]" for j, x in enumerate(dv)) + "]"
                for c, dv in zip(cols.tolist(), diffs.tolist()) if c >= 0}

    def __len__(self):
        return int(self.cols.shape[0])

    @property
    def device(self):
        return self.cols.device

    def take(self, idx):
        i = idx.to(self.cols.device, torch.long) if isinstance(idx, torch.Tensor) else \
            torch.as_tensor(np.asarray(idx, np.int64), device=self.cols.device)
        return InsightsColumn(self.cols.index_select(0, i), self.diffs.index_select(0, i), self.keys)

    def to(self, device):
        return InsightsColumn(self.cols.to(device), self.diffs.to(device), self.keys)

    def row(self, i):
        if self._values is not None:
            return self._values[i]
        return self._render(self.cols[i].cpu().numpy(), self.diffs[i].cpu().numpy())

    def null_mask(self):
        return ~(self.cols >= 0).any(1).cpu()

    @classmethod
    def _concat(cls, cols):
        if all(isinstance(c, InsightsColumn) and c.keys == cols[0].keys and c.diffs.shape[1:] == cols[0].diffs.shape[1:]
               for c in cols):
            return InsightsColumn(torch.cat([c.cols for c in cols]), torch.cat([c.diffs for c in cols]), cols[0].keys)
        return ObjectColumn(T.TextMap, np.concatenate([c.values for c in cols]))


# ---------------------------------------------------------------------------------------------- LOCO
@register_stage
class RecordInsightsLOCO(UnaryTransformer):
    """Unary (OPVector -> TextMap) transformer wrapping a fitted prediction model stage."""
    operation_name = "recordInsightsLOCO"
    output_type = T.TextMap
    _defaults = {"top_k": 20, "top_k_strategy": "abs", "vector_aggregation_strategy": "Avg"}

    def __init__(self, model=None, uid=None, **kw):
        super().__init__(None, uid=uid, **kw)
        self.model = model
        self.histories: Optional[List[dict]] = None
        self.chunk_elems = 1 << 22

    # -- model access
    def _learner_state(self):
        m = self.model
        return m.learner, m.state

    def _scores(self, X: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """(score matrix [n, C], predicted class [n])."""
        learner, state = self._learner_state()
        pred, raw, prob = learner.predict(state, X)
        if prob.shape[1] > 0:
            s = prob
        else:
            s = pred.reshape(-1, 1)
        return s.to(torch.float64), pred.reshape(-1)

    # -- groups of columns aggregated as one insight (text hashes, date unit circles)
    def _groups(self, hist: List[dict]):
        groups: Dict[str, List[int]] = {}
        for j, h in enumerate(hist):
            types = {_short(t) for t in h.get("parentFeatureType", [])}
            is_text = bool(types & TEXT_TYPES) and h.get("indicatorValue") is None and h.get("descriptorValue") is None
            is_date = bool(types & DATE_TYPES) and h.get("descriptorValue") is not None
            if not (is_text or is_date):
                continue
            origins = h.get("parentFeatureOrigins") or h.get("parentFeatureName") or [""]
            name = origins[0] + ("_" + h["grouping"] if h.get("grouping") else "")
            if is_date:
                tp = str(h.get("descriptorValue")).split("_")[-1]
                if tp.lower() in {p.lower() for p in TIME_PERIODS}:
                    name += "_" + next(p for p in TIME_PERIODS if p.lower() == tp.lower())
            groups.setdefault(name, []).append(j)
        return groups

    def _plan(self, hist: List[dict], d: int, device):
        """Candidate layout of one vector width: plain columns first (in column order), then one
        candidate per column group. Returns (cand_of_col [d], group size per candidate [m], plain
        column per candidate (-1 for groups) [m], group column tensors)."""
        groups = self._groups(hist)
        in_group = torch.zeros(d, dtype=torch.bool)
        for cols in groups.values():
            in_group[cols] = True
        plain = torch.nonzero(~in_group).flatten()
        n_plain = int(plain.numel())
        cand_of_col = torch.empty(d, dtype=torch.long)
        cand_of_col[plain] = torch.arange(n_plain)
        gsize = [1.0] * n_plain
        gcols = []
        for g, cols in enumerate(groups.values()):
            cand_of_col[torch.as_tensor(cols)] = n_plain + g
            gsize.append(float(len(cols)))
            gcols.append(torch.as_tensor(cols, device=device))
        plain_col = torch.cat([plain, torch.full((len(gcols),), -1, dtype=torch.long)])
        return (cand_of_col.to(device), torch.as_tensor(gsize, dtype=torch.float64, device=device),
                plain_col.to(device), gcols)

    def _loco_block(self, X: torch.Tensor, hist: List[dict], plan=None):
        """Top-K score changes of one block of records, all on the device: (column [n, K] (-1 = no
        insight), diffs [n, K, C]). Every (record, non-zero column) perturbation is one row of a perturbed
        batch; its score change is scattered into the record's candidate (the column itself, or its
        text / date group: ``Avg`` divides the group sum by the group size, ``LeaveOutVector`` re-scores
        the record with the whole group zeroed), then the top-K positive and negative candidates are
        merged and ordered per record by one stable sort (``RecordInsightsLOCO.scala:246-273``)."""
        n, d = X.shape
        dev = X.device
        base, pred_cls = self._scores(X)
        C = base.shape[1]
        if C == 0:
            raise RuntimeError("model does not produce scores for insights")
        if C == 1:
            ex = torch.zeros(n, dtype=torch.long, device=dev)
        elif C == 2:
            ex = torch.ones(n, dtype=torch.long, device=dev)
        else:
            ex = pred_cls.to(torch.long)
        cand_of_col, gsize, plain_col, gcols = plan if plan is not None else self._plan(hist, d, dev)
        m = int(gsize.numel())
        k = int(self.params["top_k"])
        abs_mode = self.params["top_k_strategy"] == "abs"
        kk = min(k, m)
        K = min(k if abs_mode else 2 * k, 2 * kk)
        if m == 0 or n == 0:
            return (torch.full((n, K), -1, dtype=torch.long, device=dev),
                    torch.zeros(n, K, C, dtype=torch.float64, device=dev))
        nz = X != 0
        rows, cols = torch.nonzero(nz, as_tuple=True)
        V = torch.zeros(n * m, C, dtype=torch.float64, device=dev)
        cand = cand_of_col[cols]
        # one perturbed copy per (record, non-zero column), scored in bounded chunks
        step = max(1, self.chunk_elems // max(d, 1))
        ar = torch.arange(min(step, rows.numel()), device=dev)
        for a in range(0, rows.numel(), step):
            r, c = rows[a:a + step], cols[a:a + step]
            Xp = X.index_select(0, r)
            Xp[ar[:r.numel()], c] = 0
            s, _ = self._scores(Xp)
            ca = cand[a:a + step]
            V.index_add_(0, r * m + ca, (base.index_select(0, r) - s) / gsize[ca][:, None])
        V = V.view(n, m, C)
        Cc = plain_col[None, :].expand(n, m).clone()
        n_plain = m - len(gcols)
        leave_out = self.params["vector_aggregation_strategy"] != "Avg"
        for g, gct in enumerate(gcols):
            active = nz[:, gct]
            has = active.any(1)
            Cc[:, n_plain + g] = torch.where(has, gct[active.to(torch.int8).argmax(1)], torch.full_like(has, -1,
                                                                                                    dtype=torch.long))
            if leave_out:       # LeaveOutVector: zero every active column of the group at once
                Xp = X.clone()
                Xp[:, gct] = 0
                s, _ = self._scores(Xp)
                V[:, n_plain + g] = torch.where(has[:, None], base - s, torch.zeros_like(base))
        val = V.gather(2, ex.view(n, 1, 1).expand(n, m, 1)).squeeze(2)
        valid = (Cc >= 0) & (val != 0)
        ninf = torch.full_like(val, -float("inf"))
        pv, pi = torch.topk(torch.where(valid & (val > 0), val, ninf), kk, dim=1)
        nv, ni = torch.topk(torch.where(valid & (val < 0), -val, ninf), kk, dim=1)
        idx = torch.cat([pi, ni], 1)                                   # positives first, then negatives
        ok = torch.cat([pv, nv], 1) != -float("inf")
        v = val.gather(1, idx)
        key = torch.where(ok, v.abs() if abs_mode else v, torch.full_like(v, -float("inf")))
        order = torch.sort(key, dim=1, descending=True, stable=True).indices[:, :K]
        sel = idx.gather(1, order)
        okK = ok.gather(1, order)
        colsK = torch.where(okK, Cc.gather(1, sel), torch.full_like(sel, -1))
        diffsK = V.gather(1, sel[:, :, None].expand(n, K, C))
        return colsK, diffsK

    def _run(self, X: torch.Tensor, hist: List[dict]):
        n, d = X.shape
        plan = self._plan(hist, d, X.device)
        m, C = max(int(plan[1].numel()), 1), 2
        block = max(64, (1 << 23) // (m * C))
        parts = [self._loco_block(X[a:a + block], hist, plan) for a in range(0, n, block)] or \
            [self._loco_block(X[:0], hist, plan)]
        return torch.cat([p[0] for p in parts]), torch.cat([p[1] for p in parts])

    def transform_columns(self, *cols, ds=None):
        vec: VectorColumn = cols[0]
        if vec.metadata is not None:
            self.histories = vec.metadata.column_history()
        hist = self.histories
        if hist is None:
            raise ValueError("RecordInsightsLOCO needs the input vector metadata (column histories)")
        cidx, diffs = self._run(vec.values, hist)
        return InsightsColumn(cidx, diffs, [_history_json(h) for h in hist])

    def transform_row(self, *values):
        x = torch.as_tensor(np.asarray(values[0], np.float64))[None, :]
        if self.histories is None:
            raise ValueError("RecordInsightsLOCO has not seen vector metadata yet")
        cidx, diffs = self._loco_block(x, self.histories)
        return InsightsColumn(cidx, diffs, [_history_json(h) for h in self.histories]).row(0)

    def ctor_args(self):
        from ...workflow.io import stage_to_json
        return {"model": stage_to_json(self.model) if self.model is not None else None,
                "histories": self.histories}

    def load_ctor_args(self, a):
        from ...workflow.io import _build_stage
        self.model = _build_stage(a["model"]) if a.get("model") else None
        self.histories = a.get("histories")


# ---------------------------------------------------------------------------------------------- Corr
def _pred_matrix(col) -> torch.Tensor:
    if isinstance(col, PredictionColumn):
        if col.probability.shape[1] > 0:
            return col.probability.to(torch.float64)
        return col.prediction.reshape(-1, 1).to(torch.float64)
    return col.values.to(torch.float64)


@register_stage
class RecordInsightsCorrModel(BinaryTransformer):
    operation_name = "recordInsightsCorr"
    output_type = T.TextMap
    allow_label_as_input = True

    def __init__(self, top_k=20, score_corr=None, norm=None, histories=None, uid=None, **kw):
        super().__init__(None, uid=uid, **kw)
        self.top_k = top_k
        self.score_corr = None if score_corr is None else np.asarray(score_corr, np.float64)
        self.norm = norm or {}
        self.histories = histories

    def _normalize(self, X: torch.Tensor) -> torch.Tensor:
        a = torch.as_tensor(self.norm["a"], dtype=torch.float64, device=X.device)
        b = torch.as_tensor(self.norm["b"], dtype=torch.float64, device=X.device)
        off = float(self.norm["offset"])
        Xd = X.to(torch.float64)
        return torch.where(b == 0, torch.zeros_like(Xd), (Xd - a) / torch.where(b == 0, torch.ones_like(b), b) - off)

    def _rows(self, X: torch.Tensor) -> List[Dict[str, str]]:
        d = X.shape[1]
        if self.histories is not None and len(self.histories) != d:
            raise ValueError("feature metadata size does not match feature size")
        Z = self._normalize(X)
        S = torch.as_tensor(np.nan_to_num(self.score_corr, nan=0.0), dtype=torch.float64, device=X.device)
        imp = Z[:, None, :] * S[None, :, :]                  # [n, P, d]
        k = min(int(self.top_k), d)
        _, idx = torch.topk(imp.abs(), k, dim=2)
        vals = imp.gather(2, idx)
        idx, vals = idx.cpu().numpy(), vals.cpu().numpy()
        out = []
        for i in range(X.shape[0]):
            acc: Dict[int, list] = {}
            for p in range(idx.shape[1]):
                for j, v in zip(idx[i, p], vals[i, p]):
                    acc.setdefault(int(j), []).append([p, float(v)])
            out.append({_history_json(self.histories[j]): json.dumps(v, separators=(",", ":"))
                        for j, v in acc.items()})
        return out

    def transform_columns(self, pred, vec, ds=None):
        return ObjectColumn(T.TextMap, self._rows(vec.values))

    def transform_row(self, *values):
        x = torch.as_tensor(np.asarray(values[1], np.float64))[None, :]
        return self._rows(x)[0]

    def ctor_args(self):
        return {"topK": self.top_k, "scoreCorr": None if self.score_corr is None else self.score_corr.tolist(),
                "norm": self.norm, "histories": self.histories}

    def load_ctor_args(self, a):
        self.top_k = a["topK"]
        self.score_corr = None if a["scoreCorr"] is None else np.asarray(a["scoreCorr"], np.float64)
        self.norm = a["norm"]
        self.histories = a["histories"]


@register_stage
class RecordInsightsCorr(BinaryEstimator):
    """(prediction, feature vector) -> TextMap of the top-K correlation-weighted features per record."""
    operation_name = "recordInsightsCorr"
    output_type = T.TextMap
    allow_label_as_input = True
    _defaults = {"norm_type": "minMax", "correlation_type": "pearson", "top_k": 20}

    def fit_columns(self, pred, vec, ds=None):
        from ...ops import stats as ST
        if vec.metadata is None:
            raise ValueError("second input feature must be a feature vector with OpVectorMetadata")
        P = _pred_matrix(pred)
        X = vec.values.to(torch.float64)
        psize, fsize = P.shape[1], X.shape[1]
        comb = torch.cat([X, P.to(X.device)], 1)
        C = ST.corr_matrix(comb, self.params["correlation_type"]).cpu().numpy()
        score_corr = C[fsize:fsize + psize, :fsize]
        cs = ST.col_stats(X)
        nt = self.params["norm_type"]
        mn, mx = cs["min"].cpu().numpy(), cs["max"].cpu().numpy()
        if nt == "minMax":
            norm = {"a": mn.tolist(), "b": (mx - mn).tolist(), "offset": 0.0, "name": nt}
        elif nt == "zNorm":
            norm = {"a": cs["mean"].cpu().numpy().tolist(), "b": np.sqrt(cs["variance"].cpu().numpy()).tolist(),
                    "offset": 0.0, "name": nt}
        elif nt == "minMaxCentered":
            norm = {"a": mn.tolist(), "b": ((mx - mn) / 2.0).tolist(), "offset": 1.0, "name": nt}
        else:
            raise ValueError(f"unknown norm type {nt}")
        return RecordInsightsCorrModel(self.params["top_k"], score_corr, norm, vec.metadata.column_history())

"""SanityChecker: label-aware feature validation and leakage detection.

Reference: ``SanityChecker`` (``core/.../impl/preparators/SanityChecker.scala:58-656``; sample fraction ``:356-361``,
colStats ``:407``, correlations ``:464-470``, categorical tests ``:252-348``, defaults ``:561-581``),
``DerivedFeatureFilterUtils`` (``makeColumnStatistics:80-224``, ``getFeaturesToDrop:234-281``,
``reasonsToRemove:350-420``) and the contingency statistics of ``OpStatistics`` (``utils/.../stats/OpStatistics.scala:141-382``).

Device work: one column-moment pass, one centered Gram GEMM for the full (d+1)^2 correlation matrix,
one label x column GEMM for every contingency table; the per-group chi-square / Cramer's V / PMI /
MI / rule-confidence math is tiny and runs on the host in fp64.
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Dict, List, Optional

import numpy as np
import torch

from ...data.columns import VectorColumn
from ...data.vector_metadata import OpVectorMetadata
from ...features import types as T
from ...ops import stats as ST, vector as V
from ..base import BinaryEstimator, BinaryTransformer, register_stage
from ...tuning.splitters import row_uniform


# ------------------------------------------------------------------------------- contingency math
def _filter_empties(M: np.ndarray) -> np.ndarray:
    if M.size == 0 or not np.any(M):
        return M
    M = M[M.sum(1) != 0]
    return M[:, M.sum(0) != 0]


def _chi2_cramers_v(F: np.ndarray):
    if F.shape[0] > 1 and F.shape[1] > 1:
        n = F.sum()
        E = F.sum(1, keepdims=True) * F.sum(0, keepdims=True) / n
        stat = float(((F - E) ** 2 / E).sum())
        from scipy.stats import chi2
        dof = (F.shape[0] - 1) * (F.shape[1] - 1)
        pv = float(chi2.sf(stat, dof))
        return math.sqrt(stat / n / min(F.shape[0] - 1, F.shape[1] - 1)), stat, pv
    return float("nan"), float("nan"), float("nan")


def _mutual_info(M: np.ndarray):
    rows_sum = M.sum(1)
    cols_sum = M.sum(0)
    n = rows_sum.sum()
    pmi = np.zeros_like(M, dtype=np.float64)
    ok = (M != 0) & (rows_sum[:, None] != 0) & (cols_sum[None, :] != 0)
    with np.errstate(divide="ignore", invalid="ignore"):
        val = np.log(np.maximum(M, 1e-99) * n / (rows_sum[:, None] * cols_sum[None, :])) / math.log(2.0)
    pmi = np.where(ok, val, 0.0)
    mi = float((pmi * M / n).sum()) if n > 0 else float("nan")
    return {str(j): pmi[:, j].tolist() for j in range(M.shape[1])}, mi


def _max_conf(M: np.ndarray):
    rs = M.sum(1)
    tot = rs.sum()
    sup = rs / tot if tot > 0 else np.zeros_like(rs)
    conf = np.where(rs == 0, 0.0, M.max(1) / np.where(rs == 0, 1, rs))
    return conf, sup


def contingency_stats(M: np.ndarray) -> Dict:
    F = _filter_empties(M)
    if F.size == 0 or not np.any(F):
        return {"cramersV": float("nan"), "chiSquaredStat": float("nan"), "pValue": float("nan"), "pmi": {},
                "mutualInfo": float("nan"), "maxConfidences": [], "supports": [], "contingency": {}}
    pmi, mi = _mutual_info(M)
    cv, stat, pv = _chi2_cramers_v(F)
    conf, sup = _max_conf(M)
    return {"cramersV": cv, "chiSquaredStat": stat, "pValue": pv, "pmi": pmi, "mutualInfo": mi,
            "maxConfidences": conf.tolist(), "supports": sup.tolist(),
            "contingency": {str(j): M[:, j].tolist() for j in range(M.shape[1])}}


def contingency_stats_mpl(M: np.ndarray, label_counts: np.ndarray) -> Dict:
    F = _filter_empties(M)
    singles = []
    for row in F:
        sm = np.stack([row, label_counts[:row.size] - row])
        singles.append(contingency_stats(sm))
    full = contingency_stats(M)
    if singles:
        win = max(singles, key=lambda s: -1 if math.isnan(s["cramersV"]) else s["cramersV"])
        full = dict(full, cramersV=win["cramersV"], chiSquaredStat=win["chiSquaredStat"], pValue=win["pValue"])
    return full


# ------------------------------------------------------------------------------------------- model
@register_stage
class SanityCheckerModel(BinaryTransformer):
    operation_name = "SanityChecker"
    output_type = T.OPVector
    allow_label_as_input = True

    def __init__(self, indices_to_keep=None, remove_bad_features=False, uid=None, **kw):
        super().__init__(None, uid=uid, **kw)
        self.indices_to_keep = None if indices_to_keep is None else [int(i) for i in indices_to_keep]
        self.remove_bad_features = remove_bad_features

    def transform_columns(self, *cols, ds=None):
        vec: VectorColumn = cols[1]
        meta = self.metadata.get("vector_metadata")
        if not self.remove_bad_features:
            return VectorColumn(metadata=meta or vec.metadata, blocks=vec.blocks)
        # keep-mask as a column view of the input blocks (K18): rows are gathered only by consumers
        return vec.select_columns(self.indices_to_keep, meta)

    def transform_row(self, *values):
        v = np.asarray(values[1], np.float64)
        return v[self.indices_to_keep] if self.remove_bad_features else v

    def ctor_args(self):
        return {"indicesToKeep": self.indices_to_keep, "removeBadFeatures": self.remove_bad_features}

    def load_ctor_args(self, a):
        self.indices_to_keep = list(a["indicesToKeep"])
        self.remove_bad_features = a["removeBadFeatures"]


@register_stage
class SanityChecker(BinaryEstimator):
    operation_name = "SanityChecker"
    output_type = T.OPVector
    allow_label_as_input = True
    _defaults = {"check_sample": 1.0, "sample_lower_limit": 1000, "sample_upper_limit": 1_000_000,
                 "max_correlation": 0.95, "max_feature_correlation": 0.99, "min_correlation": 0.0,
                 "min_variance": 1e-5, "max_cramers_v": 0.95, "remove_bad_features": False,
                 "remove_feature_group": True, "protect_text_shared_hash": False, "correlation_type": "pearson",
                 "max_rule_confidence": 1.0, "min_required_rule_support": 1.0,
                 "feature_feature_corr_level": "Computed", "correlation_exclusion": "NoExclusion",
                 "categorical_label": None, "sample_seed": 42}

    # parameter domains (SanityChecker.scala param validators: ParamValidators.inRange / gtEq)
    # (the correlation thresholds accept [-0.1, 1.1]: 1.1 switches a rule off, SanityChecker.scala:92-116)
    _ranges = {"check_sample": (0.0, 1.0, False), "min_correlation": (-0.1, 1.1, True),
               "max_correlation": (-0.1, 1.1, True), "max_feature_correlation": (-0.1, 1.1, True),
               "max_cramers_v": (0.0, 1.0, True), "max_rule_confidence": (0.0, 1.0, True),
               "min_required_rule_support": (0.0, 1.0, True)}

    def set(self, name, value):
        if name in self._ranges:
            lo, hi, lo_incl = self._ranges[name]
            v = float(value)
            if not ((v >= lo if lo_incl else v > lo) and v <= hi):
                raise ValueError(f"SanityChecker param {name} = {value} outside {'[' if lo_incl else '('}{lo}, {hi}]")
        # (minVariance has no validator in the reference -- DerivedFeatureFilterUtils.scala:65-70 -- and its tests set
        # it below zero to keep every column)
        if name in ("sample_lower_limit", "sample_upper_limit") and float(value) < 0:
            raise ValueError(f"SanityChecker param {name} must be >= 0, got {value}")
        return super().set(name, value)

    def set_input(self, *features):
        flat = [g for f in features for g in (f if isinstance(f, (list, tuple)) else [f])]
        if len(flat) == 2 and flat[1].is_response:
            raise ValueError("The feature vector should not contain any response features.")
        return super().set_input(*features)

    def fraction(self, total: int) -> float:
        p = self.params
        mn = min(1.0, p["sample_lower_limit"] / max(total, 1))
        mx = max(0.0, p["sample_upper_limit"] / max(total, 1))
        return max(min(p["check_sample"], mx), mn)

    # row-sharded fits reduce every statistic over the ranks (ops/stats.py: colStats, Gramian,
    # label contingency; sampling is by global row id, so the sample equals the single-process one)
    dp_aware = True

    def fit_columns(self, label_col, vec_col, ds=None):
        from ...parallel import dp
        p = self.params
        y = label_col.values
        dev = vec_col.device
        n_all = dp.count(len(vec_col))
        frac = self.fraction(n_all)
        if frac <= 0.0 or n_all == 0:
            raise ValueError("Sample size cannot be zero")
        keep = None
        if frac < 1.0:
            rid = ds.row_ids.to(dev) if ds is not None else torch.arange(n_all, device=dev)
            keep = torch.nonzero(row_uniform(rid, int(p["sample_seed"]), 9) < frac).reshape(-1)
        meta: OpVectorMetadata = vec_col.metadata
        d = vec_col.width
        if d == 0:
            raise ValueError("Feature vector passed in is empty, check your vectorizers")
        if meta is None or meta.size != d:
            raise ValueError(f"Number of columns in vector metadata ({None if meta is None else meta.size}) did not "
                             f"match number of columns in data ({d}), check your vectorizers")
        # [X | y] gathered from the vector's blocks and the label in one pass (no separate materialisation of X
        # followed by a concatenating copy); X is its leading column view
        y_full = y
        Xy = V.gather_rows_cols(vec_col.blocks + [(y_full.to(vec_col.dtype).to(dev)[:, None].contiguous(), None)],
                                None if keep is None else keep.to(dev), len(vec_col)).contiguous()
        if keep is not None:
            y = y_full.index_select(0, keep.to(y_full.device))
        X = Xy[:, :d]
        cs = ST.col_stats(Xy)
        count = cs["count"]
        cols = meta.columns
        # correlation indices (optionally excluding hashed text)
        if p["correlation_exclusion"] == "HashedText":
            hashed = {c.index for c in cols if c.grouping is None and c.indicator_value is None and any(
                t.rsplit(".", 1)[-1] in ("Text", "TextArea", "TextMap", "TextAreaMap") for t in c.parent_feature_type)}
            corr_idx = [i for i in range(d + 1) if i not in hashed]
        else:
            corr_idx = list(range(d + 1))
        ci = torch.as_tensor(corr_idx, device=X.device)
        if p["feature_feature_corr_level"] == "Off":
            C = None
            Z = Xy.index_select(1, ci)
            m = cs["mean"].index_select(0, ci.to(cs["mean"].device)).to(Z.device)
            Zc = Z.to(torch.float64) - m
            cov, ss = dp.sum_([(Zc * Zc[:, -1:]).sum(0), Zc.pow(2).sum(0)])
            cov = cov / max(count - 1, 1)
            sd = ss.div(max(count - 1, 1)).sqrt()
            corr_label = (cov / (sd * sd[-1])).cpu().numpy()
        labels_u = dp.unique_values(y)
        cat_label = p["categorical_label"]
        want_cat = cat_label is not False and (cat_label is True or labels_u.numel() < min(100.0, count * 0.1))
        pre_cat = None
        if p["feature_feature_corr_level"] != "Off":
            fused = (p["correlation_type"] == "pearson" and want_cat and len(corr_idx) == d + 1 and
                     not any(c.has_parent_of_subtype(T.MultiPickList) for c in cols))
            if fused:
                # one MFMA Gramian pass: correlations + label x column contingency + label counts
                Ct, lab, sums, cnts = ST.corr_and_label_sums(Xy, y, cs["mean"].to(Xy.device), cs["min"], cs["max"])
                C = Ct.cpu().numpy()
                pre_cat = (lab, sums[:, :d], cnts)
            else:
                C = ST.corr_matrix(Xy.index_select(1, ci), p["correlation_type"],
                                   mean=None if p["correlation_type"] == "spearman" else
                                   cs["mean"].index_select(0, ci.to(cs["mean"].device)).to(Xy.device)).cpu().numpy()
            corr_label = C[:, -1]
        # categorical tests
        cat_stats = []
        if want_cat:
            cat_stats = self._categorical_tests(X if pre_cat is not None else X.contiguous(), y, cols, pre_cat)
        label_dist = None
        if labels_u.numel() <= 100:
            lu = labels_u
            lc, = dp.sum_([(y[:, None] == lu[None, :]).sum(0).to(torch.float64)])
            label_dist = {"domain": [_label_str(v) for v in lu.cpu().tolist()],
                          "prob": (lc / max(float(lc.sum()), 1.0)).cpu().tolist()}
            for s in cat_stats:
                s["labels"] = label_dist["domain"]
        stats = self._column_statistics(cols, cs, label_col, d, corr_label, corr_idx, cat_stats, C)
        to_drop = []
        if p["remove_bad_features"]:
            to_drop = self._features_to_drop(stats)
        drop_names = {s["name"] for s, _ in to_drop}
        keep_idx = [c.index for c in cols if c.make_col_name() not in drop_names]
        if p["remove_bad_features"] and not keep_idx:
            raise ValueError("The sanity checker has dropped all of your features, check your input data quality")
        new_meta = meta.select(keep_idx if p["remove_bad_features"] else range(d), self.get_output_feature_name())
        self.metadata["vector_metadata"] = new_meta
        self.metadata["summary"] = {
            "correlationsWLabel": {"featuresIn": [cols[i].make_col_name() if i < d else self._inputs[0].name
                                                  for i in corr_idx],
                                   "values": [None if math.isnan(v) else float(v) for v in corr_label],
                                   "correlationType": p["correlation_type"]},
            "dropped": sorted(drop_names),
            "droppedReasons": {s["name"]: r for s, r in to_drop},
            "featuresStatistics": {"count": float(count), "mean": cs["mean"].tolist(), "max": cs["max"].tolist(),
                                   "min": cs["min"].tolist(), "variance": cs["variance"].tolist(),
                                   "sampleFraction": frac},
            "labelDistribution": label_dist,
            "names": [c.make_col_name() for c in cols] + [self._inputs[0].name],
            "categoricalStats": [dict(s, contingencyMatrix=s.get("contingency")) for s in cat_stats],
            "columnStatistics": [{k: v for k, v in s.items() if k not in ("column", "_ffhit")} for s in stats],
        }
        return SanityCheckerModel(keep_idx, p["remove_bad_features"])

    # ----------------------------------------------------------------------------------------
    def _categorical_tests(self, X, y, cols, pre=None) -> List[Dict]:
        if pre is not None:
            labels, sums, counts = pre
        else:
            mpl_idx = [c.index for c in cols if c.has_parent_of_subtype(T.MultiPickList)]
            Xc = X
            if mpl_idx:
                Xc = X.clone()
                mi = torch.as_tensor(mpl_idx, device=X.device)
                Xc[:, mi] = torch.clamp(Xc[:, mi], max=1.0)
            labels, sums, counts = ST.label_column_sums(Xc, y)
        cont = torch.cat([sums, counts[:, None]], 1).cpu().numpy()   # [L, d+1] rows = labels
        groups: "OrderedDict[str, list]" = OrderedDict()
        for c in cols:
            if c.grouping is not None and c.indicator_value is not None:
                groups.setdefault(c.feature_group(), []).append(c)
        out = []
        for g, cs in groups.items():
            seen = set()
            clean = []
            for c in cs:
                if c.indicator_value in seen:
                    continue
                seen.add(c.indicator_value)
                clean.append(c)
            idx = [c.index for c in clean]
            is_mpl = any(c.has_parent_of_subtype(T.MultiPickList) for c in clean)
            if len(idx) == 1:
                v = cont[:, idx[0]]
                M = np.stack([v, cont[:, -1] - v])            # rows: indicator / not, cols: labels
            else:
                M = cont[:, idx].T                            # rows: indicator values, cols: labels
            st = contingency_stats_mpl(M, cont[:, -1]) if is_mpl else contingency_stats(M)
            out.append({"group": g, "categoricalFeatures": [c.make_col_name() for c in clean], **st})
        return out

    def _column_statistics(self, cols, cs, label_col, d, corr_label, corr_idx, cat_stats, C) -> List[Dict]:
        pos = {ix: k for k, ix in enumerate(corr_idx)}
        cv_map = {}
        for s in cat_stats:
            for c in s["categoricalFeatures"]:
                cv_map[c] = s["cramersV"]

        def max_by_parent(pairs):
            out = {}
            for k, v in pairs:
                if v is None or (isinstance(v, float) and math.isnan(v)):
                    out.setdefault(k, 0.0)
                    continue
                out[k] = max(out.get(k, 0.0), abs(v))
            return out

        corr_parent = max_by_parent([(n, corr_label[pos[c.index]]) for c in cols if c.index in pos
                                     for n in c.parent_names_with_map_keys()])
        corr_parent_nk = max_by_parent([(n, corr_label[pos[c.index]]) for c in cols if c.index in pos
                                        for n in c.parent_feature_name])
        name_to_parents = {c.make_col_name(): c for c in cols}
        cv_parent = max_by_parent([(n, v) for k, v in cv_map.items()
                                   for n in name_to_parents[k].parent_names_with_map_keys()])
        cv_parent_nk = max_by_parent([(n, v) for k, v in cv_map.items()
                                      for n in name_to_parents[k].parent_feature_name])
        sup_map, conf_map = {}, {}
        for s in cat_stats:
            if len(s["categoricalFeatures"]) == 1:
                sup_map[s["categoricalFeatures"][0]] = list(s["supports"])
                conf_map[s["categoricalFeatures"][0]] = list(s["maxConfidences"])
            else:
                for f, sp, cf in zip(s["categoricalFeatures"], s["supports"], s["maxConfidences"]):
                    sup_map[f] = [sp]
                    conf_map[f] = [cf]

        def parent_val(c, m1, m2):
            vals = [m1.get(k, m2.get(k)) for k in c.parent_names_with_map_keys()]
            vals = [v for v in vals if v is not None]
            return max(vals) if vals else None

        # the feature-feature correlation rule per column, vectorised: the first earlier feature (position below
        # the column's index) whose |correlation| exceeds maxFeatureCorr (NaN never does)
        ff_hit: Dict[int, float] = {}
        if C is not None:
            thr = self.params["max_feature_correlation"]
            with np.errstate(invalid="ignore"):
                big = np.abs(C[:-1, :]) > thr
            for c in cols:
                k = pos.get(c.index)
                if k is None:
                    continue
                col = big[:min(c.index, big.shape[0]), k]
                if col.any():
                    ff_hit[c.index] = float(C[int(col.argmax()), k])
        mean, var = cs["mean"].cpu().numpy(), cs["variance"].cpu().numpy()
        mn, mx = cs["min"].cpu().numpy(), cs["max"].cpu().numpy()
        stats = [{"name": self._inputs[0].name, "column": None, "isLabel": True, "count": cs["count"],
                  "mean": float(mean[d]), "min": float(mn[d]), "max": float(mx[d]), "variance": float(var[d]),
                  "corrLabel": None, "cramersV": None, "featureCorrs": [], "parentCorr": None,
                  "parentCramersV": None, "maxRuleConfidences": [], "supports": []}]
        for c in cols:
            i = c.index
            name = c.make_col_name()
            k = pos.get(i)
            stats.append({
                "name": name, "column": c, "isLabel": False, "count": cs["count"], "mean": float(mean[i]),
                "min": float(mn[i]), "max": float(mx[i]), "variance": float(var[i]),
                "corrLabel": None if k is None else float(corr_label[k]),
                "cramersV": cv_map.get(name),
                "featureCorrs": [] if (k is None or C is None) else C[:-1, k].tolist(),
                "_ffhit": ff_hit.get(i),
                "parentCorr": parent_val(c, corr_parent, corr_parent_nk),
                "parentCramersV": parent_val(c, cv_parent, cv_parent_nk),
                "maxRuleConfidences": conf_map.get(name, []), "supports": sup_map.get(name, [])})
        return stats

    def _features_to_drop(self, stats):
        p = self.params
        groups = {}
        for s in stats:
            c = s["column"]
            g = c.feature_group() if c is not None else None
            groups.setdefault(g, []).append(s)
        rule_groups = set()
        for g, ss in groups.items():
            if g is None:
                continue
            if any(cf > p["max_rule_confidence"] and sp > p["min_required_rule_support"]
                   for s in ss for cf, sp in zip(s["maxRuleConfidences"], s["supports"])):
                rule_groups.add(g)
        out = []
        for s in stats:
            r = self._reasons(s, rule_groups)
            if r:
                out.append((s, f"Removing {s['name']} due to: {','.join(r)}"))
        return out

    def _reasons(self, s, removed_groups) -> List[str]:
        if s["isLabel"]:
            return []
        p = self.params
        R = []
        v = s["variance"]
        if v is not None and v <= p["min_variance"]:
            R.append(f"variance {v} lower than min variance {p['min_variance']}")
        cl = s["corrLabel"]
        if cl is not None and not math.isnan(cl):
            if abs(cl) < p["min_correlation"]:
                R.append(f"correlation {cl} lower than min correlation {p['min_correlation']}")
            if abs(cl) > p["max_correlation"]:
                R.append(f"correlation {cl} higher than max correlation {p['max_correlation']}")
        c = s["column"]
        if c is not None and s["featureCorrs"]:
            hit = s.get("_ffhit")
            if "_ffhit" not in s:       # statistics built elsewhere: the same rule, element by element
                prev = s["featureCorrs"][:c.index]
                hit = next((x for x in prev if not math.isnan(x) and abs(x) > p["max_feature_correlation"]), None)
            if hit is not None:
                R.append(f"this feature has correlations {hit} with another feature higher than max feature-feature"
                         f" correlation {p['max_feature_correlation']}")
        cv = s["cramersV"]
        if cv is not None and not math.isnan(cv) and cv > p["max_cramers_v"]:
            R.append(f"Cramer's V {cv} higher than max Cramer's V {p['max_cramers_v']}")
        for cf, sp in zip(s["maxRuleConfidences"], s["supports"]):
            if cf > p["max_rule_confidence"] and sp > p["min_required_rule_support"]:
                R.append(f"Max association rule confidence {cf} is above threshold of {p['max_rule_confidence']} "
                         f"and support {sp} is above the required support threshold of "
                         f"{p['min_required_rule_support']}")
                break
        if c is not None and c.feature_group() in removed_groups:
            R.append(f"other feature in indicator group {c.feature_group()} flagged for removal via rule confidence"
                     f" checks")
        if p["remove_feature_group"] and c is not None and (not _is_text_shared_hash(c) or
                                                             not p["protect_text_shared_hash"]):
            pcv = s["parentCramersV"]
            if pcv is not None and not math.isnan(pcv) and pcv > p["max_cramers_v"]:
                R.append(f"Cramer's V {pcv} for something in parent feature set higher than max Cramer's V "
                         f"{p['max_cramers_v']}")
            pc = s["parentCorr"]
            if pc is not None and not math.isnan(pc) and pc > p["max_correlation"]:
                R.append(f"correlation {pc} for something in parent feature set higher than max correlation "
                         f"{p['max_correlation']}")
        return R


def _label_str(v) -> str:
    f = float(v)
    return str(int(f)) if f.is_integer() else repr(f)


def _is_text_shared_hash(c) -> bool:
    derived = any(t.rsplit(".", 1)[-1] in ("Text", "TextArea", "TextMap", "TextAreaMap") for t in c.parent_feature_type)
    return derived and c.grouping is None and c.indicator_value is None

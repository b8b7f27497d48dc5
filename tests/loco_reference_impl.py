"""The round-2 LOCO assembly (per-record Python loop over torch top-K results), kept as the oracle of the
device-resident path in ``stages/insights/record_insights.py`` (tests/test_record_insights.py)."""
import torch

from transmogrifai_amd.stages.insights.record_insights import _history_json, insight_to_text


def loco_block(self, X, hist):
    """Score changes for one block of records: returns per record a list of (col, value, diffs)."""
    n, d = X.shape
    base, pred_cls = self._scores(X)
    C = base.shape[1]
    if C == 0:
        raise RuntimeError("model does not produce scores for insights")
    if C == 1:
        ex = torch.zeros(n, dtype=torch.long, device=X.device)
    elif C == 2:
        ex = torch.ones(n, dtype=torch.long, device=X.device)
    else:
        ex = pred_cls.to(torch.long)
    groups = self._groups(hist)
    in_group = torch.zeros(d, dtype=torch.bool)
    for cols in groups.values():
        in_group[cols] = True
    nz = X != 0
    rows, cols = torch.nonzero(nz, as_tuple=True)
    diffs = torch.zeros(rows.numel(), C, dtype=torch.float64, device=X.device)
    # one perturbed copy per (record, non-zero column), scored in bounded chunks
    step = max(1, self.chunk_elems // max(d, 1))
    for a in range(0, rows.numel(), step):
        r, c = rows[a:a + step], cols[a:a + step]
        Xp = X.index_select(0, r).clone()
        Xp[torch.arange(r.numel(), device=X.device), c] = 0
        s, _ = self._scores(Xp)
        diffs[a:a + step] = base.index_select(0, r) - s
    D = torch.zeros(n, d, C, dtype=torch.float64, device=X.device)
    D[rows, cols] = diffs
    strategy = self.params["vector_aggregation_strategy"]
    cand_vals = []       # [n] tensors of diffs (all classes) per candidate
    cand_cols = []
    plain = [j for j in range(d) if not bool(in_group[j])]
    for j in plain:
        cand_cols.append(torch.full((n,), j, dtype=torch.long, device=X.device))
        cand_vals.append(D[:, j, :])
    for name, gc in groups.items():
        gct = torch.as_tensor(gc, device=X.device)
        active = nz[:, gct]
        has = active.any(1)
        first = torch.where(has, gct[active.to(torch.int8).argmax(1)], torch.full((n,), -1, device=X.device))
        if strategy == "Avg":
            v = D[:, gct, :].sum(1) / len(gc)
        else:   # LeaveOutVector: zero every active column of the group at once
            Xp = X.clone()
            Xp[:, gct] = 0
            s, _ = self._scores(Xp)
            v = torch.where(has[:, None], base - s, torch.zeros_like(base))
        cand_cols.append(first)
        cand_vals.append(v)
    if not cand_vals:
        return [[] for _ in range(n)]
    V = torch.stack(cand_vals, 1)                      # [n, m, C]
    Cc = torch.stack(cand_cols, 1)                     # [n, m]
    val = V.gather(2, ex.view(n, 1, 1).expand(n, V.shape[1], 1)).squeeze(2)
    valid = (Cc >= 0) & (val != 0)
    k = int(self.params["top_k"])
    kk = min(k, val.shape[1])
    pos = torch.where(valid & (val > 0), val, torch.full_like(val, -float("inf")))
    neg = torch.where(valid & (val < 0), -val, torch.full_like(val, -float("inf")))
    pv, pi = torch.topk(pos, kk, dim=1)
    nv, ni = torch.topk(neg, kk, dim=1)
    out = []
    pv, pi, nv, ni = pv.cpu(), pi.cpu(), nv.cpu(), ni.cpu()
    Vc, Cc_, valc = V.cpu(), Cc.cpu(), val.cpu()
    for i in range(n):
        items = [(int(Cc_[i, m]), float(valc[i, m]), Vc[i, m].tolist())
                 for m, v in zip(pi[i].tolist(), pv[i].tolist()) if v != -float("inf")]
        items += [(int(Cc_[i, m]), float(valc[i, m]), Vc[i, m].tolist())
                  for m, v in zip(ni[i].tolist(), nv[i].tolist()) if v != -float("inf")]
        if self.params["top_k_strategy"] == "abs":
            items.sort(key=lambda t: -abs(t[1]))
            items = items[:k]
        else:
            items.sort(key=lambda t: -t[1])
            items = items[:2 * k]
        out.append(items)
    return out


def loco_maps(stage, X, hist):
    """Per-record insight maps of ``stage`` (a RecordInsightsLOCO) on ``X`` the round-2 way."""
    out = []
    for items in loco_block(stage, X, hist):
        out.append(dict(insight_to_text(_history_json(hist[c]), diffs) for c, _, diffs in items))
    return out

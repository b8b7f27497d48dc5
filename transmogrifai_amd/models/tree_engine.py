"""Batched level-wise histogram tree engine.

One engine serves every tree learner of the reference: Spark ``DecisionTree`` / ``RandomForest``
/ ``GBT`` (``OpDecisionTreeClassifier.scala:47-115``, ``OpRandomForestClassifier.scala:59-154``,
``OpGBTClassifier.scala:47-142`` and the regressors) and XGBoost (``OpXGBoostClassifier.scala:47-403``),
i.e. SURVEY.md kernels K23-K25 and K29.

MI355X-first design: instead of training one tree per Spark job, *all* trees of a batch -- every
tree of every (hyper-parameter config x CV fold) -- grow together, level by level. Per level there
is one histogram launch (work items = node row-chunks x feature groups), one split-scan launch,
one partition-count launch, a single device->host sync to collect the split decisions, and one
stable-scatter launch. Rows live in one packed ``uint32`` buffer (row id | bootstrap weight << 24)
partitioned by node, so a level touches only the rows of the nodes still being split. The same
orchestration drives the C++ host kernels when the data lives on the CPU.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..ops import _native as N

MODE_CLS, MODE_VAR, MODE_GH = 0, 1, 2
KIND_GINI, KIND_ENTROPY, KIND_VARIANCE, KIND_NEWTON = 0, 1, 2, 3
KINDS = {"gini": KIND_GINI, "entropy": KIND_ENTROPY, "variance": KIND_VARIANCE, "newton": KIND_NEWTON}

HIST_ITEM = np.dtype([("node", "<i4"), ("fg0", "<i4"), ("nf", "<i4"), ("excl", "<i4"),
                      ("begin", "<i8"), ("count", "<i8")])
PART_ITEM = np.dtype([("node", "<i4"), ("pad", "<i4"), ("begin", "<i8"), ("count", "<i8"),
                      ("out_left", "<i8"), ("out_right", "<i8")])
LEAF_ITEM = np.dtype([("begin", "<i8"), ("count", "<i8"), ("out", "<i8"), ("gid", "<i4"), ("pad", "<i4")])
assert HIST_ITEM.itemsize == 32 and PART_ITEM.itemsize == 40 and LEAF_ITEM.itemsize == 32

ROW_MASK = 0xFFFFFF
MAX_ROWS = 1 << 24


@dataclass
class TreeParams:
    max_depth: int = 5
    min_instances: float = 1.0
    min_info_gain: float = 0.0
    min_child_weight: float = 0.0
    reg_lambda: float = 0.0
    gamma: float = 0.0
    eta: float = 1.0
    feature_subset: Optional[int] = None   # features sampled per node (None = all)
    split_eps: float = 0.0                 # split only if gain > split_eps


@dataclass
class TreeJob:
    model: int                      # index into t1/t2 model axis
    params: TreeParams
    rows: torch.Tensor              # int64 row ids of the root (on the engine device)
    weights: Optional[torch.Tensor] = None   # optional integer weights per root row (bootstrap)
    seed: int = 0


@dataclass
class Forest:
    """Flat node arrays for a set of trees (children indices are global into the arrays)."""
    tree_off: np.ndarray            # int64 [T+1]
    nodes: np.ndarray               # int32 [n, 4] (feat, bin, left, right), left < 0 => leaf
    default_left: np.ndarray        # uint8 [n]
    value: np.ndarray               # float32 [n, K]
    gain: np.ndarray                # float32 [n]
    cover: np.ndarray               # float32 [n]  (weighted count / hessian)
    tree_model: np.ndarray          # int32 [T]   job.model for each tree
    missing_bin: int = -1

    @property
    def n_trees(self):
        return len(self.tree_off) - 1

    @property
    def K(self):
        return self.value.shape[1]

    def tree(self, t: int) -> "Forest":
        a, b = int(self.tree_off[t]), int(self.tree_off[t + 1])
        nodes = self.nodes[a:b].copy()
        nodes[:, 2:] = np.where(nodes[:, 2:] >= 0, nodes[:, 2:] - a, -1)
        return Forest(np.array([0, b - a], np.int64), nodes, self.default_left[a:b].copy(),
                      self.value[a:b].copy(), self.gain[a:b].copy(), self.cover[a:b].copy(),
                      self.tree_model[t:t + 1].copy(), self.missing_bin)

    @staticmethod
    def concat(forests: Sequence["Forest"]) -> "Forest":
        offs, nodes, dls, vals, gains, covs, tms = [0], [], [], [], [], [], []
        base = 0
        for f in forests:
            nd = f.nodes.copy()
            nd[:, 2:] = np.where(nd[:, 2:] >= 0, nd[:, 2:] + base, -1)
            nodes.append(nd)
            dls.append(f.default_left)
            vals.append(f.value)
            gains.append(f.gain)
            covs.append(f.cover)
            tms.append(f.tree_model)
            for t in range(f.n_trees):
                offs.append(base + int(f.tree_off[t + 1]))
            base += len(f.nodes)
        return Forest(np.asarray(offs, np.int64), np.concatenate(nodes), np.concatenate(dls),
                      np.concatenate(vals), np.concatenate(gains), np.concatenate(covs),
                      np.concatenate(tms), forests[0].missing_bin if forests else -1)

    def to_state(self) -> dict:
        return {"tree_off": self.tree_off, "nodes": self.nodes, "default_left": self.default_left,
                "value": self.value, "gain": self.gain, "cover": self.cover, "tree_model": self.tree_model,
                "missing_bin": int(self.missing_bin)}

    @staticmethod
    def from_state(d) -> "Forest":
        return Forest(np.asarray(d["tree_off"], np.int64), np.asarray(d["nodes"], np.int32).reshape(-1, 4),
                      np.asarray(d["default_left"], np.uint8), np.asarray(d["value"], np.float32).reshape(
                          len(np.asarray(d["default_left"])), -1),
                      np.asarray(d["gain"], np.float32), np.asarray(d["cover"], np.float32),
                      np.asarray(d["tree_model"], np.int32), int(d.get("missing_bin", -1)))

    def feature_importance(self, n_features: int) -> np.ndarray:
        """Total gain per feature, normalized per tree then averaged (Spark ``featureImportances``)."""
        imp = np.zeros(n_features)
        for t in range(self.n_trees):
            a, b = int(self.tree_off[t]), int(self.tree_off[t + 1])
            ti = np.zeros(n_features)
            nd = self.nodes[a:b]
            internal = nd[:, 2] >= 0
            np.add.at(ti, nd[internal, 0], (self.gain[a:b][internal] * self.cover[a:b][internal]).astype(np.float64))
            s = ti.sum()
            if s > 0:
                imp += ti / s
        s = imp.sum()
        return imp / s if s > 0 else imp


def pack_rows(rows: torch.Tensor, weights: Optional[torch.Tensor]) -> torch.Tensor:
    """Pack ``row | weight << 24`` into an int32 tensor (bit pattern read as uint32 by the kernels)."""
    r = rows.to(torch.int64)
    w = torch.ones_like(r) if weights is None else weights.to(torch.int64).clamp(0, 255)
    e = r | (w << 24)
    e = torch.where(e >= (1 << 31), e - (1 << 32), e)
    return e.to(torch.int32)


def _root_rows(jobs, dev):
    """Packed root entries of every job, zero-weight (out-of-bag) rows dropped for all weighted jobs
    with one compaction (two host syncs per call instead of one per tree)."""
    packs: List[Optional[torch.Tensor]] = [None] * len(jobs)
    counts = [0] * len(jobs)
    wj = [k for k, j in enumerate(jobs) if j.weights is not None]
    for k, j in enumerate(jobs):
        if j.weights is None:
            packs[k] = pack_rows(j.rows.to(dev), None)
            counts[k] = int(j.rows.numel())
    if wj:
        sizes = [int(jobs[k].rows.numel()) for k in wj]
        R = torch.cat([jobs[k].rows.to(dev).to(torch.int64) for k in wj])
        W = torch.cat([jobs[k].weights.to(dev).to(torch.int64) for k in wj])
        keep = W > 0
        ends = torch.as_tensor(np.cumsum(sizes) - 1, device=dev)
        csum = keep.to(torch.int64).cumsum(0)
        kc = csum[ends].cpu().numpy()
        kcount = np.diff(np.concatenate([[0], kc]))
        idx = keep.nonzero().squeeze(1)
        packed = pack_rows(R[idx], W[idx])
        for k, part, c in zip(wj, torch.split(packed, kcount.tolist()), kcount):
            packs[k] = part
            counts[k] = int(c)
    rows = torch.cat(packs) if packs else torch.zeros(0, dtype=torch.int32, device=dev)
    return rows, counts


class _Grow:
    """Growable host arrays for the created nodes."""

    def __init__(self, S):
        self.S = S
        self.n = 0
        cap = 1024
        self.tree = np.zeros(cap, np.int64)
        self.feat = np.full(cap, -1, np.int64)
        self.bin = np.full(cap, -1, np.int64)
        self.dl = np.zeros(cap, np.uint8)
        self.gain = np.zeros(cap, np.float64)
        self.tot = np.zeros((cap, S), np.float64)
        self.left = np.full(cap, -1, np.int64)
        self.right = np.full(cap, -1, np.int64)

    def add(self, trees: np.ndarray) -> np.ndarray:
        k = trees.size
        need = self.n + k
        if need > self.tree.size:
            cap = max(need, 2 * self.tree.size)
            for name, fill in (("tree", 0), ("feat", -1), ("bin", -1), ("dl", 0), ("gain", 0.0),
                               ("left", -1), ("right", -1)):
                a = getattr(self, name)
                b = np.full(cap, fill, a.dtype)
                b[:a.size] = a
                setattr(self, name, b)
            t = np.zeros((cap, self.S))
            t[:self.tot.shape[0]] = self.tot
            self.tot = t
        ids = np.arange(self.n, need, dtype=np.int64)
        self.tree[ids] = trees
        self.n = need
        return ids


def _feature_subsets(n_nodes: int, F: int, k: np.ndarray, dev, gen) -> tuple:
    """Per node j, ``k[j]`` distinct uniformly sampled features, sorted ascending.

    Returns ``(feat_list int32 [sum k], offsets int32 [n], nfeat int32 [n])``. Sampling is the
    "k smallest of F uniform keys" construction, done in node chunks with a seeded generator.
    """
    parts = [None] * n_nodes
    out = torch.empty(int(k.sum()), dtype=torch.int32, device=dev)
    offs = np.zeros(n_nodes, np.int64)
    if n_nodes > 1:
        offs[1:] = np.cumsum(k[:-1])
    for kv in np.unique(k):
        idx = np.nonzero(k == kv)[0]
        kv = int(kv)
        step = max(1, (1 << 24) // max(F, 1))
        for a in range(0, idx.size, step):
            sub = idx[a:a + step]
            keys = torch.rand((sub.size, F), generator=gen).to(dev)
            sel = torch.sort(torch.topk(keys, kv, dim=1, largest=False).indices, dim=1).values.to(torch.int32)
            pos = torch.as_tensor(offs[sub], device=dev)[:, None] + torch.arange(kv, device=dev)[None, :]
            out[pos.reshape(-1)] = sel.reshape(-1)
    del parts
    return out, offs.astype(np.int32), k.astype(np.int32)


def grow_forest(Xb: torch.Tensor, n_bins: np.ndarray, jobs: Sequence[TreeJob], *, mode: int, kind: int,
                n_classes: int = 2, y: Optional[torch.Tensor] = None, t1: Optional[torch.Tensor] = None,
                t2: Optional[torch.Tensor] = None, B: int = 32, missing_bin: int = -1,
                subtract: bool = True, chunk_rows: int = 4096, rng_seed: int = 0,
                collect_leaves: bool = False, groups: Optional[int] = None) -> Forest:
    """Grow one tree per job, all jobs level-synchronously. ``Xb`` is ``uint8 [N, F]``.

    Jobs are split into ``groups`` (default 2) contiguous groups grown as independent pipelines on
    separate HIP streams; each group draws its feature subsets from its own seeded generator.

    ``collect_leaves``: also return, as ``forest.leaf_assign``, the final leaf of every training entry
    (see ``LeafAssign``) so boosting can update margins without re-walking the new trees."""
    dev = Xb.device
    on_gpu = dev.type == "cuda"
    Nrows, F = int(Xb.shape[0]), int(Xb.shape[1])
    if Nrows >= MAX_ROWS:
        raise ValueError(f"tree engine supports < {MAX_ROWS} rows per training set, got {Nrows}")
    S = n_classes if mode == MODE_CLS else (3 if mode == MODE_VAR else 2)
    K = n_classes if mode == MODE_CLS else 1
    if missing_bin >= B:
        raise ValueError("missing_bin must be < B")
    n_bins_t = torch.as_tensor(np.asarray(n_bins, np.int32), device=dev)
    stride = int(t1.shape[1]) if (t1 is not None and t1.dim() == 2) else 0
    yf = y.to(device=dev, dtype=torch.float32).contiguous() if y is not None else None
    t1f = t1.to(device=dev, dtype=torch.float32).contiguous() if t1 is not None else None
    t2f = t2.to(device=dev, dtype=torch.float32).contiguous() if t2 is not None else None
    Xb = Xb.contiguous()
    T = len(jobs)
    all_feats = torch.arange(F, dtype=torch.int32, device=dev)
    ng = groups if groups is not None else (2 if T >= 2 else 1)
    ng = max(1, min(ng, T)) if T else 1
    cuts = np.linspace(0, T, ng + 1).astype(np.int64)
    gens = [_grow_group(Xb, n_bins_t, all_feats, list(jobs[cuts[g]:cuts[g + 1]]), mode, kind, S, K, B, missing_bin,
                        yf, t1f, t2f, stride, subtract, chunk_rows,
                        int(rng_seed) if ng == 1 else int(rng_seed) + 1000003 * g, collect_leaves)
            for g in range(ng)]
    results = [None] * ng
    if on_gpu and ng > 1:
        # two job groups on two streams: while the host reads one group's level and plans the next,
        # the GPU works on the other group's kernels
        cur = torch.cuda.current_stream(dev)
        streams = _group_streams(dev, ng)
        for st in streams:
            st.wait_stream(cur)
        alive = list(range(ng))
        while alive:
            for g in list(alive):
                with torch.cuda.stream(streams[g]):
                    try:
                        next(gens[g])
                    except StopIteration as e:
                        results[g] = e.value
                        alive.remove(g)
        for st in streams:
            cur.wait_stream(st)
    else:
        for g in range(ng):
            while True:
                try:
                    next(gens[g])
                except StopIteration as e:
                    results[g] = e.value
                    break
    if ng == 1:
        return results[0]
    forest = Forest.concat(results)
    if collect_leaves:
        las = [f.leaf_assign for f in results]
        goff = np.concatenate([[0], np.cumsum([int(la.value.shape[0]) for la in las])[:-1]])
        forest.leaf_assign = LeafAssign(
            torch.cat([la.rows for la in las]),
            torch.cat([la.gid + int(o) for la, o in zip(las, goff)]),
            torch.cat([la.value for la in las]),
            torch.cat([la.tree + int(cuts[g]) for g, la in enumerate(las)]))
    return forest


_STREAMS: dict = {}


def _group_streams(dev, n):
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    lst = _STREAMS.setdefault(key, [])
    while len(lst) < n:
        lst.append(torch.cuda.Stream(device=dev))
    return lst[:n]


def _grow_group(Xb, n_bins_t, all_feats, jobs, mode, kind, S, K, B, missing_bin, yf, t1f, t2f, stride,
                subtract, chunk_rows, rng_seed, collect_leaves):
    """Level-synchronous growth of one job group (generator: yields once per level, right before
    the level's device->host read, so another group's kernels can be queued behind this group's)."""
    dev = Xb.device
    on_gpu = dev.type == "cuda"
    Nrows, F = int(Xb.shape[0]), int(Xb.shape[1])
    T = len(jobs)
    P_depth = np.array([j.params.max_depth for j in jobs], np.int64)
    P_inst = np.array([j.params.min_instances for j in jobs], np.float64)
    P_gain = np.array([j.params.min_info_gain for j in jobs], np.float64)
    P_mcw = np.array([j.params.min_child_weight for j in jobs], np.float64)
    P_lam = np.array([j.params.reg_lambda for j in jobs], np.float64)
    P_eps = np.array([j.params.split_eps for j in jobs], np.float64)
    P_sub = np.array([F if (j.params.feature_subset is None or j.params.feature_subset >= F)
                      else max(1, int(j.params.feature_subset)) for j in jobs], np.int64)
    use_subset = bool(np.any(P_sub < F))
    gen = torch.Generator(device="cpu")
    gen.manual_seed(int(rng_seed))
    G = _Grow(S)

    # ---- roots
    rows, counts = _root_rows(jobs, dev)
    rows_alt = torch.empty_like(rows)
    lv_tree = np.arange(T, dtype=np.int64)
    lv_gid = G.add(lv_tree)
    lv_count = np.asarray(counts, np.int64)
    lv_begin = np.zeros(T, np.int64)
    if T:
        lv_begin[1:] = np.cumsum(lv_count[:-1])
    max_depth = int(P_depth.max()) if T else 0

    qscale, qinv = _quant_scales(mode, S, jobs, t1f, t2f, rows, chunk_rows, dev)
    lc = _LeafCollector(int(rows.numel()), dev, chunk_rows) if collect_leaves else None
    prev_hist = None          # previous level's histogram buffer
    pair_parent_off = None    # per sibling pair: parent's offset in prev_hist
    for depth in range(max_depth + 1):
        n = lv_gid.size
        if n == 0:
            break
        can = (depth < P_depth[lv_tree]) & (lv_count >= 2) & (lv_count >= 2 * P_inst[lv_tree] - 1e-9)
        need = can | (depth == 0)
        hist_nodes = np.nonzero(need)[0]
        if hist_nodes.size == 0:
            if lc is not None:
                lc.add(rows, lv_begin, lv_count, lv_gid)
            break
        m = hist_nodes.size
        h_tree = lv_tree[hist_nodes]
        if use_subset:
            feat_list, feat_off, nfeat = _feature_subsets(m, F, P_sub[h_tree], dev, gen)
        else:
            feat_list, feat_off, nfeat = all_feats, np.zeros(m, np.int32), np.full(m, F, np.int32)
        hsz = nfeat.astype(np.int64) * B * S
        hoff = np.zeros(m, np.int64)
        if m > 1:
            hoff[1:] = np.cumsum(hsz[:-1])
        hist = torch.empty(int(hsz.sum()), dtype=torch.int64, device=dev) if on_gpu else \
            torch.zeros(int(hsz.sum()), dtype=torch.int64, device=dev)
        loc = np.full(n, -1, np.int64)
        loc[hist_nodes] = np.arange(m)

        # subtraction trick: children come in (left, right) pairs at positions (2q, 2q+1)
        derive_big = np.zeros(0, np.int64)
        derive_small = np.zeros(0, np.int64)
        derive_poff = np.zeros(0, np.int64)
        if subtract and not use_subset and prev_hist is not None and depth > 0:
            lidx = np.arange(0, n, 2)
            both = need[lidx] & need[lidx + 1]
            q = np.nonzero(both)[0]
            li, ri = lidx[q], lidx[q] + 1
            left_big = lv_count[li] >= lv_count[ri]
            big = np.where(left_big, li, ri)
            small = np.where(left_big, ri, li)
            derive_big, derive_small, derive_poff = loc[big], loc[small], pair_parent_off[q]
        build = np.ones(m, bool)
        build[derive_big] = False
        build_local = np.nonzero(build)[0]

        node_model = np.array([jobs[t].model for t in h_tree], np.int32) if T else np.zeros(0, np.int32)
        params = np.zeros((m, 8), np.float32)
        params[:, 0] = P_inst[h_tree]
        params[:, 1] = P_gain[h_tree]
        params[:, 2] = P_mcw[h_tree]
        params[:, 3] = P_lam[h_tree]
        params[:, 5] = 1.0 if missing_bin >= 0 else 0.0
        params[:, 6] = P_eps[h_tree]
        params[:, 7] = can[hist_nodes]
        # every host->device array of the level's first half travels in one staged copy
        pk = _Pack(dev)
        i_nb, i_nc = pk.add(lv_begin[hist_nodes]), pk.add(lv_count[hist_nodes])
        i_nfo, i_nnf, i_nmd, i_nho = pk.add(feat_off), pk.add(nfeat), pk.add(node_model), pk.add(hoff)
        i_par = pk.add(params)
        if on_gpu:
            items = _hist_items(build_local, lv_begin[hist_nodes], lv_count[hist_nodes], nfeat, chunk_rows)
            citems = _part_items(np.arange(m), lv_begin[hist_nodes], lv_count[hist_nodes], chunk_rows)
            i_it, i_cit = pk.add(items.view(np.uint8)), pk.add(citems.view(np.uint8))
            multi = build_local[lv_count[hist_nodes[build_local]] > chunk_rows]
            if multi.size:
                i_z = (pk.add(hoff[multi]), pk.add(hsz[multi]))
            if derive_big.size:
                i_sub = [pk.add(derive_poff), pk.add(hoff[derive_small]), pk.add(hoff[derive_big]),
                         pk.add(hsz[derive_big])]
        dv = pk.ship()
        nb_, nc_, nfo, nnf, nmd, nho, par_t = (dv[i] for i in (i_nb, i_nc, i_nfo, i_nnf, i_nmd, i_nho, i_par))
        if on_gpu:
            if multi.size:
                N.check(N.hip().tmog_hip_zero_segments(N.ptr(hist), N.ptr(dv[i_z[0]]), N.ptr(dv[i_z[1]]),
                                                       int(multi.size), int(hsz[multi].max()), N.stream(dev)),
                        "zero_segments")
            if len(items):
                N.check(N.hip().tmog_hip_hist_build(
                    N.ptr(Xb), F, N.ptr(rows), N.ptr(dv[i_it]), len(items), N.ptr(nfo), N.ptr(feat_list),
                    N.ptr(nmd), N.ptr(nho), N.ptr(hist), B, mode, S, N.ptr(yf), N.ptr(t1f), N.ptr(t2f),
                    stride, N.ptr(qscale), N.stream(dev)), "hist_build")
            if derive_big.size:
                par, sm, oo, sz = (dv[i] for i in i_sub)
                N.check(N.hip().tmog_hip_hist_subtract(
                    N.ptr(hist), N.ptr(prev_hist), N.ptr(par), N.ptr(sm), N.ptr(oo), N.ptr(sz), int(derive_big.size),
                    int(hsz[derive_big].max()), N.stream(dev)), "hist_subtract")
        else:
            if build_local.size:
                sel = torch.as_tensor(build_local, device=dev)
                keep = [nb_[sel].contiguous(), nc_[sel].contiguous(), nfo[sel].contiguous(), nnf[sel].contiguous(),
                        nmd[sel].contiguous(), nho[sel].contiguous()]
                N.check(N.host().tmog_hist_build_cpu(
                    N.ptr(Xb), Nrows, F, N.ptr(rows), int(build_local.size), N.ptr(keep[0]), N.ptr(keep[1]),
                    N.ptr(keep[2]), N.ptr(keep[3]), N.ptr(feat_list), N.ptr(keep[4]), N.ptr(keep[5]), N.ptr(hist), B,
                    mode, S, N.ptr(yf), N.ptr(t1f), N.ptr(t2f), stride, N.ptr(qscale)), "hist_build_cpu")
            for b_, s_, p_ in zip(derive_big, derive_small, derive_poff):
                sz = int(hsz[b_])
                hist[hoff[b_]:hoff[b_] + sz] = prev_hist[p_:p_ + sz] - hist[hoff[s_]:hoff[s_] + sz]

        # ---- split scan + partition count write into one result buffer -> one device->host sync
        ncit = len(citems) if on_gpu else 0
        res = _LevelResult(m, S, ncit, dev)
        if on_gpu:
            mx = int(nfeat.max())
            cand = torch.empty(m * (-(-mx // 16)) * 24, dtype=torch.uint8, device=dev)   # Best[m][fb] workspace
            N.check(N.hip().tmog_hip_split_find(
                N.ptr(hist), m, N.ptr(nho), N.ptr(nnf), N.ptr(nfo), N.ptr(feat_list), N.ptr(n_bins_t), B, S, kind,
                N.ptr(par_t), missing_bin, N.ptr(nmd), N.ptr(qinv), mx, N.ptr(cand), N.ptr(res.feat), N.ptr(res.bin),
                N.ptr(res.gain), N.ptr(res.dl), N.ptr(res.left), N.ptr(res.tot), N.stream(dev)), "split_find")
        else:
            N.check(N.host().tmog_split_find_cpu(
                N.ptr(hist), m, N.ptr(nho), N.ptr(nnf), N.ptr(nfo), N.ptr(feat_list), N.ptr(n_bins_t), B, S, kind,
                N.ptr(par_t), missing_bin, N.ptr(nmd), N.ptr(qinv), N.ptr(res.feat), N.ptr(res.bin), N.ptr(res.gain),
                N.ptr(res.dl), N.ptr(res.left), N.ptr(res.tot)), "split_find_cpu")
        ok = (par_t[:, 7] > 0.5) & (res.feat >= 0) & (res.gain > par_t[:, 6])
        res.feat.masked_fill_(~ok, -1)
        s_feat, s_bin, s_dl = res.feat, res.bin, res.dl
        if on_gpu:
            N.check(N.hip().tmog_hip_partition_count(
                N.ptr(Xb), F, N.ptr(rows), N.ptr(dv[i_cit]), ncit, N.ptr(s_feat), N.ptr(s_bin), N.ptr(s_dl),
                missing_bin, N.ptr(res.chunk_left), N.stream(dev)), "partition_count")
        yield                                   # the other job group enqueues its level meanwhile
        h = res.fetch()
        h_chunk_left = h["chunk_left"]
        h_feat = h["feat"].astype(np.int64)
        h_bin = h["bin"].astype(np.int64)
        h_gain = h["gain"].astype(np.float64)
        h_dl = h["dl"]
        h_left = h["left"].reshape(m, S).astype(np.float64)
        h_tot = h["tot"].reshape(m, S).astype(np.float64)

        g_h = lv_gid[hist_nodes]
        G.tot[g_h] = h_tot
        spl = h_feat >= 0
        sl = np.nonzero(spl)[0]
        if lc is not None:
            leaf_mask = np.ones(n, bool)
            leaf_mask[hist_nodes[sl]] = False
            lf = np.nonzero(leaf_mask)[0]
            lc.add(rows, lv_begin[lf], lv_count[lf], lv_gid[lf])
        if sl.size == 0:
            break
        gs = g_h[sl]
        G.feat[gs], G.bin[gs], G.dl[gs], G.gain[gs] = h_feat[sl], h_bin[sl], h_dl[sl], h_gain[sl]

        counts_sl = lv_count[hist_nodes[sl]]
        out_begin = np.zeros(sl.size, np.int64)
        out_begin[1:] = np.cumsum(counts_sl[:-1])
        if on_gpu:
            nl, sitems = _scatter_items(citems, h_chunk_left, sl, m, out_begin)
            sit = _Pack(dev)
            i_s = sit.add(sitems.view(np.uint8))
            sit_t = sit.ship()[i_s]
            N.check(N.hip().tmog_hip_partition_scatter(
                N.ptr(Xb), F, N.ptr(rows), N.ptr(rows_alt), N.ptr(sit_t), len(sitems), N.ptr(s_feat), N.ptr(s_bin),
                N.ptr(s_dl), missing_bin, N.stream(dev)), "partition_scatter")
        else:
            lsel = torch.as_tensor(sl, device=dev)
            ob = torch.as_tensor(out_begin, device=dev)
            nl_t = torch.zeros(sl.size, dtype=torch.int64, device=dev)
            keep = [nb_[lsel].contiguous(), nc_[lsel].contiguous(), s_feat[lsel].contiguous(),
                    s_bin[lsel].contiguous(), s_dl[lsel].contiguous()]
            N.check(N.host().tmog_partition_cpu(
                N.ptr(Xb), F, N.ptr(rows), N.ptr(rows_alt), int(sl.size), N.ptr(keep[0]), N.ptr(keep[1]),
                N.ptr(keep[2]), N.ptr(keep[3]), N.ptr(keep[4]), missing_bin, N.ptr(ob), N.ptr(nl_t)),
                "partition_cpu")
            nl = nl_t.numpy()

        # ---- next level: children pairs (left, right) interleaved
        ptree = lv_tree[hist_nodes[sl]]
        ch_tree = np.repeat(ptree, 2)
        ch = G.add(ch_tree)
        gl, gr = ch[0::2], ch[1::2]
        G.left[gs], G.right[gs] = gl, gr
        G.tot[gl] = h_left[sl]
        G.tot[gr] = h_tot[sl] - h_left[sl]
        nlv = np.asarray(nl, np.int64)
        new_begin = np.empty(2 * sl.size, np.int64)
        new_begin[0::2] = out_begin
        new_begin[1::2] = out_begin + nlv
        new_count = np.empty(2 * sl.size, np.int64)
        new_count[0::2] = nlv
        new_count[1::2] = counts_sl - nlv
        pair_parent_off = hoff[sl]
        prev_hist = hist
        rows, rows_alt = rows_alt, rows
        lv_tree, lv_gid, lv_begin, lv_count = ch_tree, ch, new_begin, new_count

    forest = _finalize(jobs, G, mode, kind, K, S, missing_bin, with_gid_values=lc is not None)
    if lc is not None:
        gid_value, gid_tree = forest._gid_value, forest._gid_tree
        del forest._gid_value, forest._gid_tree
        forest.leaf_assign = LeafAssign(lc.rows[:lc.pos], lc.gid[:lc.pos],
                                        torch.as_tensor(gid_value, device=dev),
                                        torch.as_tensor(gid_tree, device=dev))
    return forest


@dataclass
class LeafAssign:
    """Final leaf of every training entry of a ``grow_forest`` call: ``rows`` (packed entries, as
    given to the trees), ``gid`` (node id per entry), ``value[gid]`` (leaf output, pruning applied),
    ``tree[gid]`` (job index). ``per_tree_values`` turns it into margin updates."""
    rows: torch.Tensor
    gid: torch.Tensor
    value: torch.Tensor
    tree: torch.Tensor

    def row_ids(self) -> torch.Tensor:
        return (self.rows & 0xFFFFFF).to(torch.int64)

    def entry_tree(self) -> torch.Tensor:
        return self.tree[self.gid.to(torch.int64)]

    def entry_value(self) -> torch.Tensor:
        return self.value[self.gid.to(torch.int64)]


_TORCH_OF_NP = {np.dtype(np.int64): torch.int64, np.dtype(np.int32): torch.int32,
                np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64,
                np.dtype(np.uint8): torch.uint8, np.dtype(np.bool_): torch.bool}


class _Pack:
    """Ships several small host arrays with ONE host->device copy through a pinned staging ring
    (each ``torch.as_tensor(a, device=cuda)`` is its own blocking hipMemcpy: ~10 per tree level)."""
    _ring: dict = {}
    _RING = 4

    def __init__(self, dev):
        self.dev = dev
        self.arrs: List[np.ndarray] = []

    def add(self, a) -> int:
        self.arrs.append(np.ascontiguousarray(a))
        return len(self.arrs) - 1

    def ship(self) -> List[torch.Tensor]:
        if self.dev.type != "cuda":
            return [torch.from_numpy(a) for a in self.arrs]
        offs, tot = [], 0
        for a in self.arrs:
            offs.append(tot)
            tot += (a.nbytes + 15) & ~15
        tot = max(tot, 16)
        key = self.dev.index if self.dev.index is not None else torch.cuda.current_device()
        slots = _Pack._ring.setdefault(key, {"i": 0, "bufs": [None] * self._RING, "ev": [None] * self._RING})
        k = slots["i"] = (slots["i"] + 1) % self._RING
        buf, ev = slots["bufs"][k], slots["ev"][k]
        if ev is not None:
            ev.synchronize()                 # the copy that last used this slot has finished
        if buf is None or buf.numel() < tot:
            buf = torch.empty(max(tot, 1 << 16), dtype=torch.uint8, pin_memory=True)
            slots["bufs"][k] = buf
        hb = buf.numpy()
        for a, o in zip(self.arrs, offs):
            hb[o:o + a.nbytes] = a.reshape(-1).view(np.uint8)
        d = torch.empty(tot, dtype=torch.uint8, device=self.dev)
        d.copy_(buf[:tot], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.dev))
        slots["ev"][k] = ev
        return [d[o:o + a.nbytes].view(_TORCH_OF_NP[a.dtype]).reshape(a.shape) if a.dtype in _TORCH_OF_NP
                else d[o:o + a.nbytes] for a, o in zip(self.arrs, offs)]


class _LevelResult:
    """Split-scan and partition-count outputs of one level laid out in one int32 device buffer so
    the host reads every decision of the level with a single device->host copy."""

    def __init__(self, m, S, n_chunks, dev):
        self.m, self.S, self.nc = m, S, n_chunks
        words = 2 * n_chunks + 3 * m + 2 * m * S + (m + 3) // 4
        self.buf = torch.empty(max(words, 1), dtype=torch.int32, device=dev)
        o = 0
        self.chunk_left = self.buf[o:o + 2 * n_chunks].view(torch.int64)
        self.chunk_left.zero_()
        o += 2 * n_chunks
        self.feat = self.buf[o:o + m]
        o += m
        self.bin = self.buf[o:o + m]
        o += m
        self.gain = self.buf[o:o + m].view(torch.float32)
        o += m
        self.left = self.buf[o:o + m * S].view(torch.float32)
        o += m * S
        self.tot = self.buf[o:o + m * S].view(torch.float32)
        o += m * S
        self.dl = self.buf[o:o + (m + 3) // 4].view(torch.uint8)[:m]

    def fetch(self) -> dict:
        h = self.buf.cpu().numpy()
        m, S, o = self.m, self.S, 2 * self.nc
        out = {"chunk_left": h[:o].view(np.int64)}
        out["feat"] = h[o:o + m]
        out["bin"] = h[o + m:o + 2 * m]
        out["gain"] = h[o + 2 * m:o + 3 * m].view(np.float32)
        o += 3 * m
        out["left"] = h[o:o + m * S].view(np.float32)
        out["tot"] = h[o + m * S:o + 2 * m * S].view(np.float32)
        o += 2 * m * S
        out["dl"] = h[o:o + (m + 3) // 4].view(np.uint8)[:m]
        return out


class _LeafCollector:
    def __init__(self, total, dev, chunk_rows):
        self.rows = torch.empty(total, dtype=torch.int32, device=dev)
        self.gid = torch.empty(total, dtype=torch.int32, device=dev)
        self.pos = 0
        self.dev = dev
        self.chunk = int(chunk_rows)

    def add(self, rows, begin, count, gid):
        begin, count, gid = (np.asarray(a, np.int64) for a in (begin, count, gid))
        nz = count > 0
        begin, count, gid = begin[nz], count[nz], gid[nz]
        if count.size == 0:
            return
        out = self.pos + np.concatenate([[0], np.cumsum(count[:-1])])
        self.pos += int(count.sum())
        if self.dev.type == "cuda":
            nch = -(-count // self.chunk)
            seg = np.repeat(np.arange(count.size), nch)
            c = np.arange(seg.size) - np.repeat(np.cumsum(nch) - nch, nch)
            a = np.zeros(seg.size, LEAF_ITEM)
            a["begin"] = begin[seg] + c * self.chunk
            a["count"] = np.minimum(self.chunk, count[seg] - c * self.chunk)
            a["out"] = out[seg] + c * self.chunk
            a["gid"] = gid[seg]
            pk = _Pack(self.dev)
            i_a = pk.add(a.view(np.uint8))
            it = pk.ship()[i_a]
            N.check(N.hip().tmog_hip_leaf_collect(N.ptr(rows), N.ptr(it), len(a), N.ptr(self.rows), N.ptr(self.gid),
                                                  N.stream(self.dev)), "leaf_collect")
        else:
            seg = np.repeat(np.arange(count.size), count)
            starts = np.concatenate([[0], np.cumsum(count[:-1])])
            within = np.arange(seg.size) - np.repeat(starts, count)
            src = torch.as_tensor(begin[seg] + within)
            dst = slice(int(out[0]), int(out[0]) + seg.size)
            self.rows[dst] = rows[src]
            self.gid[dst] = torch.as_tensor(gid[seg].astype(np.int32))


def _quant_scales(mode, S, jobs, t1f, t2f, rows, chunk_rows, dev):
    """Per-(model, stat) power-of-two fixed-point scales for the int64 histograms (see the
    "Fixed-point statistics" note in ops/csrc/hip/tree_kernels.hip). A row's contribution is
    ``rint(v * scale)`` with ``|v * scale| <= qmax``, so a ``chunk_rows``-row LDS partial fits int32.
    Computed on the device (no host sync); returns (float32 scales, float64 inverses), ``[n_models, S]``."""
    n_models = max([j.model for j in jobs], default=0) + 1
    if mode == MODE_CLS or rows.numel() == 0:
        one = torch.ones(n_models, S, dtype=torch.float32, device=dev)
        return one, one.to(torch.float64)
    qmax = float(min(1 << 22, (2 ** 31 - 1) // max(1, int(chunk_rows)) - 1))
    wmax = ((rows >> 24) & 0xFF).max().to(torch.float32)

    def amax(t):
        if t is None:
            return torch.zeros(n_models, dtype=torch.float32, device=dev)
        v = t.reshape(t.shape[0], -1) if t.dim() == 2 else t.reshape(1, -1)
        L = v.shape[1]
        if L >= 1 << 16:        # row-wise amax of a few long rows: split each row into 256 segments
            seg = -(-L // 256)
            a = v.abs()
            if seg * 256 != L:
                a = torch.nn.functional.pad(a, (0, seg * 256 - L))
            m = a.view(v.shape[0], 256, seg).amax(2).amax(1)
        else:
            m = v.abs().amax(1)
        return m.expand(n_models) if m.numel() == 1 else m[:n_models]

    def pow2(bound):
        x = qmax / (bound * wmax).clamp_min(1e-30)
        return torch.exp2(torch.floor(torch.log2(x))).clamp(2.0 ** -60, 2.0 ** 60)

    if mode == MODE_VAR:
        m1 = amax(t1f)
        sc = torch.stack([torch.ones_like(m1), pow2(m1), pow2(m1 * m1)], 1)
    else:
        sc = torch.stack([pow2(amax(t1f)), pow2(amax(t2f))], 1)
    sc = sc.to(torch.float32).contiguous()
    return sc, (1.0 / sc.to(torch.float64)).contiguous()


def _hist_items(build_local, begin, count, nfeat, chunk_rows):
    if build_local.size == 0:
        return np.zeros(0, HIST_ITEM)
    cnt = count[build_local]
    nf = nfeat[build_local].astype(np.int64)
    ng = np.maximum(1, -(-nf // 64))
    fg = -(-nf // ng)
    nch = np.maximum(1, -(-cnt // chunk_rows))
    rep = nch * ng
    tot = int(rep.sum())
    starts = np.zeros(build_local.size, np.int64)
    starts[1:] = np.cumsum(rep[:-1])
    within = np.arange(tot, dtype=np.int64) - np.repeat(starts, rep)
    ngr, fgr, nfr = np.repeat(ng, rep), np.repeat(fg, rep), np.repeat(nf, rep)
    c = within // ngr
    g = within % ngr
    a = np.zeros(tot, HIST_ITEM)
    a["node"] = np.repeat(build_local, rep)
    a["fg0"] = g * fgr
    a["nf"] = np.minimum(fgr, nfr - g * fgr)
    a["excl"] = np.repeat((nch == 1).astype(np.int64), rep)
    a["begin"] = np.repeat(begin[build_local], rep) + c * chunk_rows
    a["count"] = np.minimum(chunk_rows, np.repeat(cnt, rep) - c * chunk_rows)
    return a


def _part_items(local, begin, count, chunk_rows):
    cnt = count[local]
    nch = np.maximum(1, -(-cnt // chunk_rows))
    tot = int(nch.sum())
    starts = np.zeros(local.size, np.int64)
    if local.size > 1:
        starts[1:] = np.cumsum(nch[:-1])
    within = np.arange(tot, dtype=np.int64) - np.repeat(starts, nch)
    a = np.zeros(tot, PART_ITEM)
    a["node"] = np.repeat(local, nch)
    a["begin"] = np.repeat(begin[local], nch) + within * chunk_rows
    a["count"] = np.minimum(chunk_rows, np.repeat(cnt, nch) - within * chunk_rows)
    return a


def _scatter_items(citems, chunk_left, split_local, m, out_begin):
    """Per-chunk output offsets (stable scatter) for the splitting nodes; returns (left counts, items)."""
    pos = np.full(m, -1, np.int64)
    pos[split_local] = np.arange(split_local.size)
    q = pos[citems["node"]]
    keep = q >= 0
    ci = citems[keep]
    q = q[keep]
    cl = chunk_left[keep].astype(np.int64)
    cr = ci["count"] - cl
    nl = np.bincount(q, weights=cl, minlength=split_local.size).astype(np.int64)
    # exclusive running sums within each node's (contiguous) chunk run
    cum_l = np.cumsum(cl) - cl
    cum_r = np.cumsum(cr) - cr
    first = np.ones(q.size, bool)
    first[1:] = q[1:] != q[:-1]
    run_id = np.cumsum(first) - 1
    base_l = cum_l[first][run_id]
    base_r = cum_r[first][run_id]
    a = np.zeros(q.size, PART_ITEM)
    a["node"] = ci["node"]
    a["begin"] = ci["begin"]
    a["count"] = ci["count"]
    a["out_left"] = out_begin[q] + (cum_l - base_l)
    a["out_right"] = out_begin[q] + nl[q] + (cum_r - base_r)
    return nl, a


def _finalize(jobs, G: _Grow, mode, kind, K, S, missing_bin, with_gid_values: bool = False):
    n = G.n
    tot = G.tot[:n]
    left = G.left[:n].copy()
    right = G.right[:n].copy()
    feat = G.feat[:n].copy()
    gain = G.gain[:n]
    tree = G.tree[:n]
    if mode == MODE_CLS:
        s = tot.sum(1, keepdims=True)
        value = np.where(s > 0, tot / np.maximum(s, 1e-300), 0.0)
        cover = s[:, 0]
    elif mode == MODE_VAR:
        value = np.where(tot[:, :1] > 0, tot[:, 1:2] / np.maximum(tot[:, :1], 1e-300), 0.0)
        cover = tot[:, 0]
    else:
        lam = np.array([j.params.reg_lambda for j in jobs])[tree]
        eta = np.array([j.params.eta for j in jobs])[tree]
        value = (-tot[:, 0] / (tot[:, 1] + lam) * eta)[:, None]
        cover = tot[:, 1]
    if kind == KIND_NEWTON:
        gam = np.array([j.params.gamma for j in jobs])[tree]
        while True:
            idx = np.nonzero(left >= 0)[0]
            if idx.size == 0:
                break
            leafy = (left[left[idx]] < 0) & (left[right[idx]] < 0)
            prune = idx[leafy & (gain[idx] < gam[idx])]
            if prune.size == 0:
                break
            left[prune] = -1
            right[prune] = -1
            feat[prune] = -1
    # BFS renumbering per tree (drops pruned descendants); nodes of a tree are created in BFS order
    # already, so a stable filter of reachable nodes preserves it.
    reach = np.zeros(n, bool)
    T = len(jobs)
    roots = np.arange(T, dtype=np.int64)          # roots were created first, one per job
    reach[roots] = True
    # propagate reachability in creation order (parents precede children)
    internal = np.nonzero(left >= 0)[0]
    for g in internal:                             # creation order == topological order
        if reach[g]:
            reach[left[g]] = True
            reach[right[g]] = True
    keep = np.nonzero(reach)[0]
    # group by tree, keeping creation order inside a tree
    order = keep[np.argsort(tree[keep], kind="stable")]
    new_id = np.full(n, -1, np.int64)
    new_id[order] = np.arange(order.size)
    tree_off = np.zeros(T + 1, np.int64)
    tree_off[1:] = np.cumsum(np.bincount(tree[order], minlength=T))
    isint = left[order] >= 0
    nodes = np.zeros((order.size, 4), np.int32)
    nodes[:, 0] = np.where(isint, feat[order], 0)
    nodes[:, 1] = np.where(isint, G.bin[:n][order], 0)
    nodes[:, 2] = np.where(isint, new_id[np.maximum(left[order], 0)], -1)
    nodes[:, 3] = np.where(isint, new_id[np.maximum(right[order], 0)], -1)
    gid_value = None
    if with_gid_values:
        # leaf output per created node id: pruned descendants inherit their kept ancestor's leaf value
        parent = np.full(n, -1, np.int64)
        orig_int = np.nonzero(G.left[:n] >= 0)[0]
        parent[G.left[:n][orig_int]] = orig_int
        parent[G.right[:n][orig_int]] = orig_int
        gid_value = value.astype(np.float32).reshape(n, K).copy()
        for g in np.nonzero(~reach)[0]:
            gid_value[g] = gid_value[parent[g]]
    f = Forest(tree_off, nodes, np.where(isint, G.dl[:n][order], 0).astype(np.uint8),
                  value[order].astype(np.float32).reshape(order.size, K),
                  np.where(isint, gain[order], 0).astype(np.float32), cover[order].astype(np.float32),
                  np.array([j.model for j in jobs], np.int32), missing_bin)
    if with_gid_values:
        f._gid_value, f._gid_tree = gid_value, tree.astype(np.int64)
    return f


def forest_predict(forest: Forest, Xb: torch.Tensor, model_rows: Sequence[Optional[torch.Tensor]],
                   model_trees: Sequence[Sequence[int]], tree_weight: Optional[np.ndarray] = None,
                   n_rows: Optional[int] = None) -> List[torch.Tensor]:
    """Evaluate groups of trees ("models") on row subsets of ``Xb``.

    ``model_rows[m]`` = row ids (or None for all rows); ``model_trees[m]`` = tree indices of the
    forest that form model m. Returns one ``float32 [n_m, K]`` tensor per model: the weighted sum
    of leaf values over the model's trees.
    """
    dev = Xb.device
    Xb = Xb.contiguous()
    Nrows, F = int(Xb.shape[0]), int(Xb.shape[1])
    K = forest.K
    # reorder trees so each model's trees are contiguous
    order = [t for ts in model_trees for t in ts]
    mto = np.zeros(len(model_trees) + 1, np.int64)
    mto[1:] = np.cumsum([len(ts) for ts in model_trees])
    tw = np.ones(forest.n_trees, np.float32) if tree_weight is None else np.asarray(tree_weight, np.float32)
    t_off = torch.as_tensor(forest.tree_off[:-1][order].astype(np.int64), device=dev)
    t_w = torch.as_tensor(tw[order], device=dev)
    nodes = torch.as_tensor(np.ascontiguousarray(forest.nodes), device=dev)
    dl = torch.as_tensor(forest.default_left, device=dev)
    lv = torch.as_tensor(np.ascontiguousarray(forest.value), device=dev)
    counts = [Nrows if r is None else int(r.numel()) for r in model_rows]
    mro = np.zeros(len(model_rows) + 1, np.int64)
    mro[1:] = np.cumsum(counts)
    if all(r is None for r in model_rows):
        row_list = None
        if len(model_rows) > 1:
            row_list = torch.cat([torch.arange(Nrows, device=dev, dtype=torch.int32)] * len(model_rows))
    else:
        row_list = torch.cat([(torch.arange(Nrows, device=dev) if r is None else r.to(dev)).to(torch.int32)
                              for r in model_rows])
    out = torch.zeros(int(mro[-1]), K, dtype=torch.float32, device=dev)
    mro_t = torch.as_tensor(mro, device=dev)
    mto_t = torch.as_tensor(mto, device=dev)
    if dev.type == "cuda":
        # the kernel accumulates up to 8 outputs per row in registers: wider K runs in class chunks
        for c0 in range(0, K, 8):
            kc = min(8, K - c0)
            lvc = lv if kc == K else lv[:, c0:c0 + kc].contiguous()
            oc = out if kc == K else torch.empty(int(mro[-1]), kc, dtype=torch.float32, device=dev)
            N.check(N.hip().tmog_hip_forest_predict(
                N.ptr(Xb), F, len(model_rows), N.ptr(mro_t), N.ptr(row_list), max(counts) if counts else 0,
                N.ptr(mto_t), N.ptr(t_off), N.ptr(t_w), N.ptr(nodes), N.ptr(dl), forest.missing_bin, N.ptr(lvc), kc,
                N.ptr(oc), N.stream(dev)), "forest_predict")
            if kc != K:
                out[:, c0:c0 + kc] = oc
    else:
        N.check(N.host().tmog_forest_predict_cpu(
            N.ptr(Xb), F, len(model_rows), N.ptr(mro_t), N.ptr(row_list), N.ptr(mto_t), N.ptr(t_off), N.ptr(t_w),
            N.ptr(nodes), N.ptr(dl), forest.missing_bin, N.ptr(lv), K, N.ptr(out)), "forest_predict_cpu")
    return [out[int(mro[m]):int(mro[m + 1])] for m in range(len(model_rows))]

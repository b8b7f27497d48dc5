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

import ctypes as C
import math
import os
import threading
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

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
CSR_ITEM_ROWS = 1024          # rows per CSR histogram item (tree_grow.hpp kCsrRows)
MAX_ROWS = 1 << 24            # packed entries (row | weight << 24) below this many training rows
MAX_WIDE_ROWS = 1 << 31       # wide entries (32-bit row id, weight 1)


def wide_rows(n_rows: int) -> bool:
    """Entry format of a training set of ``n_rows`` rows: below 2^24 rows the row id and an 8-bit weight share
    one 32-bit entry; from 2^24 rows on (or with ``TMOG_TREE_WIDE_ROWS=1``, for tests) an entry is the row id
    alone and weights become repeated entries (``tree_kernels.hip`` ``ent_row`` / ``ent_w``)."""
    return n_rows >= MAX_ROWS or os.environ.get("TMOG_TREE_WIDE_ROWS") == "1"

# Native per-group resource slots (stream, staging, histogram buffers; tree_grow_hip.hip slots()): grower calls
# running concurrently from several host threads need disjoint slot ranges. A thread running a whole learner next
# to others (tuning/validators.py concurrent learners) takes a lane of SLOT_LANE slots; every grow_forest call of
# that thread -- and of the threads it starts through ``set_slot_lane`` -- offsets its slot_base by the lane.
N_SLOTS, SLOT_LANE = 32, 8
_lane = threading.local()


_lane_lock = threading.Lock()
_quarantined: set = set()       # lane bases held by abandoned fits (maxWait), never handed out until they exit


def slot_lane() -> int:
    """This thread's slot offset: the lane it was given, else the first lane no abandoned fit holds."""
    base = getattr(_lane, "base", None)
    if base is not None:
        return base
    free = free_lanes()
    if not free:
        raise RuntimeError("every native tree-grower slot lane is held by a fit abandoned at its maxWait deadline")
    return free[0]


def set_slot_lane(base: int) -> None:
    if base < 0 or base + SLOT_LANE > N_SLOTS:
        raise ValueError(f"slot lane {base} outside the {N_SLOTS} native slots")
    _lane.base = int(base)


def free_lanes() -> list:
    """Lane bases not held by an abandoned fit, lowest first."""
    with _lane_lock:
        return [b for b in range(0, N_SLOTS, SLOT_LANE) if b not in _quarantined]


def quarantine_lane(base: int, thread: threading.Thread, on_exit=None) -> None:
    """An abandoned fit (tuning/validators.py maxWait) still runs on lane ``base``: its grow-only native buffers
    must not be shared with another grower, so the lane is withheld until ``thread`` exits (a reaper joins it,
    then runs ``on_exit``, e.g. returning the fit's leased stream)."""
    with _lane_lock:
        _quarantined.add(int(base))

    def reap():
        thread.join()
        if on_exit is not None:
            on_exit()
        with _lane_lock:
            _quarantined.discard(int(base))

    threading.Thread(target=reap, name=f"lane-reaper-{base}", daemon=True).start()


def quarantined_lanes() -> set:
    with _lane_lock:
        return set(_quarantined)


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


def prune_forest(f: Forest, max_depth: int, min_gain: float) -> Forest:
    """The forest a grower run with a smaller ``max_depth`` and / or a larger ``min_info_gain`` would
    have produced from the same nodes: a node stays split only while its depth is below ``max_depth``
    and its recorded split gain is at least ``min_gain`` (the grower accepts a split exactly when its
    best valid candidate's gain >= min_info_gain, and a larger threshold never changes which candidate
    is best, only whether it is accepted); every other node becomes a leaf with its own statistics,
    which the grower records for internal nodes too. Node order stays BFS per tree, as ``_finalize``
    emits it. Lets the model selector grow one forest per (bootstrap, seed, minInstancesPerNode, ...)
    for all of its maxDepth x minInfoGain grid points (``models/trees.py`` ``_ForestLearner``).
    Thresholds are compared on the stored fp32 gain (a split whose fp64 gain lies within one fp32
    ulp of the threshold may be kept). Leaf statistics: a pruned node keeps the totals of its own
    histogram, where direct growth gives a max-depth right child parent - left (fp32): class counts are
    identical, regression / Newton sums agree to fp32 rounding."""
    n = len(f.nodes)
    if n == 0:
        return f
    left = f.nodes[:, 2].astype(np.int64)
    right = f.nodes[:, 3].astype(np.int64)
    keep = np.zeros(n, bool)
    split = np.zeros(n, bool)
    frontier = f.tree_off[:-1].astype(np.int64)
    frontier = frontier[frontier < f.tree_off[1:]]
    keep[frontier] = True
    mg = np.float32(min_gain)
    d = 0
    while frontier.size:
        ok = (left[frontier] >= 0) & (d < max_depth) & (f.gain[frontier] >= mg)
        sp = frontier[ok]
        split[sp] = True
        frontier = np.sort(np.concatenate([left[sp], right[sp]]))
        keep[frontier] = True
        d += 1
    order = np.nonzero(keep)[0]
    new_id = np.full(n, -1, np.int64)
    new_id[order] = np.arange(order.size)
    tree_off = np.searchsorted(order, f.tree_off).astype(np.int64)
    isint = split[order]
    nodes = np.zeros((order.size, 4), np.int32)
    nodes[:, 0] = np.where(isint, f.nodes[order, 0], 0)
    nodes[:, 1] = np.where(isint, f.nodes[order, 1], 0)
    nodes[:, 2] = np.where(isint, new_id[np.maximum(left[order], 0)], -1)
    nodes[:, 3] = np.where(isint, new_id[np.maximum(right[order], 0)], -1)
    return Forest(tree_off, nodes, np.where(isint, f.default_left[order], 0).astype(np.uint8),
                  f.value[order].copy(), np.where(isint, f.gain[order], 0).astype(np.float32),
                  f.cover[order].copy(), f.tree_model.copy(), f.missing_bin)


def pack_rows(rows: torch.Tensor, weights: Optional[torch.Tensor], wide: bool = False) -> torch.Tensor:
    """Pack ``row | weight << 24`` into an int32 tensor (bit pattern read as uint32 by the kernels). ``wide``:
    entries are the row ids themselves, a weight w > 1 repeating the row w times (zero-weight rows dropped)."""
    if wide:
        r = rows.to(torch.int64)
        if weights is not None:
            r = torch.repeat_interleave(r, weights.to(torch.int64).clamp(0, 255).to(r.device))
        return r.to(torch.int32)
    r = rows.to(torch.int64)
    w = torch.ones_like(r) if weights is None else weights.to(torch.int64).clamp(0, 255)
    e = r | (w << 24)
    e = torch.where(e >= (1 << 31), e - (1 << 32), e)
    return e.to(torch.int32)


def poisson_cdf_table(rate: float) -> List[float]:
    """Inverse-CDF steps of Poisson(rate) exactly as ``trees.bootstrap_weights_multi`` compares them."""
    out = []
    p = math.exp(-rate)
    cdf = p
    for i in range(1, 40):
        out.append(cdf)
        p = p * rate / i
        cdf += p
        if 1.0 - cdf < 1e-12:
            break
    return out


def bootstrap_pack(rows: torch.Tensor, seeds: Sequence[int], rate: float, wide: bool = False):
    """Poisson(``rate``) bootstrap of ``rows`` for one tree per seed, packed as tree-engine root
    entries (``row | w << 24``, zero draws dropped): ``(int32 entries, int64 counts per tree)``.

    Multiplicities are ``trees.bootstrap_weights_multi``'s (same per-row uniform, same CDF steps); on
    the GPU one fused HIP kernel (``boost_kernels.hip: poisson_pack_kernel``) draws and packs."""
    from ..tuning.splitters import row_uniform_multi, _s64
    dev = rows.device
    cdf = poisson_cdf_table(rate)
    rid = rows.to(torch.int64).contiguous()
    k, n = len(seeds), int(rid.numel())
    if dev.type == "cuda" and n and k and not wide:
        offs = np.asarray([_s64(int(sd) * 0x632BE59BD9B4E019 + 23 * 0x2545F4914F6CDD1D) for sd in seeds], np.int64)
        pk = _Pack(dev)
        i_o, i_c = pk.add(offs), pk.add(np.asarray(cdf, np.float64))
        dv = pk.ship()
        cnt = torch.zeros(k, dtype=torch.int64, device=dev)
        lib = N.hip()
        N.check(lib.tmog_hip_poisson_pack(N.ptr(rid), n, N.ptr(dv[i_o]), k, N.ptr(dv[i_c]), len(cdf), N.ptr(cnt),
                                          None, None, N.stream(dev)), "poisson_pack count")
        counts = cnt.cpu().numpy()
        base = torch.as_tensor(np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64), device=dev)
        out = torch.empty(max(int(counts.sum()), 1), dtype=torch.int32, device=dev)
        cnt.zero_()
        N.check(lib.tmog_hip_poisson_pack(N.ptr(rid), n, N.ptr(dv[i_o]), k, N.ptr(dv[i_c]), len(cdf), N.ptr(cnt),
                                          N.ptr(base), N.ptr(out), N.stream(dev)), "poisson_pack")
        return out[:int(counts.sum())], counts.astype(np.int64)
    u = row_uniform_multi(rid, seeds, 23)
    w = torch.zeros(u.shape, dtype=torch.int64, device=dev)
    for c in cdf:
        w += (u >= c).to(torch.int64)
    parts, counts = [], []
    for t in range(k):
        keep = w[t] > 0
        parts.append(pack_rows(rid[keep], w[t][keep], wide))
        counts.append(int(parts[-1].numel()))
    out = torch.cat(parts) if parts else torch.zeros(0, dtype=torch.int32, device=dev)
    return out, np.asarray(counts, np.int64)


def _root_rows(jobs, dev, wide: bool = False):
    """Packed root entries of every job, zero-weight (out-of-bag) rows dropped for all weighted jobs
    with one compaction (two host syncs per call instead of one per tree). ``wide``: see :func:`pack_rows`."""
    packs: List[Optional[torch.Tensor]] = [None] * len(jobs)
    counts = [0] * len(jobs)
    if wide:
        for k, j in enumerate(jobs):
            packs[k] = pack_rows(j.rows.to(dev), None if j.weights is None else j.weights.to(dev), True)
            counts[k] = int(packs[k].numel())
        rows = torch.cat(packs) if packs else torch.zeros(0, dtype=torch.int32, device=dev)
        return rows, counts
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


class _GrowArgs(C.Structure):
    """Mirror of ``tmog::GrowArgs`` (ops/csrc/common/tree_grow.hpp)."""
    _fields_ = [("Xb", C.c_void_p), ("N", C.c_int64), ("F", C.c_int32), ("mode", C.c_int32), ("kind", C.c_int32),
                ("S", C.c_int32), ("B", C.c_int32), ("missing_bin", C.c_int32), ("chunk_rows", C.c_int64),
                ("subtract", C.c_int32), ("collect_leaves", C.c_int32), ("y", C.c_void_p), ("t1", C.c_void_p),
                ("t2", C.c_void_p), ("stride", C.c_int64), ("qscale", C.c_void_p), ("qinv", C.c_void_p),
                ("n_bins", C.c_void_p), ("T", C.c_int32), ("job_model", C.c_void_p), ("job_depth", C.c_void_p),
                ("job_min_inst", C.c_void_p), ("job_min_gain", C.c_void_p), ("job_mcw", C.c_void_p),
                ("job_lambda", C.c_void_p), ("job_eps", C.c_void_p), ("job_fsub", C.c_void_p),
                ("job_count", C.c_void_p), ("rows", C.c_void_p), ("rows_alt", C.c_void_p),
                ("leaf_rows", C.c_void_p), ("leaf_gid", C.c_void_p), ("n_groups", C.c_int32),
                ("group_start", C.c_void_p), ("rng_seed", C.c_int64), ("stream", C.c_void_p),
                ("n_bins_host", C.c_void_p), ("csr_ptr", C.c_void_p), ("csr_col", C.c_void_p),
                ("csr_nf", C.c_int32), ("fp_rank", C.c_int32), ("fp_world", C.c_int32), ("fp_mlo", C.c_int32),
                ("fp_mhi", C.c_int32), ("fp_olo", C.c_int32), ("fp_ohi", C.c_int32), ("fp_comm", C.c_void_p),
                ("fp_exchange", C.c_void_p), ("fp_ctx", C.c_void_p), ("slot_base", C.c_int32),
                ("XbT", C.c_void_p), ("gh", C.c_void_p), ("gh_alt", C.c_void_p), ("n_entries", C.c_int64),
                ("wide_rows", C.c_int32), ("Xh", C.c_void_p), ("Fh", C.c_int32)]


class _ResidentIO(C.Structure):
    """Mirror of ``ResidentIO`` (ops/csrc/hip/tree_resident.hip)."""
    _fields_ = [("rec", C.c_void_p), ("gid_value", C.c_void_p), ("gid_tree", C.c_void_p), ("cap_nodes", C.c_int64),
                ("job_eta", C.c_void_p), ("job_gamma", C.c_void_p)]


REC_FIXED = 7     # record words before the S totals: tree feat bin dl gain left right (tree_resident.hip)


@dataclass
class ResidentTree:
    """One device-planned ``grow_forest`` call (``resident=True``): the leaf assignment for the boosting
    epilogue is ready on the device, the created-node records ``rec`` (``[1 + cap, 7 + S]`` int64, row 0 =
    (nodes, leaf entries, error bits)) are read back later, in bulk, by :func:`resident_forests`."""
    leaf_assign: "LeafAssign"
    rec: torch.Tensor
    jobs: list
    mode: int
    kind: int
    S: int
    missing_bin: int


def resident_forests(trees: Sequence[ResidentTree]) -> List[Forest]:
    """Host Forests of device-planned trees: ONE device->host copy of all their records, then the native
    finalisation (``tmog_tree_finalize_cpu``, the host twin of the device's ``tree_finalize_kernel``)."""
    if not trees:
        return []
    recs = [t.rec for t in trees]
    host = torch.cat([r.reshape(-1) for r in recs]).cpu().numpy() if len(recs) > 1 else recs[0].reshape(-1).cpu().numpy()
    out, off = [], 0
    for t in trees:
        W = REC_FIXED + t.S
        sz = int(t.rec.numel())
        blk = host[off:off + sz].reshape(-1, W)
        off += sz
        n, err = int(blk[0, 0]), int(blk[0, 2])
        if err:
            raise RuntimeError(f"device-planned tree growth failed (error bits {err}: 1 = partition cursor mismatch, "
                               f"2 = work-list capacity)")
        r = blk[1:1 + n]
        G = _Nodes(n, t.S)
        G.tree[:] = r[:, 0]
        G.feat[:] = r[:, 1]
        G.bin[:] = r[:, 2]
        G.dl[:] = r[:, 3].astype(np.uint8)
        G.gain[:] = r[:, 4].view(np.float64)
        G.left[:] = r[:, 5]
        G.right[:] = r[:, 6]
        G.tot[:] = np.ascontiguousarray(r[:, REC_FIXED:REC_FIXED + t.S]).view(np.float64)
        K = 1
        out.append(_finalize(t.jobs, G, t.mode, t.kind, K, t.S, t.missing_bin))
    return out


def resident_enabled() -> bool:
    """Device-planned level loop for boosting (``TMOG_TREE_RESIDENT``, default on)."""
    return os.environ.get("TMOG_TREE_RESIDENT", "1") != "0"


_ENTRY_MODELS: Dict[tuple, torch.Tensor] = {}


def _entry_models(models: tuple, counts: tuple, dev) -> torch.Tensor:
    """Model id of every root entry (job j's ``counts[j]`` entries carry ``models[j]``), cached: the boosting
    rounds of one active job set reuse it. One fill per job -- ``torch.repeat_interleave`` with a handful
    of repeats runs one thread per repeat on ROCm (~350 us for 2M entries)."""
    key = (models, counts, str(dev), _stream_key(dev))
    t = _ENTRY_MODELS.get(key)
    if t is None:
        if len(_ENTRY_MODELS) >= 32:
            _ENTRY_MODELS.clear()
        parts = [torch.full((c,), m, dtype=torch.int64, device=dev) for m, c in zip(models, counts) if c]
        t = torch.cat(parts) if parts else torch.zeros(0, dtype=torch.int64, device=dev)
        _ENTRY_MODELS[key] = t
    return t


def _stage_gh(rows: torch.Tensor, counts, jobs, t1f, t2f, qscale, stride: int, wide: bool = False) -> torch.Tensor:
    """``[total, 2]`` int32: each root entry's quantised (q(w g), q(w h)) under its job's model scales -- the
    histogram kernels' ``rintf((w * t) * qscale)`` in the same fp32 operation order (tree_kernels.hip
    stage_row), so the histograms are bit-identical to gathering t1 / t2 per row."""
    dev = rows.device
    e = rows.to(torch.int64) & 0xFFFFFFFF
    r = e if wide else e & 0xFFFFFF
    w = torch.ones_like(e, dtype=torch.float32) if wide else (e >> 24).to(torch.float32)
    model = _entry_models(tuple(int(j.model) for j in jobs), tuple(int(c) for c in counts), dev)
    idx = model * int(stride) + r
    qs = qscale.reshape(-1, qscale.shape[-1])[model]
    g = torch.round((w * t1f.reshape(-1)[idx]) * qs[:, 0]).to(torch.int32)
    h = torch.round((w * t2f.reshape(-1)[idx]) * qs[:, 1]).to(torch.int32)
    return torch.stack([g, h], 1).contiguous()


@dataclass
class FpPlan:
    """This rank's share of a feature-parallel ``grow_forest`` (see parallel/learner_parallel.py):
    positions ``[mlo, mhi)`` of the multi-bin and ``[olo, ohi)`` of the one-present-bin growth-order
    feature lists, and ``one_cols`` = the ``Xb`` columns of that one-present slice (the CSR to build)."""
    par: object                      # parallel.learner_parallel.LearnerParallel
    mlo: int
    mhi: int
    olo: int
    ohi: int
    one_cols: np.ndarray
    sparse: bool = False


def fp_plan(Xb: torch.Tensor, n_bins, par, sparse: bool, force: bool = False) -> Optional[FpPlan]:
    """Split the features of ``Xb`` over ``par``'s ranks for feature-parallel growth (None when not
    possible: one rank, or fewer multi-bin columns than ranks -- then every rank grows everything).
    ``sparse``: MODE_GH with a missing bin, where one-present-bin columns form their own list."""
    from ..parallel.learner_parallel import feature_slices
    if par is None or (par.world <= 1 and not force):
        return None
    nb = np.asarray(n_bins)
    if sparse:
        multi, one = np.nonzero(nb != 1)[0], np.nonzero(nb == 1)[0]
    else:
        multi, one = np.arange(nb.size), np.zeros(0, np.int64)
    if one.size:
        idx = torch.as_tensor(one, dtype=torch.int64, device=Xb.device)
        w = torch.zeros(one.size, dtype=torch.float64, device=Xb.device)
        for r0 in range(0, int(Xb.shape[0]), 1 << 20):
            w += (Xb[r0:r0 + (1 << 20)].index_select(1, idx) == 0).sum(0).to(torch.float64)
        weights = w.cpu().numpy()
    else:
        weights = np.zeros(0)
    sl = feature_slices(int(multi.size), weights, par.world, force=force)
    if sl is None:
        return None
    mlo, mhi, olo, ohi = sl[par.rank]
    return FpPlan(par, mlo, mhi, olo, ohi, one[olo:ohi].astype(np.int64), bool(sparse))


def onebin_csr(Xb: torch.Tensor, n_bins: np.ndarray, block_rows: int = 1 << 20, cols: Optional[np.ndarray] = None):
    """Row-wise CSR of the one-present-bin columns of ``Xb`` (``n_bins == 1``: one-hot / null indicator
    columns under a sparse missing bin), for the histogram kernel's CSR path.

    Returns ``(ptr int64 [N + 1], col int16 [max(nnz, 1)] (read as uint16), n_cols)``: the entries of
    row ``r`` are ``col[ptr[r]:ptr[r + 1]]``, the ids (in ascending column order among the one-bin
    columns) of its columns holding the present bin 0. None when there are none or ids do not fit.
    ``cols``: restrict to these one-present-bin columns (a feature-parallel rank's slice), ids local to
    the subset."""
    nb = np.asarray(n_bins)
    one = np.nonzero(nb == 1)[0] if cols is None else np.asarray(cols, np.int64)
    if one.size == 0 or one.size >= (1 << 16) or Xb.dim() != 2:
        return None
    dev = Xb.device
    idx = torch.as_tensor(one, dtype=torch.int64, device=dev)
    N = int(Xb.shape[0])
    counts, cols = [], []
    for r0 in range(0, N, block_rows):
        nz = Xb[r0:r0 + block_rows].index_select(1, idx) == 0
        counts.append(nz.sum(1))
        cols.append(nz.nonzero()[:, 1].to(torch.int16))    # row-major: sorted by row, then column
    ptr = torch.zeros(N + 1, dtype=torch.int64, device=dev)
    if N:
        torch.cumsum(torch.cat(counts), 0, out=ptr[1:])
    col = torch.cat(cols) if cols else torch.empty(0, dtype=torch.int16, device=dev)
    if col.numel() == 0:
        col = torch.zeros(1, dtype=torch.int16, device=dev)
    return ptr, col.contiguous(), int(one.size)


class _Nodes:
    """Created nodes of one job group, in creation order (what ``_finalize`` consumes)."""

    def __init__(self, n, S):
        self.n = n
        self.tree = np.empty(n, np.int64)
        self.feat = np.empty(n, np.int64)
        self.bin = np.empty(n, np.int64)
        self.dl = np.empty(n, np.uint8)
        self.gain = np.empty(n, np.float64)
        self.tot = np.empty((n, S), np.float64)
        self.left = np.empty(n, np.int64)
        self.right = np.empty(n, np.int64)


def grow_forest(Xb: torch.Tensor, n_bins: np.ndarray, jobs: Sequence[TreeJob], *, mode: int, kind: int,
                n_classes: int = 2, y: Optional[torch.Tensor] = None, t1: Optional[torch.Tensor] = None,
                t2: Optional[torch.Tensor] = None, B: int = 32, missing_bin: int = -1,
                subtract: bool = True, chunk_rows: int = 4096, rng_seed: int = 0,
                collect_leaves: bool = False, groups: Optional[int] = None, csr=None, root=None,
                fp: Optional[FpPlan] = None, slot_base: int = 0, XbT: Optional[torch.Tensor] = None,
                quant_amax: Optional[torch.Tensor] = None, quant_wmax: Optional[float] = None,
                resident: bool = False, prestaged=None, Xh: Optional[torch.Tensor] = None):
    """Grow one tree per job, all jobs level-synchronously. ``Xb`` is ``uint8 [N, F]``.

    The level loop runs natively (``ops/csrc/common/tree_grow.hpp``): on the GPU every job group gets
    its own host thread and HIP stream (default 2 groups) so one group's planning overlaps the other's
    kernels; the CPU backend grows the same groups with the same seeds, bit-identically. Per-node
    feature subsets come from a splitmix64 stream seeded with ``rng_seed + 1000003 * group``.

    ``root``: pre-packed root entries ``(int32 tensor, counts per job)`` (e.g. from ``bootstrap_pack``),
    used instead of the jobs' rows / weights; the tensor is consumed (the grower partitions it in place).

    ``csr``: ``onebin_csr(Xb, n_bins)`` (GPU, ``MODE_GH`` with a missing bin): the one-present-bin
    columns' histograms are then built from the rows' CSR lists (identical results, fewer loads).

    ``collect_leaves``: also return, as ``forest.leaf_assign``, the final leaf of every training entry
    (see ``LeafAssign``) so boosting can update margins without re-walking the new trees.

    ``slot_base``: first native per-group resource slot (stream, staging, histogram buffers) of this call;
    calls running concurrently from several host threads must use disjoint slot ranges.

    ``quant_amax`` ``[n_models, 2]`` float32 / ``quant_wmax``: the per-model max |t1|, max |t2| over all N rows
    and the max entry weight, when the caller already knows them (boosting: the round epilogue computes
    them), instead of scanning ``t1`` / ``t2`` / the entries here -- same scales.

    ``fp``: feature-parallel growth (``fp_plan``): every rank calls with the same jobs, rows and ``Xb``;
    each builds histograms of its feature slice only (``csr`` must then be the slice's, from
    ``onebin_csr(..., cols=fp.one_cols)``) and all ranks return the same forest -- the one a single
    rank would grow. Jobs must not use per-node feature subsets.

    ``Xh``: GPU, optional ``uint8 [N, Fh]`` row-major copy of ``Xb[:, :Fh]`` (``Fh`` a multiple of 64) holding the
    multi-bin columns; the wide-load histogram items read it instead of ``Xb`` (aligned row segments, a smaller
    footprint for the Infinity Cache). Same trees.

    ``resident``: on the GPU, for one job group (``groups=1``), no per-node feature subsets and leaves
    collected, grow with the device-planned level loop (``ops/csrc/hip/tree_resident.hip``): nothing is
    read back, and a :class:`ResidentTree` is returned instead of a Forest (same trees; the host Forest is
    built later by :func:`resident_forests`). Other configurations fall back to the host-planned loop.

    ``prestaged``: ``(rows, counts, gh, qscale, qinv)`` already prepared on this stream by the fused round
    prologue (``boost_prologue``): the root entries (consumed), their quantised statistics and the scales."""
    dev = Xb.device
    on_gpu = dev.type == "cuda"
    slot_base = int(slot_base) + slot_lane()
    Nrows, F = int(Xb.shape[0]), int(Xb.shape[1])
    chunk_rows = int(os.environ.get("TMOG_TREE_CHUNK", chunk_rows))
    wide = wide_rows(Nrows)
    if Nrows >= MAX_WIDE_ROWS:
        raise ValueError(f"tree engine supports < 2^31 rows per training set, got {Nrows}")
    S = n_classes if mode == MODE_CLS else (3 if mode == MODE_VAR else 2)
    K = n_classes if mode == MODE_CLS else 1
    if missing_bin >= B:
        raise ValueError("missing_bin must be < B")
    if S > 256:
        raise ValueError("tree engine supports at most 256 statistics per bin (classes)")
    if on_gpu and (S > 16 or B > 64) and B * S > 16384:
        raise ValueError(f"tree engine (GPU) supports bins x classes <= 16384, got {B} x {S}")
    n_bins_t = _const_tensor(np.asarray(n_bins, np.int32), dev)
    stride = int(t1.shape[1]) if (t1 is not None and t1.dim() == 2) else 0
    yf = y.to(device=dev, dtype=torch.float32).contiguous() if y is not None else None
    t1f = t1.to(device=dev, dtype=torch.float32).contiguous() if t1 is not None else None
    t2f = t2.to(device=dev, dtype=torch.float32).contiguous() if t2 is not None else None
    Xb = Xb.contiguous()
    T = len(jobs)
    ng = groups if groups is not None else min(T, max(1, min(8, int(os.environ.get("TMOG_TREE_GROUPS", "2")))))
    ng = max(1, min(ng, T)) if T else 1
    cuts = np.linspace(0, T, ng + 1).astype(np.int32)
    if prestaged is not None:
        rows, counts = prestaged[0], [int(c) for c in prestaged[1]]
        if len(counts) != len(jobs) or sum(counts) != int(rows.numel()):
            raise ValueError("root entries do not match the jobs")
    elif root is not None:
        rows, counts = root[0].to(device=dev, dtype=torch.int32).contiguous(), [int(c) for c in root[1]]
        if len(counts) != len(jobs) or sum(counts) != int(rows.numel()):
            raise ValueError("root entries do not match the jobs")
    else:
        rows, counts = _root_rows(jobs, dev, wide)
    rows_alt = torch.empty_like(rows)
    total = int(rows.numel())
    gh = gh_alt = None
    if prestaged is not None:
        gh, qscale, qinv = prestaged[2], prestaged[3], prestaged[4]
        gh_alt = torch.empty_like(gh)
    else:
        qscale, qinv = _quant_scales(mode, S, jobs, t1f, t2f, rows, chunk_rows, dev, quant_amax,
                                     1.0 if wide else quant_wmax)
    if gh is None and on_gpu and mode == MODE_GH and total and t1f is not None and t2f is not None \
            and os.environ.get("TMOG_GH_STAGE", "1") != "0":
        gh = _stage_gh(rows, counts, jobs, t1f, t2f, qscale, stride, wide)
        gh_alt = torch.empty_like(gh)
    leaf_rows = torch.empty(max(total, 1), dtype=torch.int32, device=dev) if collect_leaves else None
    leaf_gid = torch.empty(max(total, 1), dtype=torch.int32, device=dev) if collect_leaves else None
    host = dict(
        model=np.array([j.model for j in jobs], np.int32), depth=np.array([j.params.max_depth for j in jobs], np.int32),
        inst=np.array([j.params.min_instances for j in jobs], np.float64),
        gain=np.array([j.params.min_info_gain for j in jobs], np.float64),
        mcw=np.array([j.params.min_child_weight for j in jobs], np.float64),
        lam=np.array([j.params.reg_lambda for j in jobs], np.float64),
        eps=np.array([j.params.split_eps for j in jobs], np.float64),
        fsub=np.array([0 if j.params.feature_subset is None else int(j.params.feature_subset) for j in jobs], np.int32),
        count=np.asarray(counts, np.int64), cuts=cuts, nbins=np.ascontiguousarray(np.asarray(n_bins, np.int32)))
    hp = {k: v.ctypes.data for k, v in host.items()}
    use_csr = (csr is not None and on_gpu and mode == MODE_GH and missing_bin > 0
               and os.environ.get("TMOG_TREE_CSR") != "0")
    if use_csr and (int(csr[0].numel()) != Nrows + 1 or csr[0].device != dev or csr[1].dtype != torch.int16):
        raise ValueError("csr does not match Xb")
    fpw = 0 if fp is None else int(fp.par.world)      # 0 = not feature-parallel
    if fpw > 0:
        if fp.sparse != (mode == MODE_GH and missing_bin >= 0):
            raise ValueError("feature-parallel plan was made for another histogram mode")
        if any(j.params.feature_subset is not None and 0 < int(j.params.feature_subset) < F for j in jobs):
            raise ValueError("feature-parallel growth needs jobs without per-node feature subsets")
        if use_csr and int(csr[2]) != fp.ohi - fp.olo:
            raise ValueError("feature-parallel growth needs the CSR of this rank's one-present-bin slice")
        fp_comm = fp.par.fp.comm_array(dev, ng) if on_gpu else None
        fp_cb = None if on_gpu else fp.par.fp.exchange_fn()
    else:
        fp_comm = fp_cb = None
    a = _GrowArgs(N.ptr(Xb), Nrows, F, mode, kind, S, B, missing_bin, int(chunk_rows), int(bool(subtract)),
                  int(bool(collect_leaves)), N.ptr(yf), N.ptr(t1f), N.ptr(t2f), stride, N.ptr(qscale), N.ptr(qinv),
                  N.ptr(n_bins_t), T, hp["model"], hp["depth"], hp["inst"], hp["gain"], hp["mcw"], hp["lam"], hp["eps"],
                  hp["fsub"], hp["count"], N.ptr(rows), N.ptr(rows_alt), N.ptr(leaf_rows), N.ptr(leaf_gid), ng,
                  hp["cuts"], int(rng_seed), N.stream(dev) if on_gpu else None,
                  hp["nbins"] if (fpw > 0 or os.environ.get("TMOG_TREE_PERM") != "0") else None,
                  N.ptr(csr[0]) if use_csr else None, N.ptr(csr[1]) if use_csr else None,
                  int(csr[2]) if use_csr else 0,
                  int(fp.par.rank) if fpw else 0, fpw, fp.mlo if fpw else 0, fp.mhi if fpw else 0,
                  fp.olo if fpw else 0, fp.ohi if fpw else 0,
                  C.cast(fp_comm, C.c_void_p) if fp_comm is not None else None,
                  C.cast(fp_cb, C.c_void_p) if fp_cb is not None else None, None, int(slot_base),
                  N.ptr(XbT) if (on_gpu and XbT is not None) else None,
                  N.ptr(gh) if gh is not None else None, N.ptr(gh_alt) if gh_alt is not None else None, total,
                  int(wide), N.ptr(Xh) if (on_gpu and Xh is not None) else None,
                  int(Xh.shape[1]) if (on_gpu and Xh is not None) else 0)
    lib = N.hip() if on_gpu else N.host()
    if resident and on_gpu and ng == 1 and collect_leaves:
        rt = _grow_resident(lib, a, jobs, mode, kind, S, missing_bin, leaf_rows, leaf_gid, dev, total, wide)
        if rt is not None:
            return rt
    fn = (lambda name: getattr(lib, f"tmog_hip_{name}")) if on_gpu else (lambda name: getattr(lib, f"tmog_{name}_cpu"))
    side = []
    if on_gpu and ng > 1 and fpw == 0:
        # groups beyond the first run on side streams of the process-wide set (ops/streams.py), shared when
        # fewer are free; the grouping itself (and so every tree) does not depend on how many were free
        from ..ops import streams as SP
        null_base = int(N.stream(dev) or 0) == 0
        side = SP.lease(dev, ng if null_base else ng - 1)
        for g in range(ng):
            k = g if null_base else g - 1
            if k >= 0:
                lib.tmog_hip_slot_stream(slot_base + g, side[k % len(side)].cuda_stream if side else None,
                                         1 if side else 0)
    try:
        h = fn("grow_forest")(C.byref(a))
    finally:
        if side:
            from ..ops import streams as SP
            SP.release(dev, side)
    try:
        msg = C.create_string_buffer(512)
        if fn("grow_status")(h, msg, 512) != 0:
            raise RuntimeError(f"native tree grower failed: {msg.value.decode(errors='replace')}")
        forests, las = [], []
        entry0 = np.concatenate([[0], np.cumsum(host["count"])])
        for g in range(ng):
            n = int(fn("grow_nodes")(h, g))
            G = _Nodes(n, S)
            fn("grow_copy")(h, g, G.tree.ctypes.data, G.feat.ctypes.data, G.bin.ctypes.data, G.dl.ctypes.data,
                            G.gain.ctypes.data, G.tot.ctypes.data, G.left.ctypes.data, G.right.ctypes.data)
            gj = list(jobs[cuts[g]:cuts[g + 1]])
            f = _finalize(gj, G, mode, kind, K, S, missing_bin, with_gid_values=collect_leaves)
            if collect_leaves:
                lc = int(fn("grow_leaf_count")(h, g))
                e0 = int(entry0[cuts[g]])
                pk = _Pack(dev)
                i_v, i_t = pk.add(f._gid_value), pk.add(f._gid_tree + int(cuts[g]))
                dv = pk.ship()
                las.append((leaf_rows[e0:e0 + lc], leaf_gid[e0:e0 + lc], dv[i_v], dv[i_t]))
                del f._gid_value, f._gid_tree
            forests.append(f)
    finally:
        fn("grow_free")(h)
    forest = forests[0] if ng == 1 else Forest.concat(forests)
    if collect_leaves:
        if ng == 1:
            r_, g_, v_, t_ = las[0]
            forest.leaf_assign = LeafAssign(r_, g_, v_, t_, wide)
        else:
            goff = np.concatenate([[0], np.cumsum([int(x[2].shape[0]) for x in las])[:-1]])
            forest.leaf_assign = LeafAssign(torch.cat([x[0] for x in las]),
                                            torch.cat([x[1] + int(o) for x, o in zip(las, goff)]),
                                            torch.cat([x[2] for x in las]), torch.cat([x[3] for x in las]), wide)
    return forest


def _grow_resident(lib, a, jobs, mode, kind, S, missing_bin, leaf_rows, leaf_gid, dev, total,
                   wide: bool = False) -> Optional[ResidentTree]:
    cap = int(lib.tmog_hip_resident_cap_nodes(C.byref(a)))
    if cap <= 0:
        return None
    rec = torch.empty(1 + cap, REC_FIXED + S, dtype=torch.int64, device=dev)
    gid_value = torch.empty(cap, dtype=torch.float32, device=dev)
    gid_tree = torch.empty(cap, dtype=torch.int64, device=dev)
    eta = np.ascontiguousarray([j.params.eta for j in jobs], np.float64)
    gam = np.ascontiguousarray([j.params.gamma for j in jobs], np.float64)
    io = _ResidentIO(N.ptr(rec), N.ptr(gid_value), N.ptr(gid_tree), cap, eta.ctypes.data, gam.ctypes.data)
    rc = int(lib.tmog_hip_grow_resident(C.byref(a), C.byref(io)))
    if rc == 1:
        return None
    if rc != 0:
        msg = C.create_string_buffer(512)
        lib.tmog_hip_resident_error(msg, 512)
        raise RuntimeError(f"device-planned tree growth failed: {msg.value.decode(errors='replace')}")
    la = LeafAssign(leaf_rows[:total], leaf_gid[:total], gid_value, gid_tree, wide)
    return ResidentTree(la, rec, list(jobs), mode, kind, S, missing_bin)


@dataclass
class LeafAssign:
    """Final leaf of every training entry of a ``grow_forest`` call: ``rows`` (packed entries, as
    given to the trees), ``gid`` (node id per entry), ``value[gid]`` (leaf output, pruning applied),
    ``tree[gid]`` (job index). ``per_tree_values`` turns it into margin updates."""
    rows: torch.Tensor
    gid: torch.Tensor
    value: torch.Tensor
    tree: torch.Tensor
    wide: bool = False          # entries are plain row ids (training sets of >= 2^24 rows)

    def row_ids(self) -> torch.Tensor:
        if self.wide:
            return self.rows.to(torch.int64) & 0xFFFFFFFF
        return (self.rows & 0xFFFFFF).to(torch.int64)

    def entry_tree(self) -> torch.Tensor:
        return self.tree[self.gid.to(torch.int64)]

    def entry_value(self) -> torch.Tensor:
        return self.value[self.gid.to(torch.int64)]


from ..ops.staging import Pack as _Pack  # noqa: E402  (re-exported for the learners)


_CONST: dict = {}


def _stream_key(dev) -> int:
    """The calling thread's current stream on ``dev`` (0 on the host). The device-tensor caches below are kept
    per stream: a cached tensor is then only ever read by kernels of the stream it was allocated on, so when an
    eviction frees it the caching allocator can hand its block only to later work of that same stream. Shared
    across streams (the boosting parts, the learner lanes), an evicted tensor's block could be reused on its
    allocation stream while another stream's queued kernels still read it -- stale index tensors, and faults."""
    dev = torch.device(dev)
    return int(torch.cuda.current_stream(dev).cuda_stream) if dev.type == "cuda" else 0


def _const_tensor(a: np.ndarray, dev) -> torch.Tensor:
    """Device copy of a small constant host array, cached by content and stream (no per-call blocking copy)."""
    key = (str(dev), _stream_key(dev), a.dtype.str, a.shape, a.tobytes())
    t = _CONST.get(key)
    if t is None:
        if len(_CONST) > 256:
            _CONST.clear()
        t = _CONST[key] = torch.as_tensor(a, device=dev)
    return t


def quant_qmax(chunk_rows: int = 4096) -> float:
    """Per-row bound of a quantised statistic: an LDS partial sums at most max(chunk_rows, CSR_ITEM_ROWS) rows
    (CSR items always span 1024 rows, tree_grow.hpp kCsrRows), and must fit int32."""
    chunk_rows = int(os.environ.get("TMOG_TREE_CHUNK", chunk_rows))
    return float(min(1 << 22, (2 ** 31 - 1) // max(1, int(chunk_rows), CSR_ITEM_ROWS) - 1))


def boost_prologue(root: torch.Tensor, counts, act, G: torch.Tensor, H: torch.Tensor, amax: torch.Tensor,
                   comp: torch.Tensor, tam_prev: Optional[torch.Tensor], tam_next: torch.Tensor, out: dict,
                   wide: bool = False):
    """Set-up of one device-resident boosting round in a single launch (ops/csrc/hip/boost_kernels.hip
    boost_prologue_kernel): the quantisation maxima of the active jobs ``act`` (model index = job) from
    ``comp`` and the previous epilogue's ``tam_prev`` (None: first round, ``amax`` as it is), their
    power-of-two scales, a copy of the packed ``root`` entries and their quantised (g, h); zeroes the jobs'
    entries of ``tam_next``. ``out`` holds the reusable buffers; returns grow_forest's ``prestaged``."""
    dev = root.device
    total = int(root.numel())
    P = int(G.shape[0])
    if out.get("rows") is None or out["rows"].numel() < total:
        out["rows"] = torch.empty(max(total, 1), dtype=torch.int32, device=dev)
        out["gh"] = torch.empty(max(total, 1), 2, dtype=torch.int32, device=dev)
    if out.get("qscale") is None:
        out["qscale"] = torch.ones(P, 2, dtype=torch.float32, device=dev)
        out["qinv"] = torch.ones(P, 2, dtype=torch.float64, device=dev)
    rows, gh = out["rows"][:total], out["gh"][:total]
    act_t = _const_tensor(np.asarray(act, np.int32), dev)
    off = _const_tensor(np.concatenate([[0], np.cumsum(np.asarray(counts, np.int64))]).astype(np.int64), dev)
    rc = N.hip().tmog_hip_boost_prologue(N.ptr(tam_prev) if tam_prev is not None else None, N.ptr(tam_next),
                                         N.ptr(comp), N.ptr(amax), P, N.ptr(act_t), len(act), N.ptr(off),
                                         N.ptr(root), N.ptr(rows), total, N.ptr(G), N.ptr(H), int(G.shape[1]),
                                         N.ptr(gh), N.ptr(out["qscale"]), N.ptr(out["qinv"]), quant_qmax(),
                                         int(bool(wide)), N.stream(dev))
    if rc != 0:
        raise RuntimeError(f"boost prologue launch failed ({rc})")
    return rows, list(counts), gh, out["qscale"], out["qinv"]


def _quant_scales(mode, S, jobs, t1f, t2f, rows, chunk_rows, dev, amax_hint=None, wmax_hint=None):
    """Per-(model, stat) power-of-two fixed-point scales for the int64 histograms (see the
    "Fixed-point statistics" note in ops/csrc/hip/tree_kernels.hip). A row's contribution is
    ``rint(v * scale)`` with ``|v * scale| <= qmax``, so a ``chunk_rows``-row LDS partial fits int32.
    Computed on the device (no host sync); returns (float32 scales, float64 inverses), ``[n_models, S]``."""
    n_models = max([j.model for j in jobs], default=0) + 1
    if mode == MODE_CLS or rows.numel() == 0:
        one = torch.ones(n_models, S, dtype=torch.float32, device=dev)
        return one, one.to(torch.float64)
    qmax = quant_qmax(chunk_rows)
    wmax = torch.tensor(float(wmax_hint), dtype=torch.float32, device=dev) if wmax_hint is not None else \
        ((rows >> 24) & 0xFF).max().to(torch.float32)

    def amax(t, k=0):
        if amax_hint is not None:
            return amax_hint[:n_models, k].to(torch.float32)
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
        # 2^floor(log2 x) built from the exponent bits of x = qmax / bound (an IEEE division, not torch's
        # reciprocal-times-scalar): exact and identical on every device, and the same bits as the fused round
        # prologue (boost_kernels.hip pow2_scale)
        b = (bound * wmax).to(torch.float32).clamp_min(1e-30)
        x = torch.full_like(b, qmax) / b
        e = ((x.view(torch.int32) >> 23) & 0xFF) - 127
        return ((e.clamp(-60, 60) + 127) << 23).to(torch.int32).view(torch.float32)

    if mode == MODE_VAR:
        m1 = amax(t1f)
        sc = torch.stack([torch.ones_like(m1), pow2(m1), pow2(m1 * m1)], 1)
    else:
        sc = torch.stack([pow2(amax(t1f, 0)), pow2(amax(t2f, 1))], 1)
    sc = sc.to(torch.float32).contiguous()
    return sc, (1.0 / sc.to(torch.float64)).contiguous()


def _finalize(jobs, G: "_Nodes", mode, kind, K, S, missing_bin, with_gid_values: bool = False):
    """Created nodes -> Forest (values, gamma pruning, per-tree regrouping): native
    ``tmog_tree_finalize_cpu`` (ops/csrc/host/tree_cpu.cpp), array-identical to ``_finalize_py``."""
    if os.environ.get("TMOG_FINALIZE_PY") == "1":
        return _finalize_py(jobs, G, mode, kind, K, S, missing_bin, with_gid_values)
    n = G.n
    T = len(jobs)
    lam = np.ascontiguousarray([j.params.reg_lambda for j in jobs], np.float64)
    eta = np.ascontiguousarray([j.params.eta for j in jobs], np.float64)
    gam = np.ascontiguousarray([j.params.gamma for j in jobs], np.float64)
    tree_off = np.empty(T + 1, np.int64)
    nodes = np.empty((max(n, 1), 4), np.int32)
    dl = np.empty(max(n, 1), np.uint8)
    value = np.empty((max(n, 1), K), np.float32)
    gain = np.empty(max(n, 1), np.float32)
    cover = np.empty(max(n, 1), np.float32)
    gid_value = np.empty((max(n, 1), K), np.float32) if with_gid_values else None
    tot = np.ascontiguousarray(G.tot[:n])
    m = int(N.host().tmog_tree_finalize_cpu(
        n, T, G.tree.ctypes.data, G.feat.ctypes.data, G.bin.ctypes.data, G.dl.ctypes.data, G.gain.ctypes.data,
        tot.ctypes.data, S, G.left.ctypes.data, G.right.ctypes.data, mode, kind, K, lam.ctypes.data,
        eta.ctypes.data, gam.ctypes.data, int(bool(with_gid_values)), tree_off.ctypes.data, nodes.ctypes.data,
        dl.ctypes.data, value.ctypes.data, gain.ctypes.data, cover.ctypes.data,
        gid_value.ctypes.data if with_gid_values else None))
    f = Forest(tree_off, nodes[:m].copy(), dl[:m].copy(), value[:m].copy(), gain[:m].copy(), cover[:m].copy(),
               np.array([j.model for j in jobs], np.int32), missing_bin)
    if with_gid_values:
        f._gid_value, f._gid_tree = gid_value[:n], G.tree[:n].astype(np.int64)
    return f


def _finalize_py(jobs, G: "_Nodes", mode, kind, K, S, missing_bin, with_gid_values: bool = False):
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
    # propagate reachability one tree level per vectorized pass (children are created after parents)
    internal = np.nonzero(left >= 0)[0]
    while internal.size:
        hit = internal[reach[internal]]
        fresh = hit[~(reach[left[hit]] & reach[right[hit]])]
        if fresh.size == 0:
            break
        reach[left[fresh]] = True
        reach[right[fresh]] = True
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
        resolved = reach.copy()
        un = np.nonzero(~reach)[0]
        while un.size:      # one level below the resolved frontier per pass
            cand = un[resolved[parent[un]]]
            if cand.size == 0:
                break
            gid_value[cand] = gid_value[parent[cand]]
            resolved[cand] = True
            un = un[~resolved[un]]
    f = Forest(tree_off, nodes, np.where(isint, G.dl[:n][order], 0).astype(np.uint8),
                  value[order].astype(np.float32).reshape(order.size, K),
                  np.where(isint, gain[order], 0).astype(np.float32), cover[order].astype(np.float32),
                  np.array([j.model for j in jobs], np.int32), missing_bin)
    if with_gid_values:
        f._gid_value, f._gid_tree = gid_value, tree.astype(np.int64)
    return f


_PM_VK = 32      # tree_kernels.hip forest_predict_multi_kernel: variants x classes per model


def _pm_lds_bytes(F: int) -> int:
    """LDS of one forest_predict_multi_kernel workgroup: 64 staged rows of F bins + 64 x 4 x 32 fp32
    accumulators (tmog_hip_forest_predict_multi)."""
    return ((64 * F + 15) & ~15) + 4 * _PM_VK * 64 * 4


def _lds_limit(dev) -> int:
    """LDS one workgroup may allocate (gfx950: 160 KB; the launcher refuses more with -3)."""
    return 160 * 1024


def forest_predict_multi(forest: Forest, Xb: torch.Tensor, model_rows: Sequence[Optional[torch.Tensor]],
                         model_trees: Sequence[Sequence[int]],
                         model_variants: Sequence[Sequence[Tuple[int, float]]]) -> List[List[torch.Tensor]]:
    """Predictions of pruned variants of shared trees: model m's trees are grown trees and each of its
    variants ``(max_depth, min_info_gain)`` is the forest ``prune_forest(trees, max_depth, min_info_gain)``
    would give. On the GPU every (row, tree) is walked once for all of a model's variants
    (``forest_predict_multi_kernel``); elsewhere (or for class counts the kernel does not take) each
    variant is pruned and predicted on its own. Returns ``[model][variant] -> float32 [n_m, K]``."""
    dev = Xb.device
    K = forest.K
    F = int(Xb.shape[1]) if Xb.dim() == 2 else 0
    if dev.type != "cuda" or K not in (1, 2, 4, 8) or any(len(v) * K > _PM_VK or len(v) > 32
                                                         for v in model_variants) \
            or _pm_lds_bytes(F) > _lds_limit(dev):
        res = []
        for rows, ts, vs in zip(model_rows, model_trees, model_variants):
            sub = Forest.concat([forest.tree(int(t)) for t in ts])
            res.append([forest_predict(prune_forest(sub, d, g), Xb, [rows], [list(range(sub.n_trees))])[0]
                        for d, g in vs])
        return res
    Xb = Xb.contiguous()
    Nrows, F = int(Xb.shape[0]), int(Xb.shape[1])
    order = [t for ts in model_trees for t in ts]
    mto = np.zeros(len(model_trees) + 1, np.int64)
    mto[1:] = np.cumsum([len(ts) for ts in model_trees])
    counts = [Nrows if r is None else int(r.numel()) for r in model_rows]
    mro = np.zeros(len(model_rows) + 1, np.int64)
    mro[1:] = np.cumsum(counts)
    voff = np.zeros(len(model_variants) + 1, np.int32)
    voff[1:] = np.cumsum([len(v) for v in model_variants])
    vdep = np.asarray([d for vs in model_variants for d, _ in vs], np.int32)
    vout = np.zeros(max(1, int(voff[-1])), np.int64)
    pos = 0
    for m, vs in enumerate(model_variants):
        for k in range(len(vs)):
            vout[int(voff[m]) + k] = pos
            pos += counts[m] * K
    # per-node variant stop bits of the depth-independent part of prune_forest's rule: a grown leaf stops
    # every variant, an internal node those whose min gain exceeds its split gain (fp32 compare)
    mask = np.zeros(len(forest.nodes), np.uint32)
    leaf = forest.nodes[:, 2] < 0
    for m, vs in enumerate(model_variants):
        sel = np.zeros(len(forest.nodes), bool)
        for t in model_trees[m]:
            sel[int(forest.tree_off[t]):int(forest.tree_off[t + 1])] = True
        bits = np.zeros(len(forest.nodes), np.uint32)
        for k, (_, g) in enumerate(vs):
            bits |= ((forest.gain < np.float32(g)) | leaf).astype(np.uint32) << np.uint32(k)
        mask[sel] = bits[sel]
    pk = _Pack(dev)
    ids = [pk.add(forest.tree_off[:-1][order].astype(np.int64)), pk.add(np.ones(len(order), np.float32)),
           pk.add(np.ascontiguousarray(forest.nodes)), pk.add(forest.default_left),
           pk.add(np.ascontiguousarray(forest.value, np.float32)), pk.add(mask.view(np.int32))]
    i_v = [pk.add(voff), pk.add(vdep), pk.add(vout), pk.add(mro), pk.add(mto)]
    row_list = torch.cat([(torch.arange(Nrows, device=dev) if r is None else r.to(dev)).to(torch.int32)
                          for r in model_rows])
    dv = pk.ship()
    t_off, t_w, nodes, dl, lv, gn = (dv[i] for i in ids)
    voff_t, vdep_t, vout_t, mro_t, mto_t = (dv[i] for i in i_v)
    out = torch.empty(max(pos, 1), dtype=torch.float32, device=dev)
    N.check(N.hip().tmog_hip_forest_predict_multi(
        N.ptr(Xb), F, len(model_rows), N.ptr(mro_t), N.ptr(row_list), max(counts) if counts else 0, N.ptr(mto_t),
        N.ptr(t_off), N.ptr(t_w), N.ptr(nodes), N.ptr(dl), forest.missing_bin, N.ptr(lv), K, N.ptr(gn), N.ptr(voff_t),
        N.ptr(vdep_t), N.ptr(vout_t), N.ptr(out), N.stream(dev)), "forest_predict_multi")
    res = []
    for m, vs in enumerate(model_variants):
        res.append([out[int(vout[int(voff[m]) + k]):int(vout[int(voff[m]) + k]) + counts[m] * K].view(counts[m], K)
                    for k in range(len(vs))])
    return res


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
    pk = _Pack(dev)
    ids = [pk.add(forest.tree_off[:-1][order].astype(np.int64)), pk.add(tw[order]),
           pk.add(np.ascontiguousarray(forest.nodes)), pk.add(forest.default_left),
           pk.add(np.ascontiguousarray(forest.value, np.float32))]
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
    i_mro, i_mto = pk.add(mro), pk.add(mto)
    dv = pk.ship()
    t_off, t_w, nodes, dl, lv = (dv[i] for i in ids)
    mro_t, mto_t = dv[i_mro], dv[i_mto]
    out = torch.zeros(int(mro[-1]), K, dtype=torch.float32, device=dev)
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

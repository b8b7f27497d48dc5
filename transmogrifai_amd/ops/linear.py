"""Dense linear-algebra entry points used by the learners and statistics.

``gemm``/``gemm_t`` are the two halves of every linear-model iteration (``M = X V`` and
``G = X^T R``); on device they run on the matrix cores (hipBLASLt via torch for these plain
library-shaped GEMMs, fp32 in / fp32 accumulate), on the host through BLAS.
"""
from __future__ import annotations

import os
from typing import Optional

import torch


def _dense_mfma(X) -> bool:
    """A contiguous fp32 device design whose products run on the matrix-core row GEMMs (ops/dense.py) when
    ``TMOG_DENSE_MFMA=1`` (default: hipBLASLt, measured faster on these shapes)."""
    from .dense import enabled
    return isinstance(X, torch.Tensor) and X.is_cuda and X.dtype == torch.float32 and X.dim() == 2 and \
        X.is_contiguous() and enabled()


def gemm(X, V: torch.Tensor) -> torch.Tensor:
    """``X [N, d] @ V [d, P]`` in X's dtype (a :class:`SparseDesign` multiplies its dense and sparse parts; a dense
    fp32 device design runs ``dense_kernels.hip`` rowgemm)."""
    if isinstance(X, SparseDesign):
        return X.mm(V)
    if _dense_mfma(X):
        from . import dense as DN
        return DN.mm(X, V.to(torch.float32))
    return X @ V.to(X.dtype)


def gemm_t(X, R: torch.Tensor) -> torch.Tensor:
    """``X^T [d, N] @ R [N, P]`` in X's dtype (fp64 for a :class:`SparseDesign`, and for a dense fp32 device
    design: ``dense_kernels.hip`` xtd -- fp32 matrix-core chunks, fp64 across chunks)."""
    if isinstance(X, SparseDesign):
        return X.tmm(R)
    if _dense_mfma(X):
        from . import dense as DN
        return DN.tmm(X, R.to(torch.float32))
    return X.t() @ R.to(X.dtype)


_SPMM_MAXC = 256       # sparse_kernels.hip kMaxC: output columns per launch
_SEG_NNZ = 4096        # non-zeros per CSC segment (one wave each)


class SparseDesign:
    """A design matrix split into its dense columns (a dense fp32 block: library GEMM) and its sparse columns
    (device CSR for ``X V`` + segmented CSC for ``X^T R``, ``ops/csrc/hip/sparse_kernels.hip``). Built once per
    learner fit from the dense (compacted) matrix; the multi-class text configuration's 1352 columns are
    ~3 % non-zero, so an objective evaluation reads ~44 entries per row instead of 1352."""

    DENSE_FRAC = 0.25

    def __init__(self, X: torch.Tensor, chunk: int = 1 << 16):
        dev = X.device
        N, d = X.shape
        self.shape = (N, d)
        self.device, self.dtype = dev, torch.float32
        nz = torch.zeros(d, dtype=torch.int64, device=dev)
        for a in range(0, N, chunk):
            nz += (X[a:a + chunk] != 0).sum(0)
        dense = nz > self.DENSE_FRAC * max(N, 1)
        self.idx_d = torch.nonzero(dense).reshape(-1)
        self.idx_s = torch.nonzero(~dense).reshape(-1)
        self.Xd = X.index_select(1, self.idx_d).to(torch.float32).contiguous()
        ds = int(self.idx_s.numel())
        self.ds = ds
        rows, cols, vals = [], [], []
        for a in range(0, N, chunk):
            Xc = X[a:a + chunk].index_select(1, self.idx_s)
            ij = torch.nonzero(Xc)
            rows.append(ij[:, 0] + a)
            cols.append(ij[:, 1])
            vals.append(Xc[ij[:, 0], ij[:, 1]].to(torch.float32))
        r = torch.cat(rows) if rows else torch.zeros(0, dtype=torch.int64, device=dev)
        c = torch.cat(cols) if cols else torch.zeros(0, dtype=torch.int64, device=dev)
        v = torch.cat(vals) if vals else torch.zeros(0, dtype=torch.float32, device=dev)
        self.nnz = int(r.numel())
        self.row_ptr = torch.zeros(N + 1, dtype=torch.int64, device=dev)
        self.row_ptr[1:] = torch.cumsum(torch.bincount(r, minlength=N), 0)
        self.col = c.to(torch.int32).contiguous()
        self.val = v.contiguous()
        order = torch.argsort(c * max(N, 1) + r)
        self.csc_row = r[order].to(torch.int32).contiguous()
        self.csc_val = v[order].contiguous()
        self.csc_val_sq = (self.csc_val * self.csc_val).contiguous()
        cnt = torch.bincount(c, minlength=ds)
        col_start = torch.zeros(ds + 1, dtype=torch.int64, device=dev)
        col_start[1:] = torch.cumsum(cnt, 0)
        nseg = (cnt + _SEG_NNZ - 1) // _SEG_NNZ
        self.col_seg = torch.zeros(ds + 1, dtype=torch.int64, device=dev)
        self.col_seg[1:] = torch.cumsum(nseg, 0)
        n_seg = int(self.col_seg[-1].item()) if ds else 0
        seg_col = torch.repeat_interleave(torch.arange(ds, device=dev), nseg)
        within = torch.arange(n_seg, device=dev) - self.col_seg[seg_col]
        self.seg_begin = torch.cat([col_start[seg_col] + within * _SEG_NNZ,
                                    torch.tensor([self.nnz], dtype=torch.int64, device=dev)]).contiguous()
        self.n_seg = n_seg

    @staticmethod
    def worthwhile(X: torch.Tensor) -> bool:
        """GPU, wide and mostly zero: worth the CSR build (decided on a row sample)."""
        if not (X.is_cuda and X.dim() == 2 and X.shape[1] >= 256 and X.shape[0] >= 4096):
            return False
        samp = X[:: max(1, X.shape[0] // 8192)]
        return float((samp != 0).float().mean()) < 0.1

    def mm(self, V: torch.Tensor) -> torch.Tensor:
        from . import _native as N_
        V = V.to(torch.float32)
        M = (self.Xd @ V.index_select(0, self.idx_d)).contiguous() if self.idx_d.numel() else \
            torch.zeros(self.shape[0], V.shape[1], dtype=torch.float32, device=self.device)
        if self.ds:
            Vs = V.index_select(0, self.idx_s).contiguous()
            C = V.shape[1]
            for c0 in range(0, C, _SPMM_MAXC):
                c1 = min(C, c0 + _SPMM_MAXC)
                Vc = Vs[:, c0:c1].contiguous()
                out = M if (c0 == 0 and c1 == C) else M[:, c0:c1]
                if out.is_contiguous() or c1 - c0 == C:
                    N_.check(N_.hip().tmog_hip_csr_spmm(N_.ptr(self.row_ptr), N_.ptr(self.col), N_.ptr(self.val),
                                                        self.shape[0], N_.ptr(Vc), c1 - c0, N_.ptr(out), C, 1,
                                                        N_.stream(self.device)), "csr_spmm")
                else:       # column chunk of a wider output: row stride C, start at column c0
                    N_.check(N_.hip().tmog_hip_csr_spmm(N_.ptr(self.row_ptr), N_.ptr(self.col), N_.ptr(self.val),
                                                        self.shape[0], N_.ptr(Vc), c1 - c0, M.data_ptr() + 4 * c0,
                                                        C, 1, N_.stream(self.device)), "csr_spmm")
        return M

    def tmm(self, R: torch.Tensor, square: bool = False) -> torch.Tensor:
        """``X^T R`` (``(X*X)^T R`` with ``square``) in fp64, ``[d, C]``."""
        from . import _native as N_
        N, d = self.shape
        R = R.to(torch.float32).contiguous()
        C = R.shape[1]
        G = torch.zeros(d, C, dtype=torch.float64, device=self.device)
        if self.idx_d.numel():
            Xd = self.Xd * self.Xd if square else self.Xd
            G[self.idx_d] = (Xd.t() @ R).to(torch.float64)
        if self.ds:
            vals = self.csc_val_sq if square else self.csc_val
            Gs = torch.empty(self.ds, C, dtype=torch.float64, device=self.device)
            for c0 in range(0, C, _SPMM_MAXC):
                c1 = min(C, c0 + _SPMM_MAXC)
                Rc = R[:, c0:c1].contiguous()
                part = torch.empty(max(self.n_seg, 1), c1 - c0, dtype=torch.float32, device=self.device)
                Gc = torch.empty(self.ds, c1 - c0, dtype=torch.float64, device=self.device)
                N_.check(N_.hip().tmog_hip_csc_spmm_t(N_.ptr(self.seg_begin), N_.ptr(self.csc_row), N_.ptr(vals),
                                                      self.n_seg, N_.ptr(self.col_seg), self.ds, N_.ptr(Rc), c1 - c0,
                                                      c1 - c0, N_.ptr(part), N_.ptr(Gc), N_.stream(self.device)),
                         "csc_spmm_t")
                Gs[:, c0:c1] = Gc
            G[self.idx_s] = Gs
        return G


def softmax_objective(M: torch.Tensor, y: torch.Tensor, W: torch.Tensor, bias: torch.Tensor, P: int, K: int,
                      grad: bool):
    """Fused multinomial epilogue (``sparse_kernels.hip`` softmax_epilogue_kernel + colsum_kernel) over the margins
    ``M [N, P*K]`` (problem-major columns, no bias): returns ``(f [P] = sum_i W l, rsum [P*K] or None)`` in
    fp64; with ``grad`` M is overwritten by ``R = W (softmax - onehot(y))``."""
    from . import _native as N_
    dev = M.device
    N = M.shape[0]
    Wf = W.to(torch.float32).contiguous()
    yf = y.to(device=dev, dtype=torch.float32).contiguous()
    bf = bias.to(torch.float32).contiguous()
    Lw = torch.empty(N, P, dtype=torch.float32, device=dev)
    N_.check(N_.hip().tmog_hip_softmax_epilogue(N_.ptr(M), N, P, K, N_.ptr(bf), N_.ptr(yf), N_.ptr(Wf), P,
                                                N_.ptr(Lw), int(grad), N_.stream(dev)), "softmax_epilogue")
    nblk = max(1, min(1024, (N + 255) // 256))
    fp = torch.empty(nblk, P, dtype=torch.float64, device=dev)
    N_.check(N_.hip().tmog_hip_colsum(N_.ptr(Lw), N, P, nblk, N_.ptr(fp), N_.stream(dev)), "colsum")
    f = fp.sum(0)
    rs = None
    if grad:
        rp = torch.empty(nblk, P * K, dtype=torch.float64, device=dev)
        N_.check(N_.hip().tmog_hip_colsum(N_.ptr(M), N, P * K, nblk, N_.ptr(rp), N_.stream(dev)), "colsum")
        rs = rp.sum(0)
    return f, rs


LOSS_CODES = {"logistic": 0, "hinge": 1, "squared": 2}
_LR_DMAX = 384          # one-pass kernel: 64-row X tile + V resident in LDS
_LR_WIDE_DMAX = 2048    # wide kernel: library GEMM margins + fused epilogue / MFMA gradient
_LR_PC = 32


def fused_objective_supported(X) -> bool:
    """The fused HIP objective handles fp32 ``X`` on the GPU with ``d <= 2048`` columns (one pass over X
    up to 384 columns, a library GEMM plus one fused pass above)."""
    if isinstance(X, SparseDesign):
        return False
    return X.is_cuda and X.dtype == torch.float32 and X.dim() == 2 and 1 <= X.shape[1] <= _LR_WIDE_DMAX \
        and X.is_contiguous()


def _n_blocks(N: int, grad: bool = True) -> int:
    # persistent workgroups: as many per CU as the pass's tile fits in LDS (linear_kernels.hip: one 64-row or
    # two 32-row tiles per CU), each keeping its next tile's loads in flight
    from . import _native as N_
    props = torch.cuda.get_device_properties(torch.cuda.current_device())
    per_cu = int(N_.hip().tmog_hip_lr_blocks_per_cu(int(grad)))
    return max(1, min((N + 31) // 32, props.multi_processor_count * per_cu))


def fused_objective(X: torch.Tensor, y: torch.Tensor, W: torch.Tensor, V: torch.Tensor, bias: torch.Tensor,
                    loss: str, yscale=None, grad: bool = True):
    """One pass of the fused HIP objective (``ops/csrc/hip/linear_kernels.hip``) for P problems.

    ``m = X V + bias``; returns ``(f [P], r [P], G [d, P] or None)`` in fp64 with ``f = sum_i W l(m)``,
    ``r = sum_i W l'(m)``, ``G = X^T (W * l'(m))``. Problems are processed 32 per launch."""
    from . import _native as N_
    N, d = X.shape
    P = W.shape[1]
    dev = X.device
    if d <= _LR_DMAX and (X.data_ptr() % 16 or N * d < 16):
        # the kernel streams X in 16-byte chunks from a 16-byte aligned base (it loads a ragged end of the
        # last tile itself, so every problem column is computed the same whatever the other columns are)
        Nm = 0
        parts = []
        if Nm:
            parts.append(fused_objective(X[:Nm], y[:Nm], W[:Nm], V, bias, loss, yscale, grad))
        parts.append(_torch_objective(X[Nm:], y[Nm:], W[Nm:], V, bias, loss, yscale, grad))
        f = sum(q[0] for q in parts)
        r = sum(q[1] for q in parts)
        G = sum(q[2] for q in parts) if grad else None
        return f, r, G
    yf = y.to(device=dev, dtype=torch.float32).contiguous()
    Wf = W.to(torch.float32).contiguous()
    if d <= _LR_DMAX:
        nblk = _n_blocks(N, grad)
    else:                                   # the wide-d epilogue kernel: one 512-thread workgroup per CU
        nblk = max(1, min((N + 63) // 64, torch.cuda.get_device_properties(dev).multi_processor_count))
    dpad = ((d + 15) // 16) * 16
    f = torch.empty(P, dtype=torch.float64, device=dev)
    r = torch.empty(P, dtype=torch.float64, device=dev)
    G = torch.empty(d, P, dtype=torch.float64, device=dev) if grad else None
    fp = torch.empty(nblk, _LR_PC, dtype=torch.float64, device=dev)
    rp = torch.empty_like(fp)
    gp = torch.empty(nblk, dpad, _LR_PC, dtype=torch.float32, device=dev) if grad else fp
    single = P <= _LR_PC
    for c0 in range(0, P, _LR_PC):
        pc = min(_LR_PC, P - c0)
        # zero-padded to the kernel's 32 problem columns in one launch each (the optimiser calls this ~300
        # times per learner: allocation + slice-assign pairs were a visible share of its launch overhead)
        Vc = torch.nn.functional.pad(V[:, c0:c0 + pc].to(torch.float32), (0, _LR_PC - pc)).contiguous()
        bc = torch.nn.functional.pad(bias[c0:c0 + pc].to(torch.float32), (0, _LR_PC - pc)).contiguous()
        ys = None
        if yscale is not None:
            ys = torch.ones(_LR_PC, dtype=torch.float32, device=dev)
            ys[:pc] = yscale[c0:c0 + pc]
        md = MixedDesign.of(X, grad) if d <= _LR_DMAX else None
        if md is not None:
            # lossless mixed storage: bf16 for the bf16-exact columns, fp32 for the others; bit-identical pass
            N_.check(N_.hip().tmog_hip_lr_objective_mixed(
                N_.ptr(md.Xm), N, d, N_.ptr(md.colmap), md.cpr, md.nce, N_.ptr(yf), N_.ptr(Wf), P, c0, pc,
                N_.ptr(Vc), N_.ptr(bc), LOSS_CODES[loss], N_.ptr(ys), int(grad), N_.ptr(fp), N_.ptr(rp),
                N_.ptr(gp) if grad else None, nblk, N_.stream(dev)), "lr_objective_mixed")
        elif d <= _LR_DMAX:
            N_.check(N_.hip().tmog_hip_lr_objective(
                N_.ptr(X), N, d, N_.ptr(yf), N_.ptr(Wf), P, c0, pc, N_.ptr(Vc), N_.ptr(bc), LOSS_CODES[loss],
                N_.ptr(ys), int(grad), N_.ptr(fp), N_.ptr(rp), N_.ptr(gp) if grad else None, nblk, N_.stream(dev)),
                "lr_objective")
        else:
            M = (X @ Vc).contiguous()          # [N, 32] margins on hipBLASLt
            N_.check(N_.hip().tmog_hip_lr_epilogue_grad(
                N_.ptr(X), N, d, N_.ptr(M), N_.ptr(yf), N_.ptr(Wf), P, c0, pc, N_.ptr(bc), LOSS_CODES[loss],
                N_.ptr(ys), int(grad), N_.ptr(fp), N_.ptr(rp), N_.ptr(gp) if grad else None, nblk, N_.stream(dev)),
                "lr_epilogue_grad")
        if single:
            f, r = fp[:, :pc].sum(0), rp[:, :pc].sum(0)
            if grad:
                G = gp[:, :d, :pc].sum(0, dtype=torch.float64)
            break
        f[c0:c0 + pc] = fp[:, :pc].sum(0)
        r[c0:c0 + pc] = rp[:, :pc].sum(0)
        if grad:
            G[:, c0:c0 + pc] = gp[:, :d, :pc].sum(0, dtype=torch.float64)
    return f, r, G


class MixedDesign:
    """Lossless mixed-storage copy of an fp32 device design matrix for the fp32 objective pass
    (``linear_kernels.hip`` ``tmog_hip_lr_objective_mixed``): each row is the columns whose values are all exact in
    bf16 (one-hot, null indicators, small counts -- most of a transmogrified matrix; ``stats.bf16_exact_columns``)
    stored as bf16, then the other columns as fp32, in 16-byte chunks. The kernel widens the bf16 values (exactly)
    and scatters every value back to its own column of the fp32 LDS tile, so the pass -- margins, losses,
    gradients -- is bit-identical to the plain fp32 pass while HBM moves 2 instead of 4 bytes per exact value.

    ``colmap`` ``int32 [8 nce + 4 (cpr - nce)]``: original column of every value slot of a row (-1 = padding)."""

    def __init__(self, X: torch.Tensor, E: torch.Tensor, R: torch.Tensor):
        dev = X.device
        N = int(X.shape[0])
        nE, nR = int(E.numel()), int(R.numel())
        dE, dR = (nE + 7) // 8 * 8, (nR + 3) // 4 * 4
        self.nce = dE // 8
        self.cpr = self.nce + dR // 4
        rb = 16 * self.cpr
        Xm = torch.zeros(N, rb, dtype=torch.uint8, device=dev)
        if nE:
            Xm[:, :2 * dE].view(torch.bfloat16)[:, :nE] = X.index_select(1, E).to(torch.bfloat16)
        if nR:
            Xm[:, 2 * dE:].view(torch.float32)[:, :nR] = X.index_select(1, R)
        self.Xm = Xm
        pad = lambda t, n: torch.cat([t.to(torch.int32), torch.full((n - int(t.numel()),), -1, dtype=torch.int32,
                                                                      device=dev)])
        self.colmap = torch.cat([pad(E, dE), pad(R, dR)]).contiguous()
        self.nE, self.nR = nE, nR

    @staticmethod
    def of(X: torch.Tensor, grad: bool = False) -> Optional["MixedDesign"]:
        """The mixed copy of ``X`` (made once per tensor, shared by every pass), or None when it does not pay or
        fit: fp32 ``linear_dtype`` only, opt-in with ``TMOG_LR_MIXED=1`` (value passes) / ``2`` (gradient passes
        too). Off by default: on the headline it measured slower than the plain fp32 passes -- LR lane 0.634 s vs
        0.515 s, identical AuPR (profiles/r6b_bench_mixed1.log / r6b_bench_mixed0.log): the landing of the bf16
        half in LDS costs more than the bytes it saves."""
        from .. import config as _cfg
        mode = os.environ.get("TMOG_LR_MIXED", "0")
        if mode == "0" or (grad and mode != "2") or _cfg.linear_dtype() != "fp32":
            return None
        if not (isinstance(X, torch.Tensor) and X.is_cuda and X.dtype == torch.float32 and X.dim() == 2
                and X.is_contiguous() and 1 <= X.shape[1] <= _LR_DMAX and X.shape[0] >= 32):
            return None
        D = getattr(X, "_tmog_mixed", None)
        if D is not None and D[0] == X._version:
            return D[1]
        from . import stats as ST
        exact = ST.bf16_exact_columns(X)
        E = torch.nonzero(exact).reshape(-1)
        R = torch.nonzero(~exact).reshape(-1)
        d = int(X.shape[1])
        dm = 128 if d <= 128 else 256 if d <= 256 else 384
        cpr = (int(E.numel()) + 7) // 8 + (int(R.numel()) + 3) // 4
        md = MixedDesign(X, E, R) if (int(E.numel()) >= 16 and 16 * cpr < 4 * d and 4 * cpr <= dm) else None
        X._tmog_mixed = (X._version, md)
        return md


_BF16_DMAX = 384        # linear_bf16_kernels.hip: 12 feature blocks of 32 resident in the accumulators
_SPLIT_K = 16           # row chunks of the X^T R library GEMM (a [d, 2C] output alone is a few dozen tiles)


class Bf16Design:
    """A dense fp32 device design matrix stored once in bf16 for ``fused_objective_bf16``: ``Xb [Npad, dpad]``
    row-major, rows padded to a multiple of 32 and columns to a multiple of 32 with zeros (the kernel's 32-row
    tiles and 32-feature blocks read no ragged edges). One copy serves the value and the gradient products.

    Columns whose values are all exact in bf16 (one-hot, null indicators, small counts: most of a transmogrified
    matrix) are stored as they are. Every other column j is stored centred and scaled, ``(x - mu_j) / s_j`` with
    ``s_j`` the power of two nearest its standard deviation, so its rounding error is relative to its spread, not to
    its magnitude (a column of values near 19000 with a spread of 10 keeps its information; plain bf16 would round
    it in steps of 128). The objective folds the shift and scale back exactly: ``X v = Xs (s v) + mu . v`` and
    ``X^T r = s (Xs^T r) + mu sum(r)``."""

    def __init__(self, X: torch.Tensor, pad: bool = True):
        from . import stats as ST
        N, d = X.shape
        self.N, self.d = int(N), int(d)
        # pad=True: the binary kernel's 32-row tiles and 32-feature blocks; pad=False (multinomial): the fused
        # kernel's 64-feature chunks and a row count that also splits into _SPLIT_K equal GEMM chunks
        self.dpad = ((d + 31) // 32) * 32 if pad else ((d + 63) // 64) * 64
        npad = ((N + 31) // 32) * 32 if pad else ((N + 32 * _SPLIT_K - 1) // (32 * _SPLIT_K)) * 32 * _SPLIT_K
        dev = X.device
        # one pass for the exactness flags, one (the fp64 stable column moments) for the centres and scales, one
        # packing pass (stats_kernels.hip bf16_pack_kernel)
        exact = ST.bf16_exact_columns(X)
        n_, mean, m2 = ST._col_partials(X)[:3]          # this process's rows (no collective inside a learner)
        mean = mean.to(torch.float64)
        std = torch.sqrt((m2.to(torch.float64) / max(int(n_), 1)).clamp_min(0))
        e = torch.round(torch.log2(torch.where(std > 0, std, torch.ones_like(std))))
        self.mu = torch.where(exact, torch.zeros_like(mean), mean.to(torch.float32).to(torch.float64))
        self.scale = torch.where(exact, torch.ones_like(std), torch.pow(2.0, e))                 # fp64, exact
        self.shifted = not bool(exact.all())
        self.n_exact = int(exact.sum())
        src = torch.arange(d, device=dev)
        mode = torch.where(exact, torch.full_like(src, ST.PACK_RAW), torch.full_like(src, ST.PACK_HI))
        self.Xb = ST.bf16_pack(X, src, mode, self.mu.to(torch.float32), (1.0 / self.scale).to(torch.float32),
                               self.dpad, rows=npad)
        self.device = dev
        self.shape = X.shape

    @staticmethod
    def supported(X) -> bool:
        return (isinstance(X, torch.Tensor) and X.is_cuda and X.dtype == torch.float32 and X.dim() == 2
                and 1 <= X.shape[1] <= _BF16_DMAX and X.shape[0] >= 1)

    @staticmethod
    def of(X: torch.Tensor, pad: bool = True) -> "Bf16Design":
        """The bf16 copy of ``X``, made once per tensor (every grid point and fold of a learner shares the design
        matrix, and the learners of one selector share it too); dropped with ``X``. ``pad=False``: the unpadded
        ``[N, d]`` copy of the library-GEMM paths (``mnl_objective_bf16``)."""
        attr = "_tmog_bf16" if pad else "_tmog_bf16_plain"
        D = getattr(X, attr, None)
        if D is None or D[0] != X._version:
            D = (X._version, Bf16Design(X, pad=pad))
            setattr(X, attr, D)
        return D[1]

    def fold_in(self, V: torch.Tensor, bias: torch.Tensor):
        """Coefficients and bias on the stored (centred / scaled) columns: ``(s v, b + mu . v)`` (fp64)."""
        if not self.shifted:
            return V, bias
        V64 = V.to(torch.float64)
        return V64 * self.scale[:, None], bias.to(torch.float64) + self.mu @ V64

    def fold_out(self, G: torch.Tensor, rsum: torch.Tensor) -> torch.Tensor:
        """``X^T r`` from the stored columns' ``Xs^T r`` and ``sum(r)`` per output column."""
        if not self.shifted:
            return G
        return G * self.scale[:, None] + self.mu[:, None] * rsum[None, :]


def _bf16_blocks(dpad: int, grad: bool, N: int) -> int:
    from . import _native as N_
    props = torch.cuda.get_device_properties(torch.cuda.current_device())
    per_cu = int(N_.hip().tmog_hip_lr_bf16_blocks_per_cu(dpad, int(grad)))
    return max(1, min((N + 127) // 128, props.multi_processor_count * per_cu))


def weight_map(wcols, P: int, device) -> torch.Tensor:
    """Device ``int32 [ceil(P / 32) * 32]`` map problem -> weight column for ``fused_objective_bf16`` (padding
    entries repeat a valid column; their problems weigh nothing)."""
    wc = list(range(P)) if wcols is None else [int(c) for c in wcols]
    n = ((P + _LR_PC - 1) // _LR_PC) * _LR_PC
    wc = wc + [wc[-1]] * (n - P)
    return torch.tensor(wc, dtype=torch.int32).to(device)


def fused_objective_bf16(D: Bf16Design, y: torch.Tensor, W: torch.Tensor, V: torch.Tensor, bias: torch.Tensor,
                         loss: str, yscale=None, grad: bool = True, wmap: Optional[torch.Tensor] = None):
    """``fused_objective`` on the bf16 design copy (``ops/csrc/hip/linear_bf16_kernels.hip``): the same outputs
    ``(f [P], r [P], G [d, P] or None)`` in fp64, of the objective whose design matrix is ``X`` rounded to bf16;
    V and the residual weights enter the bf16 matrix cores as high + low bf16 parts. ``P`` is ``V``'s width;
    problem p's row weights are column ``wmap[p]`` of ``W`` (``weight_map``; default column p), so problems that
    share their training rows (the grid points of one fold) share one weight column."""
    from . import _native as N_
    N, d, dpad = D.N, D.d, D.dpad
    P = V.shape[1]
    dev = D.device
    yf = y.to(device=dev, dtype=torch.float32).contiguous()
    Wf = W.to(torch.float32).contiguous()
    if wmap is None:
        wmap = weight_map(None, P, dev)
    V, bias = D.fold_in(V, bias)        # centred / scaled columns: s v for the stored columns, mu . v in the bias
    nblk = _bf16_blocks(dpad, grad, N)
    f = torch.empty(P, dtype=torch.float64, device=dev)
    r = torch.empty(P, dtype=torch.float64, device=dev)
    G = torch.empty(d, P, dtype=torch.float64, device=dev) if grad else None
    fp = torch.empty(nblk * 4, _LR_PC, dtype=torch.float64, device=dev)
    rp = torch.empty_like(fp)
    gp = torch.empty(nblk, dpad, _LR_PC, dtype=torch.float32, device=dev) if grad else None
    single = P <= _LR_PC
    for c0 in range(0, P, _LR_PC):
        pc = min(_LR_PC, P - c0)
        Vc = torch.nn.functional.pad(V[:, c0:c0 + pc].to(torch.float32), (0, _LR_PC - pc, 0, dpad - d)).contiguous()
        bc = torch.nn.functional.pad(bias[c0:c0 + pc].to(torch.float32), (0, _LR_PC - pc)).contiguous()
        ys = None
        if yscale is not None:
            ys = torch.ones(_LR_PC, dtype=torch.float32, device=dev)
            ys[:pc] = yscale[c0:c0 + pc]
        N_.check(N_.hip().tmog_hip_lr_bf16(
            N_.ptr(D.Xb), dpad, N, dpad, N_.ptr(yf), N_.ptr(Wf), Wf.shape[1], N_.ptr(wmap[c0:c0 + _LR_PC]), pc,
            N_.ptr(Vc), N_.ptr(bc), LOSS_CODES[loss],
            N_.ptr(ys), int(grad), N_.ptr(fp), N_.ptr(rp), N_.ptr(gp) if grad else None, nblk, N_.stream(dev)),
            "lr_bf16")
        if single:
            f, r = fp[:, :pc].sum(0), rp[:, :pc].sum(0)
            if grad:
                G = gp[:, :d, :pc].sum(0, dtype=torch.float64)
            break
        f[c0:c0 + pc] = fp[:, :pc].sum(0)
        r[c0:c0 + pc] = rp[:, :pc].sum(0)
        if grad:
            G[:, c0:c0 + pc] = gp[:, :d, :pc].sum(0, dtype=torch.float64)
    if grad:
        G = D.fold_out(G, r)
    return f, r, G


def split_bf16(A: torch.Tensor) -> torch.Tensor:
    """``[A_hi | A_lo]`` side by side in bf16: ``A_hi = bf16(A)``, ``A_lo = bf16(A - A_hi)`` (~16 mantissa bits)."""
    A = A.to(torch.float32)
    hi = A.to(torch.bfloat16)
    lo = (A - hi.to(torch.float32)).to(torch.bfloat16)
    return torch.cat([hi, lo], 1).contiguous()


def mnl_objective_bf16(D: Bf16Design, V: torch.Tensor, y: torch.Tensor, W: torch.Tensor, bias: torch.Tensor,
                       P: int, K: int, grad: bool, wmap: Optional[torch.Tensor] = None):
    """Multinomial objective of P problems x K classes on the unpadded bf16 design copy ``D`` (``Bf16Design.of(X,
    pad=False)``): margins by one library GEMM ``Xs [V_hi | V_lo]`` (fp32 out), then ``ops/csrc/hip/mnl_kernels.hip``
    (softmax, weighted loss, per-block fp64 sums, ``[R_hi | R_lo]``), then the gradient GEMM ``Xs^T [R_hi | R_lo]``.
    ``V [d, C]`` and ``bias [C]`` problem-major (column ``p * K + k``). Returns ``(f [P], rsum [C], G [d, C] or
    None)`` in fp64."""
    from . import _native as N_
    Xb = D.Xb
    N, d = D.N, D.d
    npad, dpad = Xb.shape
    C = P * K
    dev = Xb.device
    V, bias = D.fold_in(V, bias)
    if 2 <= K <= _MNL_KMAX and dpad % 64 == 0 and npad % 32 == 0 and os.environ.get("TMOG_MNL_FUSED_BF16", "1") != "0":
        return _mnl_fused_bf16(D, V, y, W, bias, P, K, grad, wmap)
    if dpad > d:
        V = torch.nn.functional.pad(V, (0, 0, 0, dpad - d))
    M2 = torch.mm(Xb, split_bf16(V), out_dtype=torch.float32)                  # [npad, 2C]
    nblk = max(1, min(4096, (N + 255) // 256))
    fp = torch.empty(nblk, P, dtype=torch.float64, device=dev)
    rp = torch.empty(nblk, C, dtype=torch.float64, device=dev)
    R2 = None
    if grad:
        R2 = torch.empty(npad, 2 * C, dtype=torch.bfloat16, device=dev)
        if npad > N:
            R2[N:].zero_()
    yf = y.to(device=dev, dtype=torch.float32).contiguous()
    Wf = W.to(torch.float32).contiguous()
    bf = bias.to(torch.float32).contiguous()
    N_.check(N_.hip().tmog_hip_mnl_epilogue(N_.ptr(M2), N, P, K, N_.ptr(bf), N_.ptr(yf), N_.ptr(Wf), Wf.shape[1],
                                            N_.ptr(wmap), int(grad), N_.ptr(R2), N_.ptr(fp), N_.ptr(rp),
                                            nblk, N_.stream(dev)), "mnl_epilogue")
    del M2
    f, rs = fp.sum(0), rp.sum(0)
    G = None
    if grad:
        # split-K by hand: _SPLIT_K row chunks as one batched GEMM, chunk results summed in fp64
        S = _SPLIT_K if npad % _SPLIT_K == 0 else 1
        Xs = Xb.view(S, npad // S, dpad).transpose(1, 2)
        G2 = torch.bmm(Xs, R2.view(S, npad // S, 2 * C), out_dtype=torch.float32).sum(0, dtype=torch.float64)
        G = D.fold_out(G2[:d, :C] + G2[:d, C:], rs)
    return f, rs, G


_MNL_KMAX = 6           # mnl_kernels.hip mnl_bf16_kernel: K accumulators of 32 x 32 in two waves' VGPRs per SIMD


def _mnl_fused_bf16(D: "Bf16Design", V: torch.Tensor, y: torch.Tensor, W: torch.Tensor, bias: torch.Tensor, P: int,
                    K: int, grad: bool, wmap: Optional[torch.Tensor]):
    """``mnl_objective_bf16`` through the fused kernel (``mnl_kernels.hip`` mnl_bf16_kernel, 32 problems a launch,
    class-major columns): margins, softmax, loss and R without a margin matrix in memory; with ``grad`` the
    launch writes ``[R_hi | R_lo]`` and ``X^T R`` is one split-K library GEMM. ``V``, ``bias`` already folded."""
    from . import _native as N_
    Xb = D.Xb
    N, d = D.N, D.d
    npad, dpad = Xb.shape
    dev = Xb.device
    props = torch.cuda.get_device_properties(dev)
    nblk = max(1, min((npad // 32 + 7) // 8, props.multi_processor_count))
    V3 = V.to(torch.float32).reshape(d, P, K)
    b2 = bias.to(torch.float32).reshape(P, K)
    wm = torch.arange(P, dtype=torch.int32, device=dev) if wmap is None else wmap.to(dev, torch.int32)
    Wf = W.to(torch.float32).contiguous()
    yf = y.to(device=dev, dtype=torch.float32).contiguous()
    f = torch.empty(P, dtype=torch.float64, device=dev)
    rs = torch.empty(P * K, dtype=torch.float64, device=dev)
    G = torch.empty(d, P * K, dtype=torch.float64, device=dev) if grad else None
    NC = K * 32
    fp = torch.empty(nblk * 8, 32, dtype=torch.float64, device=dev)
    rp = torch.empty(nblk * 8, NC, dtype=torch.float64, device=dev)
    R2 = None
    if grad:
        R2 = torch.empty(npad, 2 * NC, dtype=torch.bfloat16, device=dev)
        if npad > N:
            R2[N:].zero_()
    for p0 in range(0, P, 32):
        pc = min(32, P - p0)
        # class-major V^T [K * 32, dpad] (column k * 32 + p), zero for padding problems / features
        Vt = torch.zeros(K, 32, dpad, dtype=torch.float32, device=dev)
        Vt[:, :pc, :d] = V3[:, p0:p0 + pc, :].permute(2, 1, 0)
        Vt = Vt.reshape(NC, dpad)
        hi = Vt.to(torch.bfloat16)
        Vhl = torch.cat([hi, (Vt - hi.to(torch.float32)).to(torch.bfloat16)], 0).contiguous()
        bt = torch.zeros(K, 32, dtype=torch.float32, device=dev)
        bt[:, :pc] = b2[p0:p0 + pc].t()
        wc = torch.zeros(32, dtype=torch.int32, device=dev)
        wc[:pc] = wm[p0:p0 + pc]
        wc[pc:] = wm[p0]
        N_.check(N_.hip().tmog_hip_mnl_bf16(N_.ptr(Xb), dpad, N, dpad, N_.ptr(yf), N_.ptr(Wf), Wf.shape[1], N_.ptr(wc),
                                            pc, K, N_.ptr(Vhl), N_.ptr(bt.reshape(-1)), int(grad), N_.ptr(R2),
                                            N_.ptr(fp), N_.ptr(rp), nblk, N_.stream(dev)), "mnl_bf16")
        f[p0:p0 + pc] = fp.sum(0)[:pc]
        rk = rp.sum(0).reshape(K, 32)[:, :pc]                              # [K, pc] -> problem-major
        rs[p0 * K:(p0 + pc) * K] = rk.t().reshape(-1)
        if grad:
            S = _SPLIT_K if npad % _SPLIT_K == 0 else 1
            Xs = Xb.view(S, npad // S, dpad).transpose(1, 2)
            G2 = torch.bmm(Xs, R2.view(S, npad // S, 2 * NC), out_dtype=torch.float32).sum(0, dtype=torch.float64)
            Gk = (G2[:d, :NC] + G2[:d, NC:]).reshape(d, K, 32)[:, :, :pc]      # [d, K, pc]
            G[:, p0 * K:(p0 + pc) * K] = Gk.permute(0, 2, 1).reshape(d, pc * K)
    if grad:
        G = D.fold_out(G, rs)
    return f, rs, G


def _torch_objective(X, y, W, V, bias, loss, yscale, grad):
    """Reference / tail path of ``fused_objective`` (same outputs, fp64 sums)."""
    M = X @ V.to(X.dtype) + bias.to(X.dtype)[None, :]
    yy = y.to(M.dtype)[:, None]
    if loss == "logistic":
        l = torch.nn.functional.softplus(M) - yy * M
        g = torch.sigmoid(M) - yy
    elif loss == "hinge":
        ys = 2 * yy - 1
        l = torch.clamp(1 - ys * M, min=0)
        g = torch.where(ys * M < 1, -ys, torch.zeros_like(M))
    else:
        r = M - yy / yscale.to(M.dtype)[None, :]
        l = 0.5 * r * r
        g = r
    Wm = W.to(M.dtype)
    R = g * Wm
    G = (X.t() @ R).to(torch.float64) if grad else None
    return (l * Wm).sum(0).to(torch.float64), R.sum(0).to(torch.float64), G


_OW_DMAX, _OW_MMAX = 256 * 48, 32


def owlqn_direction_supported(U: torch.Tensor, m: int) -> bool:
    return U.is_cuda and U.dtype == torch.float64 and U.dim() == 2 and U.shape[0] <= _OW_DMAX and m <= _OW_MMAX


def owlqn_direction(U, g, l1, S, Y, RHO, hist_n: int, m: int):
    """OWL-QN pseudo-gradient + two-loop L-BFGS direction + orthant projection for every column of ``U`` in
    one HIP launch (``linear_kernels.hip`` owlqn_direction_kernel); same arithmetic as the torch loop of
    ``models/linear.py`` owlqn_batched. Returns ``(D, pg, xi, dnorm)``."""
    from . import _native as N_
    U, g, l1 = U.contiguous(), g.contiguous(), l1.contiguous()
    d1, P = U.shape
    D, pg, xi = torch.empty_like(U), torch.empty_like(U), torch.empty_like(U)
    dnorm = torch.empty(P, dtype=torch.float64, device=U.device)
    N_.check(N_.hip().tmog_hip_owlqn_direction(
        N_.ptr(U), N_.ptr(g), N_.ptr(l1), N_.ptr(S), N_.ptr(Y), N_.ptr(RHO), int(d1), int(P), int(m), int(hist_n),
        N_.ptr(D), N_.ptr(pg), N_.ptr(xi), N_.ptr(dnorm), N_.stream(U.device)), "owlqn_direction")
    return D, pg, xi, dnorm


def owlqn_candidate(U, D, xi, l1, pg, alpha):
    """OWL-QN line-search candidate ``cand = project_xi(U + alpha D)`` with ``sum l1 |cand|`` and
    ``sum pg (cand - U)`` per column, one HIP launch (``owlqn_candidate_kernel``). All fp64, contiguous."""
    from . import _native as N_
    d1, P = U.shape
    cand = torch.empty_like(U)
    l1t = torch.empty(P, dtype=torch.float64, device=U.device)
    dd = torch.empty_like(l1t)
    a = alpha.to(torch.float64).contiguous()
    N_.check(N_.hip().tmog_hip_owlqn_candidate(
        N_.ptr(U), N_.ptr(D), N_.ptr(xi), N_.ptr(l1), N_.ptr(pg), N_.ptr(a), int(d1), int(P), N_.ptr(cand),
        N_.ptr(l1t), N_.ptr(dd), N_.stream(U.device)), "owlqn_candidate")
    return cand, l1t, dd


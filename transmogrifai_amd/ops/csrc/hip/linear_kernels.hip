// Fused linear-model objective for CDNA4 (gfx950): one pass over X per (value, gradient) evaluation.
//
// Replaces the per-iteration work of Spark's LogisticRegression / LinearRegression / LinearSVC
// aggregators (OpLogisticRegression.scala:54-177, OpLinearRegression.scala, OpLinearSVC.scala; Spark
// LogisticAggregator / HingeAggregator / LeastSquaresAggregator: margins, loss and gradient summed
// over rows) for P problems at once -- the (config, fold) grid of the model selector, SURVEY.md K22.
//
// Per 64-row tile of X (row-major [N][d] fp32, copied verbatim into LDS with 16-byte loads that are
// issued one tile ahead, so HBM latency overlaps the MFMA work of the current tile), 8 waves:
//   phase A  M[64, 32] = X_tile . V     v_mfma_f32_16x16x4_f32; wave w owns the 16x16 output block
//            (rows 16(w&3).., problems 16(w>>2)..) over all of d; V is staged once in LDS
//   epilogue in registers: l, dl/dm per (row, problem), R = W * dl/dm, weighted loss sums
//   phase B  G[d, 32] += X_tile^T . R   v_mfma_f32_16x16x4_f32; 16x16 output blocks round-robin
//            over the waves, accumulators resident for the whole kernel
// so X is read from HBM exactly once per evaluation (the torch path reads it twice and round-trips M
// and R through HBM). Workgroups are persistent; their G / loss partials are summed in fp64 on the
// host side (ops/linear.py). Phase-A column order inside each 64-column block is k = s + 16q (lane
// group q) so the four lane groups of an operand read land 16 banks apart; V rows are padded to 33.
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <stdint.h>
#include <math.h>

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int TM = 64;         // rows per tile
constexpr int NT = 512;        // threads per workgroup (8 waves)
constexpr int PC = 32;         // problem columns per launch
constexpr int VS = 33;         // LDS row stride of V
constexpr int DMAX = 384;      // LDS: 64*384*4 (X) + 384*33*4 (V) + 64*32*4 (R) = 155 KB

__device__ __forceinline__ void loss_and_grad(int loss, float m, float y, float ysc, float* l, float* g) {
  if (loss == 0) {              // logistic
    // log1p(e) for e in (0, 1] as log(u) * e / (u - 1) with u = 1 + e (exact-argument trick, a few ulp)
    // and sigmoid through one reciprocal: ~15 VALU instead of the ~60 of log1pf + two IEEE divisions
    const float am = fabsf(m);
    const float e = __expf(-am);
    const float u = 1.f + e;
    const float lp = (u == 1.f) ? e : __logf(u) * __fdividef(e, u - 1.f);
    *l = fmaxf(m, 0.f) + lp - y * m;
    const float inv = __builtin_amdgcn_rcpf(u);
    const float sig = m >= 0.f ? inv : e * inv;
    *g = sig - y;
  } else if (loss == 1) {       // hinge
    const float ys = 2.f * y - 1.f;
    const float marg = ys * m;
    *l = fmaxf(1.f - marg, 0.f);
    *g = marg < 1.f ? -ys : 0.f;
  } else {                      // squared, label pre-scaled per problem
    const float r = m - y / ysc;
    *l = 0.5f * r * r;
    *g = r;
  }
}

__device__ __forceinline__ int kcol(int s, int q) { return 64 * (s >> 4) + (s & 15) + 16 * q; }

// GB = phase-B output blocks per wave, NPF = prefetch float4 slots per thread, TT = rows per tile (64: one
// 512-thread workgroup per CU; 32: 256-thread workgroups, two per CU -- two tiles' loads in flight per CU).
// Waves: TT / 16 row blocks x 2 problem halves; phase-B output blocks ob = wave + NW i.
// MIX (lossless mixed storage, ops/linear.py MixedDesign): a row of X is cpr 16-byte chunks -- nce chunks of 8 bf16
// values (the columns whose values are all exact in bf16: one-hot, null indicators, small counts) then chunks of 4
// fp32 values (every other column). colmap[slot] is the original column of each value slot of a row (-1: padding).
// The landing step widens the bf16 values (exactly) and scatters every value to its original column of the fp32
// LDS tile, so the tile -- and everything computed from it -- is bit-identical to the plain fp32 pass, while HBM
// delivers 2 bytes instead of 4 for the exact columns.
template <bool GRAD, int GB, int NPF, int DM, int TT, bool MIX>
__global__ void __launch_bounds__(8 * TT) lr_objective_kernel(
    const float* __restrict__ X, int64_t N, int d, const float* __restrict__ y,
    const float* __restrict__ W, int ldw, int wcol0, int P, const float* __restrict__ V,
    const float* __restrict__ bias, int loss, const float* __restrict__ yscale, double* __restrict__ f_part,
    double* __restrict__ r_part, float* __restrict__ G_part, int dpad, const int32_t* __restrict__ colmap, int cpr,
    int nce) {
  constexpr int RB = TT / 16;               // row blocks (waves per problem half)
  constexpr int NW = 2 * RB;                // waves per workgroup
  constexpr int NTT = 64 * NW;              // threads per workgroup
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int ks_full = (d >> 6) * 16;        // phase-A k-steps over full 64-column blocks
  const int ks_tail = ((d & 63) + 3) >> 2;  // k-steps over the ragged last block
  const int xs_words = (TT * d + 64 + 3) & ~3;
  float* Xs = lds;                          // [TT][d] + 64 words of overrun (finite, times V = 0)
  float* Vs = Xs + xs_words;                // [64][VS]: V rows of the ragged last 64-column block, zero beyond d
  float* Rs = Vs + 64 * VS;                 // [TT][PC]
  int* cm = reinterpret_cast<int*>(Rs + TT * PC);   // MIX: the row's slot -> column map
  const int n_slots = MIX ? 8 * nce + 4 * (cpr - nce) : 0;
  const int tile_chunks = MIX ? TT * cpr : 0;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: SGPR, scalar branches
  const int q = lane >> 4, c = lane & 15;
  const int rb = wave % RB, pb = wave / RB;
  const int nob = 2 * ((d + 15) >> 4);
  const int nb64 = d >> 6;

  for (int i = threadIdx.x; i < xs_words; i += NTT) Xs[i] = 0.f;
  if (MIX)
    for (int i = threadIdx.x; i < n_slots; i += NTT) cm[i] = colmap[i];
  for (int i = threadIdx.x; i < 64 * VS; i += NTT) {
    const int k = 64 * nb64 + i / VS, j = i % VS;
    Vs[i] = (k < d && j < PC) ? V[(int64_t)k * PC + j] : 0.f;
  }
  f32x4 gacc[GB];
#pragma unroll
  for (int i = 0; i < GB; ++i) gacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int p = 16 * pb + c;                // this lane's problem column in phase A / epilogue
  // phase-A B operands of the full 64-column blocks live in registers for the whole kernel: lane (q, c)
  // of problem block pb only ever multiplies V[64 b + 16 q + s][16 pb + c] (s = 0..15), so per MFMA one
  // LDS read (the X element) remains instead of two
  constexpr int NB64 = DM / 64;
  float vr[NB64 * 16];
#pragma unroll
  for (int b = 0; b < NB64; ++b)
#pragma unroll
    for (int s2 = 0; s2 < 16; ++s2)
      vr[16 * b + s2] = b < nb64 ? V[(int64_t)(64 * b + 16 * q + s2) * PC + p] : 0.f;
  const float bp = bias[p];
  const float ysp = yscale ? yscale[p] : 1.f;
  double f_acc = 0.0, r_acc = 0.0;

  const int64_t ntiles = (N + TT - 1) / TT;
  const int tile_f4 = (TT * d) >> 2;
  // branch-free prefetch (a guarded load makes hipcc wait vmcnt(0) per slot): out-of-range slots
  // re-read the tile's last float4 and are zeroed at the LDS store. Host guarantees N * d % 4 == 0.
  // The epilogue's W / y values of the next tile ride along (rows clamped to N - 1, masked later).
  f32x4 pf[NPF];
  float pw[4], py[4];
  f32x4 pt = {0.f, 0.f, 0.f, 0.f};          // the last tile's 1-3 trailing floats past 4 * nval4 ((N d) % 4 != 0)
  int nval4 = 0, ntail = 0;
  auto prefetch = [&](int64_t tile) {
    const int64_t r0 = tile * TT;
    if constexpr (MIX) {
      nval4 = (int)(min((int64_t)TT, N - r0) * cpr);      // rows are whole 16-byte chunks: no ragged tail
      ntail = 0;
      const f32x4* src = reinterpret_cast<const f32x4*>(reinterpret_cast<const uint8_t*>(X) + r0 * (int64_t)cpr * 16);
#pragma unroll
      for (int i = 0; i < NPF; ++i) pf[i] = src[min((int)threadIdx.x + NTT * i, max(nval4 - 1, 0))];
    } else {
    const int nval = (int)(min((int64_t)TT, N - r0) * d);
    nval4 = nval >> 2;
    ntail = nval & 3;
    const f32x4* src = reinterpret_cast<const f32x4*>(X + r0 * (int64_t)d);
#pragma unroll
    for (int i = 0; i < NPF; ++i) pf[i] = src[min((int)threadIdx.x + NTT * i, max(nval4 - 1, 0))];
    const float* xt = X + r0 * (int64_t)d;   // every lane reads the same <= 3 words (clamped into the tile)
#pragma unroll
    for (int k = 0; k < 3; ++k) pt[k] = k < ntail ? xt[min(4 * nval4 + k, nval - 1)] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t gr = min(r0 + 16 * rb + 4 * q + j, N - 1);
      pw[j] = W[gr * ldw + wcol0 + min(p, P - 1)];
      py[j] = y[gr];
    }
  };
  if ((int64_t)blockIdx.x < ntiles) prefetch(blockIdx.x);
  __syncthreads();

  const float* va = Vs + 16 * pb + c;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t r0 = tile * TT;
    const int nrows = (int)min((int64_t)TT, N - r0);
    // ---- land the prefetched tile in LDS, then start fetching the next one
    if constexpr (MIX) {
#pragma unroll
      for (int i = 0; i < NPF; ++i) {
        const int e4 = threadIdx.x + NTT * i;
        if (e4 < tile_chunks) {
          const int row = e4 / cpr, off = e4 - row * cpr;
          const bool live = e4 < nval4;           // rows past N: zeros (finite, and their R is 0)
          float* xr = Xs + row * d;
          if (off < nce) {                        // 8 bf16: widened exactly (bf16 = the high half of an fp32)
            const uint32_t* u = reinterpret_cast<const uint32_t*>(&pf[i]);
            const int* m = cm + 8 * off;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const uint32_t w = u[k >> 1];
              const uint32_t bits = (k & 1) ? (w & 0xFFFF0000u) : (w << 16);
              const int col = m[k];
              if (col >= 0) xr[col] = live ? __uint_as_float(bits) : 0.f;
            }
          } else {                                // 4 fp32
            const int* m = cm + 8 * nce + 4 * (off - nce);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const int col = m[k];
              if (col >= 0) xr[col] = live ? pf[i][k] : 0.f;
            }
          }
        }
      }
    } else {
    f32x4* xs4 = reinterpret_cast<f32x4*>(Xs);
#pragma unroll
    for (int i = 0; i < NPF; ++i) {
      const int e4 = threadIdx.x + NTT * i;
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      if (e4 < tile_f4) xs4[e4] = e4 < nval4 ? pf[i] : (e4 == nval4 && ntail ? pt : z);
    }
    }
    float cw[4], cy[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) { cw[j] = pw[j]; cy[j] = py[j]; }
    __syncthreads();
    if (tile + gridDim.x < ntiles) prefetch(tile + gridDim.x);

    // ---- phase A: this wave's 16x16 margin block over all of d (two accumulators hide the
    // 40-cycle dependent-MFMA latency)
    // Full 64-column blocks use the bank-spread order; the ragged tail block steps 4 columns at a time.
    // Per 64-column block the 16 k-steps read at compile-time offsets from two per-block bases (column
    // 64 b + 16 q + s, s = 0..15): no per-step address arithmetic (it was ~7 VALU per MFMA, and the
    // kernel was VALU-issue bound).
    f32x4 macc = {0.f, 0.f, 0.f, 0.f}, macc2 = {0.f, 0.f, 0.f, 0.f};
    const float* xa = Xs + (16 * rb + c) * d;
#pragma unroll
    for (int b = 0; b < NB64; ++b) {
      if (b < nb64) {
        const float* xb = xa + 16 * q + 64 * b;
#pragma unroll
        for (int s2 = 0; s2 < 16; s2 += 2) {
          macc = __builtin_amdgcn_mfma_f32_16x16x4f32(xb[s2], vr[16 * b + s2], macc, 0, 0, 0);
          macc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(xb[s2 + 1], vr[16 * b + s2 + 1], macc2, 0, 0, 0);
        }
      }
    }
    for (int k = 4 * ks_full + q; k < 4 * ks_full + 4 * ks_tail; k += 8) {
      macc = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[k], va[(k - 64 * nb64) * VS], macc, 0, 0, 0);
      if (k + 4 < 4 * ks_full + 4 * ks_tail)
        macc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[k + 4], va[(k + 4 - 64 * nb64) * VS], macc2, 0, 0, 0);
    }
    macc += macc2;

    // ---- fused epilogue in registers: rows 16rb + 4q + j, problem p
    float fl = 0.f, rl = 0.f;       // this lane's 4 rows in fp32, folded into the fp64 totals once per tile
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = 16 * rb + 4 * q + j;
      float rv = 0.f;
      if (row < nrows && p < P) {
        const float w = cw[j];
        float l, g;
        loss_and_grad(loss, macc[j] + bp, cy[j], ysp, &l, &g);
        fl += l * w;
        rv = g * w;
        rl += rv;
      }
      if (GRAD) Rs[row * PC + p] = rv;
    }
    f_acc += (double)fl;
    r_acc += (double)rl;
    if (GRAD) {
      __syncthreads();
      // ---- phase B: G[16db.., 16pb'..] += X_tile^T R  (TT / 4 k-steps of 4 rows)
      // output blocks ob = wave + NW i: column block (wave >> 1) + (NW / 2) i, problem half wave & 1
      const float* xw = Xs + q * d + c + 16 * (wave >> 1);
      const float* rw = Rs + q * PC + 16 * (wave & 1) + c;
#pragma unroll 4
      for (int t = 0; t < TT / 4; ++t) {
        const float rv = rw[4 * t * PC];
        const float* xr = xw + 4 * t * d;
#pragma unroll
        for (int i = 0; i < GB; ++i) {
          if (wave + NW * i < nob)
            gacc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(xr[8 * NW * i], rv, gacc[i], 0, 0, 0);
        }
      }
    }
    __syncthreads();          // Xs / Rs are rewritten by the next tile
  }

  // ---- per-workgroup partials
  if (GRAD) {
    float* gp = G_part + (int64_t)blockIdx.x * dpad * PC;
#pragma unroll
    for (int i = 0; i < GB; ++i) {
      const int ob = wave + NW * i;
      if (ob < nob) {
        const int db = ob >> 1, pbb = ob & 1;
#pragma unroll
        for (int j = 0; j < 4; ++j) gp[(int64_t)(16 * db + 4 * q + j) * PC + 16 * pbb + c] = gacc[i][j];
      }
    }
  }
  // lanes sharing a problem column: 4 lane groups x RB row-block waves
  f_acc += __shfl_xor(f_acc, 16, 64);
  f_acc += __shfl_xor(f_acc, 32, 64);
  r_acc += __shfl_xor(r_acc, 16, 64);
  r_acc += __shfl_xor(r_acc, 32, 64);
  double* sf = reinterpret_cast<double*>(lds);
  __syncthreads();
  if (q == 0) {
    sf[wave * 16 + c] = f_acc;
    sf[128 + wave * 16 + c] = r_acc;
  }
  __syncthreads();
  if (threadIdx.x < PC) {
    const int pp = threadIdx.x, pbw = pp >> 4, cc = pp & 15;
    double fs = 0.0, rs = 0.0;
    for (int r = 0; r < RB; ++r) {            // waves RB pb + r
      fs += sf[(RB * pbw + r) * 16 + cc];
      rs += sf[128 + (RB * pbw + r) * 16 + cc];
    }
    f_part[(int64_t)blockIdx.x * PC + pp] = fs;
    r_part[(int64_t)blockIdx.x * PC + pp] = rs;
  }
}

// Wide-d variant (384 < d <= 2048; the LDS cannot hold a 64-row tile and V): the margins come from a
// library GEMM (M = X V on hipBLASLt) and this kernel fuses everything after it -- loss, dl/dm, the
// weighted sums and G += X_tile^T R on the matrix cores -- reading every X element exactly once, straight
// from global memory (one coalesced 64-byte row segment per lane group and MFMA operand; the GB
// output blocks of a wave keep that many loads in flight). Output partials as lr_objective_kernel.
template <bool GRAD, int GB>
__global__ void __launch_bounds__(NT) lr_epilogue_grad_kernel(
    const float* __restrict__ X, int64_t N, int d, const float* __restrict__ M, const float* __restrict__ y,
    const float* __restrict__ W, int ldw, int wcol0, int P, const float* __restrict__ bias, int loss,
    const float* __restrict__ yscale, double* __restrict__ f_part, double* __restrict__ r_part,
    float* __restrict__ G_part, int dpad) {
  __shared__ float Rs[TM * PC];
  __shared__ double sfr[2 * NT];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane >> 4, c = lane & 15;
  const int nob = 2 * ((d + 15) >> 4);
  f32x4 gacc[GB];
#pragma unroll
  for (int i = 0; i < GB; ++i) gacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  double f_acc = 0.0, r_acc = 0.0;
  // epilogue mapping: thread -> problem column pe, rows re, re + 16, re + 32, re + 48
  const int pe = threadIdx.x & (PC - 1), re = threadIdx.x >> 5;
  const float be = bias[pe];
  const float yse = yscale ? yscale[pe] : 1.f;
  const int64_t ntiles = (N + TM - 1) / TM;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t r0 = tile * TM;
    const int nrows = (int)min((int64_t)TM, N - r0);
#pragma unroll
    for (int k = 0; k < TM / 16; ++k) {
      const int row = re + 16 * k;
      float rv = 0.f;
      if (row < nrows && pe < P) {
        const int64_t gr = r0 + row;
        const float w = W[gr * ldw + wcol0 + pe];
        float l, g;
        loss_and_grad(loss, M[gr * PC + pe] + be, y[gr], yse, &l, &g);
        f_acc += (double)(l * w);
        rv = g * w;
        r_acc += (double)rv;
      }
      Rs[row * PC + pe] = rv;
    }
    if (GRAD) {
      __syncthreads();
#pragma unroll 2
      for (int t = 0; t < TM / 4; ++t) {
        const int row = 4 * t + q;
        const float rv0 = Rs[row * PC + c], rv1 = Rs[row * PC + 16 + c];
        const float* xr = X + (r0 + min(row, nrows - 1)) * (int64_t)d;   // rows past nrows have R = 0
#pragma unroll
        for (int i = 0; i < GB; ++i) {
          const int ob = wave + 8 * i;
          if (ob < nob) {
            const int col = 16 * (ob >> 1) + c;
            const float xv = col < d ? xr[col] : 0.f;
            gacc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv, (ob & 1) ? rv1 : rv0, gacc[i], 0, 0, 0);
          }
        }
      }
    }
    __syncthreads();          // Rs is rewritten by the next tile
  }
  if (GRAD) {
    float* gp = G_part + (int64_t)blockIdx.x * dpad * PC;
#pragma unroll
    for (int i = 0; i < GB; ++i) {
      const int ob = wave + 8 * i;
      if (ob < nob) {
        const int db = ob >> 1, pbb = ob & 1;
#pragma unroll
        for (int j = 0; j < 4; ++j) gp[(int64_t)(16 * db + 4 * q + j) * PC + 16 * pbb + c] = gacc[i][j];
      }
    }
  }
  sfr[threadIdx.x] = f_acc;
  sfr[NT + threadIdx.x] = r_acc;
  __syncthreads();
  if (threadIdx.x < PC) {
    double fs = 0.0, rs = 0.0;
    for (int k = 0; k < NT / PC; ++k) {        // threads sharing problem column pe (fixed order)
      fs += sfr[k * PC + threadIdx.x];
      rs += sfr[NT + k * PC + threadIdx.x];
    }
    f_part[(int64_t)blockIdx.x * PC + threadIdx.x] = fs;
    r_part[(int64_t)blockIdx.x * PC + threadIdx.x] = rs;
  }
}

// OWL-QN search direction for P problems in one launch (models/linear.py owlqn_batched): pseudo-gradient,
// L-BFGS two-loop recursion over the m-slot history ring, initial Hessian scaling, orthant projection,
// the orthant signs xi and |pg|. One 256-thread workgroup per problem column; the column's d1 entries
// stay in registers (QMAX per thread) and every inner product is an fp64 block reduction. Replaces ~150
// small torch launches per iteration (the optimiser was launch-bound: ~0.2 s of the LR learner's 0.3 s).
constexpr int OW_NT = 256;
constexpr int OW_QMAX = 48;      // d1 <= 12288 (16 per thread up to 4096)
constexpr int OW_MMAX = 32;      // history slots

__device__ __forceinline__ double ow_block_sum(double v, double* sh) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  __syncthreads();                       // previous readers of sh are done
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  return (sh[0] + sh[1]) + (sh[2] + sh[3]);
}
__device__ __forceinline__ double ow_sign(double x) { return (double)((x > 0.0) - (x < 0.0)); }

template <int QMAX>
__global__ void __launch_bounds__(OW_NT) owlqn_direction_kernel(
    const double* __restrict__ U, const double* __restrict__ g, const double* __restrict__ l1,
    const double* __restrict__ S, const double* __restrict__ Y, const double* __restrict__ RHO, int d1, int P,
    int m, int hist_n, double* __restrict__ D_out, double* __restrict__ pg_out, double* __restrict__ xi_out,
    double* __restrict__ dnorm_out) {
  __shared__ double sh[4];
  const int p = blockIdx.x, t = threadIdx.x;
  // q in registers; the pseudo-gradient goes straight to pg_out and is read back by the same thread at the end
  // (the multinomial columns, (d + 1) K entries, need the registers for q)
  double q[QMAX];
  double pn = 0.0;
#pragma unroll
  for (int r = 0; r < QMAX; ++r) {
    const int i = t + OW_NT * r;
    double pv = 0.0;
    if (i < d1) {
      const int64_t e = (int64_t)i * P + p;
      const double u = U[e], gg = g[e], l = l1[e];
      pv = u > 0.0 ? gg + l : (u < 0.0 ? gg - l : (gg + l < 0.0 ? gg + l : (gg - l > 0.0 ? gg - l : 0.0)));
      pg_out[e] = pv;
      pn += pv * pv;
    }
    q[r] = pv;
  }
  const int k = min(hist_n, m);
  double a[OW_MMAX];
  for (int j = 0; j < k; ++j) {
    const int idx = ((hist_n - 1 - j) % m + m) % m;
    const double* Sj = S + (int64_t)idx * d1 * P;
    double acc = 0.0;
#pragma unroll
    for (int r = 0; r < QMAX; ++r) {
      const int i = t + OW_NT * r;
      if (i < d1) acc += Sj[(int64_t)i * P + p] * q[r];
    }
    a[j] = RHO[(int64_t)idx * P + p] * ow_block_sum(acc, sh);
    const double* Yj = Y + (int64_t)idx * d1 * P;
#pragma unroll
    for (int r = 0; r < QMAX; ++r) {
      const int i = t + OW_NT * r;
      if (i < d1) q[r] -= a[j] * Yj[(int64_t)i * P + p];
    }
  }
  if (k > 0) {
    const int last = ((hist_n - 1) % m + m) % m;
    const double* Sl = S + (int64_t)last * d1 * P;
    const double* Yl = Y + (int64_t)last * d1 * P;
    double yy = 0.0, sy = 0.0;
#pragma unroll
    for (int r = 0; r < QMAX; ++r) {
      const int i = t + OW_NT * r;
      if (i < d1) {
        const double yv = Yl[(int64_t)i * P + p];
        yy += yv * yv;
        sy += Sl[(int64_t)i * P + p] * yv;
      }
    }
    yy = ow_block_sum(yy, sh);
    sy = ow_block_sum(sy, sh);
    const double gam = yy > 0.0 ? sy / fmax(yy, 1e-300) : 1.0;
#pragma unroll
    for (int r = 0; r < QMAX; ++r) q[r] *= gam;
  }
  for (int j = k - 1; j >= 0; --j) {
    const int idx = ((hist_n - 1 - j) % m + m) % m;
    const double* Sj = S + (int64_t)idx * d1 * P;
    const double* Yj = Y + (int64_t)idx * d1 * P;
    double acc = 0.0;
#pragma unroll
    for (int r = 0; r < QMAX; ++r) {
      const int i = t + OW_NT * r;
      if (i < d1) acc += Yj[(int64_t)i * P + p] * q[r];
    }
    const double b = RHO[(int64_t)idx * P + p] * ow_block_sum(acc, sh);
#pragma unroll
    for (int r = 0; r < QMAX; ++r) {
      const int i = t + OW_NT * r;
      if (i < d1) q[r] += Sj[(int64_t)i * P + p] * (a[j] - b);
    }
  }
#pragma unroll
  for (int r = 0; r < QMAX; ++r) {
    const int i = t + OW_NT * r;
    if (i < d1) {
      const int64_t e = (int64_t)i * P + p;
      const double u = U[e], l = l1[e], pv = pg_out[e];
      double dv = -q[r];
      if (l > 0.0 && ow_sign(dv) != ow_sign(-pv)) dv = 0.0;
      D_out[e] = dv;
      xi_out[e] = u != 0.0 ? ow_sign(u) : ow_sign(-pv);
    }
  }
  pn = ow_block_sum(pn, sh);
  if (t == 0) dnorm_out[p] = fmax(sqrt(pn), 1e-300);
}

// OWL-QN line-search candidate for every problem column: cand = U + alpha D projected onto the orthant
// xi (l1 > 0 coordinates whose sign left it are zeroed), with the two per-column sums the Armijo test
// needs, sum l1 |cand| and sum pg (cand - U) -- one launch instead of ~12 torch ops per trial step.
__global__ void __launch_bounds__(OW_NT) owlqn_candidate_kernel(
    const double* __restrict__ U, const double* __restrict__ D, const double* __restrict__ xi,
    const double* __restrict__ l1, const double* __restrict__ pg, const double* __restrict__ alpha, int d1, int P,
    double* __restrict__ cand, double* __restrict__ l1t_out, double* __restrict__ dd_out) {
  __shared__ double sh[4];
  const int p = blockIdx.x;
  const double a = alpha[p];
  double l1t = 0.0, dd = 0.0;
  for (int i = threadIdx.x; i < d1; i += OW_NT) {
    const int64_t e = (int64_t)i * P + p;
    const double u = U[e], l = l1[e];
    double c = u + a * D[e];
    if (l > 0.0 && ow_sign(c) != xi[e]) c = 0.0;
    cand[e] = c;
    l1t += l * fabs(c);
    dd += pg[e] * (c - u);
  }
  l1t = ow_block_sum(l1t, sh);
  dd = ow_block_sum(dd, sh);
  if (threadIdx.x == 0) {
    l1t_out[p] = l1t;
    dd_out[p] = dd;
  }
}

}  // namespace

extern "C" {

// Wide-d objective tail: M [N][32] fp32 = X V (from a library GEMM, without bias); same outputs as
// tmog_hip_lr_objective. d <= 2048.
int tmog_hip_lr_epilogue_grad(const float* X, int64_t N, int d, const float* M, const float* y, const float* W,
                              int ldw, int wcol0, int P, const float* bias, int loss, const float* yscale, int grad,
                              double* f_part, double* r_part, float* G_part, int nblk, hipStream_t stream) {
  if (d < 1 || d > 2048 || P > PC || P < 1 || nblk < 1) return -2;
  const int dpad = ((d + 15) / 16) * 16;
  const int nob = 2 * ((d + 15) / 16);
#define TM_LRE(G, GB)                                                                                       \
  hipLaunchKernelGGL((lr_epilogue_grad_kernel<G, GB>), dim3(nblk), dim3(NT), 0, stream, X, N, d, M, y, W, ldw, \
                     wcol0, P, bias, loss, yscale, f_part, r_part, G_part, dpad)
  if (!grad) TM_LRE(false, 1);
  else if (nob <= 8 * 8) TM_LRE(true, 8);
  else if (nob <= 8 * 16) TM_LRE(true, 16);
  else TM_LRE(true, 32);
#undef TM_LRE
  return (int)hipGetLastError();
}


// Weighted loss sums f[p] = sum_i W[i,p] l(m_ip), r[p] = sum_i W[i,p] l'(m_ip) and (grad != 0)
// G[:, p] = sum_i X[i,:] W[i,p] l'(m_ip), with m = X V + bias, for up to 32 problems (columns
// wcol0 .. wcol0+P-1 of W). V is [d][32] fp32 (zero-padded), bias / yscale are [32].
// Outputs are per-workgroup partials: f_part / r_part [nblk][32] fp64, G_part [nblk][dpad][32] fp32.
// Rows per tile of the value-only / gradient passes: TMOG_LR_TILE_V / TMOG_LR_TILE_G (32 or 64). Measured at
// 1M x 330 x 32 problems (scripts/bench_lr_obj.py): value pass 0.449 ms (64) vs 0.422 ms (32, two workgroups
// per CU); gradient pass 0.720 ms (64) vs 1.128 ms (32: twice the phase-B accumulators per wave, spills).
static int lr_tile(bool grad) {
  static const int tv = [] { const char* e = std::getenv("TMOG_LR_TILE_V"); return (e && std::atoi(e) == 64) ? 64 : 32; }();
  static const int tg = [] { const char* e = std::getenv("TMOG_LR_TILE_G"); return (e && std::atoi(e) == 32) ? 32 : 64; }();
  return grad ? tg : tv;
}

// Workgroups per CU of a tmog_hip_lr_objective pass (ops/linear.py sizes its persistent grid with it).
int tmog_hip_lr_blocks_per_cu(int grad) { return lr_tile(grad != 0) == 32 ? 2 : 1; }

static int lr_objective_launch(const float* X, int64_t N, int d, const float* y, const float* W, int ldw, int wcol0,
                               int P, const float* V, const float* bias, int loss, const float* yscale, int grad,
                               double* f_part, double* r_part, float* G_part, int nblk, hipStream_t stream,
                               const int32_t* colmap, int cpr, int nce) {
  if (d > DMAX || d < 1 || P > PC || P < 1 || nblk < 1) return -2;
  if ((reinterpret_cast<uintptr_t>(X) & 15) != 0) return -3;
  const bool mix = colmap != nullptr;
  const int dm = d <= 128 ? 128 : d <= 256 ? 256 : 384;
  // a mixed row must fit the prefetch slots sized for the fp32 row (NPF * NTT >= TT * cpr): cpr <= DM / 4
  if (mix && (cpr < 1 || nce < 0 || nce > cpr || 4 * cpr > dm)) return -4;
  const int dpad = ((d + 15) / 16) * 16;
  const int tt = lr_tile(grad != 0);
  const int n_slots = mix ? 8 * nce + 4 * (cpr - nce) : 0;
  const size_t lds = (size_t)(((tt * d + 64 + 3) & ~3) + 64 * VS + tt * PC) * sizeof(float) + sizeof(int) * n_slots;
#define TM_LR(G, DM, T_)                                                                                          \
  if (mix)                                                                                                        \
    hipLaunchKernelGGL((lr_objective_kernel<G, (DM / 8 + T_ / 8 - 1) / (T_ / 8), (T_ * DM / 4 + 8 * T_ - 1) / (8 * T_), \
                                            DM, T_, true>),                                                       \
                       dim3(nblk), dim3(8 * T_), lds, stream, X, N, d, y, W, ldw, wcol0, P, V, bias, loss, yscale,   \
                       f_part, r_part, G_part, dpad, colmap, cpr, nce);                                           \
  else                                                                                                            \
    hipLaunchKernelGGL((lr_objective_kernel<G, (DM / 8 + T_ / 8 - 1) / (T_ / 8), (T_ * DM / 4 + 8 * T_ - 1) / (8 * T_), \
                                            DM, T_, false>),                                                      \
                       dim3(nblk), dim3(8 * T_), lds, stream, X, N, d, y, W, ldw, wcol0, P, V, bias, loss, yscale,   \
                       f_part, r_part, G_part, dpad, (const int32_t*)nullptr, 0, 0)
#define TM_LR_D(G, T_)                \
  if (d <= 128) { TM_LR(G, 128, T_); } \
  else if (d <= 256) { TM_LR(G, 256, T_); } \
  else { TM_LR(G, 384, T_); }
  if (grad) {
    if (tt == 32) { TM_LR_D(true, 32) } else { TM_LR_D(true, 64) }
  } else {
    if (tt == 32) { TM_LR_D(false, 32) } else { TM_LR_D(false, 64) }
  }
#undef TM_LR_D
#undef TM_LR
  return (int)hipGetLastError();
}

int tmog_hip_lr_objective(const float* X, int64_t N, int d, const float* y, const float* W, int ldw, int wcol0,
                          int P, const float* V, const float* bias, int loss, const float* yscale, int grad,
                          double* f_part, double* r_part, float* G_part, int nblk, hipStream_t stream) {
  return lr_objective_launch(X, N, d, y, W, ldw, wcol0, P, V, bias, loss, yscale, grad, f_part, r_part, G_part, nblk,
                             stream, nullptr, 0, 0);
}

// The same pass over the lossless mixed-storage copy of X (Xm: N rows of cpr 16-byte chunks, nce of them bf16;
// colmap: [8 nce + 4 (cpr - nce)] original column per value slot, -1 = padding). Bit-identical to
// tmog_hip_lr_objective on the fp32 X. Returns -4 when the mixed row does not fit the pass's prefetch slots.
int tmog_hip_lr_objective_mixed(const void* Xm, int64_t N, int d, const int32_t* colmap, int cpr, int nce,
                                const float* y, const float* W, int ldw, int wcol0, int P, const float* V,
                                const float* bias, int loss, const float* yscale, int grad, double* f_part,
                                double* r_part, float* G_part, int nblk, hipStream_t stream) {
  if (colmap == nullptr) return -2;
  return lr_objective_launch((const float*)Xm, N, d, y, W, ldw, wcol0, P, V, bias, loss, yscale, grad, f_part, r_part,
                             G_part, nblk, stream, colmap, cpr, nce);
}

// OWL-QN direction (see owlqn_direction_kernel); all arrays fp64, [d1][P] / [m][d1][P] / [m][P] row-major.
int tmog_hip_owlqn_direction(const double* U, const double* g, const double* l1, const double* S, const double* Y,
                             const double* RHO, int d1, int P, int m, int hist_n, double* D, double* pg, double* xi,
                             double* dnorm, hipStream_t stream) {
  if (P < 1 || d1 < 1) return 0;
  if (d1 > OW_NT * OW_QMAX || m < 1 || m > OW_MMAX || hist_n < 0) return -2;
  if (d1 <= 16 * OW_NT)
    hipLaunchKernelGGL(owlqn_direction_kernel<16>, dim3(P), dim3(OW_NT), 0, stream, U, g, l1, S, Y, RHO, d1, P, m, hist_n,
                     D, pg, xi, dnorm);
  else
    hipLaunchKernelGGL(owlqn_direction_kernel<OW_QMAX>, dim3(P), dim3(OW_NT), 0, stream, U, g, l1, S, Y, RHO, d1, P, m, hist_n,
                     D, pg, xi, dnorm);
  return (int)hipGetLastError();
}

int tmog_hip_owlqn_candidate(const double* U, const double* D, const double* xi, const double* l1, const double* pg,
                             const double* alpha, int d1, int P, double* cand, double* l1t, double* dd,
                             hipStream_t stream) {
  if (P < 1 || d1 < 1) return 0;
  hipLaunchKernelGGL(owlqn_candidate_kernel, dim3(P), dim3(OW_NT), 0, stream, U, D, xi, l1, pg, alpha, d1, P, cand,
                     l1t, dd);
  return (int)hipGetLastError();
}

}  // extern "C"

// Multinomial (softmax) objective epilogue of the bf16 design-matrix path (Spark LogisticRegression family
// "multinomial", OpLogisticRegression.scala:46-207; models/linear.py MultinomialObjective). The margins come from
// one library GEMM of the bf16 design copy with [V_hi | V_lo] (fp32 output, [N][2C]: the high and low bf16 parts of
// the coefficients side by side, C = P * K problem-major columns). This kernel, one pass over those margins:
//   * m = M[r][c] + M[r][C + c] + bias[c], log-sum-exp over the K classes of each (row, problem), the weighted
//     loss w (lse - m_y) and R = w (softmax - onehot(y));
//   * fixed-order fp64 sums per workgroup of the loss per problem and of R per column (the intercept gradient),
//     so no margin or loss matrix is re-read by a column-sum launch;
//   * with the gradient, R as [R_hi | R_lo] bf16 [N][2C] for the gradient GEMM X^T [R_hi | R_lo] (~16 mantissa bits
//     of R through the bf16 matrix cores).
// Thread t of a workgroup owns problem p = t % P for every row it visits (rows r0 + t / P, step 256 / P), so its
// fp64 accumulators belong to one problem, and the per-problem sums over threads are taken in thread order.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

namespace {

constexpr int NT = 256;
constexpr int KMAX = 16;                 // LDS: 256 x 17 fp64 sums

__global__ void __launch_bounds__(NT) mnl_epilogue_kernel(
    const float* __restrict__ M2, int64_t N, int P, int K, const float* __restrict__ bias,
    const float* __restrict__ y, const float* __restrict__ W, int ldw, const int32_t* __restrict__ wmap,
    int64_t rows_per_blk, int grad, __bf16* __restrict__ R2, double* __restrict__ f_part,
    double* __restrict__ r_part) {
  const int C = P * K;
  const int rows_per_pass = NT / P;             // P <= NT
  const int t = threadIdx.x;
  const bool active = t < rows_per_pass * P;
  const int p = t % P, lr = t / P;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_blk;
  const int64_t r1 = min(N, r0 + rows_per_blk);
  double fs = 0.0, rs[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) rs[k] = 0.0;
  if (active) {
    const float* bb = bias + p * K;
    const int wc = wmap ? wmap[p] : p;
    for (int64_t r = r0 + lr; r < r1; r += rows_per_pass) {
      const float* mh = M2 + r * 2 * C + p * K;
      const float* ml = mh + C;
      const int yc = (int)y[r];
      float m[KMAX];
      float mx = -INFINITY, my = 0.f;
      bool has_y = false;
#pragma unroll
      for (int k = 0; k < KMAX; ++k)
        if (k < K) {
          m[k] = mh[k] + ml[k] + bb[k];
          mx = fmaxf(mx, m[k]);
          if (k == yc) {
            my = m[k];
            has_y = true;
          }
        }
      float se = 0.f;
#pragma unroll
      for (int k = 0; k < KMAX; ++k)
        if (k < K) {
          m[k] = __expf(m[k] - mx);             // m now holds exp(m - max)
          se += m[k];
        }
      const float w = W[r * ldw + wc];
      const float lse = mx + __logf(se);
      fs += (double)(w * (lse - (has_y ? my : lse)));
      const float inv = 1.f / se;
#pragma unroll
      for (int k = 0; k < KMAX; ++k)
        if (k < K) {
          const float rk = w * (m[k] * inv - (k == yc ? 1.f : 0.f));
          rs[k] += (double)rk;
          if (grad) {
            const __bf16 hi = (__bf16)rk;
            R2[r * 2 * C + p * K + k] = hi;
            R2[r * 2 * C + C + p * K + k] = (__bf16)(rk - (float)hi);
          }
        }
    }
  }
  // per-problem sums over the threads that own it, in thread order
  __shared__ double sh[NT][KMAX + 1];
  sh[t][0] = fs;
#pragma unroll
  for (int k = 0; k < KMAX; ++k)
    if (k < K) sh[t][k + 1] = rs[k];
  __syncthreads();
  for (int i = t; i < P * (K + 1); i += NT) {
    const int q = i / (K + 1), k = i - q * (K + 1);
    double a = 0.0;
    for (int u = q; u < rows_per_pass * P; u += P) a += sh[u][k];
    if (k == 0)
      f_part[(int64_t)blockIdx.x * P + q] = a;
    else
      r_part[(int64_t)blockIdx.x * C + q * K + (k - 1)] = a;
  }
}

}  // namespace

extern "C" {

// M2 [N][2C] fp32 (C = P * K: the products with V_hi then with V_lo), bias [C], y [N] class ids, W [N][ldw] with
// wmap[p] the weight column of problem p (nullptr: column p); P <= 256, K <= 16. Partials f [nblk][P],
// r [nblk][C] fp64; R2 [N][2C] bf16 (R_hi | R_lo) written when grad.
int tmog_hip_mnl_epilogue(const float* M2, int64_t N, int P, int K, const float* bias, const float* y, const float* W,
                          int ldw, const int32_t* wmap, int grad, void* R2, double* f_part, double* r_part, int nblk,
                          hipStream_t stream) {
  if (N <= 0 || nblk <= 0) return 0;
  if (P < 1 || P > NT || K < 1 || K > KMAX || (grad && R2 == nullptr)) return -2;
  const int64_t rpb = (N + nblk - 1) / nblk;
  hipLaunchKernelGGL(mnl_epilogue_kernel, dim3(nblk), dim3(NT), 0, stream, M2, N, P, K, bias, y, W, ldw, wmap, rpb,
                     grad, (__bf16*)R2, f_part, r_part);
  return (int)hipGetLastError();
}

}  // extern "C"

namespace {

// ------------------------------------------------------------------------------------------------------------
// mnl_bf16_kernel -- the fused multinomial pass: margins of 32 problems x K classes for 32-row tiles of the bf16
// design copy on the bf16 matrix cores, then the softmax epilogue straight from the accumulators; no margin matrix
// goes to memory. Columns are class-major (column k * 32 + p = class k of problem p), so the K margins of a
// (row, problem) sit in one lane, in register e of the K accumulators: the softmax needs no lane traffic.
// The coefficient image V^T [hi | lo][K * 32][dpad] (bf16) is too large for LDS at text widths, so a workgroup of
// 8 waves walks the features in 64-wide chunks in lockstep: the next chunk's V^T and X rows are loaded into
// registers while the current chunk's MFMAs run, then V^T goes to LDS between two barriers. Waves whose tile is
// past the end keep the barrier cadence on a clamped tile and write nothing. With grad, R = w (softmax - onehot)
// is written as [R_hi | R_lo] bf16 [npad][2 * K * 32] for the split-K gradient GEMM (ops/linear.py).
typedef __bf16 mbf16x8 __attribute__((ext_vector_type(8)));
typedef float mf32x16 __attribute__((ext_vector_type(16)));

constexpr int MKC = 64;               // features per chunk
constexpr int MNW = 8;                // waves per workgroup
constexpr int MVS = MKC + 8;          // LDS row stride of the V^T chunk (bf16)

template <int K, bool GRAD>
__global__ void __launch_bounds__(64 * MNW) mnl_bf16_kernel(
    const __bf16* __restrict__ X, int64_t ldx, int64_t N, int dpad, const float* __restrict__ y,
    const float* __restrict__ W, int ldw, const int32_t* __restrict__ wcol, int pc, const __bf16* __restrict__ Vt,
    const float* __restrict__ bias, __bf16* __restrict__ R2, double* __restrict__ f_part,
    double* __restrict__ r_part) {
  constexpr int NC = K * 32;                          // columns of this launch
  constexpr int VPT = 2 * NC * MKC / 8 / (64 * MNW);  // 16-byte V^T pieces per thread per chunk
  static_assert((2 * NC * MKC / 8) % (64 * MNW) == 0, "V chunk split");
  extern __shared__ __attribute__((aligned(16))) __bf16 vs[];     // [2][NC][MVS]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r31 = lane & 31, h = lane >> 5, p = r31;
  const int64_t ntiles = (N + 31) / 32;
  const int64_t per_round = (int64_t)gridDim.x * MNW;
  const int64_t rounds = (ntiles + per_round - 1) / per_round;
  const int nch = dpad / MKC;
  const int wc = wcol[p];
  float bk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) bk[k] = bias[k * 32 + p];
  double fs = 0.0, rs[K];
#pragma unroll
  for (int k = 0; k < K; ++k) rs[k] = 0.0;
  for (int64_t rd = 0; rd < rounds; ++rd) {
    const int64_t t = (rd * gridDim.x + blockIdx.x) * MNW + wv;
    const bool live = t < ntiles;
    const int64_t r0 = (live ? t : ntiles - 1) * 32;
    const __bf16* xrow = X + (r0 + r31) * ldx + 8 * h;
    mf32x16 acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = mf32x16{};
    mbf16x8 xk[MKC / 16], xn[MKC / 16], vr[VPT];
    auto load_v = [&](int ch) {
#pragma unroll
      for (int u = 0; u < VPT; ++u) {
        const int idx = u * 64 * MNW + threadIdx.x;          // piece: (part, column, 8-feature segment)
        const int seg = idx % (MKC / 8), row = idx / (MKC / 8);  // row = part * NC + column
        vr[u] = *reinterpret_cast<const mbf16x8*>(Vt + (int64_t)row * dpad + ch * MKC + seg * 8);
      }
    };
    auto store_v = [&]() {
#pragma unroll
      for (int u = 0; u < VPT; ++u) {
        const int idx = u * 64 * MNW + threadIdx.x;
        const int seg = idx % (MKC / 8), row = idx / (MKC / 8);
        *reinterpret_cast<mbf16x8*>(vs + row * MVS + seg * 8) = vr[u];
      }
    };
#pragma unroll
    for (int s = 0; s < MKC / 16; ++s) xk[s] = *reinterpret_cast<const mbf16x8*>(xrow + 16 * s);
    load_v(0);
    __syncthreads();                                   // the previous round's last chunk is no longer read
    store_v();
    __syncthreads();
    for (int ch = 0; ch < nch; ++ch) {
      const bool more = ch + 1 < nch;
      if (more) {                                      // next chunk in flight during this chunk's MFMAs
#pragma unroll
        for (int s = 0; s < MKC / 16; ++s)
          xn[s] = *reinterpret_cast<const mbf16x8*>(xrow + (ch + 1) * MKC + 16 * s);
        load_v(ch + 1);
      }
#pragma unroll
      for (int s = 0; s < MKC / 16; ++s) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const mbf16x8 bh = *reinterpret_cast<const mbf16x8*>(vs + (k * 32 + p) * MVS + 16 * s + 8 * h);
          const mbf16x8 bl = *reinterpret_cast<const mbf16x8*>(vs + (NC + k * 32 + p) * MVS + 16 * s + 8 * h);
          acc[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xk[s], bh, acc[k], 0, 0, 0);
          acc[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xk[s], bl, acc[k], 0, 0, 0);
        }
      }
      if (more) {
        __syncthreads();
        store_v();
        __syncthreads();
#pragma unroll
        for (int s = 0; s < MKC / 16; ++s) xk[s] = xn[s];
      }
    }
    if (!live) continue;
    // epilogue: register e of every accumulator = row (e & 3) + 8 (e >> 2) + 4 h of the tile, problem p
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int64_t r = r0 + (e & 3) + 8 * (e >> 2) + 4 * h;
      if (r >= N) continue;
      const float w = p < pc ? W[r * ldw + wc] : 0.f;
      const int yc = (int)y[r];
      float m[K], mx = -INFINITY, my = 0.f;
      bool has_y = false;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        m[k] = acc[k][e] + bk[k];
        mx = fmaxf(mx, m[k]);
        if (k == yc) {
          my = m[k];
          has_y = true;
        }
      }
      float se = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        m[k] = __expf(m[k] - mx);
        se += m[k];
      }
      const float lse = mx + __logf(se);
      fs += (double)(w * (lse - (has_y ? my : lse)));
      const float inv = 1.f / se;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const float rk = w * (m[k] * inv - (k == yc ? 1.f : 0.f));
        rs[k] += (double)rk;
        if constexpr (GRAD) {
          const __bf16 hi = (__bf16)rk;
          R2[r * 2 * NC + k * 32 + p] = hi;
          R2[r * 2 * NC + NC + k * 32 + p] = (__bf16)(rk - (float)hi);
        }
      }
    }
  }
  fs += __shfl_xor(fs, 32, 64);
#pragma unroll
  for (int k = 0; k < K; ++k) rs[k] += __shfl_xor(rs[k], 32, 64);
  if (h == 0) {
    const int64_t gw = (int64_t)blockIdx.x * MNW + wv;
    f_part[gw * 32 + p] = fs;
#pragma unroll
    for (int k = 0; k < K; ++k) r_part[gw * NC + k * 32 + p] = rs[k];
  }
}

}  // namespace

extern "C" {

// Fused multinomial pass (mnl_bf16_kernel): X [npad][ldx] bf16 (npad a multiple of 32, dpad a multiple of 64,
// zero padding), Vt [2][K * 32][dpad] bf16 (hi, lo; class-major columns k * 32 + p), bias [K * 32] class-major,
// wcol [32] the W column of each problem, K in 2..6 (the K accumulators and the chunk registers fill the
// 256 VGPRs of two waves per SIMD; more classes take the library-GEMM path), pc <= 32. Partials per wave: f [nblk * 8][32],
// r [nblk * 8][K * 32] fp64; R2 [npad][2 * K * 32] bf16 when grad.
int tmog_hip_mnl_bf16(const void* X, int64_t ldx, int64_t N, int dpad, const float* y, const float* W, int ldw,
                      const int32_t* wcol, int pc, int K, const void* Vt, const float* bias, int grad, void* R2,
                      double* f_part, double* r_part, int nblk, hipStream_t stream) {
  if (N <= 0 || nblk <= 0) return 0;
  if (dpad <= 0 || dpad % MKC || ldx < dpad || ldx % 8 || (uintptr_t)X % 16 || (uintptr_t)Vt % 16 || pc < 1 ||
      pc > 32 || K < 2 || K > 6 || (grad && R2 == nullptr))
    return -2;
  const size_t lds = sizeof(__bf16) * 2 * K * 32 * MVS;
  const dim3 g(nblk), b(64 * MNW);
  const __bf16* x = (const __bf16*)X;
  const __bf16* vt = (const __bf16*)Vt;
  __bf16* r2 = (__bf16*)R2;
#define TMOG_MNL_CASE(KK)                                                                                      \
  case KK:                                                                                                     \
    if (grad)                                                                                                  \
      hipLaunchKernelGGL((mnl_bf16_kernel<KK, true>), g, b, lds, stream, x, ldx, N, dpad, y, W, ldw, wcol, pc, vt, \
                         bias, r2, f_part, r_part);                                                            \
    else                                                                                                       \
      hipLaunchKernelGGL((mnl_bf16_kernel<KK, false>), g, b, lds, stream, x, ldx, N, dpad, y, W, ldw, wcol, pc,    \
                         vt, bias, r2, f_part, r_part);                                                        \
    break;
  switch (K) {
    TMOG_MNL_CASE(2) TMOG_MNL_CASE(3) TMOG_MNL_CASE(4) TMOG_MNL_CASE(5) TMOG_MNL_CASE(6)
    default: return -2;
  }
#undef TMOG_MNL_CASE
  return (int)hipGetLastError();
}

}  // extern "C"

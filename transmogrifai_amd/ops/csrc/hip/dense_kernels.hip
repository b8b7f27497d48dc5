// Dense fp32 GEMMs of the learners on the CDNA4 matrix cores (gfx950, v_mfma_f32_32x32x2_f32: exact fp32
// products, one rounding each -- the numerics of an fp32 fmaf chain).
//
// The learners' dense products are "row GEMMs": one dimension is the row count N (up to 10^8), the others are a
// feature count (<= a few thousand) and a column count (grid points x classes / hidden units, <= a few hundred):
//
//   rowgemm_kernel   C_p[n, c] = epi( sum_k A_p[n, k] B_p(k, c) + bias_p(c) )      forward products
//                    (the multinomial margins X V, every MLP layer with its bias + sigmoid fused, the MLP's
//                    back-propagated activations dZ W^T), 128 x 64 output tiles, K staged 32 at a time in LDS
//   xtd_kernel       G_p[k, c] = sum_n A_p[n, k] D_p(n, c)                          gradient products
//                    (X^T R of the multinomial / linear objectives, the MLP's weight gradients), 64 x 64 output
//                    tiles per row chunk, fp32 inside a chunk; xtd_reduce_kernel adds the chunk partials in fp64
//                    in a fixed order (deterministic, no atomics)
//
// "Grouped" columns let one launch serve P problems that share A: column c belongs to group c / g at offset c % g
// and its B / D / bias / output addresses step by a group stride -- the P jobs' weight matrices [P, K, g] and
// their outputs [P, N, g] are read and written in place, and A (the design matrix, the only large operand) is
// streamed once per 64-column tile instead of once per job. A batch index (grid z) covers products whose A differs
// per job (hidden layers). Reference: SURVEY.md K19-K22 / K27 (Spark's BLAS gemm for LogisticRegression with
// multinomial family and MultilayerPerceptronClassifier, OpLogisticRegression.scala / OpMultilayerPerceptron-
// Classifier.scala:49-144).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;

struct ColMap {             // column c of a product: group c / g, offset c % g
  int g;
  int64_t stride;           // elements between groups
  __device__ __forceinline__ int64_t off(int c) const {
    const int q = c / g;
    return (int64_t)q * stride + (c - q * g);
  }
};

constexpr int RG_BM = 128, RG_BN = 64, RG_BK = 32;
constexpr int RG_LDA = RG_BK + 1;          // A tile row pitch (33: the 32 rows of a wave's read hit 32 banks)
constexpr int RG_LDB = 96;                 // B tile row pitch (two k rows of a read land 32 banks apart)

// EPI 0: none, 1: sigmoid. B(k, c): btrans ? B[off(c) * ldb + k] : B[k * ldb + off(c)]
template <int EPI>
__global__ void __launch_bounds__(256) rowgemm_kernel(const float* __restrict__ A, int64_t lda, int64_t a_pstride,
                                                      const float* __restrict__ B, int64_t ldb, int64_t b_pstride,
                                                      int btrans, ColMap bmap, const float* __restrict__ bias,
                                                      int64_t bias_pstride, ColMap biasmap, float* __restrict__ C,
                                                      int64_t ldc, int64_t c_pstride, ColMap cmap, int64_t N, int K,
                                                      int M) {
  __shared__ float As[RG_BM * RG_LDA];
  __shared__ float Bs[RG_BK * RG_LDB];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int p = blockIdx.z;
  const int64_t n0 = (int64_t)blockIdx.x * RG_BM;
  const int c0 = blockIdx.y * RG_BN;
  const float* Ap = A + (int64_t)p * a_pstride;
  const float* Bp = B + (int64_t)p * b_pstride;
  const int wr = (w >> 1) * 64, wc = (w & 1) * 32;   // this wave's 64 x 32 block of the tile
  f32x16 acc0 = {}, acc1 = {};
  for (int k0 = 0; k0 < K; k0 += RG_BK) {
    // stage A [128 rows x 32 k] (a wave loads two contiguous 128-byte row segments) and B [32 k x 64 c]
#pragma unroll
    for (int it = 0; it < (RG_BM * RG_BK) / 256; ++it) {
      const int idx = it * 256 + t;
      const int r = idx >> 5, k = idx & 31;
      const int64_t n = n0 + r;
      As[r * RG_LDA + k] = (n < N && k0 + k < K) ? Ap[n * lda + k0 + k] : 0.f;
    }
#pragma unroll
    for (int it = 0; it < (RG_BK * RG_BN) / 256; ++it) {
      const int idx = it * 256 + t;
      const int k = idx >> 6, c = idx & 63;
      float v = 0.f;
      if (k0 + k < K && c0 + c < M) {
        const int64_t o = bmap.off(c0 + c);
        v = btrans ? Bp[o * ldb + k0 + k] : Bp[(int64_t)(k0 + k) * ldb + o];
      }
      Bs[k * RG_LDB + c] = v;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < RG_BK; kk += 2) {
      const int ka = kk + (lane >> 5);
      const float b = Bs[ka * RG_LDB + wc + (lane & 31)];
      const float a0 = As[(wr + (lane & 31)) * RG_LDA + ka];
      const float a1 = As[(wr + 32 + (lane & 31)) * RG_LDA + ka];
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b, acc1, 0, 0, 0);
    }
    __syncthreads();
  }
  // epilogue: column on the lane, rows in the 16 registers (row = 8 (r >> 2) + 4 (lane >> 5) + (r & 3))
  const int c = c0 + wc + (lane & 31);
  if (c >= M) return;
  const float bv = bias != nullptr ? bias[(int64_t)p * bias_pstride + biasmap.off(c)] : 0.f;
  float* Cp = C + (int64_t)p * c_pstride + cmap.off(c);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const f32x16& acc = h ? acc1 : acc0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t n = n0 + wr + 32 * h + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3);
      if (n < N) {
        float v = acc[r] + bv;
        if (EPI == 1) v = __builtin_amdgcn_rcpf(1.f + __expf(-v));
        Cp[n * ldc] = v;
      }
    }
  }
}

constexpr int XT_BK = 64, XT_BN = 64, XT_BR = 32;
constexpr int XT_LD = 96;                  // row pitch of both staged tiles (see RG_LDB)

// grid (k tiles x c tiles, row chunks, P): partial[((s * P + p) * K + k) * M + c] over rows [s * chunk, ...)
__global__ void __launch_bounds__(256) xtd_kernel(const float* __restrict__ A, int64_t lda, int64_t a_pstride,
                                                  const float* __restrict__ D, int64_t ldd, int64_t d_pstride,
                                                  ColMap dmap, int64_t N, int K, int M, int64_t chunk,
                                                  float* __restrict__ part) {
  __shared__ float Xs[XT_BR * XT_LD];
  __shared__ float Ds[XT_BR * XT_LD];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int ktiles = (K + XT_BK - 1) / XT_BK;
  const int k0 = (blockIdx.x % ktiles) * XT_BK, c0 = (blockIdx.x / ktiles) * XT_BN;
  const int s = blockIdx.y, p = blockIdx.z, P = gridDim.z;
  const int64_t r0 = (int64_t)s * chunk, r1 = min(N, r0 + chunk);
  const float* Ap = A + (int64_t)p * a_pstride;
  const float* Dp = D + (int64_t)p * d_pstride;
  const int wk = (w >> 1) * 32, wc = (w & 1) * 32;
  // this thread's staged columns: k0 + (t & 63) of A and the D column offset of c0 + (t & 63)
  const int sc = t & 63, sr = t >> 6;
  const bool kin = k0 + sc < K, cin = c0 + sc < M;
  const int64_t doff = cin ? dmap.off(c0 + sc) : 0;
  f32x16 acc = {};
  for (int64_t rb = r0; rb < r1; rb += XT_BR) {
#pragma unroll
    for (int it = 0; it < XT_BR / 4; ++it) {
      const int r = it * 4 + sr;
      const int64_t n = rb + r;
      const bool rin = n < r1;
      Xs[r * XT_LD + sc] = (rin && kin) ? Ap[n * lda + k0 + sc] : 0.f;
      Ds[r * XT_LD + sc] = (rin && cin) ? Dp[doff + n * ldd] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int rr = 0; rr < XT_BR; rr += 2) {
      const int r = rr + (lane >> 5);
      const float a = Xs[r * XT_LD + wk + (lane & 31)];
      const float b = Ds[r * XT_LD + wc + (lane & 31)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    __syncthreads();
  }
  const int c = c0 + wc + (lane & 31);
  if (c >= M) return;
  float* out = part + ((int64_t)s * P + p) * (int64_t)K * M;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int k = k0 + wk + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3);
    if (k < K) out[(int64_t)k * M + c] = acc[r];
  }
}

// out[e] = sum_s part[s * total + e] in fp64, s ascending
__global__ void __launch_bounds__(256) xtd_reduce_kernel(const float* __restrict__ part, int S, int64_t total,
                                                         double* __restrict__ out) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    double acc = 0.0;
    for (int s = 0; s < S; ++s) acc += (double)part[(int64_t)s * total + e];
    out[e] = acc;
  }
}

}  // namespace

extern "C" {

// C_p[n, c] = epi(A_p[n, :] . B_p(:, c) + bias_p(c)) for p < P, n < N, c < M. Group maps: g columns per group,
// *_gstride elements between groups (g = M: one group).
int tmog_hip_rowgemm(const float* A, int64_t lda, int64_t a_pstride, const float* B, int64_t ldb, int64_t b_pstride,
                     int btrans, int bg, int64_t b_gstride, const float* bias, int64_t bias_pstride, int64_t bias_gstride,
                     float* C, int64_t ldc, int64_t c_pstride, int cg, int64_t c_gstride, int64_t N, int K, int M, int P,
                     int epi, hipStream_t stream) {
  if (N <= 0 || M <= 0 || P <= 0) return 0;
  if (K < 0 || bg < 1 || cg < 1 || P > 65535 || epi < 0 || epi > 1) return -2;
  const int64_t nt = (N + RG_BM - 1) / RG_BM;
  const int ct = (M + RG_BN - 1) / RG_BN;
  if (nt > 0x7fffffff || ct > 65535) return -2;
  const ColMap bm{bg, b_gstride}, biasm{bg, bias_gstride}, cm{cg, c_gstride};
  const dim3 grid((unsigned)nt, (unsigned)ct, (unsigned)P);
  if (epi == 1)
    hipLaunchKernelGGL(rowgemm_kernel<1>, grid, dim3(256), 0, stream, A, lda, a_pstride, B, ldb, b_pstride, btrans,
                       bm, bias, bias_pstride, biasm, C, ldc, c_pstride, cm, N, K, M);
  else
    hipLaunchKernelGGL(rowgemm_kernel<0>, grid, dim3(256), 0, stream, A, lda, a_pstride, B, ldb, b_pstride, btrans,
                       bm, bias, bias_pstride, biasm, C, ldc, c_pstride, cm, N, K, M);
  return (int)hipGetLastError();
}

// Row chunks of the gradient product for a target grid size: returns S (chunk = ceil(N / S) rounded to 32).
int tmog_hip_xtd_chunks(int64_t N, int K, int M, int P, int target_blocks) {
  if (N <= 0) return 1;
  const int64_t tiles = (int64_t)((K + XT_BK - 1) / XT_BK) * ((M + XT_BN - 1) / XT_BN) * P;
  int64_t s = (target_blocks + tiles - 1) / tiles;
  s = s < 1 ? 1 : s;
  const int64_t maxs = (N + 255) / 256;     // at least 256 rows a chunk
  if (s > maxs) s = maxs;
  if (s > 65535) s = 65535;
  return (int)s;
}

// out_p[k, c] (fp64, [P, K, M]) = sum_n A_p[n, k] D_p(n, c); part: S * P * K * M floats of scratch.
int tmog_hip_xtd(const float* A, int64_t lda, int64_t a_pstride, const float* D, int64_t ldd, int64_t d_pstride,
                 int dg, int64_t d_gstride, int64_t N, int K, int M, int P, int S, float* part, double* out,
                 hipStream_t stream) {
  if (K <= 0 || M <= 0 || P <= 0) return 0;
  if (dg < 1 || S < 1 || S > 65535 || P > 65535) return -2;
  const int64_t total = (int64_t)P * K * M;
  if (N <= 0) return (int)hipMemsetAsync(out, 0, total * sizeof(double), stream);
  int64_t chunk = (N + S - 1) / S;
  chunk = (chunk + XT_BR - 1) / XT_BR * XT_BR;
  const int64_t tiles = (int64_t)((K + XT_BK - 1) / XT_BK) * ((M + XT_BN - 1) / XT_BN);
  if (tiles > 0x7fffffff) return -2;
  // every chunk s < S must start below N (the host computes S from N; a larger S leaves zero partials)
  const ColMap dm{dg, d_gstride};
  hipLaunchKernelGGL(xtd_kernel, dim3((unsigned)tiles, (unsigned)S, (unsigned)P), dim3(256), 0, stream, A, lda,
                     a_pstride, D, ldd, d_pstride, dm, N, K, M, chunk, part);
  const int64_t nb = (total + 255) / 256;
  hipLaunchKernelGGL(xtd_reduce_kernel, dim3((unsigned)(nb < 4096 ? nb : 4096)), dim3(256), 0, stream, part, S, total,
                     out);
  return (int)hipGetLastError();
}

}  // extern "C"

// Sparse design-matrix products and the fused multinomial epilogue for the linear learners (CDNA4, gfx950).
//
// The multi-class text configuration's feature matrix is ~3 % dense (hashed term frequencies and one-hot
// pivots: ~44 non-zeros of 1352 columns per row). The linear learners keep its dense columns as a dense
// block (library GEMM) and its sparse columns as CSR + segmented CSC (ops/linear.py SparseDesign), so an
// objective evaluation reads the non-zeros instead of the whole N x d matrix
// (OpLogisticRegression.scala:46-207 multinomial family; Spark aggregates sparse vectors the same way).
//
//   csr_spmm_kernel     M[N][C] (+)= Xs[N][ds] . V[ds][C]   one wave per row, lanes over the C columns,
//                       the row's (col, val) pairs broadcast from a 64-entry register batch
//   csc_spmm_t_kernel   partial[seg][C] = sum over the segment's non-zeros of val * R[row][C]; every
//                       column's non-zeros are cut into segments of <= kSegNnz, one wave each (a one-hot
//                       value present in 25 % of 1M rows is 62 waves, not one)
//   seg_reduce_kernel   G[col][C] = sum of the column's segment partials, in segment order (deterministic)
//   softmax_epilogue_kernel  per (row, problem): log-sum-exp of the K class margins, the weighted loss and
//                       R = w (softmax - onehot(y)) in place of the margins
//   colsum_kernel       fp64 per-block column sums of a row-major matrix over contiguous row slices (the
//                       loss and intercept-gradient sums, fixed order)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

namespace {

constexpr int kMaxC = 256;     // output columns per launch (lanes x 4)

// Both products walk a list of (index, value) pairs per wave and gather one row of a small dense operand per
// pair (V[col] for X V, R[row] for X^T R). The gathers of kU pairs are issued before their FMAs, so kU
// independent row loads are in flight per wave instead of one dependent load per pair (the loop was
// load-latency bound: ~25x below the kernel's memory roofline). The FMAs keep the pairs' order, so
// results are unchanged and deterministic. CU = ceil(C / 64) column chunks per lane.
constexpr int kU = 8;

template <int CU>
__device__ __forceinline__ void gather_fma(const int64_t a, const int64_t b, const int32_t* __restrict__ idx,
                                           const float* __restrict__ val, const float* __restrict__ D, int64_t ldd,
                                           int C, int lane, float* acc) {
  for (int64_t base = a; base < b; base += 64) {
    const int n = (int)min((int64_t)64, b - base);
    const int my_i = lane < n ? idx[base + lane] : 0;
    const float my_v = lane < n ? val[base + lane] : 0.f;
    int t = 0;
    for (; t + kU <= n; t += kU) {
      float xs[kU], vv[kU][CU];
#pragma unroll
      for (int k = 0; k < kU; ++k) {
        const int i = __shfl(my_i, t + k, 64);
        xs[k] = __shfl(my_v, t + k, 64);
        const float* dr = D + (int64_t)i * ldd;
#pragma unroll
        for (int u = 0; u < CU; ++u) {
          const int j = lane + 64 * u;
          vv[k][u] = j < C ? dr[j] : 0.f;
        }
      }
#pragma unroll
      for (int k = 0; k < kU; ++k)
#pragma unroll
        for (int u = 0; u < CU; ++u) acc[u] += xs[k] * vv[k][u];
    }
    for (; t < n; ++t) {
      const int i = __shfl(my_i, t, 64);
      const float x = __shfl(my_v, t, 64);
      const float* dr = D + (int64_t)i * ldd;
#pragma unroll
      for (int u = 0; u < CU; ++u) {
        const int j = lane + 64 * u;
        if (j < C) acc[u] += x * dr[j];
      }
    }
  }
}

template <int CU>
__global__ void __launch_bounds__(256) csr_spmm_kernel(const int64_t* __restrict__ row_ptr,
                                                       const int32_t* __restrict__ col,
                                                       const float* __restrict__ val, int64_t N,
                                                       const float* __restrict__ V, int C,
                                                       float* __restrict__ M, int ldm, int accumulate) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  float acc[CU];
#pragma unroll
  for (int u = 0; u < CU; ++u) acc[u] = 0.f;
  gather_fma<CU>(row_ptr[row], row_ptr[row + 1], col, val, V, C, C, lane, acc);
  float* out = M + row * ldm;
#pragma unroll
  for (int u = 0; u < CU; ++u) {
    const int j = lane + 64 * u;
    if (j < C) out[j] = accumulate ? out[j] + acc[u] : acc[u];
  }
}

template <int CU>
__global__ void __launch_bounds__(256) csc_spmm_t_kernel(const int64_t* __restrict__ seg_begin,
                                                         const int32_t* __restrict__ row, const float* __restrict__ val,
                                                         int64_t n_seg, const float* __restrict__ R, int C, int ldr,
                                                         float* __restrict__ partial) {
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= n_seg) return;
  float acc[CU];
#pragma unroll
  for (int u = 0; u < CU; ++u) acc[u] = 0.f;
  gather_fma<CU>(seg_begin[s], seg_begin[s + 1], row, val, R, ldr, C, lane, acc);
  float* out = partial + s * C;
#pragma unroll
  for (int u = 0; u < CU; ++u) {
    const int j = lane + 64 * u;
    if (j < C) out[j] = acc[u];
  }
}

// G[col][c] (fp64) = sum_{s in col's segments} partial[s][c]: one thread per (col, c), segments in order
__global__ void __launch_bounds__(256) seg_reduce_kernel(const int64_t* __restrict__ col_seg, int64_t ds,
                                                         const float* __restrict__ partial, int C,
                                                         double* __restrict__ G) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ds * C) return;
  const int64_t c = i / C, j = i - c * C;
  double acc = 0.0;
  for (int64_t s = col_seg[c]; s < col_seg[c + 1]; ++s) acc += (double)partial[s * C + j];
  G[i] = acc;
}

// Multinomial epilogue: M [N][P*K] holds the margins without bias (problem p's classes at p*K..p*K+K-1);
// bias [P*K]; y [N] class ids; W [N][P] (ldw) row weights. One thread per (row, problem): Lw[r][p] =
// w (lse - m_y) and, with grad, R = w (softmax - onehot(y)) in place of the margins. The sums over rows are
// taken by colsum_kernel in a fixed order (deterministic, no atomics).
__global__ void __launch_bounds__(256) softmax_epilogue_kernel(float* __restrict__ M, int64_t N, int P, int K,
                                                               const float* __restrict__ bias,
                                                               const float* __restrict__ y,
                                                               const float* __restrict__ W, int ldw,
                                                               float* __restrict__ Lw, int grad) {
  const int C = P * K;
  const int64_t total = N * (int64_t)P;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / P;
    const int p = (int)(e - r * P);
    float* m = M + r * C + p * K;
    const float* bb = bias + p * K;
    const float w = W[r * ldw + p];
    const int yc = (int)y[r];
    float mx = -INFINITY;
    for (int k = 0; k < K; ++k) mx = fmaxf(mx, m[k] + bb[k]);
    float se = 0.f;
    for (int k = 0; k < K; ++k) se += __expf(m[k] + bb[k] - mx);
    const float lse = mx + __logf(se);
    const float my = (yc >= 0 && yc < K) ? m[yc] + bb[yc] : lse;
    Lw[e] = w * (lse - my);
    if (grad) {
      const float inv = 1.f / se;
      for (int k = 0; k < K; ++k) {
        const float pk = __expf(m[k] + bb[k] - mx) * inv;
        m[k] = w * (pk - (k == yc ? 1.f : 0.f));
      }
    }
  }
}

// R column sums: rsum_part[blk][C] over a contiguous row slice per block (fp64, fixed order per block)
__global__ void __launch_bounds__(256) colsum_kernel(const float* __restrict__ R, int64_t N, int C,
                                                     int64_t rows_per_blk, double* __restrict__ part) {
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_blk;
  const int64_t r1 = min(N, r0 + rows_per_blk);
  for (int j = threadIdx.x; j < C; j += blockDim.x) {
    double acc = 0.0;
    for (int64_t r = r0; r < r1; ++r) acc += (double)R[r * C + j];
    part[(int64_t)blockIdx.x * C + j] = acc;
  }
}

}  // namespace

extern "C" {

int tmog_hip_csr_spmm(const int64_t* row_ptr, const int32_t* col, const float* val, int64_t N, const float* V, int C,
                      float* M, int ldm, int accumulate, hipStream_t stream) {
  if (N == 0) return 0;
  if (C <= 0 || C > kMaxC) return -2;
#define TM_CSR(CUV)                                                                                            \
  hipLaunchKernelGGL(csr_spmm_kernel<CUV>, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, stream, row_ptr, col, val, N, \
                     V, C, M, ldm, accumulate)
  if (C <= 64) TM_CSR(1);
  else if (C <= 128) TM_CSR(2);
  else if (C <= 192) TM_CSR(3);
  else TM_CSR(4);
#undef TM_CSR
  return (int)hipGetLastError();
}

int tmog_hip_csc_spmm_t(const int64_t* seg_begin, const int32_t* row, const float* val, int64_t n_seg,
                        const int64_t* col_seg, int64_t ds, const float* R, int C, int ldr, float* partial, double* G,
                        hipStream_t stream) {
  if (C <= 0 || C > kMaxC) return -2;
#define TM_CSC(CUV)                                                                                            \
  hipLaunchKernelGGL(csc_spmm_t_kernel<CUV>, dim3((unsigned)((n_seg + 3) / 4)), dim3(256), 0, stream, seg_begin,    \
                     row, val, n_seg, R, C, ldr, partial)
  if (n_seg > 0) {
    if (C <= 64) TM_CSC(1);
    else if (C <= 128) TM_CSC(2);
    else if (C <= 192) TM_CSC(3);
    else TM_CSC(4);
  }
#undef TM_CSC
  if (ds > 0)
    hipLaunchKernelGGL(seg_reduce_kernel, dim3((unsigned)((ds * C + 255) / 256)), dim3(256), 0, stream, col_seg, ds,
                       partial, C, G);
  return (int)hipGetLastError();
}

int tmog_hip_softmax_epilogue(float* M, int64_t N, int P, int K, const float* bias, const float* y, const float* W,
                              int ldw, float* Lw, int grad, hipStream_t stream) {
  if (N == 0 || P <= 0) return 0;
  const int64_t total = N * (int64_t)P;
  const unsigned nblk = (unsigned)min((total + 255) / 256, (int64_t)65536);
  hipLaunchKernelGGL(softmax_epilogue_kernel, dim3(nblk), dim3(256), 0, stream, M, N, P, K, bias, y, W, ldw, Lw, grad);
  return (int)hipGetLastError();
}

int tmog_hip_colsum(const float* R, int64_t N, int C, int nblk, double* part, hipStream_t stream) {
  if (N == 0) return 0;
  const int64_t rpb = (N + nblk - 1) / nblk;
  hipLaunchKernelGGL(colsum_kernel, dim3(nblk), dim3(256), 0, stream, R, N, C, rpb, part);
  return (int)hipGetLastError();
}

}  // extern "C"

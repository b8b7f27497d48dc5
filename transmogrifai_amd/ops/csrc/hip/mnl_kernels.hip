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

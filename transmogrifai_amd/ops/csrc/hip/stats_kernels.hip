// Column moments in one HBM pass (Spark Statistics.colStats used by SanityChecker,
// MinVarianceFilter, RecordInsightsCorr). Row-major fp32 [n][ld]; each workgroup covers 64 columns
// x a row chunk: 4 waves stride the rows, every lane owns one column (256 B coalesced per row),
// accumulating sum / sum of squares in fp64 plus min / max / non-zeros. Partials go to
// part[chunk][5][d]; a tiny second kernel folds the chunks into out[6][d].
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <float.h>

namespace {

__global__ void __launch_bounds__(256) col_partials_kernel(const float* __restrict__ X, int64_t n, int d, int64_t ld,
                                                           int64_t rows_per_chunk, double* __restrict__ part) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int ty = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
  const int64_t r1 = min(n, r0 + rows_per_chunk);
  double s = 0, q = 0, nz = 0;
  float mn = FLT_MAX, mx = -FLT_MAX;
  if (c < d) {
    for (int64_t r = r0 + ty; r < r1; r += 4) {
      const float v = X[r * ld + c];
      s += v;
      q += (double)v * v;
      mn = fminf(mn, v);
      mx = fmaxf(mx, v);
      nz += v != 0.f;
    }
  }
  __shared__ double sh[4][5][64];
  const int l = threadIdx.x & 63;
  sh[ty][0][l] = s; sh[ty][1][l] = q; sh[ty][2][l] = mn; sh[ty][3][l] = mx; sh[ty][4][l] = nz;
  __syncthreads();
  if (ty == 0 && c < d) {
    for (int k = 1; k < 4; ++k) {
      s += sh[k][0][l]; q += sh[k][1][l]; nz += sh[k][4][l];
      mn = fminf(mn, (float)sh[k][2][l]); mx = fmaxf(mx, (float)sh[k][3][l]);
    }
    double* p = part + (int64_t)blockIdx.y * 5 * d;
    p[c] = s; p[d + c] = q; p[2 * d + c] = mn; p[3 * d + c] = mx; p[4 * d + c] = nz;
  }
}

__global__ void col_fold_kernel(const double* __restrict__ part, int chunks, int d, double* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= d) return;
  double s = 0, q = 0, nz = 0, mn = DBL_MAX, mx = -DBL_MAX;
  for (int k = 0; k < chunks; ++k) {
    const double* p = part + (int64_t)k * 5 * d;
    s += p[c]; q += p[d + c]; nz += p[4 * d + c];
    mn = fmin(mn, p[2 * d + c]); mx = fmax(mx, p[3 * d + c]);
  }
  out[c] = s; out[d + c] = q; out[2 * d + c] = mn; out[3 * d + c] = mx; out[4 * d + c] = nz; out[5 * d + c] = 0;
}

}  // namespace

extern "C" int tmog_hip_col_stats(const float* X, const void* unused, int64_t n, int d, int64_t ld, double* out,
                                  hipStream_t stream) {
  (void)unused;
  if (n == 0 || d == 0) return 0;
  const int cblocks = (d + 63) / 64;
  int64_t chunks = (2048 + cblocks - 1) / cblocks;           // ~2048 workgroups in flight
  if (chunks > n / 256 + 1) chunks = n / 256 + 1;
  if (chunks < 1) chunks = 1;
  const int64_t rpc = (n + chunks - 1) / chunks;
  double* part = nullptr;
  hipError_t e = hipMallocAsync((void**)&part, sizeof(double) * 5 * d * chunks, stream);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(col_partials_kernel, dim3(cblocks, (unsigned)chunks), dim3(256), 0, stream, X, n, d, ld, rpc, part);
  hipLaunchKernelGGL(col_fold_kernel, dim3((d + 255) / 256), dim3(256), 0, stream, part, (int)chunks, d, out);
  hipFreeAsync(part, stream);
  return (int)hipGetLastError();
}

// RawFeatureFilter statistics for numeric raw columns (reference
// RawFeatureFilter.computeFeatureStats:137-200, Summary.scala:36-66, FeatureDistribution.histValues:317-351,
// PreparedFeatures.getNullLabelLeakageVector).
//
// Columns are passed as pointer arrays (one device buffer per raw feature, no N x F staging copy):
//   vals[f]  -> values of column f, element type dtype[f] (0 f32, 1 f64, 2 i64, 3 u8/bool)
//   valid[f] -> uint8 validity (nullptr = all valid)
// Pass 1 (rff_summary): per column count, nulls, min, max, sum, sum^2, sum^3, sum^4 and sum(label*null)
//   in fp64; grid (row chunks, F), wave shuffles + LDS fold, per-chunk partials, then a fold kernel.
// Pass 2 (rff_hist): per column `bins`-bin histogram with the reference bucketing (bins-1 regular
//   buckets over [min, min + step*(bins-1)), step = (max-min)/(bins-2), Left inclusion, last bucket =
//   out of range); min == max -> 2 buckets (== max, != max). Workgroup-private LDS histogram, one
//   global atomic per non-empty LDS bin.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <float.h>

namespace {

__device__ __forceinline__ double load_val(const void* p, int dt, int64_t i) {
  switch (dt) {
    case 0: return (double)((const float*)p)[i];
    case 1: return ((const double*)p)[i];
    case 2: return (double)((const int64_t*)p)[i];
    default: return (double)((const uint8_t*)p)[i];
  }
}

constexpr int NSTAT = 9;  // count, nulls, min, max, s1, s2, s3, s4, s_label_null

__device__ __forceinline__ double wave_sum(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_min(double v) {
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

__global__ void __launch_bounds__(256) rff_summary_kernel(const void* const* __restrict__ vals,
                                                          const uint8_t* const* __restrict__ valid,
                                                          const int32_t* __restrict__ dtype, int64_t n,
                                                          int64_t rows_per_chunk, const void* __restrict__ label,
                                                          int label_dt, double* __restrict__ part) {
  const int f = blockIdx.y;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_chunk;
  const int64_t r1 = min(n, r0 + rows_per_chunk);
  const void* v = vals[f];
  const uint8_t* ok = valid[f];
  const int dt = dtype[f];
  double c = 0, nul = 0, mn = DBL_MAX, mx = -DBL_MAX, s1 = 0, s2 = 0, s3 = 0, s4 = 0, sln = 0;
  for (int64_t r = r0 + threadIdx.x; r < r1; r += blockDim.x) {
    const bool good = ok == nullptr || ok[r] != 0;
    if (good) {
      const double x = load_val(v, dt, r);
      const double x2 = x * x;
      c += 1; s1 += x; s2 += x2; s3 += x2 * x; s4 += x2 * x2;
      mn = fmin(mn, x); mx = fmax(mx, x);
    } else {
      nul += 1;
      if (label) sln += load_val(label, label_dt, r);
    }
  }
  c = wave_sum(c); nul = wave_sum(nul); s1 = wave_sum(s1); s2 = wave_sum(s2); s3 = wave_sum(s3);
  s4 = wave_sum(s4); sln = wave_sum(sln); mn = wave_min(mn); mx = wave_max(mx);
  __shared__ double sh[4][NSTAT];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh[w][0] = c; sh[w][1] = nul; sh[w][2] = mn; sh[w][3] = mx; sh[w][4] = s1;
    sh[w][5] = s2; sh[w][6] = s3; sh[w][7] = s4; sh[w][8] = sln;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = blockDim.x >> 6;
    for (int k = 1; k < nw; ++k) {
      sh[0][0] += sh[k][0]; sh[0][1] += sh[k][1]; sh[0][2] = fmin(sh[0][2], sh[k][2]);
      sh[0][3] = fmax(sh[0][3], sh[k][3]);
      for (int s = 4; s < NSTAT; ++s) sh[0][s] += sh[k][s];
    }
    double* p = part + ((int64_t)f * gridDim.x + blockIdx.x) * NSTAT;
    for (int s = 0; s < NSTAT; ++s) p[s] = sh[0][s];
  }
}

__global__ void rff_summary_fold_kernel(const double* __restrict__ part, int chunks, int F, double* __restrict__ out) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F) return;
  double acc[NSTAT] = {0, 0, DBL_MAX, -DBL_MAX, 0, 0, 0, 0, 0};
  for (int k = 0; k < chunks; ++k) {
    const double* p = part + ((int64_t)f * chunks + k) * NSTAT;
    acc[0] += p[0]; acc[1] += p[1]; acc[2] = fmin(acc[2], p[2]); acc[3] = fmax(acc[3], p[3]);
    for (int s = 4; s < NSTAT; ++s) acc[s] += p[s];
  }
  for (int s = 0; s < NSTAT; ++s) out[(int64_t)f * NSTAT + s] = acc[s];
}

__global__ void __launch_bounds__(256) rff_hist_kernel(const void* const* __restrict__ vals,
                                                       const uint8_t* const* __restrict__ valid,
                                                       const int32_t* __restrict__ dtype, int64_t n,
                                                       int64_t rows_per_chunk, const double* __restrict__ lo,
                                                       const double* __restrict__ hi, int bins,
                                                       unsigned int* __restrict__ hist) {
  extern __shared__ unsigned int lh[];
  const int f = blockIdx.y;
  const double mn = lo[f], mx = hi[f];
  const bool degenerate = !(mn < mx);
  const int nb = degenerate ? 2 : bins;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) lh[i] = 0u;
  __syncthreads();
  const double step = degenerate ? 1.0 : (mx - mn) / (bins - 2.0);
  const double top = mn + step * (bins - 1);
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_chunk;
  const int64_t r1 = min(n, r0 + rows_per_chunk);
  const void* v = vals[f];
  const uint8_t* ok = valid[f];
  const int dt = dtype[f];
  for (int64_t r = r0 + threadIdx.x; r < r1; r += blockDim.x) {
    if (ok != nullptr && ok[r] == 0) continue;
    const double x = load_val(v, dt, r);
    int b;
    if (degenerate) {
      b = (x == mx) ? 0 : 1;
    } else if (x >= mn && x < top) {
      b = (int)floor((x - mn) / step);
      if (b > bins - 2) b = bins - 2;
      // exact split comparison at bucket edges (splits are min + step * k)
      if (b > 0 && x < mn + step * b) --b;
      else if (b < bins - 2 && x >= mn + step * (b + 1)) ++b;
    } else {
      b = bins - 1;
    }
    atomicAdd(&lh[b], 1u);
  }
  __syncthreads();
  unsigned int* out = hist + (int64_t)f * bins;
  for (int i = threadIdx.x; i < nb; i += blockDim.x)
    if (lh[i]) atomicAdd(&out[i], lh[i]);
}

int chunks_for(int64_t n, int F) {
  int64_t c = (2048 + F - 1) / F;
  if (c > n / 1024 + 1) c = n / 1024 + 1;
  if (c < 1) c = 1;
  return (int)c;
}

}  // namespace

extern "C" int tmog_hip_rff_summary(const void* const* vals, const uint8_t* const* valid, const int32_t* dtype,
                                    int64_t n, int F, const void* label, int label_dt, double* out,
                                    hipStream_t stream) {
  if (F == 0) return 0;
  const int chunks = chunks_for(n, F);
  const int64_t rpc = (n + chunks - 1) / chunks;
  double* part = nullptr;
  hipError_t e = hipMallocAsync((void**)&part, sizeof(double) * NSTAT * chunks * (int64_t)F, stream);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(rff_summary_kernel, dim3(chunks, F), dim3(256), 0, stream, vals, valid, dtype, n, rpc, label,
                     label_dt, part);
  hipLaunchKernelGGL(rff_summary_fold_kernel, dim3((F + 127) / 128), dim3(128), 0, stream, part, chunks, F, out);
  hipFreeAsync(part, stream);
  return (int)hipGetLastError();
}

extern "C" int tmog_hip_rff_hist(const void* const* vals, const uint8_t* const* valid, const int32_t* dtype,
                                 int64_t n, int F, const double* lo, const double* hi, int bins,
                                 unsigned int* hist, hipStream_t stream) {
  if (F == 0 || n == 0) return 0;
  if (bins < 2 || bins > 16384) return -1;   // LDS-resident histogram limit (64 KiB)
  const int chunks = chunks_for(n, F);
  const int64_t rpc = (n + chunks - 1) / chunks;
  hipLaunchKernelGGL(rff_hist_kernel, dim3(chunks, F), dim3(256), sizeof(unsigned int) * bins, stream, vals, valid,
                     dtype, n, rpc, lo, hi, bins, hist);
  return (int)hipGetLastError();
}

// Feature binning for the tree learners on CDNA4 (gfx950): uint8 bins of a row-major fp32 design matrix.
//
// Replaces the torch chain of models/binning.quantize (transpose copy of each 1M-row chunk to [F, rows], an int64
// searchsorted, isnan / where over int64, a transposing uint8 copy back: ~25 ms and ~8 GB of traffic per chunk of
// the headline's 329 columns, ~200 ms per AutoML step) with one pass that reads X once and writes the bins once.
// Spark's tree learners bin through findSplits + TreePoint (OpRandomForestClassifier.scala:59-154 /
// OpXGBoostClassifier.scala:47-403 hist binning).
//
// Block = (64 features, 64 rows): the 64 features' sorted thresholds (padded with +inf to MS) are staged in LDS
// (row stride MS + 1, odd, so lanes of different features spread over the banks); lane = feature, so a wave's
// X loads and uint8 stores are one contiguous run of the row. bin = #(thresholds < x), exactly torch.searchsorted
// (side = "left") on the fp32 thresholds: a branch-free binary search over the padded row; NaN counts every
// threshold (searchsorted's NaN-last order), and with a reserved missing bin NaN / the missing value map to it.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

namespace {

constexpr int QF = 64;     // features per block (one per lane)
constexpr int QR = 64;     // rows per block (16 per wave)

__global__ void __launch_bounds__(256) quantize_kernel(const float* __restrict__ X, int64_t N, int F,
                                                       const float* __restrict__ thr, int MS, int top,
                                                       int missing_bin, int has_mv, float missing_value,
                                                       uint8_t* __restrict__ out) {
  extern __shared__ float t_lds[];
  const int f0 = blockIdx.y * QF;
  const int nf = min(QF, F - f0);
  const int ts = MS + 1;
  for (int i = threadIdx.x; i < nf * MS; i += blockDim.x) {
    const int f = i / MS, k = i - f * MS;
    t_lds[f * ts + k] = thr[(int64_t)(f0 + f) * MS + k];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane >= nf) return;
  const float* tf = t_lds + lane * ts;
  const int64_t r0 = (int64_t)blockIdx.x * QR;
  for (int rr = wave; rr < QR; rr += 4) {
    const int64_t r = r0 + rr;
    if (r >= N) break;
    const float x = X[r * F + f0 + lane];
    int lo = 0;
    for (int step = top; step > 0; step >>= 1) {     // largest count c <= MS with tf[c - 1] < x
      const int c = lo + step;
      if (c <= MS && tf[c - 1] < x) lo = c;
    }
    int b = isnan(x) ? MS : lo;
    if (missing_bin >= 0 && (isnan(x) || (has_mv && x == missing_value))) b = missing_bin;
    out[r * F + f0 + lane] = (uint8_t)b;
  }
}

}  // namespace

extern "C" {

// thr: [F][MS] fp32 thresholds per feature, ascending, +inf padded; out: [N][F] uint8
int tmog_hip_quantize(const float* X, int64_t N, int F, const float* thr, int MS, int missing_bin, int has_mv,
                      float missing_value, uint8_t* out, hipStream_t stream) {
  if (N == 0 || F == 0) return 0;
  if (MS < 1 || MS > 255 || F < 0) return -2;
  const size_t lds = (size_t)QF * (MS + 1) * sizeof(float);
  if (lds > 64 * 1024) return -2;
  int top = 1;
  while (top * 2 <= MS) top *= 2;
  const int64_t gx = (N + QR - 1) / QR;
  const int gy = (F + QF - 1) / QF;
  if (gx > 0x7FFFFFFF || gy > 65535) return -2;
  hipLaunchKernelGGL(quantize_kernel, dim3((unsigned)gx, (unsigned)gy), dim3(256), lds, stream, X, N, F, thr, MS, top,
                     missing_bin, has_mv, missing_value, out);
  return (int)hipGetLastError();
}

}  // extern "C"

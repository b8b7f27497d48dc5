// Fused vectorizer kernels: the layer transform of RealVectorizer /
// IntegralVectorizer / BinaryVectorizer (RealVectorizer.scala:108-119) written straight into the
// row-major feature matrix -- fill + null indicator + column->row transpose in one HBM pass.
//
// Each workgroup owns a 64-row x 32-column tile: phase 1 reads every input column with 64
// consecutive rows per wave (256 B coalesced), phase 2 writes whole 64/32-float output row
// segments through LDS (padded by one word to avoid bank conflicts on the transpose).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int TR = 64;   // rows per tile
constexpr int TC = 32;   // input columns per tile

__global__ void __launch_bounds__(256) vectorize_numeric_kernel(const float* const* __restrict__ vals,
                                                                const uint8_t* const* __restrict__ valid,
                                                                const float* __restrict__ fills, int64_t n, int F,
                                                                float* __restrict__ out, int64_t W, int track) {
  __shared__ float tile[TR][2 * TC + 1];
  const int64_t row0 = (int64_t)blockIdx.x * TR;
  const int c0 = blockIdx.y * TC;
  const int per = track ? 2 : 1;
  for (int k = threadIdx.x; k < TR * TC; k += blockDim.x) {
    const int r = k % TR, cj = k / TR, c = c0 + cj;
    const int64_t row = row0 + r;
    if (c < F && row < n) {
      const bool ok = valid[c][row] != 0;
      const float v = ok ? vals[c][row] : fills[c];
      tile[r][per * cj] = v;
      if (track) tile[r][per * cj + 1] = ok ? 0.f : 1.f;
    }
  }
  __syncthreads();
  const int ncols = min(TC, F - c0) * per;
  for (int k = threadIdx.x; k < TR * TC * per; k += blockDim.x) {
    const int r = k / (TC * per), oc = k % (TC * per);
    const int64_t row = row0 + r;
    if (oc < ncols && row < n) out[row * W + (int64_t)c0 * per + oc] = tile[r][oc];
  }
}

// One-hot pivot of several categorical columns at once (OpOneHotVectorizer transform,
// OpOneHotVectorizer.scala:416-437): column c maps dictionary code -> slot through lut[c]
// (code -1 = missing uses the lut's last entry, slot -1 = no output), writing 1.0 at
// out[row, off[c] + slot]. out is zero-initialised by the caller; each (row, column) writes at most
// one element, so plain stores suffice. grid.y = column.
__global__ void __launch_bounds__(256) onehot_pivot_kernel(const int32_t* const* __restrict__ codes,
                                                           const int32_t* const* __restrict__ luts,
                                                           const int32_t* __restrict__ lut_n,
                                                           const int64_t* __restrict__ off, int64_t n,
                                                           float* __restrict__ out, int64_t W) {
  const int c = blockIdx.y;
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const int32_t code = codes[c][r];
  const int32_t ln = lut_n[c];
  const int32_t slot = luts[c][(code >= 0 && code < ln - 1) ? code : ln - 1];
  if (slot >= 0) out[r * W + off[c] + slot] = 1.f;
}

// Row x column gather from a blocked feature matrix (the SanityChecker keep-mask and
// the VectorsCombiner concatenation applied lazily): out[r, j] = col_base[j][row(r) * col_ld[j]] with
// row(r) = rows ? rows[r] : r. A workgroup covers 64 output columns x 32 rows; each lane keeps its
// column's base / stride in registers and walks 8 rows, so one wave reads 64 adjacent source words of
// a row (same block) and writes 256 B of the output row.
constexpr int kGatherRows = 32;

__global__ void __launch_bounds__(256) gather_rows_cols_kernel(const float* const* __restrict__ col_base,
                                                               const int64_t* __restrict__ col_ld,
                                                               const int64_t* __restrict__ rows, int64_t m, int k,
                                                               float* __restrict__ out) {
  const int j = blockIdx.y * 64 + (threadIdx.x & 63);
  if (j >= k) return;
  const float* base = col_base[j];
  const int64_t ld = col_ld[j];
  const int64_t r0 = (int64_t)blockIdx.x * kGatherRows + (threadIdx.x >> 6);
  // all row ids, then all values, then the stores: independent loads in flight instead of a chain of
  // (row id -> value) latencies per row
  constexpr int NR = kGatherRows / 4;
  int64_t src[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int64_t r = min(r0 + 4 * i, m - 1);
    src[i] = rows ? rows[r] : r;
  }
  float v[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) v[i] = base[src[i] * ld];
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int64_t r = r0 + 4 * i;
    if (r < m) out[r * k + j] = v[i];
  }
}

// Masked column sums of many columns in one launch (RealVectorizer fill-with-mean, RealVectorizer.scala:82-86:
// the mean of every column's non-null values). grid = (row chunks, columns); column c is fp32 (dtype 0) or fp64
// (1), its validity bytes optional (null = all valid). Each thread keeps 4 independent row loads in flight per
// step (rows r, r + 256, ...: every wave reads 256 B / 512 B runs), sums in fp64; the block's (sum, count)
// goes to part[c][chunk] and the chunks are folded by the caller in a fixed order.
constexpr int kSumUnroll = 4;

__global__ void __launch_bounds__(256) masked_colsum_kernel(const void* const* __restrict__ vals,
                                                            const uint8_t* const* __restrict__ valid,
                                                            const int32_t* __restrict__ dtype, int64_t n,
                                                            int64_t rows_per_chunk, double* __restrict__ part) {
  const int c = blockIdx.y;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_chunk;
  const int64_t r1 = min(n, r0 + rows_per_chunk);
  const uint8_t* ok = valid[c];
  const bool f64 = dtype[c] == 1;
  const float* vf = (const float*)vals[c];
  const double* vd = (const double*)vals[c];
  double s = 0.0, k = 0.0;
  for (int64_t base = r0 + threadIdx.x; base < r1; base += 256 * kSumUnroll) {
    double v[kSumUnroll];
    bool m[kSumUnroll];
#pragma unroll
    for (int u = 0; u < kSumUnroll; ++u) {
      const int64_t r = base + 256 * u;
      const int64_t rc = min(r, r1 - 1);          // clamped, loads issued together; masked below
      v[u] = f64 ? vd[rc] : (double)vf[rc];
      m[u] = r < r1 && (ok == nullptr || ok[rc] != 0);
    }
#pragma unroll
    for (int u = 0; u < kSumUnroll; ++u)
      if (m[u]) {
        s += v[u];
        k += 1.0;
      }
  }
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o, 64);
    k += __shfl_xor(k, o, 64);
  }
  __shared__ double sh[2][4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh[0][w] = s;
    sh[1][w] = k;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double* o = part + ((int64_t)c * gridDim.x + blockIdx.x) * 2;
    o[0] = (sh[0][0] + sh[0][1]) + (sh[0][2] + sh[0][3]);
    o[1] = (sh[1][0] + sh[1][1]) + (sh[1][2] + sh[1][3]);
  }
}

}  // namespace

extern "C" {

// part [n_cols][chunks][2] fp64 (sum, count) partials; chunks = ceil(n / rows_per_chunk).
int tmog_hip_masked_colsum(const void* vals, const void* valid, const int32_t* dtype, int n_cols, int64_t n,
                           int64_t rows_per_chunk, double* part, hipStream_t stream) {
  if (n <= 0 || n_cols <= 0) return 0;
  if (rows_per_chunk <= 0) return -1;
  const int64_t chunks = (n + rows_per_chunk - 1) / rows_per_chunk;
  if (chunks > (1 << 20) || n_cols > 65535) return -2;
  hipLaunchKernelGGL(masked_colsum_kernel, dim3((unsigned)chunks, (unsigned)n_cols), dim3(256), 0, stream,
                     (const void* const*)vals, (const uint8_t* const*)valid, dtype, n, rows_per_chunk, part);
  return (int)hipGetLastError();
}

int tmog_hip_gather_rows_cols(const void* col_base, const int64_t* col_ld, const int64_t* rows, int64_t m, int k,
                              float* out, hipStream_t stream) {
  if (m == 0 || k == 0) return 0;
  dim3 grid((unsigned)((m + kGatherRows - 1) / kGatherRows), (unsigned)((k + 63) / 64));
  hipLaunchKernelGGL(gather_rows_cols_kernel, grid, dim3(256), 0, stream, (const float* const*)col_base, col_ld, rows,
                     m, k, out);
  return (int)hipGetLastError();
}

int tmog_hip_onehot_pivot(const void* codes, const void* luts, const int32_t* lut_n, const int64_t* off, int n_cols,
                          int64_t n, float* out, int64_t W, hipStream_t stream) {
  if (n == 0 || n_cols == 0) return 0;
  dim3 grid((unsigned)((n + 255) / 256), (unsigned)n_cols);
  hipLaunchKernelGGL(onehot_pivot_kernel, grid, dim3(256), 0, stream, (const int32_t* const*)codes,
                     (const int32_t* const*)luts, lut_n, off, n, out, W);
  return (int)hipGetLastError();
}

int tmog_hip_vectorize_numeric(const void* vals, const void* valid, const float* fills, int64_t n, int F,
                               const void* r1, const void* r2, const void* r3, float* out, int64_t W, int track,
                               hipStream_t stream) {
  (void)r1; (void)r2; (void)r3;
  if (n == 0 || F == 0) return 0;
  dim3 grid((unsigned)((n + TR - 1) / TR), (unsigned)((F + TC - 1) / TC));
  hipLaunchKernelGGL(vectorize_numeric_kernel, grid, dim3(256), 0, stream, (const float* const*)vals,
                     (const uint8_t* const*)valid, fills, n, F, out, W, track);
  return (int)hipGetLastError();
}

}  // extern "C"

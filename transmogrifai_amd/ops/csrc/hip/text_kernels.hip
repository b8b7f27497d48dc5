// Text / categorical / calendar vectorizer kernels.
//
// * hash_tokens_kernel  -- Spark HashingTF index of every token: nonNegativeMod(murmur3_x86_32(
//   prefix || token, 42), numFeatures) with Spark's signed-byte tail mixing
//   (OPCollectionHashingVectorizer.scala:204-208, 284-305; bit-identical to host hashing_cpu.cpp).
//   One lane per token; the feature-name prefix is concatenated virtually (no string rebuild).
// * hash_tf_rows_kernel -- term-frequency rows written straight into the feature matrix: one wave
//   per row accumulates its tokens' indices in a private LDS count row (ds_add_u32), then writes the
//   whole W-wide row segment coalesced (64 lanes x 4 B). Rows reach their tokens through dictionary
//   codes (row -> distinct value -> token range), so a repeated value is tokenized once.
// * code_count_kernel   -- value counts of dictionary-coded columns (one-hot / SmartText fit,
//   integral mode): LDS-privatised histograms flushed with one 64-bit global atomic per bin.
// * bucketize_kernel    -- NumericBucketizer binary search + one-hot write (NumericBucketizer.scala:219-265).
// * date_unit_circle_kernel -- DateToUnitCircleTransformer (cos, sin) of a UTC calendar period
//   (DateToUnitCircleTransformer.scala:77-121), integer civil-date arithmetic on device.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

struct Prefix {
  uint8_t b[24];
  int32_t len;
};

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ uint32_t mix_k1(uint32_t k1) {
  k1 *= 0xcc9e2d51u;
  k1 = rotl32(k1, 15);
  return k1 * 0x1b873593u;
}
__device__ __forceinline__ uint32_t mix_h1(uint32_t h1, uint32_t k1) {
  h1 ^= k1;
  h1 = rotl32(h1, 13);
  return h1 * 5u + 0xe6546b64u;
}

__global__ void __launch_bounds__(256) hash_tokens_kernel(const uint8_t* __restrict__ data,
                                                          const int64_t* __restrict__ tok_offs, int64_t T,
                                                          Prefix pre, int32_t seed, int32_t num_features,
                                                          int32_t base, int32_t* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  const int64_t s = tok_offs[t];
  const int64_t len = (int64_t)pre.len + (tok_offs[t + 1] - s);
  const uint8_t* tok = data + s;
  auto at = [&](int64_t k) -> uint32_t { return k < pre.len ? pre.b[k] : tok[k - pre.len]; };
  uint32_t h1 = (uint32_t)seed;
  const int64_t aligned = len - (len & 3);
  for (int64_t i = 0; i < aligned; i += 4)
    h1 = mix_h1(h1, mix_k1(at(i) | (at(i + 1) << 8) | (at(i + 2) << 16) | (at(i + 3) << 24)));
  for (int64_t i = aligned; i < len; ++i) h1 = mix_h1(h1, mix_k1((uint32_t)(int32_t)(int8_t)at(i)));
  h1 ^= (uint32_t)len;
  h1 ^= h1 >> 16;
  h1 *= 0x85ebca6bu;
  h1 ^= h1 >> 13;
  h1 *= 0xc2b2ae35u;
  h1 ^= h1 >> 16;
  int32_t m = (int32_t)h1 % num_features;
  out[t] = (m < 0 ? m + num_features : m) + base;
}

struct HashFeat {
  const int32_t* codes;    // row -> distinct-value code (-1 = null); nullptr = identity
  const int64_t* row_ptr;  // code -> token range
  const int32_t* idx;      // token -> column inside the W-wide block
};

constexpr int kRowsPerBlock = 4;  // one wave per row

__global__ void __launch_bounds__(256) hash_tf_rows_kernel(const HashFeat* __restrict__ feats, int n_feats,
                                                           int64_t n, int W, int binary, float* __restrict__ out,
                                                           int64_t ld, int64_t off) {
  extern __shared__ uint32_t cnt_all[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t* cnt = cnt_all + (size_t)wave * W;
  for (int64_t r0 = (int64_t)blockIdx.x * kRowsPerBlock; r0 < n; r0 += (int64_t)gridDim.x * kRowsPerBlock) {
    const int64_t r = r0 + wave;
    for (int j = lane; j < W; j += 64) cnt[j] = 0u;
    __syncthreads();
    if (r < n) {
      for (int f = 0; f < n_feats; ++f) {
        const HashFeat hf = feats[f];
        const int64_t code = hf.codes ? (int64_t)hf.codes[r] : r;
        if (code < 0) continue;
        const int64_t a = hf.row_ptr[code], b = hf.row_ptr[code + 1];
        for (int64_t t = a + lane; t < b; t += 64) atomicAdd(&cnt[hf.idx[t]], 1u);
      }
    }
    __syncthreads();
    if (r < n) {
      float* dst = out + r * ld + off;
      for (int j = lane; j < W; j += 64) {
        const uint32_t c = cnt[j];
        dst[j] = binary ? (c ? 1.f : 0.f) : (float)c;
      }
    }
    __syncthreads();
  }
}

// Wide hash spaces (W beyond the LDS row budget): global float atomics into a zeroed block.
__global__ void __launch_bounds__(256) hash_tf_rows_global_kernel(const HashFeat* __restrict__ feats, int n_feats,
                                                                  int64_t n, int binary, float* __restrict__ out,
                                                                  int64_t ld, int64_t off) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * kRowsPerBlock + wave;
  if (r >= n) return;
  float* dst = out + r * ld + off;
  for (int f = 0; f < n_feats; ++f) {
    const HashFeat hf = feats[f];
    const int64_t code = hf.codes ? (int64_t)hf.codes[r] : r;
    if (code < 0) continue;
    const int64_t a = hf.row_ptr[code], b = hf.row_ptr[code + 1];
    for (int64_t t = a + lane; t < b; t += 64) {
      if (binary) dst[hf.idx[t]] = 1.f;
      else atomicAdd(&dst[hf.idx[t]], 1.f);
    }
  }
}

// counts[c][v] += #rows with codes[c][row] == v; code -1 (null) counts into slot nv[c].
__global__ void __launch_bounds__(256) code_count_kernel(const int32_t* const* __restrict__ codes,
                                                         const int32_t* __restrict__ nv, int64_t n,
                                                         unsigned long long* const* __restrict__ counts,
                                                         int use_lds) {
  extern __shared__ uint32_t h[];
  const int c = blockIdx.y;
  const int V = nv[c] + 1;
  const int32_t* cc = codes[c];
  unsigned long long* gc = counts[c];
  if (use_lds) {
    for (int j = threadIdx.x; j < V; j += blockDim.x) h[j] = 0u;
    __syncthreads();
  }
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    int32_t v = cc[r];
    v = (v < 0 || v >= V - 1) ? V - 1 : v;
    if (use_lds) atomicAdd(&h[v], 1u);
    else atomicAdd(&gc[v], 1ull);
  }
  if (use_lds) {
    __syncthreads();
    for (int j = threadIdx.x; j < V; j += blockDim.x)
      if (h[j]) atomicAdd(&gc[j], (unsigned long long)h[j]);
  }
}

// One-hot bucket index by binary search over `ns` sorted splits (ns - 1 buckets). left_incl: splits[i] <= x <
// splits[i+1], else splits[i] < x <= splits[i+1]. Invalid (out of range / non-finite) valid values go to the
// slot after the buckets when track_invalid, else raise `bad` (first offending row). Nulls -> last slot when
// track_nulls. `out` is zero-initialised.
__global__ void __launch_bounds__(256) bucketize_kernel(const double* __restrict__ x, const uint8_t* __restrict__ ok,
                                                        int64_t n, const double* __restrict__ splits, int ns,
                                                        int left_incl, int track_invalid, int track_nulls,
                                                        float* __restrict__ out, int64_t ld, int64_t off, int width,
                                                        unsigned long long* __restrict__ bad) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  float* dst = out + r * ld + off;
  if (!ok[r]) {
    if (track_nulls) dst[width - 1] = 1.f;
    return;
  }
  const double v = x[r];
  // searchsorted: left_incl -> first index with splits[i] > v (right=True); else first with splits[i] >= v
  int lo = 0, hi = ns;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    const bool go_right = left_incl ? (splits[mid] <= v) : (splits[mid] < v);
    if (go_right) lo = mid + 1;
    else hi = mid;
  }
  const int b = lo - 1;
  const bool finite = v == v && v != __longlong_as_double(0x7ff0000000000000LL) &&
                      v != __longlong_as_double((long long)0xfff0000000000000ULL);
  if (b >= 0 && b < ns - 1 && finite) {
    dst[b] = 1.f;
  } else if (track_invalid) {
    dst[ns - 1] = 1.f;
  } else {
    atomicMin(bad, (unsigned long long)r);
  }
}

__device__ __forceinline__ int64_t fdiv(int64_t a, int64_t b) {
  const int64_t q = a / b;
  return (a % b != 0 && ((a < 0) != (b < 0))) ? q - 1 : q;
}

__device__ __forceinline__ int64_t dow(int64_t days) {  // Monday = 1; 1970-01-01 was a Thursday
  int64_t m = (days + 3) % 7;
  if (m < 0) m += 7;
  return m + 1;
}

// period: 0 DayOfMonth, 1 DayOfWeek, 2 DayOfYear, 3 HourOfDay, 4 MonthOfYear, 5 WeekOfMonth, 6 WeekOfYear.
__device__ int64_t period_field(int64_t ms, int period) {
  const int64_t days = fdiv(ms, 86400000LL);
  if (period == 3) return fdiv(ms - days * 86400000LL, 3600000LL);
  if (period == 1) return dow(days);
  const int64_t z = days + 719468;
  const int64_t era = fdiv(z, 146097);
  const int64_t doe = z - era * 146097;
  const int64_t yoe = fdiv(doe - fdiv(doe, 1460) + fdiv(doe, 36524) - fdiv(doe, 146096), 365);
  int64_t y = yoe + era * 400;
  const int64_t doy0 = doe - (365 * yoe + fdiv(yoe, 4) - fdiv(yoe, 100));
  const int64_t mp = fdiv(5 * doy0 + 2, 153);
  const int64_t d = doy0 - fdiv(153 * mp + 2, 5) + 1;
  const int64_t m = mp < 10 ? mp + 3 : mp - 9;
  y += (m <= 2);
  if (period == 0) return d;
  if (period == 4) return m;
  const bool leap = ((y % 4 == 0) && (y % 100 != 0)) || (y % 400 == 0);
  // doy0 counts days from March 1st: March..December follow January + February
  const int64_t doy = m >= 3 ? doy0 + 60 + (leap ? 1 : 0) : doy0 - 305;
  if (period == 2) return doy;
  if (period == 6) return fdiv(doy - 1 + dow(days - (doy - 1)) - 1, 7) + 1;
  return fdiv(d - 1 + dow(days - (d - 1)) - 1, 7) + 1;  // WeekOfMonth
}

// (cos, sin)(2 pi v / size) for valid rows (v zero-based when the period starts at 1), (0, 0) for nulls.
__global__ void __launch_bounds__(256) date_unit_circle_kernel(const int64_t* __restrict__ ms,
                                                               const uint8_t* __restrict__ ok, int64_t n, int period,
                                                               int zero_based_shift, int size,
                                                               float* __restrict__ out, int64_t ld, int64_t off) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  float* dst = out + r * ld + off;
  if (!ok[r]) {
    dst[0] = 0.f;
    dst[1] = 0.f;
    return;
  }
  const int64_t v = period_field(ms[r], period) - zero_based_shift;
  const double rad = 2.0 * 3.141592653589793 * (double)v / (double)size;
  dst[0] = (float)cos(rad);
  dst[1] = (float)sin(rad);
}

}  // namespace

extern "C" {

int tmog_hip_hash_tokens(const uint8_t* data, const int64_t* tok_offs, int64_t T, const uint8_t* prefix,
                         int32_t plen, int32_t seed, int32_t num_features, int32_t base, int32_t* out,
                         hipStream_t stream) {
  if (T == 0) return 0;
  if (plen < 0 || plen > 24 || num_features <= 0) return -1;
  Prefix p{};
  for (int i = 0; i < plen; ++i) p.b[i] = prefix[i];
  p.len = plen;
  hipLaunchKernelGGL(hash_tokens_kernel, dim3((unsigned)((T + 255) / 256)), dim3(256), 0, stream, data, tok_offs, T,
                     p, seed, num_features, base, out);
  return (int)hipGetLastError();
}

int tmog_hip_hash_tf_rows(const void* feats, int n_feats, int64_t n, int W, int binary, float* out, int64_t ld,
                          int64_t off, hipStream_t stream) {
  if (n == 0 || n_feats == 0 || W == 0) return 0;
  const size_t lds = (size_t)kRowsPerBlock * W * sizeof(uint32_t);
  if (lds <= 64 * 1024) {
    const int64_t blocks = (n + kRowsPerBlock - 1) / kRowsPerBlock;
    const unsigned grid = (unsigned)(blocks < 16384 ? blocks : 16384);
    hipLaunchKernelGGL(hash_tf_rows_kernel, dim3(grid), dim3(256), lds, stream, (const HashFeat*)feats, n_feats, n,
                       W, binary, out, ld, off);
  } else {
    hipLaunchKernelGGL(hash_tf_rows_global_kernel, dim3((unsigned)((n + kRowsPerBlock - 1) / kRowsPerBlock)),
                       dim3(256), 0, stream, (const HashFeat*)feats, n_feats, n, binary, out, ld, off);
  }
  return (int)hipGetLastError();
}

int tmog_hip_hash_feat_bytes() { return (int)sizeof(HashFeat); }

int tmog_hip_code_count(const void* codes, const int32_t* nv, int max_v, int n_cols, int64_t n, void* counts,
                        hipStream_t stream) {
  if (n == 0 || n_cols == 0) return 0;
  const size_t lds = (size_t)(max_v + 1) * sizeof(uint32_t);
  const int use_lds = lds <= 48 * 1024;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(code_count_kernel, dim3((unsigned)blocks, (unsigned)n_cols), dim3(256), use_lds ? lds : 0,
                     stream, (const int32_t* const*)codes, nv, n, (unsigned long long* const*)counts, use_lds);
  return (int)hipGetLastError();
}

int tmog_hip_bucketize(const double* x, const uint8_t* ok, int64_t n, const double* splits, int ns, int left_incl,
                       int track_invalid, int track_nulls, float* out, int64_t ld, int64_t off, int width,
                       unsigned long long* bad, hipStream_t stream) {
  if (n == 0) return 0;
  if (ns < 2) return -1;
  hipLaunchKernelGGL(bucketize_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, x, ok, n, splits, ns,
                     left_incl, track_invalid, track_nulls, out, ld, off, width, bad);
  return (int)hipGetLastError();
}

int tmog_hip_date_unit_circle(const int64_t* ms, const uint8_t* ok, int64_t n, int period, int shift, int size,
                              float* out, int64_t ld, int64_t off, hipStream_t stream) {
  if (n == 0) return 0;
  if (period < 0 || period > 6 || size <= 0) return -1;
  hipLaunchKernelGGL(date_unit_circle_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, ms, ok, n,
                     period, shift, size, out, ld, off);
  return (int)hipGetLastError();
}

}  // extern "C"

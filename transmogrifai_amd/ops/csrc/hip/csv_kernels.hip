// CSV parsing on the device (readers/gpu_csv.py; the reference's default readers are CSV: CSVReaders.scala:54-122,
// DataReader.scala:173-197). The host only moves raw bytes: file chunks are read into pinned buffers and copied to
// the device, where
//   csv_fields_kernel   one wave per row walks the row in 64-byte windows (coalesced loads), finds the separators
//                       outside double quotes with two ballots (the quote parity of each lane is the popcount of
//                       the quotes below it) and writes every field's start offset;
//   csv_parse_num       one thread per (row, column): the field as a float64 or int64 with a validity byte --
//                       pandas' NA strings and empty cells are missing; decimal strings of at most 19 significant
//                       digits with |exponent| <= 22 convert exactly (one IEEE multiply or divide of two exact
//                       doubles: the correctly rounded result), anything else is flagged for the host parser;
//   csv_hash_text       one thread per (row, column): a 64-bit hash of the unquoted field bytes (0 = missing), the
//                       input of the device dictionary encoding (torch.unique + first appearance).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__device__ __forceinline__ uint64_t lanes_below(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

// buf: the chunk's bytes; row_start[r] .. row_end[r] (exclusive, the '\n' or the chunk end) are row r's bytes (a
// trailing '\r' is dropped). fstart[r * (ncols + 1) + k] = absolute offset of field k, fstart[.. + nf] = end + 1 (so
// field k is [fstart[k], fstart[k + 1] - 1)); nfields[r] = number of fields (fields past ncols are not recorded).
__global__ void __launch_bounds__(256) csv_fields_kernel(const uint8_t* __restrict__ buf,
                                                         const int64_t* __restrict__ row_start,
                                                         const int64_t* __restrict__ row_end, int64_t nrows,
                                                         int ncols, int sep, int64_t* __restrict__ fstart,
                                                         int32_t* __restrict__ nfields) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= nrows) return;
  const int64_t b0 = row_start[r];
  int64_t e = row_end[r];
  if (e > b0 && buf[e - 1] == '\r') --e;
  int64_t* fs = fstart + r * (int64_t)(ncols + 1);
  if (lane == 0) fs[0] = b0;
  int nf = 1;                   // fields so far (wave-uniform)
  int quote = 0;                // quote parity carried from the previous windows
  for (int64_t p = b0; p < e; p += 64) {
    const int64_t q = p + lane;
    const uint8_t c = q < e ? buf[q] : 0;
    const uint64_t qm = __ballot(c == '"');
    const int inq = (quote + __popcll(qm & lanes_below(lane))) & 1;
    const bool is_sep = c == (uint8_t)sep && !inq && q < e;
    const uint64_t sm = __ballot(is_sep);
    if (is_sep) {
      const int k = nf + __popcll(sm & lanes_below(lane));
      if (k <= ncols - 1) fs[k] = q + 1;
    }
    nf += __popcll(sm);
    quote = (quote + __popcll(qm)) & 1;
  }
  if (lane == 0) {
    fs[min(nf, ncols)] = e + 1;
    nfields[r] = nf;
  }
}

__device__ __forceinline__ bool is_space(uint8_t c) { return c == ' ' || c == '\t'; }

// pandas.read_csv's default NA strings (readers/columnar.py _PANDAS_NA), compared on the trimmed, unquoted field
__device__ bool is_na(const uint8_t* s, int n) {
  if (n == 0) return true;
  if (n > 8) return false;
  const uint8_t c0 = s[0];              // every NA string starts with one of these
  if (!(c0 == '#' || c0 == '-' || c0 == '1' || c0 == '<' || c0 == 'N' || c0 == 'n')) return false;
  char t[9];
  for (int i = 0; i < n; ++i) t[i] = (char)s[i];
  t[n] = 0;
  const char* na[] = {"#N/A", "#N/A N/A", "#NA", "-1.#IND", "-1.#QNAN", "-NaN", "-nan", "1.#IND", "1.#QNAN", "<NA>",
                      "N/A", "NA", "NULL", "NaN", "None", "n/a", "nan", "null"};
  for (int k = 0; k < 18; ++k) {
    const char* a = na[k];
    int i = 0;
    while (i < n && a[i] && a[i] == t[i]) ++i;
    if (i == n && a[i] == 0) return true;
  }
  return false;
}

// the field's trimmed, unquoted byte range
__device__ __forceinline__ void field_range(const uint8_t* buf, const int64_t* fs, int nf, int col, int64_t* a,
                                            int64_t* b) {
  if (col >= nf) {
    *a = *b = 0;
    return;
  }
  int64_t s = fs[col], t = fs[col + 1] - 1;
  while (s < t && is_space(buf[s])) ++s;
  while (t > s && is_space(buf[t - 1])) --t;
  if (t - s >= 2 && buf[s] == '"' && buf[t - 1] == '"') {
    ++s;
    --t;
  }
  *a = s;
  *b = t;
}

__constant__ double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                  1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// One (row, column) per thread, row-major: the threads of a wave read one row's consecutive field offsets and bytes.
// cols[j] = CSV column of output j; kind[j] = 0 float64, 1 int64. out[r * nout + j] (as double or int64 bits),
// valid[r * nout + j]; slow[r * nout + j] = 1 when the host must parse the field (the host transposes the tile to
// column-major). A field that does not parse as a number is checked against the NA strings only then.
__global__ void __launch_bounds__(256) csv_parse_num_kernel(const uint8_t* __restrict__ buf,
                                                            const int64_t* __restrict__ fstart,
                                                            const int32_t* __restrict__ nfields, int64_t nrows,
                                                            int ncols, const int32_t* __restrict__ cols,
                                                            const int32_t* __restrict__ kind, int nout,
                                                            int64_t* __restrict__ out, uint8_t* __restrict__ valid,
                                                            uint8_t* __restrict__ slow) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nrows * nout) return;
  const int64_t r = i / nout;
  const int j = (int)(i - r * nout);
  const int64_t o = i;
  int64_t a, b;
  field_range(buf, fstart + r * (int64_t)(ncols + 1), nfields[r], cols[j], &a, &b);
  const uint8_t* s = buf + a;
  const int n = (int)(b - a);
  slow[o] = 0;
  if (n == 0) {
    valid[o] = 0;
    out[o] = 0;
    return;
  }
  int k = 0;
  bool neg = false;
  if (s[k] == '+' || s[k] == '-') neg = s[k++] == '-';
  uint64_t m = 0;
  int nd = 0, e10 = 0;
  bool any = false, dot = false, bad = false;
  for (; k < n; ++k) {
    const uint8_t c = s[k];
    if (c >= '0' && c <= '9') {
      any = true;
      if (m == 0 && c == '0') {         // leading zeros do not count as significant digits
        if (dot) --e10;
        continue;
      }
      if (nd < 19) {
        m = m * 10 + (c - '0');
        ++nd;
        if (dot) --e10;
      } else {
        bad = bad || c != '0';          // a 20th significant digit that matters: host
        if (!dot) ++e10;
      }
    } else if (c == '.' && !dot) {
      dot = true;
    } else {
      break;
    }
  }
  if (k < n && (s[k] == 'e' || s[k] == 'E') && any) {
    ++k;
    bool eneg = false;
    if (k < n && (s[k] == '+' || s[k] == '-')) eneg = s[k++] == '-';
    int ev = 0;
    bool edig = false;
    for (; k < n && s[k] >= '0' && s[k] <= '9'; ++k) {
      edig = true;
      ev = min(ev * 10 + (s[k] - '0'), 100000);
    }
    bad = bad || !edig;
    e10 += eneg ? -ev : ev;
  }
  if (!any || k != n) {                 // not a plain decimal: an NA string is missing, anything else (inf,
    if (is_na(s, n)) {                  // hex, stray characters) goes to the host parser
      valid[o] = 0;
      out[o] = 0;
      return;
    }
    bad = true;
  }
  if (kind[j] == 1) {                   // int64: an integer literal (a ".0" fraction is accepted)
    if (bad || e10 < 0 || nd + e10 > 18) {
      slow[o] = 1;
      valid[o] = 0;
      out[o] = 0;
      return;
    }
    int64_t v = (int64_t)m;
    for (int t = 0; t < e10; ++t) v *= 10;
    out[o] = neg ? -v : v;
    valid[o] = 1;
    return;
  }
  double v;
  if (!bad && m == 0) {
    v = 0.0;
  } else if (!bad && m < (1ull << 53) && e10 >= -22 && e10 <= 22) {
    const double dm = (double)m;        // exact
    v = e10 >= 0 ? dm * kPow10[e10] : dm / kPow10[-e10];     // one correctly rounded IEEE operation
  } else {
    slow[o] = 1;
    valid[o] = 0;
    out[o] = 0;
    return;
  }
  v = neg ? -v : v;
  out[o] = __double_as_longlong(v);
  valid[o] = 1;
}

// 64-bit FNV-1a of the unquoted field (""-escapes kept as written: equal strings hash equally), 0 for missing.
__global__ void __launch_bounds__(256) csv_hash_text_kernel(const uint8_t* __restrict__ buf,
                                                            const int64_t* __restrict__ fstart,
                                                            const int32_t* __restrict__ nfields, int64_t nrows,
                                                            int ncols, const int32_t* __restrict__ cols, int nout,
                                                            uint64_t* __restrict__ hash, int64_t* __restrict__ span) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nrows * nout) return;
  const int64_t r = i / nout;           // row-major as csv_parse_num: out[r * nout + j]
  const int j = (int)(i - r * nout);
  const int64_t o = i;
  int64_t a, b;
  field_range(buf, fstart + r * (int64_t)(ncols + 1), nfields[r], cols[j], &a, &b);
  span[2 * o] = a;
  span[2 * o + 1] = b;
  if (is_na(buf + a, (int)(b - a))) {
    hash[o] = 0;
    return;
  }
  uint64_t h = 1469598103934665603ull;
  for (int64_t p = a; p < b; ++p) {
    h ^= buf[p];
    h *= 1099511628211ull;
  }
  hash[o] = h ? h : 1;                  // 0 is reserved for missing
}

}  // namespace

extern "C" {

int tmog_hip_csv_fields(const uint8_t* buf, const int64_t* row_start, const int64_t* row_end, int64_t nrows,
                        int ncols, int sep, int64_t* fstart, int32_t* nfields, hipStream_t stream) {
  if (nrows <= 0) return 0;
  if (ncols < 1) return -2;
  const int64_t blocks = (nrows + 3) / 4;   // 4 waves (rows) per workgroup
  hipLaunchKernelGGL(csv_fields_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, buf, row_start, row_end, nrows,
                     ncols, sep, fstart, nfields);
  return (int)hipGetLastError();
}

int tmog_hip_csv_parse_num(const uint8_t* buf, const int64_t* fstart, const int32_t* nfields, int64_t nrows, int ncols,
                           const int32_t* cols, const int32_t* kind, int nout, int64_t* out, uint8_t* valid,
                           uint8_t* slow, hipStream_t stream) {
  const int64_t n = nrows * (int64_t)nout;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(csv_parse_num_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, buf, fstart,
                     nfields, nrows, ncols, cols, kind, nout, out, valid, slow);
  return (int)hipGetLastError();
}

int tmog_hip_csv_hash_text(const uint8_t* buf, const int64_t* fstart, const int32_t* nfields, int64_t nrows,
                           int ncols, const int32_t* cols, int nout, uint64_t* hash, int64_t* span,
                           hipStream_t stream) {
  const int64_t n = nrows * (int64_t)nout;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(csv_hash_text_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, buf, fstart,
                     nfields, nrows, ncols, cols, nout, hash, span);
  return (int)hipGetLastError();
}

}  // extern "C"

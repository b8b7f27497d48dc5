// Exact areas under the PR and ROC curves of J score sets over the same labelled rows (the model
// selector's BinaryClassificationEvaluator metric, Spark BinaryClassificationMetrics with numBins = 0, as
// OpBinaryClassificationEvaluator.scala:67-135 computes it).
//
// Input: every score set sorted descending (the caller's flat radix sorts: segment-major, stable), the source
// column of every sorted element and the rows' 0/1 labels. Each score set is cut into chunks of 64 slabs of 1024
// elements, one workgroup per (set, chunk); in a slab a block scan of the (positive, negative) counts gives the
// cumulative confusion counts, the curve points are the run ends (the last element of every run of equal scores),
// and each run end adds its trapezoid against the previous run end -- inside the slab from an exclusive max-scan
// of the end positions, across slabs from the carried counts, across chunks from a first pass of per-chunk
// summaries. With P positives and N negatives:
//   AuPR  = (1 / P)     * sum_ends (tp - tp') * (prec + prec') / 2     (curve starts at (0, precision of end 1))
//   AuROC = (1 / (P N)) * sum_ends (fp - fp') * (tp + tp') / 2         ((0, 0) first; the end point is (1, 1))
// exactly the points of evaluators/metrics.py binary_curves, accumulated in fp64 in a fixed order (deterministic).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int NT = 1024;
constexpr int NW = NT / 64;

__device__ __forceinline__ int wave_incl_sum(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  return v;
}

__device__ __forceinline__ int wave_incl_max(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(v, o, 64);
    if (lane >= o) v = max(v, u);
  }
  return v;
}

// Chunk summary (pass 1, grid J x C): positives and negatives of the chunk, and the chunk-local cumulative counts at
// its last run end (-1 when the chunk holds none). A run end at a chunk's last element looks at the next chunk's
// first score, so chunks never need each other's data beyond that one element.
struct ChunkSum {
  int64_t pos, neg, end_tp, end_fp;
};

template <typename T>
__device__ __forceinline__ bool run_end(const T* ss, int64_t i, int64_t n) {
  return i == n - 1 || ss[i + 1] != ss[i];
}

// one 1024-element slab: block scans of the counts (sum) and of the last end position (max); returns this
// thread's inclusive counts and fills s_cp / s_cn / s_last
template <typename T>
__device__ __forceinline__ void slab_scan(const T* ss, const int64_t* ii, const uint8_t* lab, int64_t i, int64_t hi,
                                          int64_t n, int* s_cp, int* s_cn, int* s_last, int* w_p, int* w_n, int* w_m,
                                          int& cp, int& cn, bool& end) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const bool v = i < hi;
  const int pos = v ? (int)(lab[ii[i]] != 0) : 0;
  const int neg = v ? 1 - pos : 0;
  end = v && run_end(ss, i, n);
  cp = wave_incl_sum(pos);
  cn = wave_incl_sum(neg);
  int cm = wave_incl_max(end ? t : -1);
  if (lane == 63) {
    w_p[w] = cp;
    w_n[w] = cn;
    w_m[w] = cm;
  }
  __syncthreads();
  if (t < 64) {
    const int a = t < NW ? w_p[t] : 0, b = t < NW ? w_n[t] : 0, c = t < NW ? w_m[t] : -1;
    const int ia = wave_incl_sum(a), ib = wave_incl_sum(b), ic = wave_incl_max(c);
    const int prev = __shfl(ic, t > 0 ? t - 1 : 0, 64);     // every lane of wave 0 takes part
    if (t < NW) {
      w_p[t] = ia - a;
      w_n[t] = ib - b;
      w_m[t] = t > 0 ? prev : -1;
    }
  }
  __syncthreads();
  cp += w_p[w];
  cn += w_n[w];
  cm = max(cm, w_m[w]);
  s_cp[t] = cp;
  s_cn[t] = cn;
  s_last[t] = cm;
  __syncthreads();
}

template <typename T>
__global__ void __launch_bounds__(NT) area_chunk_kernel(const T* __restrict__ s, const int64_t* __restrict__ idx,
                                                        int64_t n, int64_t chunk, const uint8_t* __restrict__ lab,
                                                        ChunkSum* __restrict__ sums) {
  __shared__ int s_cp[NT], s_cn[NT], s_last[NT];
  __shared__ int w_p[NW], w_n[NW], w_m[NW];
  const int seg = blockIdx.y, c = blockIdx.x, C = gridDim.x;
  const T* ss = s + (int64_t)seg * n;
  const int64_t* ii = idx + (int64_t)seg * n;
  const int64_t lo = (int64_t)c * chunk, hi = min(n, lo + chunk);
  int64_t tp0 = 0, fp0 = 0, etp = -1, efp = -1;
  for (int64_t base = lo; base < hi; base += NT) {
    int cp, cn;
    bool end;
    slab_scan(ss, ii, lab, base + threadIdx.x, hi, n, s_cp, s_cn, s_last, w_p, w_n, w_m, cp, cn, end);
    const int last = s_last[NT - 1];
    if (last >= 0) {
      etp = tp0 + s_cp[last];
      efp = fp0 + s_cn[last];
    }
    tp0 += s_cp[NT - 1];
    fp0 += s_cn[NT - 1];
    __syncthreads();
  }
  if (threadIdx.x == 0) sums[(int64_t)seg * C + c] = ChunkSum{tp0, fp0, etp, efp};
}

// Pass 2 (grid J x C): the chunk's carry -- counts before it and at the last run end before it -- from the chunk
// summaries, then the trapezoids of its run ends; one fp64 partial per (segment, chunk) for the fixed-order sum.
template <typename T>
__global__ void __launch_bounds__(NT) area_sum_kernel(const T* __restrict__ s, const int64_t* __restrict__ idx,
                                                      int64_t n, int64_t chunk, const uint8_t* __restrict__ lab,
                                                      const ChunkSum* __restrict__ sums, double* __restrict__ part) {
  __shared__ int s_cp[NT], s_cn[NT], s_last[NT];
  __shared__ int w_p[NW], w_n[NW], w_m[NW];
  __shared__ double r_pr[NW], r_roc[NW];
  __shared__ int64_t s_carry[5];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int seg = blockIdx.y, c = blockIdx.x, C = gridDim.x;
  const T* ss = s + (int64_t)seg * n;
  const int64_t* ii = idx + (int64_t)seg * n;
  const ChunkSum* cs = sums + (int64_t)seg * C;
  if (t == 0) {                        // C is small (n / chunk): one thread folds the preceding chunks in order
    int64_t a = 0, b = 0, ptp = 0, pfp = 0, hp = 0;
    for (int k = 0; k < c; ++k) {
      if (cs[k].end_tp >= 0) {
        ptp = a + cs[k].end_tp;
        pfp = b + cs[k].end_fp;
        hp = 1;
      }
      a += cs[k].pos;
      b += cs[k].neg;
    }
    s_carry[0] = a;
    s_carry[1] = b;
    s_carry[2] = ptp;
    s_carry[3] = pfp;
    s_carry[4] = hp;
  }
  __syncthreads();
  int64_t tp0 = s_carry[0], fp0 = s_carry[1], ptp = s_carry[2], pfp = s_carry[3];
  bool has_prev = s_carry[4] != 0;
  const int64_t lo = (int64_t)c * chunk, hi = min(n, lo + chunk);
  double acc_pr = 0.0, acc_roc = 0.0;
  for (int64_t base = lo; base < hi; base += NT) {
    int cp, cn;
    bool end;
    slab_scan(ss, ii, lab, base + t, hi, n, s_cp, s_cn, s_last, w_p, w_n, w_m, cp, cn, end);
    if (end) {
      const int pt = t > 0 ? s_last[t - 1] : -1;        // previous run end in this slab
      const int64_t tp = tp0 + cp, fp = fp0 + cn;
      int64_t tpp, fpp;
      bool hp;
      if (pt >= 0) {
        tpp = tp0 + s_cp[pt];
        fpp = fp0 + s_cn[pt];
        hp = true;
      } else {
        tpp = ptp;
        fpp = pfp;
        hp = has_prev;
      }
      const double prec = tp + fp > 0 ? (double)tp / (double)(tp + fp) : 1.0;
      const double precp = hp ? (tpp + fpp > 0 ? (double)tpp / (double)(tpp + fpp) : 1.0) : prec;
      acc_pr += (double)(tp - tpp) * (prec + precp) * 0.5;
      acc_roc += (double)(fp - fpp) * (double)(tp + tpp) * 0.5;
    }
    const int last = s_last[NT - 1];
    if (last >= 0) {
      ptp = tp0 + s_cp[last];
      pfp = fp0 + s_cn[last];
      has_prev = true;
    }
    tp0 += s_cp[NT - 1];
    fp0 += s_cn[NT - 1];
    __syncthreads();
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    acc_pr += __shfl_down(acc_pr, o, 64);
    acc_roc += __shfl_down(acc_roc, o, 64);
  }
  if (lane == 0) {
    r_pr[w] = acc_pr;
    r_roc[w] = acc_roc;
  }
  __syncthreads();
  if (t == 0) {
    double a = 0.0, b = 0.0;
    for (int k = 0; k < NW; ++k) {
      a += r_pr[k];
      b += r_roc[k];
    }
    part[2 * ((int64_t)seg * C + c)] = a;
    part[2 * ((int64_t)seg * C + c) + 1] = b;
  }
}

// Pass 3 (one thread per segment): chunk partials summed in chunk order, normalised by P and P N.
__global__ void area_finish_kernel(const ChunkSum* __restrict__ sums, const double* __restrict__ part, int J, int C,
                                   double* __restrict__ out_pr, double* __restrict__ out_roc) {
  const int seg = blockIdx.x * blockDim.x + threadIdx.x;
  if (seg >= J) return;
  double a = 0.0, b = 0.0;
  int64_t P = 0, N = 0;
  for (int c = 0; c < C; ++c) {
    a += part[2 * ((int64_t)seg * C + c)];
    b += part[2 * ((int64_t)seg * C + c) + 1];
    P += sums[(int64_t)seg * C + c].pos;
    N += sums[(int64_t)seg * C + c].neg;
  }
  out_pr[seg] = P > 0 ? a / (double)P : 0.0;
  // no negatives: every ROC point has fpr 0 and the (1, 1) end point closes a unit-width trapezoid at tpr 1
  out_roc[seg] = P > 0 ? (N > 0 ? b / ((double)P * (double)N) : 1.0) : 0.0;
}

}  // namespace

extern "C" {

// s: [J][n] sorted scores (fp64 when is_f64, else fp32), idx: [J][n] source column, lab: [n] 0/1. The segments are
// cut into chunks of 64 slabs so the three passes run on J * C workgroups (J alone would leave most CUs idle on a
// multi-million-row validation fold). Scratch comes from the stream-ordered pool.
int tmog_hip_binary_areas(const void* s, int is_f64, const int64_t* idx, int64_t n, int J, const uint8_t* lab,
                          double* out_pr, double* out_roc, hipStream_t stream) {
  if (J <= 0) return 0;
  if (n <= 0) {
    hipMemsetAsync(out_pr, 0, sizeof(double) * J, stream);
    hipMemsetAsync(out_roc, 0, sizeof(double) * J, stream);
    return (int)hipGetLastError();
  }
  const int64_t chunk = 64 * (int64_t)NT;
  const int C = (int)((n + chunk - 1) / chunk);
  if ((int64_t)C > 65535) return -2;
  ChunkSum* sums = nullptr;
  double* part = nullptr;
  hipError_t e = hipMallocAsync((void**)&sums, sizeof(ChunkSum) * (size_t)J * C, stream);
  if (e != hipSuccess) return (int)e;
  e = hipMallocAsync((void**)&part, sizeof(double) * 2 * (size_t)J * C, stream);
  if (e != hipSuccess) {
    hipFreeAsync(sums, stream);
    return (int)e;
  }
  const dim3 grid(C, J);
  if (is_f64) {
    hipLaunchKernelGGL(area_chunk_kernel<double>, grid, dim3(NT), 0, stream, (const double*)s, idx, n, chunk, lab, sums);
    hipLaunchKernelGGL(area_sum_kernel<double>, grid, dim3(NT), 0, stream, (const double*)s, idx, n, chunk, lab, sums,
                       part);
  } else {
    hipLaunchKernelGGL(area_chunk_kernel<float>, grid, dim3(NT), 0, stream, (const float*)s, idx, n, chunk, lab, sums);
    hipLaunchKernelGGL(area_sum_kernel<float>, grid, dim3(NT), 0, stream, (const float*)s, idx, n, chunk, lab, sums,
                       part);
  }
  hipLaunchKernelGGL(area_finish_kernel, dim3((J + 63) / 64), dim3(64), 0, stream, sums, part, J, C, out_pr, out_roc);
  const int rc = (int)hipGetLastError();
  hipFreeAsync(part, stream);
  hipFreeAsync(sums, stream);
  return rc;
}

}  // extern "C"

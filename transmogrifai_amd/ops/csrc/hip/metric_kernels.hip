// Exact areas under the PR and ROC curves of J score sets over the same labelled rows (the model
// selector's BinaryClassificationEvaluator metric, Spark BinaryClassificationMetrics with numBins = 0, as
// OpBinaryClassificationEvaluator.scala:67-135 computes it).
//
// Input: every score set sorted descending (the caller's flat radix sorts: segment-major, stable), the source
// column of every sorted element and the rows' 0/1 labels. One 1024-thread workgroup walks one score set in
// 1024-element chunks: a block scan of the (positive, negative) counts gives the cumulative confusion counts,
// the curve points are the run ends (the last element of every run of equal scores), and each run end adds its
// trapezoid against the previous run end -- the previous end inside the chunk comes from an exclusive max-scan
// of the end positions, across chunks from the carried counts. With P positives and N negatives:
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

template <typename T>
__global__ void __launch_bounds__(NT) binary_area_kernel(const T* __restrict__ s, const int64_t* __restrict__ idx,
                                                         int64_t n, const uint8_t* __restrict__ lab,
                                                         double* __restrict__ out_pr, double* __restrict__ out_roc) {
  __shared__ int s_cp[NT], s_cn[NT], s_last[NT];
  __shared__ int w_p[NW], w_n[NW], w_m[NW];
  __shared__ double r_pr[NW], r_roc[NW];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t off = (int64_t)blockIdx.x * n;
  const T* ss = s + off;
  const int64_t* ii = idx + off;
  int64_t tp0 = 0, fp0 = 0;       // counts before this chunk (block-uniform)
  int64_t ptp = 0, pfp = 0;       // counts at the last run end before this chunk
  bool has_prev = false;
  double acc_pr = 0.0, acc_roc = 0.0;
  for (int64_t base = 0; base < n; base += NT) {
    const int64_t i = base + t;
    const bool v = i < n;
    const T sc = v ? ss[i] : T(0);
    const int pos = v ? (int)(lab[ii[i]] != 0) : 0;
    const int neg = v ? 1 - pos : 0;
    const bool end = v && (i == n - 1 || ss[i + 1] != sc);
    // block inclusive scans: counts (sum) and the last end position (max)
    int cp = wave_incl_sum(pos), cn = wave_incl_sum(neg), cm = wave_incl_max(end ? t : -1);
    if (lane == 63) {
      w_p[w] = cp;
      w_n[w] = cn;
      w_m[w] = cm;
    }
    __syncthreads();
    if (t < 64) {
      int a = t < NW ? w_p[t] : 0, b = t < NW ? w_n[t] : 0, c = t < NW ? w_m[t] : -1;
      // exclusive wave prefixes of the per-wave totals
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
    if (end) {
      const int pt = t > 0 ? s_last[t - 1] : -1;        // previous run end in this chunk
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
    // carry to the next chunk (every thread computes the same values from LDS)
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
  // fixed-order reduction: lanes, then waves
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
    const double P = (double)tp0, N = (double)fp0;
    out_pr[blockIdx.x] = P > 0 ? a / P : 0.0;
    // no negatives: every ROC point has fpr 0 and the (1, 1) end point closes a unit-width trapezoid at tpr 1
    out_roc[blockIdx.x] = P > 0 ? (N > 0 ? b / (P * N) : 1.0) : 0.0;
  }
}

}  // namespace

extern "C" {

// s: [J][n] sorted scores (fp64 when is_f64, else fp32), idx: [J][n] source column, lab: [n] 0/1.
int tmog_hip_binary_areas(const void* s, int is_f64, const int64_t* idx, int64_t n, int J, const uint8_t* lab,
                          double* out_pr, double* out_roc, hipStream_t stream) {
  if (J <= 0) return 0;
  if (n <= 0) {
    hipMemsetAsync(out_pr, 0, sizeof(double) * J, stream);
    hipMemsetAsync(out_roc, 0, sizeof(double) * J, stream);
    return (int)hipGetLastError();
  }
  if (is_f64)
    hipLaunchKernelGGL(binary_area_kernel<double>, dim3(J), dim3(NT), 0, stream, (const double*)s, idx, n, lab,
                       out_pr, out_roc);
  else
    hipLaunchKernelGGL(binary_area_kernel<float>, dim3(J), dim3(NT), 0, stream, (const float*)s, idx, n, lab, out_pr,
                       out_roc);
  return (int)hipGetLastError();
}

}  // extern "C"

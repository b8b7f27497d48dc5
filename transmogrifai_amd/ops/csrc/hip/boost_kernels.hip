// Boosting-round epilogue and counter-based row sampling for CDNA4 (gfx950).
//
// boost_epilogue_kernel -- one launch per boosting round replaces the ~60 small torch ops that
// followed every XGBoost / GBT round (OpXGBoostClassifier.scala:47-403 drives 200 of them per config):
// for every training entry of the round's trees (the leaf assignment the tree grower returns) it
//   1. adds the entry's leaf value to the job's margin   F[p, r] += value[gid]          (fp64)
//   2. writes next round's gradient / hessian            G[p, r], H[p, r]             (fp32)
//      (binary:logistic: p = sigmoid(F), g = p - y, h = max(p (1 - p), 1e-16); squared error: g = F - y, h = 1)
//   3. bins the new training score into the job's (label, score-bin) count table, from which the
//      early-stopping AuPR on the training rows (eval_metric aucpr) is a cumulative sum.
// Every (job, row) pair occurs exactly once among a round's entries, so the margin / gradient
// stores need no atomics; the AuPR table uses integer atomics (exact, order-independent).
//
// poisson_pack_kernel -- Poisson(rate) bootstrap multiplicities (Spark RF BaggedPoint with
// replacement) for k trees over one row list, fused with the tree engine's root packing: the uniform
// is row_uniform's, the count is the number of inverse-CDF steps it passes (the host ships the exact
// CDF table of trees.bootstrap_weights_multi), rows drawn zero times are dropped and the rest written
// as packed entries (row | w << 24) -- one pass instead of ~20 int64 [k, n] torch ops plus a
// compaction per forest. Two launches: count (per-tree totals) and pack (block-reserved output slots;
// the order inside a tree is not significant: histograms are exact integer sums).
//
// row_uniform_kernel -- the splitmix64 per-(seed, stream, global row id) uniform of
// tuning/splitters.row_uniform (hold-out split, CV folds, down-sampling, bootstrap, sanity-check
// sample) as one fused pass instead of ~12 int64 elementwise torch kernels; bit-identical results.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

namespace {

__global__ void __launch_bounds__(256) boost_epilogue_kernel(
    const uint32_t* __restrict__ entries, const int32_t* __restrict__ gid, int64_t n_entries,
    const float* __restrict__ gid_value, const int64_t* __restrict__ gid_tree, const int64_t* __restrict__ tree_job,
    int64_t N, double* __restrict__ F, float* __restrict__ G, float* __restrict__ H, const float* __restrict__ y,
    int objective, int32_t* __restrict__ auc_hist, int bins, int64_t n_gid, int64_t n_trees, int64_t P) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_entries) return;
  const int64_t r = entries[e] & 0xFFFFFFu;
  const int32_t g_id = gid[e];
  if (g_id < 0 || g_id >= n_gid || r >= N) return;                 // defensive: never index out of range
  const int64_t t = gid_tree[g_id];
  if (t < 0 || t >= n_trees) return;
  const int64_t p = tree_job[t];
  if (p < 0 || p >= P) return;
  const int64_t k = p * N + r;
  const double m = F[k] + (double)gid_value[g_id];
  F[k] = m;
  const float yr = y[r];
  if (objective == 0) {
    const double pr = 1.0 / (1.0 + exp(-m));
    G[k] = (float)(pr - (double)yr);
    H[k] = (float)fmax(pr * (1.0 - pr), 1e-16);
    if (auc_hist) {
      const float s = fminf(fmaxf((float)pr, 0.f), 1.f);
      const int b = (int)(s * (float)(bins - 1));
      atomicAdd(auc_hist + (p * 2 + (yr > 0.5f ? 1 : 0)) * bins + (bins - 1 - b), 1);
    }
  } else {
    G[k] = (float)(m - (double)yr);
    H[k] = 1.f;
  }
}

__device__ __forceinline__ double splitmix_uniform(uint64_t rid, uint64_t off) {
  const uint64_t M63 = 0x7FFFFFFFFFFFFFFFull;
  uint64_t x = rid * 0x1E3779B97F4A7C15ull + off;
  x &= M63;
  x = ((x ^ (x >> 30)) * 0x2F58476D1CE4E5B9ull) & M63;
  x = ((x ^ (x >> 27)) * 0x14C3124B4B69A5C5ull) & M63;
  x = x ^ (x >> 31);
  return (double)(x >> 10) / 9007199254740992.0;
}

__global__ void __launch_bounds__(256) poisson_pack_kernel(const int64_t* __restrict__ rows, int64_t n,
                                                           const int64_t* __restrict__ offsets,
                                                           const double* __restrict__ cdf, int ncdf,
                                                           unsigned long long* __restrict__ counts,
                                                           const int64_t* __restrict__ base,
                                                           int32_t* __restrict__ out) {
  const int t = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int w = 0;
  uint32_t r = 0;
  if (i < n) {
    r = (uint32_t)rows[i];
    const double u = splitmix_uniform((uint64_t)rows[i], (uint64_t)offsets[t]);
    for (int c = 0; c < ncdf; ++c) w += (u >= cdf[c]) ? 1 : 0;
  }
  const bool keep = w > 0;
  const unsigned long long m = __ballot(keep);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int pre = __popcll(m & ((1ull << lane) - 1ull));
  __shared__ int wtot[4];
  __shared__ unsigned long long blk;
  if (lane == 0) wtot[wv] = __popcll(m);
  __syncthreads();
  int wbase = 0, tot = 0;
  for (int k = 0; k < 4; ++k) {
    if (k < wv) wbase += wtot[k];
    tot += wtot[k];
  }
  if (out == nullptr) {
    if (threadIdx.x == 0 && tot) atomicAdd(counts + t, (unsigned long long)tot);
    return;
  }
  if (threadIdx.x == 0) blk = tot ? atomicAdd(counts + t, (unsigned long long)tot) : 0ull;
  __syncthreads();
  if (keep) out[base[t] + (int64_t)blk + wbase + pre] = (int32_t)(r | ((uint32_t)min(w, 255) << 24));
}

__global__ void __launch_bounds__(256) row_uniform_kernel(const int64_t* __restrict__ row_ids, int64_t n,
                                                          const int64_t* __restrict__ offsets, int k_seeds,
                                                          double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t M63 = 0x7FFFFFFFFFFFFFFFull;
  const uint64_t rid = (uint64_t)row_ids[i];
  for (int s = 0; s < k_seeds; ++s) {
    uint64_t x = rid * 0x1E3779B97F4A7C15ull + (uint64_t)offsets[s];
    x &= M63;
    x = ((x ^ (x >> 30)) * 0x2F58476D1CE4E5B9ull) & M63;
    x = ((x ^ (x >> 27)) * 0x14C3124B4B69A5C5ull) & M63;
    x = x ^ (x >> 31);
    out[(int64_t)s * n + i] = (double)(x >> 10) / 9007199254740992.0;
  }
}

}  // namespace


// AuPR of K score sets from their (label, score-bin) count tables [K][2][bins] (bins in descending score
// order; the boosting-round early-stopping metric, evaluators/metrics.py binned_aupr_from_counts): one
// workgroup per set. Segment sums + a block scan give every thread its cumulative (tp, fp) entering its
// 256-bin segment; the thread then walks the segment with the same per-bin arithmetic as the torch path
// (precision tp / cnt, recall tp / P, trapezoid ((r - r') * (p + p')) * 0.5, leading empty bins taking the
// first non-empty bin's precision) and the block sums the terms -- one launch instead of two 65536-long
// fp64 scans plus ~20 small kernels per round.
__global__ void __launch_bounds__(256) aupr_counts_kernel(const int32_t* __restrict__ counts, int bins,
                                                          double* __restrict__ out) {
  const int k = blockIdx.x, t = threadIdx.x;
  const int32_t* neg = counts + (int64_t)k * 2 * bins;
  const int32_t* pos = neg + bins;
  const int seg = (bins + 255) / 256;
  const int b0 = min(bins, t * seg), b1 = min(bins, b0 + seg);
  long long sp = 0, sn = 0;
  int first = 0x7fffffff;
  for (int b = b0; b < b1; ++b) {
    const int p = pos[b], n = neg[b];
    sp += p;
    sn += n;
    if (p + n > 0 && first == 0x7fffffff) first = b;
  }
  __shared__ long long s_p[256], s_n[256];
  __shared__ int s_first[256];
  __shared__ double s_area[256];
  s_p[t] = sp;
  s_n[t] = sn;
  s_first[t] = first;
  __syncthreads();
  if (t == 0) {                    // exclusive scan of 256 segment totals + global first non-empty bin
    long long ap = 0, an = 0;
    int f = 0x7fffffff;
    for (int i = 0; i < 256; ++i) {
      const long long vp = s_p[i], vn = s_n[i];
      s_p[i] = ap;
      s_n[i] = an;
      ap += vp;
      an += vn;
      f = min(f, s_first[i]);
    }
    s_first[0] = f == 0x7fffffff ? 0 : f;
    s_area[0] = (double)ap;        // total positives P
  }
  __syncthreads();
  const double Pt = s_area[0];
  const double Pm = Pt > 1.0 ? Pt : 1.0;
  const int fb = s_first[0];
  const double pf = (double)pos[fb] / fmax((double)pos[fb] + (double)neg[fb], 1.0);   // prec at the first bin
  double tp = (double)s_p[t], fp = (double)s_n[t];
  double prev_prec = (tp + fp > 0.0) ? tp / fmax(tp + fp, 1.0) : pf;
  double prev_rec = tp / Pm;
  double acc = 0.0;
  for (int b = b0; b < b1; ++b) {
    tp += (double)pos[b];
    fp += (double)neg[b];
    const double cnt = tp + fp;
    const double pr = cnt > 0.0 ? tp / fmax(cnt, 1.0) : pf;
    const double rc = tp / Pm;
    acc += ((rc - prev_rec) * (pr + prev_prec)) * 0.5;
    prev_prec = pr;
    prev_rec = rc;
  }
  __syncthreads();
  s_area[t] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) s_area[t] += s_area[t + w];
    __syncthreads();
  }
  if (t == 0) out[k] = Pt > 0.0 ? s_area[0] : 0.0;
}

extern "C" {

int tmog_hip_boost_epilogue(const uint32_t* entries, const int32_t* gid, int64_t n_entries, const float* gid_value,
                            const int64_t* gid_tree, const int64_t* tree_job, int64_t N, double* F, float* G, float* H,
                            const float* y, int objective, int32_t* auc_hist, int bins, int64_t n_gid,
                            int64_t n_trees, int64_t P, hipStream_t stream) {
  if (n_entries == 0) return 0;
  if (N >= (1 << 24)) return -2;
  hipLaunchKernelGGL(boost_epilogue_kernel, dim3((unsigned)((n_entries + 255) / 256)), dim3(256), 0, stream, entries,
                     gid, n_entries, gid_value, gid_tree, tree_job, N, F, G, H, y, objective, auc_hist, bins, n_gid,
                     n_trees, P);
  return (int)hipGetLastError();
}

// counts[k] must be zero. out == nullptr: count pass (counts = kept rows per tree); otherwise pack
// pass with base[k] = first output slot of tree k (counts, re-zeroed, act as the slot cursors).
int tmog_hip_poisson_pack(const int64_t* rows, int64_t n, const int64_t* offsets, int k, const double* cdf, int ncdf,
                          unsigned long long* counts, const int64_t* base, int32_t* out, hipStream_t stream) {
  if (n == 0 || k == 0) return 0;
  if (n >= (1 << 24) || k > 65535 || ncdf > 64 || (out != nullptr && base == nullptr)) return -2;
  hipLaunchKernelGGL(poisson_pack_kernel, dim3((unsigned)((n + 255) / 256), (unsigned)k), dim3(256), 0, stream, rows,
                     n, offsets, cdf, ncdf, counts, base, out);
  return (int)hipGetLastError();
}

int tmog_hip_row_uniform(const int64_t* row_ids, int64_t n, const int64_t* offsets, int k_seeds, double* out,
                         hipStream_t stream) {
  if (n == 0 || k_seeds == 0) return 0;
  hipLaunchKernelGGL(row_uniform_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, row_ids, n, offsets,
                     k_seeds, out);
  return (int)hipGetLastError();
}

int tmog_hip_aupr_counts(const int32_t* counts, int K, int bins, double* out, hipStream_t stream) {
  if (K <= 0) return 0;
  if (bins <= 0) return -2;
  hipLaunchKernelGGL(aupr_counts_kernel, dim3(K), dim3(256), 0, stream, counts, bins, out);
  return (int)hipGetLastError();
}

}  // extern "C"

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
#include <algorithm>
#include <stdint.h>
#include <math.h>

namespace {

constexpr int kAmaxCopies = 64;   // boost_epilogue_kernel's per-job maxima: [kAmaxCopies][P][2] (trees.py)

// Wave64 max of non-negative floats (their bit patterns order like int32) on DPP -- row_shr 1/2/4/8 inside the
// 16-lane rows, row_bcast 15/31 across them -- wave-uniform result, no ds_bpermute. Whole wave active.
__device__ __forceinline__ float wave_max_nonneg(float f) {
  int v = __float_as_int(f);
#define TM_DPP_MAX(CTRL, ROWS) v = max(v, __builtin_amdgcn_update_dpp(0, v, CTRL, ROWS, 0xF, false));
  TM_DPP_MAX(0x111, 0xF) TM_DPP_MAX(0x112, 0xF) TM_DPP_MAX(0x114, 0xF) TM_DPP_MAX(0x118, 0xF)
  TM_DPP_MAX(0x142, 0xA) TM_DPP_MAX(0x143, 0xC)
#undef TM_DPP_MAX
  return __int_as_float(__builtin_amdgcn_readlane(v, 63));
}

__global__ void __launch_bounds__(256) boost_epilogue_kernel(
    const uint32_t* __restrict__ entries, const int32_t* __restrict__ gid, int64_t n_entries,
    const float* __restrict__ gid_value, const int64_t* __restrict__ gid_tree, const int64_t* __restrict__ tree_job,
    int64_t N, double* __restrict__ F, float* __restrict__ G, float* __restrict__ H, const float* __restrict__ y,
    int objective, int32_t* __restrict__ auc_hist, int bins, int64_t n_gid, int64_t n_trees, int64_t P,
    uint32_t* __restrict__ amax, int wide) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float ag = 0.f, ah = 0.f;                    // this lane's |g| and h (for the next round's quantisation)
  // no early returns: the AuPR-count aggregation below needs every lane of the wave
  int64_t slot = -1;                           // this lane's (job, label, score-bin) counter, -1 = none
  bool ok = e < n_entries;
  int64_t r = 0, t = 0, p = 0;
  int32_t g_id = 0;
  if (ok) {
    r = wide ? (int64_t)entries[e] : (int64_t)(entries[e] & 0xFFFFFFu);   // tree_kernels.hip ent_row
    g_id = gid[e];
    ok = g_id >= 0 && g_id < n_gid && r < N;   // defensive: never index out of range
  }
  if (ok) {
    t = gid_tree[g_id];
    ok = t >= 0 && t < n_trees;
  }
  if (ok) {
    p = tree_job[t];
    ok = p >= 0 && p < P;
  }
  if (ok) {
    const int64_t k = p * N + r;
    const double m = F[k] + (double)gid_value[g_id];
    F[k] = m;
    const float yr = y[r];
    if (objective == 0) {
      const double pr = 1.0 / (1.0 + exp(-m));
      const float gk = (float)(pr - (double)yr), hk = (float)fmax(pr * (1.0 - pr), 1e-16);
      G[k] = gk;
      H[k] = hk;
      ag = fabsf(gk);
      ah = hk;
      if (auc_hist) {
        const float sc = fminf(fmaxf((float)pr, 0.f), 1.f);
        const int b = (int)(sc * (float)(bins - 1));
        slot = (p * 2 + (yr > 0.5f ? 1 : 0)) * bins + (bins - 1 - b);
      }
    } else {
      const float gk = (float)(m - (double)yr);
      G[k] = gk;
      H[k] = 1.f;
      ag = fabsf(gk);
      ah = 1.f;
    }
  }
  if (amax) {
    // per-job max |g| and max h of the new statistics (tree_engine._quant_scales of the next round): the
    // wave peels off its distinct jobs (usually one), max-reduces each over the matching lanes and issues
    // one atomicMax per job on the float bits (non-negative floats order like their bit patterns) into one
    // of kAmaxCopies copies (block-strided: same-address atomics from every wave would serialise); the
    // host takes the max over the copies
    const int lane = threadIdx.x & 63;
    bool pend = ok;
    for (int it = 0; it < 64; ++it) {
      const unsigned long long act = __ballot(pend);
      if (act == 0ull) break;
      const int leader = __ffsll((long long)act) - 1;
      const int64_t lp = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)((uint64_t)p >> 32), leader) << 32) |
                                   (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)p, leader));
      const bool mine = pend && p == lp;
      // NaN lanes contribute nothing (as fmaxf ignored them)
      const float mg = wave_max_nonneg(mine && ag == ag ? ag : 0.f), mh = wave_max_nonneg(mine && ah == ah ? ah : 0.f);
      if (lane == leader) {
        uint32_t* dst = amax + ((int64_t)(blockIdx.x % kAmaxCopies) * P + lp) * 2;
        atomicMax(dst, __float_as_uint(mg));
        atomicMax(dst + 1, __float_as_uint(mh));
      }
      pend = pend && !mine;
    }
  }
  if (auc_hist) {
    // Scores of a boosting round cluster in a few bins (eta-sized steps from a shared base margin), so
    // per-lane atomics serialise on the same counters: the wave first peels off up to 8 distinct slots
    // (ballot on the leader's slot, one atomic of the match count each), the rest go per lane.
    const int lane = threadIdx.x & 63;
    bool pend = slot >= 0;
    for (int it = 0; it < 8; ++it) {
      const unsigned long long act = __ballot(pend);
      if (act == 0ull) break;
      const int leader = __ffsll((long long)act) - 1;
      const int64_t ls = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)((uint64_t)slot >> 32), leader) << 32) |
                                   (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)slot, leader));
      const bool mine = pend && slot == ls;
      const unsigned long long mm = __ballot(mine);
      if (lane == leader) atomicAdd(auc_hist + ls, (int)__popcll(mm));
      pend = pend && !mine;
    }
    if (pend) atomicAdd(auc_hist + slot, 1);
  }
}

// boost_prologue_kernel -- the set-up of a device-resident boosting round (models/trees.py, resident grower) in
// one launch instead of ~35 small torch ops: per active job p (= its model index)
//   * the quantisation maxima of the new (g, h): max(rows outside the job's training set, the last
//     epilogue's per-copy maxima tam_prev) -> amax[p] (tree_engine._quant_scales' amax_hint),
//   * the power-of-two fixed-point scales q = 2^floor(log2(qmax / max(amax, 1e-30))) clamped to 2^[-60, 60]
//     (built from the exponent bits: exact, as tree_engine._quant_scales computes it) -> qscale[p], qinv[p],
//   * every root entry copied into the grower's row buffer and its quantised (q(w g), q(w h)) staged
//     (tree_engine._stage_gh: rintf((w * t) * q), the same fp32 operation order),
//   * the job's copies of the NEXT epilogue's maxima buffer zeroed (double buffered by the caller).
// Every block recomputes the T scales from the (tiny) maxima tables; block 0 writes them out.
__device__ __forceinline__ float pow2_scale(float qmax, float a) {
  const float x = qmax / fmaxf(a, 1e-30f);
  const int e = (int)((__float_as_uint(x) >> 23) & 0xFFu) - 127;   // floor(log2 x) for normal x
  const int k = min(60, max(-60, e));
  return __uint_as_float((uint32_t)(k + 127) << 23);
}

constexpr int kMaxProJobs = 64;

__global__ void __launch_bounds__(256) boost_prologue_kernel(
    const uint32_t* __restrict__ tam_prev, uint32_t* __restrict__ tam_next, const float* __restrict__ comp,
    float* __restrict__ amax, int P, const int32_t* __restrict__ act, int T, const int64_t* __restrict__ job_off,
    const uint32_t* __restrict__ root, uint32_t* __restrict__ rows, const float* __restrict__ G,
    const float* __restrict__ H, int64_t stride, int2* __restrict__ gh, float* __restrict__ qscale,
    double* __restrict__ qinv, float qmax, int wide) {
  __shared__ float s_sc[kMaxProJobs][2];
  __shared__ int64_t s_off[kMaxProJobs + 1];
  __shared__ int s_p[kMaxProJobs];
  for (int t = threadIdx.x; t < T; t += blockDim.x) {
    const int p = act[t];
    float a0, a1;
    if (tam_prev) {
      a0 = comp[2 * p];
      a1 = comp[2 * p + 1];
      for (int c = 0; c < kAmaxCopies; ++c) {
        a0 = fmaxf(a0, __uint_as_float(tam_prev[((int64_t)c * P + p) * 2]));
        a1 = fmaxf(a1, __uint_as_float(tam_prev[((int64_t)c * P + p) * 2 + 1]));
      }
    } else {
      a0 = amax[2 * p];
      a1 = amax[2 * p + 1];
    }
    const float q0 = pow2_scale(qmax, a0), q1 = pow2_scale(qmax, a1);
    s_sc[t][0] = q0;
    s_sc[t][1] = q1;
    s_p[t] = p;
    if (blockIdx.x == 0) {
      amax[2 * p] = a0;
      amax[2 * p + 1] = a1;
      qscale[2 * p] = q0;
      qscale[2 * p + 1] = q1;
      qinv[2 * p] = 1.0 / (double)q0;
      qinv[2 * p + 1] = 1.0 / (double)q1;
    }
  }
  for (int t = threadIdx.x; t <= T; t += blockDim.x) s_off[t] = job_off[t];
  if (blockIdx.x == 0 && tam_next)
    for (int i = threadIdx.x; i < kAmaxCopies * T; i += blockDim.x) {
      const int c = i / T, t = i - c * T;
      tam_next[((int64_t)c * P + act[t]) * 2] = 0u;
      tam_next[((int64_t)c * P + act[t]) * 2 + 1] = 0u;
    }
  __syncthreads();
  const int64_t total = s_off[T];
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    int t = 0;
    while (t + 1 < T && s_off[t + 1] <= e) ++t;
    const uint32_t en = root[e];
    rows[e] = en;
    const int64_t r = wide ? (int64_t)en : (int64_t)(en & 0xFFFFFFu);
    const float w = (float)(wide ? 1u : (en >> 24));
    const int64_t k = (int64_t)s_p[t] * stride + r;
    const float g = w * G[k];
    const float h = w * H[k];
    gh[e] = make_int2((int)rintf(g * s_sc[t][0]), (int)rintf(h * s_sc[t][1]));
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
// 1024-thread workgroup per set, thread t owning the consecutive bins [t seg, (t + 1) seg). The thread sums its
// segment (16 bins at a time, their loads issued together, 16-byte loads when aligned), one block scan of the segment totals
// gives every segment its cumulative (tp, fp) before it and the positive total P, and the thread then walks its
// bins again (L2 hits) evaluating each bin's trapezoid term with the torch path's arithmetic (precision
// tp / cnt, recall tp / P, ((r - r') * (p + p')) * 0.5). The previous bin's precision comes from the cumulative
// counts before the bin; with none before it (leading empty bins) the torch path uses the first non-empty bin's
// precision, which is this bin's own whenever the term is non-zero. Replaces a version that walked the bins in
// 16 dependent 4096-bin chunks (two barriers and a memory round trip each: ~107 us a call at 65536 bins, one
// call per boosting round on the round's serial chain).
constexpr int AUPR_NT = 1024;

__global__ void __launch_bounds__(AUPR_NT) aupr_counts_kernel(const int32_t* __restrict__ counts, int bins,
                                                              double* __restrict__ out) {
  const int k = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  constexpr int NW = AUPR_NT / 64;
  const int32_t* neg = counts + (int64_t)k * 2 * bins;
  const int32_t* pos = neg + bins;
  __shared__ long long s_p[NW], s_n[NW];
  __shared__ double s_acc[NW];
  const int seg = (bins + AUPR_NT - 1) / AUPR_NT;
  const int b0 = min(bins, t * seg), b1 = min(bins, b0 + seg);
  const bool vec = (bins & 3) == 0 && (seg & 3) == 0 && ((uintptr_t)neg & 15) == 0;
  // 16 bins of the segment at a time, all their loads issued together (bins past the segment read as 0: an
  // empty bin changes neither the cumulative counts nor the area)
  auto load16 = [&](int c, int (&pv)[16], int (&nv)[16]) {
    if (vec && c + 16 <= b1) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int4 p4 = *reinterpret_cast<const int4*>(pos + c + 4 * q);
        const int4 n4 = *reinterpret_cast<const int4*>(neg + c + 4 * q);
        pv[4 * q] = p4.x; pv[4 * q + 1] = p4.y; pv[4 * q + 2] = p4.z; pv[4 * q + 3] = p4.w;
        nv[4 * q] = n4.x; nv[4 * q + 1] = n4.y; nv[4 * q + 2] = n4.z; nv[4 * q + 3] = n4.w;
      }
    } else {
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int b = min(c + u, bins - 1);
        pv[u] = c + u < b1 ? pos[b] : 0;
        nv[u] = c + u < b1 ? neg[b] : 0;
      }
    }
  };
  long long lp = 0, ln = 0;
  for (int c = b0; c < b1; c += 16) {
    int pv[16], nv[16];
    load16(c, pv, nv);
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      lp += pv[u];
      ln += nv[u];
    }
  }
  long long ip = lp, in = ln;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const long long a = __shfl_up(ip, o, 64), c = __shfl_up(in, o, 64);
    if (lane >= o) {
      ip += a;
      in += c;
    }
  }
  if (lane == 63) {
    s_p[wv] = ip;
    s_n[wv] = in;
  }
  __syncthreads();
  long long ep = ip - lp, en = in - ln, Pi = 0;
  for (int w = 0; w < NW; ++w) {
    if (w < wv) {
      ep += s_p[w];
      en += s_n[w];
    }
    Pi += s_p[w];
  }
  const double Pt = (double)Pi;
  const double Pm = Pt > 1.0 ? Pt : 1.0;
  double tp = (double)ep, fp = (double)en, acc = 0.0;
  for (int c = b0; c < b1; c += 16) {
    int pv[16], nv[16];
    load16(c, pv, nv);
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const double tp1 = tp + (double)pv[u], fp1 = fp + (double)nv[u];
      if (pv[u] > 0) {
        const double pr = tp1 / fmax(tp1 + fp1, 1.0);
        const double prev_prec = (tp + fp > 0.0) ? tp / fmax(tp + fp, 1.0) : pr;
        acc += ((tp1 / Pm - tp / Pm) * (pr + prev_prec)) * 0.5;
      }
      tp = tp1;
      fp = fp1;
    }
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane == 0) s_acc[wv] = acc;
  __syncthreads();
  if (t == 0) {
    double a = 0.0;
    for (int w = 0; w < NW; ++w) a += s_acc[w];
    out[k] = Pt > 0.0 ? a : 0.0;
  }
}

extern "C" {

int tmog_hip_boost_epilogue(const uint32_t* entries, const int32_t* gid, int64_t n_entries, const float* gid_value,
                            const int64_t* gid_tree, const int64_t* tree_job, int64_t N, double* F, float* G, float* H,
                            const float* y, int objective, int32_t* auc_hist, int bins, int64_t n_gid,
                            int64_t n_trees, int64_t P, hipStream_t stream, uint32_t* amax, int wide_rows) {
  if (n_entries == 0) return 0;
  if (N >= (1 << 24) && !wide_rows) return -2;
  hipLaunchKernelGGL(boost_epilogue_kernel, dim3((unsigned)((n_entries + 255) / 256)), dim3(256), 0, stream, entries,
                     gid, n_entries, gid_value, gid_tree, tree_job, N, F, G, H, y, objective, auc_hist, bins, n_gid,
                     n_trees, P, amax, wide_rows);
  return (int)hipGetLastError();
}

// Round prologue of device-resident boosting (boost_prologue_kernel). tam_prev == null: first round, the
// maxima in amax are used as they are. T <= 64 active jobs.
int tmog_hip_boost_prologue(const uint32_t* tam_prev, uint32_t* tam_next, const float* comp, float* amax, int P,
                            const int32_t* act, int T, const int64_t* job_off, const uint32_t* root, uint32_t* rows,
                            int64_t total, const float* G, const float* H, int64_t stride, int32_t* gh,
                            float* qscale, double* qinv, float qmax, int wide, hipStream_t stream) {
  if (T <= 0) return 0;
  if (T > kMaxProJobs) return -2;
  const int64_t blocks = std::min<int64_t>(std::max<int64_t>(1, (total + 255) / 256), 2048);
  hipLaunchKernelGGL(boost_prologue_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, tam_prev, tam_next, comp,
                     amax, P, act, T, job_off, root, rows, G, H, stride, reinterpret_cast<int2*>(gh), qscale, qinv,
                     qmax, wide);
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
  hipLaunchKernelGGL(aupr_counts_kernel, dim3(K), dim3(AUPR_NT), 0, stream, counts, bins, out);
  return (int)hipGetLastError();
}

}  // extern "C"

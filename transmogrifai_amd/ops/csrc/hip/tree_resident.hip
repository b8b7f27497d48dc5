// Device-planned tree growth ("resident" level loop) for one job group on the caller's stream.
//
// The host-planned grower (common/tree_grow.hpp grow_group) reads every level's split decisions back to the
// host, plans the next level there (node bookkeeping, histogram / partition / leaf work items, sibling
// pairs, zero segments) and ships the plan in one staged copy: one blocking round trip per level and
// group, 66-170 us of stream idle per level on the XGBoost headline (profiles/r4_levels_base.txt). Here the
// same plan is computed ON THE DEVICE by one 1024-thread workgroup (level_plan_kernel) between the level
// kernels, and every level kernel is launched with a host upper bound of its grid and reads the real item
// count from device memory (tree_kernels.hip `dcount` arguments): the host enqueues a whole tree -- every
// level, the leaf collection and the tree finalisation (leaf values, gamma pruning; tree_finalize_kernel) --
// without a single synchronisation, and boosting (models/trees.py) enqueues round after round. The host
// reads the created-node records once per fit.
//
// The device plan reproduces grow_group's decisions exactly (same can / need rules, Newton hessian gate,
// subtraction pairing, feature groups from group_layout, item chunking), so the trees are bit-identical
// to the host-planned grower (tests/test_tree_resident_gpu.py); work-item ORDER may differ where it does not
// matter (integer histogram atomics and exclusive stores are order-independent, partition order inside a
// child is not stable on either path).
//
// Reference behaviour: XGBoost4J's hist updater as wrapped by OpXGBoostClassifier.scala:47-403.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "common/tree_grow.hpp"
#include "hip/dev_alloc.hpp"

extern "C" {
int tmog_hip_hist_build(const uint8_t* Xb, int F, const uint32_t* rows, const void* items, int n_items,
                        const int32_t* node_feat_off, const int32_t* feat_list, const int32_t* node_model,
                        const int64_t* node_hist_off, int64_t* hist, int B, int mode, int S, const float* y,
                        const float* t1, const float* t2, int64_t stride, const float* qscale, int skip_bin,
                        const int64_t* csr_ptr, const uint16_t* csr_col, int Sc, int n_wide, int need_general,
                        hipStream_t stream, const int32_t* gh, const int* dcount, int wide_rows,
                        const uint8_t* Xh, int Fh);
int tmog_hip_split_find(const int64_t* hist, int n_nodes, const int64_t* node_hist_off, const int32_t* node_nfeat,
                        const int32_t* node_feat_off, const int32_t* feat_list, const int32_t* feat_nbins, int B,
                        int S, int kind, const float* node_params, int missing_bin, const int32_t* node_model,
                        const double* qinv, int max_nfeat, void* cand_ws, int32_t* out_feat, int32_t* out_bin,
                        float* out_gain, uint8_t* out_dl, float* out_left, float* out_total, int64_t* cursors, int n_multi,
                        void* rec, int64_t rec_bytes, int fp_mlo, int fp_nml, int fp_obase, hipStream_t stream,
                        unsigned* done, const int* dm);
int tmog_hip_pair_scan(int64_t* hist, const int64_t* parent, const int64_t* parent_off, const int32_t* small_j,
                       const int32_t* big_j, int n_pairs, const int64_t* node_hist_off, const int32_t* node_nfeat,
                       const int32_t* node_feat_off, const int32_t* feat_list, const int32_t* feat_nbins, int B, int S,
                       int kind, const float* node_params, int missing_bin, const int32_t* node_model,
                       const double* qinv, int max_nfeat, void* cand_ws, int n_multi, hipStream_t stream,
                       const int* dnp);
int tmog_hip_zero_segments(int64_t* hist, const int64_t* off, const int64_t* size, int n, int64_t max_size,
                           int64_t dense, int per, int S, hipStream_t stream, int n_dense, const int* dn);
size_t tmog_hip_split_cand_bytes(int n_nodes, int max_nfeat, int B, int S);
int tmog_hip_tree_prime();
int tmog_hip_hist_stat_chunk(int B, int S);
int tmog_hip_partition_fused(const uint8_t* Xb, int F, const uint32_t* rows_in, uint32_t* rows_out, const void* items,
                             int n_items, const int64_t* node_begin, const int64_t* node_count, const int32_t* split_feat,
                             const int32_t* split_bin, const uint8_t* dl, const float* node_params,
                             const float* split_gain, int missing_bin, int64_t* cursors, const uint8_t* XbT, int64_t N,
                             hipStream_t stream, const int32_t* gh_in, int32_t* gh_out, const int* dcount,
                             int wide_rows);
int tmog_hip_leaf_collect(const uint32_t* rows, const void* items, int n_items, uint32_t* out_rows,
                          int32_t* out_gid, hipStream_t stream, const uint32_t* rows_alt, const int* dcount);
int tmog_hip_fp_allgather(const void* send, void* recv, int64_t bytes, void* comm, int world, hipStream_t stream);
int tmog_hip_fp_merge_dev(const void* recv, int R, int m_stride, int64_t rec_bytes, int S, int32_t* out_feat,
                          int32_t* out_bin, float* out_gain, uint8_t* out_dl, float* out_left, const int* dm,
                          hipStream_t stream);
}

// plan / finalisation arithmetic with the host twins' IEEE operation sequence (no FMA contraction)
#pragma clang fp contract(off)

namespace {

using tmog::HistItemH;
using tmog::LeafItemH;
using tmog::PartItemH;

// device counters of the current level (int32 each)
enum : int {
  C_N = 0,     // nodes of the current level
  C_M,         // histogram (scanned) nodes
  C_NP,        // sibling pairs
  C_NH,        // histogram items
  C_NC,        // partition items
  C_NZ,        // zero segments (C_NZ, C_NZD adjacent: zero_segments_kernel reads both)
  C_NZD,       // ... of which whole-node segments (listed first)
  C_NL,        // leaf items
  C_NCREATED,  // created nodes of the tree
  C_ERR,       // bit 0: partition cursor mismatch, bit 1: capacity overflow
  C_COUNT = 16
};

constexpr int kRecFixed = 7;   // record words before the S totals: tree feat bin dl gain left right

struct PlanArgs {
  int d, T, S, chunk_rows, n_groups, n_sc, newton, subtract, pair_fuse, F_use, has_missing;
  int64_t hsz, live_dense;
  const int4* groups;          // (f0, nf, flags): bit 0 register path, bit 1 CSR, bit 2 wide-load
  const int32_t* j_depth;
  const int32_t* j_model;
  const int64_t* j_count;
  const double* j_inst;
  const double* j_gain;
  const double* j_mcw;
  const double* j_lam;
  const double* j_eps;
  int32_t* lv_tree[2];
  int32_t* lv_gid[2];
  int64_t* lv_begin[2];
  int64_t* lv_count[2];
  int32_t* hn[2];              // histogram node j -> level node i
  int32_t* nmd[2];
  int64_t* nho[2];
  float* par[2];
  int64_t* nb[2];
  int64_t* nc[2];
  int32_t* nfo;
  int32_t* nnf;
  int32_t* sj;
  int32_t* bj;
  int64_t* poff;
  int64_t* zoff;
  int64_t* zsize;
  int64_t* ppo;                // parent histogram offset of the previous level's q-th split
  HistItemH* hitems;
  PartItemH* citems;
  LeafItemH* litems;
  const int32_t* r_feat;
  const int32_t* r_bin;
  const float* r_gain;
  const float* r_left;
  const float* r_tot;
  const uint8_t* r_dl;
  const int64_t* r_cur;
  int64_t* rec;
  int W;
  int32_t* level_off;
  int* cnt;
  int64_t* leaf_pos;
  int64_t* sa;
  int64_t* sb;
  int64_t* sc;
  int64_t* sd;
  int64_t* se;
  int64_t* sf;
  int64_t* sg;
  int32_t* flag;
  int32_t* loc;
  int64_t cap_nl, cap_m, cap_nodes, cap_h, cap_c, cap_l;
  int profile;                 // TMOG_PLAN_PROFILE: per-phase wall-clock ticks into g_plan_prof
  int64_t lds_cap;             // > 0: scratch arrays in dynamic LDS with this many entries each
};

// TMOG_PLAN_PROFILE diagnostics: wall-clock ticks (100 MHz) spent in each phase of level_plan_kernel, summed
// over calls (entry 31: calls); read with tmog_hip_plan_profile.
__device__ unsigned long long g_plan_prof[32];

__device__ __forceinline__ int64_t dbits(double v) { return __double_as_longlong(v); }
__device__ __forceinline__ double bitsd(int64_t v) { return __longlong_as_double(v); }

// Exclusive prefix sums of K arrays v[k][0, n) in place at once; every thread of the block calls it and gets the
// totals. Each thread sums a contiguous run of ceil(n / 1024) entries, the runs are scanned inside each wave on
// the lane network (6 shuffle steps, no barrier), the 16 wave totals go through LDS: two barriers per call
// whatever K, instead of 2 log2(1024) per array.
__device__ __forceinline__ int64_t wave_incl_scan(int64_t x, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  return x;
}

template <int K>
__device__ void block_scan_multi(int64_t* const (&v)[K], int64_t n, int64_t (&total)[K], int64_t* sh) {
  const int t = threadIdx.x, nt = blockDim.x, lane = t & 63, wave = t >> 6, nw = nt >> 6;
  const int64_t per = (n + nt - 1) / nt;
  const int64_t lo = min(n, (int64_t)t * per), hi = min(n, lo + per);
  int64_t s[K], incl[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    s[k] = 0;
    for (int64_t i = lo; i < hi; ++i) s[k] += v[k][i];
    incl[k] = wave_incl_scan(s[k], lane);
    if (lane == 63) sh[k * 16 + wave] = incl[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    int64_t before = 0, all = 0;
    for (int w = 0; w < nw; ++w) {
      const int64_t x = sh[k * 16 + w];
      before += w < wave ? x : 0;
      all += x;
    }
    total[k] = all;
    int64_t run = before + incl[k] - s[k];
    for (int64_t i = lo; i < hi; ++i) {
      const int64_t x = v[k][i];
      v[k][i] = run;
      run += x;
    }
  }
  __syncthreads();
}

__device__ __forceinline__ int64_t block_scan(int64_t* v, int64_t n, int64_t* sh) {
  int64_t* const a[1] = {v};
  int64_t tot[1];
  block_scan_multi<1>(a, n, tot, sh);
  return tot[0];
}

// last i in [0, n) with pre[i] <= k (pre: exclusive prefix sums, k < total): the owner of item k
__device__ __forceinline__ int64_t owner(const int64_t* pre, int64_t n, int64_t k) {
  int64_t lo = 0, hi = n - 1;
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    if (pre[mid] <= k) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ void init_node(int64_t* r, int64_t tree, int S) {
  r[0] = tree;
  r[1] = -1;
  r[2] = -1;
  r[3] = 0;
  r[4] = dbits(0.0);
  r[5] = -1;
  r[6] = -1;
  for (int s = 0; s < S; ++s) r[kRecFixed + s] = dbits(0.0);
}

__device__ __forceinline__ int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Leaf items of the nodes i in [0, n) whose sa-flag is 0 (sa == nullptr: all nodes), reading buffer `buf`.
// Appends to litems at C_NL and advances the leaf cursor (host twin: the collect lambda of grow_group).
// The planner's per-node scratch arrays (global memory, or dynamic LDS when the level capacity fits).
struct PlanScratch {
  int64_t *sa, *sb, *sc, *sd, *se, *sf, *sg;
  int32_t* flag;
};

__device__ void emit_leaves(const PlanArgs& A, const PlanScratch& Z, int lvl, int n, const int32_t* split, int buf,
                            int64_t* sh) {
  const int t = threadIdx.x, nt = blockDim.x;
  const int64_t* cnt_ = A.lv_count[lvl];
  for (int i = t; i < n; i += nt) {
    const bool leaf = split == nullptr || split[i] == 0;
    const int64_t c = cnt_[i];
    Z.sd[i] = leaf && c > 0 ? c : 0;
    Z.se[i] = leaf && c > 0 ? cdiv(c, A.chunk_rows) : 0;
  }
  __syncthreads();
  const int64_t lbase = *A.leaf_pos;
  const int64_t nl0 = A.cnt[C_NL];
  __syncthreads();
  int64_t* const arr[2] = {Z.sd, Z.se};
  int64_t tots[2];
  block_scan_multi<2>(arr, n, tots, sh);
  const int64_t tot_rows = tots[0], tot_items = tots[1];
  const int64_t n_emit = min(tot_items, A.cap_l - nl0);
  for (int64_t k = t; k < n_emit; k += nt) {
    const int64_t i = owner(Z.se, n, k);
    const int64_t o = (k - Z.se[i]) * A.chunk_rows;
    LeafItemH it;
    it.begin = A.lv_begin[lvl][i] + o;
    it.count = min((int64_t)A.chunk_rows, cnt_[i] - o);
    it.out = lbase + Z.sd[i] + o;
    it.gid = A.lv_gid[lvl][i];
    it.pad = buf;
    A.litems[nl0 + k] = it;
  }
  __syncthreads();
  if (t == 0) {
    *A.leaf_pos = lbase + tot_rows;
    A.cnt[C_NL] = (int)(nl0 + n_emit);
    if (n_emit < tot_items) A.cnt[C_ERR] |= 2;
  }
  __syncthreads();
}

// One level of planning. d > 0 first turns level d - 1's device decisions (split_find + partition) into
// the tree records, the leaf items of its non-splitting nodes and the children (level d); then level d's
// work lists are built. Host twin: common/tree_grow.hpp grow_group (GPU backend, no feature subsets).
constexpr int kPlanScratch = 7;     // int64 per-node scratch arrays of the planner (sa .. sg) + one int32 (flag)

__global__ void __launch_bounds__(1024) level_plan_kernel(PlanArgs A) {
  __shared__ int64_t sh[1024];
  // the per-node scratch arrays live in LDS when the level capacity fits (A.lds_cap > 0): every scan, owner
  // search and flag read of the plan is then an LDS access instead of an L2 round trip
  extern __shared__ int64_t dyn_scratch[];
  // the plan is the serial link between two levels of this tree while its CU usually also runs other boosting
  // parts' histogram waves: issue priority over them
  __builtin_amdgcn_s_setprio(3);
  PlanScratch Z{A.sa, A.sb, A.sc, A.sd, A.se, A.sf, A.sg, A.flag};
  if (A.lds_cap > 0) {
    int64_t* base = dyn_scratch;
    Z = PlanScratch{base, base + A.lds_cap, base + 2 * A.lds_cap, base + 3 * A.lds_cap, base + 4 * A.lds_cap,
                    base + 5 * A.lds_cap, base + 6 * A.lds_cap, reinterpret_cast<int32_t*>(base + 7 * A.lds_cap)};
  }
  __shared__ int s_n_prev, s_m_prev, s_created;
  const int t = threadIdx.x, nt = blockDim.x;
  const int d = A.d, S = A.S, T = A.T;
  auto R = [&](int64_t g) { return A.rec + (g + 1) * (int64_t)A.W; };
  uint64_t t_prev = 0;
  if (A.profile && t == 0) {
    t_prev = wall_clock64();
    atomicAdd(&g_plan_prof[31], 1ull);
  }
  auto mark = [&](int k) {
    if (A.profile && t == 0) {
      const uint64_t now = wall_clock64();
      atomicAdd(&g_plan_prof[k], (unsigned long long)(now - t_prev));
      t_prev = now;
    }
  };
  if (t == 0) {
    s_n_prev = d > 0 ? A.cnt[C_N] : 0;
    s_m_prev = d > 0 ? A.cnt[C_M] : 0;
    s_created = d > 0 ? A.cnt[C_NCREATED] : 0;
  }
  __syncthreads();
  if (t == 0) {
    A.cnt[C_NL] = 0;
    if (d == 0) {
      A.cnt[C_ERR] = 0;
      *A.leaf_pos = 0;
    }
  }
  __syncthreads();
  int n = 0;
  const int C = d & 1;
  if (d == 0) {
    if (t == 0) {
      int64_t b = 0;
      for (int j = 0; j < T; ++j) {
        A.lv_tree[0][j] = j;
        A.lv_gid[0][j] = j;
        A.lv_begin[0][j] = b;
        A.lv_count[0][j] = A.j_count[j];
        b += A.j_count[j];
      }
      A.cnt[C_NCREATED] = T;
      A.level_off[0] = 0;
    }
    for (int j = t; j < T; j += nt) init_node(R(j), j, S);
    n = T;
    __syncthreads();
    mark(0);
  } else {
    const int P = (d - 1) & 1;
    const int n_prev = s_n_prev;
    if (t == 0) A.level_off[d] = s_created;
    if (n_prev == 0) {
      if (t == 0) {
        for (int k = C_N; k <= C_NZD; ++k) A.cnt[k] = 0;
      }
      return;
    }
    // (a) per node of level d - 1 (loc[i] = its histogram node j, or -1): node totals, split flag, leaf work
    const int64_t* pcnt = A.lv_count[P];
    for (int i = t; i < n_prev; i += nt) {
      const int j = A.loc[i];
      bool split = false;
      if (j >= 0) {
        int64_t* r = R(A.lv_gid[P][i]);
        for (int s = 0; s < S; ++s) r[kRecFixed + s] = dbits((double)A.r_tot[(int64_t)j * S + s]);
        const float* Pp = A.par[P] + (int64_t)j * 8;
        split = Pp[7] > 0.5f && A.r_feat[j] >= 0 && A.r_gain[j] > Pp[6];
      }
      const int64_t c = pcnt[i];
      const bool leaf = !split && c > 0;
      Z.sd[i] = leaf ? c : 0;
      Z.se[i] = leaf ? cdiv(c, A.chunk_rows) : 0;
      Z.sf[i] = split ? 1 : 0;
      Z.flag[i] = split ? 1 : 0;
    }
    __syncthreads();
    mark(1);
    const int64_t lbase = *A.leaf_pos;
    const int64_t nl0 = A.cnt[C_NL];
    int64_t* const arr3[3] = {Z.sd, Z.se, Z.sf};
    int64_t tot3[3];
    block_scan_multi<3>(arr3, n_prev, tot3, sh);
    const int64_t tot_rows = tot3[0], tot_items = tot3[1], ns = tot3[2];
    mark(2);
    const int base = s_created;
    if (2 * ns > A.cap_nl || base + 2 * ns > A.cap_nodes) {   // (cannot happen: caps bound every level)
      if (t == 0) {
        A.cnt[C_ERR] |= 2;
        A.cnt[C_N] = 0;
        for (int k = C_M; k <= C_NZD; ++k) A.cnt[k] = 0;
      }
      return;
    }
    // (b) leaf items of the nodes that do not split (read from the buffer level d - 1 read)
    const int64_t n_emit = min(tot_items, A.cap_l - nl0);
    for (int64_t k = t; k < n_emit; k += nt) {
      const int64_t i = owner(Z.se, n_prev, k);
      const int64_t o = (k - Z.se[i]) * A.chunk_rows;
      LeafItemH it;
      it.begin = A.lv_begin[P][i] + o;
      it.count = min((int64_t)A.chunk_rows, pcnt[i] - o);
      it.out = lbase + Z.sd[i] + o;
      it.gid = A.lv_gid[P][i];
      it.pad = P;
      A.litems[nl0 + k] = it;
    }
    // (c) splits -> records + children (level d), in split order
    for (int i = t; i < n_prev; i += nt) {
      if (!Z.flag[i]) continue;
      const int j = A.loc[i];
      const int64_t q = Z.sf[i];
      int64_t* r = R(A.lv_gid[P][i]);
      r[1] = A.r_feat[j];
      r[2] = A.r_bin[j];
      r[3] = A.r_dl[j];
      r[4] = dbits((double)A.r_gain[j]);
      const int64_t ncnt = pcnt[i];
      const int64_t nl = A.r_cur[2 * j];
      if (nl < 0 || nl + A.r_cur[2 * j + 1] != ncnt) A.cnt[C_ERR] |= 1;
      const int64_t gl = base + 2 * q, gr = gl + 1;
      r[5] = gl;
      r[6] = gr;
      const int tree = A.lv_tree[P][i];
      int64_t* rl = R(gl);
      int64_t* rr = R(gr);
      init_node(rl, tree, S);
      init_node(rr, tree, S);
      for (int s = 0; s < S; ++s) {
        const double lt = (double)A.r_left[(int64_t)j * S + s];
        const double tt = (double)A.r_tot[(int64_t)j * S + s];
        rl[kRecFixed + s] = dbits(lt);
        rr[kRecFixed + s] = dbits(tt - lt);
      }
      const int64_t b0 = A.lv_begin[P][i];
      A.lv_tree[C][2 * q] = tree;
      A.lv_gid[C][2 * q] = (int32_t)gl;
      A.lv_begin[C][2 * q] = b0;
      A.lv_count[C][2 * q] = nl;
      A.lv_tree[C][2 * q + 1] = tree;
      A.lv_gid[C][2 * q + 1] = (int32_t)gr;
      A.lv_begin[C][2 * q + 1] = b0 + nl;
      A.lv_count[C][2 * q + 1] = ncnt - nl;
      A.ppo[q] = A.nho[P][j];
    }
    n = (int)(2 * ns);
    if (t == 0) {
      *A.leaf_pos = lbase + tot_rows;
      A.cnt[C_NL] = (int)(nl0 + n_emit);
      if (n_emit < tot_items) A.cnt[C_ERR] |= 2;
      A.cnt[C_NCREATED] = base + n;
    }
    __syncthreads();
    mark(3);
  }
  if (n == 0) {
    if (t == 0) {
      A.cnt[C_N] = 0;
      for (int k = C_M; k <= C_NZD; ++k) A.cnt[k] = 0;
    }
    return;
  }
  // ---- plan level d, one pass over sibling pairs (level 0: over the roots). Per node i: flag bits
  // 1 = can split, 2 = needs a histogram, 4 = left node of a histogram pair, 8 = the pair's derived (big) node;
  // counts for one multi-scan: sa need, sb wide-load hist items, sc other hist items, sd partition items,
  // se whole-node zero segments, sf CSR-region zero segments, sg pairs (at the left node)
  const int32_t* ltree = A.lv_tree[C];
  const int64_t* lcnt = A.lv_count[C];
  const bool dense_split = A.live_dense >= 0 && A.live_dense < A.hsz;
  auto can_split = [&](int i) {
    const int jt = ltree[i];
    const int64_t c = lcnt[i];
    bool can = d < A.j_depth[jt] && c >= 2 && (double)c >= 2 * A.j_inst[jt] - 1e-9;
    if (can && A.newton && d > 0 && A.j_mcw[jt] > 0 &&
        bitsd(R(A.lv_gid[C][i])[kRecFixed + 1]) < 2.0 * A.j_mcw[jt] * (1.0 - 1e-6))
      can = false;
    return can;
  };
  auto counts = [&](int i, int fl) {
    const bool need = fl & 2;
    const int64_t c = lcnt[i];
    const int64_t nch = max((int64_t)1, cdiv(c, A.chunk_rows));
    const int64_t ncsr = max((int64_t)1, cdiv(c, tmog::kCsrRows));
    const bool build = need && !(fl & 8);
    int64_t wide = 0, other = 0;
    bool has_csr = false;
    if (build)
      for (int g = 0; g < A.n_groups; ++g) {
        const int gfl = A.groups[g].z;
        const bool reg = gfl & 1, csr = gfl & 2, wd = gfl & 4;
        const int64_t k = (csr ? ncsr : nch) * ((csr || reg) ? 1 : A.n_sc);
        if (wd) wide += k;
        else other += k;
        has_csr |= csr;
      }
    Z.flag[i] = fl;
    Z.sa[i] = need ? 1 : 0;
    Z.sb[i] = wide;
    Z.sc[i] = other;
    Z.sd[i] = need ? max((int64_t)1, cdiv(c, tmog::kPartRows)) : 0;
    Z.se[i] = build && (nch > 1 || (has_csr && ncsr > 1 && !dense_split)) ? 1 : 0;
    Z.sf[i] = build && nch == 1 && has_csr && ncsr > 1 && dense_split ? 1 : 0;
    Z.sg[i] = (fl & 4) ? 1 : 0;
  };
  if (d == 0) {
    for (int i = t; i < n; i += nt) counts(i, (can_split(i) ? 1 : 0) | 2);
  } else {
    for (int q = t; 2 * q + 1 < n; q += nt) {
      const int li = 2 * q, ri = li + 1;
      const bool cl = can_split(li), cr = can_split(ri);
      bool nl = cl, nr = cr;
      // subtraction pairing: when one sibling needs a histogram, the other gets one too if it is the smaller
      // (built) one -- then the bigger one is derived from the parent
      if (nl != nr && lcnt[li] >= 1 && lcnt[ri] >= 1 && (cl ? lcnt[ri] <= lcnt[li] : lcnt[li] <= lcnt[ri]))
        nl = nr = true;
      const bool pair = nl && nr;
      const bool left_big = lcnt[li] >= lcnt[ri];
      counts(li, (cl ? 1 : 0) | (nl ? 2 : 0) | (pair ? 4 : 0) | (pair && left_big ? 8 : 0));
      counts(ri, (cr ? 1 : 0) | (nr ? 2 : 0) | (pair && !left_big ? 8 : 0));
    }
  }
  __syncthreads();
  mark(4);
  int64_t* const arr7[7] = {Z.sa, Z.sb, Z.sc, Z.sd, Z.se, Z.sf, Z.sg};
  int64_t tot7[7];
  block_scan_multi<7>(arr7, n, tot7, sh);
  const int m = (int)tot7[0];
  const int64_t n_wide = tot7[1], n_other = tot7[2], n_part = tot7[3], n_zw = tot7[4], n_zc = tot7[5];
  const int n_pairs = (int)tot7[6];
  mark(5);
  if (m > A.cap_m) {                       // (cannot happen: caps bound every level)
    if (t == 0) {
      A.cnt[C_ERR] |= 2;
      A.cnt[C_N] = 0;
      for (int k = C_M; k <= C_NZD; ++k) A.cnt[k] = 0;
    }
    return;
  }
  if (m == 0) {                            // nothing to scan: every node of level d is a leaf
    for (int i = t; i < n; i += nt) A.loc[i] = -1;
    emit_leaves(A, Z, C, n, nullptr, C, sh);
    if (t == 0) {
      A.cnt[C_N] = 0;
      for (int k = C_M; k <= C_NZD; ++k) A.cnt[k] = 0;
    }
    return;
  }
  // ---- emission: per-node tables (histogram node j = need prefix, in node order), pairs, zero segments
  for (int i = t; i < n; i += nt) {
    const int fl = Z.flag[i];
    if (!(fl & 2)) {
      A.loc[i] = -1;
      continue;
    }
    const int j = (int)Z.sa[i];
    const int jt = ltree[i];
    A.hn[C][j] = i;
    A.loc[i] = j;
    A.nmd[C][j] = A.j_model[jt];
    A.nho[C][j] = (int64_t)j * A.hsz;
    A.nb[C][j] = A.lv_begin[C][i];
    A.nc[C][j] = lcnt[i];
    A.nfo[j] = 0;
    A.nnf[j] = A.F_use;
    const bool paired = d > 0 && (((i & 1) == 0 && (fl & 4)) || ((i & 1) == 1 && (Z.flag[i - 1] & 4)));
    float* Pp = A.par[C] + (int64_t)j * 8;
    Pp[0] = (float)A.j_inst[jt];
    Pp[1] = (float)A.j_gain[jt];
    Pp[2] = (float)A.j_mcw[jt];
    Pp[3] = (float)A.j_lam[jt];
    Pp[4] = paired ? 1.f : 0.f;             // pair_fuse: the pair scan derives / scans both siblings
    Pp[5] = A.has_missing ? 1.f : 0.f;
    Pp[6] = (float)A.j_eps[jt];
    Pp[7] = (fl & 1) ? 1.f : 0.f;
    if (fl & 4) {                          // left node of a pair: (small, big) histogram nodes, parent offset
      const int jr = (int)Z.sa[i + 1];
      const bool left_big = fl & 8;
      const int64_t k = Z.sg[i];
      A.sj[k] = left_big ? jr : j;
      A.bj[k] = left_big ? j : jr;
      A.poff[k] = A.ppo[i >> 1];
    }
    const bool zw = (i + 1 < n ? Z.se[i + 1] : n_zw) != Z.se[i];
    const bool zc = (i + 1 < n ? Z.sf[i + 1] : n_zc) != Z.sf[i];
    if (zw) {
      A.zoff[Z.se[i]] = (int64_t)j * A.hsz;
      A.zsize[Z.se[i]] = A.hsz;
    }
    if (zc) {
      A.zoff[n_zw + Z.sf[i]] = (int64_t)j * A.hsz + A.live_dense;
      A.zsize[n_zw + Z.sf[i]] = A.hsz - A.live_dense;
    }
  }
  mark(6);
  const int64_t n_hist = n_wide + n_other;
  const int64_t h_emit = min(n_hist, A.cap_h), c_emit = min(n_part, A.cap_c);
  // histogram items, wide-load items first (the host's stable partition), then the others
  for (int64_t k = t; k < h_emit; k += nt) {
    const bool wsec = k < n_wide;
    const int64_t* pre = wsec ? Z.sb : Z.sc;
    const int64_t kk = wsec ? k : k - n_wide;
    const int64_t i = owner(pre, n, kk);
    int64_t local = kk - pre[i];
    const int64_t c = lcnt[i];
    const int64_t nch = max((int64_t)1, cdiv(c, A.chunk_rows));
    const int64_t ncsr = max((int64_t)1, cdiv(c, tmog::kCsrRows));
    const int64_t b0 = A.lv_begin[C][i];
    const int32_t j = (int32_t)Z.sa[i];
    for (int g = 0; g < A.n_groups; ++g) {
      const int4 gr = A.groups[g];
      const bool reg = gr.z & 1, csr = gr.z & 2, wd = gr.z & 4;
      if (wd != wsec) continue;
      const int64_t nit = csr ? ncsr : nch;
      const int64_t nchunk = (csr || reg) ? 1 : A.n_sc;
      if (local >= nit * nchunk) {
        local -= nit * nchunk;
        continue;
      }
      const int64_t sc_ = local / nit, ci = local - sc_ * nit;
      const int64_t step = csr ? tmog::kCsrRows : A.chunk_rows;
      HistItemH h;
      h.node = j;
      h.fg0 = gr.x;
      h.nf = gr.y;
      h.excl = (nit == 1 ? 1 : 0) | (reg ? 2 : 0) | (csr ? 4 : 0) | (wd ? 16 : 0) |
               ((reg || csr) && A.live_dense >= 0 ? 8 : 0) | (int32_t)(sc_ << 8);
      h.begin = b0 + ci * step;
      h.count = min(step, c - ci * step);
      A.hitems[k] = h;
      break;
    }
  }
  // partition items of every scanned node (kPartRows-row slices)
  for (int64_t k = t; k < c_emit; k += nt) {
    const int64_t i = owner(Z.sd, n, k);
    const int64_t ci = k - Z.sd[i];
    const int64_t c = lcnt[i];
    PartItemH pi;
    pi.node = (int32_t)Z.sa[i];
    pi.pad = 0;
    pi.begin = A.lv_begin[C][i] + ci * tmog::kPartRows;
    pi.count = min((int64_t)tmog::kPartRows, c - ci * tmog::kPartRows);
    pi.out_left = pi.out_right = 0;
    A.citems[k] = pi;
  }
  if (t == 0) {
    A.cnt[C_N] = n;
    A.cnt[C_M] = m;
    A.cnt[C_NP] = n_pairs;
    A.cnt[C_NH] = (int)h_emit;
    A.cnt[C_NC] = (int)c_emit;
    A.cnt[C_NZ] = (int)(n_zw + n_zc);
    A.cnt[C_NZD] = (int)n_zw;
    if (h_emit < n_hist || c_emit < n_part) A.cnt[C_ERR] |= 2;
  }
  mark(7);
}

struct FinArgs {
  int T, S, mode, kind, n_levels;
  int prune;                   // some job has gamma > 0 (Newton): pruning can happen
  int64_t* rec;
  int W;
  const int32_t* level_off;
  const int* cnt;
  const int64_t* leaf_pos;
  const double* j_lam;
  const double* j_eta;
  const double* j_gamma;
  float* gid_value;
  int64_t* gid_tree;
  int64_t* left_w;
  int64_t* right_w;
  int64_t* parent;
  int32_t* reach;
  double* value;
};

// Device twin of tmog_tree_finalize_cpu's values / gamma pruning / gid values (ops/csrc/host/tree_cpu.cpp):
// the leaf output of every created node id for the boosting epilogue, a pruned node's descendants taking
// their kept ancestor's value. The host rebuilds the Forest from the same records with tree_cpu.cpp.
// Pruning bottom-up level by level is the sequential reverse-id loop (children have higher ids than parents).
__global__ void __launch_bounds__(1024) tree_finalize_kernel(FinArgs A) {
  __builtin_amdgcn_s_setprio(3);            // serial link between two boosting rounds (see level_plan_kernel)
  const int t = threadIdx.x, nt = blockDim.x;
  const int64_t n = A.cnt[C_NCREATED];
  auto R = [&](int64_t g) { return A.rec + (g + 1) * (int64_t)A.W; };
  if (!(A.kind == 3 && A.prune)) {
    // nothing can be pruned (no gamma > 0: a recorded split's gain exceeds split_eps > 0), so every created
    // node is reachable and keeps its own value: one pass, no level loops
    for (int64_t i = t; i < n; i += nt) {
      const int64_t* r = R(i);
      const int64_t jt = r[0];
      const double t0 = bitsd(r[kRecFixed]);
      const double t1 = A.S > 1 ? bitsd(r[kRecFixed + 1]) : 0.0;
      double v;
      if (A.mode == 1) v = t0 > 0 ? t1 / fmax(t0, 1e-300) : 0.0;
      else v = -t0 / (t1 + A.j_lam[jt]) * A.j_eta[jt];
      A.gid_value[i] = (float)v;
      A.gid_tree[i] = jt;
    }
    if (t == 0) {
      A.rec[0] = n;
      A.rec[1] = *A.leaf_pos;
      A.rec[2] = A.cnt[C_ERR];
    }
    return;
  }
  for (int64_t i = t; i < n; i += nt) {
    const int64_t* r = R(i);
    const int64_t jt = r[0];
    const double t0 = bitsd(r[kRecFixed]);
    const double t1 = A.S > 1 ? bitsd(r[kRecFixed + 1]) : 0.0;
    double v;
    if (A.mode == 1) v = t0 > 0 ? t1 / fmax(t0, 1e-300) : 0.0;
    else v = -t0 / (t1 + A.j_lam[jt]) * A.j_eta[jt];
    A.value[i] = v;
    A.left_w[i] = r[5];
    A.right_w[i] = r[6];
    A.parent[i] = -1;
    A.reach[i] = i < A.T ? 1 : 0;
  }
  __syncthreads();
  for (int64_t i = t; i < n; i += nt) {
    const int64_t* r = R(i);
    if (r[5] >= 0) {
      A.parent[r[5]] = i;
      A.parent[r[6]] = i;
    }
  }
  __syncthreads();
  auto lvl_lo = [&](int L) { return (int64_t)A.level_off[L]; };
  auto lvl_hi = [&](int L) { return L + 1 < A.n_levels ? (int64_t)A.level_off[L + 1] : n; };
  if (A.kind == 3) {
    for (int L = A.n_levels - 1; L >= 0; --L) {
      for (int64_t i = lvl_lo(L) + t; i < lvl_hi(L); i += nt) {
        const int64_t l = A.left_w[i];
        if (l < 0) continue;
        const int64_t r = A.right_w[i];
        const int64_t* rr = R(i);
        if (A.left_w[l] < 0 && A.left_w[r] < 0 && bitsd(rr[4]) < A.j_gamma[rr[0]]) {
          A.left_w[i] = -1;
          A.right_w[i] = -1;
        }
      }
      __syncthreads();
    }
  }
  for (int L = 0; L < A.n_levels; ++L) {
    for (int64_t i = lvl_lo(L) + t; i < lvl_hi(L); i += nt)
      if (A.reach[i] && A.left_w[i] >= 0) {
        A.reach[A.left_w[i]] = 1;
        A.reach[A.right_w[i]] = 1;
      }
    __syncthreads();
  }
  for (int L = 0; L < A.n_levels; ++L) {
    for (int64_t i = lvl_lo(L) + t; i < lvl_hi(L); i += nt) {
      const int64_t p = A.parent[i];
      A.gid_value[i] = (A.reach[i] || p < 0) ? (float)A.value[i] : A.gid_value[p];
      A.gid_tree[i] = R(i)[0];
    }
    __syncthreads();
  }
  if (t == 0) {
    A.rec[0] = n;
    A.rec[1] = *A.leaf_pos;
    A.rec[2] = A.cnt[C_ERR];
  }
}

inline void hchk(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
inline void kchk(int rc, const char* what) {
  if (rc != 0) throw std::runtime_error(std::string("kernel ") + what + " failed with code " + std::to_string(rc));
}

// Per-slot device resources of the resident grower (grow-only; stream-ordered allocations on the caller's
// stream, which every use of the slot is ordered on).
struct Buf {
  uint8_t* p = nullptr;
  size_t cap = 0;
  void need(size_t bytes, hipStream_t s) {     // dev_alloc.hpp: a failed growth leaves the buffer empty
    tmog::grow_device(p, cap, bytes, bytes + bytes / 4 + 4096, s);
  }
};

struct ResSlot {
  Buf arena, hist0, hist1, cand, done, res, consts, fp_send, fp_recv;
  uint8_t* pin = nullptr;      // pinned staging of the per-call constants
  size_t pin_cap = 0;
  hipEvent_t copied = nullptr;
  std::vector<uint8_t> last;   // constants last shipped (skipped when unchanged)
  const uint8_t* done_zeroed = nullptr;   // the ticket-counter block last zeroed (a new block is zeroed again)
  int device = -1;
};

std::vector<ResSlot>& res_slots() {
  static std::vector<ResSlot> s(32);
  return s;
}

thread_local std::string g_err;

struct Carve {
  uint8_t* base;
  size_t off = 0;
  template <class T>
  T* take(int64_t n) {
    off = (off + 255) & ~size_t(255);
    T* p = reinterpret_cast<T*>(base + off);
    off += sizeof(T) * (size_t)std::max<int64_t>(n, 1);
    return p;
  }
};

struct Caps {
  int D = 0;
  std::vector<int64_t> nmax;   // nodes per level bound, d = 0..D + 1 (level D + 1 is empty)
  int64_t cap_nl = 0, cap_m = 0, cap_nodes = 0, cap_h = 0, cap_c = 0, cap_l = 0;
};

Caps caps_of(const tmog::GrowArgs& a, const tmog::GroupLayout& L, int n_sc) {
  Caps c;
  const int T = a.T;
  int64_t total = 0;
  for (int j = 0; j < T; ++j) {
    total += a.job_count[j];
    c.D = std::max(c.D, (int)a.job_depth[j]);
  }
  c.nmax.assign(c.D + 2, 0);
  for (int d = 0; d <= c.D; ++d) {
    int64_t s = 0;
    for (int j = 0; j < T; ++j)
      if (d <= a.job_depth[j]) s += std::min(d >= 40 ? a.job_count[j] : ((int64_t)1 << d), std::max<int64_t>(a.job_count[j], 1));
    c.nmax[d] = std::max<int64_t>(1, std::min<int64_t>(s, std::max<int64_t>(total, T)));
    c.cap_nl = std::max(c.cap_nl, c.nmax[d]);
    if (d < c.D || d == 0) c.cap_m = std::max(c.cap_m, c.nmax[d]);   // levels that build histograms
    c.cap_nodes += c.nmax[d];
  }
  c.cap_m = std::max<int64_t>(c.cap_m, 1);
  for (const tmog::FeatGroup& g : L.full_groups) {
    const int64_t step = g.csr ? tmog::kCsrRows : a.chunk_rows;
    c.cap_h += ((g.csr || g.reg) ? 1 : n_sc) * (total / step + c.cap_m + 1);
  }
  c.cap_c = total / tmog::kPartRows + c.cap_m + 1;
  c.cap_l = 2 * (total / std::max<int64_t>(a.chunk_rows, 1) + c.cap_nl + 1);
  return c;
}

// per-level grid bounds
int64_t hist_bound(const tmog::GrowArgs& a, const tmog::GroupLayout& L, int n_sc, int64_t total, int64_t m) {
  int64_t h = 0;
  for (const tmog::FeatGroup& g : L.full_groups) {
    const int64_t step = g.csr ? tmog::kCsrRows : a.chunk_rows;
    h += ((g.csr || g.reg) ? 1 : n_sc) * (total / step + m + 1);
  }
  return h;
}

// Configurations the device plan covers (everything else stays on the host-planned grower): one job group,
// no per-node feature subsets, subtraction + fused pair scan, narrow split scan with the fused reduction,
// statistics in one histogram chunk, leaves collected, Newton (MODE 2) or variance (MODE 1) values.
// Feature-parallel growth is covered: the level's split records are all-gathered and merged on the stream
// (RCCL, or the local answer of a projected rank group) between split-find and partition, so a spread job's
// levels need no host round trip either. Returns an empty string when supported.
std::string unsupported(const tmog::GrowArgs& a) {
  if (a.n_groups != 1) return "more than one job group";
  if (a.fp_world > 0 && a.fp_comm == nullptr) return "feature-parallel without a communicator array";
  if (!a.collect_leaves) return "leaves not collected";
  if (!a.subtract) return "no subtraction";
  if (a.mode == 0) return "class-count histograms";
  if (a.S > 16 || a.B > 64) return "wide statistics";
  for (int j = 0; j < a.T; ++j) {
    const int k = a.job_fsub[j];
    if (k > 0 && k < a.F) return "per-node feature subsets";
  }
  const char* ps = std::getenv("TMOG_PAIR_SCAN");
  if (ps && ps[0] == '0') return "pair scan disabled";
  const char* fr = std::getenv("TMOG_FUSED_REDUCE");
  if (fr && fr[0] == '0') return "fused reduction disabled";
  const char* ws = std::getenv("TMOG_HIST_WIDE_SPLIT");
  if (ws && ws[0] == '1') return "split wide-load launches";
  if (tmog_hip_hist_stat_chunk(a.B, a.S) < a.S) return "chunked statistics";
  return "";
}

}  // namespace

extern "C" {

// Outputs of one device-planned tree (models/tree_engine.py _ResidentIO).
struct ResidentIO {
  int64_t* rec;          // [1 + cap_nodes][7 + S] int64: header (nodes, leaf entries, error bits), then node records
  float* gid_value;      // [cap_nodes] leaf output per created node id (pruning applied)
  int64_t* gid_tree;     // [cap_nodes] job of each created node
  int64_t cap_nodes;
  const double* job_eta;    // [T]
  const double* job_gamma;  // [T]
};

int64_t tmog_hip_resident_cap_nodes(const tmog::GrowArgs* args) {
  const tmog::GrowArgs& a = *args;
  if (!unsupported(a).empty()) return -1;
  const tmog::GroupLayout L = tmog::group_layout<true>(a, false, a.fp_world > 0);
  return caps_of(a, L, 1).cap_nodes;
}

// TMOG_PLAN_PROFILE: copy the planner's per-phase tick sums (32 entries, 100 MHz wall clock; [31] = calls).
int tmog_hip_plan_profile(uint64_t* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_plan_prof), sizeof(unsigned long long) * 32, 0,
                                     hipMemcpyDeviceToHost);
  if (e != hipSuccess) return (int)e;
  if (reset) {
    static const unsigned long long zero[32] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_plan_prof), zero, sizeof(zero), 0, hipMemcpyHostToDevice);
  }
  return (int)e;
}

int tmog_hip_resident_error(char* msg, int cap) {
  if (msg && cap > 0) {
    std::strncpy(msg, g_err.c_str(), cap - 1);
    msg[cap - 1] = 0;
  }
  return (int)g_err.size();
}

// Enqueue the growth of one tree per job of the (single) group on a.stream. Returns 0 when enqueued,
// 1 when the configuration is not covered (nothing enqueued; use tmog_hip_grow_forest), -1 on error
// (tmog_hip_resident_error). No host synchronisation with the device.
int tmog_hip_grow_resident(const tmog::GrowArgs* args, const ResidentIO* io) {
  g_err.clear();
  try {
    const tmog::GrowArgs& a = *args;
    const std::string why = unsupported(a);
    if (!why.empty()) {
      g_err = why;
      return 1;
    }
    const int T = a.T, S = a.S, B = a.B;
    if (a.slot_base < 0 || a.slot_base >= (int)res_slots().size()) throw std::runtime_error("bad slot");
    hipStream_t st = (hipStream_t)a.stream;
    int dev = 0;
    hchk(hipGetDevice(&dev), "hipGetDevice");
    (void)tmog_hip_tree_prime();
    ResSlot& sl = res_slots()[a.slot_base];
    if (sl.device != dev) {
      sl = ResSlot();
      sl.device = dev;
    }
    const bool fp = a.fp_world > 0;
    const tmog::GroupLayout L = tmog::group_layout<true>(a, false, fp);
    const int n_sc = 1;
    const Caps cp = caps_of(a, L, n_sc);
    if (io->cap_nodes < cp.cap_nodes) throw std::runtime_error("record buffer too small");
    int64_t total = 0;
    for (int j = 0; j < T; ++j) total += a.job_count[j];
    const int F_use = L.F_use;
    const int64_t hsz = (int64_t)F_use * B * S;
    const int W = kRecFixed + S;
    // ---- per-call constants: groups, feature list, job table (shipped only when they change)
    std::vector<int4> groups;
    bool need_general = false;
    for (const tmog::FeatGroup& g : L.full_groups) {
      groups.push_back(make_int4(g.f0, g.nf, (g.reg ? 1 : 0) | (g.csr ? 2 : 0) | (g.wide ? 4 : 0), 0));
      need_general |= !g.csr && !g.wide;
    }
    std::vector<int32_t> flist(F_use);
    for (int f = 0; f < F_use; ++f) flist[f] = L.perm_feats.empty() ? f : L.perm_feats[f];
    tmog::Staging cs;
    const size_t o_groups = cs.add(groups), o_flist = cs.add(flist);
    const size_t o_depth = cs.add(a.job_depth, 4 * (size_t)T), o_model = cs.add(a.job_model, 4 * (size_t)T);
    const size_t o_count = cs.add(a.job_count, 8 * (size_t)T), o_inst = cs.add(a.job_min_inst, 8 * (size_t)T);
    const size_t o_gain = cs.add(a.job_min_gain, 8 * (size_t)T), o_mcw = cs.add(a.job_mcw, 8 * (size_t)T);
    const size_t o_lam = cs.add(a.job_lambda, 8 * (size_t)T), o_eps = cs.add(a.job_eps, 8 * (size_t)T);
    const size_t o_eta = cs.add(io->job_eta, 8 * (size_t)T), o_gam = cs.add(io->job_gamma, 8 * (size_t)T);
    const uint8_t* consts_before = sl.consts.p;
    sl.consts.need(cs.buf.size(), st);
    if (sl.consts.p != consts_before) sl.last.clear();     // a new block holds nothing yet
    if (cs.buf != sl.last) {
      if (sl.copied) hchk(hipEventSynchronize(sl.copied), "constants copy wait");
      else hchk(hipEventCreateWithFlags(&sl.copied, hipEventDisableTiming), "event");
      if (sl.pin_cap < cs.buf.size() || sl.pin == nullptr) {
        if (sl.pin) {
          hipError_t e = hipHostFree(sl.pin);
          sl.pin = nullptr;
          sl.pin_cap = 0;
          hchk(e, "hipHostFree");
        }
        hchk(hipHostMalloc((void**)&sl.pin, cs.buf.size() + 4096, hipHostMallocDefault), "hipHostMalloc");
        sl.pin_cap = cs.buf.size() + 4096;
      }
      std::memcpy(sl.pin, cs.buf.data(), cs.buf.size());
      hchk(hipMemcpyAsync(sl.consts.p, sl.pin, cs.buf.size(), hipMemcpyHostToDevice, st), "constants copy");
      hchk(hipEventRecord(sl.copied, st), "event record");
      sl.last = cs.buf;
    }
    const uint8_t* K = sl.consts.p;
    // ---- arena
    auto carve_all = [&](Carve& cv, PlanArgs& P, FinArgs& Fa, int** cnt, int64_t** leaf_pos, int32_t** level_off,
                         int32_t** r_feat, int32_t** r_bin, float** r_gain, float** r_left, float** r_tot,
                         uint8_t** r_dl, int64_t** r_cur) {
      for (int k = 0; k < 2; ++k) {
        P.lv_tree[k] = cv.take<int32_t>(cp.cap_nl);
        P.lv_gid[k] = cv.take<int32_t>(cp.cap_nl);
        P.lv_begin[k] = cv.take<int64_t>(cp.cap_nl);
        P.lv_count[k] = cv.take<int64_t>(cp.cap_nl);
        P.hn[k] = cv.take<int32_t>(cp.cap_m);
        P.nmd[k] = cv.take<int32_t>(cp.cap_m);
        P.nho[k] = cv.take<int64_t>(cp.cap_m);
        P.par[k] = cv.take<float>(8 * cp.cap_m);
        P.nb[k] = cv.take<int64_t>(cp.cap_m);
        P.nc[k] = cv.take<int64_t>(cp.cap_m);
      }
      P.nfo = cv.take<int32_t>(cp.cap_m);
      P.nnf = cv.take<int32_t>(cp.cap_m);
      P.sj = cv.take<int32_t>(cp.cap_m);
      P.bj = cv.take<int32_t>(cp.cap_m);
      P.poff = cv.take<int64_t>(cp.cap_m);
      P.zoff = cv.take<int64_t>(cp.cap_m);
      P.zsize = cv.take<int64_t>(cp.cap_m);
      P.ppo = cv.take<int64_t>(cp.cap_nl);
      P.hitems = cv.take<HistItemH>(cp.cap_h);
      P.citems = cv.take<PartItemH>(cp.cap_c);
      P.litems = cv.take<LeafItemH>(cp.cap_l);
      P.sa = cv.take<int64_t>(cp.cap_nl);
      P.sb = cv.take<int64_t>(cp.cap_nl);
      P.sc = cv.take<int64_t>(cp.cap_nl);
      P.sd = cv.take<int64_t>(cp.cap_nl);
      P.se = cv.take<int64_t>(cp.cap_nl);
      P.sf = cv.take<int64_t>(cp.cap_nl);
      P.sg = cv.take<int64_t>(cp.cap_nl);
      P.flag = cv.take<int32_t>(cp.cap_nl);
      P.loc = cv.take<int32_t>(cp.cap_nl);
      *cnt = cv.take<int>(C_COUNT);
      *leaf_pos = cv.take<int64_t>(1);
      *level_off = cv.take<int32_t>(cp.D + 2);
      *r_feat = cv.take<int32_t>(cp.cap_m);
      *r_bin = cv.take<int32_t>(cp.cap_m);
      *r_gain = cv.take<float>(cp.cap_m);
      *r_left = cv.take<float>((int64_t)S * cp.cap_m);
      *r_tot = cv.take<float>((int64_t)S * cp.cap_m);
      *r_dl = cv.take<uint8_t>(cp.cap_m);
      *r_cur = cv.take<int64_t>(2 * cp.cap_m);
      Fa.left_w = cv.take<int64_t>(cp.cap_nodes);
      Fa.right_w = cv.take<int64_t>(cp.cap_nodes);
      Fa.parent = cv.take<int64_t>(cp.cap_nodes);
      Fa.reach = cv.take<int32_t>(cp.cap_nodes);
      Fa.value = cv.take<double>(cp.cap_nodes);
    };
    PlanArgs P{};
    static const bool plan_prof = [] { const char* e = std::getenv("TMOG_PLAN_PROFILE"); return e && e[0] == '1'; }();
    P.profile = plan_prof ? 1 : 0;
    FinArgs Fa{};
    int* cnt;
    int64_t* leaf_pos;
    int32_t* level_off;
    int32_t *r_feat, *r_bin;
    float *r_gain, *r_left, *r_tot;
    uint8_t* r_dl;
    int64_t* r_cur;
    {
      Carve probe{nullptr};
      carve_all(probe, P, Fa, &cnt, &leaf_pos, &level_off, &r_feat, &r_bin, &r_gain, &r_left, &r_tot, &r_dl, &r_cur);
      sl.arena.need(probe.off + 256, st);
      Carve cv{sl.arena.p};
      carve_all(cv, P, Fa, &cnt, &leaf_pos, &level_off, &r_feat, &r_bin, &r_gain, &r_left, &r_tot, &r_dl, &r_cur);
    }
    sl.hist0.need(sizeof(int64_t) * (size_t)hsz * cp.cap_m, st);
    sl.hist1.need(sizeof(int64_t) * (size_t)hsz * cp.cap_m, st);
    sl.cand.need(tmog_hip_split_cand_bytes((int)cp.cap_m, F_use, B, S), st);
    sl.done.need(sizeof(unsigned) * (size_t)cp.cap_m, st);
    const size_t fp_rb = tmog::fp_rec_bytes(S);
    if (fp) {                                  // split records of this rank / of every rank of the group
      sl.fp_send.need(fp_rb * (size_t)cp.cap_m, st);
      sl.fp_recv.need(fp_rb * (size_t)cp.cap_m * (size_t)a.fp_world, st);
    }
    if (sl.done_zeroed != sl.done.p) {       // ticket counters start (and are left) at zero
      hchk(hipMemsetAsync(sl.done.p, 0, sl.done.cap, st), "memset done");
      sl.done_zeroed = sl.done.p;
    }
    int64_t* hist[2] = {(int64_t*)sl.hist0.p, (int64_t*)sl.hist1.p};
    uint32_t* rows[2] = {a.rows, a.rows_alt};
    int32_t* gh[2] = {a.gh, a.gh_alt};
    const bool use_gh = a.gh != nullptr && a.gh_alt != nullptr && a.mode == 2;
    P.T = T;
    P.S = S;
    P.chunk_rows = (int)a.chunk_rows;
    P.n_groups = (int)groups.size();
    P.n_sc = n_sc;
    P.newton = (a.mode == 2 && a.kind == 3 && S >= 2 && !(std::getenv("TMOG_TREE_HESS_GATE") &&
                                                            std::getenv("TMOG_TREE_HESS_GATE")[0] == '0')) ? 1 : 0;
    P.subtract = 1;
    P.pair_fuse = 1;
    P.F_use = F_use;
    P.hsz = hsz;
    P.live_dense = L.live_dense;
    P.groups = (const int4*)(K + o_groups);
    P.j_depth = (const int32_t*)(K + o_depth);
    P.j_model = (const int32_t*)(K + o_model);
    P.j_count = (const int64_t*)(K + o_count);
    P.j_inst = (const double*)(K + o_inst);
    P.j_gain = (const double*)(K + o_gain);
    P.j_mcw = (const double*)(K + o_mcw);
    P.j_lam = (const double*)(K + o_lam);
    P.j_eps = (const double*)(K + o_eps);
    P.r_feat = r_feat;
    P.r_bin = r_bin;
    P.r_gain = r_gain;
    P.r_left = r_left;
    P.r_tot = r_tot;
    P.r_dl = r_dl;
    P.r_cur = r_cur;
    P.rec = io->rec;
    P.W = W;
    P.level_off = level_off;
    P.cnt = cnt;
    P.leaf_pos = leaf_pos;
    P.cap_nl = cp.cap_nl;
    P.cap_m = cp.cap_m;
    P.cap_nodes = cp.cap_nodes;
    P.cap_h = cp.cap_h;
    P.cap_c = cp.cap_c;
    P.cap_l = cp.cap_l;
    P.has_missing = a.missing_bin >= 0 ? 1 : 0;
    const int32_t* flist_d = (const int32_t*)(K + o_flist);
    // levels 0..D build histograms (level D only when D == 0: deeper, no node of level D may split), and
    // planner scratch in LDS when the per-level node capacity fits (TMOG_PLAN_LDS=0: global memory)
    static const bool plan_lds_ok = [] { const char* e = std::getenv("TMOG_PLAN_LDS"); return !(e && e[0] == '0'); }();
    const size_t per_node = (size_t)kPlanScratch * sizeof(int64_t) + sizeof(int32_t);
    static const bool lds_attr = hipFuncSetAttribute((const void*)level_plan_kernel,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 148 * 1024) ==
                                 hipSuccess;   // once per process (thread-safe static initialisation)
    const bool lds_fit = plan_lds_ok && lds_attr && cp.cap_nl > 0 &&
                         per_node * (size_t)cp.cap_nl + 64 <= (size_t)148 * 1024;
    P.lds_cap = lds_fit ? cp.cap_nl : 0;
    // threads of the two single-workgroup kernels (plan, finalisation); TMOG_PLAN_THREADS = 256 / 512 / 1024: a
    // smaller workgroup finds a CU sooner while the other boosting parts' histogram waves occupy the chip
    static const int plan_nt = [] {
      const char* e = std::getenv("TMOG_PLAN_THREADS");
      const int v = e ? std::atoi(e) : 1024;
      return (v == 256 || v == 512) ? v : 1024;
    }();
    const size_t plan_lds = lds_fit ? per_node * (size_t)cp.cap_nl + 64 : 0;
    // plan D + 1 turns the last decisions into leaves
    for (int d = 0; d <= cp.D + 1; ++d) {
      P.d = d;
      hipLaunchKernelGGL(level_plan_kernel, dim3(1), dim3(plan_nt), plan_lds, st, P);
      kchk((int)hipGetLastError(), "level_plan");
      const int64_t nprev = d > 0 ? cp.nmax[d - 1] : 0;
      const int64_t lbound = (total / std::max<int64_t>(a.chunk_rows, 1) + nprev + 1) +
                             (total / std::max<int64_t>(a.chunk_rows, 1) + cp.nmax[d] + 1);
      kchk(tmog_hip_leaf_collect(rows[0], P.litems, (int)std::min(lbound, cp.cap_l), a.leaf_rows, a.leaf_gid, st,
                                 rows[1], cnt + C_NL),
           "leaf_collect");
      if (d > cp.D || (d == cp.D && d > 0)) continue;
      const int c = d & 1;
      const int64_t mb = cp.nmax[d];
      kchk(tmog_hip_zero_segments(hist[c], P.zoff, P.zsize, (int)mb, hsz, L.live_dense, B * S, S, st, 0, cnt + C_NZ),
           "zero_segments");
      kchk(tmog_hip_hist_build(a.Xb, a.F, rows[c], P.hitems, (int)std::min(hist_bound(a, L, n_sc, total, mb), cp.cap_h),
                               P.nfo, flist_d, P.nmd[c], P.nho[c], hist[c], B, a.mode, S, a.y, a.t1, a.t2, a.stride,
                               a.qscale, a.mode == 2 ? a.missing_bin : -1, a.csr_ptr, a.csr_col, S, 0,
                               need_general ? 1 : 0, st, use_gh ? gh[c] : nullptr, cnt + C_NH, a.wide_rows, a.Xh,
                               a.Fh),
           "hist_build");
      if (d > 0)
        kchk(tmog_hip_pair_scan(hist[c], hist[c ^ 1], P.poff, P.sj, P.bj, (int)std::max<int64_t>(1, mb / 2), P.nho[c],
                                P.nnf, P.nfo, flist_d, a.n_bins, B, S, a.kind, P.par[c], a.missing_bin, P.nmd[c],
                                a.qinv, F_use, sl.cand.p, L.split_n_multi, st, cnt + C_NP),
             "pair_scan");
      kchk(tmog_hip_split_find(hist[c], (int)mb, P.nho[c], P.nnf, P.nfo, flist_d, a.n_bins, B, S, a.kind, P.par[c],
                               a.missing_bin, P.nmd[c], a.qinv, F_use, sl.cand.p, r_feat, r_bin, r_gain, r_dl, r_left,
                               r_tot, r_cur, L.split_n_multi, fp ? sl.fp_send.p : nullptr, fp ? (int64_t)fp_rb : 0,
                               fp ? a.fp_mlo : 0, fp ? L.fp_nml : 0, fp ? L.fp_obase : 0, st, (unsigned*)sl.done.p,
                               cnt + C_M),
           "split_find");
      if (fp) {
        // the ranks' best split per node: all-gather the level's records (the host bound mb of them; the
        // merge reads the device count) and merge them into this level's decisions, all on the stream
        kchk(tmog_hip_fp_allgather(sl.fp_send.p, sl.fp_recv.p, (int64_t)(fp_rb * (size_t)mb), a.fp_comm[0],
                                   a.fp_world, st),
             "fp_allgather");
        kchk(tmog_hip_fp_merge_dev(sl.fp_recv.p, a.fp_world, (int)mb, (int64_t)fp_rb, S, r_feat, r_bin, r_gain,
                                   r_dl, r_left, cnt + C_M, st),
             "fp_merge");
      }
      kchk(tmog_hip_partition_fused(a.Xb, a.F, rows[c], rows[c ^ 1], P.citems,
                                    (int)std::min<int64_t>(total / tmog::kPartRows + mb + 1, cp.cap_c), P.nb[c],
                                    P.nc[c], r_feat, r_bin, r_dl, P.par[c], r_gain, a.missing_bin, r_cur, a.XbT, a.N,
                                    st, use_gh ? gh[c] : nullptr, use_gh ? gh[c ^ 1] : nullptr, cnt + C_NC,
                                    a.wide_rows),
           "partition_fused");
    }
    Fa.T = T;
    Fa.S = S;
    Fa.mode = a.mode;
    Fa.kind = a.kind;
    Fa.n_levels = cp.D + 1;
    Fa.rec = io->rec;
    Fa.W = W;
    Fa.level_off = level_off;
    Fa.cnt = cnt;
    Fa.leaf_pos = leaf_pos;
    Fa.j_lam = P.j_lam;
    Fa.j_eta = (const double*)(K + o_eta);
    Fa.j_gamma = (const double*)(K + o_gam);
    Fa.gid_value = io->gid_value;
    Fa.gid_tree = io->gid_tree;
    Fa.prune = 0;
    for (int j = 0; j < T; ++j) Fa.prune |= io->job_gamma[j] > 0.0 ? 1 : 0;
    hipLaunchKernelGGL(tree_finalize_kernel, dim3(1), dim3(plan_nt), 0, st, Fa);
    kchk((int)hipGetLastError(), "tree_finalize");
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

}  // extern "C"

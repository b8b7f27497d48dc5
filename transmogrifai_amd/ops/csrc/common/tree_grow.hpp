// Native level-synchronous tree grower (host orchestration), shared by the HIP and CPU backends.
//
// This is the runtime half of the histogram tree engine (replaces Spark MLlib's
// per-level RandomForest.findBestSplits driver loop and XGBoost4J's hist updater, e.g.
// OpRandomForestClassifier.scala:59-154, OpGBTClassifier.scala:47-142, OpXGBoostClassifier.scala:47-403).
// One call grows one tree per job, all jobs of a group level by level. Per level the grower plans the
// work items on the host, ships every host array in ONE staged copy, launches the level's kernels
// (histogram, subtraction trick, split scan, partition count), reads every decision back with ONE
// device->host copy, then launches the stable partition and the leaf collection. Job groups run on
// their own host threads and HIP streams, so one group's planning overlaps the other's kernels.
//
// Backends (template parameter BK) provide memory, staging and the kernels:
//   GPU  (hip/tree_grow_hip.hip)   : pinned staging + hipMemcpyAsync, tmog_hip_* launchers
//   CPU  (host/tree_grow_cpu.cpp)  : host memory, tmog_*_cpu functions (bit-identical results)
// Layout contracts are those of hip/tree_kernels.hip (packed rows, int64 fixed-point histograms).
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace tmog {

// Deterministic cross-group order of the feature-parallel split exchanges. Every job group grows on its
// own host thread and issues one all-gather per level on its own communicator; left to the threads'
// timing, rank A could enqueue (g0 level L, g1 level L) while rank B enqueues (g1, g0) -- collectives of
// two communicators queued in different orders on different ranks is the classic RCCL/NCCL deadlock once
// two streams share a hardware queue. The turn passes round-robin over the groups that are still
// growing: g0 L0, g1 L0, g0 L1, g1 L1, ..., a finished group drops out. Each group's exchange count is
// identical on every rank (all ranks merge the same decisions), so the global enqueue order is too.
struct FpTurns {
  std::mutex m;
  std::condition_variable cv;
  int turn = 0;
  std::vector<char> done;
  std::vector<int64_t> issued;          // exchanges issued per group (checked against the other ranks' in tests)
  explicit FpTurns(int n) : done(std::max(1, n), 0), issued(std::max(1, n), 0) {}
  void advance_locked() {
    const int n = (int)done.size();
    for (int k = 1; k <= n; ++k) {
      const int c = (turn + k) % n;
      if (!done[c]) {
        turn = c;
        return;
      }
    }
  }
  template <class Fn>
  void run(int g, Fn&& fn) {
    std::unique_lock<std::mutex> lk(m);
    cv.wait(lk, [&] { return turn == g || done[g]; });
    try {
      fn();
    } catch (...) {
      ++issued[g];
      advance_locked();
      cv.notify_all();
      throw;
    }
    ++issued[g];
    advance_locked();
    cv.notify_all();
  }
  void finish(int g) {
    std::lock_guard<std::mutex> lk(m);
    done[g] = 1;
    if (turn == g) advance_locked();
    cv.notify_all();
  }
};

// Test hook: TMOG_FP_DELAY="rank:group:ms" sleeps before every exchange of that (rank, group), so a
// multi-rank test can skew the groups' timing on one rank and check the order (and the trees) hold.
inline int fp_delay_ms(int rank, int group) {
  const char* e = std::getenv("TMOG_FP_DELAY");
  int r = -1, gg = -1, ms = 0;
  if (e == nullptr || std::sscanf(e, "%d:%d:%d", &r, &gg, &ms) != 3) return 0;
  return (r == rank && gg == group) ? ms : 0;
}

struct GrowArgs {
  const uint8_t* Xb;
  int64_t N;
  int32_t F, mode, kind, S, B, missing_bin;
  int64_t chunk_rows;
  int32_t subtract, collect_leaves;
  const float* y;
  const float* t1;
  const float* t2;
  int64_t stride;
  const float* qscale;
  const double* qinv;
  const int32_t* n_bins;
  int32_t T;
  const int32_t* job_model;
  const int32_t* job_depth;
  const double* job_min_inst;
  const double* job_min_gain;
  const double* job_mcw;
  const double* job_lambda;
  const double* job_eps;
  const int32_t* job_fsub;
  const int64_t* job_count;   // root entries per job (job-major in rows)
  uint32_t* rows;             // packed root entries (device / host), overwritten
  uint32_t* rows_alt;         // scratch of the same size
  uint32_t* leaf_rows;        // collect_leaves: final leaf of every entry (same size as rows)
  int32_t* leaf_gid;
  int32_t n_groups;
  const int32_t* group_start;  // [n_groups + 1] job boundaries
  int64_t rng_seed;
  void* stream;               // GPU: caller's stream (groups wait on it; it waits on the groups)
  const int32_t* n_bins_host; // host copy of n_bins (feature grouping for the histogram kernel), may be null
  // GPU, sparse missing bin: CSR of the one-present-bin columns (row -> local ids, in n_bins order, of
  // the columns whose bin is the present bin 0); null when absent
  const int64_t* csr_ptr;     // [N + 1]
  const uint16_t* csr_col;
  int32_t csr_nf;             // number of one-present-bin columns the CSR indexes
  // Feature-parallel growth (fp_world > 0; jobs without per-node feature subsets). Every rank runs the
  // same jobs on the same replicated rows and binned matrix but builds histograms and scans splits for
  // its own slice of the growth-order feature list only: positions [fp_mlo, fp_mhi) of the multi-bin
  // list and [fp_olo, fp_ohi) of the one-present-bin list (all features count as multi-bin outside the
  // sparse missing-bin mode). Per level the ranks all-gather one split record per node (fp_rec_bytes)
  // and every rank merges them with the split scan's total order, so all ranks partition identically
  // and the forests equal the single-rank ones bit for bit.
  int32_t fp_rank, fp_world;
  int32_t fp_mlo, fp_mhi, fp_olo, fp_ohi;
  void* const* fp_comm;       // GPU: one RCCL communicator per job group
  int (*fp_exchange)(void* ctx, int group, const void* send, void* recv, int64_t bytes);   // CPU all-gather
  void* fp_ctx;
  // GPU: first per-group resource slot (stream, staging, histogram buffers) of this call -- concurrent
  // calls (e.g. the XGBoost learner's pipelined job halves, one host thread each) use disjoint slots
  int32_t slot_base;
  // GPU, optional: feature-major copy of Xb ([F][N], row index = packed entry & 0xFFFFFF). The partition
  // reads one split-column byte per row; from the feature-major copy the bytes of a node's rows share
  // cache lines (from Xb every byte pulls its own line)
  const uint8_t* XbT;
  // GPU, MODE 2, optional: the entries' quantised statistics (int32 pairs q(w g), q(w h)), one per entry of
  // rows / rows_alt (same positions); the partition moves them with their entries so the histogram items
  // read them coalesced instead of gathering t1 / t2 by row id. n_entries = size of rows (and of these).
  int32_t* gh;
  int32_t* gh_alt;
  int64_t n_entries;
  // training sets of >= 2^24 rows: entries are plain 32-bit row ids of weight 1 instead of row | weight << 24
  // (weighted roots are expanded into repeated entries by the caller, models/tree_engine.py)
  int32_t wide_rows;
  // GPU, optional: row-major matrix the wide-load histogram items read instead of Xb -- the multi-bin columns
  // only (their Xb column positions), row stride Fh bytes (a multiple of 64: every row segment starts a cache
  // line and the matrix is smaller than Xb, so more of it stays in the Infinity Cache). Groups whose columns
  // reach past Fh stay on Xb.
  const uint8_t* Xh;
  int32_t Fh;
};

// Feature-parallel split record, one per node and rank:
//   gain f64 @0 | fpos i32 @8 (position in the full growth-order feature list, the tie-break) |
//   bin i32 @12 | dl i32 @16 | col i32 @20 (Xb column) | left f32[S] @24
inline size_t fp_rec_bytes(int S) { return (24 + 4 * (size_t)S + 7) & ~size_t(7); }

// Merge of the ranks' records of node j (host twin of tree_kernels.hip fp_merge_kernel).
inline void fp_merge_host(const uint8_t* recv, int R, int m, size_t rb, int S, int32_t* feat, int32_t* bin,
                          float* gain, uint8_t* dl, float* left) {
  for (int j = 0; j < m; ++j) {
    int w = -1;
    double bg = -INFINITY;
    int bf = 0x7fffffff, bd = 0, bb = 0;
    for (int r = 0; r < R; ++r) {
      const uint8_t* p = recv + ((size_t)r * m + j) * rb;
      double g;
      int32_t f, b, d;
      std::memcpy(&g, p, 8);
      std::memcpy(&f, p + 8, 4);
      std::memcpy(&b, p + 12, 4);
      std::memcpy(&d, p + 16, 4);
      if (f == 0x7fffffff) continue;
      const bool better = g != bg ? g > bg : (f != bf ? f < bf : (d != bd ? d < bd : b < bb));
      if (w < 0 || better) {
        w = r; bg = g; bf = f; bd = d; bb = b;
      }
    }
    if (w < 0) {
      feat[j] = -1;
      bin[j] = -1;
      gain[j] = -INFINITY;
      dl[j] = 0;
      for (int s = 0; s < S; ++s) left[(size_t)j * S + s] = 0.f;
      continue;
    }
    const uint8_t* p = recv + ((size_t)w * m + j) * rb;
    int32_t col;
    std::memcpy(&col, p + 20, 4);
    feat[j] = col;
    bin[j] = bb;
    gain[j] = (float)bg;
    dl[j] = (uint8_t)bd;
    std::memcpy(left + (size_t)j * S, p + 24, 4 * (size_t)S);
  }
}

struct GroupResult {
  std::vector<int64_t> tree, feat, bin, left, right;
  std::vector<uint8_t> dl;
  std::vector<double> gain, tot;   // tot: n * S
  int64_t leaf_count = 0;
  int S = 1;

  std::vector<int64_t> add(const std::vector<int64_t>& trees) {
    std::vector<int64_t> ids(trees.size());
    for (size_t i = 0; i < trees.size(); ++i) {
      ids[i] = (int64_t)tree.size();
      tree.push_back(trees[i]);
      feat.push_back(-1);
      bin.push_back(-1);
      left.push_back(-1);
      right.push_back(-1);
      dl.push_back(0);
      gain.push_back(0.0);
      for (int s = 0; s < S; ++s) tot.push_back(0.0);
    }
    return ids;
  }
};

struct GrowResult {
  std::vector<GroupResult> groups;
  int status = 0;
  std::string error;
};

// item layouts shared with hip/tree_kernels.hip
struct HistItemH {
  int32_t node, fg0, nf, excl;
  int64_t begin, count;
};
struct PartItemH {
  int32_t node, pad;
  int64_t begin, count, out_left, out_right;
};
struct LeafItemH {
  int64_t begin, count, out;
  int32_t gid, pad;
};
static_assert(sizeof(HistItemH) == 32 && sizeof(PartItemH) == 40 && sizeof(LeafItemH) == 32, "item layout");

// splitmix64 stream for the per-node feature subsets (identical on both backends)
struct SplitMix {
  uint64_t s;
  explicit SplitMix(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  uint64_t below(uint64_t n) { return next() % n; }
};

// Host staging: arrays appended at 16-byte aligned offsets, shipped as one block by the backend.
struct Staging {
  std::vector<uint8_t> buf;
  size_t add(const void* p, size_t bytes) {
    const size_t off = (buf.size() + 15) & ~size_t(15);
    buf.resize(off + ((bytes + 15) & ~size_t(15)));
    if (bytes) std::memcpy(buf.data() + off, p, bytes);
    return off;
  }
  template <class T>
  size_t add(const std::vector<T>& v) { return add(v.data(), v.size() * sizeof(T)); }
  void clear() { buf.clear(); }
};

// Where split_find writes the feature-parallel split records (rec == nullptr: not feature-parallel).
struct FpSlice {
  uint8_t* rec;
  int64_t rec_bytes;
  int32_t mlo, nml, obase;   // local feature f -> position f < nml ? mlo + f : obase + (f - nml)
};

struct FeatGroup {
  int f0, nf;
  bool reg;
  bool csr = false;
  bool wide = false;   // GPU: contiguous dword-aligned physical columns -> wide-load histogram items
};

constexpr int64_t kCsrRows = 1024;   // rows per CSR histogram item (GPU)
constexpr int64_t kPartRows = 1024;  // rows per partition item (GPU)

// n features in near-equal groups of at most 64
inline std::vector<FeatGroup> equal_groups(int n) {
  std::vector<FeatGroup> out;
  if (n <= 0) return out;
  const int ng = std::max(1, (n + 63) / 64);
  const int fg = (n + ng - 1) / ng;
  for (int gi = 0; gi * fg < n; ++gi) out.push_back(FeatGroup{gi * fg, std::min(fg, n - gi * fg), false, false});
  return out;
}

// Groups whose sizes are multiples of 4 (<= 64): with a dword-aligned first column every group of the
// wide-load histogram path starts on a dword boundary of the row.
inline std::vector<FeatGroup> equal_groups4(int n) {
  std::vector<FeatGroup> out;
  if (n <= 0) return out;
  const int ng = std::max(1, (n + 63) / 64);
  const int fg = std::min(64, ((n + ng - 1) / ng + 3) / 4 * 4);
  for (int gi = 0; gi * fg < n; ++gi) out.push_back(FeatGroup{gi * fg, std::min(fg, n - gi * fg), false, false});
  return out;
}

// TMOG_GROW_TIMING=1: host nanoseconds per level spent planning (building the level's work lists and
// reading the previous level's decisions), issuing (staging copy + kernel launches) and waiting for the
// level's result read-back, summed over every group and call (diagnostics; read by the C ABI)
struct GrowTiming {
  std::atomic<int64_t> plan{0}, issue{0}, wait{0}, levels{0};
};
inline GrowTiming& grow_timing() {
  static GrowTiming t;
  return t;
}

// Histogram feature groups of a job group without per-node feature subsets (or the per-node default),
// shared by the host-planned level loop (grow_group) and the device-planned one (hip/tree_resident.hip).
struct GroupLayout {
  std::vector<FeatGroup> full_groups;
  std::vector<int32_t> perm_feats;
  int split_n_multi = -1;   // GPU split scan: local features [n_multi, F) have one present bin
  int64_t live_dense = -1;  // GPU zero / subtract: words past this prefix are live only at bin 0
  int fp_nml = 0, fp_obase = 0;   // split records: local feature -> position in the full feature list
  int F_use = 0;
};

template <bool GPU>
GroupLayout group_layout(const GrowArgs& a, bool use_subset, bool fp) {
  // Feature groups of the histogram kernel (<= 64 features each). Without per-node subsets the
  // grouping is fixed: with a sparse missing bin (GPU, MODE 2) the one-present-bin columns (one-hot /
  // null indicators) go last; given their row-wise CSR they form one group whose items walk only the
  // present entries of each row (a few per row instead of one byte per column), otherwise groups of
  // their own that the kernel accumulates in registers.
  // The feature order is the same on both backends (stable: multi-bin columns first, then the
  // one-present-bin columns), so split tie-breaks by local feature index stay identical GPU vs CPU.
  GroupLayout L;
  std::vector<FeatGroup>& full_groups = L.full_groups;
  std::vector<int32_t>& perm_feats = L.perm_feats;
  int& split_n_multi = L.split_n_multi;
  int64_t& live_dense = L.live_dense;
  int& fp_nml = L.fp_nml;
  int& fp_obase = L.fp_obase;
  const int F = a.F, B = a.B, S = a.S;
  if (!use_subset && a.mode == 2 && a.missing_bin >= 0 && a.n_bins_host != nullptr) {
    std::vector<int32_t> multi, one;
    for (int f = 0; f < F; ++f) (a.n_bins_host[f] != 1 ? multi : one).push_back(f);
    int m0 = 0, m1 = (int)multi.size(), o0 = 0, o1 = (int)one.size();
    if (fp) {
      m0 = a.fp_mlo; m1 = a.fp_mhi; o0 = a.fp_olo; o1 = a.fp_ohi;
      if (m0 < 0 || m1 > (int)multi.size() || m1 <= m0 || o0 < 0 || o1 > (int)one.size() || o1 < o0)
        throw std::runtime_error("bad feature-parallel slice");
    }
    perm_feats.assign(multi.begin() + m0, multi.begin() + m1);
    const int n_multi = m1 - m0;
    fp_nml = n_multi;
    fp_obase = (int)multi.size() + o0;
    // node totals are read from local feature 0, which must be a multi-bin column: with no multi-bin
    // column at all every histogram word stays written and scanned (no CSR / reduced write-out)
    split_n_multi = n_multi > 0 ? n_multi : -1;
    if (GPU && n_multi > 0) live_dense = (int64_t)n_multi * a.B * a.S;
    perm_feats.insert(perm_feats.end(), one.begin() + o0, one.begin() + o1);
    const char* wenv = std::getenv("TMOG_HIST_WIDE");
    // (32-bit buffer offsets row * F + column: matrices below 2 GiB)
    const bool wide_ok = GPU && a.mode == 2 && S == 2 && F % 4 == 0 && !(wenv && wenv[0] == '0') &&
                         (int64_t)a.N * F < ((int64_t)1 << 31) - 64;
    for (FeatGroup g : (wide_ok ? equal_groups4(n_multi) : equal_groups(n_multi))) {
      if (wide_ok) {
        bool ok = perm_feats[g.f0] % 4 == 0;
        for (int i = 1; ok && i < g.nf; ++i) ok = perm_feats[g.f0 + i] == perm_feats[g.f0] + i;
        // with a compact histogram matrix every wide group must lie inside it (the kernel reads Xh only)
        if (ok && a.Xh != nullptr) ok = a.Fh % 4 == 0 && perm_feats[g.f0] + g.nf <= a.Fh;
        g.wide = ok;
      }
      full_groups.push_back(g);
    }
    const int n_one = o1 - o0;
    if (GPU && a.csr_ptr && a.csr_col && n_multi > 0 && n_one > 0 && a.csr_nf == n_one &&
        2 * n_one + 4 + 64 * 4 <= 64 * (B * S + 1))   // sums + list lengths of the CSR item (tree_kernels.hip)
      full_groups.push_back(FeatGroup{n_multi, n_one, false, true});   // one item walks the rows' CSR lists
    else
      for (const FeatGroup& g : equal_groups(n_one))
        full_groups.push_back(FeatGroup{n_multi + g.f0, g.nf, GPU, false});
  } else if (fp) {
    if (a.fp_mlo < 0 || a.fp_mhi > F || a.fp_mhi <= a.fp_mlo) throw std::runtime_error("bad feature-parallel slice");
    for (int f = a.fp_mlo; f < a.fp_mhi; ++f) perm_feats.push_back(f);
    fp_nml = (int)perm_feats.size();
    fp_obase = F;
    full_groups = equal_groups(fp_nml);
  } else {
    full_groups = equal_groups(F);
  }
  L.F_use = perm_feats.empty() ? F : (int)perm_feats.size();
  return L;
}

template <class BK>
void grow_group(BK& bk, const GrowArgs& a, int g, GroupResult& R, FpTurns* turns = nullptr) {
  const int j0 = a.group_start[g], j1 = a.group_start[g + 1];
  const int T = j1 - j0;
  const int F = a.F, S = a.S, B = a.B;
  R.S = S;
  if (T <= 0) return;
  int64_t entry0 = 0;
  for (int j = 0; j < j0; ++j) entry0 += a.job_count[j];
  int64_t total = 0;
  for (int j = j0; j < j1; ++j) total += a.job_count[j];
  uint32_t* rows = a.rows + entry0;
  uint32_t* rows_alt = a.rows_alt + entry0;
  uint32_t* leaf_rows = a.collect_leaves ? a.leaf_rows + entry0 : nullptr;
  int32_t* leaf_gid = a.collect_leaves ? a.leaf_gid + entry0 : nullptr;
  int64_t leaf_pos = 0;

  std::vector<int32_t> fsub(T);
  bool use_subset = false;
  int max_depth = 0;
  for (int t = 0; t < T; ++t) {
    const int k = a.job_fsub[j0 + t];
    fsub[t] = (k <= 0 || k >= F) ? F : k;
    use_subset |= fsub[t] < F;
    max_depth = std::max(max_depth, a.job_depth[j0 + t]);
  }
  SplitMix rng((uint64_t)a.rng_seed + 1000003ull * (uint64_t)g);

  std::vector<int64_t> lv_tree(T), lv_begin(T), lv_count(T);
  for (int t = 0; t < T; ++t) {
    lv_tree[t] = t;
    lv_count[t] = a.job_count[j0 + t];
    lv_begin[t] = t ? lv_begin[t - 1] + lv_count[t - 1] : 0;
  }
  std::vector<int64_t> lv_gid = R.add(lv_tree);

  const int32_t* all_feats = bk.all_features(F);
  int64_t* hist = nullptr;
  int64_t* prev_hist = nullptr;
  int cur_slot = 0;          // the backend keeps two grow-only histogram buffers per group
  std::vector<int64_t> pair_parent_off;
  Staging st1, st2, st3;   // level arrays (slot 0), scatter items (slot 1), leaf items (slot 2)

  auto collect = [&](const std::vector<int64_t>& idx) {
    if (!a.collect_leaves) return;
    std::vector<LeafItemH> items;
    for (int64_t i : idx) {
      const int64_t c = lv_count[i];
      if (c <= 0) continue;
      for (int64_t o = 0; o < c; o += a.chunk_rows) {
        LeafItemH it;
        it.begin = lv_begin[i] + o;
        it.count = std::min(a.chunk_rows, c - o);
        it.out = leaf_pos + o;
        it.gid = (int32_t)lv_gid[i];
        it.pad = 0;
        items.push_back(it);
      }
      leaf_pos += c;
    }
    if (items.empty()) return;
    st3.clear();
    const size_t o = st3.add(items);
    const uint8_t* d = bk.ship(st3, 2);
    bk.leaf_collect(rows, d + o, (int)items.size(), leaf_rows, leaf_gid);
  };

  const bool fp = a.fp_world > 0;   // 1 rank is allowed (tests run the exchange path on one GPU)
  if (fp && use_subset) throw std::runtime_error("feature-parallel growth needs jobs without feature subsets");
  GroupLayout L = group_layout<BK::kGPU>(a, use_subset, fp);
  std::vector<FeatGroup>& full_groups = L.full_groups;
  std::vector<int32_t>& perm_feats = L.perm_feats;
  const int split_n_multi = L.split_n_multi;
  const int64_t live_dense = L.live_dense;
  const int fp_nml = L.fp_nml, fp_obase = L.fp_obase;
  const int F_use = perm_feats.empty() ? F : (int)perm_feats.size();
  const bool trace = std::getenv("TMOG_GROW_TRACE") != nullptr;   // progress to stderr (debugging)
  if (trace)
    std::fprintf(stderr, "[grow g%d] T=%d F=%d F_use=%d S=%d B=%d fp=%d slice m[%d,%d) o[%d,%d)\n", g, T, F, F_use, S,
                 B, (int)fp, a.fp_mlo, a.fp_mhi, a.fp_olo, a.fp_ohi);
  // GPU histogram items accumulate a chunk of the statistics when a B x S table exceeds the LDS (many
  // classes / wide bins): one item per chunk, each writing disjoint words of the node histogram
  const int stat_sc = bk.stat_chunk(B, S);
  const int n_sc = (S + stat_sc - 1) / stat_sc;
  if (n_sc > 256) throw std::runtime_error("too many statistic chunks (classes x bins too large)");
  const int fp_mlo = fp ? a.fp_mlo : 0;
  const size_t fp_rb = fp_rec_bytes(S);
  const char* hg_env = std::getenv("TMOG_TREE_HESS_GATE");     // "0": off (A/B and the equality test)
  const bool newton = a.mode == 2 && a.kind == 3 && S >= 2 &&   // (g, h) statistics, second-order gain
                      !(hg_env && hg_env[0] == '0');
  static const bool timing = std::getenv("TMOG_GROW_TIMING") != nullptr;
  using tclock = std::chrono::steady_clock;
  auto ns_since = [](tclock::time_point t) {
    return (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(tclock::now() - t).count();
  };
  tclock::time_point t_lvl = tclock::now();
  for (int depth = 0; depth <= max_depth; ++depth) {
    const int64_t n = (int64_t)lv_gid.size();
    if (n == 0) break;
    if (timing) t_lvl = tclock::now();
    std::vector<uint8_t> can(n), need(n);
    std::vector<int64_t> hist_nodes;
    for (int64_t i = 0; i < n; ++i) {
      const int t = (int)lv_tree[i];
      can[i] = depth < a.job_depth[j0 + t] && lv_count[i] >= 2 &&
               (double)lv_count[i] >= 2 * a.job_min_inst[j0 + t] - 1e-9;
      // Newton trees: both children of a split need a hessian sum >= min_child_weight, so a node whose
      // hessian (from its parent's split statistics, fp32) is clearly below 2 mcw has no valid split --
      // skip its histogram / scan (the 1e-6 margin keeps every node that could split)
      if (can[i] && newton && depth > 0 && a.job_mcw[j0 + t] > 0 &&
          R.tot[(size_t)lv_gid[i] * S + 1] < 2.0 * a.job_mcw[j0 + t] * (1.0 - 1e-6))
        can[i] = 0;
      need[i] = can[i] || depth == 0;
    }
    // a splittable node whose sibling cannot split still gets its histogram by subtraction from the
    // parent's: build the sibling's (scan skipped, params slot 7 = 0) rather than the node's own
    if (a.subtract && !use_subset && prev_hist && depth > 0)
      for (int64_t q = 0; 2 * q + 1 < n; ++q)
        if (need[2 * q] != need[2 * q + 1] && lv_count[2 * q] >= 1 && lv_count[2 * q + 1] >= 1 &&
            (can[2 * q] ? lv_count[2 * q + 1] <= lv_count[2 * q] : lv_count[2 * q] <= lv_count[2 * q + 1]))
          need[2 * q] = need[2 * q + 1] = 1;
    for (int64_t i = 0; i < n; ++i)
      if (need[i]) hist_nodes.push_back(i);
    if (hist_nodes.empty()) {
      std::vector<int64_t> all(n);
      for (int64_t i = 0; i < n; ++i) all[i] = i;
      collect(all);
      break;
    }
    const int m = (int)hist_nodes.size();
    // ---- per-node feature lists
    std::vector<int32_t> feat_list, feat_off(m), nfeat(m);
    if (use_subset) {
      std::vector<int32_t> perm(F);
      for (int j = 0; j < m; ++j) {
        const int k = fsub[lv_tree[hist_nodes[j]]];
        for (int f = 0; f < F; ++f) perm[f] = f;
        for (int i = 0; i < k; ++i) std::swap(perm[i], perm[i + (int)rng.below((uint64_t)(F - i))]);
        std::sort(perm.begin(), perm.begin() + k);
        feat_off[j] = (int32_t)feat_list.size();
        nfeat[j] = k;
        feat_list.insert(feat_list.end(), perm.begin(), perm.begin() + k);
      }
    } else {
      for (int j = 0; j < m; ++j) {
        feat_off[j] = 0;
        nfeat[j] = F_use;
      }
      if (!perm_feats.empty()) feat_list = perm_feats;
    }
    std::vector<int64_t> hsz(m), hoff(m);
    int64_t hwords = 0;
    int max_nf = 0;
    for (int j = 0; j < m; ++j) {
      hsz[j] = (int64_t)nfeat[j] * B * S;
      hoff[j] = hwords;
      hwords += hsz[j];
      max_nf = std::max(max_nf, (int)nfeat[j]);
    }
    hist = bk.hist_buffer(cur_slot, (size_t)hwords);
    std::vector<int64_t> loc(n, -1);
    for (int j = 0; j < m; ++j) loc[hist_nodes[j]] = j;
    // ---- subtraction trick: children come in (left, right) pairs
    std::vector<int64_t> d_big, d_small, d_poff;
    if (a.subtract && !use_subset && prev_hist && depth > 0) {
      for (int64_t q = 0; 2 * q + 1 < n; ++q) {
        const int64_t li = 2 * q, ri = 2 * q + 1;
        if (!(need[li] && need[ri])) continue;
        const bool left_big = lv_count[li] >= lv_count[ri];
        d_big.push_back(loc[left_big ? li : ri]);
        d_small.push_back(loc[left_big ? ri : li]);
        d_poff.push_back(pair_parent_off[q]);
      }
    }
    std::vector<uint8_t> build(m, 1);
    for (int64_t b : d_big) build[b] = 0;
    // GPU: a sibling pair's subtraction and both children's split scans run as one pass (pair_scan_kernel)
    // -- the two nodes are flagged (params slot 4) so the node-wise scan skips them; same decisions
    const char* ps_env = std::getenv("TMOG_PAIR_SCAN");
    const bool pair_fuse = BK::kGPU && !use_subset && S <= 16 && B <= 64 && !d_big.empty() &&
                           !(ps_env && ps_env[0] == '0');
    std::vector<int32_t> d_sj, d_bj;
    if (pair_fuse)
      for (size_t q = 0; q < d_big.size(); ++q) {
        d_sj.push_back((int32_t)d_small[q]);
        d_bj.push_back((int32_t)d_big[q]);
      }
    std::vector<int64_t> nb(m), nc(m);
    std::vector<int32_t> nmd(m);
    std::vector<float> params((size_t)m * 8, 0.f);
    for (int j = 0; j < m; ++j) {
      const int64_t i = hist_nodes[j];
      const int t = (int)lv_tree[i];
      nb[j] = lv_begin[i];
      nc[j] = lv_count[i];
      nmd[j] = a.job_model[j0 + t];
      float* P = &params[(size_t)j * 8];
      P[0] = (float)a.job_min_inst[j0 + t];
      P[1] = (float)a.job_min_gain[j0 + t];
      P[2] = (float)a.job_mcw[j0 + t];
      P[3] = (float)a.job_lambda[j0 + t];
      P[5] = a.missing_bin >= 0 ? 1.f : 0.f;
      P[6] = (float)a.job_eps[j0 + t];
      P[7] = can[i] ? 1.f : 0.f;
    }
    for (size_t q = 0; q < d_sj.size(); ++q) params[(size_t)d_sj[q] * 8 + 4] = params[(size_t)d_bj[q] * 8 + 4] = 1.f;
    // ---- work items (GPU) / built-node arrays (CPU)
    std::vector<HistItemH> hitems;
    std::vector<PartItemH> citems;
    std::vector<int64_t> z_off, z_size;
    std::vector<int64_t> zc_off, zc_size;   // nodes whose only multi-item group is the CSR one: zero its words
    std::vector<int64_t> b_nb, b_nc, b_nho;
    std::vector<int32_t> b_nfo, b_nnf, b_nmd;
    for (int j = 0; j < m; ++j) {
      const int64_t cnt = nc[j];
      const int64_t nch = std::max<int64_t>(1, (cnt + a.chunk_rows - 1) / a.chunk_rows);
      // partition items: short slices (each is a chain of 256-row steps with cursor atomics)
      for (int64_t c = 0, npi = std::max<int64_t>(1, (cnt + kPartRows - 1) / kPartRows); c < npi; ++c) {
        PartItemH p;
        p.node = j;
        p.pad = 0;
        p.begin = nb[j] + c * kPartRows;
        p.count = std::min(kPartRows, cnt - c * kPartRows);
        p.out_left = p.out_right = 0;
        citems.push_back(p);
      }
      if (!build[j]) continue;
      b_nb.push_back(nb[j]);
      b_nc.push_back(nc[j]);
      b_nho.push_back(hoff[j]);
      b_nfo.push_back(feat_off[j]);
      b_nnf.push_back(nfeat[j]);
      b_nmd.push_back(nmd[j]);
      const int nf = nfeat[j];
      const std::vector<FeatGroup>& grp = use_subset ? equal_groups(nf) : full_groups;
      // CSR items take kCsrRows-row slices (each walks its rows one at a time, so shorter items keep
      // more of them in flight); a node split over several items is zeroed and accumulated atomically
      const int64_t ncsr = std::max<int64_t>(1, (cnt + kCsrRows - 1) / kCsrRows);
      bool has_csr = false;
      for (const FeatGroup& fgp : grp) has_csr |= fgp.csr;
      if (nch > 1) {
        z_off.push_back(hoff[j]);
        z_size.push_back(hsz[j]);
      } else if (has_csr && ncsr > 1) {
        // single-chunk multi-bin groups write their words exclusively: only the one-present-bin region
        // past the dense prefix (the CSR group's bin-0 words) accumulates atomically and needs zeroing
        if (live_dense >= 0 && live_dense < hsz[j]) {
          zc_off.push_back(hoff[j] + live_dense);
          zc_size.push_back(hsz[j] - live_dense);
        } else {
          z_off.push_back(hoff[j]);
          z_size.push_back(hsz[j]);
        }
      }
      for (const FeatGroup& fgp : grp) {
        const int64_t step = fgp.csr ? kCsrRows : a.chunk_rows;
        const int64_t nit = fgp.csr ? ncsr : nch;
        const int nchunk = (fgp.csr || fgp.reg) ? 1 : n_sc;
        for (int sc = 0; sc < nchunk; ++sc)
          for (int64_t c = 0; c < nit; ++c) {
            HistItemH h;
            h.node = j;
            h.fg0 = fgp.f0;
            h.nf = fgp.nf;
            h.excl = (nit == 1 ? 1 : 0) | (fgp.reg ? 2 : 0) | (fgp.csr ? 4 : 0) | (fgp.wide ? 16 : 0) |
                     ((fgp.reg || fgp.csr) && live_dense >= 0 ? 8 : 0) | (sc << 8);
            h.begin = nb[j] + c * step;
            h.count = std::min(step, cnt - c * step);
            hitems.push_back(h);
          }
      }
    }
    // wide-load items first: the GPU launches them as a kernel of their own (fewer registers)
    const auto wide_end = std::stable_partition(hitems.begin(), hitems.end(),
                                                [](const HistItemH& h) { return (h.excl & 16) != 0; });
    const int n_wide = (int)(wide_end - hitems.begin());
    int need_general = 0;          // any item on the byte-gather path (not CSR, not wide-load)?
    for (const HistItemH& h : hitems) need_general |= (h.excl & (4 | 16)) == 0;
    std::vector<int64_t> d_soff, d_ooff, d_size;
    int64_t d_max = 0;
    for (size_t q = 0; q < d_big.size(); ++q) {
      d_soff.push_back(hoff[d_small[q]]);
      d_ooff.push_back(hoff[d_big[q]]);
      d_size.push_back(hsz[d_big[q]]);
      d_max = std::max(d_max, hsz[d_big[q]]);
    }
    int64_t z_max = 0, zc_max = 0;
    for (int64_t z : z_size) z_max = std::max(z_max, z);
    for (int64_t z : zc_size) zc_max = std::max(zc_max, z);
    // ---- ship everything in one copy
    st1.clear();
    const size_t o_nfo = st1.add(feat_off), o_nnf = st1.add(nfeat), o_nmd = st1.add(nmd), o_nho = st1.add(hoff);
    const size_t o_par = st1.add(params);
    const bool own_list = use_subset || !perm_feats.empty();
    const size_t o_fl = own_list ? st1.add(feat_list) : 0;
    const size_t o_hit = st1.add(hitems), o_cit = st1.add(citems);
    std::vector<int64_t> z_off_all(z_off), z_size_all(z_size);
    z_off_all.insert(z_off_all.end(), zc_off.begin(), zc_off.end());
    z_size_all.insert(z_size_all.end(), zc_size.begin(), zc_size.end());
    const size_t o_zo = st1.add(z_off_all), o_zs = st1.add(z_size_all);
    const size_t o_dp = st1.add(d_poff), o_ds = st1.add(d_soff), o_do = st1.add(d_ooff), o_dz = st1.add(d_size);
    const size_t o_bnb = st1.add(b_nb), o_bnc = st1.add(b_nc), o_bnfo = st1.add(b_nfo), o_bnnf = st1.add(b_nnf);
    const size_t o_bnmd = st1.add(b_nmd), o_bnho = st1.add(b_nho);
    const size_t o_nb = st1.add(nb), o_nc = st1.add(nc);
    const size_t o_sj = st1.add(d_sj), o_bj = st1.add(d_bj);
    tclock::time_point t_issue = tclock::now();
    if (timing) grow_timing().plan += ns_since(t_lvl);
    const uint8_t* d1 = bk.ship(st1, 0);
#define TM_P(T_, off) ((T_*)(d1 + (off)))
    const int32_t* flist = own_list ? TM_P(const int32_t, o_fl) : all_feats;
    // ---- histograms
    // one launch: the first z_off.size() segments are whole node histograms (dense prefix live_dense), the
    // rest start at a node's one-present-bin region (dense prefix 0)
    bk.zero_segments(hist, TM_P(const int64_t, o_zo), TM_P(const int64_t, o_zs), (int)(z_off.size() + zc_off.size()),
                     std::max(z_max, zc_max), live_dense, a.B * a.S, a.S, (int)z_off.size());
    bk.hist_build(a, rows, hitems.size() ? (const void*)(d1 + o_hit) : nullptr, (int)hitems.size(),
                  TM_P(const int32_t, o_nfo), flist, TM_P(const int32_t, o_nmd), TM_P(const int64_t, o_nho), hist,
                  (int)b_nb.size(), TM_P(const int64_t, o_bnb), TM_P(const int64_t, o_bnc),
                  TM_P(const int32_t, o_bnfo), TM_P(const int32_t, o_bnnf), TM_P(const int32_t, o_bnmd),
                  TM_P(const int64_t, o_bnho), stat_sc, n_wide, need_general);
    bool pairs_done = false;
    if constexpr (BK::kGPU) {
      if (pair_fuse) {
        bk.pair_scan(a, hist, prev_hist, TM_P(const int64_t, o_dp), TM_P(const int32_t, o_sj),
                     TM_P(const int32_t, o_bj), (int)d_sj.size(), TM_P(const int64_t, o_nho),
                     TM_P(const int32_t, o_nnf), TM_P(const int32_t, o_nfo), flist, TM_P(const float, o_par),
                     TM_P(const int32_t, o_nmd), max_nf, m, split_n_multi);
        pairs_done = true;
      }
    }
    if (!d_big.empty() && !pairs_done)
      bk.hist_subtract(hist, prev_hist, TM_P(const int64_t, o_dp), TM_P(const int64_t, o_ds),
                       TM_P(const int64_t, o_do), TM_P(const int64_t, o_dz), (int)d_big.size(), d_max, live_dense,
                       a.B * a.S, a.S);
    // ---- split scan + (GPU) one-pass partition -> one result block: decisions + per-node slot cursors
    const int64_t ncit = (int64_t)citems.size();
    const size_t r_cl = 0, r_feat = r_cl + 16 * (size_t)m, r_bin = r_feat + 4 * (size_t)m, r_gain = r_bin + 4 * (size_t)m;
    const size_t r_left = r_gain + 4 * (size_t)m, r_tot = r_left + 4 * (size_t)m * S, r_dl = r_tot + 4 * (size_t)m * S;
    const size_t r_bytes = r_dl + (size_t)m;
    uint8_t* res = bk.result_buffer(r_bytes);
    uint8_t* fp_send = fp ? bk.fp_send_buffer(fp_rb * (size_t)m) : nullptr;
    const FpSlice fps{fp_send, (int64_t)fp_rb, fp_mlo, fp_nml, fp_obase};
    bk.split_find(a, hist, m, TM_P(const int64_t, o_nho), TM_P(const int32_t, o_nnf), TM_P(const int32_t, o_nfo),
                  flist, TM_P(const float, o_par), TM_P(const int32_t, o_nmd), max_nf, (int32_t*)(res + r_feat),
                  (int32_t*)(res + r_bin), (float*)(res + r_gain), res + r_dl, (float*)(res + r_left),
                  (float*)(res + r_tot), (int64_t*)(res + r_cl), use_subset ? -1 : split_n_multi, fps);
    if (trace) std::fprintf(stderr, "[grow g%d] depth %d: %d nodes split_find done\n", g, depth, m);
    if (fp) {  // all-gather the ranks' best splits, merge into this level's decisions (on-stream on the GPU)
      if (const int ms = fp_delay_ms(a.fp_rank, g)) std::this_thread::sleep_for(std::chrono::milliseconds(ms));
      auto xchg = [&] {
        bk.fp_exchange_merge(a, fp_send, m, fp_rb, (int32_t*)(res + r_feat), (int32_t*)(res + r_bin),
                             (float*)(res + r_gain), res + r_dl, (float*)(res + r_left));
      };
      if (turns != nullptr) turns->run(g, xchg);
      else xchg();
      if (trace) std::fprintf(stderr, "[grow g%d] depth %d: exchange + merge issued\n", g, depth);
    }
    if (BK::kGPU)   // partition in place of the node ranges, straight from the device decisions
      bk.partition_fused(a, rows, rows_alt, d1 + o_cit, (int)ncit, TM_P(const int64_t, o_nb),
                         TM_P(const int64_t, o_nc), (const int32_t*)(res + r_feat), (const int32_t*)(res + r_bin),
                         res + r_dl, TM_P(const float, o_par), (const float*)(res + r_gain), (int64_t*)(res + r_cl));
    tclock::time_point t_wait = tclock::now();
    if (timing) grow_timing().issue += ns_since(t_issue);
    const uint8_t* h = bk.fetch(res, r_bytes);
    if (timing) {
      grow_timing().wait += ns_since(t_wait);
      grow_timing().levels += 1;
      t_lvl = tclock::now();
    }
    const int64_t* h_cur = (const int64_t*)(h + r_cl);   // GPU: [left, right] entries per node
    const int32_t* h_feat = (const int32_t*)(h + r_feat);
    const int32_t* h_bin = (const int32_t*)(h + r_bin);
    const float* h_gain = (const float*)(h + r_gain);
    const float* h_left = (const float*)(h + r_left);
    const float* h_tot = (const float*)(h + r_tot);
    const uint8_t* h_dl = h + r_dl;
    // ---- decisions
    std::vector<int64_t> sl;
    for (int j = 0; j < m; ++j) {
      const int64_t gid = lv_gid[hist_nodes[j]];
      for (int s = 0; s < S; ++s) R.tot[(size_t)gid * S + s] = (double)h_tot[(size_t)j * S + s];
      const bool ok = params[(size_t)j * 8 + 7] > 0.5f && h_feat[j] >= 0 && h_gain[j] > params[(size_t)j * 8 + 6];
      if (ok) sl.push_back(j);
    }
    {
      std::vector<uint8_t> splits(n, 0);
      for (int64_t j : sl) splits[hist_nodes[j]] = 1;
      std::vector<int64_t> lf;
      for (int64_t i = 0; i < n; ++i)
        if (!splits[i]) lf.push_back(i);
      collect(lf);
    }
    if (sl.empty()) break;
    const int64_t ns = (int64_t)sl.size();
    std::vector<int64_t> counts_sl(ns), out_begin(ns), nl(ns, 0);
    for (int64_t q = 0; q < ns; ++q) {
      const int64_t j = sl[q], gid = lv_gid[hist_nodes[j]];
      R.feat[gid] = h_feat[j];
      R.bin[gid] = h_bin[j];
      R.dl[gid] = h_dl[j];
      R.gain[gid] = (double)h_gain[j];
      counts_sl[q] = nc[j];
      out_begin[q] = q ? out_begin[q - 1] + counts_sl[q - 1] : 0;
    }
    // ---- partition of the splitting nodes' entries
    if (BK::kGPU) {
      for (int64_t q = 0; q < ns; ++q) {
        nl[q] = h_cur[2 * sl[q]];
        if (nl[q] < 0 || nl[q] + h_cur[2 * sl[q] + 1] != nc[sl[q]])
          throw std::runtime_error("partition cursor mismatch at depth " + std::to_string(depth));
      }
    } else {
      std::vector<int64_t> s_nb(ns), s_nc(ns);
      std::vector<int32_t> s_f(ns), s_b(ns);
      std::vector<uint8_t> s_d(ns);
      for (int64_t q = 0; q < ns; ++q) {
        const int64_t j = sl[q];
        s_nb[q] = nb[j];
        s_nc[q] = nc[j];
        s_f[q] = h_feat[j];
        s_b[q] = h_bin[j];
        s_d[q] = h_dl[j];
      }
      bk.partition_nodes(a, rows, rows_alt, (int)ns, s_nb.data(), s_nc.data(), s_f.data(), s_b.data(), s_d.data(),
                         out_begin.data(), nl.data());
    }
    // ---- next level: (left, right) children pairs
    std::vector<int64_t> ch_tree(2 * ns);
    for (int64_t q = 0; q < ns; ++q) ch_tree[2 * q] = ch_tree[2 * q + 1] = lv_tree[hist_nodes[sl[q]]];
    std::vector<int64_t> ch = R.add(ch_tree);
    std::vector<int64_t> new_begin(2 * ns), new_count(2 * ns);
    pair_parent_off.assign(ns, 0);
    for (int64_t q = 0; q < ns; ++q) {
      const int64_t j = sl[q], gid = lv_gid[hist_nodes[j]];
      const int64_t gl = ch[2 * q], gr = ch[2 * q + 1];
      R.left[gid] = gl;
      R.right[gid] = gr;
      for (int s = 0; s < S; ++s) {
        const double lt = (double)h_left[(size_t)j * S + s];
        const double tt = (double)h_tot[(size_t)j * S + s];
        R.tot[(size_t)gl * S + s] = lt;
        R.tot[(size_t)gr * S + s] = tt - lt;
      }
      const int64_t b0 = BK::kGPU ? nb[j] : out_begin[q];   // GPU children stay inside the parent's range
      new_begin[2 * q] = b0;
      new_begin[2 * q + 1] = b0 + nl[q];
      new_count[2 * q] = nl[q];
      new_count[2 * q + 1] = counts_sl[q] - nl[q];
      pair_parent_off[q] = hoff[j];
    }
#undef TM_P
    if (timing) grow_timing().plan += ns_since(t_lvl);
    std::swap(hist, prev_hist);
    cur_slot ^= 1;
    std::swap(rows, rows_alt);
    lv_tree = ch_tree;
    lv_gid = ch;
    lv_begin = new_begin;
    lv_count = new_count;
  }
  bk.finish();
  R.leaf_count = leaf_pos;
}

// Result accessors shared by both C ABIs.
inline int64_t result_nodes(const GrowResult* r, int g) { return (int64_t)r->groups[g].tree.size(); }

inline void result_copy(const GrowResult* r, int g, int64_t* tree, int64_t* feat, int64_t* bin, uint8_t* dl,
                        double* gain, double* tot, int64_t* left, int64_t* right) {
  const GroupResult& R = r->groups[g];
  const size_t n = R.tree.size();
  std::memcpy(tree, R.tree.data(), n * 8);
  std::memcpy(feat, R.feat.data(), n * 8);
  std::memcpy(bin, R.bin.data(), n * 8);
  std::memcpy(dl, R.dl.data(), n);
  std::memcpy(gain, R.gain.data(), n * 8);
  std::memcpy(tot, R.tot.data(), n * R.S * 8);
  std::memcpy(left, R.left.data(), n * 8);
  std::memcpy(right, R.right.data(), n * 8);
}

}  // namespace tmog

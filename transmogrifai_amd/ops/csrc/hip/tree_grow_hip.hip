// HIP backend of the native tree grower (common/tree_grow.hpp): one host thread + one HIP stream per
// job group, pinned staging buffers (three rotating slots per group) with hipMemcpyAsync, grow-only
// device buffers kept across calls (stream-ordered hipMallocAsync when they grow), and the tmog_hip_* kernel launchers of
// tree_kernels.hip. The only host<->device synchronisation is one result read per level and group.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <csignal>
#include <cstdlib>
#include <cstring>
#include <execinfo.h>
#include <unistd.h>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
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
int tmog_hip_hist_subtract(int64_t* hist, const int64_t* parent, const int64_t* parent_off, const int64_t* small_off,
                           const int64_t* out_off, const int64_t* size, int n, int64_t max_size, int64_t dense,
                           int per, int S, hipStream_t stream);
int tmog_hip_split_find(const int64_t* hist, int n_nodes, const int64_t* node_hist_off, const int32_t* node_nfeat,
                        const int32_t* node_feat_off, const int32_t* feat_list, const int32_t* feat_nbins, int B,
                        int S, int kind, const float* node_params, int missing_bin, const int32_t* node_model,
                        const double* qinv, int max_nfeat, void* cand_ws, int32_t* out_feat, int32_t* out_bin,
                        float* out_gain, uint8_t* out_dl, float* out_left, float* out_total, int64_t* cursors, int n_multi,
                        void* rec, int64_t rec_bytes, int fp_mlo, int fp_nml, int fp_obase, hipStream_t stream,
                        unsigned* done, const int* dm);
int tmog_hip_fp_merge(const void* recv, int R, int m, int64_t rec_bytes, int S, int32_t* out_feat, int32_t* out_bin,
                      float* out_gain, uint8_t* out_dl, float* out_left, hipStream_t stream);
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
}

namespace {

inline void hchk(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
inline void kchk(int rc, const char* what) {
  if (rc != 0) throw std::runtime_error(std::string("kernel ") + what + " failed with code " + std::to_string(rc));
}

// per-(group slot) persistent resources: stream, pinned staging slots, device staging, result mirror
struct GpuSlot {
  hipStream_t stream = nullptr;
  hipStream_t ext = nullptr;                 // caller-provided stream for this slot (tmog_hip_slot_stream)
  bool ext_set = false;
  uint8_t* pin[3] = {nullptr, nullptr, nullptr};
  size_t pin_cap[3] = {0, 0, 0};
  uint8_t* dev[3] = {nullptr, nullptr, nullptr};
  size_t dev_cap[3] = {0, 0, 0};
  hipEvent_t copied[3] = {nullptr, nullptr, nullptr};   // last H2D copy out of pin[k]
  uint8_t* res_dev = nullptr;
  size_t res_cap = 0;
  uint8_t* res_pin = nullptr;
  size_t res_pin_cap = 0;
  uint8_t* cand = nullptr;
  size_t cand_cap = 0;
  unsigned* done = nullptr;                  // per-node ticket counters of the fused split reduction (zeroed)
  size_t done_cap = 0;
  int32_t* feats = nullptr;
  int feats_n = 0;
  uint8_t* fp_send = nullptr;                 // feature-parallel: this rank's split records
  size_t fp_send_cap = 0;
  uint8_t* fp_recv = nullptr;                 // feature-parallel: all-gathered split records
  size_t fp_recv_cap = 0;
  uint8_t* hist[2] = {nullptr, nullptr};     // grow-only level histogram buffers (int64 words)
  size_t hist_cap[2] = {0, 0};
  int device = -1;
};

std::mutex& rccl_mutex() {
  static std::mutex m;
  return m;
}

std::vector<GpuSlot>& slots() {
  static std::vector<GpuSlot> s(32);   // models/tree_engine.py N_SLOTS (lanes of SLOT_LANE)
  return s;
}

struct GpuBackend {
  static constexpr bool kGPU = true;
  GpuSlot& sl;
  const tmog::GrowArgs& a;
  int group;
  GpuBackend(GpuSlot& s, const tmog::GrowArgs& args, int g) : sl(s), a(args), group(g) {}

  // grow-only device buffers: dev_alloc.hpp (a failed growth leaves the buffer empty, never a stale capacity)
  static void grow_dev(uint8_t*& p, size_t& cap, size_t need, hipStream_t s) {
    tmog::grow_device(p, cap, need, need + need / 2 + 4096, s);
  }
  static void grow_pin(uint8_t*& p, size_t& cap, size_t need, hipStream_t s) {
    if (need <= cap && p != nullptr) return;
    if (p) {
      hchk(hipStreamSynchronize(s), "sync before pinned realloc");
      hipError_t e = hipHostFree(p);
      p = nullptr;
      cap = 0;
      hchk(e, "hipHostFree");
    }
    const size_t nc = need + need / 2 + 4096;
    hchk(hipHostMalloc((void**)&p, nc, hipHostMallocDefault), "hipHostMalloc");
    cap = nc;
  }
  const int32_t* all_features(int F) {
    if (sl.feats_n < F) {
      uint8_t* p = reinterpret_cast<uint8_t*>(sl.feats);
      size_t cap = sl.feats ? sizeof(int32_t) * (size_t)sl.feats_n : 0;
      sl.feats = nullptr;
      sl.feats_n = 0;
      tmog::grow_device(p, cap, sizeof(int32_t) * (size_t)F, sizeof(int32_t) * (size_t)F, sl.stream);
      std::vector<int32_t> h(F);
      for (int i = 0; i < F; ++i) h[i] = i;
      hchk(hipMemcpyAsync(p, h.data(), sizeof(int32_t) * F, hipMemcpyHostToDevice, sl.stream), "copy feats");
      hchk(hipStreamSynchronize(sl.stream), "sync feats");
      sl.feats = reinterpret_cast<int32_t*>(p);
      sl.feats_n = F;
    }
    return sl.feats;
  }
  // Staged host arrays -> device in one async copy. The pinned buffer is rewritten only after its
  // previous copy has completed: a level's leaf items (slot 2) can be shipped twice with no blocking
  // result read in between (leaves after the split read, then every node at the next level when
  // none of them can split), so the wait is explicit instead of relying on the level's fetch.
  const uint8_t* ship(const tmog::Staging& st, int k) {
    const size_t n = st.buf.size() ? st.buf.size() : 16;
    if (sl.copied[k]) hchk(hipEventSynchronize(sl.copied[k]), "stage copy wait");
    else hchk(hipEventCreateWithFlags(&sl.copied[k], hipEventDisableTiming), "event create");
    grow_pin(sl.pin[k], sl.pin_cap[k], n, sl.stream);
    grow_dev(sl.dev[k], sl.dev_cap[k], n, sl.stream);
    if (st.buf.size()) {
      std::memcpy(sl.pin[k], st.buf.data(), st.buf.size());
      hchk(hipMemcpyAsync(sl.dev[k], sl.pin[k], st.buf.size(), hipMemcpyHostToDevice, sl.stream), "stage copy");
      hchk(hipEventRecord(sl.copied[k], sl.stream), "event record");
    }
    return sl.dev[k];
  }
  int64_t* hist_buffer(int k, size_t words) {
    grow_dev(sl.hist[k], sl.hist_cap[k], words * sizeof(int64_t), sl.stream);
    return (int64_t*)sl.hist[k];
  }
  uint8_t* result_buffer(size_t bytes) {
    grow_dev(sl.res_dev, sl.res_cap, bytes, sl.stream);
    return sl.res_dev;
  }
  const uint8_t* fetch(const uint8_t* dev, size_t bytes) {
    grow_pin(sl.res_pin, sl.res_pin_cap, bytes, sl.stream);
    hchk(hipMemcpyAsync(sl.res_pin, dev, bytes, hipMemcpyDeviceToHost, sl.stream), "result copy");
    hchk(hipStreamSynchronize(sl.stream), "result sync");
    return sl.res_pin;
  }
  void zero_segments(int64_t* hist, const int64_t* off, const int64_t* size, int n, int64_t mx, int64_t dense, int per,
                     int S, int n_dense) {
    kchk(tmog_hip_zero_segments(hist, off, size, n, mx, dense, per, S, sl.stream, n_dense, nullptr), "zero_segments");
  }
  // staged statistics of the entry buffer position ``p`` points into (rows or rows_alt), or null
  int32_t* gh_of(const uint32_t* p) const {
    if (a.gh == nullptr || a.gh_alt == nullptr || a.mode != 2) return nullptr;
    if (p >= a.rows && p < a.rows + a.n_entries) return a.gh + 2 * (p - a.rows);
    if (p >= a.rows_alt && p < a.rows_alt + a.n_entries) return a.gh_alt + 2 * (p - a.rows_alt);
    return nullptr;
  }
  void hist_build(const tmog::GrowArgs& g, const uint32_t* rows, const void* items, int n_items, const int32_t* nfo,
                  const int32_t* flist, const int32_t* nmd, const int64_t* nho, int64_t* hist, int, const int64_t*,
                  const int64_t*, const int32_t*, const int32_t*, const int32_t*, const int64_t*, int Sc,
                  int n_wide, int need_general) {
    if (n_items)
      kchk(tmog_hip_hist_build(g.Xb, g.F, rows, items, n_items, nfo, flist, nmd, nho, hist, g.B, g.mode, g.S, g.y,
                               g.t1, g.t2, g.stride, g.qscale, g.mode == 2 ? g.missing_bin : -1, g.csr_ptr,
                               g.csr_col, Sc, n_wide, need_general, sl.stream, gh_of(rows), nullptr, g.wide_rows, g.Xh,
                               g.Fh),
           "hist_build");
  }
  int stat_chunk(int B, int S) const { return tmog_hip_hist_stat_chunk(B, S); }
  void hist_subtract(int64_t* hist, const int64_t* prev, const int64_t* poff, const int64_t* soff,
                     const int64_t* ooff, const int64_t* size, int n, int64_t mx, int64_t dense, int per, int S) {
    kchk(tmog_hip_hist_subtract(hist, prev, poff, soff, ooff, size, n, mx, dense, per, S, sl.stream), "hist_subtract");
  }
  void pair_scan(const tmog::GrowArgs& g, int64_t* hist, const int64_t* prev, const int64_t* poff, const int32_t* sj,
                 const int32_t* bj, int n_pairs, const int64_t* nho, const int32_t* nnf, const int32_t* nfo,
                 const int32_t* flist, const float* params, const int32_t* nmd, int max_nf, int m, int n_multi) {
    grow_dev(sl.cand, sl.cand_cap, tmog_hip_split_cand_bytes(m, max_nf, g.B, g.S), sl.stream);
    kchk(tmog_hip_pair_scan(hist, prev, poff, sj, bj, n_pairs, nho, nnf, nfo, flist, g.n_bins, g.B, g.S, g.kind, params,
                            g.missing_bin, nmd, g.qinv, max_nf, sl.cand, n_multi, sl.stream, nullptr),
         "pair_scan");
  }
  void split_find(const tmog::GrowArgs& g, const int64_t* hist, int m, const int64_t* nho, const int32_t* nnf,
                  const int32_t* nfo, const int32_t* flist, const float* params, const int32_t* nmd, int max_nf,
                  int32_t* feat, int32_t* bin, float* gain, uint8_t* dl, float* left, float* tot, int64_t* cursors,
                  int n_multi, const tmog::FpSlice& fps) {
    grow_dev(sl.cand, sl.cand_cap, tmog_hip_split_cand_bytes(m, max_nf, g.B, g.S), sl.stream);
    const char* fr_env = std::getenv("TMOG_FUSED_REDUCE");      // read per call: A/B within one process
    const bool fused_reduce = !(fr_env && fr_env[0] == '0');
    if (fused_reduce && sl.done_cap < (size_t)m) {     // grow-only, zeroed; the kernels leave it zeroed
      uint8_t* p = reinterpret_cast<uint8_t*>(sl.done);
      size_t cap = sl.done_cap * sizeof(unsigned);
      sl.done = nullptr;
      sl.done_cap = 0;
      const size_t n = (size_t)m + m / 2 + 256;
      tmog::grow_device(p, cap, (size_t)m * sizeof(unsigned), n * sizeof(unsigned), sl.stream);
      hchk(hipMemsetAsync(p, 0, n * sizeof(unsigned), sl.stream), "memset done");
      sl.done = reinterpret_cast<unsigned*>(p);
      sl.done_cap = n;
    }
    kchk(tmog_hip_split_find(hist, m, nho, nnf, nfo, flist, g.n_bins, g.B, g.S, g.kind, params, g.missing_bin, nmd,
                             g.qinv, max_nf, sl.cand, feat, bin, gain, dl, left, tot, cursors, n_multi, fps.rec,
                             fps.rec_bytes, fps.mlo, fps.nml, fps.obase, sl.stream, fused_reduce ? sl.done : nullptr,
                             nullptr),
         "split_find");
  }
  // RCCL send / receive buffers come from plain hipMalloc (grow-only; never from the stream-ordered
  // pool of grow_dev): the collective library inspects and may register the buffers it is given.
  static void grow_plain(uint8_t*& p, size_t& cap, size_t need, hipStream_t s) {
    if (need <= cap && p != nullptr) return;
    if (p) {
      hchk(hipStreamSynchronize(s), "sync before rccl buffer realloc");
      hipError_t e = hipFree(p);
      p = nullptr;
      cap = 0;
      hchk(e, "hipFree");
    }
    const size_t nc = need + need / 2 + 4096;
    hchk(hipMalloc((void**)&p, nc), "hipMalloc");
    cap = nc;
  }
  uint8_t* fp_send_buffer(size_t bytes) {
    grow_plain(sl.fp_send, sl.fp_send_cap, bytes, sl.stream);
    return sl.fp_send;
  }
  // One RCCL all-gather of the level's split records over xGMI (this group's communicator, on the
  // group's stream: no host round trip), then the merge kernel rewrites the decisions in place.
  void fp_exchange_merge(const tmog::GrowArgs& g, const uint8_t* rec, int m, size_t rb, int32_t* feat, int32_t* bin,
                         float* gain, uint8_t* dl, float* left) {
    const size_t bytes = rb * (size_t)m;
    grow_plain(sl.fp_recv, sl.fp_recv_cap, bytes * (size_t)g.fp_world, sl.stream);
    ncclComm_t comm = (ncclComm_t)g.fp_comm[group];
    if (comm == nullptr) {        // single-GPU projection of a rank group: the exchange answered locally
      for (int r = 0; r < g.fp_world; ++r)
        hchk(hipMemcpyAsync(sl.fp_recv + (size_t)r * bytes, rec, bytes, hipMemcpyDeviceToDevice, sl.stream),
             "fp local exchange");
    } else {
      ncclResult_t r;
      {
        // enqueue under a process-wide lock: the job groups' host threads issue their (independent,
        // per-communicator) collectives concurrently, and RCCL's enqueue path keeps process-global state
        std::lock_guard<std::mutex> lk(rccl_mutex());
        r = ncclAllGather(rec, sl.fp_recv, bytes, ncclUint8, comm, sl.stream);
      }
      if (r != ncclSuccess) throw std::runtime_error(std::string("ncclAllGather: ") + ncclGetErrorString(r));
    }
    kchk(tmog_hip_fp_merge(sl.fp_recv, g.fp_world, m, (int64_t)rb, g.S, feat, bin, gain, dl, left, sl.stream),
         "fp_merge");
  }
  void partition_fused(const tmog::GrowArgs& g, const uint32_t* rows, uint32_t* rows_alt, const void* items, int n,
                       const int64_t* nb, const int64_t* nc, const int32_t* feat, const int32_t* bin, const uint8_t* dl,
                       const float* params, const float* gain, int64_t* cursors) {
    int32_t* gi = gh_of(rows);
    int32_t* go = gh_of(rows_alt);
    if ((gi == nullptr) != (go == nullptr)) gi = go = nullptr;
    kchk(tmog_hip_partition_fused(g.Xb, g.F, rows, rows_alt, items, n, nb, nc, feat, bin, dl, params, gain,
                                  g.missing_bin, cursors, g.XbT, g.N, sl.stream, gi, go, nullptr, g.wide_rows),
         "partition_fused");
  }
  void partition_nodes(const tmog::GrowArgs&, const uint32_t*, uint32_t*, int, const int64_t*, const int64_t*,
                       const int32_t*, const int32_t*, const uint8_t*, const int64_t*, int64_t*) {
    throw std::logic_error("partition_nodes is the CPU backend's path");
  }
  void leaf_collect(const uint32_t* rows, const void* items, int n, uint32_t* out_rows, int32_t* out_gid) {
    kchk(tmog_hip_leaf_collect(rows, items, n, out_rows, out_gid, sl.stream, nullptr, nullptr), "leaf_collect");
  }
  void finish() {}
};

}  // namespace

extern "C" {

static void segv_backtrace(int sig) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  const char msg[] = "\n[tmog] native fault, backtrace:\n";
  (void)!write(2, msg, sizeof(msg) - 1);
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

void* tmog_hip_grow_forest(const tmog::GrowArgs* args) {
  static bool handler = false;
  if (!handler && std::getenv("TMOG_GROW_TRACE")) {   // debugging aid: name the faulting native frame
    signal(SIGSEGV, segv_backtrace);
    handler = true;
  }
  tmog::GrowResult* res = new tmog::GrowResult();
  const tmog::GrowArgs& a = *args;
  const int ng = a.n_groups;
  res->groups.resize(ng);
  std::vector<hipStream_t> own(ng, nullptr);   // each slot's own stream, restored after the call
  int swapped = 0;
  const int sb = a.slot_base;
  try {
    if (sb < 0 || sb + ng > (int)slots().size()) throw std::runtime_error("too many job groups");
    if (a.fp_world > 0 && a.fp_comm == nullptr) throw std::runtime_error("feature-parallel growth needs communicators");
    int dev = 0;
    hchk(hipGetDevice(&dev), "hipGetDevice");
    (void)tmog_hip_tree_prime();     // best effort, before the group threads' first launches (a failure here
                                     // leaves the lazy load to the first launch, as before)
    hipStream_t base = (hipStream_t)a.stream;
    static const bool base_ok = [] { const char* e = std::getenv("TMOG_GROW_ON_BASE"); return !(e && e[0] == '0'); }();
    // Group 0 runs on the caller's stream itself (no fork / join for single-group calls: boosting parts and
    // concurrent learners each call with one group). Other groups run on the stream the caller assigned to their
    // slot (tmog_hip_slot_stream: a side stream of the process-wide set, ops/streams.py -- groups may share
    // one), else on the slot's own stream. Every earlier use of a slot is ordered before `base` by the join of
    // the call that made it; this call orders each group stream after `base` again.
    const bool on_base = base_ok && base != nullptr;
    std::vector<char> joined(ng, 0);
    hipEvent_t ready;
    hchk(hipEventCreateWithFlags(&ready, hipEventDisableTiming), "event");
    hchk(hipEventRecord(ready, base), "event record");
    for (int g = 0; g < ng; ++g) {
      GpuSlot& s = slots()[sb + g];
      hipStream_t use;
      if (on_base && g == 0) {
        use = base;
      } else if (s.ext_set && a.fp_world == 0) {
        use = s.ext;           // feature-parallel groups keep streams of their own (one collective order each)
      } else {
        if (s.stream == nullptr || s.device != dev) {
          hchk(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking), "stream");
          s.device = dev;
        }
        use = s.stream;
      }
      own[g] = s.stream;
      swapped = g + 1;
      s.stream = use;
      if (use != base) {
        hchk(hipStreamWaitEvent(use, ready, 0), "wait ready");
        joined[g] = 1;
      }
    }
    std::vector<std::string> errs(ng);
    std::vector<std::thread> th;
    // feature-parallel: the groups' per-level all-gathers are enqueued in one rank-independent order
    tmog::FpTurns turns(ng);
    tmog::FpTurns* tp = a.fp_world > 0 ? &turns : nullptr;
    for (int g = 0; g < ng; ++g) {
      th.emplace_back([&, g]() {
        try {
          hchk(hipSetDevice(dev), "hipSetDevice");
          GpuBackend bk(slots()[sb + g], a, g);
          tmog::grow_group(bk, a, g, res->groups[g], tp);
        } catch (const std::exception& e) {
          errs[g] = e.what();
        }
        turns.finish(g);
      });
    }
    for (auto& t : th) t.join();
    for (int g = 0; g < ng; ++g) {
      if (!joined[g]) continue;
      hipEvent_t done;
      hchk(hipEventCreateWithFlags(&done, hipEventDisableTiming), "event");
      hchk(hipEventRecord(done, slots()[sb + g].stream), "event record");
      hchk(hipStreamWaitEvent(base, done, 0), "base wait");
      hchk(hipEventDestroy(done), "event destroy");
    }
    hchk(hipEventDestroy(ready), "event destroy");
    for (int g = 0; g < ng; ++g) slots()[sb + g].stream = own[g];
    swapped = 0;
    for (int g = 0; g < ng; ++g)
      if (!errs[g].empty()) throw std::runtime_error("group " + std::to_string(g) + ": " + errs[g]);
  } catch (const std::exception& e) {
    res->status = -1;
    res->error = e.what();
    for (int g = 0; g < swapped; ++g) slots()[sb + g].stream = own[g];
  }
  return res;
}

// TMOG_GROW_TIMING diagnostics: out = [plan, issue, wait] host nanoseconds and the level count, summed over
// every grower call since the last reset
void tmog_hip_grow_timing(int64_t* out, int reset) {
  tmog::GrowTiming& t = tmog::grow_timing();
  out[0] = t.plan.load();
  out[1] = t.issue.load();
  out[2] = t.wait.load();
  out[3] = t.levels.load();
  if (reset) t.plan = t.issue = t.wait = t.levels = 0;
}

// The stream the job group using native slot `slot` runs on in later multi-group calls (null clears: the slot's
// own stream). Set by models/tree_engine.py from the process-wide side streams before each such call.
int tmog_hip_slot_stream(int slot, void* stream, int set) {
  if (slot < 0 || slot >= (int)slots().size()) return -1;
  slots()[slot].ext = (hipStream_t)stream;
  slots()[slot].ext_set = set != 0;
  return 0;
}

// dev_alloc.hpp: the out-of-memory handler (torch.cuda.empty_cache from ops/_native.py) and the test hook
// that fails the n-th native allocation from now (0 = off).
void tmog_hip_set_oom_handler(void (*fn)()) { tmog::g_oom_handler.store(fn); }
void tmog_hip_fail_alloc(long n) { tmog::g_fail_at.store(n > 0 ? n : 0); }

int tmog_hip_grow_status(void* h, char* msg, int cap) {
  tmog::GrowResult* r = (tmog::GrowResult*)h;
  if (msg && cap > 0) {
    std::strncpy(msg, r->error.c_str(), cap - 1);
    msg[cap - 1] = 0;
  }
  return r->status;
}
int64_t tmog_hip_grow_nodes(void* h, int g) { return tmog::result_nodes((tmog::GrowResult*)h, g); }
int64_t tmog_hip_grow_leaf_count(void* h, int g) { return ((tmog::GrowResult*)h)->groups[g].leaf_count; }
void tmog_hip_grow_copy(void* h, int g, int64_t* tree, int64_t* feat, int64_t* bin, uint8_t* dl, double* gain,
                        double* tot, int64_t* left, int64_t* right) {
  tmog::result_copy((tmog::GrowResult*)h, g, tree, feat, bin, dl, gain, tot, left, right);
}
void tmog_hip_grow_free(void* h) { delete (tmog::GrowResult*)h; }

// RCCL communicators of the feature-parallel tree grower (one per job group; models/tree_engine.py
// FeatureParallel creates them once per process: rank 0's unique id is broadcast through
// torch.distributed, then every rank joins on its current device).
int tmog_hip_rccl_unique_id(char* out, int cap) {
  if (cap < (int)sizeof(ncclUniqueId)) return -2;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return -1;
  std::memcpy(out, &id, sizeof(id));
  return (int)sizeof(id);
}
void* tmog_hip_rccl_comm_init(const char* id_bytes, int world, int rank) {
  ncclUniqueId id;
  std::memcpy(&id, id_bytes, sizeof(id));
  ncclComm_t comm = nullptr;
  std::lock_guard<std::mutex> lk(rccl_mutex());
  if (ncclCommInitRank(&comm, world, id, rank) != ncclSuccess) return nullptr;
  // one small all-gather right away, from this (single) thread: RCCL finishes its lazy per-communicator
  // setup (connections, kernel resources) here instead of inside the grower's concurrent group threads
  hipStream_t s = nullptr;
  void* buf = nullptr;
  bool ok = hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess &&
            hipMalloc(&buf, 64 * (size_t)world) == hipSuccess &&
            ncclAllGather((char*)buf + 64 * (size_t)rank, buf, 64, ncclUint8, comm, s) == ncclSuccess &&
            hipStreamSynchronize(s) == hipSuccess;
  if (buf) (void)hipFree(buf);
  if (s) (void)hipStreamDestroy(s);
  if (!ok) {
    ncclCommDestroy(comm);
    return nullptr;
  }
  return (void*)comm;
}
// All-gather of `bytes` per rank on `stream` for the device-planned feature-parallel levels (tree_resident.hip).
// comm == nullptr with world > 1 is the single-GPU projection of a rank group (scripts/project_schedule.py): the
// other ranks' records are answered locally with copies of this rank's, so the level's exchange and merge run
// with the group's shapes (the trees then only see this rank's feature slice).
int tmog_hip_fp_allgather(const void* send, void* recv, int64_t bytes, void* comm, int world, hipStream_t stream) {
  if (bytes <= 0) return 0;
  if (comm == nullptr) {
    for (int r = 0; r < world; ++r) {
      const hipError_t e = hipMemcpyAsync((uint8_t*)recv + (size_t)r * (size_t)bytes, send, (size_t)bytes,
                                          hipMemcpyDeviceToDevice, stream);
      if (e != hipSuccess) return (int)e;
    }
    return 0;
  }
  std::lock_guard<std::mutex> lk(rccl_mutex());
  const ncclResult_t r = ncclAllGather(send, recv, (size_t)bytes, ncclUint8, (ncclComm_t)comm, stream);
  return r == ncclSuccess ? 0 : 1000 + (int)r;
}

int tmog_hip_rccl_comm_destroy(void* comm) {
  return comm ? (int)ncclCommDestroy((ncclComm_t)comm) : 0;
}

}  // extern "C"

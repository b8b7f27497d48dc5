// CPU backend of the native tree grower (common/tree_grow.hpp): host memory, the tmog_*_cpu twins of
// the HIP kernels (tree_cpu.cpp), groups grown one after the other with the same per-group seeds as
// the GPU backend, so both produce bit-identical forests.
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "common/tree_grow.hpp"

extern "C" {
int tmog_hist_build_cpu(const uint8_t* Xb, int64_t N, int F, const uint32_t* rows, int n_nodes,
                        const int64_t* node_begin, const int64_t* node_count, const int32_t* node_feat_off,
                        const int32_t* node_nfeat, const int32_t* feat_list, const int32_t* node_model,
                        const int64_t* node_hist_off, int64_t* hist, int B, int mode, int S, const float* y,
                        const float* t1, const float* t2, int64_t model_stride, const float* qscale, int wide);
int tmog_split_find_cpu(const int64_t* hist, int n_nodes, const int64_t* node_hist_off, const int32_t* node_nfeat,
                        const int32_t* node_feat_off, const int32_t* feat_list, const int32_t* feat_nbins, int B,
                        int S, int kind, const float* node_params, int missing_bin, const int32_t* node_model,
                        const double* qinv, int32_t* out_feat, int32_t* out_bin, float* out_gain,
                        uint8_t* out_default_left, float* out_left, float* out_total, uint8_t* rec,
                        int64_t rec_bytes, int fp_mlo, int fp_nml, int fp_obase);
int tmog_partition_cpu(const uint8_t* Xb, int F, const uint32_t* rows_in, uint32_t* rows_out, int n_nodes,
                       const int64_t* node_begin, const int64_t* node_count, const int32_t* split_feat,
                       const int32_t* split_bin, const uint8_t* default_left, int missing_bin,
                       const int64_t* out_begin, int64_t* out_left_count, int wide);
}

namespace {

struct CpuBackend {
  static constexpr bool kGPU = false;
  int group = 0;
  std::vector<uint8_t> fp_recv;
  std::vector<int32_t> feats;
  std::vector<uint8_t> res;
  std::vector<int64_t> hist[2];

  const int32_t* all_features(int F) {
    feats.resize(F);
    for (int i = 0; i < F; ++i) feats[i] = i;
    return feats.data();
  }
  const uint8_t* ship(const tmog::Staging& st, int) { return st.buf.data(); }
  int stat_chunk(int, int S) const { return S; }
  std::vector<uint8_t> fp_send;
  uint8_t* fp_send_buffer(size_t bytes) {
    fp_send.assign(bytes ? bytes : 8, 0);
    return fp_send.data();
  }
  int64_t* hist_buffer(int k, size_t words) {
    if (hist[k].size() < words) hist[k].resize(words + words / 4 + 16);
    return hist[k].data();
  }
  uint8_t* result_buffer(size_t bytes) {
    res.assign(bytes, 0);
    return res.data();
  }
  const uint8_t* fetch(const uint8_t* p, size_t) { return p; }
  void zero_segments(int64_t*, const int64_t*, const int64_t*, int, int64_t, int64_t, int, int, int) {}   // CPU hist zeroes per node
  void hist_build(const tmog::GrowArgs& g, const uint32_t* rows, const void*, int, const int32_t*,
                  const int32_t* flist, const int32_t*, const int64_t*, int64_t* hist, int nbuild,
                  const int64_t* bnb, const int64_t* bnc, const int32_t* bnfo, const int32_t* bnnf,
                  const int32_t* bnmd, const int64_t* bnho, int, int, int) {
    if (nbuild)
      tmog_hist_build_cpu(g.Xb, g.N, g.F, rows, nbuild, bnb, bnc, bnfo, bnnf, flist, bnmd, bnho, hist, g.B, g.mode,
                          g.S, g.y, g.t1, g.t2, g.stride, g.qscale, g.wide_rows);
  }
  void hist_subtract(int64_t* hist, const int64_t* prev, const int64_t* poff, const int64_t* soff,
                     const int64_t* ooff, const int64_t* size, int n, int64_t, int64_t, int, int) {
    for (int j = 0; j < n; ++j) {
      const int64_t* p = prev + poff[j];
      const int64_t* s = hist + soff[j];
      int64_t* o = hist + ooff[j];
      for (int64_t k = 0; k < size[j]; ++k) o[k] = p[k] - s[k];
    }
  }
  void split_find(const tmog::GrowArgs& g, const int64_t* hist, int m, const int64_t* nho, const int32_t* nnf,
                  const int32_t* nfo, const int32_t* flist, const float* params, const int32_t* nmd, int,
                  int32_t* feat, int32_t* bin, float* gain, uint8_t* dl, float* left, float* tot, int64_t*, int,
                  const tmog::FpSlice& fps) {
    tmog_split_find_cpu(hist, m, nho, nnf, nfo, flist, g.n_bins, g.B, g.S, g.kind, params, g.missing_bin, nmd, g.qinv,
                        feat, bin, gain, dl, left, tot, fps.rec, fps.rec_bytes, fps.mlo, fps.nml, fps.obase);
  }
  // all-gather through the caller's exchange function (torch.distributed gloo in the CPU tests)
  void fp_exchange_merge(const tmog::GrowArgs& g, const uint8_t* rec, int m, size_t rb, int32_t* feat, int32_t* bin,
                         float* gain, uint8_t* dl, float* left) {
    const size_t bytes = rb * (size_t)m;
    fp_recv.assign(bytes * (size_t)g.fp_world, 0);
    if (g.fp_exchange == nullptr) throw std::runtime_error("feature-parallel growth needs an exchange function");
    if (g.fp_exchange(g.fp_ctx, group, rec, fp_recv.data(), (int64_t)bytes) != 0)
      throw std::runtime_error("feature-parallel exchange failed");
    tmog::fp_merge_host(fp_recv.data(), g.fp_world, m, rb, g.S, feat, bin, gain, dl, left);
  }
  void partition_fused(const tmog::GrowArgs&, const uint32_t*, uint32_t*, const void*, int, const int64_t*,
                       const int64_t*, const int32_t*, const int32_t*, const uint8_t*, const float*, const float*,
                       int64_t*) {
    throw std::logic_error("partition_fused is the GPU backend's path");
  }
  void partition_nodes(const tmog::GrowArgs& g, const uint32_t* rows, uint32_t* rows_alt, int ns, const int64_t* nb,
                       const int64_t* nc, const int32_t* f, const int32_t* b, const uint8_t* d, const int64_t* ob,
                       int64_t* nl) {
    tmog_partition_cpu(g.Xb, g.F, rows, rows_alt, ns, nb, nc, f, b, d, g.missing_bin, ob, nl, g.wide_rows);
  }
  void leaf_collect(const uint32_t* rows, const void* items, int n, uint32_t* out_rows, int32_t* out_gid) {
    const tmog::LeafItemH* it = (const tmog::LeafItemH*)items;
    for (int i = 0; i < n; ++i) {
      std::memcpy(out_rows + it[i].out, rows + it[i].begin, sizeof(uint32_t) * it[i].count);
      for (int64_t k = 0; k < it[i].count; ++k) out_gid[it[i].out + k] = it[i].gid;
    }
  }
  void finish() {}
};

}  // namespace

extern "C" {

void* tmog_grow_forest_cpu(const tmog::GrowArgs* args) {
  tmog::GrowResult* res = new tmog::GrowResult();
  res->groups.resize(args->n_groups);
  try {
    const int ng = args->n_groups;
    if (args->fp_world > 0 && ng > 1 && std::getenv("TMOG_CPU_GROUP_THREADS") != nullptr) {
      // one host thread per group, as the GPU backend runs them: exercises the exchange turn order
      // (tmog::FpTurns) across ranks on the CPU (gloo) path
      tmog::FpTurns turns(ng);
      std::vector<std::string> errs(ng);
      std::vector<std::thread> th;
      for (int g = 0; g < ng; ++g) {
        th.emplace_back([&, g]() {
          try {
            CpuBackend bk;
            bk.group = g;
            tmog::grow_group(bk, *args, g, res->groups[g], &turns);
          } catch (const std::exception& e) {
            errs[g] = e.what();
          }
          turns.finish(g);
        });
      }
      for (auto& t : th) t.join();
      for (int g = 0; g < ng; ++g)
        if (!errs[g].empty()) throw std::runtime_error("group " + std::to_string(g) + ": " + errs[g]);
    } else {
      for (int g = 0; g < ng; ++g) {
        CpuBackend bk;
        bk.group = g;
        tmog::grow_group(bk, *args, g, res->groups[g]);
      }
    }
  } catch (const std::exception& e) {
    res->status = -1;
    res->error = e.what();
  }
  return res;
}

int tmog_grow_status_cpu(void* h, char* msg, int cap) {
  tmog::GrowResult* r = (tmog::GrowResult*)h;
  if (msg && cap > 0) {
    std::strncpy(msg, r->error.c_str(), cap - 1);
    msg[cap - 1] = 0;
  }
  return r->status;
}
int64_t tmog_grow_nodes_cpu(void* h, int g) { return tmog::result_nodes((tmog::GrowResult*)h, g); }
int64_t tmog_grow_leaf_count_cpu(void* h, int g) { return ((tmog::GrowResult*)h)->groups[g].leaf_count; }
void tmog_grow_copy_cpu(void* h, int g, int64_t* tree, int64_t* feat, int64_t* bin, uint8_t* dl, double* gain,
                        double* tot, int64_t* left, int64_t* right) {
  tmog::result_copy((tmog::GrowResult*)h, g, tree, feat, bin, dl, gain, tot, left, right);
}
void tmog_grow_free_cpu(void* h) { delete (tmog::GrowResult*)h; }

}  // extern "C"

// Histogram tree engine kernels for CDNA4 (gfx950).
//
// Replaces the per-level statistics aggregation of Spark MLlib trees (DTStatsAggregator, used by
// OpRandomForestClassifier.scala:59-154 / OpGBTClassifier.scala:47-142 / DT) and XGBoost4J's
// hist updater (OpXGBoostClassifier.scala:47-403): SURVEY.md kernels K23 (histogram, split scan,
// partition), K24/K25 (GBT / Newton stats) and K29 (ensemble traversal).
//
// Layout contract (identical to ../host/tree_cpu.cpp, orchestrated by models/tree_engine.py):
//   Xb    uint8 [N][F] row-major bins          rows  uint32 (row | weight<<24)
//   hist  int64 fixed point, node j at node_hist_off[j], index ((fl * B) + bin) * S + s;
//         value = hist * qinv[model][s] (see "Fixed-point statistics" below)
//
// Histogram kernel mapping (wave64-first): a wave-instruction covers R = 64 / FG rows x FG
// features -- lane (r, f) handles feature f of row r, so lanes of one instruction touch distinct LDS
// histogram rows (feature-major, padded by one word so bank = f + bin*S + s spreads). All waves of
// the workgroup share the table through integer LDS atomics; the R copies are folded on the way out
// and a node covered by one row-chunk stores with plain stores, otherwise 64-bit integer atomics.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdlib>
#include <stdint.h>
#include <math.h>

#define TM_MAX_S 16          // narrow split scan / staged-record path: S <= 16 statistics
#define TM_WIDE_MAX_S 256    // wide path (many classes): statistic-chunked histograms, LDS split scan
#define TM_WIDE_MAX_BS 16384 // wide split scan keeps one feature's B x S int64 histogram in LDS

namespace {

struct HistItem {
  int32_t node;     // node slot
  int32_t fg0;      // first local feature of this group
  int32_t nf;       // features in this group (<= 64)
  int32_t excl;     // bit 0: this item alone covers node rows for its features (plain stores)
                    // bit 1: every feature of the group has one present bin (register accumulation)
  int64_t begin;    // first row entry
  int64_t count;    // row entries in this chunk
};

// Fixed-point statistics. Every per-row contribution is quantised to an integer,
//   q = rint(v * qscale[model][s]),  |q| <= qmax = (2^31 - 1) / chunk_rows - 1,
// with power-of-two scales chosen on the device from the per-model max |v| (tree_engine._quant_scales).
// Workgroup LDS partials are int32 (ds_add_u32: ~17x the throughput of ds_add_f32 on gfx950, see
// benchmarks/lds_atomic_bench.hip) and cannot overflow for a chunk of <= chunk_rows rows; the
// global histogram is int64, so sums, the subtraction trick and the split scan's prefix sums are
// exact and order-independent -- GPU and CPU (../host/tree_cpu.cpp) histograms are bit-identical and
// runs are deterministic. Class counts (MODE 0) and the variance count are integer weights (scale 1).
//
// Staged row record (entry bits, q0, q1, q2):
//   MODE 0 (class counts):   q0 = w, q1 = class
//   MODE 1 (variance stats): q0 = w, q1 = q(w*t), q2 = q(w*t*t)
//   MODE 2 (grad / hess):    q0 = q(w*g), q1 = q(w*h)
// Entry decoding. Packed (default): row | weight << 24 (rows < 2^24). Wide rows (training sets of >= 2^24
// rows, GrowArgs.wide_rows): the entry is the 32-bit row id and every entry weighs 1 -- weighted roots are
// expanded into repeated entries by the host (models/tree_engine.py), which adds the same integer
// statistics to every histogram.
__device__ __forceinline__ uint32_t ent_row(uint32_t e, int wide) { return wide ? e : (e & 0xFFFFFFu); }
__device__ __forceinline__ uint32_t ent_w(uint32_t e, int wide) { return wide ? 1u : (e >> 24); }

template <int MODE>
__device__ __forceinline__ int4 stage_row(uint32_t e, int64_t model, int64_t stride, const float* __restrict__ y,
                                          const float* __restrict__ t1, const float* __restrict__ t2,
                                          const float* __restrict__ qs, int wide) {
  const int64_t r = ent_row(e, wide);
  const float w = (float)ent_w(e, wide);
  int4 s;
  s.x = (int)e;
  if (MODE == 0) {
    s.y = (int)ent_w(e, wide); s.z = (int)y[r]; s.w = 0;
  } else if (MODE == 1) {
    const float t = t1[model * stride + r];
    const float wt = w * t;
    s.y = (int)ent_w(e, wide);
    s.z = (int)rintf(wt * qs[1]);
    s.w = (int)rintf((wt * t) * qs[2]);
  } else {
    s.y = (int)rintf((w * t1[model * stride + r]) * qs[0]);
    s.z = (int)rintf((w * t2[model * stride + r]) * qs[1]);
    s.w = 0;
  }
  return s;
}

// Statistic chunk [s0, s0 + Sc) of a histogram item (Sc < S when B * S does not fit the LDS table:
// many classes or wide bins -- each chunk is its own item, writing disjoint words).
template <int MODE>
__device__ __forceinline__ void add_row(int* my, int bin, int S, int s0, int Sc, const int4& st) {
  if (MODE == 0) {
    const int c = st.z - s0;
    if (c >= 0 && c < Sc) atomicAdd(my + bin * Sc + c, st.y);
  } else if (MODE == 1) {
    int* hb = my + bin * Sc;
    const int v[3] = {st.y, st.z, st.w};
    for (int k = 0; k < Sc; ++k) atomicAdd(hb + k, v[s0 + k]);
  } else {
    int* hb = my + bin * Sc;
    if (Sc == 2) {
      atomicAdd(hb, st.y); atomicAdd(hb + 1, st.z);
    } else {
      atomicAdd(hb, s0 ? st.z : st.y);
    }
  }
}

// Histogram build. Lane mapping (wave64): a wave-instruction covers R = 64 / FG rows x FG features;
// lane (rsub, fidx) owns histogram row (rsub, fidx) of the workgroup's LDS table, shared by its 4
// waves through integer LDS atomics -- lanes of one instruction never address the same word.
//  1. each wave takes 64 row entries at once (one coalesced load of the packed (row, weight) list)
//     and every lane gathers + quantises the statistics of *its* row (64 independent gathers);
//  2. the 64 records are staged in a wave-private LDS slot (one ds_write_b128 per lane);
//  3. lane (rsub, fidx) walks the staged rows R at a time, 8 rows unrolled: 8 broadcast ds_read_b128,
//     8 independent bin gathers Xb[row*F + feat] in flight, then the ds_add_u32s.
//
// Sparse missing bin (MODE 2, skip_bin >= 0; XGBoost's sparsity-aware histogram): entries whose bin is
// the reserved missing bin (XGBoost ``missing`` = 0.0 in the reference grid, i.e. every zero of the
// one-hot / null-indicator columns) issue no LDS atomic. Each wave instead folds its 64 staged rows'
// (g, h) into the chunk total with two wave reductions, and before the write-out the missing bin of
// every feature is recovered exactly as chunk total - sum of the other bins (integer arithmetic, so
// the histogram stays bit-identical to the CPU twin). Masking lanes does not shorten an LDS atomic
// wave-instruction, so this alone saves little; what it enables is the register path below.
//
// Register path (excl bit 1, sparse mode only): when every feature of the group has a single present
// bin (one-hot and null-indicator columns under ``missing`` = 0: value 1 -> bin 0, value 0 -> missing
// bin) a lane just sums the (g, h) of its rows with bin 0 in two registers -- no LDS atomics in the
// row loop at all, one per lane at the end. The tree grower groups such columns together
// (common/tree_grow.hpp), so on the headline table ~40 % of the feature groups skip the atomics.
// PMC on the tree micro-benchmark: ~0.064 LDS wave-instructions per CU-cycle at ~11 cycles each for
// a ds_add_u32 -> the LDS atomic unit is ~70 % busy; VALU ~12 % busy, so trading atomics for VALU pays.
// CSR path (excl bit 2, MODE 2 with a sparse missing bin): one item covers ALL one-present-bin columns
// of a node row-chunk. Such a column's histogram has two non-zero bins -- the present bin 0 and the
// missing bin -- and the missing bin is the chunk total minus bin 0, so only the entries with bin 0
// matter: the row's CSR list (csr_ptr / csr_col, local column ids). The wave walks its 64 staged
// rows one at a time with the lanes spread over that row's list (coalesced 2-byte id loads; the ids
// of one row are distinct, so an LDS atomic wave-instruction never conflicts), kCsrU rows in flight.
// On the headline table that is ~50 entries per row instead of ~530 byte gathers.
constexpr int kCsrU = 16;
constexpr int kCsrG = 8;     // row slots per lane group in flight (register budget of the whole kernel)

// Wave64 inclusive prefix sum of an int64 on the DPP lane network (GFX9 sequence: row_shr 1 / 2 / 4 / 8 inside
// the 16-lane rows, then row_bcast:15 into rows 1 and 3 and row_bcast:31 into rows 2 and 3), two 32-bit halves
// moved per step and added as one 64-bit value: 12 DPP moves + 6 adds instead of 6 x 2 ds_bpermute (LDS
// crossbar) + selects. Lanes without a source keep `old` = 0. Integer sums: identical to any other order.
template <int CTRL, int ROWS>
__device__ __forceinline__ int64_t dpp_shift64(int64_t v) {
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(uint64_t)v, CTRL, ROWS, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)((uint64_t)v >> 32), CTRL, ROWS, 0xF, false);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint64_t)(uint32_t)lo);
}
__device__ __forceinline__ int64_t wave_scan64(int64_t v) {
  v += dpp_shift64<0x111, 0xF>(v);    // row_shr:1
  v += dpp_shift64<0x112, 0xF>(v);    // row_shr:2
  v += dpp_shift64<0x114, 0xF>(v);    // row_shr:4
  v += dpp_shift64<0x118, 0xF>(v);    // row_shr:8
  v += dpp_shift64<0x142, 0xA>(v);    // row_bcast:15 -> rows 1, 3
  v += dpp_shift64<0x143, 0xC>(v);    // row_bcast:31 -> rows 2, 3
  return v;
}

// Wave64 int32 sum / max of non-negatives on DPP, result wave-uniform (the inclusive scan ends in lane 63): 6 DPP
// adds + one readlane instead of 6 ds_bpermute round trips through the LDS crossbar. Whole wave active.
template <bool MAX>
__device__ __forceinline__ int wave_reduce32(int v) {
#define TM_DPP_STEP(CTRL, ROWS)                                                         \
  {                                                                                     \
    const int t = __builtin_amdgcn_update_dpp(0, v, CTRL, ROWS, 0xF, false);           \
    v = MAX ? max(v, t) : v + t;                                                        \
  }
  TM_DPP_STEP(0x111, 0xF) TM_DPP_STEP(0x112, 0xF) TM_DPP_STEP(0x114, 0xF) TM_DPP_STEP(0x118, 0xF)
  TM_DPP_STEP(0x142, 0xA) TM_DPP_STEP(0x143, 0xC)
#undef TM_DPP_STEP
  return __builtin_amdgcn_readlane(v, 63);
}

__device__ __forceinline__ int64_t readlane64(int64_t v, int l) {
  const int lo = __builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)v, l);
  const int hi = __builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint64_t)(uint32_t)lo);
}

__device__ __forceinline__ void hist_csr_item(const HistItem& it, const uint32_t* __restrict__ rows,
                                              const int32_t* __restrict__ node_model,
                                              const int64_t* __restrict__ node_hist_off, int64_t* __restrict__ hist,
                                              int B, int S, const float* __restrict__ t1,
                                              const float* __restrict__ t2, int64_t stride,
                                              const float* __restrict__ qscale, int skip_bin,
                                              const int64_t* __restrict__ csr_ptr,
                                              const uint16_t* __restrict__ csr_col, int* lds,
                                              const int2* __restrict__ gh, int wide) {
  const int nf = it.nf;
  int* a0 = lds;            // bin-0 sum of q(w g) per column
  int* a1 = lds + nf;       // bin-0 sum of q(w h)
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int nwaves = blockDim.x >> 6;
  const int soff = (2 * nf + 3) & ~3;        // per-wave row stage + list lengths after the sums
  int4* stg = reinterpret_cast<int4*>(lds + soff) + wave * 64;
  int* lens = lds + soff + 4 * 64 * nwaves + wave * 64;
  for (int i = threadIdx.x; i < 2 * nf; i += blockDim.x) lds[i] = 0;
  __syncthreads();
  const int64_t model = node_model ? node_model[it.node] : 0;
  const float* qs = qscale + model * S;
  const uint32_t* rp = rows + it.begin;
  const int64_t cnt = it.count;
  const float* t1m = t1 + model * stride;
  const float* t2m = t2 + model * stride;
  // One-chunk-ahead pipeline (as in hist_wide_item): the next chunk's entry is loaded before this
  // chunk's list walk, its statistics and list bounds after the first batch of id loads.
  const int64_t step = (int64_t)nwaves * 64;
  // staged statistics (gh != null): the entry's quantised (g, h) ride with the entry in node order, one
  // coalesced 8-byte load instead of two scattered 4-byte gathers per row
  const int2* ghp = gh ? gh + it.begin : nullptr;
  uint32_t e_n = 0;
  float g_n = 0.f, h_n = 0.f;
  int2 q_n = make_int2(0, 0);
  int64_t p0_n = 0, p1_n = 0;
  if ((int64_t)wave * 64 < cnt) {
    const int64_t i0 = min((int64_t)wave * 64 + lane, cnt - 1);
    e_n = rp[i0];
    const int64_t r = ent_row(e_n, wide);
    if (ghp) q_n = ghp[i0];
    else { g_n = t1m[r]; h_n = t2m[r]; }
    p0_n = csr_ptr[r]; p1_n = csr_ptr[r + 1];
  }
  for (int64_t base = (int64_t)wave * 64; base < cnt; base += step) {
    const int nrows = (int)min((int64_t)64, cnt - base);
    const float wt = (float)ent_w(e_n, wide);
    int4 mine;
    mine.x = (int)e_n;
    mine.y = ghp ? q_n.x : (int)rintf((wt * g_n) * qs[0]);
    mine.z = ghp ? q_n.y : (int)rintf((wt * h_n) * qs[1]);
    mine.w = 0;
    const int64_t q0 = p0_n;
    const int len = lane < nrows ? (int)(p1_n - p0_n) : 0;
    const bool more = base + step < cnt;             // wave-uniform
    const int64_t i_n = min(base + step + lane, cnt - 1);
    if (more) e_n = rp[i_n];
    // Row records go through the wave's LDS stage (q(g), q(h), list start) + list length: the lane groups
    // read them with plain LDS loads (no cross-lane shuffles, whose sources must all be active) and keep
    // only the entry ids in registers across the id gathers.
    stg[lane] = make_int4(mine.y, mine.z, (int)(uint32_t)(uint64_t)q0, (int)((uint64_t)q0 >> 32));
    lens[lane] = len;
    // Lane groups of W (a power of two >= this chunk's longest list, <= 64) take one row each, so a
    // wave-instruction covers 64 / W rows at (nearly) full lane use instead of one row per instruction
    // (the headline's rows carry ~17 entries).
    const int mx = wave_reduce32<true>(len);
    const int W = mx <= 8 ? 8 : mx <= 16 ? 16 : mx <= 32 ? 32 : 64;
    const int RPI = 64 / W;
    const int rs = lane / W, k = lane - rs * W;
    __builtin_amdgcn_s_waitcnt(0xC07F);        // lgkmcnt(0): staged records visible to the wave
    __builtin_amdgcn_wave_barrier();
    for (int j0 = 0; j0 < nrows; j0 += RPI * kCsrG) {
      int col[kCsrG];
      bool ok[kCsrG];
#pragma unroll
      for (int u = 0; u < kCsrG; ++u) {
        const int src = j0 + u * RPI + rs;
        const int sl = min(src, 63);
        const int ln = src < nrows ? lens[sl] : 0;
        const int4 rr = stg[sl];
        const int64_t k0 = (int64_t)(((uint64_t)(uint32_t)rr.w << 32) | (uint64_t)(uint32_t)rr.z);
        ok[u] = k < ln;
        col[u] = csr_col[ok[u] ? k0 + k : k0 > 0 ? k0 - 1 : 0];   // unpredicated load of a valid id
      }
      __builtin_amdgcn_sched_barrier(0);
      if (j0 == 0 && more) {
        const int64_t r = ent_row(e_n, wide);
        if (ghp) q_n = ghp[i_n];
        else { g_n = t1m[r]; h_n = t2m[r]; }
        p0_n = csr_ptr[r]; p1_n = csr_ptr[r + 1];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < kCsrG; ++u)
        if (ok[u]) {
          const int2 gh = *reinterpret_cast<const int2*>(&stg[min(j0 + u * RPI + rs, 63)]);
          atomicAdd(a0 + col[u], gh.x);
          atomicAdd(a1 + col[u], gh.y);
        }
      if (W == 64) {                       // lists longer than the lane group
#pragma unroll
        for (int u = 0; u < kCsrG; ++u) {
          const int src = j0 + u * RPI + rs;
          const int sl = min(src, 63);
          const int ln = src < nrows ? lens[sl] : 0;
          if (ln <= 64) continue;
          const int4 rr = stg[sl];
          const int64_t k0 = (int64_t)(((uint64_t)(uint32_t)rr.w << 32) | (uint64_t)(uint32_t)rr.z);
          for (int kk = k + 64; kk < ln; kk += 64) {
            const int c = csr_col[k0 + kk];
            atomicAdd(a0 + c, rr.x);
            atomicAdd(a1 + c, rr.y);
          }
        }
      }
    }
    __builtin_amdgcn_wave_barrier();           // the stage is rewritten by the next chunk
  }
  __syncthreads();
  // Only bin 0 of these columns is written: the split scan and split reduce evaluate a one-present-bin
  // column from its bin 0 and the node totals (read from a multi-bin column), and zero_segments /
  // hist_subtract maintain only that word, so no other word of these columns is ever live.
  int64_t* out = hist + node_hist_off[it.node] + (int64_t)it.fg0 * B * S;
  const int per = B * S;
  const bool excl = (it.excl & 1) != 0;
  for (int k = threadIdx.x; k < nf * S; k += blockDim.x) {
    const int f = k / S, s = k - f * S;
    const int v = s ? a1[f] : a0[f];
    int64_t* w = out + (int64_t)f * per + s;
    if (excl) *w = v;
    else if (v != 0) atomicAdd(reinterpret_cast<unsigned long long*>(w), (unsigned long long)(int64_t)v);
  }
}


// Wide-load path (MODE 2, excl bit 4): a dense group of FG <= 64 multi-bin columns that are physically
// contiguous and dword aligned in Xb (col0 % 4 == 0, row stride % 4 == 0; the XGBoost learner pads its
// growth-order matrix to that). Lane (rs, d) loads dword d of the group's row segment -- 4 bins of one
// row in one 4-byte load -- so a wave-instruction covers 64 / ceil(FG/4) rows (4 for FG = 64) and
// kWideU instructions keep 4x the bytes of the byte-gather path in flight for the same registers (the
// kernel is gather-latency bound: MI355X_MICROARCH.md "72 KiB in flight per CU"). The statistics are
// packed as one 64-bit word (q(g) << 32) + q(h) per (feature, bin) -- h >= 0 and its per-item sum stays
// below 2^31 (qmax), so the low half never carries -- and added with ONE ds_add_u64 instead of two
// ds_add_u32. Output is identical (integer sums) to the byte path and the CPU twin.
constexpr int kWideU = 16;

// LDS table layout (bank-conflict free): the ds_add_u64 of a wave-instruction is serviced in 4 groups of 16
// contiguous lanes, and a group conflicts when two of its lanes hit one bank (byte address / 4 mod 32). Lanes are
// (rs, d) with the dword count padded to NP = 16 / 8 / 4 / 2 / 1 (a power of two), so a 16-lane group holds
// 16 / NP rows of one group of NP dwords; lane position p = lane % 16 is unique in its group. Word
// (k, b, p) = k * (B + 1) * 16 + b * 16 + p holds feature 4 d + k, bin b, for row slot p / NP: its bank pair
// 2 p mod 32 depends on the lane position only, never on the (data-dependent) bin -- the feature-major layout
// put lanes of random bins on random banks (~3.5-way per group). Row slots of one group are separate copies,
// folded before the write-out; the table stays 64 x (B + 1) words.
__device__ __forceinline__ void hist_wide_item(const HistItem& it, const uint8_t* __restrict__ Xb, int F, int col0,
                                               const uint32_t* __restrict__ rows,
                                               const int32_t* __restrict__ node_model,
                                               const int64_t* __restrict__ node_hist_off, int64_t* __restrict__ hist,
                                               int B, const float* __restrict__ t1, const float* __restrict__ t2,
                                               int64_t stride, const float* __restrict__ qscale, int skip_bin,
                                               int* lds, const int2* __restrict__ gh, int wide) {
  const int FG = it.nf;
  const int ND = (FG + 3) >> 2;                    // dwords of the group's row segment (<= 16)
  const int NP = ND <= 1 ? 1 : ND <= 2 ? 2 : ND <= 4 ? 4 : ND <= 8 ? 8 : 16;
  const int RPI = 64 / NP;                         // rows per wave-instruction (>= 4)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
  const int rs = lane / NP, d = lane - rs * NP;
  const int pos = lane & 15;
  const int sub = (B + 1) * 16;                    // words per k-plane
  unsigned long long* tab = reinterpret_cast<unsigned long long*>(lds);
  const int twords = 4 * sub;                      // == 64 * (B + 1): the launcher's LDS size
  const int toff = (2 * twords + 3) & ~3;
  int4* stage = reinterpret_cast<int4*>(lds + toff) + wave * 64;
  int* tot = lds + toff + 4 * 64 * nwaves;
  for (int i = threadIdx.x; i < twords; i += blockDim.x) tab[i] = 0ull;
  if (threadIdx.x < 2) tot[threadIdx.x] = 0;
  __syncthreads();
  const bool sparse = skip_bin >= 0;
  const int64_t model = node_model ? node_model[it.node] : 0;
  const float* qs = qscale + model * 2;
  const uint32_t* rp = rows + it.begin;
  const int64_t cnt = it.count;
  // buffer loads: one descriptor for the group's first column (wave-uniform) and a 32-bit per-lane byte
  // offset row * F + 4 d (the grower takes this path only for matrices below 2 GiB) -- one VGPR per
  // gather address instead of two. Pad lanes (d >= ND) re-read the last dword and add 0.
  const uint64_t xbase = (uint64_t)(uintptr_t)(Xb + col0);
  const uint32_t xlo = __builtin_amdgcn_readfirstlane((uint32_t)xbase);
  const uint32_t xhi = __builtin_amdgcn_readfirstlane((uint32_t)(xbase >> 32));
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(uintptr_t)(((uint64_t)xhi << 32) | xlo), (short)0, 0x7FFFFFFF, 0x00020000);
  const uint32_t lane_off = 4u * (uint32_t)min(d, ND - 1);
  const float* t1m = t1 + model * stride;
  const float* t2m = t2 + model * stride;
  // Software pipeline over the wave's 64-row chunks: the next chunk's row entry is loaded before this
  // chunk's bin gathers and its (g, h) right after them, so the dependent entry -> statistic -> bin
  // latency chain of a chunk overlaps the previous chunk's gathers and atomics instead of adding up.
  const int64_t step = (int64_t)nwaves * 64;
  const int2* ghp = gh ? gh + it.begin : nullptr;   // staged (g, h): coalesced with the entries
  uint32_t e_n = 0;
  float g_n = 0.f, h_n = 0.f;
  int2 q_n = make_int2(0, 0);
  if ((int64_t)wave * 64 < cnt) {
    const int64_t i0 = min((int64_t)wave * 64 + lane, cnt - 1);
    e_n = rp[i0];
    if (ghp) q_n = ghp[i0];
    else {
      g_n = t1m[ent_row(e_n, wide)];
      h_n = t2m[ent_row(e_n, wide)];
    }
  }
  for (int64_t base = (int64_t)wave * 64; base < cnt; base += step) {
    const int nrows = (int)min((int64_t)64, cnt - base);
    const float wt = (float)ent_w(e_n, wide);
    int4 mine;
    mine.x = (int)e_n;
    mine.y = ghp ? q_n.x : (int)rintf((wt * g_n) * qs[0]);
    mine.z = ghp ? q_n.y : (int)rintf((wt * h_n) * qs[1]);
    mine.w = 0;
    const bool more = base + step < cnt;             // wave-uniform
    const int64_t i_n = min(base + step + lane, cnt - 1);
    if (more) {
      e_n = rp[i_n];
      if (ghp) q_n = ghp[i_n];                 // independent of the entry: issued with it
    }
    stage[lane] = make_int4(mine.y, mine.z, mine.x, 0);   // (q(g), q(h), entry): (g, h) 8-byte aligned
    if (sparse) {
      const int a = wave_reduce32<false>(lane < nrows ? mine.y : 0);
      const int b = wave_reduce32<false>(lane < nrows ? mine.z : 0);
      if (lane == 0) {
        atomicAdd(tot, a);
        atomicAdd(tot + 1, b);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);        // lgkmcnt(0): staged records visible to the wave
    __builtin_amdgcn_wave_barrier();
    {                                          // RPI * kWideU >= 64 (NP <= 16): one pass covers the chunk
      // only the row ids stay in registers across the gathers; (g, h) are re-read from the LDS stage
      // at the atomics (fewer VGPRs -> more waves, i.e. more gathers in flight per CU)
      uint32_t off[kWideU], w[kWideU];
#pragma unroll
      for (int u = 0; u < kWideU; ++u)
        off[u] = (wide ? (uint32_t)stage[min(u * RPI + rs, 63)].z * (uint32_t)F     // < 2^31 (grower guard)
                       : __umul24((uint32_t)stage[min(u * RPI + rs, 63)].z & 0xFFFFFFu, (uint32_t)F)) + lane_off;
#pragma unroll
      for (int u = 0; u < kWideU; ++u) w[u] = __builtin_amdgcn_raw_buffer_load_b32(xrs, (int)off[u], 0, 0);
      __builtin_amdgcn_sched_barrier(0);       // keep the next chunk's statistic loads behind the gathers
      if (more && !ghp) {
        g_n = t1m[ent_row(e_n, wide)];
        h_n = t2m[ent_row(e_n, wide)];
      }
      __builtin_amdgcn_sched_barrier(0);
      // branch-free: masked-off work (rows past the chunk, pad features) adds 0 to the lane's own word
      // instead of toggling EXEC around every atomic (a masked lane costs the same)
#pragma unroll
      for (int u = 0; u < kWideU; ++u) {
        const bool live = u * RPI + rs < nrows;
        const int2 st = *reinterpret_cast<const int2*>(&stage[min(u * RPI + rs, 63)]);
        const unsigned long long pk = live ? ((unsigned long long)(uint32_t)st.x << 32) + (unsigned long long)(uint32_t)st.y
                                           : 0ull;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int bin = (int)((w[u] >> (8 * k)) & 0xFFu);
          atomicAdd(tab + k * sub + bin * 16 + pos, 4 * d + k < FG ? pk : 0ull);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  // fold the 16 / NP row-slot copies of every (k, bin) row into its first NP words
  if (NP < 16) {
    for (int i = threadIdx.x; i < 4 * B * NP; i += blockDim.x) {
      const int r = i / NP, dd = i - r * NP;                   // r = k * B + bin
      unsigned long long* row = tab + (r / B) * sub + (r % B) * 16;
      unsigned long long acc = row[dd];
      for (int c = NP; c < 16; c += NP) acc += row[c + dd];
      row[dd] = acc;
    }
    __syncthreads();
  }
  auto tix = [sub](int f, int b) { return (f & 3) * sub + b * 16 + (f >> 2); };
  if (sparse) {       // missing bin = chunk totals - the other bins, packed into the spare bin-B word
    for (int f = threadIdx.x; f < FG; f += blockDim.x) {
      long long g = 0, h = 0;
      for (int b = 0; b < B; ++b) {
        if (b == skip_bin) continue;
        const unsigned long long v = tab[tix(f, b)];
        g += (long long)v >> 32;
        h += (long long)(v & 0xFFFFFFFFull);
      }
      const long long mg = (long long)tot[0] - g, mh = (long long)tot[1] - h;
      tab[tix(f, B)] = ((unsigned long long)mg << 32) + (unsigned long long)(uint32_t)mh;
    }
    __syncthreads();
  }
  int64_t* out = hist + node_hist_off[it.node] + (int64_t)it.fg0 * B * 2;
  const bool excl = (it.excl & 1) != 0;
  for (int k = threadIdx.x; k < FG * B; k += blockDim.x) {
    const int f = k / B, b = k - f * B;
    const unsigned long long v = tab[tix(f, (sparse && b == skip_bin) ? B : b)];
    const int64_t g = (long long)v >> 32, h = (long long)(v & 0xFFFFFFFFull);
    int64_t* o = out + (int64_t)k * 2;
    if (excl) {
      o[0] = g;
      o[1] = h;
    } else {
      if (g != 0) atomicAdd(reinterpret_cast<unsigned long long*>(o), (unsigned long long)g);
      if (h != 0) atomicAdd(reinterpret_cast<unsigned long long*>(o + 1), (unsigned long long)h);
    }
  }
}

constexpr int HIST_U = 16;   // row bins gathered per lane before their LDS atomics (loads in flight)

// Diagnostics only (tmog_hip_debug_flags, TMOG_HIST_DEBUG): bit 0 skips CSR items, bit 1 skips wide /
// dense multi-bin items -- the trees are then wrong; used to time the item kinds separately.
__device__ int g_hist_debug = 0;

// Wide-load items in a kernel of their own (TMOG_HIST_WIDE_SPLIT=1; the grower puts them first): the mixed
// kernel's register budget is set by its general and CSR paths, this one's by the wide path alone, so
// more waves -- more row gathers in flight -- fit on a CU (OCC = requested waves per SIMD: 7 is
// the LDS limit of these 21 KB workgroups, at a couple of spilled registers; TMOG_HIST_WIDE_OCC picks).
template <int OCC>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC))) hist_wide_kernel(
    const uint8_t* __restrict__ Xb, int F, const uint32_t* __restrict__ rows, const HistItem* __restrict__ items,
    const int32_t* __restrict__ node_feat_off, const int32_t* __restrict__ feat_list,
    const int32_t* __restrict__ node_model, const int64_t* __restrict__ node_hist_off, int64_t* __restrict__ hist,
    int B, const float* __restrict__ t1, const float* __restrict__ t2, int64_t stride,
    const float* __restrict__ qscale, int skip_bin, const int2* __restrict__ gh, int wide,
    const uint8_t* __restrict__ Xh, int Fh) {
  extern __shared__ int lds_w[];
  if (g_hist_debug & 2) return;
  const HistItem it = items[blockIdx.x];
  hist_wide_item(it, Xh, Fh, feat_list[node_feat_off[it.node] + it.fg0], rows, node_model, node_hist_off, hist, B,
                 t1, t2, stride, qscale, skip_bin, lds_w, gh, wide);
}


// GEN = false (MODE 2 launches whose items are all CSR / wide-load, the XGBoost case): the byte-gather
// path is not compiled in, so its registers do not cap the occupancy of the other two (106 -> ~74 VGPRs).
template <int MODE, bool GEN = true>
__global__ void __launch_bounds__(256) hist_build_kernel(
    const uint8_t* __restrict__ Xb, int F, const uint32_t* __restrict__ rows, const HistItem* __restrict__ items,
    const int32_t* __restrict__ node_feat_off, const int32_t* __restrict__ feat_list,
    const int32_t* __restrict__ node_model, const int64_t* __restrict__ node_hist_off, int64_t* __restrict__ hist,
    int B, int S, const float* __restrict__ y, const float* __restrict__ t1, const float* __restrict__ t2,
    int64_t stride, const float* __restrict__ qscale, int skip_bin, const int64_t* __restrict__ csr_ptr,
    const uint16_t* __restrict__ csr_col, int Sc, const int2* __restrict__ gh, const int* __restrict__ dcount,
    int wide, const uint8_t* __restrict__ Xh, int Fh) {
  extern __shared__ __attribute__((aligned(16))) int lds[];
  // dcount (device-planned levels, tree_resident.hip): the grid is an upper bound, the item count is on the device
  if (dcount != nullptr && (int)blockIdx.x >= *dcount) return;
  const HistItem it = items[blockIdx.x];
  const int s0 = ((it.excl >> 8) & 0xFF) * Sc;   // statistic chunk of this item (excl bits 8..15)
  const int sc = min(Sc, S - s0);
  if (MODE == 2 && g_hist_debug) {
    if ((g_hist_debug & 1) && (it.excl & 4)) return;
    if ((g_hist_debug & 2) && !(it.excl & 4)) return;
  }
  if (MODE == 2 && (it.excl & 4)) {
    hist_csr_item(it, rows, node_model, node_hist_off, hist, B, S, t1, t2, stride, qscale, skip_bin, csr_ptr,
                  csr_col, lds, gh, wide);
    return;
  }
  if (MODE == 2 && (it.excl & 16)) {        // wide-load items read the compact matrix (GrowArgs.Xh, or Xb)
    hist_wide_item(it, Xh, Fh, feat_list[node_feat_off[it.node] + it.fg0], rows, node_model, node_hist_off, hist, B,
                   t1, t2, stride, qscale, skip_bin, lds, gh, wide);
    return;
  }
  if constexpr (!GEN) {
    return;
  } else {
  const int FG = it.nf;
  const int R = 64 / FG;
  const int rowstride = B * sc + 1;           // padded feature row (this item's statistic chunk)
  const int ncopy_words = R * FG * rowstride;  // <= 64 * rowstride
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int nwaves = blockDim.x >> 6;
  int4* stage = reinterpret_cast<int4*>(lds + ((ncopy_words + 3) & ~3)) + wave * 64;
  int* tot = lds + ((ncopy_words + 3) & ~3) + 4 * 64 * 4;     // chunk totals (sparse missing bin)
  const bool sparse = MODE == 2 && skip_bin >= 0;
  const bool regacc = sparse && (it.excl & 2);
  const bool excl = (it.excl & 1) != 0;
  for (int i = threadIdx.x; i < ncopy_words; i += blockDim.x) lds[i] = 0;
  if (threadIdx.x < TM_MAX_S) tot[threadIdx.x] = 0;
  __syncthreads();

  const int rsub = lane / FG;
  const int fidx = lane - rsub * FG;
  const bool active = rsub < R;
  const int feat = active ? feat_list[node_feat_off[it.node] + it.fg0 + fidx] : 0;
  const int64_t model = node_model ? node_model[it.node] : 0;
  const float* qs = qscale + model * S;
  int* my = lds + (rsub * FG + fidx) * rowstride;
  const uint32_t* rp = rows + it.begin;
  const int64_t cnt = it.count;

  int racc0 = 0, racc1 = 0;     // register path sums (bin 0 of this lane's feature)
  // Loads are never predicated (a masked "load or skip" makes hipcc branch around every load and wait
  // vmcnt(0) per element): out-of-range slots read a valid dummy record and are masked at the atomic.
  for (int64_t base = (int64_t)wave * 64; base < cnt; base += (int64_t)nwaves * 64) {
    const int64_t ri = min(base + lane, cnt - 1);
    const int nrows = (int)min((int64_t)64, cnt - base);
    int4 mine;
    if (MODE == 2 && gh) {
      const int2 q = gh[it.begin + ri];
      mine = make_int4((int)rp[ri], q.x, q.y, 0);
    } else {
      mine = stage_row<MODE>(rp[ri], model, stride, y, t1, t2, qs, wide);
    }
    stage[lane] = mine;
    if (sparse) {
      // chunk totals: one wave reduction of the 64 staged (g, h) records, one LDS add per wave
      const int a = wave_reduce32<false>(lane < nrows ? mine.y : 0);
      const int b = wave_reduce32<false>(lane < nrows ? mine.z : 0);
      if (lane == 0) {
        atomicAdd(tot, a);
        atomicAdd(tot + 1, b);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);        // lgkmcnt(0): staged records visible to the wave
    __builtin_amdgcn_wave_barrier();
    if (regacc) {
      for (int j0 = 0; j0 < nrows; j0 += R * 8) {
        int4 st[8];
        int bin[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) st[u] = stage[min(j0 + u * R + rsub, 63)];
#pragma unroll
        for (int u = 0; u < 8; ++u) bin[u] = (int)Xb[(int64_t)ent_row((uint32_t)st[u].x, wide) * F + feat];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const bool hit = j0 + u * R + rsub < nrows && bin[u] == 0;
          racc0 += hit ? st[u].y : 0;
          racc1 += hit ? st[u].z : 0;
        }
      }
      __builtin_amdgcn_wave_barrier();
      continue;
    }
    for (int j0 = 0; j0 < nrows; j0 += R * HIST_U) {
      int4 st[HIST_U];
      int bin[HIST_U];
#pragma unroll
      for (int u = 0; u < HIST_U; ++u) st[u] = stage[min(j0 + u * R + rsub, 63)];
#pragma unroll
      for (int u = 0; u < HIST_U; ++u) bin[u] = (int)Xb[(int64_t)ent_row((uint32_t)st[u].x, wide) * F + feat];
#pragma unroll
      for (int u = 0; u < HIST_U; ++u)
        if (active && j0 + u * R + rsub < nrows && bin[u] != skip_bin) add_row<MODE>(my, bin[u], S, s0, sc, st[u]);
    }
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();

  int64_t* out = hist + node_hist_off[it.node] + (int64_t)it.fg0 * B * S;
  const int words = FG * B * S;
  if (regacc) {
    if (active) {
      atomicAdd(my, racc0);
      atomicAdd(my + 1, racc1);
    }
    __syncthreads();
  }
  if (sparse) {
    // fold the R copies into copy 0, then recover each feature's missing bin from the chunk totals
    if (R > 1) {
      for (int k = threadIdx.x; k < words; k += blockDim.x) {
        const int f = k / (B * S);
        const int rem = k - f * (B * S);
        int acc = 0;
        for (int r = 0; r < R; ++r) acc += lds[(r * FG + f) * rowstride + rem];
        lds[f * rowstride + rem] = acc;
      }
      __syncthreads();
    }
    for (int t = threadIdx.x; t < FG * S; t += blockDim.x) {
      const int f = t / S, s = t - (t / S) * S;
      int* row = lds + f * rowstride;
      int sum = 0;
      for (int b = 0; b < B; ++b) sum += (b == skip_bin) ? 0 : row[b * S + s];
      row[skip_bin * S + s] = tot[s] - sum;
    }
    __syncthreads();
    // excl bit 3: the group's columns have one present bin and only their bin 0 is live (the grower
    // orders multi-bin columns first and zero / subtract maintain bin 0 alone, see hist_csr_item)
    const int wlimit = (it.excl & 8) ? S : B * S;
    for (int k = threadIdx.x; k < words; k += blockDim.x) {
      const int f = k / (B * S);
      if (k - f * (B * S) >= wlimit) continue;
      const int64_t acc = lds[f * rowstride + (k - f * (B * S))];
      if (excl) out[k] = acc;
      else if (acc != 0) atomicAdd(reinterpret_cast<unsigned long long*>(out + k), (unsigned long long)acc);
    }
    return;
  }
  // fold the R private copies and write the node histogram of this feature group (chunk slots only)
  const int cwords = FG * B * sc;
  for (int k = threadIdx.x; k < cwords; k += blockDim.x) {
    const int f = k / (B * sc);
    const int rem = k - f * (B * sc);
    int64_t acc = 0;
    for (int r = 0; r < R; ++r) acc += lds[(r * FG + f) * rowstride + rem];
    const int bin = rem / sc, c = rem - bin * sc;
    int64_t* w = out + ((int64_t)f * B + bin) * S + s0 + c;
    if (excl) *w = acc;
    else if (acc != 0) atomicAdd(reinterpret_cast<unsigned long long*>(w), (unsigned long long)acc);
  }
  }   // GEN
}

// sibling = parent - small (histogram subtraction trick), size words each
// Word k of a node's live region: with dense >= 0 the region is the first `dense` words (the multi-bin
// columns, every bin) followed by bin 0 of each one-present-bin column -- the only words the split scan,
// the split reduce and the next level's subtraction read of those columns (tree_grow.hpp orders the
// multi-bin columns first), so ~530 of the headline table's ~730 columns move S words instead of B * S.
__device__ __forceinline__ int64_t live_words(int64_t sz, int64_t dense, int per, int S) {
  return (dense < 0 || sz <= dense) ? sz : dense + (sz - dense) / per * S;
}
// 32-bit index math (a node's histogram is < 2^31 words; int64 division is a long software sequence)
__device__ __forceinline__ int live_word(int k, int dense, int per, int S) {
  if (dense < 0 || k < dense) return k;
  const int t = k - dense, f = t / S;
  return dense + f * per + (t - f * S);
}

__global__ void hist_subtract_kernel(int64_t* __restrict__ hist, const int64_t* __restrict__ parent,
                                     const int64_t* __restrict__ parent_off, const int64_t* __restrict__ small_off,
                                     const int64_t* __restrict__ out_off, const int64_t* __restrict__ size, int n,
                                     int64_t dense, int per, int S) {
  const int j = blockIdx.y;
  if (j >= n) return;
  const int sz = (int)live_words(size[j], dense, per, S);
  const int dn = (int)dense;
  const int64_t* p = parent + parent_off[j];
  const int64_t* s = hist + small_off[j];
  int64_t* o = hist + out_off[j];
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < sz; k += gridDim.x * blockDim.x) {
    const int w = live_word(k, dn, per, S);
    o[w] = p[w] - s[w];
  }
}

// zero the histograms of nodes built from several row chunks (their items accumulate atomically);
// single-chunk and derived nodes are fully overwritten, so the level buffer is never memset whole
__global__ void zero_segments_kernel(int64_t* __restrict__ hist, const int64_t* __restrict__ off,
                                     const int64_t* __restrict__ size, int n, int64_t dense, int per, int S,
                                     int n_dense, const int* __restrict__ dcnt) {
  const int j = blockIdx.y;
  if (dcnt != nullptr) {       // device-planned level: [segments, whole-node segments] on the device
    n = dcnt[0];
    n_dense = dcnt[1];
  }
  if (j >= n) return;
  int64_t* o = hist + off[j];
  const int64_t dj = j < n_dense ? dense : 0;      // segments past n_dense start at a one-present-bin region
  const int sz = (int)live_words(size[j], dj, per, S);
  const int dn = (int)dj;
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < sz; k += gridDim.x * blockDim.x)
    o[live_word(k, dn, per, S)] = 0;
}

// ------------------------------------------------------------------------------- split finding
// No FMA contraction from here on: gains are evaluated with exactly the CPU twin's IEEE operation
// sequence, so near-tied candidates resolve identically on both paths (hipcc contracts by default).
#pragma clang fp contract(off)
__device__ __forceinline__ double impurity_dev(const double* st, int S, int kind, double* cnt) {
  if (kind == 0 || kind == 1) {
    double n = 0;
    for (int s = 0; s < S; ++s) n += st[s];
    *cnt = n;
    if (n <= 0) return 0.0;
    double imp = kind == 0 ? 1.0 : 0.0;
    for (int s = 0; s < S; ++s) {
      const double p = st[s] / n;
      if (kind == 0) imp -= p * p;
      else if (p > 0) imp -= p * log2(p);
    }
    return imp;
  }
  if (kind == 2) {
    const double n = st[0];
    *cnt = n;
    if (n <= 0) return 0.0;
    const double m = st[1] / n;
    return st[2] / n - m * m;
  }
  *cnt = st[1];
  return 0.0;
}

// Loops over the statistics of a node inside the SM-templated scans: unrolled to the compile-time bound with a
// runtime guard, so the per-statistic arrays (totals, scales, left / right sums) stay in registers -- a loop to
// the runtime S indexes them dynamically and puts them in scratch memory
#define TM_FOR_S(s) _Pragma("unroll") for (int s = 0; s < SM; ++s) if (s < S)

// impurity_dev over a register array of at most SM statistics (same operation order)
template <int SM>
__device__ __forceinline__ double impurity_reg(const double* st, int S, int kind, double* cnt) {
  if (kind == 0 || kind == 1) {
    double n = 0;
    TM_FOR_S(s) n += st[s];
    *cnt = n;
    if (n <= 0) return 0.0;
    double imp = kind == 0 ? 1.0 : 0.0;
    TM_FOR_S(s) {
      const double p = st[s] / n;
      if (kind == 0) imp -= p * p;
      else if (p > 0) imp -= p * log2(p);
    }
    return imp;
  }
  if (kind == 2) {
    const double n = st[0];
    *cnt = n;
    if (n <= 0) return 0.0;
    const double m = st[1] / n;
    return st[2] / n - m * m;
  }
  *cnt = st[1];
  return 0.0;
}

struct Best {
  double gain;
  int f;    // local feature index (tie-break)
  int b;
  int dl;
};
static_assert(sizeof(Best) == 24, "candidate record: three 8-byte words (store_best_sc1 / load_best_sc1)");

// A candidate as three 8-byte agent-scope (sc1) words -- stores that bypass the XCD-local caching and
// loads served from L2, for the hand-off between workgroups of the fused split reduction
__device__ __forceinline__ void store_best_sc1(Best* p, const Best& b) {
  uint64_t* w = reinterpret_cast<uint64_t*>(p);
  __hip_atomic_store(w, (uint64_t)__double_as_longlong(b.gain), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(w + 1, (uint64_t)(uint32_t)b.f | ((uint64_t)(uint32_t)b.b << 32), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(w + 2, (uint64_t)(uint32_t)b.dl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ Best load_best_sc1(const Best* p) {
  const uint64_t* w = reinterpret_cast<const uint64_t*>(p);
  const uint64_t g = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t fb = __hip_atomic_load(w + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t dl = __hip_atomic_load(w + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return Best{__longlong_as_double((long long)g), (int)(uint32_t)fb, (int)(uint32_t)(fb >> 32), (int)(uint32_t)dl};
}

__device__ __forceinline__ bool better(const Best& a, const Best& b) {
  if (a.gain != b.gain) return a.gain > b.gain;
  if (a.f != b.f) return a.f < b.f;
  if (a.dl != b.dl) return a.dl < b.dl;
  return a.b < b.b;
}

// Split scan, two kernels. split_scan_kernel: grid (node, feature block of FPB = 16 features); each
// of the 4 waves scans 4 features (lane = bin, B <= 64) with an exact int64 wave prefix sum of the
// fixed-point histogram, converting to double only to evaluate gains (identical arithmetic to
// tmog_split_find_cpu, so both pick the same split bit for bit); the block's best candidate goes to
// cand[node][fb]. split_reduce_kernel: one wave per node picks the best candidate with the CPU's
// tie-break (gain, then lowest feature, dl, bin) and sums the winner's left statistics. Spreading a
// node over feature blocks fills the chip at the shallow levels (6 root nodes = 6 workgroups before).
// SM = compile-time bound on S (register arrays sized to it).
constexpr int FPB = 16;      // default features per scan workgroup (TMOG_SPLIT_FPB: 4, 8 or 16; 4 waves)

// Candidate slots per node: the node's feature blocks rounded up to 16 (16 x 24 B = 3 whole 128-B lines), so
// no cache line holds two nodes' candidates -- a reducer's L2 never caches a line of a node it has not
// finished (the fused split reduction's sc1 hand-off)
static inline int cand_stride(int fbmax) { return (fbmax + 15) & ~15; }

static int split_fpb() {
  static const int v = [] {
    const char* e = std::getenv("TMOG_SPLIT_FPB");
    const int x = e ? std::atoi(e) : FPB;
    return (x == 4 || x == 8 || x == 16) ? x : FPB;
  }();
  return v;
}

// Everything the per-node split reduction reads and writes (split_reduce_kernel, or the last scan block of a
// node when the reduction is fused into the scan).
struct ReduceArgs {
  const int64_t* hist;
  const int64_t* node_hist_off;
  const int32_t* node_feat_off;
  const int32_t* feat_list;
  int B, S, missing_bin;
  const int32_t* node_model;
  const double* qinv;
  int fbmax;
  int cstride;      // candidate slots per node (fbmax rounded up to 16: 384 B, whole 128-B lines per node)
  const Best* cand;
  int32_t* out_feat;
  int32_t* out_bin;
  float* out_gain;
  uint8_t* out_dl;
  float* out_left;
  float* out_total;
  unsigned long long* cursors;
  uint8_t* rec;
  int64_t rec_bytes;
  int fp_mlo, fp_nml, fp_obase;
};

// One wave: node j's best candidate under the CPU twin's tie-break (gain, then lowest feature, dl, bin), the
// node totals and the winner's left statistics.
__device__ __forceinline__ void reduce_node(const ReduceArgs& ra, int j, int lane, bool sc1 = false) {
  const int B = ra.B, S = ra.S, fbmax = ra.fbmax, missing_bin = ra.missing_bin;
  if (ra.cursors && lane < 2) ra.cursors[2 * j + lane] = 0;   // partition_fused_kernel's per-node slot cursors
  Best b{-INFINITY, 0x7fffffff, 0, 0};
  for (int i = lane; i < fbmax; i += 64) {      // any number of feature blocks
    const Best* cp = ra.cand + (int64_t)j * ra.cstride + i;
    const Best c = sc1 ? load_best_sc1(cp) : *cp;
    if (better(c, b)) b = c;
  }
  for (int off = 32; off > 0; off >>= 1) {
    Best o;
    o.gain = __shfl_xor(b.gain, off, 64);
    o.f = __shfl_xor(b.f, off, 64);
    o.b = __shfl_xor(b.b, off, 64);
    o.dl = __shfl_xor(b.dl, off, 64);
    if (better(o, b)) b = o;
  }
  const bool found = b.f != 0x7fffffff && b.gain > -INFINITY;
  const int64_t* h = ra.hist + ra.node_hist_off[j];
  const double* qi = ra.qinv + (int64_t)(ra.node_model ? ra.node_model[j] : 0) * S;
  if (lane == 0) {
    ra.out_feat[j] = found ? ra.feat_list[ra.node_feat_off[j] + b.f] : -1;
    ra.out_bin[j] = found ? b.b : -1;
    ra.out_gain[j] = found ? (float)b.gain : -INFINITY;
    ra.out_dl[j] = (uint8_t)(found ? b.dl : 0);
  }
  for (int s = 0; s < S; ++s) {
    int64_t t = 0, l = 0;
    const int64_t* hf = h + (int64_t)(found ? b.f : 0) * B * S;
    for (int bb = lane; bb < B; bb += 64) {       // any number of bins
      t += h[(int64_t)bb * S + s];
      if (found && bb <= b.b) l += hf[(int64_t)bb * S + s];
    }
    if (found && b.dl && lane == 0) l += hf[(int64_t)missing_bin * S + s];
    for (int off = 32; off > 0; off >>= 1) {
      t += __shfl_xor(t, off, 64);
      l += __shfl_xor(l, off, 64);
    }
    if (lane == 0) {
      ra.out_total[(int64_t)j * S + s] = (float)((double)t * qi[s]);
      ra.out_left[(int64_t)j * S + s] = (float)((double)l * qi[s]);
      if (ra.rec) reinterpret_cast<float*>(ra.rec + (int64_t)j * ra.rec_bytes + 24)[s] = (float)((double)l * qi[s]);
    }
  }
  if (ra.rec && lane == 0) {   // feature-parallel split record (common/tree_grow.hpp fp_rec_bytes)
    uint8_t* r = ra.rec + (int64_t)j * ra.rec_bytes;
    *reinterpret_cast<double*>(r) = found ? b.gain : -INFINITY;
    reinterpret_cast<int32_t*>(r)[2] =
        found ? (b.f < ra.fp_nml ? ra.fp_mlo + b.f : ra.fp_obase + (b.f - ra.fp_nml)) : 0x7fffffff;
    reinterpret_cast<int32_t*>(r)[3] = found ? b.b : -1;
    reinterpret_cast<int32_t*>(r)[4] = found ? b.dl : 0;
    reinterpret_cast<int32_t*>(r)[5] = found ? ra.feat_list[ra.node_feat_off[j] + b.f] : -1;
  }
}

// Per-node split evaluation state of the narrow scans (split_scan_kernel, pair_scan_kernel): node totals
// (fixed point and scaled), the node's parameters, and this thread's best candidate so far.
template <int SM>
struct NodeScan {
  int64_t totq[SM];
  double tot[SM], q[SM];
  double tcount, pimp, parent_gain, min_inst, min_gain, mcw, lambda;
  int S, kind;
  bool allow_missing;
  Best best;

  // totq_in: the node's fixed-point totals (every lane holds the same values)
  __device__ __forceinline__ void init(const int64_t* totq_in, const double* qi, const float* P, int S_, int kind_,
                                       int missing_bin) {
    S = S_;
    kind = kind_;
    best = Best{-INFINITY, 0x7fffffff, 0, 0};
    min_inst = P[0];
    min_gain = P[1];
    mcw = P[2];
    lambda = P[3];
    allow_missing = P[5] > 0.5f && missing_bin >= 0;
    TM_FOR_S(s) {
      totq[s] = totq_in[s];
      q[s] = qi[s];
      tot[s] = (double)totq[s] * q[s];
    }
    pimp = impurity_reg<SM>(tot, S, kind, &tcount);
    parent_gain = kind == 3 ? tot[0] * tot[0] / (tot[1] + lambda) : 0.0;
  }

  // one candidate (left statistics lq, bin b, missing direction dl) with the CPU twin's arithmetic
  __device__ __forceinline__ void consider(const int64_t* lq, int f, int b, int dl) {
    double left[SM], right[SM];
    TM_FOR_S(s) {
      left[s] = (double)lq[s] * q[s];
      right[s] = (double)(totq[s] - lq[s]) * q[s];
    }
    double gain;
    bool ok = true;
    if (kind == 3) {
      // invalid by min_child_weight: skip the two fp64 divisions (whole waves skip at small nodes)
      if (left[1] < mcw || right[1] < mcw) return;
      gain = left[0] * left[0] / (left[1] + lambda) + right[0] * right[0] / (right[1] + lambda) - parent_gain;
    } else {
      double lc, rc;
      const double li = impurity_reg<SM>(left, S, kind, &lc);
      const double ri = impurity_reg<SM>(right, S, kind, &rc);
      if (lc < min_inst || rc < min_inst || lc <= 0 || rc <= 0) ok = false;
      gain = pimp - (lc / tcount) * li - (rc / tcount) * ri;
      if (gain < min_gain) ok = false;
    }
    if (ok) {
      Best c{gain, f, b, dl};
      if (better(c, best)) best = c;
    }
  }

  // multi-bin feature f: lane = bin, v = this lane's bin statistics (0 past nb), miss = the missing bin's
  // (same on every lane). Exact int64 wave prefix sum, then the lane's (bin, dl) candidates.
  __device__ __forceinline__ void scan_feature(int64_t* v, const int64_t* miss, int nb, int f, int lane) {
    TM_FOR_S(s) v[s] = wave_scan64(v[s]);
    // candidates b < nb - 1; with a missing bin dl = 0 also b = nb - 1 (present left, missing right).
    // An empty missing bin makes every dl = 1 candidate equal to its dl = 0 twin, which wins the tie
    // (better(): dl ascending; the CPU twin's first-wins scan order) -- skip them.
    bool any_miss = false;
    TM_FOR_S(s) any_miss |= miss[s] != 0;
    const int n_dl = allow_missing ? (any_miss ? 2 : 1) : 1;
    if (lane < nb - 1 + (allow_missing ? 1 : 0)) {
      for (int dl = 0; dl < n_dl; ++dl) {
        if (lane == nb - 1 && dl) continue;
        int64_t lq[SM];
        TM_FOR_S(s) lq[s] = v[s] + (dl ? miss[s] : 0);
        consider(lq, f, lane, dl);
      }
    }
  }

  // wave-level best (every lane ends with it)
  __device__ __forceinline__ void wave_best() {
    for (int off = 32; off > 0; off >>= 1) {
      Best o;
      o.gain = __shfl_xor(best.gain, off, 64);
      o.f = __shfl_xor(best.f, off, 64);
      o.b = __shfl_xor(best.b, off, 64);
      o.dl = __shfl_xor(best.dl, off, 64);
      if (better(o, best)) best = o;
    }
  }
};

// node totals from local feature 0 of a histogram (every row is counted once per feature, including the
// missing bin), on every lane of the wave
template <int SM>
__device__ __forceinline__ void node_totals(const int64_t* h, int B, int S, int lane, int64_t* totq) {
  int64_t v[SM];
  TM_FOR_S(s) v[s] = lane < B ? h[lane * S + s] : 0;     // all loads before the reductions
  TM_FOR_S(s) totq[s] = readlane64(wave_scan64(v[s]), 63);
}

template <int SM>
__global__ void __launch_bounds__(256) split_scan_kernel(
    const int64_t* __restrict__ hist, const int64_t* __restrict__ node_hist_off, const int32_t* __restrict__ node_nfeat,
    const int32_t* __restrict__ node_feat_off, const int32_t* __restrict__ feat_list,
    const int32_t* __restrict__ feat_nbins, int B, int S, int kind, const float* __restrict__ node_params,
    int missing_bin, const int32_t* __restrict__ node_model, const double* __restrict__ qinv, int fbmax,
    Best* __restrict__ cand, int n_multi, int fpb, unsigned* __restrict__ done, ReduceArgs ra,
    const int* __restrict__ dm) {
  const int cstride = ra.cstride;
  const int j = blockIdx.x / fbmax;
  const int fb = blockIdx.x - j * fbmax;
  if (dm != nullptr && j >= *dm) return;      // device-planned level: node count on the device
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // params slot 4: the node was scanned with its subtraction partner by pair_scan_kernel (same cand slots, all
  // written by that earlier launch): with the fused reduction its block 0 reduces it, the others have nothing to do
  if (node_params[(int64_t)j * 8 + 4] > 0.5f) {
    if (done && fb == 0 && wave == 0) reduce_node(ra, j, lane);
    return;
  }
  const int nf = node_nfeat[j];
  // n_multi >= 0: local features [n_multi, nf) have one present bin; their blocks (fb >= fb_multi)
  // take 256 features each, one thread per feature, instead of 16 per block through the scan
  const int f_lim = n_multi >= 0 ? min(n_multi, nf) : nf;
  const int fb_multi = n_multi >= 0 ? (n_multi + fpb - 1) / fpb : fbmax;
  const bool one_blk = fb >= fb_multi;
  __shared__ Best s_best[4];
  NodeScan<SM> ns;
  ns.best = Best{-INFINITY, 0x7fffffff, 0, 0};
  // params slot 7 = "may split" (tree_grow.hpp): nodes built only as a subtraction partner are not scanned
  if (node_params[(int64_t)j * 8 + 7] > 0.5f &&
      (one_blk ? (n_multi + (fb - fb_multi) * 256 < nf) : (fb * fpb < f_lim))) {
    const int64_t* h = hist + node_hist_off[j];
    const int32_t* fl = feat_list + node_feat_off[j];
    int64_t totq[SM];
    node_totals<SM>(h, B, S, lane, totq);
    ns.init(totq, qinv + (int64_t)(node_model ? node_model[j] : 0) * S, node_params + (int64_t)j * 8, S, kind,
            missing_bin);
    const int f_end = one_blk ? 0 : min(f_lim, (fb + 1) * fpb);
    if (one_blk) {
      const int f = n_multi + (fb - fb_multi) * 256 + (int)threadIdx.x;
      if (f < nf && ns.allow_missing && feat_nbins[fl[f]] == 1) {
        const int64_t* hf = h + (int64_t)f * B * S;
        int64_t lq[SM];
        TM_FOR_S(s) lq[s] = hf[s];
        ns.consider(lq, f, 0, 0);
      }
    }
    for (int f = fb * fpb + wave; f < f_end; f += 4) {
      const int nb = feat_nbins[fl[f]];
      const int64_t* hf = h + (int64_t)f * B * S;
      if (nb == 1) {
        // one present bin (one-hot / null indicator): the only candidate is present-left,
        // missing-right -- no scan, one lane
        if (ns.allow_missing && lane == 0) {
          int64_t lq[SM];
          TM_FOR_S(s) lq[s] = hf[s];
          ns.consider(lq, f, 0, 0);
        }
        continue;
      }
      int64_t v[SM], miss[SM];
      const int bl = lane < nb ? lane : 0;
      const int mbin = missing_bin >= 0 ? missing_bin : 0;
      TM_FOR_S(s) {          // unconditional loads, selected afterwards (issued together)
        v[s] = hf[bl * S + s];
        miss[s] = hf[mbin * S + s];
      }
      TM_FOR_S(s) {
        v[s] = lane < nb ? v[s] : 0;
        miss[s] = ns.allow_missing ? miss[s] : 0;
      }
      ns.scan_feature(v, miss, nb, f, lane);
    }
  }
  ns.wave_best();
  if (lane == 0) s_best[wave] = ns.best;
  __syncthreads();
  if (done == nullptr) {
    if (threadIdx.x == 0) {
      Best b = s_best[0];
      for (int w = 1; w < 4; ++w)
        if (better(s_best[w], b)) b = s_best[w];
      cand[(int64_t)j * cstride + fb] = b;
    }
    return;
  }
  // Fused reduction: the last of the node's fbmax blocks to finish reduces it -- one launch per level fewer.
  // Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, first row of the sc1 table): the candidate
  // goes out as agent-scope (sc1) stores by wave 0, which waits for them (vmcnt(0)) before its agent-scope
  // ticket add; the block whose add returns fbmax - 1 reads every candidate of the node with sc1 loads in
  // that same wave. No L2 write-back / L1 invalidate fences.
  // HARDWARE ASSUMPTION (not a HIP memory-model guarantee -- every access here is relaxed): on gfx950 an
  // sc1 store is written through to the coherence point before vmcnt reaches 0, an sc1 load is served from
  // it, and the reader's loads cannot be hoisted above the ticket add (they are issued after the wave-uniform
  // branch on its result, and the atomics are volatile to the compiler). The portable form -- release on
  // the ticket add, an agent-scope acquire fence in the winning block -- costs an L2 write-back per node on
  // this part (agent scope spans the 8 XCDs' L2s). TMOG_FUSED_REDUCE=0 selects the separate reduce launch;
  // tests/test_gpu_kernels.py checks the two paths give identical trees over many nodes and levels.
  if (wave == 0) {
    unsigned last = 0;
    if (lane == 0) {
      Best b = s_best[0];
      for (int w = 1; w < 4; ++w)
        if (better(s_best[w], b)) b = s_best[w];
      store_best_sc1(cand + (int64_t)j * cstride + fb, b);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // the sc1 stores have left before the ticket
      last = __hip_atomic_fetch_add(done + j, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             (unsigned)(fbmax - 1);
    }
    last = __shfl(last, 0, 64);
    if (last) {
      reduce_node(ra, j, lane, true);
      if (lane == 0) __hip_atomic_store(done + j, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Subtraction + split scan of a sibling pair in one pass (replaces hist_subtract_kernel + the two nodes'
// split_scan blocks). Block (q, fb) covers feature block fb of pair q exactly as split_scan_kernel does for
// one node: it loads the parent's and the built (small) child's rows, stores big = parent - small, and
// scans both children from registers -- the histograms the subtraction already streams are not read
// again by a separate scan. Node totals: small from its feature 0, big = parent's - small's. Writes
// cand[j_small][fb] and cand[j_big][fb]; the two nodes carry params slot 4 = 1 so split_scan_kernel skips
// them. Words outside the live set (one-present-bin columns above bin 0) are left alone, as before.
template <int SM>
__global__ void __launch_bounds__(256) pair_scan_kernel(
    int64_t* __restrict__ hist, const int64_t* __restrict__ parent, const int64_t* __restrict__ parent_off,
    const int32_t* __restrict__ small_j, const int32_t* __restrict__ big_j, int n_pairs,
    const int64_t* __restrict__ node_hist_off, const int32_t* __restrict__ node_nfeat,
    const int32_t* __restrict__ node_feat_off, const int32_t* __restrict__ feat_list,
    const int32_t* __restrict__ feat_nbins, int B, int S, int kind, const float* __restrict__ node_params,
    int missing_bin, const int32_t* __restrict__ node_model, const double* __restrict__ qinv, int fbmax,
    Best* __restrict__ cand, int n_multi, int fpb, int cstride, const int* __restrict__ dnp) {
  const int q = blockIdx.x / fbmax;
  const int fb = blockIdx.x - q * fbmax;
  if (dnp != nullptr) n_pairs = *dnp;          // device-planned level: pair count on the device
  if (q >= n_pairs) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int js = small_j[q], jb = big_j[q];
  const int nf = node_nfeat[js];           // no per-node feature subsets on this path: same list for both
  const int f_lim = n_multi >= 0 ? min(n_multi, nf) : nf;
  const int fb_multi = n_multi >= 0 ? (n_multi + fpb - 1) / fpb : fbmax;
  const bool one_blk = fb >= fb_multi;
  const int64_t* P = parent + parent_off[q];
  const int64_t* Hs = hist + node_hist_off[js];
  int64_t* Hb = hist + node_hist_off[jb];
  const int32_t* fl = feat_list + node_feat_off[js];
  const bool scan_s = node_params[(int64_t)js * 8 + 7] > 0.5f;
  const bool scan_b = node_params[(int64_t)jb * 8 + 7] > 0.5f;
  __shared__ Best s_best[2][4];
  NodeScan<SM> ns, nb_;
  {
    int64_t ts[SM], tp[SM], tb[SM];
    node_totals<SM>(Hs, B, S, lane, ts);
    node_totals<SM>(P, B, S, lane, tp);
    TM_FOR_S(s) tb[s] = tp[s] - ts[s];
    ns.init(ts, qinv + (int64_t)(node_model ? node_model[js] : 0) * S, node_params + (int64_t)js * 8, S, kind,
            missing_bin);
    nb_.init(tb, qinv + (int64_t)(node_model ? node_model[jb] : 0) * S, node_params + (int64_t)jb * 8, S, kind,
             missing_bin);
  }
  if (one_blk) {
    const int f = n_multi + (fb - fb_multi) * 256 + (int)threadIdx.x;
    if (f < nf) {
      const int64_t o = (int64_t)f * B * S;      // live words of a one-present-bin column: bin 0
      int64_t ls[SM], lb[SM];
      TM_FOR_S(s) {
        ls[s] = Hs[o + s];
        lb[s] = P[o + s] - ls[s];
        Hb[o + s] = lb[s];
      }
      if (feat_nbins[fl[f]] == 1) {
        if (scan_s && ns.allow_missing) ns.consider(ls, f, 0, 0);
        if (scan_b && nb_.allow_missing) nb_.consider(lb, f, 0, 0);
      }
    }
  } else {
    const int f_end = min(f_lim, (fb + 1) * fpb);
    for (int f = fb * fpb + wave; f < f_end; f += 4) {
      const int nbins = feat_nbins[fl[f]];
      const int64_t o = (int64_t)f * B * S;
      int64_t vs[SM], vb[SM], ms[SM], mb[SM], pa[SM], pp[SM];
      const int bl = lane < B ? lane : 0;           // every load unconditional (issued together)
      TM_FOR_S(s) {
        pa[s] = Hs[o + bl * S + s];
        pp[s] = P[o + bl * S + s];
      }
      TM_FOR_S(s) {
        const int64_t a = lane < B ? pa[s] : 0;
        const int64_t c = lane < B ? pp[s] - pa[s] : 0;
        if (lane < B) Hb[o + lane * S + s] = c;
        // missing bin statistics from the lane holding it
        ms[s] = missing_bin >= 0 ? readlane64(a, missing_bin) : 0;   // kernel argument: wave-uniform lane
        mb[s] = missing_bin >= 0 ? readlane64(c, missing_bin) : 0;
        vs[s] = lane < nbins ? a : 0;
        vb[s] = lane < nbins ? c : 0;
      }
      if (nbins == 1) {
        if (lane == 0) {
          if (scan_s && ns.allow_missing) ns.consider(vs, f, 0, 0);
          if (scan_b && nb_.allow_missing) nb_.consider(vb, f, 0, 0);
        }
        continue;
      }
      if (scan_s) {
        if (!ns.allow_missing)
          TM_FOR_S(s) ms[s] = 0;
        ns.scan_feature(vs, ms, nbins, f, lane);
      }
      if (scan_b) {
        if (!nb_.allow_missing)
          TM_FOR_S(s) mb[s] = 0;
        nb_.scan_feature(vb, mb, nbins, f, lane);
      }
    }
  }
  ns.wave_best();
  nb_.wave_best();
  if (lane == 0) {
    s_best[0][wave] = ns.best;
    s_best[1][wave] = nb_.best;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    Best b = s_best[threadIdx.x][0];
    for (int w = 1; w < 4; ++w)
      if (better(s_best[threadIdx.x][w], b)) b = s_best[threadIdx.x][w];
    cand[(int64_t)(threadIdx.x ? jb : js) * cstride + fb] = b;
  }
}

// Wide split scan (S > 16 classes or B > 64 bins): one workgroup per (node, local feature). The
// feature's B x S fixed-point histogram is copied into LDS and prefix-summed over bins per statistic
// (one thread per statistic), node totals come from local feature 0 as in the narrow kernel, then the
// threads stride over the (bin, missing direction) candidates and evaluate each with exactly the CPU
// twin's operation order (impurity sums over s in order), so both paths pick the same split.
__global__ void __launch_bounds__(256) split_scan_wide_kernel(
    const int64_t* __restrict__ hist, const int64_t* __restrict__ node_hist_off, const int32_t* __restrict__ node_nfeat,
    const int32_t* __restrict__ node_feat_off, const int32_t* __restrict__ feat_list,
    const int32_t* __restrict__ feat_nbins, int B, int S, int kind, const float* __restrict__ node_params,
    int missing_bin, const int32_t* __restrict__ node_model, const double* __restrict__ qinv, int fbmax,
    Best* __restrict__ cand, int n_multi, int cstride) {
  extern __shared__ __attribute__((aligned(16))) int64_t wl[];
  int64_t* H = wl;                       // [B][S] prefix sums
  int64_t* totq = H + (int64_t)B * S;    // [S]
  int64_t* miss = totq + S;              // [S]
  double* q = reinterpret_cast<double*>(miss + S);   // [S]
  __shared__ Best s_best[4];
  const int j = blockIdx.x / fbmax;
  const int f = blockIdx.x - j * fbmax;
  const int nf = node_nfeat[j];
  Best best{-INFINITY, 0x7fffffff, 0, 0};
  const bool live = f < nf && node_params[(int64_t)j * 8 + 7] > 0.5f;   // slot 7: node may split
  const int64_t* h = hist + node_hist_off[j];
  const int32_t* fl = feat_list + node_feat_off[j];
  const float* P = node_params + (int64_t)j * 8;
  const double* qi = qinv + (int64_t)(node_model ? node_model[j] : 0) * S;
  const double min_inst = P[0], min_gain = P[1], mcw = P[2], lambda = P[3];
  const bool allow_missing = P[5] > 0.5f && missing_bin >= 0;
  const int nb = live ? feat_nbins[fl[f]] : 0;
  const bool one = live && n_multi >= 0 && f >= n_multi;     // one-present-bin column: bin 0 only
  const int64_t* hf = h + (int64_t)f * B * S;
  if (live) {
    for (int i = threadIdx.x; i < B * S; i += blockDim.x) H[i] = (one && i >= S) ? 0 : hf[i];
    for (int s = threadIdx.x; s < S; s += blockDim.x) {
      int64_t t = 0;
      for (int bb = 0; bb < B; ++bb) t += h[(int64_t)bb * S + s];
      totq[s] = t;
      miss[s] = allow_missing ? hf[(int64_t)missing_bin * S + s] : 0;
      q[s] = qi[s];
    }
  }
  __syncthreads();
  if (live)
    for (int s = threadIdx.x; s < S; s += blockDim.x)
      for (int bb = 1; bb < B; ++bb) H[(int64_t)bb * S + s] += H[(int64_t)(bb - 1) * S + s];
  __syncthreads();
  if (live) {
    // parent impurity with the CPU twin's arithmetic
    double tcount = 0, pimp = 0, parent_gain = 0;
    if (kind == 0 || kind == 1) {
      for (int s = 0; s < S; ++s) tcount += (double)totq[s] * q[s];
      if (tcount > 0) {
        pimp = kind == 0 ? 1.0 : 0.0;
        for (int s = 0; s < S; ++s) {
          const double p = ((double)totq[s] * q[s]) / tcount;
          if (kind == 0) pimp -= p * p;
          else if (p > 0) pimp -= p * log2(p);
        }
      }
    } else {
      double tot[4] = {0, 0, 0, 0};
      for (int s = 0; s < S && s < 4; ++s) tot[s] = (double)totq[s] * q[s];
      pimp = impurity_dev(tot, S, kind, &tcount);
      parent_gain = kind == 3 ? tot[0] * tot[0] / (tot[1] + lambda) : 0.0;
    }
    const int nd = allow_missing ? 2 : 1;
    const int nbc = one ? 1 : nb - 1 + (allow_missing ? 1 : 0);   // candidate bins per direction
    for (int c = threadIdx.x; c < nbc * nd; c += blockDim.x) {
      const int dl = c / nbc, b = one ? 0 : c - dl * nbc;
      if (one && (dl || !allow_missing)) continue;
      if (!one && b == nb - 1 && dl) continue;
      const int64_t* lp = H + (int64_t)b * S;
      double gain;
      bool ok = true;
      if (kind == 0 || kind == 1) {
        double lc = 0, rc = 0;
        for (int s = 0; s < S; ++s) {
          const int64_t lq = lp[s] + (dl ? miss[s] : 0);
          lc += (double)lq * q[s];
          rc += (double)(totq[s] - lq) * q[s];
        }
        double li = 0, ri = 0;
        if (lc > 0) {
          li = kind == 0 ? 1.0 : 0.0;
          for (int s = 0; s < S; ++s) {
            const double p = ((double)(lp[s] + (dl ? miss[s] : 0)) * q[s]) / lc;
            if (kind == 0) li -= p * p;
            else if (p > 0) li -= p * log2(p);
          }
        }
        if (rc > 0) {
          ri = kind == 0 ? 1.0 : 0.0;
          for (int s = 0; s < S; ++s) {
            const double p = ((double)(totq[s] - lp[s] - (dl ? miss[s] : 0)) * q[s]) / rc;
            if (kind == 0) ri -= p * p;
            else if (p > 0) ri -= p * log2(p);
          }
        }
        if (lc < min_inst || rc < min_inst || lc <= 0 || rc <= 0) ok = false;
        gain = pimp - (lc / tcount) * li - (rc / tcount) * ri;
        if (gain < min_gain) ok = false;
      } else {
        double left[4] = {0, 0, 0, 0}, right[4] = {0, 0, 0, 0};
        for (int s = 0; s < S && s < 4; ++s) {
          const int64_t lq = lp[s] + (dl ? miss[s] : 0);
          left[s] = (double)lq * q[s];
          right[s] = (double)(totq[s] - lq) * q[s];
        }
        if (kind == 3) {
          if (left[1] < mcw || right[1] < mcw) ok = false;
          gain = left[0] * left[0] / (left[1] + lambda) + right[0] * right[0] / (right[1] + lambda) - parent_gain;
        } else {
          double lc, rc;
          const double li = impurity_dev(left, S, kind, &lc);
          const double ri = impurity_dev(right, S, kind, &rc);
          if (lc < min_inst || rc < min_inst || lc <= 0 || rc <= 0) ok = false;
          gain = pimp - (lc / tcount) * li - (rc / tcount) * ri;
          if (gain < min_gain) ok = false;
        }
      }
      if (ok) {
        const Best cb{gain, f, b, dl};
        if (better(cb, best)) best = cb;
      }
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int off = 32; off > 0; off >>= 1) {
    Best o;
    o.gain = __shfl_xor(best.gain, off, 64);
    o.f = __shfl_xor(best.f, off, 64);
    o.b = __shfl_xor(best.b, off, 64);
    o.dl = __shfl_xor(best.dl, off, 64);
    if (better(o, best)) best = o;
  }
  if (lane == 0) s_best[wave] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    Best bb = s_best[0];
    for (int w = 1; w < 4; ++w)
      if (better(s_best[w], bb)) bb = s_best[w];
    cand[(int64_t)j * cstride + f] = bb;
  }
}

__global__ void __launch_bounds__(64) split_reduce_kernel(ReduceArgs ra) { reduce_node(ra, blockIdx.x, threadIdx.x); }

// Feature-parallel merge: node j's decision is the best of the R ranks' records under the split scan's
// order (gain, then lowest full-list position, dl, bin) -- the candidate a single rank scanning every
// feature would pick. Host twin: common/tree_grow.hpp fp_merge_host.
// m_stride: records per rank in recv (the all-gather's count; >= m); dm (device-planned levels): the real node count
// is read from device memory, the grid covers the host bound m.
__global__ void fp_merge_kernel(const uint8_t* __restrict__ recv, int R, int m, int64_t rb, int S,
                                int32_t* __restrict__ out_feat, int32_t* __restrict__ out_bin,
                                float* __restrict__ out_gain, uint8_t* __restrict__ out_dl,
                                float* __restrict__ out_left, int64_t m_stride, const int* __restrict__ dm) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m || (dm != nullptr && j >= *dm)) return;
  int w = -1;
  Best best{-INFINITY, 0x7fffffff, 0, 0};
  for (int r = 0; r < R; ++r) {
    const uint8_t* p = recv + ((int64_t)r * m_stride + j) * rb;
    const int32_t* pi = reinterpret_cast<const int32_t*>(p);
    const Best c{*reinterpret_cast<const double*>(p), pi[2], pi[3], pi[4]};
    if (c.f == 0x7fffffff) continue;
    if (w < 0 || better(c, best)) {
      w = r;
      best = c;
    }
  }
  if (w < 0) {
    out_feat[j] = -1;
    out_bin[j] = -1;
    out_gain[j] = -INFINITY;
    out_dl[j] = 0;
    for (int s = 0; s < S; ++s) out_left[(int64_t)j * S + s] = 0.f;
    return;
  }
  const uint8_t* p = recv + ((int64_t)w * m_stride + j) * rb;
  out_feat[j] = reinterpret_cast<const int32_t*>(p)[5];
  out_bin[j] = best.b;
  out_gain[j] = (float)best.gain;
  out_dl[j] = (uint8_t)best.dl;
  for (int s = 0; s < S; ++s) out_left[(int64_t)j * S + s] = reinterpret_cast<const float*>(p + 24)[s];
}

// ----------------------------------------------------------------------------------- partition
struct PartItem {
  int32_t node;
  int32_t pad;
  int64_t begin;      // absolute position of the chunk in rows_in
  int64_t count;
  int64_t out_left;   // absolute output position for this chunk's first left row
  int64_t out_right;  // absolute output position for this chunk's first right row
};

constexpr int PART_U = 4;

__device__ __forceinline__ bool goes_left(uint8_t bin, int sb, bool dl, int missing_bin) {
  return (missing_bin >= 0 && bin == missing_bin) ? dl : ((int)bin <= sb);
}

// One-pass partition (replaces count + scatter): every chunk of every node reads its split decision
// straight from split_find's device output (no host round trip before the partition), and each
// 256-row step reserves its left / right output slots with two atomics on the node's cursors: left
// entries fill the node's own range [begin, begin + nl) upward, right entries fill it downward from
// the end. The order inside a child is not stable, which changes nothing downstream: histograms are
// exact integer sums (order-independent) and leaf assignments are keyed by row id. Nodes that do not
// split (feat < 0) are skipped; their ranges are collected as leaves from the input buffer.
__global__ void __launch_bounds__(256) partition_fused_kernel(
    const uint8_t* __restrict__ Xb, int F, const uint32_t* __restrict__ rows_in, uint32_t* __restrict__ rows_out,
    const PartItem* __restrict__ items, const int64_t* __restrict__ node_begin, const int64_t* __restrict__ node_count,
    const int32_t* __restrict__ split_feat, const int32_t* __restrict__ split_bin, const uint8_t* __restrict__ dl,
    const float* __restrict__ node_params, const float* __restrict__ split_gain, int missing_bin,
    unsigned long long* __restrict__ cursors, const uint8_t* __restrict__ XbT, int64_t Nt,
    const int2* __restrict__ gh_in, int2* __restrict__ gh_out, const int* __restrict__ dcount, int wide) {
  if (dcount != nullptr && (int)blockIdx.x >= *dcount) return;
  const PartItem it = items[blockIdx.x];
  const int j = it.node;
  const int f = split_feat[j], sb = split_bin[j];
  // the host's split decision, evaluated identically: splittable node, a split found, gain above eps
  if (f < 0 || !(node_params[(int64_t)j * 8 + 7] > 0.5f) || !(split_gain[j] > node_params[(int64_t)j * 8 + 6])) return;
  const bool d = dl[j] != 0;
  const int64_t nb = node_begin[j], nend = nb + node_count[j];
  // PART_U rows per thread per pass: their row / bin loads are all in flight together and one pair
  // of cursor atomics reserves the slots of 256 * PART_U rows (the dependent load -> load -> atomic
  // chain runs once per pass instead of once per 256 rows)
  __shared__ int s_cnt[PART_U][4];
  __shared__ unsigned long long s_base[2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned long long below = (1ull << lane) - 1ull;
  for (int64_t base = 0; base < it.count; base += (int64_t)blockDim.x * PART_U) {
    uint32_t e[PART_U];
    int2 q[PART_U];
    bool vd[PART_U], lf[PART_U];
#pragma unroll
    for (int u = 0; u < PART_U; ++u) {
      const int64_t i = base + (int64_t)u * blockDim.x + threadIdx.x;
      vd[u] = i < it.count;
      e[u] = rows_in[it.begin + (vd[u] ? i : 0)];     // unpredicated: row 0 of the item is valid
      if (gh_in) q[u] = gh_in[it.begin + (vd[u] ? i : 0)];   // the staged (g, h) move with their entry
    }
    uint8_t bn[PART_U];
#pragma unroll
    for (int u = 0; u < PART_U; ++u)
      bn[u] = XbT ? XbT[(int64_t)f * Nt + ent_row(e[u], wide)] : Xb[(int64_t)ent_row(e[u], wide) * F + f];
    int wpre[PART_U];
#pragma unroll
    for (int u = 0; u < PART_U; ++u) {
      lf[u] = vd[u] && goes_left(bn[u], sb, d, missing_bin);
      const unsigned long long m = __ballot(lf[u]);
      wpre[u] = __popcll(m & below);
      if (lane == 0) s_cnt[u][wave] = __popcll(m);
    }
    __syncthreads();
    int tot = 0, before[PART_U];
#pragma unroll
    for (int u = 0; u < PART_U; ++u) {
      int b = tot;
      for (int w = 0; w < 4; ++w) {
        if (w < wave) b += s_cnt[u][w];
        tot += s_cnt[u][w];
      }
      before[u] = b;
    }
    const int nvalid = (int)min((int64_t)blockDim.x * PART_U, it.count - base);
    if (threadIdx.x == 0) {
      s_base[0] = atomicAdd(cursors + 2 * j, (unsigned long long)tot);
      s_base[1] = atomicAdd(cursors + 2 * j + 1, (unsigned long long)(nvalid - tot));
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < PART_U; ++u) {
      if (!vd[u]) continue;
      const int lpos = before[u] + wpre[u];               // left rows before this one (row order)
      const int idx = u * (int)blockDim.x + (int)threadIdx.x;  // rows before this one
      // guarded: a slot outside the node's range (impossible unless the cursors were not reset) is
      // dropped; the host checks every node's left + right count against its size
      const int64_t pos = lf[u] ? nb + (int64_t)s_base[0] + lpos : nend - 1 - (int64_t)s_base[1] - (idx - lpos);
      if (pos >= nb && pos < nend) {
        rows_out[pos] = e[u];
        if (gh_in) gh_out[pos] = q[u];
      }
    }
    __syncthreads();
  }
}

// ----------------------------------------------------------------------------- leaf collection
// When a node stops splitting, its row entries (still contiguous in the level's row buffer) are
// copied out with the node id: after the last level every training entry sits in exactly one
// (entry, leaf) pair, so boosting updates its margins by a gather instead of re-walking the tree.
struct LeafItem {
  int64_t begin;    // first entry in rows
  int64_t count;
  int64_t out;      // output position
  int32_t gid;      // node id
  int32_t buf;      // row buffer: 0 = rows, 1 = rows_alt (device-planned levels collect from both)
};

__global__ void __launch_bounds__(256) leaf_collect_kernel(const uint32_t* __restrict__ rows,
                                                           const uint32_t* __restrict__ rows_alt,
                                                           const LeafItem* __restrict__ items,
                                                           uint32_t* __restrict__ out_rows,
                                                           int32_t* __restrict__ out_gid,
                                                           const int* __restrict__ dcount) {
  if (dcount != nullptr && (int)blockIdx.x >= *dcount) return;
  const LeafItem it = items[blockIdx.x];
  const uint32_t* src = (it.buf && rows_alt) ? rows_alt : rows;
  for (int64_t i = threadIdx.x; i < it.count; i += blockDim.x) {
    out_rows[it.out + i] = src[it.begin + i];
    out_gid[it.out + i] = it.gid;
  }
}

// ------------------------------------------------------------------------------------- predict
// LDS-row variant (F <= 512): the workgroup first copies its 128 rows' bins (row-major, F bytes each)
// into LDS with coalesced byte loads, then four lanes per row each walk a quarter of the model's
// trees (chunks of eight interleaved) reading bins from LDS, and the four partial sums are folded in a
// fixed order. 512-thread workgroups keep 16 waves per CU busy on the dependent node-fetch chains
// (128-thread groups left 4 waves per CU with the 64 KB of staged rows). Without it each tree step paid a dependent L2/Infinity-cache round trip for
// a single byte (64 lanes = 64 different rows = 64 cache lines per step); now only the node fetch
// (shared by the wave near the root, L2/L1 resident) stays global. grid.y = model.
constexpr int PRED_ROWS = 128;
constexpr int PRED_TU = 8;
constexpr int PRED_TPR = 4;   // threads per row (tree slices), 512-thread workgroups sharing the staged rows

__global__ void __launch_bounds__(PRED_ROWS * PRED_TPR) forest_predict_lds_kernel(
    const uint8_t* __restrict__ Xb, int F, const int64_t* __restrict__ model_row_off,
    const int32_t* __restrict__ row_list, const int64_t* __restrict__ model_tree_off,
    const int64_t* __restrict__ tree_off, const float* __restrict__ tree_weight, const int4* __restrict__ nodes,
    const uint8_t* __restrict__ default_left, int missing_bin, const float* __restrict__ leaf_value, int K,
    float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t srows[];
  const int m = blockIdx.y;
  const int64_t r0 = model_row_off[m], r1 = model_row_off[m + 1];
  const int64_t blk0 = r0 + (int64_t)blockIdx.x * PRED_ROWS;
  if (blk0 >= r1) return;                                   // whole workgroup out of range (uniform)
  const int nrow = (int)min((int64_t)PRED_ROWS, r1 - blk0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
  for (int r = wave; r < nrow; r += nwaves) {
    const int64_t row = row_list ? row_list[blk0 + r] : (blk0 + r - r0);
    const uint8_t* src = Xb + row * F;
    for (int b = lane; b < F; b += 64) srows[r * F + b] = src[b];
  }
  __syncthreads();
  // thread (rr, q): row rr of the block, tree chunks q, q + PRED_TPR, ... of PRED_TU trees each
  const int rr = threadIdx.x % PRED_ROWS, q = threadIdx.x / PRED_ROWS;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (rr < nrow) {
    const uint8_t* xr = srows + rr * F;
    const int64_t t_end = model_tree_off[m + 1];
    for (int64_t t = model_tree_off[m] + (int64_t)q * PRED_TU; t < t_end; t += (int64_t)PRED_TU * PRED_TPR) {
      const int nu = (int)min((int64_t)PRED_TU, t_end - t);
      int64_t k[PRED_TU];
      int4 nd[PRED_TU];
#pragma unroll
      for (int u = 0; u < PRED_TU; ++u) {
        k[u] = u < nu ? tree_off[t + u] : tree_off[t];
        nd[u] = nodes[k[u]];
      }
      bool active = true;
      while (active) {
        active = false;
#pragma unroll
        for (int u = 0; u < PRED_TU; ++u) {
          if (nd[u].z >= 0) {
            const uint8_t b = xr[nd[u].x];
            const bool gl = (missing_bin >= 0 && b == missing_bin) ? (default_left[k[u]] != 0) : ((int)b <= nd[u].y);
            k[u] = gl ? nd[u].z : nd[u].w;
            nd[u] = nodes[k[u]];
            active = true;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < PRED_TU; ++u) {
        if (u < nu) {
          const float w = tree_weight[t + u];
          for (int c = 0; c < K && c < 8; ++c) acc[c] += w * leaf_value[k[u] * K + c];
        }
      }
    }
  }
  // fold the PRED_TPR partial sums in q order (deterministic)
  float* red = reinterpret_cast<float*>(srows + ((PRED_ROWS * F + 15) & ~15));
  for (int c = 0; c < 8; ++c) red[(q * PRED_ROWS + rr) * 8 + c] = acc[c];
  __syncthreads();
  if (q == 0 && rr < nrow) {
    float* o = out + (blk0 + rr) * K;
    for (int c = 0; c < K && c < 8; ++c) {
      float v = red[rr * 8 + c];
      for (int qq = 1; qq < PRED_TPR; ++qq) v += red[(qq * PRED_ROWS + rr) * 8 + c];
      o[c] = v;
    }
  }
}

// Shared-forest prediction for pruned variants (models/trees.py: RF grid points that differ only in
// maxDepth / minInfoGain share one grown forest, tree_engine.prune_forest). Model m walks the grown
// trees once per (row, tree) and serves all of its variants v in [var_off[m], var_off[m+1]) on the way
// down: variant v stops at the first node that is a leaf of the grown tree, lies at depth >= var_depth[v]
// or has a split gain < the variant's min gain (exactly prune_forest's rule; the leaf / gain part comes
// precomputed as a per-node variant bitmask) and adds that node's value. One walk
// instead of one per variant (~5x fewer node visits for the default RF grid). Rows staged in LDS as in
// forest_predict_lds_kernel; 4 trees interleaved per thread; out[var_out_off[v] + (row - r0) * K + c].
constexpr int PM_ROWS = 64;
constexpr int PM_TPR = 4;
constexpr int PM_TU = 4;
constexpr int PM_VK = 32;      // variants x classes accumulated per thread

template <int KT>     // classes (compile-time: the per-thread accumulators stay in registers)
__global__ void __launch_bounds__(PM_ROWS * PM_TPR) forest_predict_multi_kernel(
    const uint8_t* __restrict__ Xb, int F, const int64_t* __restrict__ model_row_off,
    const int32_t* __restrict__ row_list, const int64_t* __restrict__ model_tree_off,
    const int64_t* __restrict__ tree_off, const float* __restrict__ tree_weight, const int4* __restrict__ nodes,
    const uint8_t* __restrict__ default_left, int missing_bin, const float* __restrict__ leaf_value, int K,
    const uint32_t* __restrict__ node_mask, const int32_t* __restrict__ var_off, const int32_t* __restrict__ var_depth,
    const int64_t* __restrict__ var_out_off, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t srows[];
  const int m = blockIdx.y;
  const int64_t r0 = model_row_off[m], r1 = model_row_off[m + 1];
  const int64_t blk0 = r0 + (int64_t)blockIdx.x * PM_ROWS;
  if (blk0 >= r1) return;
  const int nrow = (int)min((int64_t)PM_ROWS, r1 - blk0);
  const int v0 = var_off[m], V = var_off[m + 1] - v0;        // host guarantees V * K <= PM_VK
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
  for (int r = wave; r < nrow; r += nwaves) {
    const int64_t row = row_list ? row_list[blk0 + r] : (blk0 + r - r0);
    const uint8_t* src = Xb + row * F;
    for (int b = lane; b < F; b += 64) srows[r * F + b] = src[b];
  }
  __syncthreads();
  // per-thread accumulators live in the LDS reduction area (dynamic variant index, no register arrays)
  // depth stop masks: s_dmask[d] = variants whose max depth is <= d (the gain / grown-leaf part of the
  // rule is precomputed per node by the host: node_mask[k] = variants that stop at node k regardless of depth)
  __shared__ uint32_t s_dmask[33];
  if (threadIdx.x < 33) {
    uint32_t mk = 0u;
    for (int v = 0; v < V; ++v) mk |= (var_depth[v0 + v] <= (int)threadIdx.x ? 1u : 0u) << v;
    s_dmask[threadIdx.x] = mk;
  }
  const int rr = threadIdx.x % PM_ROWS, q = threadIdx.x / PM_ROWS;
  float* red = reinterpret_cast<float*>(srows + ((PM_ROWS * F + 15) & ~15));
  float* acc = red + (q * PM_ROWS + rr) * PM_VK;
  for (int i = 0; i < PM_VK; ++i) acc[i] = 0.f;
  __syncthreads();
  if (rr < nrow) {
    const uint8_t* xr = srows + rr * F;
    const int64_t t_end = model_tree_off[m + 1];
    const uint32_t all = V >= 32 ? 0xFFFFFFFFu : (1u << V) - 1u;     // V == 32: a 32-bit shift by 32 is undefined
    for (int64_t t = model_tree_off[m] + (int64_t)q * PM_TU; t < t_end; t += (int64_t)PM_TU * PM_TPR) {
      const int nu = (int)min((int64_t)PM_TU, t_end - t);
      int64_t k[PM_TU];
      int4 nd[PM_TU];
      uint32_t live[PM_TU];
      int dep[PM_TU];
#pragma unroll
      for (int u = 0; u < PM_TU; ++u) {
        k[u] = u < nu ? tree_off[t + u] : tree_off[t];
        nd[u] = nodes[k[u]];
        live[u] = u < nu ? all : 0u;
        dep[u] = 0;
      }
      bool active = true;
      while (active) {
        active = false;
#pragma unroll
        for (int u = 0; u < PM_TU; ++u) {
          if (live[u] != 0u) {
            const uint32_t stop = (node_mask[k[u]] | s_dmask[min(dep[u], 32)]) & live[u];
            if (stop) {
              const float w = tree_weight[t + u];
              for (int c = 0; c < KT; ++c) {
                const float val = w * leaf_value[k[u] * KT + c];
                for (uint32_t sm = stop; sm; sm &= sm - 1u) acc[(__ffs(sm) - 1) * KT + c] += val;
              }
              live[u] &= ~stop;
            }
            if (live[u] != 0u) {
              const uint8_t b = xr[nd[u].x];
              const bool gl = (missing_bin >= 0 && b == missing_bin) ? (default_left[k[u]] != 0) : ((int)b <= nd[u].y);
              k[u] = gl ? nd[u].z : nd[u].w;
              nd[u] = nodes[k[u]];
              dep[u] += 1;
              active = true;
            }
          }
        }
      }
    }
  }
  __syncthreads();
  if (q == 0 && rr < nrow) {
    for (int v = 0; v < V; ++v) {
      float* o = out + var_out_off[v0 + v] + (blk0 + rr - r0) * KT;
      for (int c = 0; c < KT; ++c) {
        float x = red[rr * PM_VK + v * KT + c];
        for (int qq = 1; qq < PM_TPR; ++qq) x += red[(qq * PM_ROWS + rr) * PM_VK + v * KT + c];
        o[c] = x;
      }
    }
  }
}

// grid.y = model; each thread walks every tree of its model for one of the model's rows.
__global__ void __launch_bounds__(256) forest_predict_kernel(
    const uint8_t* __restrict__ Xb, int F, const int64_t* __restrict__ model_row_off,
    const int32_t* __restrict__ row_list, const int64_t* __restrict__ model_tree_off,
    const int64_t* __restrict__ tree_off, const float* __restrict__ tree_weight, const int4* __restrict__ nodes,
    const uint8_t* __restrict__ default_left, int missing_bin, const float* __restrict__ leaf_value, int K,
    float* __restrict__ out) {
  const int m = blockIdx.y;
  const int64_t r0 = model_row_off[m], r1 = model_row_off[m + 1];
  const int64_t i = r0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= r1) return;
  const int64_t row = row_list ? row_list[i] : (i - r0);
  const uint8_t* xr = Xb + row * F;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int64_t t_end = model_tree_off[m + 1];
  int64_t t = model_tree_off[m];
  // four trees walked together: four independent node-fetch -> bin-fetch chains in flight per lane
  for (; t + 4 <= t_end; t += 4) {
    int64_t k[4];
    int4 nd[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      k[u] = tree_off[t + u];
      nd[u] = nodes[k[u]];
    }
    bool active = true;
    while (active) {
      active = false;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (nd[u].z >= 0) {
          const uint8_t b = xr[nd[u].x];
          const bool gl = (missing_bin >= 0 && b == missing_bin) ? (default_left[k[u]] != 0) : ((int)b <= nd[u].y);
          k[u] = gl ? nd[u].z : nd[u].w;
          nd[u] = nodes[k[u]];
          active = true;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float w = tree_weight[t + u];
      for (int c = 0; c < K && c < 8; ++c) acc[c] += w * leaf_value[k[u] * K + c];
    }
  }
  for (; t < t_end; ++t) {
    int64_t k = tree_off[t];
    int4 nd = nodes[k];  // (feat, bin, left, right)
    while (nd.z >= 0) {
      const uint8_t b = xr[nd.x];
      const bool gl = (missing_bin >= 0 && b == missing_bin) ? (default_left[k] != 0) : ((int)b <= nd.y);
      k = gl ? nd.z : nd.w;
      nd = nodes[k];
    }
    const float w = tree_weight[t];
    for (int c = 0; c < K && c < 8; ++c) acc[c] += w * leaf_value[k * K + c];
  }
  float* o = out + i * K;
  for (int c = 0; c < K && c < 8; ++c) o[c] = acc[c];
}

}  // namespace

// ------------------------------------------------------------------------------------- C ABI
extern "C" {

int tmog_hip_debug_flags(int flags) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_hist_debug), &flags, sizeof(int));
}

int tmog_hip_hist_build(const uint8_t* Xb, int F, const uint32_t* rows, const void* items, int n_items,
                        const int32_t* node_feat_off, const int32_t* feat_list, const int32_t* node_model,
                        const int64_t* node_hist_off, int64_t* hist, int B, int mode, int S, const float* y,
                        const float* t1, const float* t2, int64_t stride, const float* qscale, int skip_bin,
                        const int64_t* csr_ptr, const uint16_t* csr_col, int Sc, int n_wide, int need_general,
                        hipStream_t stream, const int32_t* gh_words, const int* dcount, int wide_rows,
                        const uint8_t* Xh, int Fh) {
  if (n_items == 0) return 0;
  if (Xh == nullptr) {
    Xh = Xb;
    Fh = F;
  }
  if (dcount != nullptr && n_wide != 0) return -2;   // device-counted launches: one mixed launch
  const int2* gh = reinterpret_cast<const int2*>(gh_words);
  if (gh && mode != 2) return -2;
  if (Sc <= 0 || Sc > S) Sc = S;
  size_t lds = (size_t)(((64 * (B * Sc + 1)) + 3) & ~3) * sizeof(int) + 4 * 64 * sizeof(int4) +
               TM_MAX_S * sizeof(int);
  if (mode == 2 && S == 2) {   // wide-load items: 64 features x (B + 1) packed int64 words + stage + totals
    const size_t wl = (size_t)((2 * (64 * (B + 1) + 17) + 3) & ~3) * sizeof(int) + 4 * 64 * sizeof(int4) +
                      4 * sizeof(int);
    if (wl > lds) lds = wl;
  }
  if (lds > 160 * 1024) return -2;
  if (skip_bin >= B || (mode == 2 && skip_bin >= 0 && (S != 2 || Sc != S))) return -2;
  if (mode == 0 && S > TM_WIDE_MAX_S) return -2;
  if ((csr_ptr != nullptr) != (csr_col != nullptr) || (csr_ptr && (mode != 2 || skip_bin <= 0))) return -2;
  const HistItem* it = (const HistItem*)items;
  if (n_wide < 0 || n_wide > n_items || (n_wide > 0 && (mode != 2 || S != 2))) return -2;
  // The grower lists the wide-load items first. By default they share the launch with the other items
  // (the mixed kernel runs them concurrently with the CSR items); TMOG_HIST_WIDE_SPLIT=1 launches them
  // as hist_wide_kernel -- measured slower on the headline (1086 vs 974 ms per step: the two launches
  // serialise and each has its own tail), kept for experiments.
  static const bool split_wide = [] { const char* e = std::getenv("TMOG_HIST_WIDE_SPLIT"); return e && e[0] == '1'; }();
  if (!split_wide) n_wide = 0;
  if (n_wide > 0) {
    static const int occ = [] { const char* e = std::getenv("TMOG_HIST_WIDE_OCC"); return e ? std::atoi(e) : 6; }();
    if (occ >= 7)
      hipLaunchKernelGGL(hist_wide_kernel<7>, dim3(n_wide), dim3(256), lds, stream, Xb, F, rows, it, node_feat_off,
                         feat_list, node_model, node_hist_off, hist, B, t1, t2, stride, qscale, skip_bin, gh, wide_rows, Xh, Fh);
    else
      hipLaunchKernelGGL(hist_wide_kernel<6>, dim3(n_wide), dim3(256), lds, stream, Xb, F, rows, it, node_feat_off,
                         feat_list, node_model, node_hist_off, hist, B, t1, t2, stride, qscale, skip_bin, gh, wide_rows, Xh, Fh);
    it += n_wide;
    n_items -= n_wide;
    if (n_items == 0) return (int)hipGetLastError();
  }
  dim3 grid(n_items), block(256);
  if (mode == 0)
    hipLaunchKernelGGL(hist_build_kernel<0>, grid, block, lds, stream, Xb, F, rows, it, node_feat_off, feat_list,
                       node_model, node_hist_off, hist, B, S, y, t1, t2, stride, qscale, -1, nullptr, nullptr, Sc,
                       nullptr, dcount, wide_rows, Xh, Fh);
  else if (mode == 1)
    hipLaunchKernelGGL(hist_build_kernel<1>, grid, block, lds, stream, Xb, F, rows, it, node_feat_off, feat_list,
                       node_model, node_hist_off, hist, B, S, y, t1, t2, stride, qscale, -1, nullptr, nullptr, Sc,
                       nullptr, dcount, wide_rows, Xh, Fh);
  else if (need_general)
    hipLaunchKernelGGL(hist_build_kernel<2>, grid, block, lds, stream, Xb, F, rows, it, node_feat_off, feat_list,
                       node_model, node_hist_off, hist, B, S, y, t1, t2, stride, qscale, skip_bin, csr_ptr,
                       csr_col, Sc, gh, dcount, wide_rows, Xh, Fh);
  else
    hipLaunchKernelGGL((hist_build_kernel<2, false>), grid, block, lds, stream, Xb, F, rows, it, node_feat_off,
                       feat_list, node_model, node_hist_off, hist, B, S, y, t1, t2, stride, qscale, skip_bin, csr_ptr,
                       csr_col, Sc, gh, dcount, wide_rows, Xh, Fh);
  return (int)hipGetLastError();
}

// live words of the largest node: the grids of the subtract / zero kernels are sized to what they touch
// (sized from the full B x S words they launched ~4x the workgroups the live region needs)
static int64_t host_live_words(int64_t sz, int64_t dense, int per, int S) {
  return (dense < 0 || sz <= dense) ? sz : dense + (sz - dense) / per * S;
}

int tmog_hip_hist_subtract(int64_t* hist, const int64_t* parent, const int64_t* parent_off, const int64_t* small_off,
                           const int64_t* out_off, const int64_t* size, int n, int64_t max_size, int64_t dense,
                           int per, int S, hipStream_t stream) {
  if (n == 0) return 0;
  if (max_size >= (int64_t)1 << 31) return -2;
  int gx = (int)min((host_live_words(max_size, dense, per, S) + 255) / 256, (int64_t)1024);
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL(hist_subtract_kernel, dim3(gx, n), dim3(256), 0, stream, hist, parent, parent_off, small_off,
                     out_off, size, n, dense, per, S);
  return (int)hipGetLastError();
}

int tmog_hip_split_find(const int64_t* hist, int n_nodes, const int64_t* node_hist_off, const int32_t* node_nfeat,
                        const int32_t* node_feat_off, const int32_t* feat_list, const int32_t* feat_nbins, int B,
                        int S, int kind, const float* node_params, int missing_bin, const int32_t* node_model,
                        const double* qinv, int max_nfeat, void* cand_ws, int32_t* out_feat, int32_t* out_bin,
                        float* out_gain, uint8_t* out_dl, float* out_left, float* out_total, int64_t* cursors,
                        int n_multi, void* rec, int64_t rec_bytes, int fp_mlo, int fp_nml, int fp_obase,
                        hipStream_t stream, unsigned* done, const int* dm) {
  if (n_nodes == 0) return 0;
  // device-counted launches take the narrow scan with the fused reduction (no separate per-node launch)
  if (dm != nullptr && (done == nullptr || S > TM_MAX_S || B > 64)) return -2;
  if (n_multi > max_nfeat) n_multi = -1;
  Best* cand = (Best*)cand_ws;   // >= tmog_hip_split_cand_bytes(n_nodes, max_nfeat, B, S) bytes
  const bool wide = S > TM_MAX_S || B > 64;
  int fbmax;
  // done (n_nodes zeroed counters, left zeroed): the node reduction runs inside the narrow scan's last block
  auto make_ra = [&](int fbm) {
    return ReduceArgs{hist, node_hist_off, node_feat_off, feat_list, B, S, missing_bin, node_model, qinv, fbm,
                      cand_stride(fbm), cand,
                      out_feat, out_bin, out_gain, out_dl, out_left, out_total, (unsigned long long*)cursors,
                      (uint8_t*)rec, rec_bytes, fp_mlo, fp_nml, fp_obase};
  };
  ReduceArgs ra{};
  if (wide) {
    if (S > TM_WIDE_MAX_S || B * S > TM_WIDE_MAX_BS) return -2;
    fbmax = max_nfeat;        // one workgroup per (node, feature)
    const size_t lds = ((size_t)B * S + 3 * (size_t)S) * 8;
    hipLaunchKernelGGL(split_scan_wide_kernel, dim3(n_nodes * fbmax), dim3(256), lds, stream, hist, node_hist_off,
                       node_nfeat, node_feat_off, feat_list, feat_nbins, B, S, kind, node_params, missing_bin,
                       node_model, qinv, fbmax, cand, n_multi, cand_stride(fbmax));
  } else {
  const int fpb = split_fpb();
  fbmax = n_multi >= 0 ? (n_multi + fpb - 1) / fpb + (max_nfeat - n_multi + 255) / 256
                       : (max_nfeat + fpb - 1) / fpb;
  ra = make_ra(fbmax);
#define TM_SPLIT(SMV)                                                                                          \
  hipLaunchKernelGGL(split_scan_kernel<SMV>, dim3(n_nodes * fbmax), dim3(256), 0, stream, hist, node_hist_off,  \
                     node_nfeat, node_feat_off, feat_list, feat_nbins, B, S, kind, node_params, missing_bin,    \
                     node_model, qinv, fbmax, cand, n_multi, fpb, done, ra, dm)
  if (S <= 2) TM_SPLIT(2);
  else if (S == 3) TM_SPLIT(3);
  else if (S <= 4) TM_SPLIT(4);
  else TM_SPLIT(TM_MAX_S);
#undef TM_SPLIT
  }
  if (wide) ra = make_ra(fbmax);
  if (wide || done == nullptr)
    hipLaunchKernelGGL(split_reduce_kernel, dim3(n_nodes), dim3(64), 0, stream, ra);
  return (int)hipGetLastError();
}

// Fused subtraction + split scan of sibling pairs (pair_scan_kernel); the same candidate layout as
// tmog_hip_split_find, whose scan then skips the pairs' nodes (params slot 4). Narrow path only.
int tmog_hip_pair_scan(int64_t* hist, const int64_t* parent, const int64_t* parent_off, const int32_t* small_j,
                       const int32_t* big_j, int n_pairs, const int64_t* node_hist_off, const int32_t* node_nfeat,
                       const int32_t* node_feat_off, const int32_t* feat_list, const int32_t* feat_nbins, int B, int S,
                       int kind, const float* node_params, int missing_bin, const int32_t* node_model,
                       const double* qinv, int max_nfeat, void* cand_ws, int n_multi, hipStream_t stream,
                       const int* dnp) {
  if (n_pairs == 0) return 0;
  if (S > TM_MAX_S || B > 64) return -2;
  if (n_multi > max_nfeat) n_multi = -1;
  const int fpb = split_fpb();
  const int fbmax = n_multi >= 0 ? (n_multi + fpb - 1) / fpb + (max_nfeat - n_multi + 255) / 256
                                 : (max_nfeat + fpb - 1) / fpb;
#define TM_PAIR(SMV)                                                                                           \
  hipLaunchKernelGGL(pair_scan_kernel<SMV>, dim3(n_pairs * fbmax), dim3(256), 0, stream, hist, parent, parent_off, \
                     small_j, big_j, n_pairs, node_hist_off, node_nfeat, node_feat_off, feat_list, feat_nbins, B, S, \
                     kind, node_params, missing_bin, node_model, qinv, fbmax, (Best*)cand_ws, n_multi, fpb,    \
                     cand_stride(fbmax), dnp)
  if (S <= 2) TM_PAIR(2);
  else if (S == 3) TM_PAIR(3);
  else if (S <= 4) TM_PAIR(4);
  else TM_PAIR(TM_MAX_S);
#undef TM_PAIR
  return (int)hipGetLastError();
}

int tmog_hip_fp_merge(const void* recv, int R, int m, int64_t rec_bytes, int S, int32_t* out_feat, int32_t* out_bin,
                      float* out_gain, uint8_t* out_dl, float* out_left, hipStream_t stream) {
  if (m == 0) return 0;
  hipLaunchKernelGGL(fp_merge_kernel, dim3((m + 255) / 256), dim3(256), 0, stream, (const uint8_t*)recv, R, m,
                     rec_bytes, S, out_feat, out_bin, out_gain, out_dl, out_left, (int64_t)m, (const int*)nullptr);
  return (int)hipGetLastError();
}

// Device-planned levels: recv holds m_stride records per rank (the level's host bound), the merged nodes are the
// first *dm of them.
int tmog_hip_fp_merge_dev(const void* recv, int R, int m_stride, int64_t rec_bytes, int S, int32_t* out_feat,
                          int32_t* out_bin, float* out_gain, uint8_t* out_dl, float* out_left, const int* dm,
                          hipStream_t stream) {
  if (m_stride == 0) return 0;
  hipLaunchKernelGGL(fp_merge_kernel, dim3((m_stride + 255) / 256), dim3(256), 0, stream, (const uint8_t*)recv, R,
                     m_stride, rec_bytes, S, out_feat, out_bin, out_gain, out_dl, out_left, (int64_t)m_stride, dm);
  return (int)hipGetLastError();
}

int tmog_hip_zero_segments(int64_t* hist, const int64_t* off, const int64_t* size, int n, int64_t max_size,
                           int64_t dense, int per, int S, hipStream_t stream, int n_dense, const int* dn) {
  if (n == 0) return 0;
  if (max_size >= (int64_t)1 << 31) return -2;
  const int64_t lw = std::max(host_live_words(max_size, dense, per, S), host_live_words(max_size, 0, per, S));
  int gx = (int)min((lw + 255) / 256, (int64_t)1024);
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL(zero_segments_kernel, dim3(gx, n), dim3(256), 0, stream, hist, off, size, n, dense, per, S,
                     n_dense, dn);
  return (int)hipGetLastError();
}

// Loads this file's code object on the current device from the calling thread. The HIP runtime loads a
// translation unit's kernels at the first launch of any of them; the tree grower's first launches come from
// its concurrent job-group threads, and that first load racing on two threads crashed inside the runtime
// under the profiler (rocprofv3 --kernel-trace, XGBoost-only run). The grower calls this before it spawns them.
int tmog_hip_tree_prime() {
  hipFuncAttributes at;
  return (int)hipFuncGetAttributes(&at, reinterpret_cast<const void*>(&zero_segments_kernel));
}

size_t tmog_hip_split_cand_bytes(int n_nodes, int max_nfeat, int B, int S) {
  const bool wide = S > TM_MAX_S || B > 64;
  const int fpb = split_fpb();       // (max_nfeat + fpb - 1) / fpb + 1 bounds fbmax for any n_multi split
  return (size_t)n_nodes * cand_stride(wide ? max_nfeat : (max_nfeat + fpb - 1) / fpb + 1) * sizeof(Best);
}

// Largest statistic chunk whose per-workgroup LDS table (64 copies of B x Sc words) fits the LDS.
int tmog_hip_hist_stat_chunk(int B, int S) {
  int sc = S;
  while (sc > 1 && (size_t)(((64 * (B * sc + 1)) + 3) & ~3) * sizeof(int) + 4 * 64 * sizeof(int4) +
                       TM_MAX_S * sizeof(int) > 160 * 1024)
    --sc;
  return sc;
}

int tmog_hip_partition_fused(const uint8_t* Xb, int F, const uint32_t* rows_in, uint32_t* rows_out, const void* items,
                             int n_items, const int64_t* node_begin, const int64_t* node_count, const int32_t* split_feat,
                             const int32_t* split_bin, const uint8_t* dl, const float* node_params,
                             const float* split_gain, int missing_bin, int64_t* cursors, const uint8_t* XbT,
                             int64_t N, hipStream_t stream, const int32_t* gh_in, int32_t* gh_out, const int* dcount,
                             int wide_rows) {
  if (n_items == 0) return 0;
  if ((gh_in != nullptr) != (gh_out != nullptr)) return -2;
  hipLaunchKernelGGL(partition_fused_kernel, dim3(n_items), dim3(256), 0, stream, Xb, F, rows_in, rows_out,
                     (const PartItem*)items, node_begin, node_count, split_feat, split_bin, dl, node_params,
                     split_gain, missing_bin, (unsigned long long*)cursors, XbT, N,
                     reinterpret_cast<const int2*>(gh_in), reinterpret_cast<int2*>(gh_out), dcount, wide_rows);
  return (int)hipGetLastError();
}

int tmog_hip_leaf_collect(const uint32_t* rows, const void* items, int n_items, uint32_t* out_rows,
                          int32_t* out_gid, hipStream_t stream, const uint32_t* rows_alt, const int* dcount) {
  if (n_items == 0) return 0;
  hipLaunchKernelGGL(leaf_collect_kernel, dim3(n_items), dim3(256), 0, stream, rows, rows_alt, (const LeafItem*)items,
                     out_rows, out_gid, dcount);
  return (int)hipGetLastError();
}

// Shared-forest multi-variant prediction (forest_predict_multi_kernel). Every model's V x K <= 32 (V <= 32).
int tmog_hip_forest_predict_multi(const uint8_t* Xb, int F, int n_models, const int64_t* model_row_off,
                                  const int32_t* row_list, int64_t max_rows, const int64_t* model_tree_off,
                                  const int64_t* tree_off, const float* tree_weight, const int32_t* nodes,
                                  const uint8_t* default_left, int missing_bin, const float* leaf_value, int K,
                                  const uint32_t* node_mask, const int32_t* var_off, const int32_t* var_depth,
                                  const int64_t* var_out_off, float* out, hipStream_t stream) {
  if (n_models == 0 || max_rows == 0) return 0;
  if (K != 1 && K != 2 && K != 4 && K != 8) return -2;
  const size_t lds = (((size_t)PM_ROWS * F + 15) & ~(size_t)15) + sizeof(float) * PM_VK * PM_ROWS * PM_TPR;
  if (lds > 160 * 1024) return -3;
  dim3 g2((unsigned)((max_rows + PM_ROWS - 1) / PM_ROWS), n_models);
#define TM_PM(KV)                                                                                               \
  hipLaunchKernelGGL(forest_predict_multi_kernel<KV>, g2, dim3(PM_ROWS * PM_TPR), lds, stream, Xb, F,           \
                     model_row_off, row_list, model_tree_off, tree_off, tree_weight, (const int4*)nodes,         \
                     default_left, missing_bin, leaf_value, K, node_mask, var_off, var_depth, var_out_off,      \
                     out)
  if (K == 1) TM_PM(1);
  else if (K == 2) TM_PM(2);
  else if (K == 4) TM_PM(4);
  else TM_PM(8);
#undef TM_PM
  return (int)hipGetLastError();
}

int tmog_hip_forest_predict(const uint8_t* Xb, int F, int n_models, const int64_t* model_row_off,
                            const int32_t* row_list, int64_t max_rows, const int64_t* model_tree_off,
                            const int64_t* tree_off, const float* tree_weight, const int32_t* nodes,
                            const uint8_t* default_left, int missing_bin, const float* leaf_value, int K, float* out,
                            hipStream_t stream) {
  if (n_models == 0 || max_rows == 0) return 0;
  if (K > 8) return -2;
  if ((size_t)PRED_ROWS * F <= 64 * 1024) {
    dim3 g2((unsigned)((max_rows + PRED_ROWS - 1) / PRED_ROWS), n_models);
    const size_t lds = (((size_t)PRED_ROWS * F + 15) & ~(size_t)15) + sizeof(float) * 8 * PRED_ROWS * PRED_TPR;
    hipLaunchKernelGGL(forest_predict_lds_kernel, g2, dim3(PRED_ROWS * PRED_TPR), lds, stream, Xb, F,
                       model_row_off, row_list, model_tree_off, tree_off, tree_weight, (const int4*)nodes,
                       default_left, missing_bin, leaf_value, K, out);
    return (int)hipGetLastError();
  }
  dim3 grid((unsigned)((max_rows + 255) / 256), n_models);
  hipLaunchKernelGGL(forest_predict_kernel, grid, dim3(256), 0, stream, Xb, F, model_row_off, row_list,
                     model_tree_off, tree_off, tree_weight, (const int4*)nodes, default_left, missing_bin, leaf_value,
                     K, out);
  return (int)hipGetLastError();
}

}  // extern "C"

// SanityChecker statistics (SanityChecker.scala:407-470, OpStatistics.scala:71-97).
//
// * col_partials_kernel / col_fold_kernel -- Spark Statistics.colStats in one HBM pass with a
//   numerically stable variance: each workgroup covers 64 columns x a row chunk (4 waves stride the
//   rows, one lane per column, 256 B coalesced per row) and accumulates fp64 sums of (x - K) and
//   (x - K)^2 around a per-chunk shift K (the chunk's first value of the column), giving the chunk's
//   (count, mean, M2) without the sum-of-squares cancellation; chunks are folded with Chan's pairwise
//   update. Also min / max / non-zeros.
// * gram_aug_kernel / gram_fold_kernel -- the centred Gramian of [X - mu | onehot(y)] on the matrix
//   cores (v_mfma_f32_32x32x2_f32, exact fp32 products): 128x128 output tiles (upper triangle of tile
//   pairs) x row chunks, 4 waves each owning a 64x64 quadrant (2x2 accumulators of 32x32), 32-row
//   stages of both column tiles centred into double-buffered LDS. The fp32 accumulators are flushed into fp64
//   registers every 256 rows; chunks are summed in fp64 by the fold kernel, which also mirrors the
//   tiles into the full symmetric matrix. The X-block gives Pearson correlations, the label block
//   gives the label x column contingency sums (onehot(y)^T (X - mu), + n_l mu on the host) and the
//   label counts -- all in one pass over the sampled rows.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdlib>
#include <stdint.h>
#include <float.h>

namespace {

__global__ void __launch_bounds__(256) col_partials_kernel(const float* __restrict__ X, int64_t n, int d, int64_t ld,
                                                           int64_t rows_per_chunk, double* __restrict__ part) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int ty = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
  const int64_t r1 = min(n, r0 + rows_per_chunk);
  double s = 0, q = 0, nz = 0;
  float mn = FLT_MAX, mx = -FLT_MAX;
  const double K = (c < d && r0 < r1) ? (double)X[r0 * ld + c] : 0.0;
  if (c < d) {
    for (int64_t r = r0 + ty; r < r1; r += 4) {
      const float v = X[r * ld + c];
      const double e = (double)v - K;
      s += e;
      q += e * e;
      mn = fminf(mn, v);
      mx = fmaxf(mx, v);
      nz += v != 0.f;
    }
  }
  __shared__ double sh[4][5][64];
  const int l = threadIdx.x & 63;
  sh[ty][0][l] = s; sh[ty][1][l] = q; sh[ty][2][l] = mn; sh[ty][3][l] = mx; sh[ty][4][l] = nz;
  __syncthreads();
  if (ty == 0 && c < d) {
    for (int k = 1; k < 4; ++k) {
      s += sh[k][0][l]; q += sh[k][1][l]; nz += sh[k][4][l];
      mn = fminf(mn, (float)sh[k][2][l]); mx = fmaxf(mx, (float)sh[k][3][l]);
    }
    const double cnt = (double)(r1 > r0 ? r1 - r0 : 0);
    const double mean = cnt > 0 ? K + s / cnt : 0.0;
    const double m2 = cnt > 0 ? fmax(q - s * s / cnt, 0.0) : 0.0;
    double* p = part + (int64_t)blockIdx.y * 6 * d;
    p[c] = mean; p[d + c] = m2; p[2 * d + c] = mn; p[3 * d + c] = mx; p[4 * d + c] = nz; p[5 * d + c] = cnt;
  }
}

// out rows: 0 sum, 1 M2 (sum of squared deviations), 2 min, 3 max, 4 non-zeros, 5 mean
__global__ void col_fold_kernel(const double* __restrict__ part, int chunks, int d, double* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= d) return;
  double na = 0, ma = 0, m2 = 0, nz = 0, mn = DBL_MAX, mx = -DBL_MAX;
  // the merge is a serial chain in chunk order (the CPU twin's order); the partials of the next 8 chunks are
  // loaded together first, so the chain waits on one load round trip per 8 chunks instead of one per chunk
  constexpr int U = 8;
  for (int k0 = 0; k0 < chunks; k0 += U) {
    double pn[U], pm[U], pq[U], pz[U], pl[U], ph[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = min(k0 + u, chunks - 1);
      const double* p = part + (int64_t)k * 6 * d;
      pn[u] = k0 + u < chunks ? p[5 * d + c] : 0.0;
      pm[u] = p[c];
      pq[u] = p[d + c];
      pl[u] = p[2 * d + c];
      ph[u] = p[3 * d + c];
      pz[u] = p[4 * d + c];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const double nb = pn[u];
      if (nb <= 0) continue;
      const double n = na + nb, delta = pm[u] - ma;
      ma += delta * (nb / n);
      m2 += pq[u] + delta * delta * (na * nb / n);
      na = n;
      nz += pz[u];
      mn = fmin(mn, pl[u]);
      mx = fmax(mx, ph[u]);
    }
  }
  out[c] = ma * na; out[d + c] = m2; out[2 * d + c] = mn; out[3 * d + c] = mx; out[4 * d + c] = nz;
  out[5 * d + c] = ma;
}

// ------------------------------------------------------------------------------------ Gramian
using f32x16 = __attribute__((ext_vector_type(16))) float;

constexpr int GT = 128;     // output tile edge (columns of the augmented matrix)
constexpr int GK = 32;      // rows per LDS stage
constexpr int kFlush = 8;   // stages between fp32 -> fp64 accumulator flushes (256 rows)

struct TilePair {
  int32_t i, j;
};

// p-th tile pair (i <= j) of the upper triangle of an nt x nt tile grid, row by row.
__device__ __forceinline__ TilePair tile_pair(int p, int nt) {
  int i = 0;
  while (p >= nt - i) {
    p -= nt - i;
    ++i;
  }
  return TilePair{i, i + p};
}

// Loads of one 32-row stage: thread t owns column t % 128 of both tiles and rows 2u + t / 128 (u < 16), so the
// column's kind (data / label / padding) and centre are per-thread constants and its 16 row loads are
// independent (all in flight at once).
struct AugCol {
  int kind;      // 0: X[r][c] - mu, 1: (y[r] == lbl), 2: zero
  int c;
  int lbl;
  float mu;
};

__device__ __forceinline__ AugCol aug_col(int c, int d, int L, const float* __restrict__ mu) {
  if (c < d) return AugCol{0, c, 0, mu[c]};
  if (c < d + L) return AugCol{1, c, c - d, 0.f};
  return AugCol{2, c, 0, 0.f};
}

__device__ __forceinline__ void aug_stage(const float* __restrict__ X, int64_t ld, const int32_t* __restrict__ y,
                                          const AugCol& col, int64_t rs, int64_t r1, int rsub, float* v) {
  // branch-free per row: all 16 loads (row clamped into the chunk) are issued before any is used -- a
  // conditional load per row made the compiler wait for each one in turn (16 serial memory latencies)
  if (col.kind == 0) {
    float t[GK / 2];
#pragma unroll
    for (int u = 0; u < GK / 2; ++u) t[u] = X[min(rs + 2 * u + rsub, r1 - 1) * ld + col.c];
#pragma unroll
    for (int u = 0; u < GK / 2; ++u) v[u] = rs + 2 * u + rsub < r1 ? t[u] - col.mu : 0.f;
  } else if (col.kind == 1) {
    int t[GK / 2];
#pragma unroll
    for (int u = 0; u < GK / 2; ++u) t[u] = y[min(rs + 2 * u + rsub, r1 - 1)];
#pragma unroll
    for (int u = 0; u < GK / 2; ++u) v[u] = (rs + 2 * u + rsub < r1 && t[u] == col.lbl) ? 1.f : 0.f;
  } else {
#pragma unroll
    for (int u = 0; u < GK / 2; ++u) v[u] = 0.f;
  }
}

// Double-buffered: the next stage's rows are loaded into registers while the matrix cores work on the
// current LDS stage, then stored into the other LDS buffer -- one barrier per stage, global-load latency
// hidden behind the MFMAs instead of serialised with them.
__global__ void __launch_bounds__(256) gram_aug_kernel(const float* __restrict__ X, int64_t n, int d, int64_t ld,
                                                       const float* __restrict__ mu, const int32_t* __restrict__ y,
                                                       int L, int nt, int64_t rows_per_chunk,
                                                       double* __restrict__ part, int flush) {
  __shared__ float tA[2][GK][GT + 4];
  __shared__ float tB[2][GK][GT + 4];
  const TilePair tp = tile_pair(blockIdx.x, nt);
  const int ca = tp.i * GT, cb = tp.j * GT;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
  const int64_t r1 = min(n, r0 + rows_per_chunk);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int qa = (wave >> 1) * 64, qb = (wave & 1) * 64;   // this wave's 64x64 quadrant
  const int li = lane & 31, lk = lane >> 5;
  const int cc = threadIdx.x & (GT - 1), rsub = threadIdx.x >> 7;
  const AugCol colA = aug_col(ca + cc, d, L, mu), colB = aug_col(cb + cc, d, L, mu);
  f32x16 acc[2][2];
  double dacc[2][2][16];
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b) {
      acc[a][b] = f32x16{};
      for (int e = 0; e < 16; ++e) dacc[a][b][e] = 0.0;
    }
  float va[GK / 2], vb[GK / 2];
  if (r0 < r1) {
    aug_stage(X, ld, y, colA, r0, r1, rsub, va);
    aug_stage(X, ld, y, colB, r0, r1, rsub, vb);
  }
  int stage = 0;
  for (int64_t rs = r0; rs < r1; rs += GK, ++stage) {
    const int buf = stage & 1;
#pragma unroll
    for (int u = 0; u < GK / 2; ++u) {
      tA[buf][2 * u + rsub][cc] = va[u];
      tB[buf][2 * u + rsub][cc] = vb[u];
    }
    __syncthreads();
    if (rs + GK < r1) {                          // next stage in flight during this stage's MFMAs
      aug_stage(X, ld, y, colA, rs + GK, r1, rsub, va);
      aug_stage(X, ld, y, colB, rs + GK, r1, rsub, vb);
    }
#pragma unroll 4
    for (int k = 0; k < GK; k += 2) {
      const float a0 = tA[buf][k + lk][qa + li], a1 = tA[buf][k + lk][qa + 32 + li];
      const float b0 = tB[buf][k + lk][qb + li], b1 = tB[buf][k + lk][qb + 32 + li];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    if ((stage + 1) % flush == 0) {
      for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b) {
          for (int e = 0; e < 16; ++e) dacc[a][b][e] += (double)acc[a][b][e];
          acc[a][b] = f32x16{};
        }
    }
  }
  // C/D map of 32x32: col = lane & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5)
  double* out = part + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * GT * GT;
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b)
      for (int e = 0; e < 16; ++e) {
        const int row = qa + a * 32 + (e & 3) + 8 * (e >> 2) + 4 * lk;
        const int col = qb + b * 32 + li;
        out[row * GT + col] = dacc[a][b][e] + (double)acc[a][b][e];
      }
}

// ------------------------------------------------------------------------------ bf16 Gramian
// gram_bf16_kernel -- A^T A of a bf16 matrix A [n][lda] on the bf16 matrix cores (v_mfma_f32_32x32x16_bf16:
// products of bf16 values are exact in fp32). ops/stats.py builds A from the SanityChecker input: the columns
// whose values are exact in bf16 (one-hot, indicators, counts) as they are, a ones column, and every other column
// centred and split into three bf16 parts (hi + mid + lo = the fp32 value exactly), so the Gramian of the
// original columns is assembled exactly from A's blocks in fp64 (8x the K per instruction of the fp32 MFMA of
// gram_aug_kernel, half the bytes). Same tiling and fp64 flush / chunk fold as gram_aug_kernel: 128 x 128 output
// tile pairs (upper triangle) x row chunks, 4 waves owning 64 x 64 quadrants; each 32-row stage is stored
// row-major into double-buffered LDS with 16-byte writes and read back transposed (row on the k axis) with
// ds_read_b64_tr_b16 (cdna_hip_programming.md T10), rows padded to 320 B so the four rows of a read fall on
// distinct banks.
typedef __bf16 gbf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 gbf16x4 __attribute__((ext_vector_type(4)));
typedef short gs16x4 __attribute__((ext_vector_type(4)));
constexpr int GS = GT + 32;           // LDS row stride (bf16 elements)

__device__ __forceinline__ gbf16x4 gtr_read(const __bf16* p) {
  const gs16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) gs16x4*)(p));
  return __builtin_bit_cast(gbf16x4, v);
}

// operand fragment of k-step s for the 32 columns c0 .. c0 + 31 of a [32 rows][GS] stage: lane l holds column
// c0 + (l & 31), rows 16 s + 8 (l >> 5) + j (j = 0..7)
__device__ __forceinline__ gbf16x8 gram_frag(const __bf16* T, int c0, int s, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const __bf16* a = T + (16 * s + 8 * (g >> 1) + q) * GS + c0 + 16 * (g & 1) + 4 * p;
  const gbf16x4 lo = gtr_read(a), hi = gtr_read(a + 4 * GS);
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

__global__ void __launch_bounds__(256) gram_bf16_kernel(const __bf16* __restrict__ A, int64_t n, int64_t lda, int nt,
                                                        int64_t rows_per_chunk, double* __restrict__ part, int flush) {
  __shared__ __attribute__((aligned(16))) __bf16 tA[2][GK * GS];
  __shared__ __attribute__((aligned(16))) __bf16 tB[2][GK * GS];
  const TilePair tp = tile_pair(blockIdx.x, nt);
  const int ca = tp.i * GT, cb = tp.j * GT;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
  const int64_t r1 = min(n, r0 + rows_per_chunk);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int qa = (wave >> 1) * 64, qb = (wave & 1) * 64;
  const int li = lane & 31, lk = lane >> 5;
  const int lr = threadIdx.x >> 4, c8 = (threadIdx.x & 15) * 8;      // stage loads: rows lr, lr + 16
  f32x16 acc[2][2];
  double dacc[2][2][16];
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b) {
      acc[a][b] = f32x16{};
      for (int e = 0; e < 16; ++e) dacc[a][b][e] = 0.0;
    }
  gbf16x8 va[2], vb[2];
  auto load = [&](int64_t rs) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t r = rs + lr + 16 * u;
      const int64_t rc = r < r1 ? r : r1 - 1;                 // clamped, then zeroed: loads issued together
      const gbf16x8 xa = *reinterpret_cast<const gbf16x8*>(A + rc * lda + ca + c8);
      const gbf16x8 xb = *reinterpret_cast<const gbf16x8*>(A + rc * lda + cb + c8);
      va[u] = r < r1 ? xa : gbf16x8{};
      vb[u] = r < r1 ? xb : gbf16x8{};
    }
  };
  if (r0 < r1) load(r0);
  int stage = 0;
  for (int64_t rs = r0; rs < r1; rs += GK, ++stage) {
    const int buf = stage & 1;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      *reinterpret_cast<gbf16x8*>(&tA[buf][(lr + 16 * u) * GS + c8]) = va[u];
      *reinterpret_cast<gbf16x8*>(&tB[buf][(lr + 16 * u) * GS + c8]) = vb[u];
    }
    __syncthreads();
    if (rs + GK < r1) load(rs + GK);                          // next stage in flight during this stage's MFMAs
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const gbf16x8 a0 = gram_frag(tA[buf], qa, s, lane), a1 = gram_frag(tA[buf], qa + 32, s, lane);
      const gbf16x8 b0 = gram_frag(tB[buf], qb, s, lane), b1 = gram_frag(tB[buf], qb + 32, s, lane);
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[1][1], 0, 0, 0);
    }
    if ((stage + 1) % flush == 0) {
      for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b) {
          for (int e = 0; e < 16; ++e) dacc[a][b][e] += (double)acc[a][b][e];
          acc[a][b] = f32x16{};
        }
    }
  }
  double* out = part + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * GT * GT;
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b)
      for (int e = 0; e < 16; ++e) {
        const int row = qa + a * 32 + (e & 3) + 8 * (e >> 2) + 4 * lk;
        const int col = qb + b * 32 + li;
        out[row * GT + col] = dacc[a][b][e] + (double)acc[a][b][e];
      }
}

// col_bf16_exact_kernel -- per column, whether every value of the column is exact in bf16 (the low 16 bits of its
// fp32 pattern are zero): lane = column, waves stride a row chunk, one atomic OR per thread (order-free).
__global__ void __launch_bounds__(256) col_bf16_exact_kernel(const float* __restrict__ X, int64_t n, int d,
                                                             int64_t ld, int64_t rows_per_chunk,
                                                             unsigned* __restrict__ low_bits) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  if (c >= d) return;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
  const int64_t r1 = min(n, r0 + rows_per_chunk);
  unsigned acc = 0;
  for (int64_t r = r0 + (threadIdx.x >> 6); r < r1; r += 4) acc |= __float_as_uint(X[r * ld + c]) & 0xFFFFu;
  if (acc) atomicOr(low_bits + c, acc);
}

// bf16_pack_kernel -- B[r][j] (bf16, row stride ldb) from the fp32 rows of X per output column j:
//   mode 0 zero, 1 one, 2 X[r][src] as is, 3 / 4 / 5 the high / middle / low bf16 part of (X[r][src] - mu) * sc
//   (the three parts sum to the fp32 value exactly), 6 (y[r] == src) -- the operand images of gram_bf16_kernel
// and of the linear learners' bf16 design copy (ops/stats.py, ops/linear.py).
// Thread = 8 consecutive output columns (one 16-byte store per row); a wave covers 64 column groups of a row and
// the block's 4 waves walk the rows of its row chunk, so the column descriptors (mode, source, shift, scale) are
// loaded once into registers per thread instead of once per element. Eight sources that are consecutive X columns
// (the usual case: design columns in order) are read as two 16-byte loads instead of eight 4-byte gathers.
__global__ void __launch_bounds__(256) bf16_pack_kernel(const float* __restrict__ X, int64_t n, int64_t ld,
                                                        const int32_t* __restrict__ y, const int32_t* __restrict__ src,
                                                        const int32_t* __restrict__ mode, const float* __restrict__ mu,
                                                        const float* __restrict__ sc, __bf16* __restrict__ B,
                                                        int64_t ldb, int64_t rows_per_blk) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t g = (int64_t)blockIdx.y * 64 + lane;
  if (g >= ldb / 8) return;                       // whole lanes idle: no barrier below
  const int j0 = (int)g * 8;
  int m[8], s[8];
  float sh[8], sf[8];
  bool contig = true, need_y = false;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    m[u] = mode[j0 + u];
    s[u] = src[j0 + u];
    sh[u] = mu[j0 + u];
    sf[u] = sc[j0 + u];
  }
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    contig &= m[u] >= 2 && m[u] <= 5 && s[u] == s[0] + u;
    need_y |= m[u] == 6;
  }
  contig &= (s[0] & 3) == 0 && (ld & 3) == 0 && ((uintptr_t)X & 15) == 0;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_blk, r1 = min(n, r0 + rows_per_blk);
  for (int64_t r = r0 + wave; r < r1; r += 4) {
    const float* xr = X + r * ld;
    float xv[8];
    if (contig) {
      const float4 a = *reinterpret_cast<const float4*>(xr + s[0]);
      const float4 b = *reinterpret_cast<const float4*>(xr + s[0] + 4);
      xv[0] = a.x; xv[1] = a.y; xv[2] = a.z; xv[3] = a.w;
      xv[4] = b.x; xv[5] = b.y; xv[6] = b.z; xv[7] = b.w;
    } else {
#pragma unroll
      for (int u = 0; u < 8; ++u) xv[u] = (m[u] >= 2 && m[u] <= 5) ? xr[s[u]] : 0.f;
    }
    const int yr = need_y ? y[r] : 0;
    gbf16x8 out;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      float v = 0.f;
      if (m[u] == 1) {
        v = 1.f;
      } else if (m[u] == 2) {
        v = xv[u];
      } else if (m[u] >= 3 && m[u] <= 5) {
        const float c = (xv[u] - sh[u]) * sf[u];
        const float h = (float)(__bf16)c;
        const float mid = (float)(__bf16)(c - h);
        v = m[u] == 3 ? h : (m[u] == 4 ? mid : c - h - mid);
      } else if (m[u] == 6) {
        v = yr == s[u] ? 1.f : 0.f;
      }
      out[u] = (__bf16)v;
    }
    *reinterpret_cast<gbf16x8*>(B + r * ldb + j0) = out;
  }
}

// G[D][D] (D = d + L) = sum over chunks of the tile partials, mirrored into the lower triangle.
__global__ void __launch_bounds__(256) gram_fold_kernel(const double* __restrict__ part, int chunks, int npairs,
                                                        int nt, int D, double* __restrict__ G) {
  const int p = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= GT * GT) return;
  double s = 0.0;
  for (int c = 0; c < chunks; ++c) s += part[((int64_t)c * npairs + p) * GT * GT + e];
  const TilePair tp = tile_pair(p, nt);
  const int i = tp.i * GT + e / GT, j = tp.j * GT + e % GT;
  if (i < D && j < D) {
    G[(int64_t)i * D + j] = s;
    G[(int64_t)j * D + i] = s;
  }
}

// ------------------------------------------------------------------------------- weighted fp64 Grams
// wgram_kernel / wgram_fold_kernel -- the normal-equation statistics of the linear learners (SURVEY.md K22:
// Spark WeightedLeastSquares / IRLS, OpLinearRegression.scala:48-209, OpGeneralizedLinearRegression.scala:
// 49-203): G_k = A_k^T diag(w_k) A_k with A_k = [X | 1 | y_k] for K weight columns at once, on the fp64
// matrix cores (v_mfma_f64_16x16x4_f64: exact fp64 products and sums, the numerics of the fp64 library GEMM
// it replaces). X is read as fp32 and widened in LDS; the weights and the optional per-weight (or shared)
// response are fp64. Workgroup = one 64x64 output tile pair (upper triangle) x one row chunk x KW weights;
// 4 waves each own a 32x32 quadrant (2x2 accumulators of 16x16 per weight), the weight scales the A
// operand in registers and the response column is substituted per weight, so one LDS stage of X serves all
// KW weights. Chunk partials are summed in a fixed order by the fold kernel (deterministic), which mirrors
// the tiles into the full symmetric matrices.
using f64x4 = __attribute__((ext_vector_type(4))) double;

constexpr int WT = 64;      // output tile edge
constexpr int WK = 16;      // rows per LDS stage
constexpr int KW = 4;       // weight columns per workgroup

struct WGramArgs {
  const float* X;
  int64_t n;
  int d;
  int64_t ldx;
  const double* W;          // [n][ldw], columns 0..K-1
  int64_t ldw;
  const double* Y;          // [n][ldy] or null; column k (per_weight) or 0
  int64_t ldy;
  int per_weight;
  int D;                    // d + 1 (+ 1 with Y)
  int K;
  int nt;
  int npairs;
  int64_t rpc;
  double* part;             // [chunks][npairs][K][WT][WT]
};

__device__ __forceinline__ TilePair wtile_pair(int p, int nt) { return tile_pair(p, nt); }

__global__ void __launch_bounds__(256) wgram_kernel(WGramArgs a) {
  __shared__ double tA[WK][WT + 1];
  __shared__ double tB[WK][WT + 1];
  __shared__ double tw[WK][KW];
  __shared__ double ty[WK][KW];
  const TilePair tp = wtile_pair(blockIdx.x, a.nt);
  const int ca = tp.i * WT, cb = tp.j * WT;
  const int w0 = blockIdx.z * KW;
  const int64_t r0 = (int64_t)blockIdx.y * a.rpc;
  const int64_t r1 = min(a.n, r0 + a.rpc);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int qa = (wave >> 1) * 32, qb = (wave & 1) * 32;
  const int li = lane & 15, lk = lane >> 4;
  const int ycol = a.Y ? a.d + 1 : -1;
  const int cc = threadIdx.x & (WT - 1), rsub = threadIdx.x >> 6;   // loader: column cc, rows rsub + 4u
  f64x4 acc[KW][2][2];
#pragma unroll
  for (int k = 0; k < KW; ++k)
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y) acc[k][x][y] = f64x4{0.0, 0.0, 0.0, 0.0};
  // this lane's operand columns (fixed for the whole kernel)
  int colA[2], colB[2];
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    colA[x] = ca + qa + 16 * x + li;
    colB[x] = cb + qb + 16 * x + li;
  }
  for (int64_t rs = r0; rs < r1; rs += WK) {
#pragma unroll
    for (int u = 0; u < WK / 4; ++u) {
      const int rr = rsub + 4 * u;
      const int64_t r = rs + rr;
      const int64_t rc = min(r, r1 - 1);
      const int c1 = ca + cc, c2 = cb + cc;
      const float x1 = a.X[rc * a.ldx + min(c1, a.d - 1)];
      const float x2 = a.X[rc * a.ldx + min(c2, a.d - 1)];
      const bool in = r < r1;
      tA[rr][cc] = !in ? 0.0 : (c1 < a.d ? (double)x1 : (c1 == a.d ? 1.0 : 0.0));
      tB[rr][cc] = !in ? 0.0 : (c2 < a.d ? (double)x2 : (c2 == a.d ? 1.0 : 0.0));
    }
    if (threadIdx.x < WK * KW) {
      const int rr = threadIdx.x / KW, k = threadIdx.x % KW;
      const int64_t r = rs + rr;
      const bool ok = r < r1 && w0 + k < a.K;
      tw[rr][k] = ok ? a.W[r * a.ldw + w0 + k] : 0.0;
      ty[rr][k] = (ok && a.Y) ? a.Y[r * a.ldy + (a.per_weight ? w0 + k : 0)] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < WK / 4; ++s) {
      const int kk = 4 * s + lk;
      double av[2], bv[2];
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        av[x] = tA[kk][qa + 16 * x + li];
        bv[x] = tB[kk][qb + 16 * x + li];
      }
#pragma unroll
      for (int k = 0; k < KW; ++k) {
        const double w = tw[kk][k], yk = ty[kk][k];
#pragma unroll
        for (int x = 0; x < 2; ++x) {
          const double aw = (colA[x] == ycol ? yk : av[x]) * w;
#pragma unroll
          for (int y = 0; y < 2; ++y) {
            const double b = colB[y] == ycol ? yk : bv[y];
            acc[k][x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(aw, b, acc[k][x][y], 0, 0, 0);
          }
        }
      }
    }
    __syncthreads();
  }
  // f64 16x16x4 C/D map: col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
  for (int k = 0; k < KW; ++k) {
    if (w0 + k >= a.K) break;
    double* out = a.part + (((int64_t)blockIdx.y * a.npairs + blockIdx.x) * a.K + w0 + k) * WT * WT;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = qa + 16 * x + lk + 4 * e;
          const int col = qb + 16 * y + li;
          out[row * WT + col] = acc[k][x][y][e];
        }
  }
}

// G[k][D][D] = sum over chunks of the tile partials, mirrored into the lower triangle. grid (WT*WT/256, npairs, K)
__global__ void __launch_bounds__(256) wgram_fold_kernel(const double* __restrict__ part, int chunks, int npairs,
                                                         int K, int nt, int D, double* __restrict__ G) {
  const int p = blockIdx.y, k = blockIdx.z;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= WT * WT) return;
  double s = 0.0;
  for (int c = 0; c < chunks; ++c) s += part[(((int64_t)c * npairs + p) * K + k) * WT * WT + e];
  const TilePair tp = tile_pair(p, nt);
  // a diagonal tile holds both (i, j) and (j, i), computed with different roundings (the weight scales the
  // A operand): its upper triangle alone is mirrored, so the result is symmetric and race-free
  if (tp.i == tp.j && e / WT > e % WT) return;
  const int i = tp.i * WT + e / WT, j = tp.j * WT + e % WT;
  if (i < D && j < D) {
    double* g = G + (int64_t)k * D * D;
    g[(int64_t)i * D + j] = s;
    g[(int64_t)j * D + i] = s;
  }
}

// weighted_colsums_kernel / weighted_colsums_fold_kernel -- per problem p and column j the fp64 sums
// s1 = sum_r W[r, p] X[r, j] and s2 = sum_r W[r, p] X[r, j]^2 (the linear learners' feature standardisation,
// Spark's weighted summarizer; models/linear.py _feature_std). Lane = column, 4 waves stride the rows of a
// fixed 4096-row chunk, 16 problems per workgroup; the chunk partials are folded in chunk order. Neither the
// chunking nor the arithmetic of a problem depends on the other problems of the launch, so a problem's
// statistics are the same bits whatever batch it is fitted in (the selector's speculative refits).
constexpr int kWcsRows = 4096;
constexpr int kWcsP = 16;

__global__ void __launch_bounds__(256) weighted_colsums_kernel(const float* __restrict__ X, int64_t n, int d,
                                                               int64_t ldx, const float* __restrict__ W,
                                                               int64_t ldw, int P, double* __restrict__ part) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + lane;
  const int64_t chunk = blockIdx.y;
  const int p0 = blockIdx.z * kWcsP;
  const int np = min(kWcsP, P - p0);
  const int64_t r0 = chunk * kWcsRows, r1 = min(n, r0 + kWcsRows);
  double s1[kWcsP], s2[kWcsP];
#pragma unroll
  for (int q = 0; q < kWcsP; ++q) s1[q] = s2[q] = 0.0;
  const int jc = min(j, d - 1);
  for (int64_t r = r0 + wave; r < r1; r += 4) {
    const double x = (double)X[r * ldx + jc];
    const double xx = x * x;
#pragma unroll
    for (int q = 0; q < kWcsP; ++q) {
      const double w = q < np ? (double)W[r * ldw + p0 + q] : 0.0;
      s1[q] += w * x;
      s2[q] += w * xx;
    }
  }
  __shared__ double sh[4][2][kWcsP][64];
#pragma unroll
  for (int q = 0; q < kWcsP; ++q) {
    sh[wave][0][q][lane] = s1[q];
    sh[wave][1][q][lane] = s2[q];
  }
  __syncthreads();
  if (wave == 0 && j < d) {
    for (int q = 0; q < np; ++q)
      for (int k = 0; k < 2; ++k) {
        const double v = ((sh[0][k][q][lane] + sh[1][k][q][lane]) + sh[2][k][q][lane]) + sh[3][k][q][lane];
        part[((chunk * P + p0 + q) * 2 + k) * (int64_t)d + j] = v;
      }
  }
}

// out[p][k][j] = sum over chunks in chunk order of part[chunk][p][k][j]
__global__ void weighted_colsums_fold_kernel(const double* __restrict__ part, int64_t chunks, int64_t words,
                                             double* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= words) return;
  double s = 0.0;
  for (int64_t c = 0; c < chunks; ++c) s += part[c * words + e];
  out[e] = s;
}

// Per-problem, per-class column sums (the label x column contingency and the
// NaiveBayes class feature sums): part[chunk][p * L + c][j] = sum of X[r][j] over rows r of the chunk with
// codes[p][r] == c (-1 = row not in problem p). Lane = column (64 per workgroup), wave = row stride; every
// wave keeps private fp64 accumulators in LDS, summed in a fixed order -- no atomics, deterministic.
__global__ void __launch_bounds__(256) class_colsum_kernel(const float* __restrict__ X, int64_t n, int d, int64_t ld,
                                                           const int32_t* __restrict__ codes, int P, int L,
                                                           int64_t rows_per_chunk, double* __restrict__ part) {
  extern __shared__ double acc[];                 // [4 waves][P * L][64]
  const int PL = P * L;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + lane;
  double* my = acc + (size_t)wave * PL * 64;
  for (int k = 0; k < PL; ++k) my[k * 64 + lane] = 0.0;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
  const int64_t r1 = min(n, r0 + rows_per_chunk);
  if (j < d) {
    for (int64_t r = r0 + wave; r < r1; r += 4) {
      const double v = (double)X[r * ld + j];
      for (int p = 0; p < P; ++p) {
        const int c = codes[(int64_t)p * n + r];
        if (c >= 0 && c < L) my[(p * L + c) * 64 + lane] += v;
      }
    }
  }
  __syncthreads();
  if (wave == 0 && j < d) {
    double* out = part + (int64_t)blockIdx.y * PL * d;
    for (int k = 0; k < PL; ++k) {
      double t = 0.0;
      for (int w = 0; w < 4; ++w) t += acc[((size_t)w * PL + k) * 64 + lane];
      out[(int64_t)k * d + j] = t;
    }
  }
}

__global__ void colsum_fold_kernel(const double* __restrict__ part, int chunks, int64_t words,
                                   double* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= words) return;
  double t = 0.0;
  for (int c = 0; c < chunks; ++c) t += part[(int64_t)c * words + k];
  out[k] = t;
}

}  // namespace

extern "C" {

// out[p][c][j] (fp64, P*L*d) = sum over rows with codes[p][row] == c of X[row][j]; P * L <= 64.
int tmog_hip_class_colsum(const float* X, int64_t n, int d, int64_t ld, const int32_t* codes, int P, int L, double* out,
                          hipStream_t stream) {
  if (n <= 0 || d <= 0 || P <= 0 || L <= 0) return -1;
  if (P * L > 64) return -2;
  const int cblocks = (d + 63) / 64;
  int64_t chunks = (1024 + cblocks - 1) / cblocks;
  if (chunks > (n + 255) / 256) chunks = (n + 255) / 256;
  if (chunks < 1) chunks = 1;
  const int64_t rpc = (n + chunks - 1) / chunks;
  chunks = (n + rpc - 1) / rpc;
  const int64_t words = (int64_t)P * L * d;
  double* part = nullptr;
  hipError_t e = hipMallocAsync((void**)&part, sizeof(double) * words * chunks, stream);
  if (e != hipSuccess) return (int)e;
  const size_t lds = (size_t)4 * P * L * 64 * sizeof(double);
  hipLaunchKernelGGL(class_colsum_kernel, dim3(cblocks, (unsigned)chunks), dim3(256), lds, stream, X, n, d, ld, codes, P,
                     L, rpc, part);
  hipLaunchKernelGGL(colsum_fold_kernel, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, stream, part, (int)chunks,
                     words, out);
  hipFreeAsync(part, stream);
  return (int)hipGetLastError();
}

int tmog_hip_col_stats(const float* X, const void* unused, int64_t n, int d, int64_t ld, double* out,
                       hipStream_t stream) {
  (void)unused;
  if (n == 0 || d == 0) return 0;
  const int cblocks = (d + 63) / 64;
  int64_t chunks = (2048 + cblocks - 1) / cblocks;           // ~2048 workgroups in flight
  if (chunks > n / 256 + 1) chunks = n / 256 + 1;
  if (chunks < 1) chunks = 1;
  const int64_t rpc = (n + chunks - 1) / chunks;
  double* part = nullptr;
  hipError_t e = hipMallocAsync((void**)&part, sizeof(double) * 6 * d * chunks, stream);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(col_partials_kernel, dim3(cblocks, (unsigned)chunks), dim3(256), 0, stream, X, n, d, ld, rpc, part);
  hipLaunchKernelGGL(col_fold_kernel, dim3((d + 255) / 256), dim3(256), 0, stream, part, (int)chunks, d, out);
  hipFreeAsync(part, stream);
  return (int)hipGetLastError();
}

// out [P][2][d] fp64: sum_r W[r, p] X[r, j] and sum_r W[r, p] X[r, j]^2 (fixed 4096-row chunks, chunk-ordered fold).
int tmog_hip_weighted_colsums(const float* X, int64_t n, int d, int64_t ldx, const float* W, int64_t ldw, int P,
                              double* out, hipStream_t stream) {
  if (n <= 0 || d <= 0 || P <= 0) return -1;
  const int64_t chunks = (n + kWcsRows - 1) / kWcsRows;
  if (chunks > 65535) return -2;
  const int64_t words = (int64_t)P * 2 * d;
  double* part = nullptr;
  hipError_t e = hipMallocAsync((void**)&part, sizeof(double) * words * chunks, stream);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(weighted_colsums_kernel, dim3((unsigned)((d + 63) / 64), (unsigned)chunks,
                                                   (unsigned)((P + kWcsP - 1) / kWcsP)),
                     dim3(256), 0, stream, X, n, d, ldx, W, ldw, P, part);
  hipLaunchKernelGGL(weighted_colsums_fold_kernel, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, stream, part,
                     chunks, words, out);
  hipFreeAsync(part, stream);
  return (int)hipGetLastError();
}

// G (fp64, [K][D][D], fully written; D = d + 1 + (Y != null)) = A_k^T diag(W[:, k]) A_k, A_k = [X | 1 | Y[:, k]]
// (Y column 0 for every k unless per_weight). X fp32 [n][ldx]; W, Y fp64.
int tmog_hip_wgram(const float* X, int64_t n, int d, int64_t ldx, const double* W, int64_t ldw, int K,
                   const double* Y, int64_t ldy, int per_weight, double* G, hipStream_t stream) {
  if (n <= 0 || d <= 0 || K <= 0) return -1;
  const int D = d + 1 + (Y ? 1 : 0);
  const int nt = (D + WT - 1) / WT;
  const int npairs = nt * (nt + 1) / 2;
  const int kg = (K + KW - 1) / KW;
  // partials bounded to ~128 MB; >= ~512 workgroups when the rows allow
  const int64_t per_chunk = (int64_t)npairs * K * WT * WT * (int64_t)sizeof(double);
  int64_t chunks = (512 + (int64_t)npairs * kg - 1) / ((int64_t)npairs * kg);
  const int64_t max_chunks = std::max<int64_t>(1, ((int64_t)128 << 20) / per_chunk);
  chunks = std::min(chunks, max_chunks);
  chunks = std::min(chunks, (n + 255) / 256);
  chunks = std::max<int64_t>(chunks, 1);
  int64_t rpc = (n + chunks - 1) / chunks;
  rpc = (rpc + WK - 1) / WK * WK;
  chunks = (n + rpc - 1) / rpc;
  double* part = nullptr;
  hipError_t e = hipMallocAsync((void**)&part, per_chunk * chunks, stream);
  if (e != hipSuccess) return (int)e;
  WGramArgs a{X, n, d, ldx, W, ldw, Y, ldy, per_weight, D, K, nt, npairs, rpc, part};
  hipLaunchKernelGGL(wgram_kernel, dim3((unsigned)npairs, (unsigned)chunks, (unsigned)kg), dim3(256), 0, stream, a);
  hipLaunchKernelGGL(wgram_fold_kernel, dim3(WT * WT / 256, (unsigned)npairs, (unsigned)K), dim3(256), 0, stream, part,
                     (int)chunks, npairs, K, nt, D, G);
  hipFreeAsync(part, stream);
  return (int)hipGetLastError();
}

// G (fp64, [(d+L)^2], fully written) = [X - mu | onehot(y)]^T [X - mu | onehot(y)] over n rows.
int tmog_hip_gram_aug(const float* X, int64_t n, int d, int64_t ld, const float* mu, const int32_t* y, int L,
                      double* G, hipStream_t stream) {
  if (n <= 0 || d <= 0 || L < 0 || (L > 0 && y == nullptr)) return -1;
  const int D = d + L;
  const int nt = (D + GT - 1) / GT;
  const int npairs = nt * (nt + 1) / 2;
  int64_t chunks = (1024 + npairs - 1) / npairs;             // >= ~1024 workgroups
  const int64_t max_chunks = 4096 / npairs > 1 ? 4096 / npairs : 1;  // partials <= 512 MB
  if (chunks > max_chunks) chunks = max_chunks;
  if (chunks > (n + 1023) / 1024) chunks = (n + 1023) / 1024;
  if (chunks < 1) chunks = 1;
  int64_t rpc = (n + chunks - 1) / chunks;
  rpc = (rpc + GK - 1) / GK * GK;
  chunks = (n + rpc - 1) / rpc;
  double* part = nullptr;
  hipError_t e = hipMallocAsync((void**)&part, sizeof(double) * GT * GT * npairs * chunks, stream);
  if (e != hipSuccess) return (int)e;
  static const int flush = [] {              // TMOG_GRAM_FLUSH: stages between fp64 flushes (diagnostics)
    const char* e = std::getenv("TMOG_GRAM_FLUSH");
    const int v = e ? std::atoi(e) : kFlush;
    return v > 0 ? v : kFlush;
  }();
  hipLaunchKernelGGL(gram_aug_kernel, dim3((unsigned)npairs, (unsigned)chunks), dim3(256), 0, stream, X, n, d, ld, mu,
                     y, L, nt, rpc, part, flush);
  hipLaunchKernelGGL(gram_fold_kernel, dim3(GT * GT / 256, (unsigned)npairs), dim3(256), 0, stream, part,
                     (int)chunks, npairs, nt, D, G);
  hipFreeAsync(part, stream);
  return (int)hipGetLastError();
}

// low_bits[c] (zeroed here) = OR over the rows of the low 16 bits of column c: zero <=> the column is exact in bf16.
int tmog_hip_col_bf16_exact(const float* X, int64_t n, int d, int64_t ld, unsigned* low_bits, hipStream_t stream) {
  if (d <= 0) return 0;
  hipError_t e = hipMemsetAsync(low_bits, 0, sizeof(unsigned) * d, stream);
  if (e != hipSuccess) return (int)e;
  if (n <= 0) return 0;
  const int cblocks = (d + 63) / 64;
  int64_t chunks = (2048 + cblocks - 1) / cblocks;
  if (chunks > (n + 1023) / 1024) chunks = (n + 1023) / 1024;
  if (chunks < 1) chunks = 1;
  const int64_t rpc = (n + chunks - 1) / chunks;
  chunks = (n + rpc - 1) / rpc;
  hipLaunchKernelGGL(col_bf16_exact_kernel, dim3(cblocks, (unsigned)chunks), dim3(256), 0, stream, X, n, d, ld, rpc,
                     low_bits);
  return (int)hipGetLastError();
}

// B [n][ldb] bf16 (ldb a multiple of 8, B 16-byte aligned) from X per output column: src / mode / mu / sc have ldb
// entries (bf16_pack_kernel).
int tmog_hip_bf16_pack(const float* X, int64_t n, int64_t ld, const int32_t* y, const int32_t* src, const int32_t* mode,
                       const float* mu, const float* sc, void* B, int64_t ldb, hipStream_t stream) {
  if (n <= 0) return 0;
  if (ldb <= 0 || ldb % 8 || (uintptr_t)B % 16) return -2;
  const int64_t gy = (ldb / 8 + 63) / 64;         // column tiles of 64 groups (512 columns)
  if (gy > 65535) return -2;
  // ~4096 workgroups in all, at least 16 rows each
  const int64_t gx = max((int64_t)1, min((n + 15) / 16, (int64_t)4096 / gy));
  const int64_t rpb = (n + gx - 1) / gx;
  hipLaunchKernelGGL(bf16_pack_kernel, dim3((unsigned)((n + rpb - 1) / rpb), (unsigned)gy), dim3(256), 0, stream, X, n,
                     ld, y, src, mode, mu, sc, (__bf16*)B, ldb, rpb);
  return (int)hipGetLastError();
}

// G (fp64, [D][D], fully written) = A^T A for a bf16 A [n][lda] whose columns D .. nt * 128 - 1 are zero (lda >=
// nt * 128, a multiple of 8; A 16-byte aligned).
int tmog_hip_gram_bf16(const void* A, int64_t n, int64_t lda, int D, double* G, hipStream_t stream) {
  if (n <= 0 || D <= 0) return -1;
  const int nt = (D + GT - 1) / GT;
  if (lda < (int64_t)nt * GT || lda % 8 || (uintptr_t)A % 16) return -2;
  const int npairs = nt * (nt + 1) / 2;
  int64_t chunks = (1024 + npairs - 1) / npairs;
  const int64_t max_chunks = 4096 / npairs > 1 ? 4096 / npairs : 1;
  if (chunks > max_chunks) chunks = max_chunks;
  if (chunks > (n + 1023) / 1024) chunks = (n + 1023) / 1024;
  if (chunks < 1) chunks = 1;
  int64_t rpc = (n + chunks - 1) / chunks;
  rpc = (rpc + GK - 1) / GK * GK;
  chunks = (n + rpc - 1) / rpc;
  double* part = nullptr;
  hipError_t e = hipMallocAsync((void**)&part, sizeof(double) * GT * GT * npairs * chunks, stream);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(gram_bf16_kernel, dim3((unsigned)npairs, (unsigned)chunks), dim3(256), 0, stream,
                     (const __bf16*)A, n, lda, nt, rpc, part, kFlush);
  hipLaunchKernelGGL(gram_fold_kernel, dim3(GT * GT / 256, (unsigned)npairs), dim3(256), 0, stream, part,
                     (int)chunks, npairs, nt, D, G);
  hipFreeAsync(part, stream);
  return (int)hipGetLastError();
}

}  // extern "C"

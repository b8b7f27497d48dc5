// bf16 linear-model objective for CDNA4 (gfx950): the "--dtype bf16" path of the linear learners (BASELINE config
// "1M-row synthetic binary-class, LR + RandomForest selector, 1 MI355X bf16"; OpLogisticRegression.scala:46-207,
// Spark LogisticAggregator / HingeAggregator / LeastSquaresAggregator). Same contract as linear_kernels.hip
// lr_objective_kernel -- per problem f = sum_i W l(m), r = sum_i W l'(m), G = X^T (W l'(m)) with m = X V + b --
// with X stored once in bf16 (rounded once per fit: half the bytes of every pass, value AND gradient) and the
// products on the bf16 matrix cores (v_mfma_f32_32x32x16_bf16, fp32 accumulate). V and R stay (nearly) fp32: each
// is split into a bf16 high part and a bf16 residual, two MFMAs per step (~16 mantissa bits), so the objective is
// the exact objective of the bf16-rounded design matrix up to fp32 accumulation.
//
// One wave owns a 32-row tile at a time (persistent waves, no workgroup barriers in the tile loop):
//   phase A  M[32 rows, 32 problems] = X_tile . V: A = the tile's rows straight from HBM (one 16-byte load per
//            lane and k-step, all issued up front and kept in registers for phase B), B = V^T hi / lo from LDS
//   epilogue per (row, problem) in the accumulator registers: loss, derivative, weighted sums, R = W l'(m)
//   phase B  G^T[32 problems, 32 features] += R^T . X_tile per 32-feature block. A = R straight from the phase-A
//            accumulator (column = problem on the lane, rows in the registers, permuted k order:
//            cdna_hip_programming.md "an accumulator tile as the next MFMA's operand"). B needs the tile with the
//            row on the k axis: the block's two k-steps are written to a 2 KB per-wave LDS image and read back
//            transposed with ds_read_b64_tr_b16 (T10), so X is read from HBM once per pass.
// The four waves' G accumulators are summed in LDS at the end; one [dpad][32] fp32 partial per workgroup and fp64
// f / r partials per wave are summed on the host side in fixed order (ops/linear.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int PC = 32;      // problem columns per launch
constexpr int NWB = 4;      // waves per workgroup
constexpr int TR = 32;      // rows per tile
constexpr int NFB_MAX = 12; // dpad <= 384

__device__ __forceinline__ void loss_grad(int loss, float m, float y, float ysc, float* l, float* g) {
  if (loss == 0) {              // logistic (numerics of linear_kernels.hip loss_and_grad)
    const float am = fabsf(m);
    const float e = __expf(-am);
    const float u = 1.f + e;
    const float lp = (u == 1.f) ? e : __logf(u) * __fdividef(e, u - 1.f);
    *l = fmaxf(m, 0.f) + lp - y * m;
    const float inv = __builtin_amdgcn_rcpf(u);
    const float sig = m >= 0.f ? inv : e * inv;
    *g = sig - y;
  } else if (loss == 1) {       // hinge
    const float ys = 2.f * y - 1.f;
    const float marg = ys * m;
    *l = fmaxf(1.f - marg, 0.f);
    *g = marg < 1.f ? -ys : 0.f;
  } else {                      // squared, label pre-scaled per problem
    const float r = m - y / ysc;
    *l = 0.5f * r * r;
    *g = r;
  }
}

__device__ __forceinline__ bf16x4 tr_read(const __bf16* p) {
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
  return __builtin_bit_cast(bf16x4, v);
}

// LDS bytes of a workgroup: V^T hi / lo [32][dpad + 8] bf16 (re-used for the G reduction: dpad x 32 fp32 fits)
// + one 32 x 32 bf16 transpose image per wave
__host__ __device__ constexpr size_t lds_bytes(int dpad) {
  return sizeof(__bf16) * 2 * PC * (size_t)(dpad + 8) + sizeof(__bf16) * NWB * TR * 32;
}

template <bool GRAD, int NFB>
__global__ void __launch_bounds__(64 * NWB) lr_bf16_kernel(
    const __bf16* __restrict__ Xr, int64_t ldr, int64_t N, const float* __restrict__ y,
    const float* __restrict__ W, int ldw, const int32_t* __restrict__ wcol, int pc, const float* __restrict__ V,
    const float* __restrict__ bias, int loss, const float* __restrict__ yscale, double* __restrict__ f_part,
    double* __restrict__ r_part, float* __restrict__ G_part) {
  constexpr int dpad = 32 * NFB;
  constexpr int KS = 2 * NFB;                    // 16-wide k-steps
  constexpr int ldv = dpad + 8;                  // 16-byte row pad: the 32 problem rows fall on different banks
  extern __shared__ __attribute__((aligned(16))) __bf16 lds_v[];
  __bf16* vh = lds_v;
  __bf16* vl = lds_v + PC * ldv;
  for (int i = threadIdx.x; i < dpad * PC; i += blockDim.x) {     // V [dpad][32] fp32 -> V^T hi / lo
    const int f = i >> 5, p = i & 31;
    const float v = V[i];
    const __bf16 hi = (__bf16)v;
    vh[p * ldv + f] = hi;
    vl[p * ldv + f] = (__bf16)(v - (float)hi);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r31 = lane & 31, h = lane >> 5;
  const int p = r31;                             // this lane's problem column in phase A / the epilogue
  const float bp = bias[p];
  const float ysp = yscale ? yscale[p] : 1.f;
  double f_acc = 0.0, r_acc = 0.0;
  f32x16 gacc[GRAD ? NFB : 1];
#pragma unroll
  for (int b = 0; b < (GRAD ? NFB : 1); ++b) gacc[b] = f32x16{};
  // transpose image of this wave: [32 rows][32 features] bf16, 64-byte rows
  __bf16* ti = lds_v + 2 * PC * ldv + wv * TR * 32;
  // ds_read_b64_tr_b16 addresses (T10): lane 4q + pp of 16-lane group g supplies row 4 (g >> 1) + q, columns
  // 16 (g & 1) + 4 pp of the 4-row block; lane i of the group receives column 16 (g & 1) + i = r31
  const int g16 = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const __bf16* tr0 = ti + (4 * (g16 >> 1) + q) * 32 + 16 * (g16 & 1) + 4 * pp;
  const int voff = p * ldv + 8 * h;
  const int wc = wcol[p];                        // W column of problem p (dead lanes: any valid column, weigh 0)
  const int64_t ntiles = (N + TR - 1) / TR;
  const int64_t gw = (int64_t)blockIdx.x * NWB + wv, nw = (int64_t)gridDim.x * NWB;
  // Software pipeline over the wave's tiles: the next tile's rows are in flight while this tile computes. Issue
  // order per tile: this tile's W / y (the epilogue's), then the next tile's rows, so the epilogue waits only for
  // the older loads (vmcnt is in order). Plain cached loads: one load instruction takes 32 B of each of 32 rows,
  // and the other k-steps' loads find the rest of each 128-byte line in the cache.
  bf16x8 xf[KS], xn[KS];
  if (gw < ntiles) {
    const __bf16* xa = Xr + (gw * TR + r31) * ldr + 8 * h;
#pragma unroll
    for (int k = 0; k < KS; ++k) xf[k] = *reinterpret_cast<const bf16x8*>(xa + 16 * k);
  }
  for (int64_t t = gw; t < ntiles; t += nw) {
    const int64_t r0 = t * TR;
    float wv_[16], yv_[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      int64_t r = r0 + (e & 3) + 8 * (e >> 2) + 4 * h;
      r = r < N ? r : N - 1;
      yv_[e] = y[r];
      wv_[e] = W[r * ldw + wc];
    }
    const int64_t tn = t + nw;
    if (tn < ntiles) {
      const __bf16* xa = Xr + (tn * TR + r31) * ldr + 8 * h;
#pragma unroll
      for (int k = 0; k < KS; ++k) xn[k] = *reinterpret_cast<const bf16x8*>(xa + 16 * k);
    }
    __builtin_amdgcn_sched_barrier(0);
    // ---- phase A: margins of the 32 rows for the 32 problems (rows past N are zero rows of the padded copy);
    // V^T is re-read from LDS every tile (an opaque offset keeps the compiler from pinning 2 x KS fragments in
    // registers, which cost the occupancy and serialised the loads)
    int vo = voff;
    asm volatile("" : "+v"(vo));
    const __bf16* vrow_h = vh + vo;
    const __bf16* vrow_l = vl + vo;
    f32x16 ah = f32x16{}, al = f32x16{};
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const bf16x8 bh = *reinterpret_cast<const bf16x8*>(vrow_h + 16 * k);
      const bf16x8 bl = *reinterpret_cast<const bf16x8*>(vrow_l + 16 * k);
      ah = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xf[k], bh, ah, 0, 0, 0);
      al = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xf[k], bl, al, 0, 0, 0);
    }
    // ---- epilogue: register e holds row (e & 3) + 8 (e >> 2) + 4 h of the tile, problem p
    float rr[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int64_t r = r0 + (e & 3) + 8 * (e >> 2) + 4 * h;
      const bool live = r < N && p < pc;
      const float yv = yv_[e];
      const float w = live ? wv_[e] : 0.f;
      float l, g;
      loss_grad(loss, ah[e] + al[e] + bp, yv, ysp, &l, &g);
      f_acc += (double)(w * l);
      r_acc += (double)(w * g);
      rr[e] = w * g;
    }
    if constexpr (GRAD) {
      // ---- phase B: k-step s of R^T = registers 8s..8s+7; element j of lane half h is tile row
      // 16 s + 8 (j >> 2) + 4 h + (j & 3), which is what the two transposed reads deliver
      bf16x8 rh[2], rl[2];
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = rr[8 * s + j];
          const __bf16 hi = (__bf16)v;
          rh[s][j] = hi;
          rl[s][j] = (__bf16)(v - (float)hi);
        }
#pragma unroll
      for (int fb = 0; fb < NFB; ++fb) {
        // the block's two k-steps as [row][32 features]: lane (r31, h) holds features 8h..8h+7 and 16+8h..
        *reinterpret_cast<bf16x8*>(ti + r31 * 32 + 8 * h) = xf[2 * fb];
        *reinterpret_cast<bf16x8*>(ti + r31 * 32 + 16 + 8 * h) = xf[2 * fb + 1];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bf16x4 b0 = tr_read(tr0 + 16 * s * 32);
          const bf16x4 b1 = tr_read(tr0 + (16 * s + 8) * 32);
          const bf16x8 b = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
          gacc[fb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rh[s], b, gacc[fb], 0, 0, 0);
          gacc[fb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rl[s], b, gacc[fb], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < KS; ++k) xf[k] = xn[k];
  }
  // ---- partials: lanes p and p + 32 hold the two row halves of problem p
  f_acc += __shfl_xor(f_acc, 32, 64);
  r_acc += __shfl_xor(r_acc, 32, 64);
  if (h == 0) {
    f_part[gw * PC + p] = f_acc;
    r_part[gw * PC + p] = r_acc;
  }
  if constexpr (GRAD) {
    // the waves' accumulators summed in a fixed order into LDS (the V image is dead), one partial per workgroup;
    // accumulator: column = feature 32 fb + r31 on the lane, row = problem (e & 3) + 8 (e >> 2) + 4 h
    float* gs = reinterpret_cast<float*>(lds_v);
    __syncthreads();
    for (int w = 0; w < NWB; ++w) {
      if (wv == w) {
#pragma unroll
        for (int fb = 0; fb < NFB; ++fb)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            float* c = gs + (32 * fb + r31) * PC + (e & 3) + 8 * (e >> 2) + 4 * h;
            *c = (w == 0 ? 0.f : *c) + gacc[fb][e];
          }
      }
      __syncthreads();
    }
    float* gout = G_part + (int64_t)blockIdx.x * dpad * PC;
    for (int i = threadIdx.x; i < dpad * PC; i += blockDim.x) gout[i] = gs[i];
  }
}

template <bool GRAD>
int launch(int nfb, const __bf16* xr, int64_t ldr, int64_t N, const float* y, const float* W, int ldw,
           const int32_t* wcol, int pc, const float* V, const float* bias, int loss, const float* yscale, double* fp, double* rp,
           float* gp, int nblk, hipStream_t stream) {
  const dim3 g(nblk), b(64 * NWB);
  const size_t lds = lds_bytes(32 * nfb);
#define TMOG_LR_BF16_CASE(K)                                                                                   \
  case K:                                                                                                      \
    hipLaunchKernelGGL((lr_bf16_kernel<GRAD, K>), g, b, lds, stream, xr, ldr, N, y, W, ldw, wcol, pc, V, bias, \
                       loss, yscale, fp, rp, gp);                                                              \
    break;
  switch (nfb) {
    TMOG_LR_BF16_CASE(1) TMOG_LR_BF16_CASE(2) TMOG_LR_BF16_CASE(3) TMOG_LR_BF16_CASE(4)
    TMOG_LR_BF16_CASE(5) TMOG_LR_BF16_CASE(6) TMOG_LR_BF16_CASE(7) TMOG_LR_BF16_CASE(8)
    TMOG_LR_BF16_CASE(9) TMOG_LR_BF16_CASE(10) TMOG_LR_BF16_CASE(11) TMOG_LR_BF16_CASE(12)
    default: return -2;
  }
#undef TMOG_LR_BF16_CASE
  return (int)hipGetLastError();
}

template <bool GRAD>
int occupancy(int nfb) {
  int per_cu = 0;
  hipError_t e = hipErrorInvalidValue;
  const size_t lds = lds_bytes(32 * nfb);
#define TMOG_LR_BF16_OCC(K)                                                                                  \
  case K:                                                                                                    \
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lr_bf16_kernel<GRAD, K>, 64 * NWB, lds);       \
    break;
  switch (nfb) {
    TMOG_LR_BF16_OCC(1) TMOG_LR_BF16_OCC(2) TMOG_LR_BF16_OCC(3) TMOG_LR_BF16_OCC(4)
    TMOG_LR_BF16_OCC(5) TMOG_LR_BF16_OCC(6) TMOG_LR_BF16_OCC(7) TMOG_LR_BF16_OCC(8)
    TMOG_LR_BF16_OCC(9) TMOG_LR_BF16_OCC(10) TMOG_LR_BF16_OCC(11) TMOG_LR_BF16_OCC(12)
    default: return 1;
  }
#undef TMOG_LR_BF16_OCC
  return (e == hipSuccess && per_cu > 0) ? per_cu : 1;
}

}  // namespace

extern "C" {

// Workgroups per CU of a pass over a dpad-column design (ops/linear.py sizes the persistent grid with it).
int tmog_hip_lr_bf16_blocks_per_cu(int dpad, int grad) {
  if (dpad <= 0 || dpad % 32 || dpad > 32 * NFB_MAX) return 1;
  return grad ? occupancy<true>(dpad / 32) : occupancy<false>(dpad / 32);
}

// Xr: [Npad][ldr] bf16 row-major, Npad a multiple of 32 rows, columns d..dpad-1 and rows N..Npad-1 zero; dpad a
// multiple of 32 up to 384; V: [dpad][32] fp32 (zero beyond d and pc); bias / yscale / wcol: 32 entries (wcol[p]
// = the column of W [N][ldw] holding problem p's row weights: problems that share their training rows share one
// column, so a pass reads a few weight columns instead of one per problem). Partials:
// f / r [nblk * 4][32] fp64 per wave, G [nblk][dpad][32] fp32 per workgroup.
int tmog_hip_lr_bf16(const void* Xr, int64_t ldr, int64_t N, int dpad, const float* y, const float* W, int ldw,
                     const int32_t* wcol, int pc, const float* V, const float* bias, int loss, const float* yscale, int grad,
                     double* fp, double* rp, float* gp, int nblk, hipStream_t stream) {
  if (N <= 0 || nblk <= 0) return 0;
  if (dpad <= 0 || dpad % 32 || dpad > 32 * NFB_MAX || ldr < dpad || ldr % 8 || (uintptr_t)Xr % 16 || pc < 1 ||
      pc > PC || (grad && gp == nullptr))
    return -2;
  const __bf16* xr = (const __bf16*)Xr;
  return grad ? launch<true>(dpad / 32, xr, ldr, N, y, W, ldw, wcol, pc, V, bias, loss, yscale, fp, rp, gp, nblk,
                             stream)
              : launch<false>(dpad / 32, xr, ldr, N, y, W, ldw, wcol, pc, V, bias, loss, yscale, fp, rp, gp, nblk,
                              stream);
}

}  // extern "C"

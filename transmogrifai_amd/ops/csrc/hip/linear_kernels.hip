// Fused linear-model objective for CDNA4 (gfx950): one pass over X per (value, gradient) evaluation.
//
// Replaces the per-iteration work of Spark's LogisticRegression / LinearRegression / LinearSVC
// aggregators (OpLogisticRegression.scala:54-177, OpLinearRegression.scala, OpLinearSVC.scala; Spark
// LogisticAggregator / HingeAggregator / LeastSquaresAggregator: margins, loss and gradient summed
// over rows) for P problems at once -- the (config, fold) grid of the model selector, SURVEY.md K22.
//
// Per 32-row tile of X (row-major [N][d] fp32, staged once in LDS):
//   phase A  M[32, 32] = X_tile . V           v_mfma_f32_32x32x2_f32, K (= d) split across the 4 waves
//   epilogue l, dl/dm per (row, problem), R = W * dl/dm, weighted loss sums   (fused, LDS resident)
//   phase B  G[d, 32] += X_tile^T . R         v_mfma_f32_32x32x2_f32, d split across the waves
// so X is read from HBM exactly once per evaluation (the torch path reads it twice and round-trips M
// and R through HBM). Workgroups are persistent and keep their G partial in accumulator registers;
// the per-workgroup partials are summed in fp64 on the host side (ops/linear.py).
//
// LDS tile rows use a stride ds = d rounded up to 2 mod 4: the 32 rows of a phase-A operand read
// land on 32 distinct even banks and the k+1 half on the odd ones (conflict-free ds_read_b32).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int TM = 32;         // rows per tile
constexpr int PC = 32;         // problem columns per launch
constexpr int DMAX = 512;      // KSW = max phase-A k-steps (column pairs) per wave, GTW = max phase-B
                               // 32-column d tiles per wave: instantiated for d <= 256 / 384 / 512

__device__ __forceinline__ void loss_and_grad(int loss, float m, float y, float ysc, float* l, float* g) {
  if (loss == 0) {              // logistic
    const float am = fabsf(m);
    *l = fmaxf(m, 0.f) + log1pf(expf(-am)) - y * m;
    const float e = expf(-am);
    const float sig = m >= 0.f ? 1.f / (1.f + e) : e / (1.f + e);
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

template <bool GRAD, int KSW, int GTW>
__global__ void __launch_bounds__(256) lr_objective_kernel(
    const float* __restrict__ X, int64_t N, int d, int ds, const float* __restrict__ y,
    const float* __restrict__ W, int ldw, int wcol0, int P, const float* __restrict__ V,
    const float* __restrict__ bias, int loss, const float* __restrict__ yscale, double* __restrict__ f_part,
    double* __restrict__ r_part, float* __restrict__ G_part, int dpad) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* Xs = lds;                          // [TM][ds]
  float* Mp = Xs + TM * ds;                 // [4][TM][PC] phase-A partials
  float* Rs = Mp + 4 * TM * PC;             // [TM][PC]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, c32 = lane & 31;
  const int ksteps = (d + 1) >> 1;
  const int dtiles = (d + 31) >> 5;

  // phase-A B operand (V) for this wave's k-steps s = wave + 4i, held in registers for the whole kernel
  float vreg[KSW];
#pragma unroll
  for (int i = 0; i < KSW; ++i) {
    const int s = wave + 4 * i;
    const int k = 2 * s + h;
    vreg[i] = (s < ksteps && k < d) ? V[(int64_t)k * PC + c32] : 0.f;
  }
  f32x16 gacc[GTW];
#pragma unroll
  for (int c = 0; c < GTW; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) gacc[c][r] = 0.f;

  // epilogue ownership: thread t handles problem column p = t & 31, rows (t >> 5) + 8 j
  const int ep = threadIdx.x & 31;
  const int er = threadIdx.x >> 5;
  const float bp = bias[ep];
  const float ysp = yscale ? yscale[ep] : 1.f;
  double f_acc = 0.0, r_acc = 0.0;

  const int64_t ntiles = (N + TM - 1) / TM;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t r0 = tile * TM;
    const int nrows = (int)min((int64_t)TM, N - r0);
    // ---- stage the tile (contiguous in global memory) into LDS with row stride ds
    const float* src = X + r0 * (int64_t)d;
    const int n = nrows * d;
    for (int e = threadIdx.x; e < TM * ds; e += blockDim.x) {
      const int row = e / ds, col = e - row * ds;
      Xs[e] = (row < nrows && col < d) ? src[row * d + col] : 0.f;
    }
    (void)n;
    __syncthreads();

    // ---- phase A: partial margins over this wave's k-steps
    f32x16 macc;
#pragma unroll
    for (int r = 0; r < 16; ++r) macc[r] = 0.f;
#pragma unroll
    for (int i = 0; i < KSW; ++i) {
      const int s = wave + 4 * i;
      if (s < ksteps) {
        const float a = Xs[c32 * ds + 2 * s + h];
        macc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, vreg[i], macc, 0, 0, 0);
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
      Mp[(wave * TM + row) * PC + c32] = macc[r];
    }
    __syncthreads();

    // ---- fused epilogue: loss, derivative, weights
#pragma unroll
    for (int j = 0; j < TM / 8; ++j) {
      const int row = er + 8 * j;
      const int idx = row * PC + ep;
      const float m = Mp[idx] + Mp[TM * PC + idx] + Mp[2 * TM * PC + idx] + Mp[3 * TM * PC + idx] + bp;
      float rv = 0.f;
      if (row < nrows && ep < P) {
        const int64_t gr = r0 + row;
        const float w = W[gr * ldw + wcol0 + ep];
        float l, g;
        loss_and_grad(loss, m, y[gr], ysp, &l, &g);
        f_acc += (double)(l * w);
        rv = g * w;
        r_acc += (double)rv;
      }
      if (GRAD) Rs[idx] = rv;
    }
    if (GRAD) {
      __syncthreads();
      // ---- phase B: G[d-tile, p] += X_tile^T R over the 32 rows (16 k-steps of 2 rows)
#pragma unroll
      for (int c = 0; c < GTW; ++c) {
        const int dt = wave + 4 * c;
        if (dt < dtiles) {
          const int col = 32 * dt + c32;
          const bool okc = col < d;
#pragma unroll
          for (int t = 0; t < TM / 2; ++t) {
            const int row = 2 * t + h;
            const float a = okc ? Xs[row * ds + col] : 0.f;
            const float b = Rs[row * PC + c32];
            gacc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, gacc[c], 0, 0, 0);
          }
        }
      }
    }
    __syncthreads();          // Xs / Mp / Rs reused by the next tile
  }

  // ---- per-workgroup partials
  if (GRAD) {
    float* gp = G_part + (int64_t)blockIdx.x * dpad * PC;
#pragma unroll
    for (int c = 0; c < GTW; ++c) {
      const int dt = wave + 4 * c;
      if (dt < dtiles) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int dcol = 32 * dt + (r & 3) + 8 * (r >> 2) + 4 * h;
          gp[(int64_t)dcol * PC + c32] = gacc[c][r];
        }
      }
    }
  }
  double* sf = reinterpret_cast<double*>(lds);   // reuse LDS: [256] f, [256] r
  sf[threadIdx.x] = f_acc;
  sf[256 + threadIdx.x] = r_acc;
  __syncthreads();
  if (threadIdx.x < PC) {
    double fs = 0.0, rs = 0.0;
    for (int k = 0; k < 8; ++k) {
      fs += sf[threadIdx.x + 32 * k];
      rs += sf[256 + threadIdx.x + 32 * k];
    }
    f_part[(int64_t)blockIdx.x * PC + threadIdx.x] = fs;
    r_part[(int64_t)blockIdx.x * PC + threadIdx.x] = rs;
  }
}

}  // namespace

extern "C" {

// Weighted loss sums f[p] = sum_i W[i,p] l(m_ip), r[p] = sum_i W[i,p] l'(m_ip) and (grad != 0)
// G[:, p] = sum_i X[i,:] W[i,p] l'(m_ip), with m = X V + bias, for up to 32 problems (columns
// wcol0 .. wcol0+P-1 of W). V is [d][32] fp32 (zero-padded), bias / yscale are [32].
// Outputs are per-workgroup partials: f_part / r_part [nblk][32] fp64, G_part [nblk][dpad][32] fp32.
int tmog_hip_lr_objective(const float* X, int64_t N, int d, const float* y, const float* W, int ldw, int wcol0,
                          int P, const float* V, const float* bias, int loss, const float* yscale, int grad,
                          double* f_part, double* r_part, float* G_part, int nblk, hipStream_t stream) {
  if (d > DMAX || d < 1 || P > PC || P < 1 || nblk < 1) return -2;
  int ds = d;
  while (ds % 4 != 2) ++ds;
  const int dpad = ((d + 31) / 32) * 32;
  size_t lds = (size_t)(TM * ds + 5 * TM * PC) * sizeof(float);
  if (lds < 512 * sizeof(double)) lds = 512 * sizeof(double);
#define TM_LR(G, K, T)                                                                                     \
  hipLaunchKernelGGL((lr_objective_kernel<G, K, T>), dim3(nblk), dim3(256), lds, stream, X, N, d, ds, y, W, ldw, \
                     wcol0, P, V, bias, loss, yscale, f_part, r_part, G_part, dpad)
  if (grad) {
    if (d <= 256) TM_LR(true, 32, 2);
    else if (d <= 384) TM_LR(true, 48, 3);
    else TM_LR(true, 64, 4);
  } else {
    if (d <= 256) TM_LR(false, 32, 2);
    else if (d <= 384) TM_LR(false, 48, 3);
    else TM_LR(false, 64, 4);
  }
#undef TM_LR
  return (int)hipGetLastError();
}

}  // extern "C"

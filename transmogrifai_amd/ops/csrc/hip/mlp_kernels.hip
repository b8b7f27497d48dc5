// Multilayer-perceptron layer epilogues for CDNA4 (gfx950).
//
// OpMultilayerPerceptronClassifier (OpMultilayerPerceptronClassifier.scala:49-144; Spark
// MultilayerPerceptronClassifier: sigmoid hidden layers, softmax output, L-BFGS) for P problems at once --
// the (grid point x fold) jobs of the model selector, SURVEY.md K27. The layer products are plain batched
// GEMMs on hipBLASLt; these kernels fuse what follows each of them, so no layer activation makes an extra
// round trip through HBM:
//   mlp_bias_sigmoid_kernel      A[p][n][j] = sigmoid(Z[p][n][j] + b[p][j])      in place (forward)
//   mlp_sigmoid_backprop_kernel  D[p][n][j] *= A (1 - A)                         in place (backward), plus the
//                                bias gradient: fp64 column sums of the result over a fixed row slice per block
//                                (deterministic, no atomics; the host adds the block partials)
// The softmax / cross-entropy output epilogue is sparse_kernels.hip softmax_epilogue_kernel (shared with the
// multinomial logistic regression).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

namespace {

__global__ void __launch_bounds__(256) mlp_bias_sigmoid_kernel(float* __restrict__ Z, int P, int64_t N, int B,
                                                               const float* __restrict__ bias) {
  const int64_t per = N * (int64_t)B;
  const int64_t total = per * P;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = e / per;
    const int j = (int)(e % B);
    const float z = Z[e] + bias[p * B + j];
    // 1 / (1 + e^-z) through one reciprocal; saturates cleanly (e^-z = inf -> 0)
    Z[e] = __builtin_amdgcn_rcpf(1.f + __expf(-z));
  }
}

// grid (row blocks, P); thread = column j (strided by the block): the 256 threads of a row read one
// contiguous run of the row's B activations
__global__ void __launch_bounds__(256) mlp_sigmoid_backprop_kernel(float* __restrict__ D, const float* __restrict__ A,
                                                                   int64_t N, int B, int64_t rows_per_blk,
                                                                   double* __restrict__ part) {
  const int p = blockIdx.y;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_blk;
  const int64_t r1 = min(N, r0 + rows_per_blk);
  float* Dp = D + (int64_t)p * N * B;
  const float* Ap = A + (int64_t)p * N * B;
  for (int j = threadIdx.x; j < B; j += blockDim.x) {
    double acc = 0.0;
    for (int64_t r = r0; r < r1; ++r) {
      const int64_t i = r * B + j;
      const float a = Ap[i];
      const float d = Dp[i] * (a * (1.f - a));
      Dp[i] = d;
      acc += (double)d;
    }
    part[((int64_t)p * gridDim.x + blockIdx.x) * B + j] = acc;
  }
}

}  // namespace

extern "C" {

int tmog_hip_mlp_bias_sigmoid(float* Z, int P, int64_t N, int B, const float* bias, hipStream_t stream) {
  const int64_t total = N * (int64_t)B * P;
  if (total == 0) return 0;
  const unsigned nblk = (unsigned)min((total + 255) / 256, (int64_t)65536);
  hipLaunchKernelGGL(mlp_bias_sigmoid_kernel, dim3(nblk), dim3(256), 0, stream, Z, P, N, B, bias);
  return (int)hipGetLastError();
}

// part: [P][nblk][B] doubles
int tmog_hip_mlp_sigmoid_backprop(float* D, const float* A, int P, int64_t N, int B, int nblk, double* part,
                                  hipStream_t stream) {
  if (P <= 0 || B <= 0 || nblk <= 0 || nblk > 65535 || P > 65535) return -2;
  const int64_t rpb = (N + nblk - 1) / nblk;
  hipLaunchKernelGGL(mlp_sigmoid_backprop_kernel, dim3((unsigned)nblk, (unsigned)P), dim3(256), 0, stream, D, A, N,
                     B, rpb, part);
  return (int)hipGetLastError();
}

}  // extern "C"

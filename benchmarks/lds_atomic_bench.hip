// Micro-benchmark: LDS accumulate throughput on gfx950 for the histogram inner loop.
// Variants (each wave-instruction: 64 lanes, lane-distinct rows of a padded [64][129] LDS table):
//   0: ds_add_f32 (float LDS atomic)       1: ds_add_u32 (integer LDS atomic)
//   2: ds_add_u64 (packed 2x32 fixed point) 3: wave-private non-atomic read-add-write (float)
// Prints cycles per wave-instruction per CU, measured with hipEvents over a grid filling the chip.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 4096

template <int V>
__global__ void __launch_bounds__(256) k(const uint32_t* __restrict__ seed, float* out) {
  __shared__ __attribute__((aligned(16))) uint32_t tab[4][64 * 129 + 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 4 * (64 * 129 + 64); i += blockDim.x) (&tab[0][0])[i] = 0;
  __syncthreads();
  uint32_t x = seed[blockIdx.x * blockDim.x + threadIdx.x] | 1u;
  uint32_t* base = V == 3 ? tab[wave] : tab[0];
  float accf = 0.f;
  for (int it = 0; it < ITERS; ++it) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    const int bin = (x >> 8) & 63;
    uint32_t* p = base + lane * 129 + bin * 2;
    if (V == 0) {
      atomicAdd(reinterpret_cast<float*>(p), 1.0f);
      atomicAdd(reinterpret_cast<float*>(p) + 1, 0.5f);
    } else if (V == 1) {
      atomicAdd(p, 1u);
      atomicAdd(p + 1, 3u);
    } else if (V == 2) {
      unsigned long long* t64 = reinterpret_cast<unsigned long long*>(&tab[0][0]);
      atomicAdd(t64 + lane * 65 + bin, 0x0000000300000001ull);
    } else {
      float* q = reinterpret_cast<float*>(p);
      q[0] += 1.0f;
      q[1] += 0.5f;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 129; i += blockDim.x) accf += __uint_as_float(tab[0][i]);
  if (accf == 12345.f) out[0] = accf;
}

template <int V>
float run(const uint32_t* seed, float* out, int blocks) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(256), 0, 0, seed, out);
  hipEventRecord(a);
  hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(256), 0, 0, seed, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  const int blocks = 256 * 4;
  uint32_t* seed;
  float* out;
  hipMalloc(&seed, sizeof(uint32_t) * blocks * 256);
  hipMalloc(&out, 16);
  uint32_t* h = (uint32_t*)malloc(sizeof(uint32_t) * blocks * 256);
  for (int i = 0; i < blocks * 256; ++i) h[i] = 2654435761u * (i + 1);
  hipMemcpy(seed, h, sizeof(uint32_t) * blocks * 256, hipMemcpyHostToDevice);
  const double waves_per_cu = (double)blocks * 4 / 256;
  const char* names[] = {"ds_add_f32 x2", "ds_add_u32 x2", "ds_add_u64 x1", "private rmw f32 x2"};
  float t[4] = {run<0>(seed, out, blocks), run<1>(seed, out, blocks), run<2>(seed, out, blocks),
                run<3>(seed, out, blocks)};
  for (int v = 0; v < 4; ++v) {
    const double rows = waves_per_cu * ITERS;       // wave-row updates per CU
    const double cyc = t[v] * 1e-3 * 2.4e9;
    printf("{\"variant\": \"%s\", \"ms\": %.3f, \"cycles_per_wave_row_per_cu\": %.2f}\n", names[v], t[v], cyc / rows);
  }
  return 0;
}

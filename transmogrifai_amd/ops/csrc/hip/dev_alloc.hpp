// One allocation path for the grow-only device buffers of the native tree growers (tree_grow_hip.hip,
// tree_resident.hip).
//
// * A buffer that grows frees its old block first and is left EMPTY (nullptr, capacity 0) until the new
//   allocation has succeeded: a failed growth can then never leave a capacity that describes freed memory
//   (the round-4 "out of memory, then illegal address on the next learner" fault: the next call saw
//   need <= cap and launched on the freed pointer).
// * On hipErrorOutOfMemory the process-wide handler runs once and the allocation is retried. The Python
//   side registers a handler that returns torch's cached-but-unused blocks to the device
//   (torch.cuda.empty_cache), so the native buffers and torch's caching allocator draw on one budget
//   instead of the native growth failing while torch holds free cache.
// * Test hook: tmog_hip_fail_alloc(n) makes the n-th native allocation from now fail with
//   hipErrorOutOfMemory (without the handler), to prove a failed growth leaves a usable slot.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>

namespace tmog {

inline std::atomic<void (*)()> g_oom_handler{nullptr};
inline std::atomic<long> g_fail_at{0};

inline hipError_t dev_malloc_async(void** p, size_t bytes, hipStream_t s) {
  *p = nullptr;
  if (g_fail_at.load(std::memory_order_relaxed) > 0 && g_fail_at.fetch_sub(1) == 1) return hipErrorOutOfMemory;
  hipError_t e = hipMallocAsync(p, bytes, s);
  if (e == hipErrorOutOfMemory) {
    (void)hipGetLastError();                 // not sticky: clear it before the retry
    if (auto h = g_oom_handler.load()) {
      h();
      e = hipMallocAsync(p, bytes, s);
    }
  }
  if (e != hipSuccess) *p = nullptr;
  return e;
}

// Grow ``p`` (capacity ``cap`` bytes) to hold ``need`` bytes, allocating ``new_cap`` >= need.
inline void grow_device(uint8_t*& p, size_t& cap, size_t need, size_t new_cap, hipStream_t s) {
  if (need <= cap && p != nullptr) return;
  if (p) {
    hipError_t ef = hipFreeAsync(p, s);
    p = nullptr;
    cap = 0;
    if (ef != hipSuccess) throw std::runtime_error(std::string("hipFreeAsync: ") + hipGetErrorString(ef));
  }
  void* q = nullptr;
  hipError_t e = dev_malloc_async(&q, new_cap, s);
  if (e != hipSuccess)
    throw std::runtime_error(std::string("hipMallocAsync(") + std::to_string(new_cap) + " B): " +
                             hipGetErrorString(e));
  p = static_cast<uint8_t*>(q);
  cap = new_cap;
}

}  // namespace tmog

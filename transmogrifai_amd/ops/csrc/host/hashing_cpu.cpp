// Host string hashing: bit-exact murmur3_x86_32 as used by Spark MLlib HashingTF
// (Murmur3_x86_32.hashUnsafeBytes with seed 42, including Spark's per-byte tail mixing of
// *signed* bytes), plus a term-frequency scatter. Reference call sites:
// OPCollectionHashingVectorizer.scala:204-208 and HashingFun.hash:244-272.
#include <cstdint>
#include <cstring>
#include <omp.h>

static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

static inline uint32_t mix_k1(uint32_t k1) {
  k1 *= 0xcc9e2d51u;
  k1 = rotl32(k1, 15);
  k1 *= 0x1b873593u;
  return k1;
}

static inline uint32_t mix_h1(uint32_t h1, uint32_t k1) {
  h1 ^= k1;
  h1 = rotl32(h1, 13);
  h1 = h1 * 5u + 0xe6546b64u;
  return h1;
}

static inline uint32_t fmix(uint32_t h1, uint32_t len) {
  h1 ^= len;
  h1 ^= h1 >> 16;
  h1 *= 0x85ebca6bu;
  h1 ^= h1 >> 13;
  h1 *= 0xc2b2ae35u;
  h1 ^= h1 >> 16;
  return h1;
}

static inline int32_t spark_murmur3(const uint8_t* p, int64_t len, int32_t seed) {
  uint32_t h1 = (uint32_t)seed;
  const int64_t aligned = len - len % 4;
  for (int64_t i = 0; i < aligned; i += 4) {
    uint32_t w;
    std::memcpy(&w, p + i, 4);  // little-endian getInt
    h1 = mix_h1(h1, mix_k1(w));
  }
  for (int64_t i = aligned; i < len; ++i) {
    const int32_t half = (int32_t)(int8_t)p[i];  // Platform.getByte is signed
    h1 = mix_h1(h1, mix_k1((uint32_t)half));
  }
  return (int32_t)fmix(h1, (uint32_t)len);
}

extern "C" {

int tmog_murmur3_batch(const uint8_t* bytes, const int64_t* offsets, int64_t n, int32_t seed, int32_t* out) {
#pragma omp parallel for schedule(static) if (n > 4096)
  for (int64_t i = 0; i < n; ++i) out[i] = spark_murmur3(bytes + offsets[i], offsets[i + 1] - offsets[i], seed);
  return 0;
}

// nonNegativeMod(hash, num_features) per term.
int tmog_hash_index_batch(const uint8_t* bytes, const int64_t* offsets, int64_t n, int32_t seed,
                          int32_t num_features, int32_t* out) {
#pragma omp parallel for schedule(static) if (n > 4096)
  for (int64_t i = 0; i < n; ++i) {
    const int32_t h = spark_murmur3(bytes + offsets[i], offsets[i + 1] - offsets[i], seed);
    int32_t m = h % num_features;
    out[i] = m < 0 ? m + num_features : m;
  }
  return 0;
}

}  // extern "C"

// Batch string cleaning and first-appearance grouping for the text statistics of the vectorizers
// (SmartTextVectorizer / pivot fits over dictionary vocabularies of 10^5..10^6 distinct strings).
//
// tmog_clean_ascii_lens: TextUtils.cleanString (lower-case, punctuation -> ' ', split on runs of ' ', capitalise
// each part, concatenate) of every ASCII string of a batch, each written in place of its input bytes (a cleaned
// string is never longer), in parallel over string ranges; strings holding any byte >= 0x80 are flagged and left
// to the Python implementation (Unicode case mapping can change lengths).
// tmog_first_ids: id of every string in order of first appearance (identical bytes -> identical id). Large
// batches: 64-bit hashes in parallel, indices bucketed by hash shard (stable, so ascending inside a shard), each
// shard deduplicated by its own open-addressing table in parallel (representative = first index of the value),
// then one ordered pass numbers the representatives -- the same ids as the serial map.
#include <omp.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string_view>
#include <unordered_map>
#include <vector>

namespace {

inline bool is_punct(uint8_t c) {
  // !"#$%&'()*+,-./:;<=>?@[\]^_`{|}~
  return (c >= 33 && c <= 47) || (c >= 58 && c <= 64) || (c >= 91 && c <= 96) || (c >= 123 && c <= 126);
}

inline uint64_t hash_bytes(const uint8_t* p, size_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (n * 0xC2B2AE3D27D4EB4Full);
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    std::memcpy(&w, p + i, 8);
    h = (h ^ (w * 0x87C37B91114253D5ull)) * 0x4CF5AD432745937Full;
    h ^= h >> 29;
  }
  uint64_t t = 0;
  for (size_t k = 0; i + k < n; ++k) t |= (uint64_t)p[i + k] << (8 * k);
  h = (h ^ (t * 0x87C37B91114253D5ull)) * 0x4CF5AD432745937Full;
  h ^= h >> 32;
  h *= 0xD6E8FEB86659FD93ull;
  return h ^ (h >> 32);
}

int64_t first_ids_serial(const uint8_t* buf, const int64_t* starts, const int64_t* ends, int64_t n, int64_t* ids) {
  std::unordered_map<std::string_view, int64_t> seen;
  seen.reserve((size_t)n * 2 + 16);
  for (int64_t i = 0; i < n; ++i) {
    std::string_view s(reinterpret_cast<const char*>(buf + starts[i]), (size_t)(ends[i] - starts[i]));
    auto it = seen.emplace(s, (int64_t)seen.size()).first;
    ids[i] = it->second;
  }
  return (int64_t)seen.size();
}

}  // namespace

extern "C" {

// out must hold offs[n] bytes: cleaned string i is written at out[offs[i], offs[i] + lens[i]); fallback n bytes
// (1 = not ASCII, not cleaned, lens[i] = 0)
void tmog_clean_ascii_lens(const uint8_t* buf, const int64_t* offs, int64_t n, uint8_t* out, int64_t* lens,
                           uint8_t* fallback) {
  const int nt = n > 4096 ? omp_get_max_threads() : 1;
#pragma omp parallel for num_threads(nt) schedule(static, 1024)
  for (int64_t i = 0; i < n; ++i) {
    const int64_t a = offs[i], b = offs[i + 1];
    bool ascii = true;
    for (int64_t p = a; p < b; ++p) ascii &= buf[p] < 0x80;
    fallback[i] = ascii ? 0 : 1;
    int64_t w = a;
    if (ascii) {
      bool start = true;   // next kept character begins a part
      for (int64_t p = a; p < b; ++p) {
        uint8_t c = buf[p];
        if (c >= 'A' && c <= 'Z') c = (uint8_t)(c - 'A' + 'a');
        if (c == ' ' || is_punct(c)) {
          start = true;
          continue;
        }
        if (start && c >= 'a' && c <= 'z') c = (uint8_t)(c - 'a' + 'A');
        start = false;
        out[w++] = c;
      }
    }
    lens[i] = w - a;
  }
}

// ids[i] = first-appearance id of string i = bytes [starts[i], ends[i]) of buf; returns the number of
// distinct strings
int64_t tmog_first_ids(const uint8_t* buf, const int64_t* starts, const int64_t* ends, int64_t n, int64_t* ids) {
  const int T = omp_get_max_threads();
  if (n < 65536 || T < 2) return first_ids_serial(buf, starts, ends, n, ids);
  constexpr int kShardBits = 8, kShards = 1 << kShardBits;
  std::vector<uint64_t> h((size_t)n);
  std::vector<int64_t> order((size_t)n), rep((size_t)n);
  std::vector<int64_t> cnt((size_t)T * kShards, 0), shard_off(kShards + 1, 0);
  auto len = [&](int64_t i) { return (size_t)(ends[i] - starts[i]); };
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num(), TT = omp_get_num_threads();   // the team may be smaller than T
    const int64_t lo = n * t / TT, hi = n * (t + 1) / TT;
    int64_t* c = cnt.data() + (size_t)t * kShards;
    for (int64_t i = lo; i < hi; ++i) {
      h[i] = hash_bytes(buf + starts[i], len(i));
      ++c[h[i] >> (64 - kShardBits)];
    }
#pragma omp barrier
#pragma omp single
    {
      int64_t run = 0;
      for (int sh = 0; sh < kShards; ++sh) {
        shard_off[sh] = run;
        for (int u = 0; u < TT; ++u) {
          const int64_t x = cnt[(size_t)u * kShards + sh];
          cnt[(size_t)u * kShards + sh] = run;   // this thread's first slot in the shard
          run += x;
        }
      }
      shard_off[kShards] = run;
    }
    for (int64_t i = lo; i < hi; ++i) order[c[h[i] >> (64 - kShardBits)]++] = i;   // stable: ascending per shard
#pragma omp barrier
    std::vector<int64_t> table;
#pragma omp for schedule(dynamic, 4)
    for (int sh = 0; sh < kShards; ++sh) {
      const int64_t a = shard_off[sh], b = shard_off[sh + 1];
      if (a == b) continue;
      size_t cap = 16;
      while (cap < (size_t)(b - a) * 2) cap <<= 1;
      table.assign(cap, -1);
      const size_t mask = cap - 1;
      for (int64_t k = a; k < b; ++k) {
        const int64_t i = order[k];
        size_t slot = (size_t)h[i] & mask;
        while (true) {
          const int64_t j = table[slot];
          if (j < 0) {
            table[slot] = i;
            rep[i] = i;
            break;
          }
          if (h[j] == h[i] && len(j) == len(i) && std::memcmp(buf + starts[j], buf + starts[i], len(i)) == 0) {
            rep[i] = j;          // j < i: the shard is walked in index order
            break;
          }
          slot = (slot + 1) & mask;
        }
      }
    }
  }
  int64_t k = 0;
  for (int64_t i = 0; i < n; ++i) ids[i] = rep[i] == i ? k++ : ids[rep[i]];
  return k;
}

}  // extern "C"

// Batch string cleaning and first-appearance grouping for the text statistics of the vectorizers
// (SmartTextVectorizer / pivot fits over dictionary vocabularies of 10^5..10^6 distinct strings).
//
// tmog_clean_ascii: TextUtils.cleanString (lower-case, punctuation -> ' ', split on runs of ' ', capitalise
// each part, concatenate) of every ASCII string of a batch; strings holding any byte >= 0x80 are flagged
// and left to the Python implementation (Unicode case mapping can change lengths).
// tmog_first_ids: id of every string in order of first appearance (identical bytes -> identical id).
#include <cstdint>
#include <cstring>
#include <string_view>
#include <unordered_map>

namespace {

inline bool is_punct(uint8_t c) {
  // !"#$%&'()*+,-./:;<=>?@[\]^_`{|}~
  return (c >= 33 && c <= 47) || (c >= 58 && c <= 64) || (c >= 91 && c <= 96) || (c >= 123 && c <= 126);
}

}  // namespace

extern "C" {

// out must hold offs[n] bytes; out_offs n + 1 entries; fallback n bytes (1 = not ASCII, not cleaned)
void tmog_clean_ascii(const uint8_t* buf, const int64_t* offs, int64_t n, uint8_t* out, int64_t* out_offs,
                      uint8_t* fallback) {
  int64_t w = 0;
  out_offs[0] = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t a = offs[i], b = offs[i + 1];
    bool ascii = true;
    for (int64_t p = a; p < b; ++p) ascii &= buf[p] < 0x80;
    fallback[i] = ascii ? 0 : 1;
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
    out_offs[i + 1] = w;
  }
}

// ids[i] = first-appearance id of string i = bytes [starts[i], ends[i]) of buf; returns the number of
// distinct strings
int64_t tmog_first_ids(const uint8_t* buf, const int64_t* starts, const int64_t* ends, int64_t n, int64_t* ids) {
  std::unordered_map<std::string_view, int64_t> seen;
  seen.reserve((size_t)n * 2 + 16);
  for (int64_t i = 0; i < n; ++i) {
    std::string_view s(reinterpret_cast<const char*>(buf + starts[i]), (size_t)(ends[i] - starts[i]));
    auto it = seen.emplace(s, (int64_t)seen.size()).first;
    ids[i] = it->second;
  }
  return (int64_t)seen.size();
}

}  // extern "C"

// Native multithreaded text tokenizer: the word rules of the default
// LuceneTextAnalyzer / StandardAnalyzer path used by TextTokenizer.tokenizeString
// (core/.../TextTokenizer.scala:160-188, core/.../utils/text/LuceneTextAnalyzer.scala:160-166):
// letter-led words (letters may be joined by ' or .), digit-led numbers (digits joined by . or ,),
// underscore-led words, StandardTokenizer split of CJK tokens (ideographs and hiragana one token each, katakana
// and hangul runs words), lowercase, 255-char cap, English stop
// words, minimum token length.
//
// The executable spec is transmogrifai_amd/utils/text.py:analyze; the character classes and the
// lowercase map come from unicode_tables.inc, generated from that interpreter's own `re`/`str`
// semantics, so the two agree code point for code point on the BMP. Strings holding a code point
// whose lowercase is context-dependent or multi-char, or one outside the BMP, are flagged and
// tokenized by the Python path instead (flag[i] = 1, no tokens emitted).
//
// Output is a flat token list (UTF-8 bytes + token end offsets) and a per-string token count, the
// layout the HIP hashing-TF kernels consume directly (text_kernels.hip).
#include <omp.h>

#include <cstdint>
#include <cstring>
#include <functional>
#include <string>
#include <unordered_set>
#include <vector>

namespace {

#include "unicode_tables.inc"

struct Tables {
  uint8_t cls[65536];
  uint16_t lower[65536];
  Tables() {
    const int nr = sizeof(kClassRuns) / sizeof(kClassRuns[0]);
    for (int r = 0; r < nr; ++r) {
      const uint32_t a = kClassRuns[r][0], b = r + 1 < nr ? kClassRuns[r + 1][0] : 65536u;
      for (uint32_t c = a; c < b; ++c) cls[c] = (uint8_t)kClassRuns[r][1];
    }
    for (uint32_t c = 0; c < 65536; ++c) lower[c] = (uint16_t)c;
    for (const auto& p : kLowerPairs) lower[p[0]] = p[1];
  }
};
const Tables& tables() {
  static const Tables t;
  return t;
}

constexpr uint8_t kWord = 1, kDigit = 2, kFallback = 4, kCjk = 8, kMark = 16;

const char* kStop[] = {
    "i", "me", "my", "myself", "we", "our", "ours", "ourselves", "you", "your", "yours", "yourself", "yourselves",
    "he", "him", "his", "himself", "she", "her", "hers", "herself", "it", "its", "itself", "they", "them", "their",
    "theirs", "themselves", "what", "which", "who", "whom", "this", "that", "these", "those", "am", "is", "are",
    "was", "were", "be", "been", "being", "have", "has", "had", "having", "do", "does", "did", "doing", "would",
    "should", "could", "ought", "i'm", "you're", "he's", "she's", "it's", "we're", "they're", "i've", "you've",
    "we've", "they've", "i'd", "you'd", "he'd", "she'd", "we'd", "they'd", "i'll", "you'll", "he'll", "she'll",
    "we'll", "they'll", "isn't", "aren't", "wasn't", "weren't", "hasn't", "haven't", "hadn't", "doesn't", "don't",
    "didn't", "won't", "wouldn't", "shan't", "shouldn't", "can't", "cannot", "couldn't", "mustn't", "let's",
    "that's", "who's", "what's", "here's", "there's", "when's", "where's", "why's", "how's", "a", "an", "the",
    "and", "but", "if", "or", "because", "as", "until", "while", "of", "at", "by", "for", "with", "about",
    "against", "between", "into", "through", "during", "before", "after", "above", "below", "to", "from", "up",
    "down", "in", "out", "on", "off", "over", "under", "again", "further", "then", "once", "here", "there", "when",
    "where", "why", "how", "all", "any", "both", "each", "few", "more", "most", "other", "some", "such", "no", "nor",
    "not", "only", "own", "same", "so", "than", "too", "very"};

const std::unordered_set<std::string>& stopwords() {
  static const std::unordered_set<std::string> s(std::begin(kStop), std::end(kStop));
  return s;
}

// Decode UTF-8 into BMP code points; false on a 4-byte sequence or malformed input.
bool decode(const uint8_t* p, int64_t n, std::vector<uint16_t>& cps) {
  cps.clear();
  for (int64_t i = 0; i < n;) {
    const uint8_t b = p[i];
    if (b < 0x80) {
      cps.push_back(b);
      i += 1;
    } else if ((b & 0xE0) == 0xC0 && i + 1 < n) {
      cps.push_back((uint16_t)(((b & 0x1F) << 6) | (p[i + 1] & 0x3F)));
      i += 2;
    } else if ((b & 0xF0) == 0xE0 && i + 2 < n) {
      cps.push_back((uint16_t)(((b & 0x0F) << 12) | ((p[i + 1] & 0x3F) << 6) | (p[i + 2] & 0x3F)));
      i += 3;
    } else {
      return false;
    }
  }
  return true;
}

inline void put_utf8(std::vector<uint8_t>& out, uint16_t c) {
  if (c < 0x80) {
    out.push_back((uint8_t)c);
  } else if (c < 0x800) {
    out.push_back((uint8_t)(0xC0 | (c >> 6)));
    out.push_back((uint8_t)(0x80 | (c & 0x3F)));
  } else {
    out.push_back((uint8_t)(0xE0 | (c >> 12)));
    out.push_back((uint8_t)(0x80 | ((c >> 6) & 0x3F)));
    out.push_back((uint8_t)(0x80 | (c & 0x3F)));
  }
}

struct Sink {
  std::vector<uint8_t> bytes;
  std::vector<int64_t> ends;  // end offset of every token inside `bytes`
};

// Tokenize one string; returns the number of tokens appended, or -1 if it needs the Python path.
int64_t tokenize_one(const uint8_t* p, int64_t n, bool lowercase, int min_len, bool use_stop,
                     std::vector<uint16_t>& cps, std::string& scratch, Sink& sink) {
  const Tables& T = tables();
  if (!decode(p, n, cps)) return -1;
  for (uint16_t c : cps)
    if (T.cls[c] & kFallback) return -1;
  if (lowercase)
    for (auto& c : cps) c = T.lower[c];
  const int64_t L = (int64_t)cps.size();
  int64_t emitted = 0;
  // CJK script of a code point (utils/text.py cjk_class: the kCjk ranges): 1 Han, 2 hiragana, 3 katakana, 4 hangul
  auto cjk_cls = [](uint32_t o) -> int {
    if ((o >= 0x4E00 && o <= 0x9FFF) || (o >= 0x3400 && o <= 0x4DBF)) return 1;
    if (o >= 0x3040 && o <= 0x309F) return 2;
    if (o >= 0x30A0 && o <= 0x30FF) return 3;
    if (o >= 0xAC00 && o <= 0xD7AF) return 4;
    return 0;
  };
  auto emit_word = [&](int64_t i, int64_t j) {
    if (j - i > 255 || j - i < min_len) return;
    const size_t start = sink.bytes.size();
    for (int64_t k = i; k < j; ++k) put_utf8(sink.bytes, T.lower[cps[k]]);
    bool stop = false;
    if (use_stop) {
      scratch.assign((const char*)sink.bytes.data() + start, sink.bytes.size() - start);
      stop = stopwords().count(scratch) != 0;
    }
    if (stop) {
      sink.bytes.resize(start);
    } else {
      sink.ends.push_back((int64_t)sink.bytes.size());
      ++emitted;
    }
  };
  // word rules over cps[lo, hi); a word holding CJK characters is split as StandardTokenizer does (every
  // ideograph and hiragana a token, katakana / hangul runs words, the other characters scanned again)
  std::function<void(int64_t, int64_t)> scan = [&](int64_t lo, int64_t hi) {
    auto is_w = [&](int64_t i) { return i < hi && (T.cls[cps[i]] & kWord); };
    // continues a word: a word character or a combining mark / ZWJ / ZWNJ (UAX#29 Extend)
    auto is_wc = [&](int64_t i) { return i < hi && (T.cls[cps[i]] & (kWord | kMark)); };
    auto is_d = [&](int64_t i) { return i < hi && (T.cls[cps[i]] & kDigit); };
    auto is_letter = [&](int64_t i) { return is_w(i) && !is_d(i) && cps[i] != '_'; };
    int64_t i = lo;
    while (i < hi) {
      int64_t j;
      if (is_letter(i)) {
        j = i + 1;
        for (;;) {
          if (is_wc(j)) ++j;
          else if (j < hi && (cps[j] == '\'' || cps[j] == '.') && is_letter(j + 1)) ++j;
          else break;
        }
      } else if (is_d(i)) {
        j = i + 1;
        for (;;) {
          if (is_wc(j)) ++j;
          else if (j < hi && (cps[j] == '.' || cps[j] == ',') && is_d(j + 1)) ++j;
          else break;
        }
      } else if (cps[i] == '_') {
        j = i + 1;
        while (is_wc(j)) ++j;
      } else {
        ++i;
        continue;
      }
      bool cjk = false;
      for (int64_t k = i; k < j; ++k) cjk |= (T.cls[cps[k]] & kCjk) != 0;
      if (cjk) {
        int64_t k = i;
        while (k < j) {
          const int c = cjk_cls(cps[k]);
          int64_t e = k + 1;
          if (c == 3 || c == 4) {
            while (e < j && cjk_cls(cps[e]) == c) ++e;
          } else if (c == 0) {
            while (e < j && cjk_cls(cps[e]) == 0) ++e;
          }
          if (c == 0) {
            scan(k, e);
          } else if (e - k >= min_len && e - k <= 255) {   // not lowercased beyond the string-level pass
            for (int64_t q = k; q < e; ++q) put_utf8(sink.bytes, cps[q]);
            sink.ends.push_back((int64_t)sink.bytes.size());
            ++emitted;
          }
          k = e;
        }
      } else {
        emit_word(i, j);
      }
      i = j;
    }
  };
  scan(0, L);
  return emitted;
}

struct Result {
  std::vector<uint8_t> bytes;
  std::vector<int64_t> tok_offs;  // T + 1
  std::vector<int64_t> row_ptr;   // n + 1
  std::vector<uint8_t> fallback;  // n
};

}  // namespace

extern "C" {

// Tokenize n UTF-8 strings (bytes[offs[i]:offs[i+1]]). Returns an opaque handle; read the sizes with
// tmog_tok_sizes, copy out with tmog_tok_copy, release with tmog_tok_free.
void* tmog_tok_run(const uint8_t* bytes, const int64_t* offs, int64_t n, int32_t lowercase, int32_t min_len,
                   int32_t use_stop) {
  tables();
  stopwords();
  auto* R = new Result();
  const int nt = n > 2048 ? omp_get_max_threads() : 1;
  std::vector<Sink> sinks(nt);
  std::vector<int64_t> counts(n);
  R->fallback.assign(n, 0);
#pragma omp parallel num_threads(nt)
  {
    const int t = omp_get_thread_num(), T = omp_get_num_threads();
    const int64_t a = n * t / T, b = n * (t + 1) / T;
    std::vector<uint16_t> cps;
    std::string scratch;
    for (int64_t i = a; i < b; ++i) {
      const int64_t c = tokenize_one(bytes + offs[i], offs[i + 1] - offs[i], lowercase != 0, min_len, use_stop != 0,
                                     cps, scratch, sinks[t]);
      if (c < 0) {
        R->fallback[i] = 1;
        counts[i] = 0;
      } else {
        counts[i] = c;
      }
    }
  }
  int64_t total_b = 0, total_t = 0;
  for (auto& s : sinks) total_b += (int64_t)s.bytes.size(), total_t += (int64_t)s.ends.size();
  R->bytes.resize(total_b);
  R->tok_offs.resize(total_t + 1);
  R->tok_offs[0] = 0;
  int64_t bo = 0, to = 0;
  for (auto& s : sinks) {
    if (!s.bytes.empty()) std::memcpy(R->bytes.data() + bo, s.bytes.data(), s.bytes.size());
    for (size_t k = 0; k < s.ends.size(); ++k) R->tok_offs[to + 1 + k] = bo + s.ends[k];
    bo += (int64_t)s.bytes.size();
    to += (int64_t)s.ends.size();
  }
  R->row_ptr.resize(n + 1);
  R->row_ptr[0] = 0;
  for (int64_t i = 0; i < n; ++i) R->row_ptr[i + 1] = R->row_ptr[i] + counts[i];
  return R;
}

void tmog_tok_sizes(void* h, int64_t* n_tokens, int64_t* n_bytes) {
  auto* R = (Result*)h;
  *n_tokens = (int64_t)R->tok_offs.size() - 1;
  *n_bytes = (int64_t)R->bytes.size();
}

void tmog_tok_copy(void* h, uint8_t* bytes, int64_t* tok_offs, int64_t* row_ptr, uint8_t* fallback) {
  auto* R = (Result*)h;
  if (!R->bytes.empty()) std::memcpy(bytes, R->bytes.data(), R->bytes.size());
  std::memcpy(tok_offs, R->tok_offs.data(), R->tok_offs.size() * sizeof(int64_t));
  std::memcpy(row_ptr, R->row_ptr.data(), R->row_ptr.size() * sizeof(int64_t));
  if (!R->fallback.empty()) std::memcpy(fallback, R->fallback.data(), R->fallback.size());
}

void tmog_tok_free(void* h) { delete (Result*)h; }

}  // extern "C"

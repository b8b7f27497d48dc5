// Bounded-bin streaming histogram (Ben-Haim & Tom-Tov), host C++.
//
// Parity target: the reference's Java StreamingHistogram + builder
// (utils/src/main/java/com/salesforce/op/utils/stats/StreamingHistogram.java:30-299) used by
// RawFeatureFilter-style summaries: points first land in a sorted spool (exact counts), the spool is
// drained into at most max_bins centroids in key order, and every overflow merges the two closest
// centroids into their count-weighted mean. `sum(b)` is the paper's trapezoid estimate of the number
// of points <= b. Exposed through a small C ABI (handles) for ctypes.
#include <cstdint>
#include <cmath>
#include <iterator>
#include <map>

namespace {

struct Hist {
  int max_bins;
  int max_spool;
  int64_t round;
  std::map<double, int64_t> bin;
  std::map<double, int64_t> spool;

  void flush() {
    for (const auto& kv : spool) {
      bin[kv.first] += kv.second;
      if ((int)bin.size() > max_bins) {
        auto it = bin.begin();
        auto best = it;
        double smallest = INFINITY;
        for (auto nx = std::next(it); nx != bin.end(); ++it, ++nx) {
          const double d = nx->first - it->first;
          if (d < smallest) {
            smallest = d;
            best = it;
          }
        }
        auto second = std::next(best);
        const double q1 = best->first, q2 = second->first;
        const int64_t k1 = best->second, k2 = second->second;
        bin.erase(best);
        bin.erase(second);
        bin[(q1 * k1 + q2 * k2) / (double)(k1 + k2)] += k1 + k2;
      }
    }
    spool.clear();
  }

  void update(double p, int64_t m) {
    if (round > 1) {
      const int64_t lp = (int64_t)p;
      const int64_t d = lp % round;
      if (d > 0) p = (double)(lp + (round - d));
    }
    spool[p] += m;
    if ((int)spool.size() > max_spool) flush();
  }

  double sum(double b) const {
    auto next = bin.upper_bound(b);
    double s = 0;
    if (next == bin.end()) {
      for (const auto& kv : bin) s += (double)kv.second;
      return s;
    }
    if (next == bin.begin()) return 0.0;
    auto pi = std::prev(next);
    const double w = (b - pi->first) / (next->first - pi->first);
    const double mb = pi->second + (next->second - pi->second) * w;
    s += (pi->second + mb) * w / 2;
    s += pi->second / 2.0;
    for (auto it = bin.begin(); it != pi; ++it) s += (double)it->second;
    return s;
  }
};

}  // namespace

extern "C" {

void* tmog_shist_new(int max_bins, int max_spool, int64_t round_to) {
  Hist* h = new Hist();
  h->max_bins = max_bins < 2 ? 2 : max_bins;
  h->max_spool = max_spool < 0 ? 0 : max_spool;
  h->round = round_to < 1 ? 1 : round_to;
  return h;
}

void tmog_shist_free(void* h) { delete static_cast<Hist*>(h); }

void tmog_shist_update(void* h, const double* p, const int64_t* m, int64_t n) {
  Hist* H = static_cast<Hist*>(h);
  for (int64_t i = 0; i < n; ++i)
    if (!std::isnan(p[i])) H->update(p[i], m ? m[i] : 1);
}

void tmog_shist_flush(void* h) { static_cast<Hist*>(h)->flush(); }

// merge = update with the other histogram's (flushed) centroids
void tmog_shist_merge(void* h, void* other) {
  Hist* O = static_cast<Hist*>(other);
  O->flush();
  Hist* H = static_cast<Hist*>(h);
  for (const auto& kv : O->bin) H->update(kv.first, kv.second);
}

int64_t tmog_shist_size(void* h) {
  Hist* H = static_cast<Hist*>(h);
  H->flush();
  return (int64_t)H->bin.size();
}

void tmog_shist_bins(void* h, double* points, int64_t* counts) {
  Hist* H = static_cast<Hist*>(h);
  H->flush();
  int64_t i = 0;
  for (const auto& kv : H->bin) {
    points[i] = kv.first;
    counts[i] = kv.second;
    ++i;
  }
}

double tmog_shist_sum(void* h, double b) {
  Hist* H = static_cast<Hist*>(h);
  H->flush();
  return H->sum(b);
}

}  // extern "C"

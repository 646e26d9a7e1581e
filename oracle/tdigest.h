// ORACLE / TEST INFRASTRUCTURE ONLY — never linked into the product (pixie_amd/).
//
// CPU restatement of the "merging digest" t-digest that QuantilesUDA wraps
// (src/carnot/funcs/builtins/math_sketches.h:33-82: `TDigest(1000)`, `add`, `merge`,
// `quantile` x7).  The implementation itself is the third-party header `tdigest/tdigest.h`
// from github.com/pixie-io/tdigest @ 85e0f70092460e60236821db4c25143768d3da12
// (bazel/repository_locations.bzl:243-247, bazel/external/tdigest.BUILD:25-37), a fork of
// derrickburns/tdigest.  It is NOT vendored in /root/reference and not present in this
// container, so this file restates the published algorithm:
//   * compression delta; maxProcessed = 2*ceil(delta), maxUnprocessed = 8*ceil(delta);
//   * add(x): NaN ignored, append to unprocessed, process() when dirty
//     (processed > maxProcessed || unprocessed > maxUnprocessed);
//   * process(): sort unprocessed by mean, merge with processed, greedy merge while
//     wSoFar + w <= wLimit with wLimit = W * integratedQ(k1 + 1),
//     k1 = integratedLocation(wSoFar / W); centroid add is the incremental mean update;
//   * merge(other): k-way merge of processed centroids + append unprocessed, process if dirty;
//   * quantile(q): process if anything is unprocessed, then interpolate on cumulative
//     midpoints with the min/max tails (including the upstream last-tail expression).
// Pinned against the reference's own known answers (math_sketches_test.cc:30-70), see
// tests/test_oracle_golden.py.  Beyond those two vectors the behaviour is "parity unpinned"
//  and device parity uses the rank-error bound stated in DESIGN.md.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <limits>
#include <queue>
#include <vector>

namespace oracle {

struct Centroid {
  double mean = 0;
  double weight = 0;
  Centroid() = default;
  Centroid(double m, double w) : mean(m), weight(w) {}
  void add(const Centroid& c) {
    if (weight != 0.0) {
      weight += c.weight;
      mean += c.weight * (c.mean - mean) / weight;
    } else {
      weight = c.weight;
      mean = c.mean;
    }
  }
};

class TDigest {
 public:
  static constexpr size_t kHighWater = 40000;

  explicit TDigest(double compression = 1000)
      : compression_(compression),
        max_processed_(static_cast<size_t>(2 * std::ceil(compression))),
        max_unprocessed_(static_cast<size_t>(8 * std::ceil(compression))) {}

  void add(double x) { add(x, 1.0); }
  bool add(double x, double w) {
    if (std::isnan(x)) return false;
    unprocessed_.emplace_back(x, w);
    unprocessed_weight_ += w;
    ProcessIfNecessary();
    return true;
  }

  void merge(const TDigest* other) {
    std::vector<const TDigest*> batch{other};
    // Single-digest form of add(iter, end): one batch regardless of kHighWater.
    MergeProcessed(batch);
    MergeUnprocessed(batch);
    ProcessIfNecessary();
    UpdateCumulative();
  }

  double quantile(double q) {
    if (HaveUnprocessed() || IsDirty()) Process();
    return QuantileProcessed(q);
  }

  // The digest one rank ships for a group of more than 8 * delta values (pxg export v2,
  // DESIGN.md §5): every value added unprocessed and ONE process() over them, i.e. the same
  // single-pass digest the device emulates for one group on one node.
  static TDigest FromValuesOnce(const std::vector<double>& v, double compression = 1000) {
    TDigest d = Unprocessed(v, compression);
    d.Process();
    return d;
  }
  // A digest holding `v` as unprocessed centroids of weight 1 (NaN skipped, as add() does):
  // a rank's raw contribution of <= 8 * delta values.
  static TDigest Unprocessed(const std::vector<double>& v, double compression = 1000) {
    TDigest d(compression);
    for (double x : v)
      if (!std::isnan(x)) {
        d.unprocessed_.emplace_back(x, 1.0);
        d.unprocessed_weight_ += 1.0;
      }
    return d;
  }
  // A digest whose processed centroids are `cs` (sorted by mean), as the shipping rank's
  // process() left them: min/max are the first / last centroid means.
  static TDigest FromCentroids(const std::vector<Centroid>& cs, double compression = 1000) {
    TDigest d(compression);
    d.processed_ = cs;
    for (const auto& c : cs) d.processed_weight_ += c.weight;
    if (!cs.empty()) {
      d.min_ = cs.front().mean;
      d.max_ = cs.back().mean;
    }
    d.UpdateCumulative();
    return d;
  }
  // The same list carrying the shipping rank's true extremes (the min / max of the values it
  // added, as the incremental digest on that rank tracks them).  The published merge
  // (MergeProcessed below) never reads another digest's min_ / max_, and the 7 quantiles read the
  // merged min_ / max_ only when the first / last centroid holds >= 2% of the weight (W <= 50 for
  // delta = 1000): tests/test_digest_minmax.py checks both forms agree bit for bit.
  static TDigest FromCentroids(const std::vector<Centroid>& cs, double compression, double true_min, double true_max) {
    TDigest d = FromCentroids(cs, compression);
    if (!cs.empty()) {
      d.min_ = std::min(d.min_, true_min);
      d.max_ = std::max(d.max_, true_max);
    }
    return d;
  }
  // A merged digest whose min_ / max_ are then set to the given extremes (the "carried" reading
  // of merge(&other)): min_ = min(min_, lo), max_ = max(max_, hi).
  void carry_extremes(double lo, double hi) {
    min_ = std::min(min_, lo);
    max_ = std::max(max_, hi);
  }
  // add(first, last) of the merging digest: a whole batch of digests merged at once (one k-way
  // merge of their processed centroids, their unprocessed ones appended, process when dirty).
  void merge_batch(const std::vector<const TDigest*>& batch) {
    MergeProcessed(batch);
    MergeUnprocessed(batch);
    ProcessIfNecessary();
    UpdateCumulative();
  }

  const std::vector<Centroid>& processed() const { return processed_; }
  double processed_weight() const { return processed_weight_; }
  double min() const { return min_; }
  double max() const { return max_; }
  void compress() { Process(); }

 private:
  double compression_;
  double min_ = std::numeric_limits<double>::max();
  double max_ = std::numeric_limits<double>::min();
  size_t max_processed_;
  size_t max_unprocessed_;
  double processed_weight_ = 0.0;
  double unprocessed_weight_ = 0.0;
  std::vector<Centroid> processed_;
  std::vector<Centroid> unprocessed_;
  std::vector<double> cumulative_;

  bool HaveUnprocessed() const { return !unprocessed_.empty(); }
  bool IsDirty() const {
    return processed_.size() > max_processed_ || unprocessed_.size() > max_unprocessed_;
  }
  void ProcessIfNecessary() {
    if (IsDirty()) Process();
  }
  double IntegratedLocation(double q) const {
    return compression_ * (std::asin(2.0 * q - 1.0) + M_PI / 2) / M_PI;
  }
  double IntegratedQ(double k) const {
    return (std::sin(std::min(k, compression_) * M_PI / compression_ - M_PI / 2) + 1) / 2;
  }
  static double WeightedAverageSorted(double x1, double w1, double x2, double w2) {
    const double x = (x1 * w1 + x2 * w2) / (w1 + w2);
    return std::max(x1, std::min(x, x2));
  }
  static double WeightedAverage(double x1, double w1, double x2, double w2) {
    return (x1 <= x2) ? WeightedAverageSorted(x1, w1, x2, w2) : WeightedAverageSorted(x2, w2, x1, w1);
  }

  void UpdateCumulative() {
    cumulative_.clear();
    double previous = 0.0;
    for (const auto& c : processed_) {
      cumulative_.push_back(previous + c.weight / 2.0);
      previous = previous + c.weight;
    }
    cumulative_.push_back(previous);
  }

  void MergeUnprocessed(const std::vector<const TDigest*>& digests) {
    for (const auto* td : digests) {
      unprocessed_.insert(unprocessed_.end(), td->unprocessed_.begin(), td->unprocessed_.end());
      unprocessed_weight_ += td->unprocessed_weight_;
    }
  }

  void MergeProcessed(const std::vector<const TDigest*>& digests) {
    struct Cursor {
      const std::vector<Centroid>* v;
      size_t i;
    };
    auto cmp = [](const Cursor& a, const Cursor& b) { return (*a.v)[a.i].mean > (*b.v)[b.i].mean; };
    std::priority_queue<Cursor, std::vector<Cursor>, decltype(cmp)> pq(cmp);
    size_t total = 0;
    for (const auto* td : digests) {
      if (!td->processed_.empty()) {
        pq.push({&td->processed_, 0});
        total += td->processed_.size();
        processed_weight_ += td->processed_weight_;
      }
    }
    if (total == 0) return;
    if (!processed_.empty()) pq.push({&processed_, 0});
    std::vector<Centroid> sorted;
    sorted.reserve(total + processed_.size());
    while (!pq.empty()) {
      Cursor best = pq.top();
      pq.pop();
      sorted.push_back((*best.v)[best.i]);
      if (++best.i < best.v->size()) pq.push(best);
    }
    processed_ = std::move(sorted);
    if (!processed_.empty()) {
      min_ = std::min(min_, processed_.front().mean);
      max_ = std::max(max_, processed_.back().mean);
    }
  }

  void Process() {
    auto cc = [](const Centroid& a, const Centroid& b) { return a.mean < b.mean; };
    std::sort(unprocessed_.begin(), unprocessed_.end(), cc);
    size_t count = unprocessed_.size();
    unprocessed_.insert(unprocessed_.end(), processed_.begin(), processed_.end());
    std::inplace_merge(unprocessed_.begin(), unprocessed_.begin() + count, unprocessed_.end(), cc);

    processed_weight_ += unprocessed_weight_;
    unprocessed_weight_ = 0;
    processed_.clear();
    if (unprocessed_.empty()) {
      UpdateCumulative();
      return;
    }

    processed_.push_back(unprocessed_[0]);
    double w_so_far = unprocessed_[0].weight;
    double w_limit = processed_weight_ * IntegratedQ(1.0);
    for (size_t i = 1; i < unprocessed_.size(); ++i) {
      const Centroid& c = unprocessed_[i];
      double projected = w_so_far + c.weight;
      if (projected <= w_limit) {
        w_so_far = projected;
        processed_.back().add(c);
      } else {
        double k1 = IntegratedLocation(w_so_far / processed_weight_);
        w_limit = processed_weight_ * IntegratedQ(k1 + 1.0);
        w_so_far += c.weight;
        processed_.push_back(c);
      }
    }
    unprocessed_.clear();
    min_ = std::min(min_, processed_.front().mean);
    max_ = std::max(max_, processed_.back().mean);
    UpdateCumulative();
  }

  double QuantileProcessed(double q) const {
    if (q < 0 || q > 1) return NAN;
    if (processed_.empty()) return NAN;
    if (processed_.size() == 1) return processed_[0].mean;
    const size_t n = processed_.size();
    const double index = q * processed_weight_;
    if (index <= processed_[0].weight / 2.0) {
      return min_ + 2.0 * index / processed_[0].weight * (processed_[0].mean - min_);
    }
    auto it = std::lower_bound(cumulative_.begin(), cumulative_.end(), index);
    if (it + 1 != cumulative_.end()) {
      size_t i = static_cast<size_t>(it - cumulative_.begin());
      double z1 = index - *(it - 1);
      double z2 = *it - index;
      return WeightedAverage(processed_[i - 1].mean, z2, processed_[i].mean, z1);
    }
    double z1 = index - processed_weight_ - processed_[n - 1].weight / 2.0;
    double z2 = processed_[n - 1].weight / 2 - z1;
    return WeightedAverage(processed_[n - 1].mean, z1, max_, z2);
  }
};

}  // namespace oracle

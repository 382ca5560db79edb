// Native search methods.  Semantics follow the reference Go implementation
// (master/pkg/searcher/*.go; file:function noted per method) so experiments behave the same.
#include "searcher.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <stdexcept>

namespace damd_native {

// ---------------------------------------------------------------- SV helpers
int64_t SV::i() const {
  if (auto p = std::get_if<int64_t>(&v)) return *p;
  if (auto p = std::get_if<double>(&v)) return static_cast<int64_t>(*p);
  if (auto p = std::get_if<bool>(&v)) return *p ? 1 : 0;
  throw std::runtime_error("snapshot: expected integer");
}
double SV::d() const {
  if (auto p = std::get_if<double>(&v)) return *p;
  if (auto p = std::get_if<int64_t>(&v)) return static_cast<double>(*p);
  throw std::runtime_error("snapshot: expected number");
}
bool SV::b() const {
  if (auto p = std::get_if<bool>(&v)) return *p;
  return i() != 0;
}
const SVList& SV::list() const {
  if (auto p = std::get_if<SVList>(&v)) return *p;
  throw std::runtime_error("snapshot: expected list");
}
const SVMap& SV::map() const {
  if (auto p = std::get_if<SVMap>(&v)) return *p;
  throw std::runtime_error("snapshot: expected map");
}
const SV& SV::at(const std::string& k) const {
  const auto& m = map();
  auto it = m.find(k);
  if (it == m.end()) throw std::runtime_error("snapshot: missing key " + k);
  return it->second;
}

static SV sample_to_sv(const Sample& s) {
  SVList l;
  for (const auto& kv : s) {
    SVMap m;
    m["path"] = SV(kv.first);
    m["kind"] = SV(static_cast<int64_t>(kv.second.kind));
    m["i"] = SV(kv.second.i);
    m["d"] = SV(kv.second.d);
    l.emplace_back(std::move(m));
  }
  return SV(std::move(l));
}
static Sample sample_from_sv(const SV& sv) {
  Sample s;
  for (const auto& e : sv.list()) {
    HPValue v;
    v.kind = static_cast<int>(e.at("kind").i());
    v.i = e.at("i").i();
    v.d = e.at("d").d();
    s.emplace_back(std::get<std::string>(e.at("path").v), v);
  }
  return s;
}

// ---------------------------------------------------------------- hyperparameters
// reference: hyperparameters.go:sampleAll / sampleOne
Sample sample_all(const std::vector<HParam>& hps, std::mt19937_64& rng) {
  Sample s;
  for (const auto& h : hps) {
    HPValue v;
    switch (h.type) {
      case HPType::Const:
        v.kind = 2;
        v.i = 0;
        break;
      case HPType::Int: {
        std::uniform_int_distribution<int64_t> d(static_cast<int64_t>(h.minval), static_cast<int64_t>(h.maxval));
        v.kind = 0;
        v.i = d(rng);
        break;
      }
      case HPType::Double: {
        std::uniform_real_distribution<double> d(h.minval, h.maxval);
        v.kind = 1;
        v.d = h.minval == h.maxval ? h.minval : d(rng);
        break;
      }
      case HPType::Log: {
        std::uniform_real_distribution<double> d(h.minval, h.maxval);
        v.kind = 1;
        v.d = std::pow(h.base, h.minval == h.maxval ? h.minval : d(rng));
        break;
      }
      case HPType::Categorical: {
        std::uniform_int_distribution<int64_t> d(0, std::max<int64_t>(h.n_vals, 1) - 1);
        v.kind = 2;
        v.i = d(rng);
        break;
      }
    }
    s.emplace_back(h.path, v);
  }
  return s;
}

// reference: grid.go:getGridAxes / cartesianProduct
std::vector<Sample> grid_samples(const std::vector<HParam>& hps) {
  std::vector<std::vector<HPValue>> axes;
  for (const auto& h : hps) {
    std::vector<HPValue> axis;
    switch (h.type) {
      case HPType::Const: {
        HPValue v;
        v.kind = 2;
        axis.push_back(v);
        break;
      }
      case HPType::Int: {
        const int64_t lo = static_cast<int64_t>(h.minval), hi = static_cast<int64_t>(h.maxval);
        const int64_t count = std::min<int64_t>(std::max<int64_t>(h.count, 1), hi - lo + 1);
        for (int64_t i = 0; i < count; ++i) {
          HPValue v;
          v.kind = 0;
          v.i = count == 1 ? static_cast<int64_t>(std::llround((lo + hi) / 2.0))
                           : static_cast<int64_t>(std::llround(lo + static_cast<double>(i * (hi - lo)) / (count - 1)));
          axis.push_back(v);
        }
        break;
      }
      case HPType::Double:
      case HPType::Log: {
        const int64_t count = std::max<int64_t>(h.count, 1);
        for (int64_t i = 0; i < count; ++i) {
          double x = count == 1 ? (h.minval + h.maxval) / 2.0 : h.minval + i * (h.maxval - h.minval) / (count - 1);
          HPValue v;
          v.kind = 1;
          v.d = h.type == HPType::Log ? std::pow(h.base, x) : x;
          axis.push_back(v);
        }
        break;
      }
      case HPType::Categorical:
        for (int64_t i = 0; i < h.n_vals; ++i) {
          HPValue v;
          v.kind = 2;
          v.i = i;
          axis.push_back(v);
        }
        break;
    }
    axes.push_back(std::move(axis));
  }
  std::vector<Sample> out(1);
  for (size_t a = 0; a < axes.size(); ++a) {
    std::vector<Sample> next;
    for (const auto& partial : out)
      for (const auto& v : axes[a]) {
        Sample s = partial;
        s.emplace_back(hps[a].path, v);
        next.push_back(std::move(s));
      }
    out = std::move(next);
  }
  if (hps.empty()) return {Sample{}};
  return out;
}

static Operation op_create(Context& ctx, Sample s) {
  Operation o;
  o.type = OpType::Create;
  o.request_id = ctx.new_request_id();
  o.sample = std::move(s);
  return o;
}
static Operation op_validate(uint64_t rid, uint64_t length) {
  Operation o;
  o.type = OpType::ValidateAfter;
  o.request_id = rid;
  o.length = length;
  return o;
}
static Operation op_close(uint64_t rid) {
  Operation o;
  o.type = OpType::Close;
  o.request_id = rid;
  return o;
}

// ---------------------------------------------------------------- random / single
// reference: random.go
class RandomSearch : public SearchMethod {
 public:
  RandomSearch(const SearcherConfig& c, bool single) : cfg_(c), single_(single) {
    if (single_) {
      cfg_.max_trials = 1;
      cfg_.max_concurrent_trials = 1;
    }
  }
  std::vector<Operation> initial_operations(Context& ctx) override {
    std::vector<Operation> ops;
    int64_t n = cfg_.max_trials;
    if (cfg_.max_concurrent_trials > 0) n = std::min(n, cfg_.max_concurrent_trials);
    for (int64_t t = 0; t < n; ++t) add_trial(ctx, ops);
    return ops;
  }
  std::vector<Operation> trial_closed(Context& ctx, uint64_t) override {
    pending_--;
    std::vector<Operation> ops;
    if (created_ < cfg_.max_trials) add_trial(ctx, ops);
    return ops;
  }
  std::vector<Operation> trial_exited_early(Context&, uint64_t, ExitedReason r) override {
    pending_--;
    if (!single_ && (r == ExitedReason::InvalidHP || r == ExitedReason::InitInvalidHP)) created_--;
    return {};
  }
  double progress(const std::map<uint64_t, double>& tp, const std::set<uint64_t>& closed) override {
    double done = 0;
    for (const auto& kv : tp) done += closed.count(kv.first) ? static_cast<double>(cfg_.max_length) : kv.second;
    const double expected = static_cast<double>(cfg_.max_length) * static_cast<double>(cfg_.max_trials);
    return expected > 0 ? done / expected : 0.0;
  }
  SV snapshot() const override {
    SVMap m;
    m["created_trials"] = SV(created_);
    m["pending_trials"] = SV(pending_);
    m["search_method_type"] = SV(std::string(single_ ? "single" : "random"));
    return SV(m);
  }
  void restore(const SV& s) override {
    created_ = s.at("created_trials").i();
    pending_ = s.at("pending_trials").i();
  }
  std::string name() const override { return single_ ? "single" : "random"; }

 private:
  void add_trial(Context& ctx, std::vector<Operation>& ops) {
    Operation c = op_create(ctx, sample_all(*ctx.hparams, *ctx.rng));
    const uint64_t rid = c.request_id;
    ops.push_back(std::move(c));
    ops.push_back(op_validate(rid, cfg_.max_length));
    ops.push_back(op_close(rid));
    created_++;
    pending_++;
  }
  SearcherConfig cfg_;
  bool single_;
  int64_t created_ = 0, pending_ = 0;
};

// ---------------------------------------------------------------- grid
// reference: grid.go
class GridSearch : public SearchMethod {
 public:
  explicit GridSearch(const SearcherConfig& c) : cfg_(c) {}
  std::vector<Operation> initial_operations(Context& ctx) override {
    remaining_ = grid_samples(*ctx.hparams);
    trials_ = static_cast<int64_t>(remaining_.size());
    int64_t n = trials_;
    if (cfg_.max_concurrent_trials > 0) n = std::min(n, cfg_.max_concurrent_trials);
    std::vector<Operation> ops;
    for (int64_t t = 0; t < n; ++t) add_trial(ctx, ops);
    return ops;
  }
  std::vector<Operation> trial_closed(Context& ctx, uint64_t) override {
    pending_--;
    std::vector<Operation> ops;
    if (!remaining_.empty()) add_trial(ctx, ops);
    return ops;
  }
  double progress(const std::map<uint64_t, double>& tp, const std::set<uint64_t>& closed) override {
    double done = static_cast<double>(closed.size()) * static_cast<double>(cfg_.max_length);
    for (const auto& kv : tp)
      if (!closed.count(kv.first)) done += kv.second;
    const double expected = static_cast<double>(cfg_.max_length) * static_cast<double>(trials_);
    return expected > 0 ? done / expected : 0.0;
  }
  SV snapshot() const override {
    SVMap m;
    SVList rem;
    for (const auto& s : remaining_) rem.push_back(sample_to_sv(s));
    m["remaining_trials"] = SV(rem);
    m["pending_trials"] = SV(pending_);
    m["trials"] = SV(trials_);
    m["search_method_type"] = SV(std::string("grid"));
    return SV(m);
  }
  void restore(const SV& s) override {
    remaining_.clear();
    for (const auto& e : s.at("remaining_trials").list()) remaining_.push_back(sample_from_sv(e));
    pending_ = s.at("pending_trials").i();
    trials_ = s.at("trials").i();
  }
  std::string name() const override { return "grid"; }

 private:
  void add_trial(Context& ctx, std::vector<Operation>& ops) {
    Sample s = std::move(remaining_.back());
    remaining_.pop_back();
    Operation c = op_create(ctx, std::move(s));
    const uint64_t rid = c.request_id;
    ops.push_back(std::move(c));
    ops.push_back(op_validate(rid, cfg_.max_length));
    ops.push_back(op_close(rid));
    pending_++;
  }
  SearcherConfig cfg_;
  std::vector<Sample> remaining_;
  int64_t pending_ = 0, trials_ = 0;
};

// ---------------------------------------------------------------- ASHA (promotion + stopping)
// reference: asha.go (promotion-based) and asha_stopping.go (stop_once)
constexpr double kExitedMetric = std::numeric_limits<double>::max();

struct TrialMetric {
  uint64_t rid;
  double metric;
  bool promoted;
};

struct Rung {
  uint64_t units_needed = 0;
  std::vector<TrialMetric> metrics;  // sorted ascending (smaller is better after sign flip)
  int64_t outstanding = 0;

  // asha.go:promotionsAsync
  std::vector<uint64_t> promotions_async(uint64_t rid, double metric, double divisor) {
    const int old_np = static_cast<int>(static_cast<double>(metrics.size()) / divisor);
    const int np = static_cast<int>(static_cast<double>(metrics.size() + 1) / divisor);
    auto it = std::upper_bound(metrics.begin(), metrics.end(), metric,
                               [](double m, const TrialMetric& t) { return m < t.metric; });
    const int idx = static_cast<int>(it - metrics.begin());
    const bool promote_now = idx < np;
    metrics.insert(it, TrialMetric{rid, metric, promote_now});
    if (promote_now) return {rid};
    if (np != old_np && !metrics[old_np].promoted) {
      metrics[old_np].promoted = true;
      return {metrics[old_np].rid};
    }
    return {};
  }
  // asha_stopping.go:continueTraining
  bool continue_training(uint64_t rid, double metric, double divisor) {
    const int np = std::max(static_cast<int>(static_cast<double>(metrics.size() + 1) / divisor), 1);
    auto it = std::lower_bound(metrics.begin(), metrics.end(), metric,
                               [](const TrialMetric& t, double m) { return t.metric < m; });
    const int idx = static_cast<int>(it - metrics.begin());
    const bool promote_now = idx < np;
    metrics.insert(it, TrialMetric{rid, metric, promote_now});
    return promote_now;
  }
};

class AsyncHalving : public SearchMethod {
 public:
  AsyncHalving(const SearcherConfig& c, bool stopping) : cfg_(c), stopping_(stopping) {
    uint64_t units = 0;
    for (int64_t id = 0; id < cfg_.num_rungs; ++id) {
      const double rate = std::pow(cfg_.divisor, static_cast<double>(cfg_.num_rungs - id - 1));
      units += std::max<uint64_t>(static_cast<uint64_t>(static_cast<double>(cfg_.max_length) / rate), 1);
      Rung r;
      r.units_needed = units;
      rungs_.push_back(r);
    }
  }

  std::vector<Operation> initial_operations(Context& ctx) override {
    int64_t n;
    if (cfg_.max_concurrent_trials > 0) {
      n = std::min(cfg_.max_concurrent_trials, cfg_.max_trials);
    } else {
      n = std::clamp<int64_t>(static_cast<int64_t>(std::pow(cfg_.divisor, static_cast<double>(cfg_.num_rungs - 1))),
                              1, cfg_.max_trials);
    }
    std::vector<Operation> ops;
    for (int64_t t = 0; t < n; ++t) add_trial(ctx, ops);
    return ops;
  }
  std::vector<Operation> trial_created(Context&, uint64_t rid) override {
    rungs_[0].outstanding++;
    trial_rungs_[rid] = 0;
    return {};
  }
  std::vector<Operation> trial_closed(Context&, uint64_t rid) override {
    trials_completed_++;
    closed_.insert(rid);
    return {};
  }
  std::vector<Operation> validation_completed(Context& ctx, uint64_t rid, double metric, uint64_t) override {
    if (!stopping_) pending_--;
    if (!cfg_.smaller_is_better) metric *= -1;
    return stopping_ ? promote_stopping(ctx, rid, metric) : promote(ctx, rid, metric);
  }
  std::vector<Operation> trial_exited_early(Context& ctx, uint64_t rid, ExitedReason reason) override {
    if (!stopping_) pending_--;
    if (reason == ExitedReason::InvalidHP || reason == ExitedReason::InitInvalidHP) {
      std::vector<Operation> ops;
      early_exit_.insert(rid);
      ops.push_back(op_close(rid));
      closed_.insert(rid);
      invalid_trials_++;
      const int hi = trial_rungs_.count(rid) ? trial_rungs_[rid] : 0;
      rungs_[hi].outstanding--;
      for (int r = 0; r <= hi; ++r) {
        auto& m = rungs_[r].metrics;
        for (auto it = m.begin(); it != m.end(); ++it)
          if (it->rid == rid) {
            m.erase(it);
            break;
          }
      }
      add_trial(ctx, ops);
      return ops;
    }
    early_exit_.insert(rid);
    closed_.insert(rid);
    return stopping_ ? promote_stopping(ctx, rid, kExitedMetric) : promote(ctx, rid, kExitedMetric);
  }
  double progress(const std::map<uint64_t, double>&, const std::set<uint64_t>&) override {
    const double all = static_cast<double>(rungs_[0].metrics.size());
    double p = all / (1.2 * static_cast<double>(cfg_.max_trials));
    if (static_cast<int64_t>(rungs_[0].metrics.size()) == cfg_.max_trials) {
      const double valid = static_cast<double>(trials_completed_ - invalid_trials_);
      p = std::max(valid / static_cast<double>(cfg_.max_trials), p);
    }
    return p;
  }
  SV snapshot() const override {
    SVMap m;
    SVList rungs;
    for (const auto& r : rungs_) {
      SVMap rm;
      rm["units_needed"] = SV(r.units_needed);
      rm["outstanding_trials"] = SV(r.outstanding);
      SVList ms;
      for (const auto& t : r.metrics) {
        SVMap tm;
        tm["request_id"] = SV(t.rid);
        tm["metric"] = SV(t.metric);
        tm["promoted"] = SV(t.promoted);
        ms.emplace_back(tm);
      }
      rm["metrics"] = SV(ms);
      rungs.emplace_back(rm);
    }
    m["rungs"] = SV(rungs);
    SVMap tr;
    for (const auto& kv : trial_rungs_) tr[std::to_string(kv.first)] = SV(static_cast<int64_t>(kv.second));
    m["trial_rungs"] = SV(tr);
    SVList ee, cl;
    for (auto r : early_exit_) ee.emplace_back(SV(r));
    for (auto r : closed_) cl.emplace_back(SV(r));
    m["early_exit_trials"] = SV(ee);
    m["closed_trials"] = SV(cl);
    m["trials_completed"] = SV(trials_completed_);
    m["invalid_trials"] = SV(invalid_trials_);
    m["pending_trials"] = SV(pending_);
    m["search_method_type"] = SV(std::string("asha"));
    return SV(m);
  }
  void restore(const SV& s) override {
    rungs_.clear();
    for (const auto& rv : s.at("rungs").list()) {
      Rung r;
      r.units_needed = static_cast<uint64_t>(rv.at("units_needed").i());
      r.outstanding = rv.at("outstanding_trials").i();
      for (const auto& tv : rv.at("metrics").list())
        r.metrics.push_back(TrialMetric{static_cast<uint64_t>(tv.at("request_id").i()), tv.at("metric").d(),
                                        tv.at("promoted").b()});
      rungs_.push_back(r);
    }
    trial_rungs_.clear();
    for (const auto& kv : s.at("trial_rungs").map())
      trial_rungs_[std::stoull(kv.first)] = static_cast<int>(kv.second.i());
    early_exit_.clear();
    closed_.clear();
    for (const auto& v : s.at("early_exit_trials").list()) early_exit_.insert(static_cast<uint64_t>(v.i()));
    for (const auto& v : s.at("closed_trials").list()) closed_.insert(static_cast<uint64_t>(v.i()));
    trials_completed_ = s.at("trials_completed").i();
    invalid_trials_ = s.at("invalid_trials").i();
    pending_ = s.at("pending_trials").i();
  }
  std::string name() const override { return stopping_ ? "async_halving_stopping" : "async_halving"; }

 private:
  void add_trial(Context& ctx, std::vector<Operation>& ops) {
    Operation c = op_create(ctx, sample_all(*ctx.hparams, *ctx.rng));
    const uint64_t rid = c.request_id;
    trial_rungs_[rid] = 0;
    ops.push_back(std::move(c));
    ops.push_back(op_validate(rid, rungs_[0].units_needed));
    if (!stopping_) pending_++;
  }

  // asha.go:promoteAsync
  std::vector<Operation> promote(Context& ctx, uint64_t rid, double metric) {
    const int ri = trial_rungs_[rid];
    Rung& rung = rungs_[ri];
    rung.outstanding--;
    bool added = false;
    std::vector<Operation> ops;
    if (ri == static_cast<int>(cfg_.num_rungs) - 1) {
      rung.metrics.push_back(TrialMetric{rid, metric, false});
      if (!early_exit_.count(rid)) {
        ops.push_back(op_close(rid));
        closed_.insert(rid);
      }
    } else {
      Rung& next = rungs_[ri + 1];
      for (uint64_t pid : rung.promotions_async(rid, metric, cfg_.divisor)) {
        trial_rungs_[pid] = ri + 1;
        next.outstanding++;
        if (!early_exit_.count(pid)) {
          // rung k's own term max_length/divisor^(R-k-1) (= reference asha.go's
          // nextRung.UnitsNeeded - rung.UnitsNeeded), which is the absolute train target.
          const uint64_t units = std::max<uint64_t>(next.units_needed - rung.units_needed, 1);
          ops.push_back(op_validate(pid, units));
          added = true;
          pending_++;
        } else {
          auto more = promote(ctx, pid, kExitedMetric);
          ops.insert(ops.end(), more.begin(), more.end());
          return ops;
        }
      }
    }
    const int64_t all = static_cast<int64_t>(trial_rungs_.size()) - invalid_trials_;
    if (!added && all < cfg_.max_trials) add_trial(ctx, ops);
    if (static_cast<int64_t>(rungs_[0].metrics.size()) == cfg_.max_trials) {
      auto more = close_out_rungs();
      ops.insert(ops.end(), more.begin(), more.end());
    }
    return ops;
  }

  // asha.go:closeOutRungs
  std::vector<Operation> close_out_rungs() {
    std::vector<Operation> ops;
    for (auto& r : rungs_) {
      if (r.outstanding > 0) break;
      for (auto& t : r.metrics)
        if (!t.promoted && !closed_.count(t.rid) && !early_exit_.count(t.rid)) {
          ops.push_back(op_close(t.rid));
          closed_.insert(t.rid);
        }
    }
    return ops;
  }

  // asha_stopping.go:promoteAsync
  std::vector<Operation> promote_stopping(Context& ctx, uint64_t rid, double metric) {
    const int ri = trial_rungs_[rid];
    Rung& rung = rungs_[ri];
    rung.outstanding--;
    bool added = false;
    std::vector<Operation> ops;
    if (ri == static_cast<int>(cfg_.num_rungs) - 1) {
      rung.metrics.push_back(TrialMetric{rid, metric, false});
      if (!early_exit_.count(rid)) {
        ops.push_back(op_close(rid));
        closed_.insert(rid);
      }
    } else {
      Rung& next = rungs_[ri + 1];
      const bool go_on = rung.continue_training(rid, metric, cfg_.divisor);
      if (!early_exit_.count(rid)) {
        if (go_on) {
          trial_rungs_[rid] = ri + 1;
          next.outstanding++;
          ops.push_back(op_validate(rid, std::max<uint64_t>(next.units_needed - rung.units_needed, 1)));
          added = true;
        } else {
          ops.push_back(op_close(rid));
          closed_.insert(rid);
        }
      }
    }
    const int64_t all = static_cast<int64_t>(trial_rungs_.size()) - invalid_trials_;
    if (!added && all < cfg_.max_trials) add_trial(ctx, ops);
    return ops;
  }

  SearcherConfig cfg_;
  bool stopping_;
  std::vector<Rung> rungs_;
  std::map<uint64_t, int> trial_rungs_;
  std::set<uint64_t> early_exit_, closed_;
  int64_t trials_completed_ = 0, invalid_trials_ = 0, pending_ = 0;
};

// ---------------------------------------------------------------- tournament (adaptive ASHA)
// reference: tournament.go + adaptive_asha.go
class Tournament : public SearchMethod {
 public:
  explicit Tournament(std::vector<std::unique_ptr<SearchMethod>> subs) : subs_(std::move(subs)) {}
  std::vector<Operation> initial_operations(Context& ctx) override {
    std::vector<Operation> all;
    for (size_t i = 0; i < subs_.size(); ++i) {
      auto ops = subs_[i]->initial_operations(ctx);
      mark(i, ops);
      all.insert(all.end(), ops.begin(), ops.end());
    }
    return all;
  }
  std::vector<Operation> trial_created(Context& ctx, uint64_t rid) override {
    const size_t i = table_.at(rid);
    auto ops = subs_[i]->trial_created(ctx, rid);
    return mark(i, ops);
  }
  std::vector<Operation> validation_completed(Context& ctx, uint64_t rid, double m, uint64_t len) override {
    const size_t i = table_.at(rid);
    auto ops = subs_[i]->validation_completed(ctx, rid, m, len);
    return mark(i, ops);
  }
  std::vector<Operation> trial_closed(Context& ctx, uint64_t rid) override {
    const size_t i = table_.at(rid);
    auto ops = subs_[i]->trial_closed(ctx, rid);
    return mark(i, ops);
  }
  std::vector<Operation> trial_exited_early(Context& ctx, uint64_t rid, ExitedReason r) override {
    const size_t i = table_.at(rid);
    auto ops = subs_[i]->trial_exited_early(ctx, rid, r);
    return mark(i, ops);
  }
  double progress(const std::map<uint64_t, double>& tp, const std::set<uint64_t>& closed) override {
    double sum = 0;
    for (size_t i = 0; i < subs_.size(); ++i) {
      std::map<uint64_t, double> p;
      std::set<uint64_t> c;
      for (const auto& kv : tp)
        if (table_.count(kv.first) && table_.at(kv.first) == i) p[kv.first] = kv.second;
      for (auto r : closed)
        if (table_.count(r) && table_.at(r) == i) c.insert(r);
      sum += subs_[i]->progress(p, c);
    }
    return subs_.empty() ? 0.0 : sum / static_cast<double>(subs_.size());
  }
  SV snapshot() const override {
    SVMap m;
    SVMap t;
    for (const auto& kv : table_) t[std::to_string(kv.first)] = SV(static_cast<int64_t>(kv.second));
    m["trial_table"] = SV(t);
    SVList subs;
    for (const auto& s : subs_) subs.push_back(s->snapshot());
    m["sub_search_states"] = SV(subs);
    m["search_method_type"] = SV(std::string("adaptive_asha"));
    return SV(m);
  }
  void restore(const SV& s) override {
    table_.clear();
    for (const auto& kv : s.at("trial_table").map()) table_[std::stoull(kv.first)] = static_cast<size_t>(kv.second.i());
    const auto& subs = s.at("sub_search_states").list();
    for (size_t i = 0; i < subs.size() && i < subs_.size(); ++i) subs_[i]->restore(subs[i]);
  }
  std::string name() const override { return "adaptive_asha"; }
  size_t n_brackets() const { return subs_.size(); }

 private:
  std::vector<Operation>& mark(size_t i, std::vector<Operation>& ops) {
    for (const auto& o : ops)
      if (o.type == OpType::Create) table_[o.request_id] = i;
    return ops;
  }
  std::vector<std::unique_ptr<SearchMethod>> subs_;
  std::map<uint64_t, size_t> table_;
};

// adaptive_asha.go:getBracketMaxTrials
std::vector<int64_t> bracket_max_trials(int64_t max_trials, double divisor, const std::vector<int64_t>& br) {
  std::vector<double> w;
  double tot = 0;
  for (auto r : br) {
    w.push_back(std::pow(divisor, static_cast<double>(r - 1)) / static_cast<double>(r));
    tot += w.back();
  }
  std::vector<int64_t> out;
  int64_t alloc = 0;
  for (size_t i = 0; i < br.size(); ++i) {
    out.push_back(std::max<int64_t>(static_cast<int64_t>(w[i] / tot * static_cast<double>(max_trials)), 1));
    alloc += out.back();
  }
  out[0] += std::max<int64_t>(max_trials - alloc, 0);
  return out;
}

// adaptive_asha.go:getBracketMaxConcurrentTrials
std::vector<int64_t> bracket_max_concurrent(int64_t mct, double divisor, const std::vector<int64_t>& mt) {
  const int64_t nb = static_cast<int64_t>(mt.size());
  int64_t min_trials, rem = 0;
  if (mct == 0) {
    min_trials = std::max<int64_t>(mt.back(), static_cast<int64_t>(divisor));
  } else {
    mct = std::max<int64_t>(mct, nb);
    min_trials = mct / nb;
    rem = mct % nb;
  }
  std::vector<int64_t> out(nb, min_trials);
  for (int64_t i = 0; i < rem; ++i) out[i]++;
  return out;
}

std::unique_ptr<SearchMethod> make_search_method(const SearcherConfig& c) {
  if (c.name == "single") return std::make_unique<RandomSearch>(c, true);
  if (c.name == "random") return std::make_unique<RandomSearch>(c, false);
  if (c.name == "grid") return std::make_unique<GridSearch>(c);
  if (c.name == "async_halving") return std::make_unique<AsyncHalving>(c, c.stop_once);
  if (c.name == "adaptive_asha") {
    std::vector<int64_t> brackets = c.bracket_rungs;
    if (brackets.empty()) {
      int64_t max_rungs = std::min<int64_t>(
          {c.max_rungs,
           static_cast<int64_t>(std::log(static_cast<double>(std::max<uint64_t>(c.max_length, 1))) / std::log(c.divisor)) + 1,
           static_cast<int64_t>(std::log(static_cast<double>(std::max<int64_t>(c.max_trials, 1))) / std::log(c.divisor)) + 1});
      if (c.mode == "conservative") {
        for (int64_t i = 1; i <= max_rungs; ++i) brackets.push_back(i);
      } else if (c.mode == "aggressive") {
        brackets.push_back(max_rungs);
      } else {
        for (int64_t i = (max_rungs - 1) / 2 + 1; i <= max_rungs; ++i) brackets.push_back(i);
      }
    }
    std::sort(brackets.rbegin(), brackets.rend());
    const auto mt = bracket_max_trials(c.max_trials, c.divisor, brackets);
    const auto mct = bracket_max_concurrent(c.max_concurrent_trials, c.divisor, mt);
    std::vector<std::unique_ptr<SearchMethod>> subs;
    for (size_t i = 0; i < brackets.size(); ++i) {
      SearcherConfig sc = c;
      sc.name = "async_halving";
      sc.num_rungs = brackets[i];
      sc.max_trials = mt[i];
      sc.max_concurrent_trials = mct[i];
      subs.push_back(std::make_unique<AsyncHalving>(sc, c.stop_once));
    }
    return std::make_unique<Tournament>(std::move(subs));
  }
  throw std::invalid_argument("unknown search method: " + c.name);
}

}  // namespace damd_native

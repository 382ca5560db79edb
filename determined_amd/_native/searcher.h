// Native search-method engine (C++17): the algorithmic core of hyperparameter search.
//
// Counterpart of the reference Go package master/pkg/searcher (search_method.go, random.go,
// grid.go, asha.go, asha_stopping.go, adaptive_asha.go, tournament.go, hyperparameters.go).
// The experiment/trial bookkeeping around it (request-id <-> trial mapping, op queues,
// persistence) lives in determined_amd/master; this layer is pure state machines.
//
// Hyperparameter values that are not numbers (const values, categorical choices) are
// opaque to C++: a sample carries the INDEX of the chosen value and the Python side maps
// it back.  State snapshots are returned as a small variant tree (SV) that the binding
// converts to/from Python dicts (stored as JSON by the master).
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <random>
#include <set>
#include <string>
#include <variant>
#include <vector>

namespace damd_native {

// ---------------------------------------------------------------- snapshot value tree
struct SV;
using SVList = std::vector<SV>;
using SVMap = std::map<std::string, SV>;
struct SV {
  std::variant<std::monostate, bool, int64_t, double, std::string, SVList, SVMap> v;
  SV() = default;
  SV(bool b) : v(b) {}
  SV(int64_t i) : v(i) {}
  SV(int i) : v(static_cast<int64_t>(i)) {}
  SV(uint64_t i) : v(static_cast<int64_t>(i)) {}
  SV(double d) : v(d) {}
  SV(std::string s) : v(std::move(s)) {}
  SV(SVList l) : v(std::move(l)) {}
  SV(SVMap m) : v(std::move(m)) {}
  int64_t i() const;
  double d() const;
  bool b() const;
  const SVList& list() const;
  const SVMap& map() const;
  const SV& at(const std::string& k) const;
};

// ---------------------------------------------------------------- hyperparameters
enum class HPType { Const = 0, Int = 1, Double = 2, Log = 3, Categorical = 4 };

struct HParam {
  std::string path;  // dotted path for nested hyperparameters ("optimizer.lr")
  HPType type = HPType::Const;
  double minval = 0, maxval = 0, base = 10;
  int64_t count = 0;  // grid count (0 = unset)
  int64_t n_vals = 1; // categorical: number of choices
};

struct HPValue {
  int kind = 2;  // 0 = int, 1 = double, 2 = index into the const/categorical value list
  int64_t i = 0;
  double d = 0;
};

using Sample = std::vector<std::pair<std::string, HPValue>>;

// ---------------------------------------------------------------- operations
enum class OpType { Create = 0, ValidateAfter = 1, Close = 2, Shutdown = 3 };

struct Operation {
  OpType type;
  uint64_t request_id = 0;
  uint64_t length = 0;   // ValidateAfter: absolute units to reach before validating
  Sample sample;         // Create
  bool cancel = false, failure = false;  // Shutdown
};

enum class ExitedReason { Errored = 0, UserCanceled = 1, InvalidHP = 2, InitInvalidHP = 3, UserRequestedStop = 4 };

struct Context {
  std::mt19937_64* rng;
  const std::vector<HParam>* hparams;
  uint64_t* next_request_id;
  uint64_t new_request_id() { return ++(*next_request_id); }
};

Sample sample_all(const std::vector<HParam>& hps, std::mt19937_64& rng);
std::vector<Sample> grid_samples(const std::vector<HParam>& hps);

// ---------------------------------------------------------------- search methods
class SearchMethod {
 public:
  virtual ~SearchMethod() = default;
  virtual std::vector<Operation> initial_operations(Context& ctx) = 0;
  virtual std::vector<Operation> trial_created(Context&, uint64_t) { return {}; }
  virtual std::vector<Operation> validation_completed(Context&, uint64_t, double, uint64_t) { return {}; }
  virtual std::vector<Operation> trial_closed(Context&, uint64_t) { return {}; }
  virtual std::vector<Operation> trial_exited_early(Context&, uint64_t, ExitedReason) { return {}; }
  virtual double progress(const std::map<uint64_t, double>& trial_progress, const std::set<uint64_t>& closed) = 0;
  virtual SV snapshot() const = 0;
  virtual void restore(const SV& state) = 0;
  virtual std::string name() const = 0;
};

struct SearcherConfig {
  std::string name;            // single | random | grid | async_halving | adaptive_asha
  uint64_t max_length = 0;     // units
  int64_t max_trials = 1;
  int64_t max_concurrent_trials = 16;
  double divisor = 4;
  int64_t num_rungs = 0;       // async_halving
  int64_t max_rungs = 5;       // adaptive_asha
  std::string mode = "standard";
  std::vector<int64_t> bracket_rungs;
  bool stop_once = false;
  bool smaller_is_better = true;
};

std::unique_ptr<SearchMethod> make_search_method(const SearcherConfig& cfg);

}  // namespace damd_native

// pybind11 bindings for the native control plane (_native.so).
#include <pybind11/pybind11.h>
#include <tuple>
#include <pybind11/stl.h>

#include <sstream>

#include "scheduler.h"
#include "searcher.h"

namespace py = pybind11;
using namespace damd_native;

namespace {

py::object sv_to_py(const SV& s) {
  struct V {
    py::object operator()(std::monostate) const { return py::none(); }
    py::object operator()(bool b) const { return py::bool_(b); }
    py::object operator()(int64_t i) const { return py::int_(i); }
    py::object operator()(double d) const { return py::float_(d); }
    py::object operator()(const std::string& x) const { return py::str(x); }
    py::object operator()(const SVList& l) const {
      py::list out;
      for (const auto& e : l) out.append(sv_to_py(e));
      return out;
    }
    py::object operator()(const SVMap& m) const {
      py::dict out;
      for (const auto& kv : m) out[py::str(kv.first)] = sv_to_py(kv.second);
      return out;
    }
  };
  return std::visit(V{}, s.v);
}

SV py_to_sv(const py::handle& o) {
  if (o.is_none()) return SV();
  if (py::isinstance<py::bool_>(o)) return SV(o.cast<bool>());
  if (py::isinstance<py::int_>(o)) return SV(o.cast<int64_t>());
  if (py::isinstance<py::float_>(o)) return SV(o.cast<double>());
  if (py::isinstance<py::str>(o)) return SV(o.cast<std::string>());
  if (py::isinstance<py::dict>(o)) {
    SVMap m;
    for (auto kv : o.cast<py::dict>()) m[py::str(kv.first).cast<std::string>()] = py_to_sv(kv.second);
    return SV(m);
  }
  if (py::isinstance<py::list>(o) || py::isinstance<py::tuple>(o)) {
    SVList l;
    for (auto e : o) l.push_back(py_to_sv(e));
    return SV(l);
  }
  throw std::invalid_argument("unsupported snapshot value");
}

const char* op_name(OpType t) {
  switch (t) {
    case OpType::Create: return "create";
    case OpType::ValidateAfter: return "validate_after";
    case OpType::Close: return "close";
    case OpType::Shutdown: return "shutdown";
  }
  return "?";
}

py::list ops_to_py(const std::vector<Operation>& ops) {
  py::list out;
  for (const auto& o : ops) {
    py::dict d;
    d["type"] = op_name(o.type);
    d["request_id"] = o.request_id;
    if (o.type == OpType::ValidateAfter) d["length"] = o.length;
    if (o.type == OpType::Create) {
      py::list hp;
      for (const auto& kv : o.sample) hp.append(py::make_tuple(kv.first, kv.second.kind, kv.second.i, kv.second.d));
      d["hparams"] = hp;
    }
    if (o.type == OpType::Shutdown) {
      d["cancel"] = o.cancel;
      d["failure"] = o.failure;
    }
    out.append(d);
  }
  return out;
}

// Owns a search method + its RNG / hyperparameter space / request-id counter.
class SearchEngine {
 public:
  SearchEngine(const py::dict& cfg, const py::list& hparams, uint64_t seed) : rng_(seed) {
    SearcherConfig c;
    c.name = cfg["name"].cast<std::string>();
    auto get = [&](const char* k) -> py::object { return cfg.contains(k) ? py::object(cfg[k]) : py::object(py::none()); };
    if (!get("max_length").is_none()) c.max_length = get("max_length").cast<uint64_t>();
    if (!get("max_trials").is_none()) c.max_trials = get("max_trials").cast<int64_t>();
    if (!get("max_concurrent_trials").is_none()) c.max_concurrent_trials = get("max_concurrent_trials").cast<int64_t>();
    if (!get("divisor").is_none()) c.divisor = get("divisor").cast<double>();
    if (!get("num_rungs").is_none()) c.num_rungs = get("num_rungs").cast<int64_t>();
    if (!get("max_rungs").is_none()) c.max_rungs = get("max_rungs").cast<int64_t>();
    if (!get("mode").is_none()) c.mode = get("mode").cast<std::string>();
    if (!get("bracket_rungs").is_none()) c.bracket_rungs = get("bracket_rungs").cast<std::vector<int64_t>>();
    if (!get("stop_once").is_none()) c.stop_once = get("stop_once").cast<bool>();
    if (!get("smaller_is_better").is_none()) c.smaller_is_better = get("smaller_is_better").cast<bool>();
    for (auto h : hparams) {
      auto d = h.cast<py::dict>();
      HParam p;
      p.path = d["path"].cast<std::string>();
      p.type = static_cast<HPType>(d["type"].cast<int>());
      if (d.contains("minval")) p.minval = d["minval"].cast<double>();
      if (d.contains("maxval")) p.maxval = d["maxval"].cast<double>();
      if (d.contains("base")) p.base = d["base"].cast<double>();
      if (d.contains("count") && !d["count"].is_none()) p.count = d["count"].cast<int64_t>();
      if (d.contains("n_vals")) p.n_vals = d["n_vals"].cast<int64_t>();
      hps_.push_back(p);
    }
    method_ = make_search_method(c);
  }
  Context ctx() { return Context{&rng_, &hps_, &next_id_}; }
  py::list initial_operations() {
    auto c = ctx();
    return ops_to_py(method_->initial_operations(c));
  }
  py::list trial_created(uint64_t rid) {
    auto c = ctx();
    return ops_to_py(method_->trial_created(c, rid));
  }
  py::list validation_completed(uint64_t rid, double metric, uint64_t length) {
    auto c = ctx();
    return ops_to_py(method_->validation_completed(c, rid, metric, length));
  }
  py::list trial_closed(uint64_t rid) {
    auto c = ctx();
    return ops_to_py(method_->trial_closed(c, rid));
  }
  py::list trial_exited_early(uint64_t rid, int reason) {
    auto c = ctx();
    return ops_to_py(method_->trial_exited_early(c, rid, static_cast<ExitedReason>(reason)));
  }
  double progress(const std::map<uint64_t, double>& tp, const std::set<uint64_t>& closed) {
    return method_->progress(tp, closed);
  }
  py::dict snapshot() const {
    py::dict d;
    d["method"] = sv_to_py(method_->snapshot());
    std::ostringstream os;
    os << rng_;
    d["rng"] = os.str();
    d["next_request_id"] = next_id_;
    return d;
  }
  void restore(const py::dict& d) {
    method_->restore(py_to_sv(d["method"]));
    std::istringstream is(d["rng"].cast<std::string>());
    is >> rng_;
    next_id_ = d["next_request_id"].cast<uint64_t>();
  }
  std::string name() const { return method_->name(); }

 private:
  std::mt19937_64 rng_;
  std::vector<HParam> hps_;
  uint64_t next_id_ = 0;
  std::unique_ptr<SearchMethod> method_;
};

py::dict request_to_py(const Request& r) {
  py::dict d;
  d["alloc_id"] = r.alloc_id;
  d["job_id"] = r.job_id;
  d["slots"] = r.slots;
  d["priority"] = r.priority;
  d["weight"] = r.weight;
  d["order"] = r.order;
  d["preemptible"] = r.preemptible;
  d["allocated"] = r.allocated;
  d["preempting"] = r.preempting;
  py::list as;
  for (const auto& a : r.assignment) as.append(py::make_tuple(a.first, a.second));
  d["assignment"] = as;
  return d;
}

}  // namespace

namespace damd_native {
void register_loader(py::module& m);
// searcher.cpp (adaptive_asha.go getBracketMaxTrials / getBracketMaxConcurrentTrials), exposed for the
// Go test vectors in tests/test_searcher_go_vectors.py
std::vector<int64_t> bracket_max_trials(int64_t max_trials, double divisor, const std::vector<int64_t>& br);
std::vector<int64_t> bracket_max_concurrent(int64_t mct, double divisor, const std::vector<int64_t>& mt);
}  // namespace damd_native

PYBIND11_MODULE(_native, m) {
  damd_native::register_loader(m);
  m.doc() = "determined_amd native control plane: search methods + scheduler";
  m.def("bracket_max_trials", &damd_native::bracket_max_trials, py::arg("max_trials"), py::arg("divisor"), py::arg("rungs"));
  m.def("bracket_max_concurrent", &damd_native::bracket_max_concurrent, py::arg("max_concurrent_trials"), py::arg("divisor"),
        py::arg("max_trials"));
  py::class_<SearchEngine>(m, "SearchEngine")
      .def(py::init<const py::dict&, const py::list&, uint64_t>(), py::arg("config"), py::arg("hparams"),
           py::arg("seed"))
      .def("initial_operations", &SearchEngine::initial_operations)
      .def("trial_created", &SearchEngine::trial_created)
      .def("validation_completed", &SearchEngine::validation_completed)
      .def("trial_closed", &SearchEngine::trial_closed)
      .def("trial_exited_early", &SearchEngine::trial_exited_early)
      .def("progress", &SearchEngine::progress)
      .def("snapshot", &SearchEngine::snapshot)
      .def("restore", &SearchEngine::restore)
      .def_property_readonly("name", &SearchEngine::name);

  py::enum_<Policy>(m, "Policy")
      .value("PRIORITY", Policy::Priority)
      .value("FAIR_SHARE", Policy::FairShare)
      .value("ROUND_ROBIN", Policy::RoundRobin);
  py::enum_<Fit>(m, "Fit").value("BEST", Fit::Best).value("WORST", Fit::Worst);

  // fair_share.go fairshareSchedule over an explicit snapshot (tests replay the Go vectors with it):
  // tasks = [(alloc_id, job_id, slots, allocated, preemptible, blocked_agents)] in queue order,
  // groups = {job_id: (weight, max_slots or -1)}, agents = {agent_id: free slot count}.
  m.def("fairshare_decide",
        [](const std::vector<std::tuple<std::string, std::string, int, bool, bool, std::vector<std::string>>>& tasks,
           const std::map<std::string, std::pair<double, int>>& groups, const std::map<std::string, int>& agents,
           Fit fit) {
          std::vector<Request> reqs;
          int64_t order = 0;
          for (const auto& t : tasks) {
            Request r;
            r.alloc_id = std::get<0>(t);
            r.job_id = std::get<1>(t);
            r.slots = std::get<2>(t);
            r.allocated = std::get<3>(t);
            r.preemptible = std::get<4>(t);
            r.excluded_agents = std::get<5>(t);
            r.order = order++;
            reqs.push_back(r);
          }
          std::map<std::string, FairShareGroup> gs;
          for (const auto& kv : groups) gs[kv.first] = FairShareGroup{kv.second.first, kv.second.second};
          std::map<std::string, AgentState> as;
          for (const auto& kv : agents) {
            AgentState a;
            a.id = kv.first;
            a.num_slots = kv.second;
            a.slot_owner.assign(kv.second, "");
            a.slot_disabled.assign(kv.second, 0);
            a.max_zero_slot_containers = 0;  // the Go mock agents' default
            as[kv.first] = a;
          }
          Decision d = fairshare_decide(reqs, gs, as, fit);
          return py::make_tuple(d.allocated, d.preempt);
        },
        py::arg("tasks"), py::arg("groups"), py::arg("agents"), py::arg("fit") = Fit::Best);

  py::class_<Scheduler>(m, "Scheduler")
      .def(py::init<Policy, Fit, bool>(), py::arg("policy"), py::arg("fit") = Fit::Best,
           py::arg("preemption") = true)
      .def("add_agent", &Scheduler::add_agent)
      .def("remove_agent", &Scheduler::remove_agent)
      .def("set_agent_enabled", &Scheduler::set_agent_enabled)
      .def("set_slot_enabled", &Scheduler::set_slot_enabled)
      .def("add_request",
           [](Scheduler& s, const std::string& alloc_id, const std::string& job_id, int slots, int priority,
              double weight, int64_t order, bool preemptible, const std::vector<std::string>& excluded_agents) {
             Request r;
             r.excluded_agents = excluded_agents;
             r.alloc_id = alloc_id;
             r.job_id = job_id;
             r.slots = slots;
             r.priority = priority;
             r.weight = weight;
             r.order = order;
             r.preemptible = preemptible;
             s.add_request(r);
           },
           py::arg("alloc_id"), py::arg("job_id"), py::arg("slots"), py::arg("priority") = 42,
           py::arg("weight") = 1.0, py::arg("order") = 0, py::arg("preemptible") = true,
           py::arg("excluded_agents") = std::vector<std::string>())
      .def("remove_request", &Scheduler::remove_request)
      .def("set_priority", &Scheduler::set_priority)
      .def("set_weight", &Scheduler::set_weight)
      .def("set_max_slots", &Scheduler::set_max_slots)
      .def("set_agent_max_zero_slot", &Scheduler::set_agent_max_zero_slot)
      .def("schedule",
           [](Scheduler& s) {
             Decision d = s.schedule();
             py::dict out;
             out["allocated"] = d.allocated;
             out["preempt"] = d.preempt;
             return out;
           })
      .def("requests",
           [](const Scheduler& s) {
             py::dict out;
             for (const auto& kv : s.requests()) out[py::str(kv.first)] = request_to_py(kv.second);
             return out;
           })
      .def("agents",
           [](const Scheduler& s) {
             py::dict out;
             for (const auto& kv : s.agents()) {
               py::dict a;
               a["num_slots"] = kv.second.num_slots;
               a["slot_owner"] = kv.second.slot_owner;
               a["enabled"] = kv.second.enabled;
               py::list dis;
               for (int i = 0; i < kv.second.num_slots; ++i)
                 if (kv.second.slot_disabled[i]) dis.append(i);
               a["disabled_slots"] = dis;
               out[py::str(kv.first)] = a;
             }
             return out;
           })
      .def_property_readonly("total_slots", &Scheduler::total_slots)
      .def_property_readonly("used_slots", &Scheduler::used_slots);
}

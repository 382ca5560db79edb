// Native resource scheduler for a resource pool of agents and their slots.
//
// Counterpart of the reference's agent resource manager schedulers
// (master/internal/rm/agentrm/{priority,fair_share,round_robin,fitting,fitting_methods}.go).
// An MI355X node is one agent with 8 slots (one per GPU, 288 GB HBM each); the scheduler packs
// concurrent 1-slot trials onto free GPUs or gang-schedules an N-slot distributed trial, and
// decides which running allocations to preempt.  Pure state machine: the master calls
// schedule() after every change and acts on the returned decisions.
#pragma once

#include <cstdint>
#include <map>
#include <algorithm>
#include <string>
#include <vector>

namespace damd_native {

enum class Policy { Priority = 0, FairShare = 1, RoundRobin = 2 };
enum class Fit { Best = 0, Worst = 1 };

struct AgentState {
  std::string id;
  int num_slots = 0;
  std::vector<std::string> slot_owner;  // allocation id or "" per slot
  std::vector<char> slot_disabled;      // `det slot disable` (reference agentrm slot enable/disable)
  int zero_slot_containers = 0;
  int max_zero_slot_containers = 1 << 30;  // reference agent max_zero_slot_containers (unlimited here)
  bool enabled = true;
  int empty() const;  // free and enabled slots
  int disabled() const;
  int usable() const { return num_slots - disabled(); }
  int used() const { return usable() - empty(); }
  bool free_slot(int i) const { return slot_owner[i].empty() && !slot_disabled[i]; }
};

struct Request {
  std::string alloc_id;
  std::string job_id;
  int slots = 1;
  int priority = 42;      // smaller value = more important (reference: 1..99, default 42)
  double weight = 1.0;    // fair share weight
  int64_t order = 0;      // submission order (queue position)
  bool preemptible = true;
  bool allocated = false;
  bool preempting = false;  // release already requested
  std::vector<std::string> excluded_agents;  // log-policy exclude_node blocklist
  // agent id -> slot indices
  std::vector<std::pair<std::string, std::vector<int>>> assignment;
};

struct Decision {
  std::vector<std::string> allocated;  // alloc ids newly allocated this round
  std::vector<std::string> preempt;    // alloc ids that must release their resources
};

struct Fitting {
  std::vector<std::pair<std::string, std::vector<int>>> assignment;
};

// fitting.go findFits: a shared fit on one agent (best / worst fit), else whole idle agents of equal
// free-slot count (multi-slot requests only).
bool find_fit_in(const Request& r, const std::map<std::string, AgentState>& agents, Fit fit, Fitting* out);

// A job's fair-share parameters (reference tasklist.Group: Weight, MaxSlots).
struct FairShareGroup {
  double weight = 0.0;
  int max_slots = -1;  // < 0: no cap
};

// fair_share.go fairshareSchedule on a snapshot, decision for decision: ``tasks`` in queue order
// (``allocated`` = already scheduled), ``groups`` by job id (a job missing from it is a group of
// weight 0 with no cap, like the Go zero value).  Returns the tasks to start and the preemptible
// allocations to release.  Like the Go function it checks fits against the unchanged ``agents``
// (starting several tasks in one call may over-commit; the caller places them one by one).
Decision fairshare_decide(const std::vector<Request>& tasks, const std::map<std::string, FairShareGroup>& groups,
                          const std::map<std::string, AgentState>& agents, Fit fit);

class Scheduler {
 public:
  Scheduler(Policy policy, Fit fit, bool preemption) : policy_(policy), fit_(fit), preemption_(preemption) {}

  void add_agent(const std::string& id, int slots);
  void remove_agent(const std::string& id);  // allocations on it become unallocated (returned lost)
  void set_agent_enabled(const std::string& id, bool enabled);
  // Disable / enable one slot of an agent: a disabled slot is never offered to new allocations
  // (a running allocation on it keeps it until it ends).  Returns false for an unknown slot.
  bool set_slot_enabled(const std::string& id, int slot, bool enabled);
  void add_request(const Request& r);
  void remove_request(const std::string& alloc_id);  // frees its slots
  void set_priority(const std::string& job_id, int priority);
  void set_weight(const std::string& job_id, double weight);
  void set_max_slots(const std::string& job_id, int max_slots);  // fair share group cap (< 0: none)
  void set_agent_max_zero_slot(const std::string& id, int n);

  Decision schedule();

  const std::map<std::string, Request>& requests() const { return reqs_; }
  const std::map<std::string, AgentState>& agents() const { return agents_; }
  int total_slots() const;
  int used_slots() const;

 private:
  bool find_fit(const Request& r, const std::map<std::string, AgentState>& agents, Fitting* out) const;
  void apply(std::map<std::string, AgentState>& agents, const std::string& alloc_id, const Fitting& f) const;
  void release(std::map<std::string, AgentState>& agents, const Request& r) const;
  double score(const Request& r, const AgentState& a) const;

  Decision schedule_priority();
  Decision schedule_fair_share();
  Decision schedule_round_robin();

  Policy policy_;
  Fit fit_;
  bool preemption_;
  std::map<std::string, AgentState> agents_;
  std::map<std::string, Request> reqs_;
  std::map<std::string, int> max_slots_;
};

}  // namespace damd_native

// Native scheduler implementation (see scheduler.h; reference rm/agentrm/*.go).
#include "scheduler.h"

#include <algorithm>
#include <cmath>
#include <functional>
#include <set>
#include <stdexcept>

namespace damd_native {

int AgentState::empty() const {
  int n = 0;
  for (int i = 0; i < num_slots; ++i) n += free_slot(i) ? 1 : 0;
  return n;
}

int AgentState::disabled() const {
  int n = 0;
  for (int i = 0; i < num_slots; ++i) n += (slot_disabled[i] && slot_owner[i].empty()) ? 1 : 0;
  return n;
}

void Scheduler::add_agent(const std::string& id, int slots) {
  AgentState a;
  a.id = id;
  a.num_slots = slots;
  a.slot_owner.assign(slots, "");
  a.slot_disabled.assign(slots, 0);
  auto it = agents_.find(id);
  if (it != agents_.end()) {
    // re-registration keeps existing ownership (and disabled slots) where possible
    for (int i = 0; i < std::min<int>(slots, it->second.num_slots); ++i) {
      a.slot_owner[i] = it->second.slot_owner[i];
      a.slot_disabled[i] = it->second.slot_disabled[i];
    }
    a.enabled = it->second.enabled;
    a.zero_slot_containers = it->second.zero_slot_containers;
  }
  agents_[id] = a;
}

void Scheduler::remove_agent(const std::string& id) {
  agents_.erase(id);
  for (auto& kv : reqs_) {
    Request& r = kv.second;
    for (const auto& as : r.assignment)
      if (as.first == id) {
        r.allocated = false;
        r.assignment.clear();
        break;
      }
  }
}

void Scheduler::set_agent_enabled(const std::string& id, bool enabled) {
  auto it = agents_.find(id);
  if (it != agents_.end()) it->second.enabled = enabled;
}

bool Scheduler::set_slot_enabled(const std::string& id, int slot, bool enabled) {
  auto it = agents_.find(id);
  if (it == agents_.end() || slot < 0 || slot >= it->second.num_slots) return false;
  it->second.slot_disabled[slot] = enabled ? 0 : 1;
  return true;
}

void Scheduler::add_request(const Request& r) { reqs_[r.alloc_id] = r; }

void Scheduler::remove_request(const std::string& alloc_id) {
  auto it = reqs_.find(alloc_id);
  if (it == reqs_.end()) return;
  release(agents_, it->second);
  reqs_.erase(it);
}

void Scheduler::set_priority(const std::string& job_id, int priority) {
  for (auto& kv : reqs_)
    if (kv.second.job_id == job_id) kv.second.priority = priority;
}

void Scheduler::set_weight(const std::string& job_id, double weight) {
  for (auto& kv : reqs_)
    if (kv.second.job_id == job_id) kv.second.weight = weight;
}

void Scheduler::set_max_slots(const std::string& job_id, int max_slots) {
  if (max_slots < 0)
    max_slots_.erase(job_id);
  else
    max_slots_[job_id] = max_slots;
}

void Scheduler::set_agent_max_zero_slot(const std::string& id, int n) {
  auto it = agents_.find(id);
  if (it != agents_.end()) it->second.max_zero_slot_containers = n;
}

int Scheduler::total_slots() const {
  int n = 0;
  for (const auto& kv : agents_)
    if (kv.second.enabled) n += kv.second.usable();
  return n;
}

int Scheduler::used_slots() const {
  int n = 0;
  for (const auto& kv : agents_) n += kv.second.used();
  return n;
}

// fitting_methods.go: BestFit / WorstFit affinity scores (higher is better)
static double fit_score(const Request& r, const AgentState& a, Fit fit) {
  if (a.used() != 0 || r.slots != 0) {
    if (fit == Fit::Best) return 1.0 / (1.0 + a.empty());
    return a.usable() ? static_cast<double>(a.empty()) / a.usable() : 0.0;
  }
  return 1.0 / (1.0 + a.zero_slot_containers);
}

double Scheduler::score(const Request& r, const AgentState& a) const { return fit_score(r, a, fit_); }

// fitting.go: findFits = shared-agent fit if the request fits one agent, else dedicated
// whole-agent fits with equal free-slot counts (slots must be a multiple of per-agent slots).
bool find_fit_in(const Request& r, const std::map<std::string, AgentState>& agents, Fit fit, Fitting* out) {
  out->assignment.clear();
  // shared fit
  const AgentState* best = nullptr;
  double best_score = -1;
  auto excluded = [&r](const std::string& id) {
    return std::find(r.excluded_agents.begin(), r.excluded_agents.end(), id) != r.excluded_agents.end();
  };
  for (const auto& kv : agents) {
    const AgentState& a = kv.second;
    if (!a.enabled || excluded(a.id)) continue;
    if (r.slots > a.empty()) continue;
    if (r.slots == 0 && a.zero_slot_containers >= a.max_zero_slot_containers) continue;
    const double s = fit_score(r, a, fit);
    if (s > best_score || (s == best_score && best && a.id < best->id)) {
      best = &a;
      best_score = s;
    }
  }
  if (best) {
    std::vector<int> slots;
    for (int i = 0; i < best->num_slots && static_cast<int>(slots.size()) < r.slots; ++i)
      if (best->free_slot(i)) slots.push_back(i);
    out->assignment.emplace_back(best->id, slots);
    return true;
  }
  if (r.slots <= 1) return false;
  // dedicated multi-agent fit: group fully idle agents by slot count
  std::map<int, std::vector<const AgentState*>, std::greater<int>> by_slots;
  for (const auto& kv : agents) {
    const AgentState& a = kv.second;
    // whole-agent fits use every slot of the agent: agents with disabled slots only take shared fits
    if (!a.enabled || a.used() != 0 || a.num_slots == 0 || a.disabled() != 0 || excluded(a.id)) continue;
    by_slots[a.num_slots].push_back(&a);
  }
  for (auto& g : by_slots) {
    const int per = g.first;
    if (r.slots % per != 0) continue;
    const size_t need = static_cast<size_t>(r.slots / per);
    if (g.second.size() < need) continue;
    std::sort(g.second.begin(), g.second.end(), [](const AgentState* x, const AgentState* y) { return x->id < y->id; });
    for (size_t k = 0; k < need; ++k) {
      std::vector<int> slots(per);
      for (int i = 0; i < per; ++i) slots[i] = i;
      out->assignment.emplace_back(g.second[k]->id, slots);
    }
    return true;
  }
  return false;
}

bool Scheduler::find_fit(const Request& r, const std::map<std::string, AgentState>& agents, Fitting* out) const {
  return find_fit_in(r, agents, fit_, out);
}

void Scheduler::apply(std::map<std::string, AgentState>& agents, const std::string& alloc_id, const Fitting& f) const {
  for (const auto& as : f.assignment) {
    AgentState& a = agents.at(as.first);
    if (as.second.empty()) a.zero_slot_containers++;
    for (int s : as.second) a.slot_owner.at(s) = alloc_id;
  }
}

void Scheduler::release(std::map<std::string, AgentState>& agents, const Request& r) const {
  for (const auto& as : r.assignment) {
    auto it = agents.find(as.first);
    if (it == agents.end()) continue;
    if (as.second.empty()) it->second.zero_slot_containers = std::max(0, it->second.zero_slot_containers - 1);
    for (int s : as.second)
      if (s < it->second.num_slots && it->second.slot_owner[s] == r.alloc_id) it->second.slot_owner[s] = "";
  }
}

Decision Scheduler::schedule() {
  switch (policy_) {
    case Policy::Priority: return schedule_priority();
    case Policy::FairShare: return schedule_fair_share();
    case Policy::RoundRobin: return schedule_round_robin();
  }
  return {};
}

// priority.go:prioritySchedulerWithFilter -- per priority level (most important first), place
// pending tasks in queue order; once a level leaves work unplaced, lower levels may only
// backfill preemptible tasks; with preemption enabled an unplaced task evicts preemptible tasks
// of lower (or equal, later-queued) priority, newest first, until it fits.
Decision Scheduler::schedule_priority() {
  Decision d;
  std::vector<Request*> pending, running;
  for (auto& kv : reqs_) (kv.second.allocated ? running : pending).push_back(&kv.second);
  auto by_prio = [](const Request* a, const Request* b) {
    if (a->priority != b->priority) return a->priority < b->priority;
    return a->order < b->order;
  };
  std::sort(pending.begin(), pending.end(), by_prio);
  std::map<std::string, AgentState> local = agents_;
  std::set<std::string> to_release;
  for (auto* r : running)
    if (r->preempting) to_release.insert(r->alloc_id);
  bool backfilling = false;
  size_t i = 0;
  while (i < pending.size()) {
    const int prio = pending[i]->priority;
    std::vector<Request*> level;
    while (i < pending.size() && pending[i]->priority == prio) level.push_back(pending[i++]);
    std::vector<Request*> failed;
    for (auto* r : level) {
      Fitting f;
      if (to_release.empty() && find_fit(*r, local, &f) && (!backfilling || (preemption_ && r->preemptible))) {
        apply(local, r->alloc_id, f);
        r->allocated = true;
        r->assignment = f.assignment;
        d.allocated.push_back(r->alloc_id);
      } else {
        failed.push_back(r);
      }
    }
    if (!failed.empty()) backfilling = true;
    if (!preemption_) continue;
    for (auto* r : failed) {
      Fitting f;
      if (find_fit(*r, local, &f)) {
        apply(local, "(reserved)" + r->alloc_id, f);  // will fit once pending releases finish
        continue;
      }
      // candidates: lowest priority first (largest value), newest first
      std::vector<Request*> cands;
      for (auto* c : running)
        if (c->preemptible && !to_release.count(c->alloc_id) &&
            (c->priority > r->priority || (c->priority == r->priority && c->order > r->order)))
          cands.push_back(c);
      std::sort(cands.begin(), cands.end(), [](const Request* a, const Request* b) {
        if (a->priority != b->priority) return a->priority > b->priority;
        return a->order > b->order;
      });
      std::map<std::string, AgentState> trial = local;
      std::vector<std::string> victims;
      bool placed = false;
      for (auto* c : cands) {
        release(trial, *c);
        victims.push_back(c->alloc_id);
        if (find_fit(*r, trial, &f)) {
          apply(trial, "(reserved)" + r->alloc_id, f);
          placed = true;
          break;
        }
      }
      if (placed) {
        local = trial;
        for (const auto& v : victims) {
          to_release.insert(v);
          reqs_.at(v).preempting = true;
          d.preempt.push_back(v);
        }
      }
    }
  }
  // commit placements
  for (const auto& id : d.allocated) apply(agents_, id, Fitting{reqs_.at(id).assignment});
  return d;
}

// ---------------------------------------------------------------------------------- fair share
// fair_share.go, step for step: (1) zero-slot tasks start wherever they fit; (2) tasks grouped by job
// (slot demand capped at the group's max_slots; non-preemptible running slots are "presubscribed");
// (3) progressive filling (max-min fairness) of slot offers in weight proportion, groups sorted by
// (demand, registration), with the multi-slot deadlock breaker that disables the newest group that
// cannot start its smallest task; (4) groups above their offer release preemptible tasks, groups
// below it start pending tasks that fit.
namespace {

struct GroupState {
  std::string job;
  double weight = 0;
  int max_slots = -1;
  bool disabled = false;
  int demand = 0, active = 0, presubscribed = 0, offered = 0;
  int64_t registered = 0;  // queue position of the group's first task (JobSubmissionTime)
  std::vector<const Request*> pending, allocated;
};

double total_weight(const std::vector<GroupState*>& st) {
  double t = 0;
  for (auto* g : st)
    if (!g->disabled && g->offered < g->demand) t += g->weight;
  return t;
}

// Go: int(float64(capacity) * weight / totalWeight) truncates toward zero; a NaN / Inf quotient
// (all weights 0) converts to the minimum int64 on amd64, so Max(1, .) makes it 1.
int fair_quota(int capacity, double weight, double total) {
  const double v = static_cast<double>(capacity) * weight / total;
  if (!std::isfinite(v)) return 1;
  return std::max(1, static_cast<int>(v));
}

void account_preoffers(int& pre, int& offer) {
  if (pre > 0) {
    if (pre == offer) {
      pre = 0;
      offer = 0;
    }
    if (pre > offer) {
      pre -= offer;
      offer = 0;
    }
    if (pre < offer) {
      pre = 0;
      offer -= pre;
    }
  }
}

// The reference sorts its by-time copy with a comparator that indexes the demand-sorted slice
// (``states[i]``) instead of the copy being sorted; Go's sort.Slice runs insertion sort for fewer
// than 13 elements, which this reproduces exactly.  Larger lists fall back to the intended order
// (newest registration first).
std::vector<GroupState*> go_by_time(const std::vector<GroupState*>& states) {
  std::vector<GroupState*> out = states;
  const int n = static_cast<int>(states.size());
  if (n <= 12) {
    auto less = [&](int i, int j) { return states[i]->registered > states[j]->registered; };
    for (int i = 1; i < n; ++i)
      for (int j = i; j > 0 && less(j, j - 1); --j) std::swap(out[j], out[j - 1]);
  } else {
    std::stable_sort(out.begin(), out.end(),
                     [](const GroupState* a, const GroupState* b) { return a->registered > b->registered; });
  }
  return out;
}

void allocate_offers(std::vector<GroupState*>& states, int capacity) {
  std::map<GroupState*, int> pre;
  for (auto* g : states) {
    if (g->presubscribed == 0) continue;
    g->offered = g->presubscribed;
    pre[g] = g->presubscribed;
    capacity -= g->presubscribed;
  }
  std::sort(states.begin(), states.end(), [](const GroupState* a, const GroupState* b) {
    if (a->demand != b->demand) return a->demand < b->demand;
    return a->registered < b->registered;
  });
  const std::vector<GroupState*> by_time = go_by_time(states);
  double tw = total_weight(states);
  for (int left = static_cast<int>(states.size()); left > 0;) {
    bool progress = false;
    const int start = capacity;
    for (auto* g : states) {
      if (g->disabled || g->offered == g->demand) continue;
      const int share = fair_quota(start, g->weight, tw);
      progress = true;
      int offer = std::min({share, capacity, g->demand - g->offered});
      account_preoffers(pre[g], offer);
      g->offered += offer;
      capacity -= offer;
      if (g->offered == g->demand) {
        --left;
        tw = total_weight(states);
      }
    }
    if (capacity == 0) {
      bool adjusted = false;
      for (auto* g : by_time) {
        const Request* smallest = nullptr;
        for (const Request* r : g->pending)
          if (!smallest || r->slots < smallest->slots) smallest = r;
        if (!g->disabled && g->offered != g->demand && smallest && smallest->slots > g->offered) {
          capacity += g->offered;
          g->offered = 0;
          g->disabled = true;
          adjusted = true;
          --left;
          tw = total_weight(states);
          break;
        }
      }
      if (!adjusted) return;
    } else if (!progress) {
      return;
    }
  }
}

}  // namespace

Decision fairshare_decide(const std::vector<Request>& tasks, const std::map<std::string, FairShareGroup>& groups,
                          const std::map<std::string, AgentState>& agents, Fit fit) {
  Decision d;
  Fitting f;
  for (const Request& r : tasks)
    if (r.slots == 0 && !r.allocated && find_fit_in(r, agents, fit, &f)) d.allocated.push_back(r.alloc_id);
  int capacity = 0;
  for (const auto& kv : agents)
    if (kv.second.enabled) capacity += kv.second.usable();
  std::vector<GroupState> store;
  store.reserve(tasks.size());
  std::map<std::string, size_t> index;
  for (const Request& r : tasks) {
    if (r.slots == 0 || r.slots > capacity) continue;
    if (!r.allocated && !find_fit_in(r, agents, fit, &f)) continue;
    auto it = index.find(r.job_id);
    if (it == index.end()) {
      GroupState g;
      g.job = r.job_id;
      g.registered = r.order;
      auto gi = groups.find(r.job_id);
      if (gi != groups.end()) {
        g.weight = gi->second.weight;
        g.max_slots = gi->second.max_slots;
      }
      it = index.emplace(r.job_id, store.size()).first;
      store.push_back(g);
    }
    GroupState& g = store[it->second];
    g.demand += r.slots;
    if (!r.allocated) {
      g.pending.push_back(&r);
    } else {
      if (!r.preemptible) g.presubscribed += r.slots;
      g.allocated.push_back(&r);
      g.active += r.slots;
    }
  }
  std::vector<GroupState*> states;
  for (auto& g : store) {
    if (g.max_slots >= 0) g.demand = std::min(g.demand, g.max_slots);
    states.push_back(&g);
  }
  allocate_offers(states, capacity);
  for (auto* g : states) {
    if (g->active > g->offered) {
      for (const Request* r : g->allocated) {
        if (!r->preemptible) continue;
        d.preempt.push_back(r->alloc_id);
        g->active -= r->slots;
        if (g->active <= g->offered) break;
      }
    } else if (g->active < g->offered) {
      g->offered -= g->active;
      for (const Request* r : g->pending) {
        if (r->slots > g->offered || !find_fit_in(*r, agents, fit, &f)) continue;
        d.allocated.push_back(r->alloc_id);
        g->offered -= r->slots;
      }
    }
  }
  return d;
}

// The live pool: the fair-share decision on the current queue, then each started task placed on
// the agents as they are now (one the decision over-committed stays queued for the next pass).
Decision Scheduler::schedule_fair_share() {
  std::vector<Request> tasks;
  for (const auto& kv : reqs_) tasks.push_back(kv.second);
  std::sort(tasks.begin(), tasks.end(), [](const Request& a, const Request& b) {
    if (a.order != b.order) return a.order < b.order;
    return a.alloc_id < b.alloc_id;
  });
  std::map<std::string, FairShareGroup> groups;
  for (const Request& r : tasks) {
    FairShareGroup& g = groups[r.job_id];
    g.weight = std::max(g.weight, r.weight);
    auto ms = max_slots_.find(r.job_id);
    g.max_slots = ms == max_slots_.end() ? -1 : ms->second;
  }
  const Decision raw = fairshare_decide(tasks, groups, agents_, fit_);
  Decision d;
  if (preemption_)
    for (const auto& id : raw.preempt) {
      Request& r = reqs_.at(id);
      if (r.preempting) continue;
      r.preempting = true;
      d.preempt.push_back(id);
    }
  for (const auto& id : raw.allocated) {
    Request& r = reqs_.at(id);
    Fitting f;
    if (r.allocated || !find_fit(r, agents_, &f)) continue;
    apply(agents_, id, f);
    r.allocated = true;
    r.assignment = f.assignment;
    d.allocated.push_back(id);
  }
  return d;
}

// round_robin.go: FIFO by queue position; first task that does not fit blocks the queue.
Decision Scheduler::schedule_round_robin() {
  Decision d;
  std::vector<Request*> pending;
  for (auto& kv : reqs_)
    if (!kv.second.allocated) pending.push_back(&kv.second);
  std::sort(pending.begin(), pending.end(), [](const Request* a, const Request* b) { return a->order < b->order; });
  for (auto* r : pending) {
    Fitting f;
    if (!find_fit(*r, agents_, &f)) break;
    apply(agents_, r->alloc_id, f);
    r->allocated = true;
    r->assignment = f.assignment;
    d.allocated.push_back(r->alloc_id);
  }
  return d;
}

}  // namespace damd_native

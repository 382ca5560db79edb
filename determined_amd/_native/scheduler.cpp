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
double Scheduler::score(const Request& r, const AgentState& a) const {
  if (a.used() != 0 || r.slots != 0) {
    if (fit_ == Fit::Best) return 1.0 / (1.0 + a.empty());
    return a.usable() ? static_cast<double>(a.empty()) / a.usable() : 0.0;
  }
  return fit_ == Fit::Best ? 1.0 / (1.0 + a.zero_slot_containers) : 1.0 / (1.0 + a.zero_slot_containers);
}

// fitting.go: findFits = shared-agent fit if the request fits one agent, else dedicated
// whole-agent fits with equal free-slot counts (slots must be a multiple of per-agent slots).
bool Scheduler::find_fit(const Request& r, const std::map<std::string, AgentState>& agents, Fitting* out) const {
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
    const double s = score(r, a);
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

// fair_share.go: slots are offered to jobs in proportion to their weight (capped at demand,
// redistributed when a job wants less than its share); tasks of a job start in queue order while
// the job is under its share; jobs running above their share are preempted (newest task first)
// when another job is starved.
Decision Scheduler::schedule_fair_share() {
  Decision d;
  struct Group {
    double weight = 0;
    int demand = 0, running = 0, share = 0;
    int64_t first_order = 0;
    std::vector<Request*> pending, active;
  };
  std::map<std::string, Group> groups;
  for (auto& kv : reqs_) {
    Request& r = kv.second;
    Group& g = groups[r.job_id];
    g.weight = std::max(g.weight, r.weight);
    g.demand += r.slots;
    if (g.pending.empty() && g.active.empty()) g.first_order = r.order;
    g.first_order = std::min(g.first_order, r.order);
    if (r.allocated) {
      g.active.push_back(&r);
      g.running += r.slots;
    } else {
      g.pending.push_back(&r);
    }
  }
  const int capacity = total_slots();
  // water-filling: give each group min(demand, weight share); redistribute leftovers
  std::vector<Group*> gs;
  for (auto& kv : groups) gs.push_back(&kv.second);
  int remaining = capacity;
  std::vector<Group*> open = gs;
  while (remaining > 0 && !open.empty()) {
    double tw = 0;
    for (auto* g : open) tw += g->weight;
    if (tw <= 0) break;
    std::vector<Group*> next;
    int handed = 0;
    for (auto* g : open) {
      const int want = g->demand - g->share;
      const int offer = std::max(1, static_cast<int>(std::floor(remaining * g->weight / tw)));
      const int give = std::min(want, offer);
      g->share += give;
      handed += give;
      if (g->share < g->demand) next.push_back(g);
    }
    remaining -= handed;
    if (handed == 0) break;
    open = next;
  }
  std::sort(gs.begin(), gs.end(), [](const Group* a, const Group* b) { return a->first_order < b->first_order; });
  std::map<std::string, AgentState> local = agents_;
  bool starved = false;
  for (auto* g : gs) {
    std::sort(g->pending.begin(), g->pending.end(), [](const Request* a, const Request* b) { return a->order < b->order; });
    for (auto* r : g->pending) {
      if (g->running + r->slots > std::max(g->share, r->slots)) {
        starved = true;
        break;
      }
      Fitting f;
      if (!find_fit(*r, local, &f)) {
        starved = true;
        break;
      }
      apply(local, r->alloc_id, f);
      r->allocated = true;
      r->assignment = f.assignment;
      g->running += r->slots;
      d.allocated.push_back(r->alloc_id);
    }
  }
  if (preemption_ && starved) {
    for (auto* g : gs) {
      if (g->running <= g->share) continue;
      std::sort(g->active.begin(), g->active.end(), [](const Request* a, const Request* b) { return a->order > b->order; });
      for (auto* r : g->active) {
        if (g->running <= g->share) break;
        if (!r->preemptible || r->preempting) continue;
        r->preempting = true;
        g->running -= r->slots;
        d.preempt.push_back(r->alloc_id);
      }
    }
  }
  for (const auto& id : d.allocated) apply(agents_, id, Fitting{reqs_.at(id).assignment});
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

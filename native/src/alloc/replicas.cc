#include "alloc/replicas.h"

#include <algorithm>
#include <map>
#include <set>

namespace adp::alloc {

std::string ReplicaId(std::string_view device_id, unsigned index, std::string_view join) {
  std::string out;
  out.reserve(device_id.size() + join.size() + 6);
  out.append(device_id);
  out.append(join);
  out.append(std::to_string(index));
  return out;
}

std::string StripReplica(std::string_view id, std::string_view join) {
  size_t p = join.empty() ? std::string_view::npos : id.find(join);
  return std::string(p == std::string_view::npos ? id : id.substr(0, p));
}

std::vector<std::string> StripReplicas(const std::vector<std::string>& ids, std::string_view join) {
  std::set<std::string> uniq;
  for (const auto& id : ids) uniq.insert(StripReplica(id, join));
  return std::vector<std::string>(uniq.begin(), uniq.end());
}

const char* ReplicaPolicyName(ReplicaPolicy p) {
  return p == ReplicaPolicy::kPack ? "pack" : "spread";
}

bool ParseReplicaPolicy(std::string_view s, ReplicaPolicy* out) {
  if (s == "spread") { *out = ReplicaPolicy::kSpread; return true; }
  if (s == "pack") { *out = ReplicaPolicy::kPack; return true; }
  return false;
}

namespace {

// Replicas still available on one physical device.
struct PhysicalPool {
  bool allocated = false;
  std::vector<std::string> replicas;  // sorted at construction

  // Take a specific replica. The reference removes by swapping the last element
  // into the hole (replica.go:55-59); that order is observable through later
  // TakeAny() calls, so it is reproduced exactly.
  bool Take(const std::string& id) {
    auto it = std::find(replicas.begin(), replicas.end(), id);
    if (it == replicas.end()) return false;
    *it = replicas.back();
    replicas.pop_back();
    allocated = true;
    return true;
  }
  std::string TakeAny() {
    std::string id = replicas.front();
    replicas.erase(replicas.begin());
    allocated = true;
    return id;
  }
};

std::string MissingMsg(const std::string& id) {
  return "device '" + id + "' in mustIncludeDeviceIDs is missing from availableDeviceIDs";
}

}  // namespace

Result<Prioritized> PrioritizeDevices(const std::vector<std::string>& available,
                                      const std::vector<std::string>& must_include,
                                      int allocation_size, ReplicaPolicy policy,
                                      std::string_view join) {
  if (allocation_size < 0) return InvalidArgument("negative allocation size");
  if (static_cast<int>(must_include.size()) > allocation_size) {
    return InvalidArgument("mustIncludeDeviceIDs (" + std::to_string(must_include.size()) +
                           ") exceeds allocation size (" + std::to_string(allocation_size) + ")");
  }

  // Ordered map == the reference's sorted key walk (replica.go:142-147).
  std::map<std::string, PhysicalPool> pools;
  for (const auto& id : available) pools[StripReplica(id, join)].replicas.push_back(id);
  for (auto& [_, p] : pools) std::sort(p.replicas.begin(), p.replicas.end());

  Prioritized out;
  out.ids.reserve(allocation_size);
  bool unique = true;
  for (const auto& id : must_include) {
    auto it = pools.find(StripReplica(id, join));
    if (it == pools.end()) return NotFound(MissingMsg(id));
    if (it->second.allocated) unique = false;
    if (!it->second.Take(id)) return NotFound(MissingMsg(id));
    out.ids.push_back(id);
  }

  if (policy == ReplicaPolicy::kSpread) {
    for (int i = static_cast<int>(out.ids.size()); i < allocation_size; ++i) {
      // First priority: a physical device not yet used by this request; second:
      // the one with the most replicas left. Ties -> lexicographically first.
      PhysicalPool* best_unalloc = nullptr;
      PhysicalPool* best_alloc = nullptr;
      size_t hi_unalloc = 0, hi_alloc = 0;
      for (auto& [_, p] : pools) {
        size_t n = p.replicas.size();
        if (p.allocated) {
          if (n > hi_alloc) { best_alloc = &p; hi_alloc = n; }
        } else {
          if (n > hi_unalloc) { best_unalloc = &p; hi_unalloc = n; }
        }
      }
      PhysicalPool* pick = best_unalloc ? best_unalloc : best_alloc;
      if (!pick) return FailedPrecondition("no devices left to allocate");
      if (pick->allocated) unique = false;
      out.ids.push_back(pick->TakeAny());
    }
    out.non_unique = !unique;
  } else {
    // Pack: finish on devices this request already touches, then best-fit the
    // remainder onto as few untouched devices as possible.
    int need = allocation_size - static_cast<int>(out.ids.size());
    for (auto& [_, p] : pools) {
      while (need > 0 && p.allocated && !p.replicas.empty()) {
        out.ids.push_back(p.TakeAny());
        --need;
      }
    }
    while (need > 0) {
      PhysicalPool* fit = nullptr;     // smallest pool that fits the remainder
      PhysicalPool* largest = nullptr; // otherwise drain the largest
      for (auto& [_, p] : pools) {
        if (p.allocated || p.replicas.empty()) continue;
        size_t n = p.replicas.size();
        if (n >= static_cast<size_t>(need) && (!fit || n < fit->replicas.size())) fit = &p;
        if (!largest || n > largest->replicas.size()) largest = &p;
      }
      PhysicalPool* pick = fit ? fit : largest;
      if (!pick) return FailedPrecondition("no devices left to allocate");
      while (need > 0 && !pick->replicas.empty()) {
        out.ids.push_back(pick->TakeAny());
        --need;
      }
    }
  }
  std::sort(out.ids.begin(), out.ids.end());
  return out;
}

}  // namespace adp::alloc

#include "alloc/replicas.h"

#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstring>
#include <map>
#include <set>
#include <unordered_map>

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
  return p == ReplicaPolicy::kPack ? "pack" : p == ReplicaPolicy::kAuto ? "auto" : "spread";
}

bool ParseReplicaPolicy(std::string_view s, ReplicaPolicy* out) {
  if (s == "spread") { *out = ReplicaPolicy::kSpread; return true; }
  if (s == "pack") { *out = ReplicaPolicy::kPack; return true; }
  if (s == "auto") { *out = ReplicaPolicy::kAuto; return true; }
  return false;
}

namespace {

// Replicas still available on one physical device. Views point into the
// caller's request buffer; nothing is copied until the result is built.
struct PhysicalPool {
  std::string_view prefix;
  // prefix + join can only split at prefix.size() (no occurrence of join starts
  // inside prefix and runs into the join), so IDs of this pool can be matched
  // by two memcmps instead of a substring search.
  bool join_safe = false;
  bool allocated = false;
  std::vector<std::string_view> replicas;  // [head, end) are still available
  size_t head = 0;
  size_t sorted_upto = 0;  // [head, sorted_upto) is sorted and holds the smallest
  bool fully_sorted = false;

  size_t size() const { return replicas.size() - head; }

  // Replicas share `prefix`, so comparing the suffixes gives the reference's
  // lexicographic order (sort.Strings) at a fraction of the cost.
  bool Less(std::string_view a, std::string_view b) const {
    return a.substr(prefix.size()) < b.substr(prefix.size());
  }
  void SortAll() {
    if (fully_sorted) return;
    std::sort(replicas.begin() + head, replicas.end(),
              [this](std::string_view a, std::string_view b) { return Less(a, b); });
    fully_sorted = true;
    sorted_upto = replicas.size();
  }
  // Take a specific replica. The reference removes by swapping the last element
  // into the hole (replica.go:55-59); that order is observable through later
  // TakeAny() calls, so it is reproduced exactly (on the fully sorted list).
  bool Take(std::string_view id) {
    SortAll();
    auto it = std::find(replicas.begin() + head, replicas.end(), id);
    if (it == replicas.end()) return false;
    *it = replicas.back();
    replicas.pop_back();
    sorted_upto = replicas.size();
    allocated = true;
    return true;
  }
  // Smallest remaining replica (sort.Strings order). Sorts lazily in growing
  // chunks: a spread request takes one replica per GPU, so a 294-replica pool
  // usually needs a partial sort of a handful of elements, not a full sort.
  std::string_view TakeAny() {
    if (head == sorted_upto) {
      size_t chunk = std::min(size(), std::max<size_t>(8, 2 * (sorted_upto - 0)));
      std::partial_sort(replicas.begin() + head, replicas.begin() + head + chunk, replicas.end(),
                        [this](std::string_view a, std::string_view b) { return Less(a, b); });
      sorted_upto = head + chunk;
    }
    allocated = true;
    return replicas[head++];
  }
  // The n smallest remaining replicas, in order -- what n TakeAny() calls
  // return -- with one partial sort instead of growing chunks.
  size_t TakeSmallest(size_t n, std::vector<std::string_view>* out) {
    n = std::min(n, size());
    if (n == 0) return 0;
    if (sorted_upto < head + n) {
      std::partial_sort(replicas.begin() + head, replicas.begin() + head + n, replicas.end(),
                        [this](std::string_view a, std::string_view b) { return Less(a, b); });
      sorted_upto = head + n;
    }
    allocated = true;
    out->insert(out->end(), replicas.begin() + head, replicas.begin() + head + n);
    head += n;
    return n;
  }
};

std::string MissingMsg(std::string_view id) {
  return "device '" + std::string(id) + "' in mustIncludeDeviceIDs is missing from availableDeviceIDs";
}

std::string_view StripView(std::string_view id, std::string_view join) {
  size_t p = join.empty() ? std::string_view::npos : id.find(join);
  return p == std::string_view::npos ? id : id.substr(0, p);
}

}  // namespace

Result<Prioritized> PrioritizeDevices(const std::vector<std::string>& available,
                                      const std::vector<std::string>& must_include,
                                      int allocation_size, ReplicaPolicy policy,
                                      std::string_view join) {
  std::vector<std::string_view> a(available.begin(), available.end());
  std::vector<std::string_view> m(must_include.begin(), must_include.end());
  return PrioritizeDeviceViews(a, m, allocation_size, policy, join);
}

Result<Prioritized> PrioritizeDeviceViews(const std::vector<std::string_view>& available,
                                      const std::vector<std::string_view>& must_include,
                                      int allocation_size, ReplicaPolicy policy,
                                      std::string_view join, const DeviceAffinity* affinity) {
  if (allocation_size < 0) return InvalidArgument("negative allocation size");
  if (static_cast<int>(must_include.size()) > allocation_size) {
    return InvalidArgument("mustIncludeDeviceIDs (" + std::to_string(must_include.size()) +
                           ") exceeds allocation size (" + std::to_string(allocation_size) + ")");
  }

  // Group by physical device. Pools are then visited in lexicographic order of
  // the device ID, the reference's sorted key walk (replica.go:142-147).
  // A node has few physical devices (8 GPUs, 64 partitions) and thousands of
  // replicas: find the pool by a linear scan keyed on (length, first 8 bytes),
  // confirmed with one memcmp, instead of hashing every ID.
  std::vector<PhysicalPool> pools;
  std::vector<uint64_t> tags;
  pools.reserve(64);
  auto tag_of = [](std::string_view s) {
    uint64_t t = 0;
    memcpy(&t, s.data(), std::min<size_t>(8, s.size()));
    return t ^ (static_cast<uint64_t>(s.size()) << 56);
  };
  size_t last = SIZE_MAX;
  for (std::string_view id : available) {
    // Runs of the same device are common (the kubelet sends sorted lists):
    // check "<last prefix><join>..." before searching for the join.
    if (last != SIZE_MAX && pools[last].join_safe) {
      std::string_view pre = pools[last].prefix;
      if (id.size() >= pre.size() + join.size() &&
          memcmp(id.data(), pre.data(), pre.size()) == 0 &&
          memcmp(id.data() + pre.size(), join.data(), join.size()) == 0) {
        pools[last].replicas.push_back(id);
        continue;
      }
    }
    std::string_view dev = StripView(id, join);
    size_t at = SIZE_MAX;
    if (last != SIZE_MAX && pools[last].prefix == dev) {
      at = last;
    } else {
      uint64_t t = tag_of(dev);
      for (size_t i = 0; i < pools.size(); ++i)
        if (tags[i] == t && pools[i].prefix == dev) { at = i; break; }
      if (at == SIZE_MAX) {
        at = pools.size();
        pools.emplace_back();
        pools.back().prefix = dev;
        if (!join.empty()) {
          std::string probe(dev.substr(dev.size() - std::min(dev.size(), join.size() - 1)));
          size_t tail = probe.size();
          probe.append(join);
          pools.back().join_safe = probe.find(join) == tail;
        }
        pools.back().replicas.reserve(available.size() / 8 + 1);
        tags.push_back(t);
      }
    }
    pools[at].replicas.push_back(id);
    last = at;
  }
  auto find_pool = [&](std::string_view dev) -> PhysicalPool* {
    for (auto& p : pools)
      if (p.prefix == dev) return &p;
    return nullptr;
  };
  std::vector<PhysicalPool*> order;
  order.reserve(pools.size());
  for (auto& p : pools) order.push_back(&p);
  std::sort(order.begin(), order.end(),
            [](const PhysicalPool* x, const PhysicalPool* y) { return x->prefix < y->prefix; });

  std::vector<std::string_view> chosen;
  chosen.reserve(allocation_size);
  bool unique = true;
  for (std::string_view id : must_include) {
    PhysicalPool* found = find_pool(StripView(id, join));
    if (!found) return NotFound(MissingMsg(id));
    PhysicalPool& pool = *found;
    if (pool.allocated) unique = false;
    if (!pool.Take(id)) return NotFound(MissingMsg(id));
    chosen.push_back(id);
  }

  Prioritized out;
  out.devices.reserve(pools.size());
  for (const auto& p : pools) out.devices.emplace_back(p.prefix);
  if (policy != ReplicaPolicy::kPack) {
    for (int i = static_cast<int>(chosen.size()); i < allocation_size; ++i) {
      // First priority: a physical device not yet used by this request; second:
      // the one with the most replicas left. Ties -> lexicographically first.
      PhysicalPool* best_unalloc = nullptr;
      PhysicalPool* best_alloc = nullptr;
      size_t hi_unalloc = 0, hi_alloc = 0;
      for (PhysicalPool* p : order) {
        size_t n = p->size();
        if (p->allocated) {
          if (n > hi_alloc) { best_alloc = p; hi_alloc = n; }
        } else {
          if (n > hi_unalloc) { best_unalloc = p; hi_unalloc = n; }
        }
      }
      PhysicalPool* pick = best_unalloc ? best_unalloc : best_alloc;
      if (!pick) return FailedPrecondition("no devices left to allocate");
      if (pick->allocated) unique = false;
      chosen.push_back(pick->TakeAny());
    }
    out.non_unique = !unique;
  } else {
    // Pack: finish on devices this request already touches, then best-fit the
    // remainder onto as few untouched devices as possible.
    int need = allocation_size - static_cast<int>(chosen.size());
    for (PhysicalPool* p : order)
      if (need > 0 && p->allocated) need -= static_cast<int>(p->TakeSmallest(static_cast<size_t>(need), &chosen));
    while (need > 0) {
      // With devices already in the request, only the closest untouched ones
      // compete (NUMA/xGMI affinity); among those: best fit, else the largest.
      long best_aff = LONG_MIN;
      if (affinity) {
        for (PhysicalPool* p : order) {
          if (p->allocated || p->size() == 0) continue;
          long aff = 0;
          for (PhysicalPool* q : order)
            if (q->allocated) aff += (*affinity)(p->prefix, q->prefix);
          best_aff = std::max(best_aff, aff);
        }
      }
      PhysicalPool* fit = nullptr;      // smallest pool that fits the remainder
      PhysicalPool* largest = nullptr;  // otherwise drain the largest
      for (PhysicalPool* p : order) {
        if (p->allocated || p->size() == 0) continue;
        if (affinity) {
          long aff = 0;
          for (PhysicalPool* q : order)
            if (q->allocated) aff += (*affinity)(p->prefix, q->prefix);
          if (aff < best_aff) continue;
        }
        size_t n = p->size();
        if (n >= static_cast<size_t>(need) && (!fit || n < fit->size())) fit = p;
        if (!largest || n > largest->size()) largest = p;
      }
      PhysicalPool* pick = fit ? fit : largest;
      if (!pick) return FailedPrecondition("no devices left to allocate");
      need -= static_cast<int>(pick->TakeSmallest(static_cast<size_t>(need), &chosen));
    }
  }
  std::sort(chosen.begin(), chosen.end());
  out.ids.assign(chosen.begin(), chosen.end());
  return out;
}

}  // namespace adp::alloc

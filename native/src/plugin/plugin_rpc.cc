// The kubelet-facing RPCs of a plugin (api.proto DevicePlugin service):
// GetDevicePluginOptions, PreStartContainer, Allocate -- with the pieces it
// builds per container -- and GetPreferredAllocation. plugin.cc builds the
// units they serve and runs the plugin. Parity: the reference's
// cmd/nvidia-device-plugin/server.go:243-359.
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <charconv>
#include <chrono>
#include <cstring>

#include "common/log.h"
#include "common/strings.h"
#include "memcap/usage.h"
#include "memcap_area.h"
#include "plugin/plugin.h"
#include "proto/messages.h"
#include "proto/wire.h"

namespace adp::plugin {
namespace {

constexpr const char* kComp = "plugin";

uint64_t NowNs() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// Whether an ID occurs twice (a pod's k is small: pairwise up to 16, else sorted).
bool HasDuplicate(const std::vector<std::string>& ids) {
  if (ids.size() <= 16) {
    for (size_t i = 1; i < ids.size(); ++i)
      for (size_t j = 0; j < i; ++j)
        if (ids[i] == ids[j]) return true;
    return false;
  }
  std::vector<std::string_view> v(ids.begin(), ids.end());
  std::sort(v.begin(), v.end());
  return std::adjacent_find(v.begin(), v.end()) != v.end();
}

}  // namespace

Status Plugin::HandleGetOptions(std::string_view, std::string* resp) {
  // Preferred allocation is always offered: replicas use the prioritizer, whole
  // GPUs and partitions use the topology policy (server.go:243-248 offered it
  // only with a policy or replicas).
  pb::DevicePluginOptions o;
  o.pre_start_required = opts_.prestart_health_check;
  o.get_preferred_allocation_available = true;
  pb::Encode(o, resp);
  return Status::Ok();
}

Status Plugin::HandlePreStart(std::string_view req, std::string*) {
  pb::PreStartContainerRequest r;
  ADP_RETURN_IF_ERROR(pb::Decode(req, &r));
  if (!opts_.prestart_health_check) return Status::Ok();  // the reference's no-op (server.go:356-358)
  // --prestart-health-check: the kubelet asks right before it starts each
  // container; a device that went Unhealthy since admission stops the start
  // (the kubelet retries the container) instead of handing the workload a
  // resetting or failed GPU.
  auto law = CurrentLaw();
  for (const auto& id : r.device_ids) {
    auto it = advertised_index_.find(id);
    if (it == advertised_index_.end())
      return InvalidArgument("PreStartContainer for '" + spec_.resource_name + "': unknown device: " + id);
    if (law->healthy[it->second]) continue;
    stats_.prestart_refusals.Add(1);
    LOG_WARN(kComp, "PreStartContainer '%s': device %s is Unhealthy; container start refused",
             spec_.resource_name.c_str(), units_[it->second].id.c_str());
    return FailedPrecondition("device " + units_[it->second].id + " of '" + spec_.resource_name +
                              "' is Unhealthy; not starting the container on it");
  }
  return Status::Ok();
}

Status Plugin::HandleAllocate(std::string_view req, std::string* resp) {
  uint64_t t0 = NowNs();
  std::vector<std::vector<std::string_view>> containers;
  ADP_RETURN_IF_ERROR(pb::DecodeView(req, &containers));
  std::vector<int> us, units_per;
  // The index entry of each requested ID: one node per advertised ID, so equal
  // addresses are the same ID (distinct IDs counted without comparing strings).
  std::vector<const std::pair<const std::string_view, int>*> entries;
  std::vector<std::pair<int, uint32_t>> shares;  // (unit, replica) of CU-partitioned units
  std::string c, joined, cu_mask;
  MemoryGrant grant;
  for (const auto& ids : containers) {
    us.clear();
    shares.clear();
    entries.clear();
    for (std::string_view id : ids) {
      auto it = advertised_index_.find(id);
      if (it == advertised_index_.end())
        return InvalidArgument("invalid allocation request for '" + spec_.resource_name +
                               "': unknown device: " + std::string(id));
      us.push_back(it->second);
      if (hbm_grants_) entries.push_back(&*it);
      if (!units_[it->second].replica_cus.empty()) {
        // An advertised replica ID ends in "<join><r>" (alloc::ReplicaId).
        uint32_t r = 0, scale = 1;
        for (size_t k = id.size(); k > 0 && id[k - 1] >= '0' && id[k - 1] <= '9'; --k, scale *= 10)
          r += static_cast<uint32_t>(id[k - 1] - '0') * scale;
        shares.emplace_back(it->second, r);
      }
    }
    // Unique physical devices. uuid strategy: sorted by ID (stripReplicas order,
    // server.go:325); index strategy: enumeration order (server.go:406-411),
    // which here is unit order = KFD-node order = the container's HIP order.
    std::sort(us.begin(), us.end());
    if (hbm_grants_) {
      // Replicas (memory units / HBM shares) granted per device: distinct IDs
      // only (an ID listed twice is one unit, never twice the HBM).
      units_per.assign(units_.size(), 0);
      std::sort(entries.begin(), entries.end());
      entries.erase(std::unique(entries.begin(), entries.end()), entries.end());
      for (const auto* e : entries) ++units_per[e->second];
    }
    us.erase(std::unique(us.begin(), us.end()), us.end());
    if (unhealthy_units_.load(std::memory_order_relaxed) != 0) ADP_RETURN_IF_ERROR(CheckAllocatedHealth(us));
    grant.Clear();
    if (hbm_grants_) BuildMemoryGrant(us, units_per, &grant);
    cu_mask.clear();
    if (!shares.empty()) BuildCuMask(us, &shares, &cu_mask);
    if (opts_.id_strategy == DeviceIdStrategy::kUuid)
      std::sort(us.begin(), us.end(), [&](int a, int b) { return units_[a].id < units_[b].id; });

    c.clear();
    joined.clear();
    for (size_t i = 0; i < us.size(); ++i) {
      if (i) joined += ',';
      joined += units_[us[i]].visible_id;
    }
    AppendDeviceList(us, joined, &c);
    if (!grant.mib.empty()) {
      pb::PutMapEntry(&c, 1, kMemoryLimitEnv, grant.mib);
      pb::PutMapEntry(&c, 1, kMemoryFractionEnv, grant.frac);
      pb::PutMapEntry(&c, 1, kMemoryDevicesEnv, grant.devs);
      c += memcap_bytes_;  // the container enforces the grant (empty unless --enforce-memory-units)
      if (!memcap_bytes_.empty()) AppendGrantMounts(grant.bytes, &c);
      if (!memcap_bytes_.empty() && !opts_.memcap_usage_dir.empty()) AddUsageFile(ids, grant.bytes, &c);
    }
    if (!cu_mask.empty()) pb::PutMapEntry(&c, 1, kCuMaskEnv, cu_mask);
    if (opts_.pass_device_specs) {
      c += kfd_spec_bytes_;
      for (int u : us) c += units_[u].spec_bytes;
    }
    pb::PutLen(resp, 1, c);
    LOG_DEBUG(kComp, "allocate '%s': %zu IDs -> [%s]", spec_.resource_name.c_str(), ids.size(),
              joined.c_str());
  }
  uint64_t dt = NowNs() - t0;
  stats_.allocate_hist.Observe(dt);
  stats_.allocate_calls.Add(1);
  stats_.allocate_ns_total.Add(dt);
  stats_.allocate_ns_max.Observe(dt);
  return Status::Ok();
}

// A kubelet racing a health transition (or holding a stale device list) can
// name a device that is Unhealthy right now.
Status Plugin::CheckAllocatedHealth(const std::vector<int>& us) {
  auto law = CurrentLaw();
  for (int u : us) {
    if (law->healthy[u]) continue;
    stats_.unhealthy_allocations.Add(1);
    if (opts_.reject_unhealthy)
      return FailedPrecondition("allocation request for '" + spec_.resource_name + "': device " + units_[u].id +
                                " is Unhealthy");
    if (warned_law_[u].exchange(law->version, std::memory_order_relaxed) != law->version)
      LOG_WARN(kComp, "allocate '%s': device %s is Unhealthy (allocated anyway; --reject-unhealthy refuses)",
               spec_.resource_name.c_str(), units_[u].id.c_str());
  }
  return Status::Ok();
}

// Memory-unit resources (replicas = -1): tell the container how much HBM it
// was granted on each device so frameworks can cap themselves (e.g.
// torch.cuda.set_per_process_memory_fraction). Listed in enumeration order
// (us sorted by unit) -- the order HIP numbers the container's devices and
// HSA_CU_MASK uses -- whatever order the ID strategy gives AMD_VISIBLE_DEVICES.
// The reference hands out memory units without telling the workload.
void Plugin::BuildMemoryGrant(const std::vector<int>& us, const std::vector<int>& units_per,
                              MemoryGrant* g) const {
  char buf[32];
  for (size_t i = 0; i < us.size(); ++i) {
    const Unit& u = units_[us[i]];
    uint64_t granted = static_cast<uint64_t>(units_per[us[i]]) * u.grant_mib;
    if (i) { g->mib += ','; g->frac += ','; g->devs += ','; }
    g->devs += u.visible_id;
    g->mib += std::to_string(granted);
    g->bytes.push_back(granted << 20);
    // Under the HBM-cap shim the device reports the grant as its memory, so
    // the grant is all of what the workload sees.
    double frac = !memcap_bytes_.empty() ? 1.0 : u.vram_mib ? std::min(1.0, double(granted) / u.vram_mib) : 0.0;
    snprintf(buf, sizeof(buf), "%.4f", frac);
    g->frac += buf;
  }
}

// HSA_CU_MASK="<agent>:<first>-<last>,...;...": agents are numbered in the
// container in KFD-node order (= unit order, us is sorted by unit), and
// devices without an entry keep all their CUs. Adjacent replica shares merge.
void Plugin::BuildCuMask(const std::vector<int>& us, std::vector<std::pair<int, uint32_t>>* shares_in,
                         std::string* cu_mask) {
  auto& shares = *shares_in;
  // By unit, then by where the replica's range starts (memory-unit ranges
  // follow the IDs' lexicographic order, not the replica number).
  std::sort(shares.begin(), shares.end(), [&](const auto& a, const auto& b) {
    if (a.first != b.first) return a.first < b.first;
    const auto& ra = units_[a.first].replica_cus[a.second];
    const auto& rb = units_[b.first].replica_cus[b.second];
    return ra != rb ? ra < rb : a.second < b.second;
  });
  shares.erase(std::unique(shares.begin(), shares.end()), shares.end());
  size_t k = 0;
  for (size_t ord = 0; ord < us.size(); ++ord) {
    while (k < shares.size() && shares[k].first < us[ord]) ++k;
    if (k == shares.size() || shares[k].first != us[ord]) continue;
    const Unit& unit = units_[us[ord]];
    const auto& ranges = unit.replica_cus;
    size_t end = k;
    while (end < shares.size() && shares[end].first == us[ord]) ++end;
    // Shares are sorted by range and distinct; memory units share slots, so a
    // run of equal ranges is the units of one slot this container holds.
    auto run_end = [&](size_t g) {
      size_t h = g + 1;
      while (h < end && ranges[shares[h].second] == ranges[shares[g].second]) ++h;
      return h;
    };
    auto filled = [&](size_t g, size_t h) {
      return h - g == unit.slot_units[ranges[shares[g].second].first / unit.xcds];
    };
    // --memory-unit-cu-slots whole: keep only the slots whose units are all
    // this container's, so no neighbour runs on them. A container filling no
    // slot keeps its partial ones (it needs some CUs) and is counted.
    bool whole_only = false;
    if (!unit.slot_units.empty()) {
      for (size_t g = k; g < end && !whole_only;) {
        size_t h = run_end(g);
        whole_only = filled(g, h);
        g = h;
      }
      if (!whole_only) stats_.partial_cu_slot_allocations.Add(1);
    }
    if (!cu_mask->empty()) *cu_mask += ';';
    *cu_mask += std::to_string(ord);
    char sep = ':';
    bool open = false;
    uint32_t lo = 0, hi = 0;
    auto emit = [&] {
      *cu_mask += sep;
      *cu_mask += std::to_string(lo) + "-" + std::to_string(hi);
      sep = ',';
    };
    for (size_t g = k; g < end;) {
      size_t h = run_end(g);
      const auto& rg = ranges[shares[g].second];
      bool keep = !whole_only || filled(g, h);
      g = h;
      if (!keep) continue;
      if (open && rg.first <= hi + 1) {  // equal and adjacent ranges merge
        hi = std::max(hi, rg.second);
        continue;
      }
      if (open) emit();
      lo = rg.first;
      hi = rg.second;
      open = true;
    }
    if (open) emit();
    k = end;
  }
}

// The device list in the --device-list-strategy's form (server.go:338-346, apiEnvs/apiMounts at
// server.go:423-441; the CDI forms are this plugin's own).
void Plugin::AppendDeviceList(const std::vector<int>& us, const std::string& joined, std::string* c) const {
  switch (opts_.list_strategy) {
    case DeviceListStrategy::kEnvvar:
      pb::PutMapEntry(c, 1, opts_.envvar, joined);
      break;
    case DeviceListStrategy::kVolumeMounts:
      pb::PutMapEntry(c, 1, opts_.envvar, kVolumeMountRoot);
      for (int u : us) *c += units_[u].mount_bytes;
      break;
    case DeviceListStrategy::kCdiAnnotations: {
      if (us.empty()) break;
      std::string names;
      for (size_t i = 0; i < us.size(); ++i) {
        if (i) names += ',';
        names += std::string(kCdiVendorClass) + "=" + units_[us[i]].visible_id;
      }
      pb::PutMapEntry(c, 4, "cdi.k8s.io/amd-gpu-device-plugin_" + units_[us[0]].visible_id, names);
      break;
    }
    case DeviceListStrategy::kCdiCri:
      for (int u : us) {
        std::string n;
        pb::PutStr(&n, 1, std::string(kCdiVendorClass) + "=" + units_[u].visible_id);
        pb::PutLen(c, 5, n);
      }
      break;
  }
}

// The grant itself, read-only: the shim's caps (the env can only lower them).
// Encoded in place (a Mount: container path, host path, read-only).
void Plugin::AppendGrantMounts(const std::vector<uint64_t>& grant_bytes, std::string* c) const {
  static thread_local std::string gm, cpath, hpath;
  for (size_t i = 0; i < grant_bytes.size(); ++i) {
    char num[24];
    cpath.assign(adp_memcap::kGrantDir).push_back('/');
    cpath.append(num, static_cast<size_t>(std::to_chars(num, num + sizeof(num), i).ptr - num));
    hpath.assign(grant_dir_prefix_);
    hpath.append(num, static_cast<size_t>(std::to_chars(num, num + sizeof(num), grant_bytes[i] >> 20).ptr - num));
    hpath.append(".mib");
    gm.clear();
    pb::PutStr(&gm, 1, cpath);
    pb::PutStr(&gm, 2, hpath);
    pb::PutBool(&gm, 3, true);
    pb::PutLen(c, 2, gm);
  }
}

// The grant's accounting file (memcap/usage.h), mounted read-write where the
// shim looks for it; written by a background thread, long before the runtime
// mounts it. Without it the shim counts in the pod's /dev/shm: the cap holds
// either way, only /metrics does not see the container's use.
void Plugin::AddUsageFile(const std::vector<std::string_view>& ids, const std::vector<uint64_t>& grant_bytes,
                          std::string* c) {
  std::vector<std::string_view> sorted(ids);
  std::sort(sorted.begin(), sorted.end());
  std::string key = memcap::AllocationKeySorted(sorted);
  size_t len = sorted.size();
  for (std::string_view id : sorted) len += id.size();
  std::string joined;
  joined.reserve(len);
  for (size_t i = 0; i < sorted.size(); ++i) {
    if (i) joined += ',';
    joined += sorted[i];
  }
  std::string host;
  host.reserve(opts_.memcap_usage_dir.size() + 24);
  host.append(opts_.memcap_usage_dir).append("/").append(key).append(".memcap");
  memcap::CreateGrantFileAsync(opts_.memcap_usage_dir, std::move(key), grant_bytes, std::move(joined),
                               /*wake=*/false);  // WakeWriter() after the response is written
  pb::PutMapEntry(c, 1, kMemcapFileEnv, kMemcapUsageContainerPath);
  pb::Mount m{kMemcapUsageContainerPath, std::move(host), false};
  std::string mb;
  pb::Encode(m, &mb);
  pb::PutLen(c, 2, mb);
}

Status Plugin::HandlePreferred(std::string_view req, std::string* resp) {
  uint64_t t0 = NowNs();
  Status st = PreferredImpl(req, resp);
  uint64_t dt = NowNs() - t0;
  stats_.preferred_hist.Observe(dt);
  stats_.preferred_ns_total.Add(dt);
  stats_.preferred_ns_max.Observe(dt);
  return st;
}

Status Plugin::PreferredImpl(std::string_view req, std::string* resp) {
  // Per loop thread, kept across calls: a memory-unit request names every free
  // unit of the node (2,352 IDs on 8 MI355X), decoded into reused capacity.
  static thread_local std::vector<pb::ContainerPreferredAllocationRequestView> reqs;
  ADP_RETURN_IF_ERROR(pb::DecodeView(req, &reqs));
  pb::PreferredAllocationResponse out;
  stats_.preferred_calls.Add(1);
  for (const auto& cr : reqs) {
    if (replicated_) {
      // Multi-device pack requests grow towards the devices already chosen
      // (same NUMA node / xGMI score), the memory-unit analogue of the
      // best-effort policy below.
      alloc::DeviceAffinity affinity = [this](std::string_view a, std::string_view b) -> long {
        auto ia = unit_index_by_id_.find(a), ib = unit_index_by_id_.find(b);
        if (ia == unit_index_by_id_.end() || ib == unit_index_by_id_.end()) return 0;
        return graph_.Score(ia->second, ib->second);
      };
      auto res = alloc::PrioritizeDeviceViews(cr.available, cr.must_include, cr.allocation_size,
                                              replica_policy_, alloc::kReplicaJoin, &affinity);
      if (!res.ok()) return res.status();
      if (HasDuplicate(res->ids)) {
        // An ID listed twice in availableDeviceIDs was chosen twice: choose
        // again from the de-duplicated list (off the common path).
        std::vector<std::string_view> avail(cr.available.begin(), cr.available.end());
        std::sort(avail.begin(), avail.end());
        avail.erase(std::unique(avail.begin(), avail.end()), avail.end());
        res = alloc::PrioritizeDeviceViews(avail, cr.must_include, cr.allocation_size, replica_policy_,
                                           alloc::kReplicaJoin, &affinity);
        if (!res.ok()) return res.status();
      }
      // Physical devices must be ours (reference: NewDevicesFrom fails on an
      // unknown UUID, server.go:274-278) -- one lookup per device, not per
      // replica -- and so must every ID handed back (of the final choice: an
      // ID the kubelet made up, e.g. "<uuid>-replica-1x", names a device of
      // ours but was never advertised).
      for (const auto& dev : res->devices)
        if (!unit_index_by_id_.count(dev))
          return InvalidArgument("unable to retrieve list of available devices: unknown device " + dev);
      for (const auto& id : res->ids)
        if (!advertised_index_.count(id))
          return InvalidArgument("unable to retrieve list of available devices: unknown device " + id);
      if (res->non_unique) LOG_DEBUG(kComp, "ignoring: %s", alloc::kNonUniqueMessage);
      out.container_responses.push_back(std::move(res->ids));
      continue;
    }
    std::vector<int> avail, must;
    for (std::string_view id : cr.available) {
      auto it = advertised_index_.find(id);
      if (it == advertised_index_.end())
        return InvalidArgument("unable to retrieve list of available devices: unknown device " +
                               std::string(id));
      avail.push_back(it->second);
    }
    for (std::string_view id : cr.must_include) {
      auto it = advertised_index_.find(id);
      if (it == advertised_index_.end())
        return InvalidArgument("unable to retrieve list of required devices: unknown device " +
                               std::string(id));
      must.push_back(it->second);
    }
    std::vector<std::string> ids;
    for (int u : CachedBestEffort(avail, must, cr.allocation_size))
      ids.push_back(units_[u].id);  // advertised ID (no replica suffix here), fixes B6
    out.container_responses.push_back(std::move(ids));
  }
  pb::Encode(out, resp);
  return Status::Ok();
}

void Plugin::Unmap::operator()(std::atomic<uint16_t>* p) const { munmap(p, kBestEffortCacheBytes); }

std::vector<int> Plugin::CachedBestEffort(const std::vector<int>& avail, const std::vector<int>& must,
                                          int size) {
  // Up to 8 devices the answer is a pure function of (available set, required
  // set, size) over an immutable graph: 256 x 256 x 9 entries of 16 bits,
  // filled lazily (0 = not computed, else 1 + result mask, kEmpty = no answer).
  constexpr int kMax = 8;
  constexpr uint16_t kEmpty = 0x200;
  const int n = static_cast<int>(units_.size());
  if (n > kMax || size < 0 || size > kMax || !best_effort_cache_)
    return alloc::BestEffortAllocate(graph_, avail, must, size);
  uint32_t am = 0, rm = 0;
  for (int u : avail) am |= 1u << u;
  for (int u : must) rm |= 1u << u;
  if ((rm & ~am) != 0) return {};
  std::atomic<uint16_t>& slot =
      best_effort_cache_.get()[(am * 256u + rm) * (kMax + 1) + static_cast<uint32_t>(size)];
  uint16_t v = slot.load(std::memory_order_relaxed);
  if (v == 0) {
    std::vector<int> r = alloc::BestEffortAllocate(graph_, avail, must, size);
    uint32_t mask = 0;
    for (int u : r) mask |= 1u << u;
    v = r.empty() ? kEmpty : static_cast<uint16_t>(1 + mask);
    slot.store(v, std::memory_order_relaxed);  // racing writers store the same value
  }
  std::vector<int> out;
  if (v == kEmpty) return out;
  for (uint32_t m = v - 1u; m; m &= m - 1) out.push_back(__builtin_ctz(m));
  return out;
}

}  // namespace adp::plugin

#include "strategy/strategy.h"

#include <set>

#include "common/log.h"
#include "common/strings.h"

namespace adp::strategy {
namespace {
constexpr const char* kComp = "strategy";
}

bool ValidResourceName(std::string_view n) {
  // Kubernetes qualified-name part: [A-Za-z0-9]([-A-Za-z0-9_.]*[A-Za-z0-9])?, <= 63 chars.
  if (n.empty() || n.size() > 63) return false;
  auto alnum = [](char c) { return std::isalnum(static_cast<unsigned char>(c)) != 0; };
  if (!alnum(n.front()) || !alnum(n.back())) return false;
  for (char c : n)
    if (!alnum(c) && c != '-' && c != '_' && c != '.') return false;
  return true;
}

Result<ResourceConfig> ResourceConfig::Parse(std::string_view spec) {
  ResourceConfig rc;
  for (const auto& raw : Split(spec, ',')) {
    std::string entry = Trim(raw);
    if (entry.empty()) continue;
    auto parts = Split(entry, ':');
    if (parts.size() != 3 && parts.size() != 4)
      return InvalidArgument("'" + entry + "': an entry must have three parts separated by a colon "
                             "(<original>:<new>:<replicas>), optionally a fourth (:spread or :pack)");
    std::string orig = Trim(parts[0]), name = Trim(parts[1]);
    if (!ValidResourceName(orig)) return InvalidArgument("'" + entry + "': invalid original resource name");
    if (!ValidResourceName(name)) return InvalidArgument("'" + entry + "': invalid new resource name");
    auto n = ParseInt(Trim(parts[2]));
    if (!n || *n > INT32_MAX || *n < INT32_MIN) return InvalidArgument("'" + entry + "': replica must be an integer");
    Variant v;
    v.name = name;
    if (*n == -1) {
      v.auto_replicas = true;
      v.replicas = 1;
    } else if (*n >= 1) {
      v.replicas = static_cast<unsigned>(*n);
    } else {
      return InvalidArgument("'" + entry + "': replicas must be a positive integer or -1 (auto)");
    }
    if (parts.size() == 4) {
      std::string pol = Trim(parts[3]);
      if (!alloc::ParseReplicaPolicy(pol, &v.policy))
        return InvalidArgument("'" + entry + "': replica policy must be spread, pack or auto");
    }
    if (rc.entries_.count(orig)) LOG_WARN(kComp, "duplicate resource-config entry for '%s'; last wins", orig.c_str());
    rc.entries_[orig] = v;
  }
  return rc;
}

Variant ResourceConfig::Get(const std::string& original) const {
  auto it = entries_.find(original);
  if (it != entries_.end()) return it->second;
  Variant v;
  v.name = original;
  return v;
}

std::string ResourceConfig::ToJson() const {
  std::string out = "{";
  bool first = true;
  for (const auto& [k, v] : entries_) {
    if (!first) out += ", ";
    first = false;
    out += "\"" + JsonEscape(k) + "\": {\"Name\": \"" + JsonEscape(v.name) +
           "\", \"Replicas\": " + std::to_string(v.replicas) +
           ", \"AutoReplicas\": " + (v.auto_replicas ? "true" : "false") +
           (v.policy == alloc::ReplicaPolicy::kAuto ? std::string()
                                                    : std::string(", \"Policy\": \"") + alloc::ReplicaPolicyName(v.policy) + "\"") +
           "}";
  }
  return out + "}";
}

bool ParsePartitionStrategy(std::string_view s, PartitionStrategy* out) {
  if (s == "none") { *out = PartitionStrategy::kNone; return true; }
  if (s == "single") { *out = PartitionStrategy::kSingle; return true; }
  if (s == "mixed") { *out = PartitionStrategy::kMixed; return true; }
  return false;
}

std::string PartitionInvalidReason(const inventory::PhysicalGpu& g) {
  if (!g.partitioned()) return "not partitioned";
  // Memory partitions (NPSn) must split evenly over compute partitions: NPS4
  // with DPX (2 partitions) has no consistent per-partition memory domain.
  if (StartsWith(g.memory_mode, "NPS")) {
    auto nps = ParseInt(std::string_view(g.memory_mode).substr(3));
    if (nps && *nps > 0 && g.partitions.size() % static_cast<size_t>(*nps) != 0)
      return "memory mode " + g.memory_mode + " incompatible with " +
             std::to_string(g.partitions.size()) + " compute partitions";
  }
  const auto& p0 = g.partitions.front();
  for (const auto& p : g.partitions) {
    if (p.render_path.empty()) return "partition without render node";
    if (p.vram_mib != p0.vram_mib || p.xcds != p0.xcds) return "partitions are not uniform";
  }
  return "";
}

namespace {
Result<std::vector<PluginSpec>> BuildSpecs(const inventory::Snapshot& snap, PartitionStrategy strategy,
                                           const ResourceConfig& rc, const std::string& prefix);
}  // namespace

Result<std::vector<PluginSpec>> BuildPluginSpecs(const inventory::Snapshot& snap,
                                                 PartitionStrategy strategy,
                                                 const ResourceConfig& rc,
                                                 const std::string& prefix) {
  auto specs = BuildSpecs(snap, strategy, rc, prefix);
  if (!specs.ok()) return specs;
  // An entry keyed by something that is neither "gpu" nor a partition profile
  // present on this node renames nothing (typo, or a profile of another node).
  std::set<std::string> known = {"gpu"};
  for (const auto& g : snap.gpus)
    if (g.partitioned()) known.insert(g.PartitionProfile());
  for (const auto& [orig, v] : rc.entries())
    if (!known.count(orig))
      LOG_WARN(kComp, "resource-config entry '%s:%s' matches no resource on this node (known: %s)", orig.c_str(),
               v.name.c_str(), Join(std::vector<std::string>(known.begin(), known.end()), ", ").c_str());
  return specs;
}

namespace {
Result<std::vector<PluginSpec>> BuildSpecs(const inventory::Snapshot& snap, PartitionStrategy strategy,
                                           const ResourceConfig& rc, const std::string& prefix) {
  auto full_gpu_plugin = [&](bool skip_partitioned) {
    PluginSpec s;
    s.original = "gpu";
    s.variant = rc.Get("gpu");
    s.resource_name = prefix + "/" + s.variant.name;
    s.socket_name = "amd-gpu.sock";
    for (const auto& g : snap.gpus) {
      if (skip_partitioned && g.partitioned()) continue;
      s.devices.push_back({g.index, -1});
    }
    return s;
  };

  std::vector<PluginSpec> out;
  switch (strategy) {
    case PartitionStrategy::kNone:
      // Whole GPUs even if partitioned (mig-strategy.go:99 "Enumerate device even
      // if MIG enabled"): a partitioned GPU is handed out with all its render nodes.
      out.push_back(full_gpu_plugin(false));
      return out;

    case PartitionStrategy::kSingle: {
      std::vector<const inventory::PhysicalGpu*> parted, whole;
      for (const auto& g : snap.gpus) (g.partitioned() ? parted : whole).push_back(&g);
      if (parted.empty()) {
        LOG_INFO(kComp, "no partitioned GPUs found; falling back to partitionStrategy=none");
        return BuildSpecs(snap, PartitionStrategy::kNone, rc, prefix);
      }
      if (!whole.empty())
        return FailedPrecondition(
            "for partitionStrategy=single all GPUs on the node must be in the same compute "
            "partition mode (found SPX and partitioned GPUs)");
      std::set<std::string> profiles;
      for (const auto* g : parted) {
        std::string why = PartitionInvalidReason(*g);
        if (!why.empty())
          return FailedPrecondition("GPU " + g->bdf + " has an unsupported partition layout: " + why);
        profiles.insert(g->PartitionProfile());
      }
      if (profiles.size() != 1)
        return FailedPrecondition("more than one partition profile present on node: " +
                                  Join(std::vector<std::string>(profiles.begin(), profiles.end()), ", "));
      PluginSpec s;
      s.original = "gpu";
      // Rename: a profile-specific entry wins, else the "gpu" entry (fix B3).
      s.variant = rc.Has(*profiles.begin()) ? rc.Get(*profiles.begin()) : rc.Get("gpu");
      s.resource_name = prefix + "/" + s.variant.name;
      s.socket_name = "amd-gpu.sock";
      for (const auto* g : parted)
        for (size_t p = 0; p < g->partitions.size(); ++p) s.devices.push_back({g->index, static_cast<int>(p)});
      out.push_back(std::move(s));
      return out;
    }

    case PartitionStrategy::kMixed: {
      out.push_back(full_gpu_plugin(true));
      std::map<std::string, std::vector<alloc::DeviceRef>> by_profile;
      for (const auto& g : snap.gpus) {
        if (!g.partitioned()) continue;
        std::string why = PartitionInvalidReason(g);
        if (!why.empty()) {
          LOG_WARN(kComp, "skipping partitions of GPU %s: %s", g.bdf.c_str(), why.c_str());
          continue;
        }
        auto& v = by_profile[g.PartitionProfile()];
        for (size_t p = 0; p < g.partitions.size(); ++p) v.push_back({g.index, static_cast<int>(p)});
      }
      for (auto& [profile, devs] : by_profile) {
        PluginSpec s;
        s.original = profile;
        s.variant = rc.Get(profile);  // fix B3: rename applies to partition resources
        s.resource_name = prefix + "/" + s.variant.name;
        s.socket_name = "amd-" + profile + ".sock";
        s.devices = std::move(devs);
        out.push_back(std::move(s));
      }
      return out;
    }
  }
  return InvalidArgument("unknown partition strategy");
}
}  // namespace

}  // namespace adp::strategy

// Resource configuration (rename + time-slice replicas) and the partition
// strategy that turns an inventory snapshot into a set of device plugins.
//
// Parity:
//  * `--resource-config "<orig>:<new>:<replicas>,..."`, `-1` = auto replicas from
//    memory: reference cmd/nvidia-device-plugin/main.go:123-129 (flag),
//    main.go:171-203 (parser), mig-strategy.go:58-76 (variant / Get()).
//  * migStrategy none|single|mixed: mig-strategy.go:31-56, 94-278, re-expressed as
//    partitionStrategy over MI355X compute partitions (SPX/DPX/QPX/CPX) x memory
//    partitions (NPS1/2/4/8).
//
// Deliberate fixes:
//  B2  a resource without an entry gets 1 replica (reference: 0 -> nothing advertised)
//  B3  renames apply to partition resources in single and mixed mode
//  B4  auto replicas use each partition's own VRAM share, not the parent GPU's
//  B10 the parse error names the right separator (':')
//  B11 replicas < -1 (or 0) are rejected instead of wrapping to a huge uint
#pragma once

#include <map>
#include <string>
#include <string_view>
#include <vector>

#include "alloc/replicas.h"
#include "alloc/topology.h"
#include "common/status.h"
#include "inventory/inventory.h"

namespace adp::strategy {

struct Variant {
  std::string name;
  unsigned replicas = 1;
  bool auto_replicas = false;
  // Optional 4th field of the entry, "<orig>:<new>:<replicas>:<policy>": how
  // GetPreferredAllocation picks this resource's replicas (spread | pack),
  // overriding --replica-policy. kAuto = not given.
  alloc::ReplicaPolicy policy = alloc::ReplicaPolicy::kAuto;
};

class ResourceConfig {
 public:
  static Result<ResourceConfig> Parse(std::string_view spec);
  // The entry for `original`, or {original, 1 replica, no auto}.
  Variant Get(const std::string& original) const;
  bool Has(const std::string& original) const { return entries_.count(original) > 0; }
  const std::map<std::string, Variant>& entries() const { return entries_; }
  std::string ToJson() const;

 private:
  std::map<std::string, Variant> entries_;
};

bool ValidResourceName(std::string_view name);

enum class PartitionStrategy { kNone, kSingle, kMixed };
bool ParsePartitionStrategy(std::string_view s, PartitionStrategy* out);

struct PluginSpec {
  std::string original;       // "gpu" or a partition profile such as "cpx-1xcd.36gb"
  std::string resource_name;  // "amd.com/<variant name>"
  std::string socket_name;    // "amd-gpu.sock", "amd-<profile>.sock"
  Variant variant;
  std::vector<alloc::DeviceRef> devices;
};

// Returns the plugins to run (possibly with zero devices; the supervisor skips
// those, like main.go:264-268). Errors are configuration errors (e.g. single
// strategy on a node with mixed partition modes).
Result<std::vector<PluginSpec>> BuildPluginSpecs(const inventory::Snapshot& snap,
                                                 PartitionStrategy strategy,
                                                 const ResourceConfig& rc,
                                                 const std::string& prefix = "amd.com");

// Why a partitioned GPU cannot be exposed as a partition resource ("" = valid).
std::string PartitionInvalidReason(const inventory::PhysicalGpu& g);

}  // namespace adp::strategy

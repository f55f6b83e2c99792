// Time-slice replica IDs and the replica-aware preferred-allocation prioritizer.
//
// Parity:
//  * ID scheme `<device-id>-replica-<i>`: reference cmd/nvidia-device-plugin/replica.go:26
//    and server.go:98-111.
//  * StripReplica / StripReplicas (dedupe + sort): replica.go:28-45.
//  * PrioritizeDevices (spread): replica.go:96-198, including its determinism
//    (lexicographic device order, sorted replica lists, swap-remove when a
//    must-include replica is taken) and its error strings
//    ("no devices left to allocate", "device '%s' in mustIncludeDeviceIDs is
//    missing from availableDeviceIDs"). The 15 reference test vectors
//    (replica_test.go:37-96) are pinned in tests/test_replicas.py and
//    native/tests/unit_tests.cc.
//
// Differences (deliberate):
//  * `len(mustInclude) > size` returns InvalidArgument instead of panicking in
//    make() (defect B12); a negative size likewise.
//  * ReplicaPolicy::kPack: for memory-unit resources (e.g. `gpu-mem-gb`, one
//    replica = 1000 MiB of one GPU) spreading a 20-unit request over 8 GPUs is
//    wrong -- the memory must come from one device. Pack keeps the request on
//    as few physical devices as possible, best-fit first (defect B19).
#pragma once

#include <functional>
#include <string>
#include <string_view>
#include <vector>

#include "common/status.h"

namespace adp::alloc {

inline constexpr std::string_view kReplicaJoin = "-replica-";

std::string ReplicaId(std::string_view device_id, unsigned index,
                      std::string_view join = kReplicaJoin);
// Everything before the first occurrence of `join` (the whole string if absent).
std::string StripReplica(std::string_view id, std::string_view join = kReplicaJoin);
// Physical IDs, de-duplicated and sorted.
std::vector<std::string> StripReplicas(const std::vector<std::string>& ids,
                                       std::string_view join = kReplicaJoin);

// kAuto is resolved per resource by the plugin (memory units -> pack, time-slice
// replicas -> spread); the prioritizer itself treats it as spread.
enum class ReplicaPolicy { kSpread, kPack, kAuto };
const char* ReplicaPolicyName(ReplicaPolicy p);
bool ParseReplicaPolicy(std::string_view s, ReplicaPolicy* out);

struct Prioritized {
  std::vector<std::string> ids;  // sorted
  // The physical devices the available IDs name (replica suffix stripped), in
  // first-seen order: callers check them against their device table, as the
  // reference does with gpuallocator.NewDevicesFrom (server.go:274-278).
  std::vector<std::string> devices;
  // True when more than one replica of the same physical device was chosen in
  // spread mode (the reference's NonUniqueError, which the caller only logs).
  bool non_unique = false;
};

inline constexpr const char* kNonUniqueMessage =
    "allocation resulted in non-unique devices due to requesting multiple GPU replicas and not "
    "having enough physical GPUs";

// Zero-copy variant (views into the request buffer); the daemon's RPC path.
// Affinity between two physical devices (by ID), higher = closer. Used by the
// pack policy when a request spans several devices: after the first device,
// the next one is the closest to those already chosen (NUMA / xGMI), and only
// then the best fit.
using DeviceAffinity = std::function<long(std::string_view a, std::string_view b)>;

Result<Prioritized> PrioritizeDeviceViews(const std::vector<std::string_view>& available,
                                      const std::vector<std::string_view>& must_include,
                                      int allocation_size,
                                      ReplicaPolicy policy = ReplicaPolicy::kSpread,
                                      std::string_view join = kReplicaJoin,
                                      const DeviceAffinity* affinity = nullptr);
Result<Prioritized> PrioritizeDevices(const std::vector<std::string>& available,
                                      const std::vector<std::string>& must_include,
                                      int allocation_size,
                                      ReplicaPolicy policy = ReplicaPolicy::kSpread,
                                      std::string_view join = kReplicaJoin);

}  // namespace adp::alloc

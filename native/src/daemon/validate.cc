#include "daemon/validate.h"

#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "alloc/replicas.h"
#include "common/log.h"
#include "common/strings.h"
#include "health/health.h"
#include "health/relay.h"
#include "inventory/inventory.h"
#include "memcap/usage.h"
#include "plugin/plugin.h"
#include "smi/smi.h"
#include "strategy/strategy.h"

namespace adp::daemon {

// The HBM-cap shim shipped with the daemon: --memcap-lib, else next to the
// binary, else the image's library directory. "" if none exists.
std::string MemcapSource(const Flags& f) {
  struct stat st;
  if (!f.memcap_lib.empty()) return stat(f.memcap_lib.c_str(), &st) == 0 ? f.memcap_lib : "";
  char exe[4096];
  ssize_t n = readlink("/proc/self/exe", exe, sizeof(exe) - 1);
  std::vector<std::string> cands;
  if (n > 0) {
    std::string self(exe, static_cast<size_t>(n));
    cands.push_back(self.substr(0, self.rfind('/') + 1) + "libadp_memcap.so");
  }
  cands.push_back("/usr/lib/amdgpu-device-plugin/libadp_memcap.so");
  for (const auto& c : cands)
    if (stat(c.c_str(), &st) == 0) return c;
  return "";
}

Result<Validated> Validate(const Config& cfg) {
  Validated v;
  const Flags& f = cfg.flags;
  if (!strategy::ParsePartitionStrategy(f.partition_strategy, &v.partition))
    return InvalidArgument("invalid --partition-strategy option: " + f.partition_strategy);
  if (!plugin::ParseDeviceListStrategy(f.device_list_strategy, &v.popts.list_strategy))
    return InvalidArgument("invalid --device-list-strategy option: " + f.device_list_strategy);
  if (!plugin::ParseDeviceIdStrategy(f.device_id_strategy, &v.popts.id_strategy))
    return InvalidArgument("invalid --device-id-strategy option: " + f.device_id_strategy);
  if (!alloc::ParseReplicaPolicy(f.replica_policy, &v.popts.replica_policy))
    return InvalidArgument("invalid --replica-policy option: " + f.replica_policy);
  auto rc = strategy::ResourceConfig::Parse(f.resource_config);
  if (!rc.ok())
    return InvalidArgument("invalid --resource-config option: '" + f.resource_config + "' " +
                           rc.status().message());
  v.rc = std::move(*rc);
  v.popts.plugin_dir = f.plugin_dir;
  v.popts.kubelet_socket = f.kubelet_socket;
  v.popts.pass_device_specs = f.pass_device_specs;
  v.popts.replica_cu_mask = f.replica_cu_mask;
  if (f.memory_unit_cu_slots != "proportional" && f.memory_unit_cu_slots != "whole")
    return InvalidArgument("invalid --memory-unit-cu-slots option: " + f.memory_unit_cu_slots +
                           " (proportional | whole)");
  v.popts.whole_cu_slots = f.memory_unit_cu_slots == "whole";
  if (f.http2_server != "native" && f.http2_server != "nghttp2")
    return InvalidArgument("invalid --http2-server option: " + f.http2_server);
  v.popts.native_http2 = f.http2_server == "native";
  if (f.loop_affinity != "peer-l3" && f.loop_affinity != "none")
    return InvalidArgument("invalid --loop-affinity option: " + f.loop_affinity);
  v.popts.follow_peer_l3 = f.loop_affinity == "peer-l3";
  v.popts.driver_root = f.driver_root;
  v.popts.auto_replica_unit_mib = f.auto_replica_unit_mib;
  if (f.auto_replica_unit != "auto" && f.auto_replica_unit != "mib" && f.auto_replica_unit != "cu-slot")
    return InvalidArgument("invalid --auto-replica-unit option: " + f.auto_replica_unit + " (auto | mib | cu-slot)");
  v.popts.cu_slot_units = f.auto_replica_unit == "cu-slot" || (f.auto_replica_unit == "auto" && f.replica_cu_mask);
  v.popts.server_threads = static_cast<int>(std::min<uint64_t>(f.server_threads, 64));
  v.popts.trace = f.trace;
  v.popts.busy_poll_us = static_cast<int>(std::min<uint64_t>(f.busy_poll_us, 100000));
  v.popts.cdi_spec_dir = f.cdi_spec_dir;
  v.popts.reject_unhealthy = f.reject_unhealthy;
  v.popts.replica_hbm_share = f.replica_hbm_share;
  v.popts.prestart_health_check = f.prestart_health_check;
  if (f.enforce_memory_units && MemcapSource(f).empty())
    return InvalidArgument("--enforce-memory-units: libadp_memcap.so not found (" +
                           (f.memcap_lib.empty() ? std::string("next to the binary or in /usr/lib/amdgpu-device-plugin")
                                                 : f.memcap_lib) + "); set --memcap-lib");
  auto extra = health::ParseEventTypes(f.health_event_extra_types);
  if (!extra.ok()) return InvalidArgument("invalid --health-event-extra-types option: " + extra.status().message());
  v.extra_event_types = std::move(*extra);
  v.bopts.driver_root = f.driver_root;
  v.bopts.sysfs_root = f.sysfs_root;
  v.bopts.include_card_nodes = f.include_card_nodes;
  std::string devs = Trim(f.devices);
  if (!devs.empty() && devs != "all") {
    for (const auto& d : Split(devs, ',')) {
      std::string t = Trim(d);
      if (t.empty()) continue;
      if (auto n = ParseUint(t)) v.bopts.only_gpus.push_back(static_cast<int>(*n));
      else v.bopts.only_ids.push_back(t);  // GPU UUID or PCI address
    }
  }
  return v;
}

}  // namespace adp::daemon

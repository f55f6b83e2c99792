// The daemon's own Prometheus families: everything /metrics serves that is not
// a plugin's -- build and restarts, the health machinery (events, polls, ECC
// and retired-page reads, event gaps), per-GPU failure causes and polled
// recoveries, amdsmi events per GPU, HBM per GPU, device-node access, the
// kubelet PodResources link and the driver-side HBM check. The plugins'
// families (resources, RPCs, allocations, grants) are plugin_metrics.cc.
//
// Parity: the reference serves no metrics; its supervisor is
// /root/reference/cmd/nvidia-device-plugin/main.go:205-326. Fed by a plain
// struct the supervisor fills, so the exposition is testable on its own.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "health/health.h"
#include "inventory/inventory.h"
#include "memcap/driver_usage.h"

namespace adp::daemon {

struct DaemonMetricsInput {
  std::string smi_version;
  uint64_t restarts = 0;
  const health::HealthCounters* health = nullptr;  // required
  // The served GPUs: failure bits (health::FailBits) and whether the GPU waits
  // for GPU_POST_RESET across an event gap (the polled check will end it).
  struct Gpu {
    std::string bdf;
    uint32_t fail = 0;
    bool awaiting_polled_recovery = false;
  };
  std::vector<Gpu> gpus;
  std::vector<inventory::NodeAccess> node_access;
  int pod_resources_up = -1;  // -1: no PodResources socket configured
  const memcap::DriverHbmMonitor::Snapshot* driver_hbm = nullptr;  // null: the check is off
  // Per resource: restarts that changed what its IDs mean while running pods held some.
  std::map<std::string, uint64_t> layout_changes_live;
  // --defer-layout-changes: resources whose config change waits for running pods.
  std::vector<std::string> deferred_layouts;
};

void AppendDaemonMetrics(const DaemonMetricsInput& in, std::string* out);

}  // namespace adp::daemon

// A synthetic MI355X node snapshot (no amdsmi): `gpus` GPUs of `parts` compute
// partitions each, fully connected by xGMI, NUMA 0 for the first four GPUs and
// 1 for the rest. Shared by the handler microbenchmark and the fuzz targets.
// `kfd`: the KFD topology nodes (the order HIP numbers a container's devices):
// 0 unreported, 1 in amdsmi's enumeration order, 2 in the reverse order.
#pragma once

#include <cstdio>
#include <memory>
#include <vector>

#include "inventory/inventory.h"

namespace adp::testing {

inline std::shared_ptr<const inventory::Snapshot> NodeModel(int gpus, int parts, int kfd = 0) {
  std::vector<smi::ProcessorInfo> procs;
  for (int g = 0; g < gpus; ++g) {
    for (int p = 0; p < parts; ++p) {
      smi::ProcessorInfo pi;
      char uuid[64];
      snprintf(uuid, sizeof(uuid), "%08x-0000-1%x00-80c0-bf9907890000", 0x75a30000 + g, p);
      pi.uuid = uuid;
      pi.bdf_id = (static_cast<uint64_t>(0x0c + 0x20 * g) << 8) | static_cast<uint64_t>(p);
      pi.render_minor = 128 + 8 * g + p;
      pi.numa_node = g < 4 ? 0 : 1;
      pi.vram_mib = 294896 / parts;
      pi.compute_partition = parts == 1 ? "SPX" : "CPX";
      pi.memory_partition = parts == 1 ? "NPS1" : "NPS2";
      pi.partition_id = p;
      pi.num_cu = 256 / parts;
      pi.xcd_count = 8 / parts;
      if (kfd == 1) pi.kfd_node = static_cast<uint32_t>(2 + g * parts + p);
      if (kfd == 2) pi.kfd_node = static_cast<uint32_t>(2 + (gpus - 1 - g) * parts + p);
      procs.push_back(pi);
    }
  }
  inventory::BuildOptions opt;
  opt.sysfs_root = "";  // nothing of this machine's /sys
  auto s = inventory::GroupProcessors(procs, opt);
  auto& snap = *s;
  size_t n = snap->gpus.size();
  for (size_t a = 0; a < n; ++a)
    for (size_t b = 0; b < n; ++b)
      if (a != b) {
        snap->gpu_links[a * n + b] = inventory::LinkClass::kXgmi;
        snap->gpu_hops[a * n + b] = 1;
      }
  return snap;
}

}  // namespace adp::testing

// Immutable node inventory: physical GPUs, their compute partitions, device
// nodes, NUMA affinity, VRAM and the device-to-device link matrix.
//
// Parity (what the reference enumerates, and where):
//  * Device{ID, Health, Topology(NUMA), Paths, Index, TotalMemory}:
//    cmd/nvidia-device-plugin/nvidia.go:40-46, buildDevice nvidia.go:162-179.
//  * Full GPUs: GpuDeviceManager.Devices nvidia.go:87-111 (index "i").
//  * MIG slices: MigDeviceManager.Devices nvidia.go:114-150 (index "i:j"),
//    capability-device resolution mig.go:121-226.
//  * gpuallocator device graph: vendor/github.com/NVIDIA/go-gpuallocator/gpuallocator/device.go:15-95.
//
// MI355X-native design:
//  * A physical GPU in SPX mode is one amdsmi processor handle with one render
//    node. In DPX/QPX/CPX mode amdsmi reports one handle per compute partition,
//    each with its own /dev/dri/renderD<N> and its own share of HBM3E. There are
//    no capability files: a partition is handed to a container purely by its
//    render node plus the shared /dev/kfd.
//  * Partitions of one GPU share the PCI bus/device (function differs), which is
//    how they are grouped back into a physical GPU.
//  * The snapshot is built once per (re)start with cheap queries only and never
//    touched again on the RPC path (the reference re-enumerates NVML on every
//    GetPreferredAllocation call, defect B5).
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "common/status.h"
#include "smi/smi.h"

namespace adp::inventory {

inline constexpr uint32_t kNoKfdNode = 0xffffffffu;  // amdsmi did not report the KFD node

struct Partition {
  int handle = -1;            // index into Snapshot::procs
  uint32_t partition_id = 0;  // amdsmi kfd current_partition_id
  std::string uuid;           // stable device ID for this partition
  std::string bdf;            // the partition's PCI address as amdsmi reports it (a function of the GPU's)
  std::string render_path;    // /dev/dri/renderD<N>
  std::string card_path;      // /dev/dri/card<N> ("" if unknown)
  int numa = -1;
  uint64_t vram_mib = 0;      // this partition's share of HBM
  uint32_t xcds = 0;
  uint32_t cus = 0;
  uint32_t kfd_node = kNoKfdNode;  // KFD topology node (the HIP/ROCr order key)
};

struct PhysicalGpu {
  int index = 0;                  // position in Snapshot::gpus
  int node_index = 0;             // node-local GPU index in amdsmi order (what "index" IDs use)
  std::string uuid;               // ID of the whole GPU
  std::string bdf;                // function-0 BDF
  int numa = -1;
  uint64_t vram_mib = 0;          // total HBM of the GPU
  uint32_t xcds = 0;
  uint32_t cus = 0;
  std::string compute_mode;       // SPX / DPX / TPX / QPX / CPX ("SPX" if unknown)
  std::string memory_mode;        // NPS1 / NPS2 / ... ("" if unknown)
  // The modes exactly as amdsmi reported them at enumeration (upper-cased; ""
  // if not reported): the health monitor compares live queries against these
  // to detect re-partitioning.
  std::string reported_compute, reported_memory;
  std::string market_name;
  // Lowest KFD topology node of its partitions (kNoKfdNode if unreported): a
  // container's HIP/ROCr device numbering follows this, not node_index.
  uint32_t kfd_node = kNoKfdNode;
  std::vector<Partition> partitions;  // one per amdsmi handle; sorted by partition_id
  int xgmi_links_down = 0;
  // How vram_mib (the physical HBM) was established, most authoritative first:
  // "memory-partition-config" (sum of the driver's NUMA memory ranges), "spx"
  // (the one handle's vram_info), "share"/"pool"/"whole" (what each partition
  // handle's vram_info turned out to mean, pinned by the model's known HBM),
  // "share-unpinned" (no reference to check against; assumed per-partition).
  std::string vram_source;
  // The driver's accelerator partition profile ("CPX", ...; "" if unavailable).
  std::string driver_profile;

  bool partitioned() const { return compute_mode != "SPX"; }
  // Resource name of this GPU's partitions, e.g. "cpx-1xcd.36gb" (empty if SPX).
  std::string PartitionProfile() const;
};

// Known HBM of a GPU model by market name (MiB), 0 if unknown. The sanity
// bound for what partition handles report (MI355X/MI350X: 288 GB, 294,896 MiB
// as amdsmi reports it on the MI355X box).
uint64_t ModelHbmMib(const std::string& market_name);

// Link classification between two physical GPUs, the analogue of NVML's P2P
// level + NVLink count (vendor/.../nvml/nvml.go:132-154,592-658).
enum class LinkClass { kSame = 0, kXgmi = 1, kPcieSameNuma = 2, kPcieCrossNuma = 3, kUnknown = 4 };

struct Snapshot {
  std::vector<smi::ProcessorInfo> procs;   // raw amdsmi handles
  std::vector<PhysicalGpu> gpus;
  // gpu_links[a * gpus.size() + b]
  std::vector<LinkClass> gpu_links;
  std::vector<uint64_t> gpu_hops;
  std::vector<uint64_t> gpu_weights;  // amdsmi_topo_get_link_weight (0 = unknown)
  std::vector<int> gpu_link_types;    // raw smi::LinkType, -1 = query failed
  std::string smi_path;
  std::string smi_version;
  // Processors whose CU count came from KFD topology (asic_info unanswered),
  // and those whose count stayed unknown.
  size_t cus_from_topology = 0;
  size_t cus_unknown = 0;

  LinkClass Link(int a, int b) const { return gpu_links[a * gpus.size() + b]; }
  uint64_t Hops(int a, int b) const { return gpu_hops[a * gpus.size() + b]; }
  // Physical GPU that owns amdsmi handle index `h` (-1 if none).
  int GpuOfHandle(int h) const;
};

// Node-feature labels describing the GPUs of a snapshot, for Kubernetes
// node-feature-discovery's local source (key=value lines): product, count,
// HBM per GPU, compute/memory partition modes, partitions, xGMI connectivity.
// Values are sanitised to label syntax ([A-Za-z0-9._-], <= 63 chars).
std::vector<std::pair<std::string, std::string>> NodeLabels(const Snapshot& snap);

// Whether this process can open each device node the plugin and amdsmi use
// (<driver root>/dev/kfd, every GPU's render node): a container's device
// cgroup answers EPERM for nodes it does not allow -- an unprivileged pod that
// only hostPath-mounts /dev -- and amdsmi's event notification and libdrm
// queries need them. err = 0: openable.
struct NodeAccess {
  std::string path;
  int err = 0;
};
std::vector<NodeAccess> ProbeDeviceAccess(const Snapshot& snap, const std::string& driver_root);
// errno of opening <driver root>/dev/kfd read-write (0 = ok).
int KfdAccessErrno(const std::string& driver_root);
// One line for the log: "ok" or what failed and the likely cause.
std::string DescribeAccess(const std::vector<NodeAccess>& access);

struct BuildOptions {
  std::string driver_root = "/";
  // Restrict to these physical GPU indices (empty = all). Used by the benchmark
  // to serve exactly N GPUs of a node, and by operators to carve a node.
  std::vector<int> only_gpus;
  // ... or by GPU UUID / PCI address ("0000:0c:00.0", function ignored).
  std::vector<std::string> only_ids;
  bool include_card_nodes = false;
  // sysfs, for what amdsmi's asic_info gives only with the render node (which
  // an unprivileged pod's device cgroup denies): the CU count from KFD's
  // topology (class/kfd/kfd/topology/nodes/<node>/properties) and the board's
  // product name (bus/pci/devices/<bdf>/product_name, the FRU name: "AMD
  // Instinct MI355 OAM" where asic_info says "AMD Radeon Graphics"). "" = neither.
  std::string sysfs_root = "/sys";
};

// CUs of KFD topology node `node` (simd_count / simd_per_cu of its properties
// file), 0 when unreadable.
uint32_t KfdTopologyCus(const std::string& topology_dir, uint32_t node);
// <sysfs root>/bus/pci/devices/<bdf, function 0>/product_name, "" when absent.
std::string PciProductName(const std::string& sysfs_root, const std::string& bdf);

// Builds a snapshot from the loaded library (one enumeration + link queries).
Result<std::shared_ptr<const Snapshot>> BuildSnapshot(smi::Library* lib, const BuildOptions& opt);

// Exposed for tests: grouping + profile naming on raw processor records.
Result<std::shared_ptr<Snapshot>> GroupProcessors(std::vector<smi::ProcessorInfo> procs,
                                                  const BuildOptions& opt);

std::string RenderPath(uint32_t minor);
std::string CardPath(uint32_t minor);
// ceil(mib / 1024): the reference's GB rounding for MIG names (mig-strategy.go:185).
uint64_t GbCeil(uint64_t mib);

}  // namespace adp::inventory

// One kubelet device plugin: a resource name, its devices (+ time-slice replicas)
// and the v1beta1 DevicePlugin gRPC service on its own Unix socket.
//
// Parity: reference cmd/nvidia-device-plugin/server.go
//   NvidiaDevicePlugin fields :56-71, initialize/replicas :95-116, Start :129-151,
//   Stop :154-165, Register :218-240, GetDevicePluginOptions :243-248,
//   ListAndWatch :251-265, GetPreferredAllocation :268-313, Allocate :316-353,
//   PreStartContainer :356-358, device-list/ID strategies :37-53,397-441,
//   DeviceSpecs :443-480.
//
// MI355X-native design:
//  * Containers get GPUs as device nodes: /dev/kfd (shared compute interface)
//    plus each allocated GPU's/partition's /dev/dri/renderD<N>. There is no
//    container-runtime hook, so DeviceSpecs are the primary mechanism; the
//    AMD_VISIBLE_DEVICES env / volume-mount list is kept for deviceListStrategy
//    compatibility (and the AMD container toolkit).
//  * Everything the RPCs need is precomputed at Start(): replica-ID -> device
//    hash map, pre-encoded DeviceSpec / Mount protobuf fragments per device, the
//    encoded ListAndWatch response, the topology graph. Allocate is O(k) hash
//    lookups plus byte concatenation with zero SMI calls (reference: linear
//    scans over all replicas, server.go:377-394, and os.Stat per call :453-462).
//  * The socket is served by `server_threads` epoll loops (concurrent kubelet /
//    benchmark clients are handled in parallel). Allocate/GetPreferredAllocation
//    only read immutable tables. Health lives on loop 0 (other threads reach it
//    through Server::Post); each health transition publishes a new immutable,
//    versioned ListAndWatch snapshot that every loop pushes to the streams it
//    owns -- no locks on the Allocate path, no data races (reference B13/B14).
//  * Health propagates to every replica of a device and recovers (B1, B15).
#pragma once

#include <atomic>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "alloc/replicas.h"
#include "alloc/topology.h"
#include "grpc/grpc.h"
#include "inventory/inventory.h"
#include "metrics/metrics.h"
#include "memcap/driver_usage.h"
#include "memcap/usage.h"
#include "podresources/podresources.h"
#include "strategy/strategy.h"

namespace adp::plugin {

enum class DeviceListStrategy { kEnvvar, kVolumeMounts, kCdiAnnotations, kCdiCri };
enum class DeviceIdStrategy { kUuid, kIndex };
bool ParseDeviceListStrategy(std::string_view s, DeviceListStrategy* out);
bool ParseDeviceIdStrategy(std::string_view s, DeviceIdStrategy* out);

inline constexpr const char* kDefaultPluginDir = "/var/lib/kubelet/device-plugins/";
inline constexpr const char* kVisibleDevicesEnv = "AMD_VISIBLE_DEVICES";
inline constexpr const char* kVolumeMountHostPath = "/dev/null";
inline constexpr const char* kVolumeMountRoot = "/var/run/amd-container-devices";
inline constexpr const char* kCdiVendorClass = "amd.com/gpu";
// Set on Allocate for memory-unit resources: MiB granted per allocated device and
// that share of the device's HBM, comma separated in enumeration order -- the
// order HIP numbers the container's devices (and HSA_CU_MASK uses) -- which is
// not AMD_VISIBLE_DEVICES order under the uuid ID strategy (that list is
// sorted by ID). AMD_GPU_MEMORY_DEVICES names the devices of both lists.
inline constexpr const char* kMemoryLimitEnv = "AMD_GPU_MEMORY_LIMIT_MIB";
inline constexpr const char* kMemoryFractionEnv = "AMD_GPU_MEMORY_FRACTION";
// The device IDs the two lists above refer to, in the same (enumeration) order.
inline constexpr const char* kMemoryDevicesEnv = "AMD_GPU_MEMORY_DEVICES";
// Set on Allocate for CU-partitioned time-slice replicas (--replica-cu-mask): the
// ROCm runtime restricts every queue of the container to the listed CUs.
inline constexpr const char* kCuMaskEnv = "HSA_CU_MASK";
// --enforce-memory-units: where the HBM-cap shim is mounted in the container.
inline constexpr const char* kMemcapContainerPath = "/usr/local/lib/amdgpu-dp/libadp_memcap.so";
// ... and where the grant's accounting file is mounted (memcap/usage.h), named
// to the shim by ADP_MEMCAP_FILE.
inline constexpr const char* kMemcapUsageContainerPath = "/run/amdgpu-dp/memcap";
inline constexpr const char* kMemcapFileEnv = "ADP_MEMCAP_FILE";

struct PluginOptions {
  std::string plugin_dir = kDefaultPluginDir;
  std::string kubelet_socket;  // "" -> plugin_dir + "kubelet.sock"
  DeviceListStrategy list_strategy = DeviceListStrategy::kEnvvar;
  DeviceIdStrategy id_strategy = DeviceIdStrategy::kUuid;
  bool pass_device_specs = true;
  std::string driver_root = "/";
  std::string envvar = kVisibleDevicesEnv;
  // kAuto: per resource, pack for memory units and spread for time-slice
  // replicas; a resource-config entry's own policy wins over this.
  alloc::ReplicaPolicy replica_policy = alloc::ReplicaPolicy::kAuto;
  uint64_t auto_replica_unit_mib = 1000;  // reference: TotalMemory / 1000 (server.go:102)
  // Memory units are CU slots instead: one unit = one CU on every XCD plus
  // VRAM / (CUs per XCD) of HBM (--auto-replica-unit cu-slot; the default with
  // --replica-cu-mask), so every grant fills whole slots.
  bool cu_slot_units = false;
  int dial_timeout_ms = 5000;             // server.go:208,219
  bool register_with_kubelet = true;
  // Built only to see what it would advertise (Plugin::ReplicaLayout): no log lines.
  bool quiet = false;
  bool trace = false;                     // log every RPC with its handler time
  std::string cdi_spec_dir = "/var/run/cdi";  // where cdi-* strategies write the CDI spec
  int server_threads = 0;                 // gRPC loops; <=0 -> DefaultServerThreads()
  int busy_poll_us = 50;                  // loop keeps polling this long after activity
  // Time-slice replicas also split the device's CUs: replica r of R gets its own
  // 1/R of every XCD's CUs (HSA_CU_MASK), so co-scheduled pods stop contending
  // for the same CUs -- the MI355X analogue of an MPS active-thread share.
  bool replica_cu_mask = false;
  // With replica_cu_mask, memory units: a container gets only the CU slots all
  // of whose units it holds (isolating), not every slot it touches.
  bool whole_cu_slots = false;
  bool native_http2 = true;  // HTTP/2 engine of the plugin sockets (false: nghttp2)
  bool follow_peer_l3 = true;  // loops serve a connection from the caller's L3
  // Allocate() of a device currently advertised Unhealthy: false = allocate it
  // and log a warning (the reference allocates silently, server.go:316-353);
  // true = fail the call with FAILED_PRECONDITION naming the device.
  bool reject_unhealthy = false;
  // Time-slice replicas also hold 1/R of the device's HBM each: Allocate()
  // reports it like a memory-unit grant (and --enforce-memory-units caps it).
  bool replica_hbm_share = false;
  // Ask the kubelet for PreStartContainer and refuse to start a container on a
  // device that is Unhealthy at that moment.
  bool prestart_health_check = false;
  // Host path of the HBM-cap shim; non-empty: memory-unit resources mount it
  // read-only at kMemcapContainerPath and set LD_PRELOAD to it.
  std::string memcap_host_path;
  // Non-empty (with the shim): a host file naming the shim, mounted read-only
  // at /etc/ld.so.preload, so the pod's own LD_PRELOAD cannot drop it.
  std::string memcap_preload_list;
  // Non-empty (with the shim): each such Allocate() creates the grant's
  // accounting file here and mounts it, so /metrics reports what the
  // container uses (memcap/usage.h).
  std::string memcap_usage_dir;
};

// With the HBM-cap shim: the grant's MiB per device, one read-only file per
// device mounted at <kGrantDir>/<HIP ordinal> (memcap_area.h). The host files
// are <plugin dir>/amdgpu-dp/grants/<mib>.mib, one per grant size a device of
// the plugin can be given, written before the plugin registers -- Allocate()
// only adds mounts, and a container can never start before its grant exists.
std::string GrantFileName(uint64_t mib);

// HSA_CU_MASK bit ranges [first, last] of each of `replicas` CU shares of a device
// with `cus` CUs over `xcds` XCDs. The kernel driver deals mask bit i to XCD
// i % xcds (measured on MI355X: profiles/r1/session18/), so ranges whose ends are
// multiples of `xcds` give every replica the same CUs on every XCD and never
// leave an XCD without CUs. Empty when the split is impossible (unknown shape,
// fewer than one CU per XCD per replica) or pointless (replicas < 2).
std::vector<std::pair<uint32_t, uint32_t>> ReplicaCuRanges(uint32_t cus, uint32_t xcds, unsigned replicas);

// Memory units (replicas = -1) with --replica-cu-mask: the unit whose ID is
// k-th in lexicographic order owns CU slot floor(k * per / units) (per = CUs per
// XCD; a slot is one CU on every XCD), so a pod gets compute in proportion to
// the HBM it holds, and a packed request, which takes IDs in that order, gets
// contiguous slots. Proportional, not isolating: about units/per units share a
// slot, so two pods may share one boundary slot (never more than one per side
// of a contiguous range). Indexed by replica number; empty when the shape is
// unknown or not uniform.
std::vector<std::pair<uint32_t, uint32_t>> MemoryUnitCuRanges(uint32_t cus, uint32_t xcds, unsigned units);

// min(8, online CPUs): one loop per GPU of an 8-GPU node. Idle loops sit in
// epoll_wait and cost no CPU; they only matter under concurrent clients.
// CPUs this process may use: its affinity mask, bounded by a cgroup CPU quota
// (cgroup v2 cpu.max / v1 cfs quota; fractional).
double CpuBudget();
// gRPC loops per plugin socket when --server-threads is 0: the CPU budget
// rounded up, at most 8.
int DefaultServerThreads();

// One allocatable device (whole GPU or partition) after snapshot resolution.
struct Unit {
  std::string id;          // advertised physical ID
  std::string index;       // "<gpu>" or "<gpu>:<partition>"
  int numa = -1;
  uint64_t vram_mib = 0;
  std::vector<std::string> paths;  // device nodes inside the container
  std::vector<int> handles;        // amdsmi handle indices (health routing)
  int gpu = 0;
  std::string visible_id;          // id or index, per DeviceIdStrategy
  std::string spec_bytes;          // pre-encoded ContainerAllocateResponse.devices entries
  std::string mount_bytes;         // pre-encoded ContainerAllocateResponse.mounts entry
  unsigned replicas = 1;
  uint64_t grant_mib = 0;          // HBM one replica holds (memory units, --replica-hbm-share); 0 = none
  uint32_t cus = 0, xcds = 0;      // compute units / XCDs of this GPU or partition
  // --replica-cu-mask: CU bit range of each replica (empty = whole device).
  std::vector<std::pair<uint32_t, uint32_t>> replica_cus;
  // --memory-unit-cu-slots whole: how many units own each CU slot (empty otherwise).
  std::vector<uint16_t> slot_units;
};

// Written by every server loop on every call: sharded per thread (metrics.h).
struct RpcStats {
  metrics::Counter allocate_calls;
  metrics::Counter allocate_ns_total;
  metrics::MaxGauge allocate_ns_max;
  metrics::Counter preferred_calls;
  metrics::Counter preferred_ns_total;
  metrics::MaxGauge preferred_ns_max;
  metrics::Counter law_sends;
  metrics::Counter unhealthy_allocations;  // Allocate() calls that named an Unhealthy device
  metrics::Counter partial_cu_slot_allocations;  // whole CU slots asked for, none filled on a device
  metrics::Counter prestart_refusals;      // container starts refused by --prestart-health-check
  metrics::Histogram allocate_hist;   // handler time (decode + lookup + encode)
  metrics::Histogram preferred_hist;
};

class Plugin {
 public:
  Plugin(std::shared_ptr<const inventory::Snapshot> snap, strategy::PluginSpec spec,
         PluginOptions opts);
  ~Plugin();
  Plugin(const Plugin&) = delete;
  Plugin& operator=(const Plugin&) = delete;

  const std::string& resource_name() const { return spec_.resource_name; }
  std::string socket_path() const;
  size_t device_count() const { return units_.size(); }
  size_t advertised_count() const { return advertised_.size(); }
  bool replicated() const { return replicated_; }
  // Units (and every per-device list Allocate() returns) follow KFD topology
  // node order -- how HIP numbers a container's devices -- rather than a guess.
  bool hip_order_known() const { return hip_order_known_; }
  // Allocate() can set HSA_CU_MASK / the AMD_GPU_MEMORY_* lists.
  bool sets_cu_masks() const {
    for (const auto& u : units_)
      if (!u.replica_cus.empty()) return true;
    return false;
  }
  bool grants_hbm() const { return hbm_grants_; }
  // Memory-unit resources (replicas -1): what one unit is -- "cu-slot" (a CU on
  // every XCD and its share of the HBM) or "mib" -- and its size in MiB when
  // every device has the same (0 when they differ or this is not a memory-unit
  // resource). Published as node labels and amdgpu_dp_memory_unit_mib.
  bool memory_units() const { return memory_units_; }
  const char* memory_unit_kind() const { return memory_unit_kind_; }
  uint64_t memory_unit_mib() const { return memory_unit_mib_; }
  // Replicated resources: what their IDs mean -- the kind and size of a unit
  // and every device's replica count -- as one comparable line ("" when the
  // resource is not replicated). A change while pods hold the IDs re-means them.
  std::string ReplicaLayout() const;
  // GetPreferredAllocation's replica policy for this resource (never kAuto).
  alloc::ReplicaPolicy replica_policy() const { return replica_policy_; }
  const std::vector<Unit>& units() const { return units_; }
  const std::vector<std::string>& advertised_ids() const { return advertised_; }

  // Serve -> self-dial -> Register. On failure everything is torn down again.
  Status Start(std::function<void()> on_fatal = nullptr);
  void Stop();
  bool running() const {
    std::lock_guard<std::mutex> lk(server_mu_);
    return server_ != nullptr;
  }
  // Running, and the socket file is still the one this plugin bound (false
  // once another process has bound the same path).
  bool owns_socket() const;

  // Thread-safe. Marks every device of physical GPU `gpu` (health is per GPU:
  // a reset or an ECC failure takes all of its partitions).
  void SetGpuHealth(int gpu, bool healthy, const std::string& reason);

  const RpcStats& stats() const { return stats_; }
  std::string StatsJson() const;
  bool registered() const { return registered_.load(); }
  size_t healthy_count() const;
  // Prometheus text for a set of plugins (one HELP/TYPE header per family).
  // `assignments` (kubelet PodResources, may be null) adds per-device usage.
  static void AppendPrometheus(const std::vector<const Plugin*>& plugins, std::string* out,
                               const std::vector<podresources::Assignment>* assignments = nullptr,
                               const memcap::DriverHbmMonitor::Snapshot* driver = nullptr,
                               const std::vector<memcap::Usage>* grant_files = nullptr);
  // Every live enforced grant (accounting files in `dir` whose IDs hash to
  // their name) -> PCI address of each GPU -> bytes granted there, from this
  // daemon's own units (never from the container-writable file's cap[]).
  static std::map<std::string, std::map<std::string, uint64_t>> GrantedByKey(
      const std::vector<const Plugin*>& plugins, const std::string& dir);
  // The same from accounting files read beforehand (no I/O: only ID lookups).
  static std::map<std::string, std::map<std::string, uint64_t>> GrantedByKey(
      const std::vector<const Plugin*>& plugins, const std::vector<memcap::Usage>& files);
  // Bytes `ids` grant per unit, in HIP order (sorted unit index); empty when an
  // ID is not this plugin's or the plugin grants no HBM.
  std::vector<std::pair<int, uint64_t>> GrantedUnits(const std::vector<std::string_view>& ids) const;

  // Handlers (public for in-process tests and benchmarks; loop thread only when serving).
  Status HandleGetOptions(std::string_view req, std::string* resp);
  Status HandleAllocate(std::string_view req, std::string* resp);
  Status HandlePreferred(std::string_view req, std::string* resp);
  Status HandlePreStart(std::string_view req, std::string* resp);

 private:
  void BuildUnits();
  Unit MakeUnit(const alloc::DeviceRef& ref) const;
  void BuildAdvertised();
  void BuildMemcapBytes();
  Status PreferredImpl(std::string_view req, std::string* resp);
  std::vector<int> CachedBestEffort(const std::vector<int>& avail, const std::vector<int>& must, int size);
  void RebuildListAndWatch();
  bool ApplyHealth(const std::vector<int>& units, bool healthy, const std::string& reason);
  void PostHealth(std::vector<int> units, bool healthy, const std::string& reason);
  Status Register();
  static void AppendMemcapUsage(const std::vector<const Plugin*>& plugins, const std::string& dir,
                                const std::vector<podresources::Assignment>* assignments, std::string* out,
                                const memcap::DriverHbmMonitor::Snapshot* driver,
                                const std::vector<memcap::Usage>* grant_files);
  void AddUsageFile(const std::vector<std::string_view>& ids, const std::vector<uint64_t>& grant_bytes,
                    std::string* c);
  // Allocate's pieces, per container (HandleAllocate).
  struct MemoryGrant {
    std::string mib, frac, devs;   // the AMD_GPU_MEMORY_* env values
    std::vector<uint64_t> bytes;   // per device, in enumeration order
    void Clear() { mib.clear(); frac.clear(); devs.clear(); bytes.clear(); }
  };
  Status CheckAllocatedHealth(const std::vector<int>& us);
  void BuildMemoryGrant(const std::vector<int>& us, const std::vector<int>& units_per, MemoryGrant* g) const;
  void BuildCuMask(const std::vector<int>& us, std::vector<std::pair<int, uint32_t>>* shares, std::string* cu_mask);
  void AppendDeviceList(const std::vector<int>& us, const std::string& joined, std::string* c) const;
  void AppendGrantMounts(const std::vector<uint64_t>& grant_bytes, std::string* c) const;

 public:
  // With the shim: writes every grant file this plugin's Allocate() can mount
  // (idempotent; also after a kubelet wiped the directory). Empty Ok otherwise.
  Status InstallGrantFiles() const;
  std::string GrantDir() const;

 private:

 public:
  // CDI (Container Device Interface) spec describing this plugin's devices, for
  // the cdi-annotations / cdi-cri device-list strategies. Returns its JSON text.
  std::string CdiSpecJson() const;
  std::string CdiSpecPath() const;
  Status WriteCdiSpec() const;

 private:

  std::shared_ptr<const inventory::Snapshot> snap_;
  strategy::PluginSpec spec_;
  PluginOptions opts_;
  bool replicated_ = false;
  bool UnitIsCuSlot(const Unit& u) const;
  void CheckMemoryUnitName();
  bool memory_units_ = false;  // auto replicas: one ID per auto_replica_unit_mib of HBM
  const char* memory_unit_kind_ = "";
  uint64_t memory_unit_mib_ = 0;
  bool hbm_grants_ = false;    // Allocate() reports (and may enforce) HBM per replica: memory units or HBM shares
  bool hip_order_known_ = true;
  alloc::ReplicaPolicy replica_policy_ = alloc::ReplicaPolicy::kSpread;  // resolved for this resource  // units are in KFD-node (HIP) order; false: amdsmi order, nodes unreported

  std::vector<Unit> units_;
  std::unordered_map<std::string, int> unit_by_id_;
  std::unordered_map<std::string_view, int> unit_index_by_id_;  // keys view units_[i].id
  std::vector<std::string> advertised_;       // advertised IDs (replicas or plain)
  std::vector<int> advertised_unit_;
  // advertised ID -> unit; keys view into advertised_ (never modified after build)
  std::unordered_map<std::string_view, int> advertised_index_;
  std::string kfd_spec_bytes_;
  std::string memcap_bytes_;  // pre-encoded LD_PRELOAD env + shim mount (--enforce-memory-units)
  std::string grant_dir_prefix_;  // GrantDir() + "/": host paths of the read-only grant files
  alloc::DeviceGraph graph_;
  // Memoised best-effort answers for <= 8 whole devices (see CachedBestEffort),
  // in anonymous zero-filled pages (an all-zero atomic<uint16_t> is "empty").
  static constexpr size_t kBestEffortCacheBytes = 256u * 256u * 9u * sizeof(uint16_t);
  struct Unmap {
    void operator()(std::atomic<uint16_t>* p) const;
  };
  std::unique_ptr<std::atomic<uint16_t>, Unmap> best_effort_cache_;

  struct LawSnapshot {
    uint64_t version = 0;
    std::string bytes;             // encoded ListAndWatchResponse
    std::vector<uint8_t> healthy;  // per unit, as advertised in `bytes`
  };
  struct LawStream {
    std::shared_ptr<grpc::ServerStream> stream;
    uint64_t sent_version = 0;
  };
  std::shared_ptr<const LawSnapshot> CurrentLaw() const;
  void BroadcastLaw(int loop);  // on loop `loop`: push the newest snapshot to its streams

  // Health: loop 0 (or under server_mu_ when not serving).
  std::vector<uint8_t> healthy_;
  uint64_t law_version_ = 0;
  mutable std::mutex law_mu_;  // guards law_ (the pointer; snapshots are immutable)
  std::shared_ptr<const LawSnapshot> law_;
  std::atomic<size_t> law_bytes_size_{0};  // readable from any thread (stats)
  // Units advertised Unhealthy in law_: Allocate() only looks health up when
  // this is non-zero, so the healthy fast path costs one relaxed load.
  std::atomic<size_t> unhealthy_units_{0};
  // Per unit: the ListAndWatch version of the last "allocated while Unhealthy"
  // warning, so a kubelet retrying the same device logs once per transition.
  std::unique_ptr<std::atomic<uint64_t>[]> warned_law_;
  // law_streams_[i] is confined to server loop i.
  std::vector<std::vector<LawStream>> law_streams_;

  // Guards server_ itself (not the loop-thread state): health updates arrive from
  // the monitor thread while the supervisor may be stopping the plugin.
  mutable std::mutex server_mu_;
  std::unique_ptr<grpc::Server> server_;
  RpcStats stats_;
  std::atomic<bool> registered_{false};
};

}  // namespace adp::plugin

// libamd_smi, loaded at run time with dlopen, wrapped in typed calls.
//
// Parity: the reference's NVML layer -- dlopen("libnvidia-ml.so.1") + nvmlInit_v2
// (vendor/.../gpu-monitoring-tools/bindings/go/nvml/nvml_dl.go:29-36), thin C
// wrappers (bindings.go:94-859) and the high-level Device (nvml.go:294-822).
// MI355X-native replacement: amdsmi (/opt/rocm/include/amd_smi/amdsmi.h), only the
// cheap queries the plugin needs. The reference calls ~14 NVML
// queries per GPU via Status() just to read total memory (nvidia.go:96-98); here
// enumeration is uuid + bdf + enumeration info (render/card minors) + NUMA +
// VRAM + partition mode, once per snapshot.
//
// The library path is overridable (AMD_SMI_LIB / --amdsmi-lib) so tests load
// native/mock/libamdsmi_mock.so, which exports the same C symbols driven by a
// JSON fixture. Every call returns a Status; nothing
// panics (reference defect B16).
#pragma once

#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "common/status.h"

namespace adp::smi {

// One amdsmi processor handle: a whole GPU (SPX) or one compute partition.
struct ProcessorInfo {
  void* handle = nullptr;
  std::string uuid;
  std::string bdf;           // "dddd:bb:dd.f"
  uint64_t bdf_id = 0;       // amdsmi_bdf_t.as_uint
  uint32_t render_minor = 0; // /dev/dri/renderD<minor>; 0 = unknown
  uint32_t card_minor = 0xffffffff;
  uint32_t hip_id = 0xffffffff;
  int32_t numa_node = -1;
  uint64_t vram_mib = 0;
  std::string compute_partition;  // "SPX", "DPX", "TPX", "QPX", "CPX" or "" if unknown
  std::string memory_partition;   // "NPS1", "NPS2", ... or ""
  uint32_t partition_id = 0;      // kfd current_partition_id (0 when not reported)
  // KFD topology node (amdsmi_get_gpu_kfd_info().node_id; 0xffffffff = not
  // reported). ROCr creates its GPU agents -- and HIP numbers a container's
  // devices -- in this order, over the nodes whose render node the process can
  // open; it need not be amdsmi's enumeration order.
  uint32_t kfd_node = 0xffffffff;
  uint32_t num_cu = 0;
  uint32_t xcd_count = 0;         // 0 = unknown
  std::string market_name;
  std::string asic_serial;        // same for every partition of one physical GPU ("" if unknown)
  // amdsmi_get_gpu_accelerator_partition_profile (+ _config for the XCC count):
  // the driver's own description of the current compute partitioning.
  std::string profile_type;       // "SPX".."CPX" ("" = query unavailable)
  uint32_t profile_partitions = 0;  // partitions of that profile (0 = unknown)
  uint32_t profile_xccs = 0;        // XCCs per partition (0 = unknown)
  // amdsmi_get_gpu_memory_partition_config: the GPU's NUMA memory ranges.
  uint32_t mem_ranges = 0;        // number of ranges (= memory partitions; 0 = unknown)
  uint64_t mem_ranges_mib = 0;    // their total size
};

enum class LinkType { kInternal = 0, kPcie = 1, kXgmi = 2, kNotApplicable = 3, kUnknown = 4 };

struct Link {
  bool valid = false;
  LinkType type = LinkType::kUnknown;
  uint64_t hops = 0;
  uint64_t weight = 0;
};

enum EventType : uint32_t {  // amdsmi_evt_notification_type_t values
  kEvtVmFault = 1,
  kEvtThermalThrottle = 2,
  kEvtGpuPreReset = 3,
  kEvtGpuPostReset = 4,
  // 5..13: KFD's informational events (migration, page faults, queue
  // eviction/restore, unmap, process start/end) -- never a device failure.
  kEvtProcessStart = 12,
  kEvtProcessEnd = 13,
  kEvtLast = 13,
};

// "GPU_PRE_RESET", "PROCESS_START", ... (amdsmi's names without the
// AMDSMI_EVT_NOTIF_ prefix); "EVENT_<n>" for a type amdsmi does not define.
std::string EventTypeName(uint32_t type);

struct Event {
  void* handle = nullptr;
  uint32_t type = 0;
  std::string message;
};

// Every query is virtual: a test harness (native/tests/health_model.cc)
// subclasses it with a scripted fake instead of a dlopen'ed library.
class Library {
 public:
  virtual ~Library();
  Library(const Library&) = delete;
  Library& operator=(const Library&) = delete;

  // dlopen(path or default) + resolve + amdsmi_init(AMD_GPUS). `path` empty ->
  // $AMD_SMI_LIB, then libamd_smi.so on the loader path, then
  // <rocm_root>/lib/libamd_smi.so.
  static Result<std::unique_ptr<Library>> Open(const std::string& path,
                                               const std::string& rocm_root = "/opt/rocm");

  const std::string& path() const { return path_; }
  std::string Version() const;

  virtual Result<std::vector<ProcessorInfo>> Enumerate();
  Link GetLink(void* src, void* dst);
  // Number of xGMI links reported down (0 when unsupported).
  virtual int XgmiLinksDown(void* h);

  // Event notification (health). Init registers `mask` on each handle, all or
  // nothing: when one handle's registration fails, the handles it had already
  // registered are stopped again before it returns, so a failed init leaves no
  // registration behind (a reload re-registering them would otherwise leak
  // the kernel's event file of each). A handle already registered by an
  // earlier EventsInit only gets the new mask.
  virtual Status EventsInit(const std::vector<void*>& handles, uint64_t mask);
  // Waits up to timeout_ms; appends received events.
  virtual Status EventsWait(int timeout_ms, std::vector<Event>* out);
  // Stops the registrations among `handles` (the others: nothing to stop).
  virtual void EventsStop(const std::vector<void*>& handles);
  // Stops every registration this Library holds (before a Reinit).
  virtual void EventsStopAll();
  // Registrations held (tests; /metrics).
  size_t EventsRegistered() const;

  // RAS polling (fallback health when events are unavailable).
  virtual Result<uint64_t> UncorrectableErrors(void* h);
  // HBM pages the driver retired after uncorrectable errors, and the count at
  // which the driver itself gives up on the GPU (needs root on current drivers).
  virtual Result<uint32_t> RetiredPages(void* h);
  virtual Result<uint32_t> RetiredPageThreshold(void* h);
  // HBM in use on the device (bytes, every process: amdsmi_get_gpu_memory_usage).
  virtual Result<uint64_t> VramUsed(void* h);
  // Graphics-engine activity in percent (amdsmi_get_gpu_activity: the SMU's
  // gpu_metrics, which the driver does not serve while the GPU is in reset).
  virtual Result<uint32_t> Activity(void* h);
  virtual bool Responsive(void* h);

  // Every query the plugin uses, run once per processor, with its amdsmi
  // status: what works in this container (device cgroup, privileges) and what
  // does not. JSON object text; `--smi-report`.
  std::string QueryReport();

  // Current compute/memory partition mode of a processor, e.g. {"CPX", "NPS2"}
  // (empty strings when the query is unavailable).
  virtual std::pair<std::string, std::string> PartitionModes(void* h);

  // amdsmi_shut_down + amdsmi_init: picks up a changed partition layout (the
  // driver re-creates processors when a GPU is re-partitioned). Invalidates all
  // handles; callers must have stopped every user of the old ones.
  virtual Status Reinit();

 protected:
  Library();  // (out of line: Fns is incomplete here)

 private:
  void ReadPartitionProfile(void* h, ProcessorInfo* p);
  struct Fns;
  void* dl_ = nullptr;
  std::unique_ptr<Fns> f_;
  std::string path_;
  bool initialized_ = false;
  mutable std::mutex evt_mu_;
  std::vector<void*> evt_live_;  // handles with a live event registration
};

std::string FormatBdf(uint64_t bdf_id);
uint64_t EventMask(uint32_t event_type);

}  // namespace adp::smi

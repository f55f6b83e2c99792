#include "daemon/config.h"

#include <cctype>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <json.hpp>
#include <sstream>

#include "common/strings.h"
#include "daemon/yaml.h"

extern char** environ;

namespace adp::daemon {
namespace {

enum class Kind { kString, kBool, kUint };

struct FlagDef {
  const char* name;      // command line, without "--"
  const char* env;       // environment variable ("" = none)
  const char* file_key;  // key under `flags:` in the config file ("" = none)
  Kind kind;
  const char* help;
  std::function<void*(Flags&)> field;
  bool allow_zero = false;  // kUint: 0 is a meaningful value ("auto")
};

// Names the reference (NVIDIA-derived) deployment used for the same settings, so
// an existing DaemonSet/config file keeps working when switched to this plugin.
// The canonical name wins when both are given at the same precedence level.
struct AliasDef {
  const char* name;       // command line alias
  const char* env;        // environment alias ("" = none)
  const char* file_key;   // config-file alias ("" = none)
  const char* canonical;  // FlagDef::name
};

const std::vector<AliasDef>& Aliases() {
  static const std::vector<AliasDef> t = {
      {"mig-strategy", "MIG_STRATEGY", "migStrategy", "partition-strategy"},  // main.go:63-71
      {"nvidia-driver-root", "NVIDIA_DRIVER_ROOT", "nvidiaDriverRoot", "driver-root"},  // :108-116
      {"", "NVIDIA_DRIVER_RESOURCE_CONFIG", "", "resource-config"},  // main.go:123-129
  };
  return t;
}

const std::vector<FlagDef>& Table() {
  static const std::vector<FlagDef> t = {
      {"partition-strategy", "PARTITION_STRATEGY", "partitionStrategy", Kind::kString,
       "strategy for exposing compute partitions (SPX/DPX/QPX/CPX): [none | single | mixed]",
       [](Flags& f) -> void* { return &f.partition_strategy; }},
      {"fail-on-init-error", "FAIL_ON_INIT_ERROR", "failOnInitError", Kind::kBool,
       "fail the plugin if an error is encountered during initialization, otherwise block "
       "indefinitely",
       [](Flags& f) -> void* { return &f.fail_on_init_error; }},
      {"pass-device-specs", "PASS_DEVICE_SPECS", "passDeviceSpecs", Kind::kBool,
       "pass /dev/kfd and the render nodes as DeviceSpecs on Allocate()",
       [](Flags& f) -> void* { return &f.pass_device_specs; }},
      {"device-list-strategy", "DEVICE_LIST_STRATEGY", "deviceListStrategy", Kind::kString,
       "how the device list is also passed to the runtime: [envvar | volume-mounts | "
       "cdi-annotations | cdi-cri]",
       [](Flags& f) -> void* { return &f.device_list_strategy; }},
      {"device-id-strategy", "DEVICE_ID_STRATEGY", "deviceIDStrategy", Kind::kString,
       "how device IDs are passed to the runtime: [uuid | index]",
       [](Flags& f) -> void* { return &f.device_id_strategy; }},
      {"driver-root", "DRIVER_ROOT", "driverRoot", Kind::kString,
       "root path of the host driver installation (device nodes are <driver-root>/dev/...)",
       [](Flags& f) -> void* { return &f.driver_root; }},
      {"resource-config", "RESOURCE_CONFIG", "resourceConfig", Kind::kString,
       "rename/replicate resources: <original>:<new>:<replicas>,... e.g. "
       "'gpu:sharedgpu:4,cpx-1xcd.36gb:small:2'; replicas -1 = one per 1000 MiB of VRAM",
       [](Flags& f) -> void* { return &f.resource_config; }},
      {"replica-policy", "REPLICA_POLICY", "replicaPolicy", Kind::kString,
       "preferred allocation over replicas: [auto | spread | pack] (auto: pack for memory-unit resources "
       "(replicas -1), spread for time-slice replicas; a resource-config entry's 4th field overrides it)",
       [](Flags& f) -> void* { return &f.replica_policy; }},
      {"replica-cu-mask", "REPLICA_CU_MASK", "replicaCuMask", Kind::kBool,
       "replicas also split the device's compute units (HSA_CU_MASK on Allocate): time-slice "
       "replica r of R runs on its own 1/R of every XCD's CUs; memory units become CU slots "
       "(--auto-replica-unit auto), each a CU on every XCD with its share of the HBM, so every "
       "pod owns whole slots",
       [](Flags& f) -> void* { return &f.replica_cu_mask; }},
      {"memory-unit-cu-slots", "DP_MEMORY_UNIT_CU_SLOTS", "memoryUnitCuSlots", Kind::kString,
       "with --replica-cu-mask and MiB memory units (--auto-replica-unit mib), which CU slots a container "
       "gets: [proportional | whole] (whole: only the slots all of whose units it holds, so no two "
       "containers share a CU; a container that fills no slot on a device falls back to its partial slots, "
       "counted in amdgpu_dp_partial_cu_slot_allocations_total). CU-slot units need neither",
       [](Flags& f) -> void* { return &f.memory_unit_cu_slots; }},
      {"device-plugin-path", "DP_PLUGIN_DIR", "devicePluginPath", Kind::kString,
       "kubelet device-plugin directory",
       [](Flags& f) -> void* { return &f.plugin_dir; }},
      {"kubelet-socket", "DP_KUBELET_SOCKET", "kubeletSocket", Kind::kString,
       "kubelet registration socket (default <device-plugin-path>/kubelet.sock)",
       [](Flags& f) -> void* { return &f.kubelet_socket; }},
      {"amdsmi-lib", "AMD_SMI_LIB", "amdsmiLib", Kind::kString,
       "path of libamd_smi.so to load (default: search the loader path and /opt/rocm/lib)",
       [](Flags& f) -> void* { return &f.amdsmi_lib; }},
      {"devices", "AMD_DP_DEVICES", "devices", Kind::kString,
       "only serve these GPUs: node indices, UUIDs or PCI addresses, comma separated (default: all)",
       [](Flags& f) -> void* { return &f.devices; }},
      {"auto-replica-unit-mib", "AUTO_REPLICA_UNIT_MIB", "autoReplicaUnitMiB", Kind::kUint,
       "MiB of VRAM per replica when replicas=-1 (MiB units)",
       [](Flags& f) -> void* { return &f.auto_replica_unit_mib; }},
      {"auto-replica-unit", "AUTO_REPLICA_UNIT", "autoReplicaUnit", Kind::kString,
       "what one memory unit (replicas=-1) is: [auto | mib | cu-slot] (mib: --auto-replica-unit-mib of "
       "VRAM, the reference's rule; cu-slot: one CU on every XCD plus VRAM / (CUs per XCD) of HBM -- 32 "
       "units of ~9 GiB on an SPX MI355X -- so CU shares line up with grants; auto: cu-slot with "
       "--replica-cu-mask, else mib)",
       [](Flags& f) -> void* { return &f.auto_replica_unit; }},
      {"resource-prefix", "RESOURCE_PREFIX", "resourcePrefix", Kind::kString,
       "extended-resource domain", [](Flags& f) -> void* { return &f.resource_prefix; }},
      {"include-card-nodes", "INCLUDE_CARD_NODES", "includeCardNodes", Kind::kBool,
       "also pass /dev/dri/card<N> nodes (not needed for compute)",
       [](Flags& f) -> void* { return &f.include_card_nodes; }},
      {"trace", "ADP_TRACE", "trace", Kind::kBool,
       "log every RPC (method, status, sizes, handler time)",
       [](Flags& f) -> void* { return &f.trace; }},
      {"dry-run", "ADP_DRY_RUN", "", Kind::kBool,
       "print the resources/devices this node would advertise as JSON and exit",
       [](Flags& f) -> void* { return &f.dry_run; }},
      {"list-grants", "ADP_LIST_GRANTS", "", Kind::kBool,
       "print the HBM use of enforced grants (the accounting files under <device-plugin-path>/amdgpu-dp/usage) "
       "as JSON and exit",
       [](Flags& f) -> void* { return &f.list_grants; }},
      {"smi-report", "ADP_SMI_REPORT", "", Kind::kBool,
       "print, as JSON, the status of every amdsmi query the plugin uses and whether each device node "
       "opens (what this container's privileges and device cgroup allow) and exit",
       [](Flags& f) -> void* { return &f.smi_report; }},
      {"relay-ping", "ADP_RELAY_PING", "", Kind::kBool,
       "liveness check of the event relay at --health-event-socket (the relay container's probe): exit 0 "
       "when it greets within 5 s with a working event wait, 1 otherwise; loads no amdsmi",
       [](Flags& f) -> void* { return &f.relay_ping; }},
      {"doctor", "ADP_DOCTOR", "", Kind::kBool,
       "check what this deployment needs on this node -- amdsmi, enumeration, resources, device-node "
       "access, health events, ECC, the kubelet socket, the plugin directory, the HBM-cap shim, the host "
       "/proc, the CPU budget -- print one line per check with what to change, and exit (1 on a failure)",
       [](Flags& f) -> void* { return &f.doctor; }},
      {"health-events", "DP_HEALTH_EVENTS", "healthEvents", Kind::kBool,
       "register amdsmi event notification (GPU_PRE_RESET / GPU_POST_RESET: Unhealthy and back); "
       "it needs /dev/kfd, which an unprivileged pod's device cgroup denies (false = polling only)",
       [](Flags& f) -> void* { return &f.health_events; }},
      {"health-event-socket", "DP_HEALTH_EVENT_SOCKET", "healthEventSocket", Kind::kString,
       "receive amdsmi health events from the event relay listening on this Unix socket instead of "
       "registering them in this process, which then needs no /dev/kfd access (privilege separation: "
       "only the relay runs privileged; empty = register in-process)",
       [](Flags& f) -> void* { return &f.health_event_socket; }},
      {"health-event-extra-types", "DP_HEALTH_EVENT_EXTRA_TYPES", "healthEventExtraTypes", Kind::kString,
       "amdsmi event types to register on top of GPU_PRE_RESET/POST_RESET, VMFAULT and THERMAL_THROTTLE, by number "
       "or name, comma separated (e.g. '12,13' = KFD PROCESS_START/PROCESS_END, which every HIP process causes): "
       "counted per GPU in amdgpu_dp_gpu_events_total, never a health verdict; the event relay registers its own "
       "(empty = none)",
       [](Flags& f) -> void* { return &f.health_event_extra_types; }},
      {"event-relay", "DP_EVENT_RELAY", "", Kind::kBool,
       "run as the event relay: register amdsmi event notification (needs /dev/kfd) and forward every "
       "event to daemons connecting to --health-event-socket; nothing else (no kubelet, no network)",
       [](Flags& f) -> void* { return &f.event_relay; }},
      {"driver-hbm-poll-ms", "DP_DRIVER_HBM_POLL_MS", "driverHbmPollMs", Kind::kUint,
       "with enforced memory units and /metrics: every N ms, read what each process holds on each GPU by the "
       "driver's count (DRM fdinfo under --host-proc), attribute it to grants and flag grants over their HBM "
       "(0 = off)",
       [](Flags& f) -> void* { return &f.driver_hbm_poll_ms; }},
      {"driver-hbm-slack-mib", "DP_DRIVER_HBM_SLACK_MIB", "driverHbmSlackMib", Kind::kUint,
       "HBM per process the driver-side check allows above the grant: the HIP runtime's own allocations, "
       "which never pass through hipMalloc",
       [](Flags& f) -> void* { return &f.driver_hbm_slack_mib; }},
      {"host-proc", "DP_HOST_PROC", "hostProc", Kind::kString,
       "the /proc of the PID namespace the pods run in, for the driver-side HBM check: /proc with hostPID, "
       "else a hostPath mount of the host's /proc (with --health-event-socket the event relay runs the scans, "
       "with its own --host-proc)",
       [](Flags& f) -> void* { return &f.host_proc; }},
      {"kfd-proc-dir", "DP_KFD_PROC_DIR", "kfdProcDir", Kind::kString,
       "KFD's list of GPU processes (host PIDs) for the driver-side HBM check: only those processes' "
       "descriptors are read, not every process's (empty = always walk every process under --host-proc)",
       [](Flags& f) -> void* { return &f.kfd_proc_dir; }},
      {"drain", "ADP_DRAIN", "", Kind::kString,
       "add these GPUs (PCI addresses, UUIDs or node indices, comma separated; checked against this node's "
       "GPUs) to --drain-file, print the drain list and exit: from the plugin pod, `amdgpu-device-plugin --drain "
       "0000:0c:00.0` takes a GPU out of service at the next health poll",
       [](Flags& f) -> void* { return &f.drain; }},
      {"undrain", "ADP_UNDRAIN", "", Kind::kString,
       "remove these GPUs from --drain-file (their names only: other GPUs named on the same line, and its "
       "comment, stay), print the drain list and exit",
       [](Flags& f) -> void* { return &f.undrain; }},
      {"return-to-service", "ADP_RETURN_TO_SERVICE", "", Kind::kString,
       "return these GPUs (named as for --drain) to service and exit: the running daemon clears what its health "
       "monitor holds against them -- a GPU_PRE_RESET without its GPU_POST_RESET, a flapping quarantine and its "
       "reset count, an ECC verdict (re-baselined at the current count), an event -- at its next poll, as if their "
       "lines were deleted from --health-state-file. A drain stays (--undrain); a failure still present (no "
       "answer, retired pages) comes back at that poll. The request is written next to --drain-file",
       [](Flags& f) -> void* { return &f.return_to_service; }},
      {"drain-file", "DP_DRAIN_FILE", "drainFile", Kind::kString,
       "operator drain list: every GPU named in this file (PCI address, UUID, partition UUID or node index; "
       "whitespace or comma separated, '#' comments) is advertised Unhealthy until it is removed from the file "
       "(read when the health monitor starts and at every poll; a reset does not clear it; empty = off)",
       [](Flags& f) -> void* { return &f.drain_file; }},
      {"reset-recovery-hold-ms", "DP_RESET_RECOVERY_HOLD_MS", "resetRecoveryHoldMs", Kind::kUint,
       "a GPU waiting for GPU_POST_RESET across an event gap (events lost: relay restarted or re-registered, "
       "events off, a new in-process registration) is back in service once amdsmi has answered every health "
       "poll for this long with no new GPU_PRE_RESET (0 = only the event brings it back)",
       [](Flags& f) -> void* { return &f.reset_recovery_hold_ms; }, true},
      {"reset-flap-limit", "DP_RESET_FLAP_LIMIT", "resetFlapLimit", Kind::kUint,
       "a GPU that resets this many times within --reset-flap-window-ms is kept Unhealthy (cause "
       "\"flapping\"), its GPU_POST_RESETs notwithstanding, until a whole window passes without a reset (0 = off; "
       "a reset counts once, however many partitions report its GPU_PRE_RESET)",
       [](Flags& f) -> void* { return &f.reset_flap_limit; }, true},
      {"defer-layout-changes", "DP_DEFER_LAYOUT_CHANGES", "deferLayoutChanges", Kind::kBool,
       "a live config change (config file, SIGHUP) that would change what a replicated resource's IDs mean "
       "(memory unit, replica count, CU masks) while running pods hold some of them (kubelet PodResources) "
       "waits: the current layout keeps being served, amdgpu_dp_deferred_layout_change says so, and the "
       "change applies once no pod holds those IDs (looked at every 30 s); a change is applied, with a "
       "warning, when PodResources cannot say (no --pod-resources-socket, or it does not answer). Off: it "
       "applies at once and the node may be over-committed until those pods end",
       [](Flags& f) -> void* { return &f.defer_layout_changes; }},
      {"reset-flap-window-ms", "DP_RESET_FLAP_WINDOW_MS", "resetFlapWindowMs", Kind::kUint,
       "the window of --reset-flap-limit, and the quiet time that ends a quarantine",
       [](Flags& f) -> void* { return &f.reset_flap_window_ms; }},
      {"sysfs-root", "DP_SYSFS_ROOT", "sysfsRoot", Kind::kString,
       "where sysfs is mounted: without the render node (an unprivileged pod's device cgroup denies it) "
       "amdsmi's asic_info fails, and the CU count comes from <root>/class/kfd/kfd/topology and the product "
       "name from <root>/bus/pci/devices/<bdf>/product_name, both readable unprivileged (empty = neither)",
       [](Flags& f) -> void* { return &f.sysfs_root; }},
      {"cdi-spec-dir", "CDI_SPEC_DIR", "cdiSpecDir", Kind::kString,
       "directory for the generated CDI spec (cdi-annotations / cdi-cri strategies)",
       [](Flags& f) -> void* { return &f.cdi_spec_dir; }},
      {"server-threads", "DP_SERVER_THREADS", "serverThreads", Kind::kUint,
       "gRPC loop threads per plugin socket (0 = the CPU budget -- affinity mask and cgroup CPU quota -- "
       "rounded up, at most 8)",
       [](Flags& f) -> void* { return &f.server_threads; }, true},
      {"busy-poll-us", "DP_BUSY_POLL_US", "busyPollUs", Kind::kUint,
       "after serving a request a gRPC loop polls without sleeping for this many "
       "microseconds, so follow-up calls skip a scheduler wake-up (0 = always sleep; off under a CPU "
       "budget below 2 CPUs)",
       [](Flags& f) -> void* { return &f.busy_poll_us; }, true},
      {"http2-server", "DP_HTTP2_SERVER", "http2Server", Kind::kString,
       "HTTP/2 engine of the plugin sockets: [native | nghttp2] (native: hand-written framing "
       "and flow control, nghttp2 HPACK decoding; nghttp2: its full session layer)",
       [](Flags& f) -> void* { return &f.http2_server; }},
      {"loop-affinity", "DP_LOOP_AFFINITY", "loopAffinity", Kind::kString,
       "where a gRPC loop runs once it takes a connection: [peer-l3 | none] (peer-l3: on the "
       "CPUs sharing the L3 cache with the caller's last CPU, when the caller is visible)",
       [](Flags& f) -> void* { return &f.loop_affinity; }},
      {"node-labels-file", "DP_NODE_LABELS_FILE", "nodeLabelsFile", Kind::kString,
       "write node-feature labels (amd.com/gpu.product, .count, .memory-mib, partition modes, "
       "interconnect; amd.com/<resource>.memory-unit and .memory-unit-mib for memory-unit resources) to this "
       "file for node-feature-discovery's local source (empty = off)",
       [](Flags& f) -> void* { return &f.node_labels_file; }},
      {"pod-resources-socket", "DP_POD_RESOURCES_SOCKET", "podResourcesSocket", Kind::kString,
       "kubelet PodResources socket; with --metrics-addr, per-device allocations and "
       "sharing (pods per GPU) are exported (empty = off)",
       [](Flags& f) -> void* { return &f.pod_resources_socket; }},
      {"health-state-file", "DP_HEALTH_STATE_FILE", "healthStateFile", Kind::kString,
       "persist per-GPU health verdicts (ECC baseline, failures awaiting GPU_POST_RESET) in this "
       "file so they survive a container restart; outside the kubelet's device-plugin directory, "
       "which the kubelet empties when it restarts (empty = kept in memory across plugin restarts only)",
       [](Flags& f) -> void* { return &f.health_state_file; }},
      {"reject-unhealthy", "DP_REJECT_UNHEALTHY", "rejectUnhealthy", Kind::kBool,
       "fail Allocate() for a device currently advertised Unhealthy (default: allocate it and log a "
       "warning, as the reference does)",
       [](Flags& f) -> void* { return &f.reject_unhealthy; }},
      {"prestart-health-check", "DP_PRESTART_HEALTH_CHECK", "prestartHealthCheck", Kind::kBool,
       "ask the kubelet to call PreStartContainer before each container start and refuse the start when one "
       "of the container's devices is Unhealthy at that moment (the reference's PreStartContainer is a no-op)",
       [](Flags& f) -> void* { return &f.prestart_health_check; }},
      {"replica-hbm-share", "DP_REPLICA_HBM_SHARE", "replicaHbmShare", Kind::kBool,
       "time-slice replicas (replicas > 1) each hold 1/R of the device's HBM: Allocate() reports the grant "
       "like a memory unit's (AMD_GPU_MEMORY_LIMIT_MIB ...), and --enforce-memory-units caps it",
       [](Flags& f) -> void* { return &f.replica_hbm_share; }},
      {"enforce-memory-units", "DP_ENFORCE_MEMORY_UNITS", "enforceMemoryUnits", Kind::kBool,
       "memory-unit resources (replicas -1): mount and preload libadp_memcap.so in the container, which caps "
       "each device's HIP allocations at the HBM the pod was granted (AMD_GPU_MEMORY_LIMIT_MIB)",
       [](Flags& f) -> void* { return &f.enforce_memory_units; }},
      {"memcap-ld-so-preload", "DP_MEMCAP_LD_SO_PRELOAD", "memcapLdSoPreload", Kind::kBool,
       "with --enforce-memory-units: also mount a read-only /etc/ld.so.preload naming the shim, so a pod that "
       "sets its own LD_PRELOAD still loads it (replaces the image's /etc/ld.so.preload, if any)",
       [](Flags& f) -> void* { return &f.memcap_ld_so_preload; }},
      {"memcap-lib", "DP_MEMCAP_LIB", "memcapLib", Kind::kString,
       "path of libadp_memcap.so in the plugin's filesystem (default: next to the binary, then "
       "/usr/lib/amdgpu-device-plugin/)",
       [](Flags& f) -> void* { return &f.memcap_lib; }},
      {"container-hbm-metrics", "DP_CONTAINER_HBM_METRICS", "containerHbmMetrics", Kind::kBool,
       "with --enforce-memory-units and --metrics-addr: mount a per-grant accounting file (read-write) into "
       "each memory-unit container so /metrics reports the HBM it uses, its peak and refused allocations",
       [](Flags& f) -> void* { return &f.container_hbm_metrics; }},
      {"metrics-addr", "DP_METRICS_ADDR", "metricsAddr", Kind::kString,
       "serve Prometheus /metrics and /healthz on this TCP address, e.g. ':9400' (empty = off)",
       [](Flags& f) -> void* { return &f.metrics_addr; }},
  };
  return t;
}

Status Assign(const FlagDef& d, Flags& f, const std::string& value, const std::string& origin) {
  void* p = d.field(f);
  switch (d.kind) {
    case Kind::kString:
      *static_cast<std::string*>(p) = value;
      return Status::Ok();
    case Kind::kBool: {
      auto b = ParseBool(value);
      if (!b) return InvalidArgument("invalid boolean '" + value + "' for " + d.name + " (" + origin + ")");
      *static_cast<bool*>(p) = *b;
      return Status::Ok();
    }
    case Kind::kUint: {
      auto u = ParseUint(Trim(value));
      if (!u || (*u == 0 && !d.allow_zero)) return InvalidArgument("invalid value '" + value + "' for " + d.name + " (" + origin + ")");
      *static_cast<uint64_t*>(p) = *u;
      return Status::Ok();
    }
  }
  return Internal("bad flag kind");
}

std::string ValueOf(const FlagDef& d, Flags& f) {
  void* p = d.field(f);
  switch (d.kind) {
    case Kind::kString: return "\"" + JsonEscape(*static_cast<std::string*>(p)) + "\"";
    case Kind::kBool: return *static_cast<bool*>(p) ? "true" : "false";
    case Kind::kUint: return std::to_string(*static_cast<uint64_t*>(p));
  }
  return "null";
}

// A config-file value into a flag: the reference unmarshals the YAML into
// typed Go fields (a string where a bool belongs is an error, and vice versa);
// here a quoted "true"/"false" is also accepted for a bool, a quoted number
// for an integer and a number for a string. null leaves the flag unset.
Status AssignFile(const FlagDef& d, Flags& f, const FileValue& v, const std::string& key,
                  const std::string& origin) {
  if (v.type == 'n') return Status::Ok();
  auto mismatch = [&](const char* want) {
    const char* have = v.type == 'b' ? "bool" : v.type == 's' ? "string" : "number";
    return InvalidArgument("unmarshal error: line " + std::to_string(v.line) + ": cannot unmarshal " + have +
                           " into " + key + " of type " + want + " (" + origin + ")");
  };
  switch (d.kind) {
    case Kind::kString:
      // Numbers are taken as their text (`devices: 0`); a YAML boolean is not
      // (`on` would silently become "true").
      if (v.type == 'b') return mismatch("string");
      break;
    case Kind::kBool:
      if (v.type != 'b' && v.type != 's') return mismatch("bool");
      break;
    case Kind::kUint:
      if (v.type != 'i' && v.type != 's') return mismatch("integer");
      break;
  }
  return Assign(d, f, v.text, origin);
}

}  // namespace

namespace {

// JSON documents when libyaml is unavailable (with libyaml, JSON is parsed as
// the YAML flow document it is).
yaml::Node FromJson(const nlohmann::json& j) {
  yaml::Node n;
  if (j.is_object()) {
    n.kind = yaml::Node::kMap;
    for (auto it = j.begin(); it != j.end(); ++it) n.map.emplace_back(it.key(), FromJson(it.value()));
  } else if (j.is_array()) {
    n.kind = yaml::Node::kSeq;
    for (const auto& v : j) n.seq.push_back(FromJson(v));
  } else if (j.is_null()) {
    n.kind = yaml::Node::kNull;
  } else if (j.is_string()) {
    n.kind = yaml::Node::kScalar;
    n.value = j.get<std::string>();
  } else {
    n.kind = yaml::Node::kScalar;
    n.plain = true;  // true/false/numbers resolve as in YAML
    n.value = j.dump();
  }
  return n;
}

bool KnownFileKey(const std::string& key) {
  for (const auto& d : Table())
    if (*d.file_key && key == d.file_key) return true;
  for (const auto& a : Aliases())
    if (*a.file_key && key == a.file_key) return true;
  return false;
}

char TypeCode(yaml::ScalarType t) {
  switch (t) {
    case yaml::ScalarType::kNull: return 'n';
    case yaml::ScalarType::kBool: return 'b';
    case yaml::ScalarType::kInt: return 'i';
    case yaml::ScalarType::kFloat: return 'f';
    case yaml::ScalarType::kString: return 's';
  }
  return 's';
}

}  // namespace

Result<ConfigFile> ParseConfigFile(const std::string& body) {
  Result<yaml::Node> doc = Unavailable("unparsed");
  bool extra_docs = false;
  std::string t = Trim(body);
  if (!yaml::Available() && !t.empty() && t[0] == '{') {
    try {
      doc = FromJson(nlohmann::json::parse(t));
    } catch (const std::exception& e) {
      return InvalidArgument(std::string("unmarshal error: ") + e.what());
    }
  } else {
    doc = yaml::Parse(body, &extra_docs);
  }
  if (!doc.ok()) return InvalidArgument("unmarshal error: " + doc.status().message());
  const yaml::Node& root = *doc;
  ConfigFile out;
  if (extra_docs) out.warnings.push_back("config file: only the first YAML document is read");
  if (root.kind == yaml::Node::kNull) return InvalidArgument("missing version field");
  if (root.kind != yaml::Node::kMap)
    return InvalidArgument("unmarshal error: the config file must be a mapping (version: v1, flags: {...})");
  auto scalar = [](const yaml::Node& n, const std::string& key, FileValue* v) -> Status {
    if (n.kind == yaml::Node::kMap || n.kind == yaml::Node::kSeq)
      return InvalidArgument("unmarshal error: line " + std::to_string(n.line) + ": " + key + " must be a scalar, not a " +
                             (n.kind == yaml::Node::kMap ? "mapping" : "sequence"));
    std::string canon;
    v->type = TypeCode(yaml::Resolve(n, &canon));
    v->text = canon;
    v->line = n.line;
    return Status::Ok();
  };
  for (const auto& [k, v] : root.map) {
    if (k == "version") {
      FileValue fv;
      ADP_RETURN_IF_ERROR(scalar(v, "version", &fv));
      out.values["version"] = fv;
    } else if (k == "flags") {
      if (v.kind == yaml::Node::kNull) continue;
      if (v.kind != yaml::Node::kMap)
        return InvalidArgument("unmarshal error: line " + std::to_string(v.line) + ": flags must be a mapping");
      for (const auto& [fk, fv_node] : v.map) {
        if (!KnownFileKey(fk)) {
          out.warnings.push_back("config file line " + std::to_string(fv_node.line) + ": unknown key flags." + fk +
                                 " (ignored)");
          continue;
        }
        FileValue fv;
        ADP_RETURN_IF_ERROR(scalar(fv_node, "flags." + fk, &fv));
        out.values["flags." + fk] = fv;
      }
    } else {
      out.warnings.push_back("config file line " + std::to_string(v.line) + ": unknown key " + k + " (ignored)");
    }
  }
  auto ver = out.values.find("version");
  if (ver == out.values.end() || ver->second.type == 'n' || ver->second.text.empty())
    return InvalidArgument("missing version field");
  if (ver->second.text != "v1") return InvalidArgument("unknown version: " + ver->second.text);
  return out;
}

Result<Config> LoadConfig(int argc, const char* const* argv,
                          const std::map<std::string, std::string>* env_in) {
  std::map<std::string, std::string> env;
  if (env_in) {
    env = *env_in;
  } else {
    for (char** e = environ; e && *e; ++e) {
      const char* eq = strchr(*e, '=');
      if (eq) env[std::string(*e, eq - *e)] = eq + 1;
    }
  }
  Config cfg;
  std::map<std::string, std::string> cli;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--help" || a == "-h") { cfg.show_help = true; continue; }
    if (a == "--version" || a == "-v") { cfg.show_version = true; continue; }
    if (!StartsWith(a, "--")) return InvalidArgument("unexpected argument: " + a);
    std::string name = a.substr(2), value;
    bool has_value = false;
    size_t eq = name.find('=');
    if (eq != std::string::npos) {
      value = name.substr(eq + 1);
      name = name.substr(0, eq);
      has_value = true;
    }
    if (name == "config-file") {
      if (!has_value) {
        if (i + 1 >= argc) return InvalidArgument("flag needs an argument: --config-file");
        value = argv[++i];
      }
      cfg.config_file = value;
      continue;
    }
    const FlagDef* def = nullptr;
    for (const auto& d : Table())
      if (name == d.name) def = &d;
    std::string key = name;
    for (const auto& al : Aliases()) {
      if (def || !*al.name || name != al.name) continue;
      for (const auto& d : Table())
        if (std::string(al.canonical) == d.name) def = &d;
      key = std::string("alias:") + al.canonical;
      cfg.deprecations.push_back("--" + name + " is accepted for compatibility; use --" + al.canonical);
    }
    if (!def) return InvalidArgument("flag provided but not defined: --" + name);
    if (!has_value) {
      if (def->kind == Kind::kBool) {
        value = "true";
      } else {
        if (i + 1 >= argc) return InvalidArgument("flag needs an argument: --" + name);
        value = argv[++i];
      }
    }
    cli[key] = value;
  }
  if (cfg.config_file.empty() && env.count("CONFIG_FILE")) cfg.config_file = env["CONFIG_FILE"];

  std::map<std::string, FileValue> file;
  if (!cfg.config_file.empty()) {
    std::ifstream in(cfg.config_file);
    if (!in) return InvalidArgument("unable to parse config file: error opening config file: " + cfg.config_file);
    std::stringstream ss;
    ss << in.rdbuf();
    auto parsed = ParseConfigFile(ss.str());
    if (!parsed.ok())
      return InvalidArgument("unable to parse config file: error parsing config file: " +
                             parsed.status().message());
    file = std::move(parsed->values);
    cfg.warnings = std::move(parsed->warnings);
  }

  // Precedence: command line > environment > config file > default; at each
  // level the canonical name beats its compatibility alias.
  for (const auto& d : Table()) {
    const AliasDef* alias = nullptr;
    for (const auto& a : Aliases())
      if (std::string(a.canonical) == d.name) alias = &a;
    std::string alias_cli = std::string("alias:") + d.name;
    std::string file_key = std::string("flags.") + d.file_key;
    std::string alias_file = alias && *alias->file_key ? std::string("flags.") + alias->file_key : "";
    Status st;
    if (cli.count(d.name)) {
      st = Assign(d, cfg.flags, cli[d.name], std::string("--") + d.name);
    } else if (alias && cli.count(alias_cli)) {
      st = Assign(d, cfg.flags, cli[alias_cli], std::string("--") + alias->name);
    } else if (*d.env && env.count(d.env)) {
      st = Assign(d, cfg.flags, env[d.env], d.env);
    } else if (alias && *alias->env && env.count(alias->env)) {
      st = Assign(d, cfg.flags, env[alias->env], alias->env);
      cfg.deprecations.push_back(std::string(alias->env) + " is accepted for compatibility; use " + d.env);
    } else if (*d.file_key && file.count(file_key) && file[file_key].type != 'n') {
      st = AssignFile(d, cfg.flags, file[file_key], file_key, cfg.config_file);
    } else if (alias && !alias_file.empty() && file.count(alias_file) && file[alias_file].type != 'n') {
      st = AssignFile(d, cfg.flags, file[alias_file], alias_file, cfg.config_file);
      cfg.deprecations.push_back(std::string("config key ") + alias->file_key +
                                 " is accepted for compatibility; use " + d.file_key);
    }
    if (!st.ok()) return st;
  }
  return cfg;
}

std::string Config::ToJson() const {
  Flags f = flags;
  std::string out = "{\n  \"version\": \"" + version + "\",\n  \"flags\": {";
  bool first = true;
  for (const auto& d : Table()) {
    out += first ? "\n" : ",\n";
    first = false;
    out += "    \"" + std::string(*d.file_key ? d.file_key : d.name) + "\": " + ValueOf(d, f);
  }
  return out + "\n  }\n}";
}

std::vector<FlagInfo> FlagTable() {
  std::vector<FlagInfo> out;
  for (const auto& d : Table()) {
    FlagInfo fi;
    fi.name = d.name;
    fi.env = d.env;
    fi.file_key = d.file_key;
    fi.kind = d.kind == Kind::kBool ? 'b' : d.kind == Kind::kUint ? 'u' : 's';
    fi.allow_zero = d.allow_zero;
    for (const auto& a : Aliases())
      if (fi.name == a.canonical) {
        fi.alias_name = a.name;
        fi.alias_env = a.env;
        fi.alias_file_key = a.file_key;
      }
    out.push_back(std::move(fi));
  }
  return out;
}

std::string UsageText() {
  std::string s =
      "amdgpu-device-plugin: Kubernetes device plugin for AMD Instinct MI355X GPUs\n\n"
      "Usage: amdgpu-device-plugin [flags]\n\nFlags:\n";
  Flags defaults;
  for (const auto& d : Table()) {
    s += "  --" + std::string(d.name) + "  (env " + d.env +
         (*d.file_key ? std::string(", file flags.") + d.file_key : std::string()) + ", default " +
         ValueOf(d, defaults) + ")\n      " + d.help + "\n";
  }
  s += "  --config-file  (env CONFIG_FILE)\n      versioned YAML/JSON config (version: v1, flags: {...})\n";
  s += "\nCompatibility aliases (reference deployments):\n";
  for (const auto& a : Aliases()) {
    s += "  ";
    if (*a.name) s += std::string("--") + a.name + "  ";
    if (*a.env) s += std::string("(env ") + a.env + ")  ";
    s += std::string("-> --") + a.canonical + "\n";
  }
  s += "  --version, --help\n";
  return s;
}

}  // namespace adp::daemon

// Daemon configuration: command-line flags, environment variables and an
// optional versioned config file (YAML or JSON).
//
// Parity: reference cmd/nvidia-device-plugin/main.go:62-130 (flag table with env
// mirrors), main.go:140-169 (validation), api/config/v1/config.go:30-144 (versioned
// file, `version: v1`, precedence CLI > env > file).
//
// Renames for MI355X: --mig-strategy -> --partition-strategy (PARTITION_STRATEGY),
// --nvidia-driver-root -> --driver-root (DRIVER_ROOT), NVIDIA_DRIVER_RESOURCE_CONFIG
// -> RESOURCE_CONFIG. Kept as-is: FAIL_ON_INIT_ERROR, PASS_DEVICE_SPECS,
// DEVICE_LIST_STRATEGY, DEVICE_ID_STRATEGY, CONFIG_FILE.
//
// Fixes: boolean values from the file can be false (B7); resourceConfig can come
// from the file (B8). --pass-device-specs defaults to true: on AMD the device
// nodes are the only thing that makes a GPU usable inside a container (there is
// no runtime hook reading an env var).
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "common/status.h"

namespace adp::daemon {

struct Flags {
  std::string partition_strategy = "none";
  bool fail_on_init_error = true;
  bool pass_device_specs = true;
  std::string device_list_strategy = "envvar";
  std::string device_id_strategy = "uuid";
  std::string driver_root = "/";
  std::string resource_config;
  std::string replica_policy = "auto";
  bool replica_cu_mask = false;
  std::string memory_unit_cu_slots = "proportional";
  std::string plugin_dir = "/var/lib/kubelet/device-plugins/";
  std::string kubelet_socket;  // default: <plugin_dir>/kubelet.sock
  std::string amdsmi_lib;
  std::string devices;         // GPU index filter, e.g. "0,1,2,3" (empty = all)
  uint64_t auto_replica_unit_mib = 1000;
  std::string auto_replica_unit = "auto";  // auto | mib | cu-slot
  std::string resource_prefix = "amd.com";
  bool include_card_nodes = false;
  bool trace = false;
  std::string cdi_spec_dir = "/var/run/cdi";
  bool dry_run = false;
  bool list_grants = false;
  bool smi_report = false;       // print every amdsmi query's status + device-node access, exit
  bool relay_ping = false;       // liveness check of the event relay at --health-event-socket, exit
  bool doctor = false;           // check what a deployment needs on this node, say what to change, exit
  bool health_events = true;     // register amdsmi event notification (needs /dev/kfd access)
  std::string health_event_socket;  // events from the relay at this socket ("" = in-process)
  std::string health_event_extra_types;  // amdsmi event types registered on top, counted only
  bool event_relay = false;         // run as that relay
  uint64_t driver_hbm_poll_ms = 10000;  // driver-side check of enforced grants (0 = off)
  uint64_t driver_hbm_slack_mib = 512;  // HIP runtime allowance per process in that check
  std::string host_proc = "/proc";      // the host's /proc (hostPID, or a hostPath mount)
  std::string kfd_proc_dir = "/sys/class/kfd/kfd/proc";  // GPU processes by host PID ("" = walk all)
  std::string sysfs_root = "/sys";
  std::string drain_file;  // operator drain list: GPUs named in it are advertised Unhealthy
  uint64_t reset_recovery_hold_ms = 120000;  // polled recovery of a GPU_POST_RESET lost in an event gap (0 = off)
  uint64_t reset_flap_limit = 3;             // resets within the window that quarantine a GPU (0 = off)
  uint64_t reset_flap_window_ms = 600000;
  bool defer_layout_changes = false;  // keep serving the old layout while pods hold IDs it would re-mean
  std::string drain, undrain;  // one-shot: add / remove GPUs in the drain file, then exit
  std::string return_to_service;  // one-shot: ask the running daemon to clear GPUs' verdicts, then exit
  uint64_t server_threads = 0;  // 0 -> plugin::DefaultServerThreads()
  std::string metrics_addr;     // "" = no metrics endpoint
  std::string node_labels_file; // "" = no NFD feature file
  std::string pod_resources_socket = "/var/lib/kubelet/pod-resources/kubelet.sock";
  uint64_t busy_poll_us = 50;
  std::string http2_server = "native";
  std::string loop_affinity = "none";  // peer-l3 only helps a visible, single-threaded caller
  std::string health_state_file;  // "" = health verdicts kept in memory only
  bool reject_unhealthy = false;  // Allocate() of an Unhealthy device fails instead of warning
  bool enforce_memory_units = false;  // memory-unit pods get the HBM-cap shim (LD_PRELOAD)
  bool replica_hbm_share = false;     // time-slice replicas hold 1/R of the HBM each
  bool container_hbm_metrics = true;   // per-container HBM use in /metrics (with the HBM-cap shim)
  bool prestart_health_check = false;  // PreStartContainer refuses Unhealthy devices
  bool memcap_ld_so_preload = false;  // also mount /etc/ld.so.preload naming the shim
  std::string memcap_lib;  // the shim in the plugin's filesystem ("" = next to the binary, then /usr/lib/...)
};

struct Config {
  std::string version = "v1";
  Flags flags;
  std::string config_file;
  bool show_version = false;
  bool show_help = false;
  std::vector<std::string> deprecations;  // compatibility aliases that were used
  std::vector<std::string> warnings;      // e.g. unknown config-file keys (logged at startup)
  std::string ToJson() const;
};

// A config-file value: its text and the YAML type it resolved to
// ('s' string, 'b' bool, 'i' int, 'f' float, 'n' null).
struct FileValue {
  std::string text;
  char type = 's';
  int line = 0;
};

struct ConfigFile {
  std::map<std::string, FileValue> values;  // "version", "flags.<key>"
  std::vector<std::string> warnings;
};

// Parses argv + environment (+ the config file they name). `env` lets tests
// inject an environment; nullptr means the process environment.
Result<Config> LoadConfig(int argc, const char* const* argv,
                          const std::map<std::string, std::string>* env = nullptr);

// Parses a versioned config file body (any YAML document, JSON included) into
// (dotted camelCase key -> scalar value). Unknown keys become warnings; a
// `flags` that is not a mapping, or a mapping/sequence where a setting's
// scalar belongs, is an error.
Result<ConfigFile> ParseConfigFile(const std::string& body);

std::string UsageText();

// Every setting and where it can come from (tests, docs): its command-line
// name, environment variable and config-file key ("" = none), its type
// ('s' string, 'b' bool, 'u' unsigned; `allow_zero`: 0 is a value), and the
// compatibility alias of each kind, if any.
struct FlagInfo {
  std::string name, env, file_key;
  char kind = 's';
  bool allow_zero = false;
  std::string alias_name, alias_env, alias_file_key;
};
std::vector<FlagInfo> FlagTable();

}  // namespace adp::daemon

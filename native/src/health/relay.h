// Privilege separation for health events: a minimal relay process registers
// amdsmi event notification -- the one thing the plugin does that needs
// /dev/kfd, which an unprivileged pod's device cgroup denies -- and forwards
// every event record to the daemon over a Unix socket. The daemon (gRPC to the
// kubelet, /metrics on the network) then runs with every capability dropped.
//
// Parity: the reference runs its whole plugin with SYS_ADMIN when MIG
// monitoring needs it, else drop-ALL
// (/root/reference/deployments/helm/nvidia-device-plugin/templates/daemonset.yml:80-93);
// here only the relay container is privileged, and it parses no network or
// kubelet input -- one line per client, "reinit", is all it reads.
//
// Wire protocol (text lines over SOCK_STREAM):
//   relay -> daemon  "hello v1 events=ok processors=<n>"         (on connect)
//                    "hello v1 events=off reason=<text>"       (registration failed)
//                    "hello v1 reinit events=ok processors=<n>" (after a "reinit")
//                    "hello v1 reinit events=off reason=..."   (watchdog: the amdsmi
//                                 wait has not returned, or has kept failing, for
//                                 ADP_RELAY_STUCK_MS, default 10 s; "events=ok"
//                                 again once waits succeed)
//                    "event node=<kfd node|-> bdf=<bdf> part=<partition id> type=<t> <message>"
//   daemon -> relay  "reinit"   re-enumerate (amdsmi_shut_down + init) and register
//                               again, then a "reinit" hello to every client (a new
//                               daemon generation, e.g. after a re-partition). A
//                               daemon takes its event state from that hello only:
//                               the connect hello predates the re-registration.
//                    "scan\t<usage dir>\t<daemon cgroup>"
//                               one driver-side HBM scan (memcap/driver_usage.h) of
//                               the relay's --host-proc: the reply is SerializeScan's
//                               text, then the relay closes that connection (it gets
//                               no events). Reading other containers' /proc/<pid>/fd
//                               needs CAP_SYS_PTRACE; with the scan here the daemon
//                               needs no capability at all.
#pragma once

#include <string>
#include <string_view>

#include "smi/smi.h"

namespace adp::health {

// One parsed relay line (ParseRelayLine). kind: "hello", "event" or "" (malformed).
struct RelayLine {
  std::string kind;
  bool events_ok = false;
  bool after_reinit = false;  // hello sent after a re-enumeration a daemon asked for
  std::string reason;      // hello with events=off
  uint32_t node = 0xffffffffu;  // KFD topology node of the processor ("-" = unreported)
  std::string bdf;
  uint32_t part = 0;
  uint32_t type = 0;
  std::string message;
};
RelayLine ParseRelayLine(std::string_view line);
std::string FormatRelayEvent(const smi::ProcessorInfo& p, uint32_t type, const std::string& message);

// Runs the relay until SIGTERM/SIGINT/SIGQUIT (the caller blocked them and
// passes their signalfd): binds `socket_path` (owner-only; connections from
// another uid are refused by their SO_PEERCRED too), registers events on
// every amdsmi processor and forwards them to every connected daemon. Returns
// the process exit code.
// `proc_root` / `kfd_proc_dir`: where scans read processes (ScanDriverHbm).
struct RelayOptions {
  std::string driver_root = "/";
  std::string proc_root = "/proc";
  std::string kfd_proc_dir = "/sys/class/kfd/kfd/proc";
};
int RunEventRelay(smi::Library* lib, const std::string& socket_path, int signal_fd, const RelayOptions& opts = {});

// Daemon side: connects to the relay (non-blocking), -1 when not reachable.
int ConnectRelay(const std::string& socket_path);

// Liveness probe of a relay (--relay-ping): 0 when it greets within
// `timeout_ms` and its event wait is not stuck (events off for another reason
// -- no /dev/kfd -- is alive: restarting would not help), else 1. Prints the
// greeting or what went wrong.
int PingRelay(const std::string& socket_path, int timeout_ms);

}  // namespace adp::health

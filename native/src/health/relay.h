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
// kubelet input -- one line per client, "reinit" or "scan", is all it reads.
//
// A GPU_POST_RESET nobody is registered for is lost for good (a GPU waiting
// for it stays out of service, health.h), so the relay is built not to lose
// events itself:
//  * every forwarded event carries a sequence number and the relay keeps the
//    last kRelayRingSize of them; a daemon that reconnects (a new monitor
//    generation: SIGHUP, config reload, kubelet restart, re-partition) names
//    the last one it handled and gets the ones it missed replayed;
//  * a daemon's reinit re-enumerates amdsmi only when the daemon's view of the
//    processors (ProcessorFingerprint) differs from the relay's registration --
//    a re-partition -- or the event wait is failing; otherwise the registration,
//    and the kernel's event queue behind it, is kept;
//  * re-enumeration (amdsmi shut_down + init) runs on a thread of its own: the
//    poll loop keeps greeting, scanning and forwarding meanwhile.
// What cannot be replayed is reported as a gap ("gap=1"), and the daemon
// falls back to its polled recovery check for GPUs waiting across it.
//
// Wire protocol (text lines over SOCK_STREAM):
//   relay -> daemon  "hello v1 events=ok processors=<n> relay=<id> gen=<g> seq=<s>"   (on connect)
//                    "hello v1 events=off relay=<id> gen=<g> seq=<s> reason=<text>"
//                    "hello v1 reinit events=ok processors=<n> relay=<id> gen=<g> seq=<s> gap=<0|1>"
//                          the answer to a reinit (to every subscribed client when
//                          the registration was renewed, gap=1 then), and the
//                          watchdog's "events=off ... reason=the amdsmi event wait
//                          has not returned / has failed for <ms> ms" when the wait
//                          hangs or keeps failing for ADP_RELAY_STUCK_MS (default
//                          10 s), "events=ok" again once waits succeed
//                    "event seq=<n> node=<kfd node|-> bdf=<bdf> part=<partition id> type=<t> <message>"
//                          ("node=- bdf=-": on a handle amdsmi never enumerated --
//                          forwarded all the same, the daemon applies its rule for
//                          an event it cannot place)
//                          relay: a random ID of this relay process; gen: its
//                          registration generation (+1 on each re-registration);
//                          seq: the last event sequence number it forwarded;
//                          every hello also carries fp=<the registration's
//                          ProcessorFingerprint> and renew_ms=<how long its last
//                          renewal took>
//   daemon -> relay  "reinit fp=<fingerprint> since=<relay>:<seq>:<gen>|-"
//                          subscribe to events: replays the events after <seq>
//                          that were forwarded while this daemon was away (when
//                          <relay> is this relay and they are still held),
//                          re-enumerates only if <fingerprint> differs from the
//                          registration's (or the wait fails), then answers with a
//                          reinit hello; gap=0 when nothing can have been missed
//                          since <seq>. A bare "reinit" (older daemons) always
//                          re-enumerates and is answered gap=1. A daemon takes its
//                          event state from that hello only: the connect hello
//                          predates its request.
//                    "scan\t<usage dir>\t<daemon cgroup>"
//                          one driver-side HBM scan (memcap/driver_usage.h) of
//                          the relay's --host-proc: the reply is SerializeScan's
//                          text, then the relay closes that connection (it gets
//                          no events). Reading other containers' /proc/<pid>/fd
//                          needs CAP_SYS_PTRACE; with the scan here the daemon
//                          needs no capability at all.
#pragma once

#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

#include "smi/smi.h"

namespace adp::health {

constexpr size_t kRelayRingSize = 1024;

// One parsed relay line (ParseRelayLine). kind: "hello", "event" or "" (malformed).
struct RelayLine {
  std::string kind;
  bool events_ok = false;
  bool after_reinit = false;  // hello sent after a re-enumeration a daemon asked for
  std::string reason;      // hello with events=off
  std::string relay;       // hello: the relay's instance ID ("" = an older relay)
  uint64_t gen = 0;        // hello: registration generation
  uint64_t seq = 0;        // hello: last event forwarded; event: its sequence number (0 = none)
  int gap = -1;            // reinit hello: 0 nothing missed, 1 events may have been missed, -1 not said
  uint32_t node = 0xffffffffu;  // KFD topology node of the processor ("-" = unreported)
  std::string bdf;
  uint32_t part = 0;
  uint32_t type = 0;
  std::string message;
};
RelayLine ParseRelayLine(std::string_view line);
// One daemon -> relay request line, as the (privileged) relay reads it.
// kind: "reinit", "scan" or "" (anything else: ignored).
struct RelayRequest {
  std::string kind;
  std::string fp;                 // reinit: 16 hex digits, "" when absent or not that shape
  bool has_since = false;         // reinit: a well-formed cursor was given
  std::string since_relay;        // (hex, at most 32 characters)
  uint64_t since_seq = 0, since_gen = 0;
  std::string usage_dir, cgroup;  // scan
  bool malformed = false;         // a scan the relay drops: the directory is relative or climbs ("..")
};
RelayRequest ParseRelayRequest(std::string_view line);
// Without the sequence number (the relay's waiter thread; the poll loop numbers the lines).
std::string FormatRelayEvent(const smi::ProcessorInfo& p, uint32_t type, const std::string& message);
// An event on a handle amdsmi never enumerated: "event node=- bdf=- part=0 type=<t> <message>".
std::string FormatUnplacedRelayEvent(uint32_t type, const std::string& message);

// 16 hex digits identifying a processor layout: every processor's PCI address,
// partition ID, KFD node and partition modes, order-independent. Daemon and
// relay compute it from their own enumerations; equal means the relay's event
// registration covers the daemon's processors.
std::string ProcessorFingerprint(const std::vector<smi::ProcessorInfo>& procs);

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
  // --health-event-extra-types of the relay: registered too, forwarded like the rest.
  uint64_t extra_mask = 0;
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

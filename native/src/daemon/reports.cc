#include "daemon/reports.h"

#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <fstream>
#include <iterator>
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
#include "memcap/driver_usage.h"
#include "memcap/usage.h"
#include "plugin/plugin.h"
#include "smi/smi.h"
#include "strategy/strategy.h"

namespace adp::daemon {
namespace {

constexpr const char* kComp = "daemon";

// A Unix socket something listens on (a connect is accepted or queued); a
// stale file refuses.
bool SocketLive(const std::string& path) {
  sockaddr_un addr{};
  if (path.size() >= sizeof(addr.sun_path)) return false;
  int fd = socket(AF_UNIX, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (fd < 0) return false;
  addr.sun_family = AF_UNIX;
  memcpy(addr.sun_path, path.c_str(), path.size());
  int rc = connect(fd, reinterpret_cast<sockaddr*>(&addr), sizeof(addr));
  bool live = rc == 0 || errno == EINPROGRESS || errno == EAGAIN;
  close(fd);
  return live;
}

}  // namespace

// --list-grants: the enforced grants' accounting files, as JSON on stdout
// (kubectl exec into the plugin pod; the numbers /metrics reports per pod).
int ListGrants(const std::string& dir) {
  std::string out = "{\"dir\": \"" + JsonEscape(dir) + "\", \"grants\": [";
  auto list = [&out](const std::vector<uint64_t>& v) {
    out += '[';
    for (size_t i = 0; i < v.size(); ++i) out += (i ? ", " : "") + std::to_string(v[i]);
    out += ']';
  };
  bool first = true;
  for (const auto& u : memcap::ReadAll(dir)) {
    out += first ? "\n  " : ",\n  ";
    first = false;
    out += "{\"key\": \"" + u.key + "\", \"ids\": \"" + JsonEscape(u.ids) + "\", \"used\": ";
    list(u.used);
    out += ", \"granted\": ";
    list(u.cap);
    out += ", \"peak\": ";
    list(u.peak);
    out += ", \"refused\": ";
    list(u.refused);
    out += ", \"processes\": " + std::to_string(u.processes) + ", \"mtime\": " + std::to_string(u.mtime_s) + "}";
  }
  out += first ? "]}\n" : "\n]}\n";
  fputs(out.c_str(), stdout);
  return 0;
}

// --dry-run: what this node would advertise, as JSON on stdout.
int DryRun(smi::Library* lib, const Validated& v, const Config& cfg) {
  auto snap = inventory::BuildSnapshot(lib, v.bopts);
  if (!snap.ok()) {
    LOG_ERROR(kComp, "device enumeration failed: %s", snap.status().ToString().c_str());
    return 1;
  }
  auto specs = strategy::BuildPluginSpecs(**snap, v.partition, v.rc, cfg.flags.resource_prefix);
  if (!specs.ok()) {
    LOG_ERROR(kComp, "error creating partition strategy: %s", specs.status().message().c_str());
    return 1;
  }
  std::string out = "{\"amdsmi\": \"" + JsonEscape((*snap)->smi_version) + "\", \"gpus\": [";
  for (size_t i = 0; i < (*snap)->gpus.size(); ++i) {
    const auto& g = (*snap)->gpus[i];
    out += (i ? ", " : "") + std::string("{\"index\": ") + std::to_string(g.node_index) + ", \"uuid\": \"" +
           JsonEscape(g.uuid) + "\", \"bdf\": \"" + g.bdf + "\", \"mode\": \"" + g.compute_mode + "/" +
           g.memory_mode + "\", \"partitions\": " + std::to_string(g.partitions.size()) +
           ", \"vram_mib\": " + std::to_string(g.vram_mib) + ", \"vram_source\": \"" + g.vram_source +
           "\", \"profile\": \"" + JsonEscape(g.PartitionProfile()) + "\", \"numa\": " + std::to_string(g.numa) +
           ", \"xcds\": " + std::to_string(g.xcds) + ", \"cus\": " + std::to_string(g.cus) + "}";
  }
  out += "], \"labels\": {";
  bool first_label = true;
  for (const auto& [k, val] : inventory::NodeLabels(**snap)) {
    out += std::string(first_label ? "" : ", ") + "\"" + JsonEscape(k) + "\": \"" + JsonEscape(val) + "\"";
    first_label = false;
  }
  out += "}, \"resources\": [";
  bool first = true;
  for (const auto& s : *specs) {
    plugin::Plugin p(*snap, s, v.popts);
    if (p.device_count() == 0) continue;
    out += std::string(first ? "" : ", ") + "{\"resource\": \"" + JsonEscape(s.resource_name) +
           "\", \"socket\": \"" + JsonEscape(p.socket_path()) + "\", \"devices\": " +
           std::to_string(p.device_count()) + ", \"allocatable\": " + std::to_string(p.advertised_count()) +
           ", \"replicated\": " + (p.replicated() ? "true" : "false");
    // --replica-cu-mask: CUs of each replica's share per device ([] = not CU-partitioned).
    out += ", \"replica_cus\": [";
    for (size_t i = 0; i < p.units().size(); ++i) {
      const auto& rc = p.units()[i].replica_cus;
      out += (i ? ", " : "") + std::to_string(rc.empty() ? 0 : rc[0].second - rc[0].first + 1);
    }
    out += "]}";
    first = false;
  }
  out += "]}";
  printf("%s\n", out.c_str());
  fflush(stdout);
  return 0;
}

// --smi-report: every amdsmi query's status per processor, and which device
// nodes open -- what a pod's privileges and device cgroup leave working.
int SmiReport(smi::Library* lib, const Validated& v, const Config& cfg) {
  std::string out = lib->QueryReport();
  out.pop_back();  // the closing brace
  out += ", \"device_access\": [";
  auto snap = inventory::BuildSnapshot(lib, v.bopts);
  if (snap.ok()) {
    auto access = inventory::ProbeDeviceAccess(**snap, cfg.flags.driver_root);
    for (size_t i = 0; i < access.size(); ++i)
      out += std::string(i ? ", " : "") + "{\"node\": \"" + JsonEscape(access[i].path) + "\", \"errno\": " +
             std::to_string(access[i].err) + ", \"error\": \"" + (access[i].err ? strerror(access[i].err) : "") +
             "\"}";
  }
  // What sysfs answers without the render node: KFD topology CUs and the
  // board's PCI product name, per processor (the fallbacks for asic_info).
  out += "], \"sysfs\": [";
  if (snap.ok() && !cfg.flags.sysfs_root.empty()) {
    const std::string topo = cfg.flags.sysfs_root + "/class/kfd/kfd/topology/nodes";
    bool first = true;
    for (const auto& p : (*snap)->procs) {
      out += std::string(first ? "" : ", ") + "{\"bdf\": \"" + JsonEscape(p.bdf) + "\", \"kfd_node\": " +
             (p.kfd_node == inventory::kNoKfdNode ? std::string("null") : std::to_string(p.kfd_node)) +
             ", \"topology_cus\": " +
             std::to_string(p.kfd_node == inventory::kNoKfdNode ? 0 : inventory::KfdTopologyCus(topo, p.kfd_node)) +
             ", \"pci_product_name\": \"" + JsonEscape(inventory::PciProductName(cfg.flags.sysfs_root, p.bdf)) +
             "\"}";
      first = false;
    }
  }
  out += "], \"enumeration\": \"" + std::string(snap.ok() ? "ok" : JsonEscape(snap.status().ToString())) + "\"}";
  printf("%s\n", out.c_str());
  fflush(stdout);
  return 0;
}

void DoctorReport::Line(const char* level, const std::string& what) {
  printf("%-5s %s\n", level, what.c_str());
  if (!strcmp(level, "ok")) ++ok;
  else if (!strcmp(level, "warn")) ++warn;
  else ++fail;
}

int DoctorReport::Finish() {
  printf("doctor: %d ok, %d warning(s), %d failure(s)\n", ok, warn, fail);
  fflush(stdout);
  return fail ? 1 : 0;
}

int Doctor(smi::Library* lib, const Validated& v, const Config& cfg, DoctorReport& d) {
  const Flags& f = cfg.flags;
  d.Line("ok", "amdsmi " + lib->Version() + " (" + lib->path() + ")");
  auto snap = inventory::BuildSnapshot(lib, v.bopts);
  if (!snap.ok()) {
    d.Line("FAIL", "enumeration: " + snap.status().ToString() + " -- is the amdgpu driver loaded, and are the "
                   "GPUs visible to this container?");
    return d.Finish();
  }
  const auto& s = **snap;
  if (s.gpus.empty()) {
    d.Line("FAIL", "enumeration: no GPU" + std::string(f.devices.empty() ? "" : " matches --devices " + f.devices));
    return d.Finish();
  }
  size_t parts = 0;
  for (const auto& g : s.gpus) parts += g.partitions.size();
  d.Line("ok", "enumeration: " + std::to_string(s.gpus.size()) + " GPU(s), " + std::to_string(parts) +
                   " compute partition(s), " + s.gpus[0].compute_mode + "/" + s.gpus[0].memory_mode);
  if (s.cus_unknown)
    d.Line(f.replica_cu_mask ? "FAIL" : "warn",
           "CU counts: unknown on " + std::to_string(s.cus_unknown) + " processor(s) -- amdsmi's asic_info needs the "
           "render node and KFD topology (under --sysfs-root " + f.sysfs_root + ") is not readable" +
           (f.replica_cu_mask ? ", so --replica-cu-mask cuts no CU shares" : ""));
  else if (s.cus_from_topology)
    d.Line("ok", "CU counts: from KFD topology on " + std::to_string(s.cus_from_topology) +
                     " processor(s) (asic_info needs the render node, which this container may not open)");
  {
    // How a container numbers its GPUs: KFD topology-node order (what every
    // per-device list Allocate() returns follows), not necessarily amdsmi's.
    std::vector<std::pair<uint32_t, int>> nodes;
    bool known = true;
    for (const auto& g : s.gpus) {
      known = known && g.kfd_node != inventory::kNoKfdNode;
      nodes.emplace_back(g.kfd_node, g.node_index);
    }
    std::sort(nodes.begin(), nodes.end());
    std::string order;
    bool differs = false;
    for (size_t i = 0; i < nodes.size(); ++i) {
      order += (i ? "," : "") + std::to_string(nodes[i].second);
      differs = differs || nodes[i].second != s.gpus[i].node_index;
    }
    if (!known)
      d.Line("warn", "device order: amdsmi reports no KFD topology node for some GPU -- per-device container lists "
                     "(HSA_CU_MASK, AMD_GPU_MEMORY_*) assume HIP numbers GPUs in amdsmi order");
    else
      d.Line("ok", "device order: containers number GPUs in KFD-node order (amdsmi indices " + order + ")" +
                       (differs ? ", which differs from amdsmi's order: per-device container lists follow KFD order"
                                : ""));
  }
  auto specs = strategy::BuildPluginSpecs(s, v.partition, v.rc, f.resource_prefix);
  if (!specs.ok()) {
    d.Line("FAIL", "partition strategy: " + specs.status().message());
  } else {
    std::string what, unit_cus;
    for (const auto& spec : *specs) {
      plugin::Plugin p(*snap, spec, v.popts);
      if (p.device_count() == 0) continue;
      what += (what.empty() ? "" : ", ") + spec.resource_name + " x" + std::to_string(p.advertised_count());
      if (spec.variant.auto_replicas && !p.units().empty() && !p.units().front().replica_cus.empty())
        unit_cus = spec.resource_name;
    }
    if (what.empty()) d.Line("FAIL", "resources: none would be advertised (partition strategy / --devices)");
    else d.Line("ok", "resources: " + what);
    if (!unit_cus.empty() && v.popts.cu_slot_units)
      d.Line("ok", "CU shares: " + unit_cus + " units are CU slots, so every pod owns whole slots (disjoint, "
                   "none idle)");
    else if (!unit_cus.empty() && v.popts.whole_cu_slots)
      d.Line("warn", "CU shares: " + unit_cus + " pods get only the CU slots their units fill (disjoint), but "
                     "MiB units do not line up with slots, so CUs of partly held slots sit idle -- "
                     "--auto-replica-unit cu-slot makes every unit a slot");
    else if (!unit_cus.empty())
      d.Line("warn", "CU shares: " + unit_cus + " pods get proportional CU slots, so packed neighbours can share "
                     "a boundary slot and slow each other's kernels -- --auto-replica-unit cu-slot (helm "
                     "autoReplicaUnit: cu-slot) makes every unit a whole slot");
  }
  auto nodes = inventory::ProbeDeviceAccess(s, f.driver_root);
  std::string acc = inventory::DescribeAccess(nodes);
  bool only_denied = !nodes.empty();
  for (const auto& n : nodes) only_denied = only_denied && (n.err == 0 || n.err == EPERM || n.err == EACCES);
  if (acc == "ok") {
    d.Line("ok", "device nodes: " + std::to_string(nodes.size()) + " openable");
  } else if (only_denied && !f.health_event_socket.empty()) {
    // The chart's layout: an unprivileged plugin next to the event relay needs
    // none of them (events and scans are the relay's, CU counts and product
    // names come from sysfs).
    d.Line("ok", "device nodes: denied by this container's device cgroup, as expected for the unprivileged "
                 "plugin next to the event relay");
  } else {
    d.Line("warn", "device nodes: " + acc);
  }
  if (!f.health_events) {
    d.Line("warn", "health events: off by configuration -- resets are seen by polling only");
  } else if (!f.health_event_socket.empty()) {
    // Privilege separation: the relay holds the registration; ask it.
    int fd = health::ConnectRelay(f.health_event_socket);
    std::string hello;
    if (fd >= 0) {
      pollfd p{fd, POLLIN, 0};
      char buf[512];
      if (poll(&p, 1, 2000) > 0) {
        ssize_t n = recv(fd, buf, sizeof(buf) - 1, 0);
        if (n > 0) hello.assign(buf, static_cast<size_t>(n));
      }
      close(fd);
    }
    hello = hello.substr(0, hello.find('\n'));
    auto line = health::ParseRelayLine(hello);
    if (fd < 0)
      d.Line("warn", "health events: the event relay at " + f.health_event_socket + " is not reachable -- is the "
                     "event-relay container running? Resets are seen by polling until it is");
    else if (line.kind == "hello" && line.events_ok)
      d.Line("ok", "health events: through the event relay at " + f.health_event_socket + " (" + hello + ")");
    else
      d.Line("warn", "health events: the event relay at " + f.health_event_socket + " reports " +
                         (line.reason.empty() ? "no hello" : line.reason));
  } else {
    std::vector<void*> handles;
    for (const auto& p : s.procs) handles.push_back(p.handle);
    uint64_t mask = smi::EventMask(smi::kEvtGpuPreReset) | smi::EventMask(smi::kEvtGpuPostReset);
    Status es = lib->EventsInit(handles, mask);
    if (es.ok()) {
      lib->EventsStop(handles);
      d.Line("ok", "health events: amdsmi event notification registers (GPU_PRE_RESET / GPU_POST_RESET)");
    } else {
      int kerr = inventory::KfdAccessErrno(f.driver_root);
      d.Line("warn", "health events: " + es.ToString() +
                         (kerr == EPERM ? " -- /dev/kfd denied by the device cgroup: run the plugin privileged "
                                          "(helm healthEvents: true)"
                                        : ""));
    }
  }
  size_t ecc_ok = 0;
  for (const auto& g : s.gpus)
    if (lib->UncorrectableErrors(s.procs[g.partitions.front().handle].handle).ok()) ++ecc_ok;
  if (ecc_ok == s.gpus.size()) d.Line("ok", "uncorrectable ECC readable on every GPU");
  else d.Line("warn", "uncorrectable ECC readable on " + std::to_string(ecc_ok) + " of " +
                          std::to_string(s.gpus.size()) + " GPU(s): ECC failures are not detected on the others");
  std::string ksock = v.popts.kubelet_socket.empty() ? PathJoin(f.plugin_dir, "kubelet.sock") : v.popts.kubelet_socket;
  struct stat st;
  if (stat(ksock.c_str(), &st) == 0 && S_ISSOCK(st.st_mode)) d.Line("ok", "kubelet socket " + ksock);
  else d.Line("warn", "kubelet socket " + ksock + " not found -- is the kubelet's device-plugin directory mounted "
                      "(--device-plugin-path)? The plugin waits for it");
  std::string probe = PathJoin(f.plugin_dir, ".amdgpu-dp-doctor-" + std::to_string(getpid()));
  int fd = open(probe.c_str(), O_WRONLY | O_CREAT | O_EXCL | O_CLOEXEC, 0600);
  if (fd >= 0) {
    close(fd);
    unlink(probe.c_str());
    d.Line("ok", "plugin directory " + f.plugin_dir + " writable");
  } else {
    d.Line("FAIL", "plugin directory " + f.plugin_dir + " not writable (" + strerror(errno) +
                       "): the plugin sockets go there");
  }
  // Who else serves in the kubelet's directory: another instance of this
  // plugin (a rollout, or a second DaemonSet with the same resources), or
  // other device plugins -- a second AMD GPU plugin advertising amd.com/gpu
  // makes the kubelet keep whichever registered last.
  {
    std::set<std::string> ours;
    if (specs.ok())
      for (const auto& spec : *specs) ours.insert(spec.socket_name);
    std::string mine, others;
    bool gpu_like = false;
    if (DIR* dir = opendir(f.plugin_dir.c_str())) {
      while (dirent* e = readdir(dir)) {
        std::string name = e->d_name, path = PathJoin(f.plugin_dir, name);
        struct stat sst;
        if (path == ksock || stat(path.c_str(), &sst) != 0 || !S_ISSOCK(sst.st_mode) || !SocketLive(path)) continue;
        std::string& list = ours.count(name) ? mine : others;
        list += (list.empty() ? "" : ", ") + name;
        if (!ours.count(name) && (ToLower(name).find("amd") != std::string::npos ||
                                  ToLower(name).find("gpu") != std::string::npos))
          gpu_like = true;
      }
      closedir(dir);
    }
    if (!mine.empty())
      d.Line("warn", "plugin sockets: another instance of this plugin serves " + mine +
                         " (a rollout in progress, or a second DaemonSet); starting this one takes them over");
    if (!others.empty())
      d.Line(gpu_like ? "warn" : "ok",
             "other device plugins serve here: " + others +
                 (gpu_like ? " -- if one of them also advertises this plugin's resources, the kubelet keeps "
                             "whichever registered last: run one GPU plugin per node"
                           : ""));
  }
  if (f.enforce_memory_units) {
    std::string src = MemcapSource(f);
    if (src.empty()) d.Line("FAIL", "--enforce-memory-units: libadp_memcap.so not found (--memcap-lib)");
    else d.Line("ok", "HBM-cap shim " + src);
    if (!f.metrics_addr.empty() && f.driver_hbm_poll_ms > 0 && !f.health_event_socket.empty()) {
      // The scan runs in the event relay (its privilege, its --host-proc).
      int rfd = health::ConnectRelay(f.health_event_socket);
      if (rfd >= 0) fcntl(rfd, F_SETFL, fcntl(rfd, F_GETFL) & ~O_NONBLOCK);
      auto scan = rfd < 0 ? Result<memcap::DriverScan>(Unavailable("not reachable"))
                          : memcap::RemoteScan(rfd, PathJoin(f.plugin_dir, "amdgpu-dp/usage"), memcap::SelfCgroup(),
                                               10000);
      if (rfd >= 0) close(rfd);
      if (!scan.ok())
        d.Line("warn", "driver-side HBM check: the event relay at " + f.health_event_socket + " ran no scan (" +
                           scan.status().ToString() + ") -- start the relay container (--event-relay)");
      else if (scan->pid_source == "proc" && scan->pids_scanned < 5)
        d.Line("warn", "driver-side HBM check: the event relay sees only " + std::to_string(scan->pids_scanned) +
                           " process(es) -- mount the host's /proc into it and point its --host-proc there");
      else if (scan->fd_dirs_unreadable == 0)
        d.Line("ok", "driver-side HBM check: the event relay reads " + std::to_string(scan->pids_scanned) +
                         " processes (" + scan->pid_source + " list)");
      else
        d.Line("warn", "driver-side HBM check: " + std::to_string(scan->fd_dirs_unreadable) + " of " +
                           std::to_string(scan->pids_scanned) + " processes not readable by the event relay -- "
                           "run it privileged, with the host's /proc at --host-proc");
    } else if (!f.metrics_addr.empty() && f.driver_hbm_poll_ms > 0) {
      memcap::DriverScan scan = memcap::ScanDriverHbm(f.host_proc, {}, memcap::SelfCgroup());
      if (scan.fd_dirs_unreadable == 0)
        d.Line("ok", "driver-side HBM check: " + std::to_string(scan.pids_scanned) + " processes readable under " +
                         f.host_proc);
      else
        d.Line("warn", "driver-side HBM check: " + std::to_string(scan.fd_dirs_unreadable) + " of " +
                           std::to_string(scan.pids_scanned) + " processes under " + f.host_proc +
                           " not readable -- run privileged, with hostPID or the host's /proc at --host-proc");
    }
  }
  if (!f.health_state_file.empty()) {
    std::string dir = f.health_state_file.substr(0, f.health_state_file.rfind('/'));
    if (access(dir.empty() ? "/" : dir.c_str(), W_OK) == 0) d.Line("ok", "health state file " + f.health_state_file);
    else d.Line("warn", "health state file " + f.health_state_file + ": directory not writable -- verdicts will "
                        "not outlive a container restart");
    // What it holds against this node's GPUs now (the operator's next question).
    health::Ledger ledger(f.health_state_file);
    for (const auto& [gpu, reason] : ledger.Failed(s)) {
      const std::string gap = ledger.Get(health::Ledger::KeyOf(s.gpus[gpu])).gap;
      d.Line("warn", "GPU " + s.gpus[gpu].bdf + " is out of service by the state file: " + reason +
                         (gap.empty() ? "" : " (after an event gap -- " + gap + " -- the polled check returns it)") +
                         " -- once repaired, --return-to-service " + s.gpus[gpu].bdf);
    }
  }
  if (!f.drain_file.empty()) {
    // The drain list: what it takes out of service here, and names that match
    // no GPU of this node (a typo drains nothing, silently otherwise).
    std::ifstream in(f.drain_file);
    std::string text((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    std::set<std::string> names = health::DrainTokens(text), known;
    std::vector<std::string> drained;
    for (const auto& g : s.gpus) {
      const std::set<std::string> own = health::DrainNames(g);
      known.insert(own.begin(), own.end());
      if (std::any_of(own.begin(), own.end(), [&](const std::string& n) { return names.count(n) > 0; }))
        drained.push_back(g.bdf);
    }
    std::vector<std::string> unknown;
    for (const auto& n : names)
      if (!known.count(n)) unknown.push_back(n);
    if (!drained.empty())
      d.Line("warn", "drained by the operator (" + f.drain_file + "): " + Join(drained, ", ") +
                         " -- advertised Unhealthy until --undrain");
    if (!unknown.empty())
      d.Line("warn", "the drain file " + f.drain_file + " names no GPU of this node as: " + Join(unknown, ", ") +
                         " -- those entries drain nothing here (PCI address, UUID, partition UUID or node index)");
    if (access((f.drain_file + ".return").c_str(), F_OK) == 0)
      d.Line("warn", "a return-to-service request is waiting in " + f.drain_file + ".return: no running daemon "
                     "with health checks has taken it");
  }
  double budget = plugin::CpuBudget();
  char b[160];
  snprintf(b, sizeof(b), "CPU budget %.2f CPUs: %d gRPC loop(s) per socket, busy-poll %s", budget,
           f.server_threads > 0 ? static_cast<int>(f.server_threads) : plugin::DefaultServerThreads(),
           budget < 2.0 ? "off (under 2 CPUs)" : "on");
  d.Line("ok", b);
  return d.Finish();
}

int DrainCommand(smi::Library* lib, const Validated& v, const Config& cfg) {
  const Flags& f = cfg.flags;
  if (f.drain_file.empty()) {
    fprintf(stderr, "--drain/--undrain/--return-to-service need --drain-file (DP_DRAIN_FILE)\n");
    return 1;
  }
  auto snap = inventory::BuildSnapshot(lib, v.bopts);
  if (!snap.ok()) {
    fprintf(stderr, "enumeration failed: %s\n", snap.status().ToString().c_str());
    return 1;
  }
  auto resolve = [&](const std::string& list, std::vector<const inventory::PhysicalGpu*>* out) -> bool {
    for (const auto& id : Split(list, ',')) {
      std::string t = Trim(id);
      if (t.empty()) continue;
      const inventory::PhysicalGpu* hit = nullptr;
      for (const auto& g : (*snap)->gpus)
        if (health::DrainNames(g).count(t)) hit = &g;
      if (!hit) {
        fprintf(stderr, "no GPU of this node is named %s\n", t.c_str());
        return false;
      }
      out->push_back(hit);
    }
    return true;
  };
  std::vector<const inventory::PhysicalGpu*> add, remove, back;
  if (!resolve(f.drain, &add) || !resolve(f.undrain, &remove) || !resolve(f.return_to_service, &back)) return 1;
  if (!back.empty()) {
    // A request, not an edit of the state file the daemon keeps writing: the
    // monitor takes the file (rename) at its next poll and clears the GPUs.
    const std::string req = f.drain_file + ".return";
    std::string body;
    {
      std::ifstream in(req);
      for (std::string line; std::getline(in, line);) body += line + "\n";
    }
    const std::set<std::string> listed = health::DrainTokens(body);
    for (const auto* g : back) {
      bool already = false;
      for (const auto& n : health::DrainNames(*g)) already = already || listed.count(n);
      if (!already) body += g->bdf + "  # " + g->uuid + "\n";
    }
    std::string tmp = req + ".tmp." + std::to_string(getpid());
    int fd = open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    bool ok = fd >= 0 && write(fd, body.data(), body.size()) == static_cast<ssize_t>(body.size());
    if (fd >= 0) close(fd);
    if (!ok || rename(tmp.c_str(), req.c_str()) != 0) {
      fprintf(stderr, "cannot write %s: %s\n", req.c_str(), strerror(errno));
      unlink(tmp.c_str());
      return 1;
    }
    for (const auto* g : back)
      printf("%s (%s): back in service at the daemon's next health poll (request in %s)\n", g->bdf.c_str(),
             g->uuid.c_str(), req.c_str());
    fflush(stdout);
    // Wait (a little) for the daemon to take it: two poll intervals, 2..30 s.
    const health::HealthConfig hc = health::HealthConfig::FromEnv();
    const int wait_ms = hc.disabled || hc.poll_interval_ms <= 0
                            ? 0
                            : std::min(30000, std::max(2000, 2 * hc.poll_interval_ms));
    struct stat st;
    for (int waited = 0; waited < wait_ms && stat(req.c_str(), &st) == 0; waited += 50) usleep(50000);
    if (stat(req.c_str(), &st) == 0)
      fprintf(stderr, "the request is still waiting after %d ms: is the plugin running here with health checks on "
              "(DP_DISABLE_HEALTHCHECKS unset, DP_HEALTH_POLL_MS > 0) and this --drain-file? It stays queued.\n",
              wait_ms);
    else
      printf("taken by the running daemon\n");
    if (add.empty() && remove.empty()) return 0;
  }

  std::vector<std::string> lines;
  {
    std::ifstream in(f.drain_file);
    for (std::string line; std::getline(in, line);) lines.push_back(line);
  }
  auto names_line = [&](const std::string& line, const inventory::PhysicalGpu* g) {
    auto tokens = health::DrainTokens(line);
    for (const auto& n : health::DrainNames(*g))
      if (tokens.count(n)) return true;
    return false;
  };
  // Only this GPU's names leave a line; other GPUs named with it stay drained.
  for (const auto* g : remove) {
    const std::set<std::string> names = health::DrainNames(*g);
    std::vector<std::string> next;
    for (const auto& l : lines) {
      if (!names_line(l, g)) {
        next.push_back(l);
        continue;
      }
      std::string rest = health::RemoveDrainNames(l, names);
      if (!rest.empty()) {
        fprintf(stderr, "kept on the same line: %s\n", rest.c_str());
        next.push_back(rest);
      }
    }
    lines = std::move(next);
  }
  for (const auto* g : add) {
    bool listed = false;
    for (const auto& l : lines) listed = listed || names_line(l, g);
    if (!listed) lines.push_back(g->bdf + "  # " + g->uuid);
  }
  std::string body;
  for (const auto& l : lines) body += l + "\n";
  std::string tmp = f.drain_file + ".tmp." + std::to_string(getpid());
  int fd = open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  bool ok = fd >= 0 && write(fd, body.data(), body.size()) == static_cast<ssize_t>(body.size());
  if (fd >= 0) close(fd);
  if (!ok || rename(tmp.c_str(), f.drain_file.c_str()) != 0) {
    fprintf(stderr, "cannot write %s: %s\n", f.drain_file.c_str(), strerror(errno));
    unlink(tmp.c_str());
    return 1;
  }
  printf("%s", body.c_str());
  fflush(stdout);
  return 0;
}

}  // namespace adp::daemon

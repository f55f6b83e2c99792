#include "daemon/supervisor.h"

#include "daemon/reports.h"
#include "daemon/validate.h"

#include <dirent.h>
#include <errno.h>
#include <poll.h>
#include <signal.h>
#include <fcntl.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/inotify.h>
#include <sys/signalfd.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <sys/timerfd.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <memory>
#include <tuple>
#include <set>
#include <map>
#include <mutex>
#include <vector>

#include "alloc/replicas.h"
#include "common/log.h"
#include "common/strings.h"
#include "health/health.h"
#include "health/relay.h"
#include "inventory/inventory.h"
#include "metrics/metrics.h"
#include "memcap/driver_usage.h"
#include "memcap/usage.h"
#include "podresources/podresources.h"
#include "plugin/plugin.h"
#include "smi/smi.h"
#include "strategy/strategy.h"

namespace adp::daemon {
namespace {

constexpr const char* kComp = "daemon";
constexpr int kMaxBackoffMs = 30000;

// --enforce-memory-units: copies the shim into <plugin dir>/amdgpu-dp/ -- a
// host path the container runtime can bind-mount into pods (the kubelet wipes
// the directory when it restarts; every plugin (re)start installs it again) --
// and returns that path, or "" (logged) when it cannot.
std::string InstallMemcap(const Flags& f) {
  std::string src = MemcapSource(f);
  FILE* in = src.empty() ? nullptr : fopen(src.c_str(), "rb");
  if (!in) {
    LOG_ERROR(kComp, "--enforce-memory-units: cannot read %s: %s; memory units are not enforced",
              src.empty() ? "libadp_memcap.so" : src.c_str(), strerror(errno));
    return "";
  }
  std::string body;
  char buf[65536];
  for (size_t n; (n = fread(buf, 1, sizeof(buf), in)) > 0;) body.append(buf, n);
  fclose(in);
  std::string dir = PathJoin(f.plugin_dir, "amdgpu-dp");
  std::string dst = PathJoin(dir, "libadp_memcap.so");
  if (FILE* cur = fopen(dst.c_str(), "rb")) {  // already there and identical: keep the inode
    std::string have;
    for (size_t n; (n = fread(buf, 1, sizeof(buf), cur)) > 0;) have.append(buf, n);
    fclose(cur);
    if (have == body) return dst;
  }
  mkdir(dir.c_str(), 0755);
  std::string tmp = dst + ".tmp";
  FILE* out = fopen(tmp.c_str(), "wb");
  bool ok = out && fwrite(body.data(), 1, body.size(), out) == body.size();
  if (out) ok = (fclose(out) == 0) && ok;
  // A new inode each time: running containers keep the library they mapped.
  if (!ok || chmod(tmp.c_str(), 0644) != 0 || rename(tmp.c_str(), dst.c_str()) != 0) {
    LOG_ERROR(kComp, "--enforce-memory-units: cannot install %s: %s; memory units are not enforced", dst.c_str(),
              strerror(errno));
    unlink(tmp.c_str());
    return "";
  }
  LOG_INFO(kComp, "HBM-cap shim installed at %s (from %s)", dst.c_str(), src.c_str());
  return dst;
}

// --memcap-ld-so-preload: <plugin dir>/amdgpu-dp/ld.so.preload naming the
// shim's path in the container; returns its path, or "" (logged).
std::string InstallPreloadList(const Flags& f) {
  std::string path = PathJoin(PathJoin(f.plugin_dir, "amdgpu-dp"), "ld.so.preload");
  std::string want = std::string(plugin::kMemcapContainerPath) + "\n";
  if (FILE* cur = fopen(path.c_str(), "rb")) {
    char buf[512];
    size_t n = fread(buf, 1, sizeof(buf), cur);
    fclose(cur);
    if (std::string(buf, n) == want) return path;
  }
  std::string tmp = path + ".tmp";
  FILE* out = fopen(tmp.c_str(), "wb");
  bool ok = out && fwrite(want.data(), 1, want.size(), out) == want.size();
  if (out) ok = (fclose(out) == 0) && ok;
  if (!ok || chmod(tmp.c_str(), 0644) != 0 || rename(tmp.c_str(), path.c_str()) != 0) {
    LOG_ERROR(kComp, "--memcap-ld-so-preload: cannot write %s: %s", path.c_str(), strerror(errno));
    unlink(tmp.c_str());
    return "";
  }
  return path;
}

// Atomically replaces `path` with one `key=value` line per label.
void WriteLabels(const std::string& path, const inventory::Snapshot& snap) {
  std::string body;
  for (const auto& [k, v] : inventory::NodeLabels(snap)) body += k + "=" + v + "\n";
  std::string tmp = path + ".tmp";
  FILE* f = fopen(tmp.c_str(), "w");
  bool ok = f && fwrite(body.data(), 1, body.size(), f) == body.size();
  if (f) ok = (fclose(f) == 0) && ok;
  if (!ok || rename(tmp.c_str(), path.c_str()) != 0) {
    LOG_WARN(kComp, "cannot write node labels to %s: %s", path.c_str(), strerror(errno));
    unlink(tmp.c_str());
    return;
  }
  LOG_INFO(kComp, "wrote node labels to %s", path.c_str());
}

// Two resources that both hand a container per-device lists numbered from HIP
// device 0 (HSA_CU_MASK agents, AMD_GPU_MEMORY_*): a container requesting both
// gets one value per name (the kubelet merges the plugins' envs), numbered as
// if that plugin's devices were all it had.
void WarnSharedDeviceLists(const std::vector<std::unique_ptr<plugin::Plugin>>& plugins) {
  std::vector<std::string> masks, grants;
  for (const auto& p : plugins) {
    if (p->device_count() == 0) continue;
    if (p->sets_cu_masks()) masks.push_back(p->resource_name());
    if (p->grants_hbm()) grants.push_back(p->resource_name());
  }
  auto warn = [](const std::vector<std::string>& rs, const char* what) {
    if (rs.size() < 2) return;
    std::string names;
    for (const auto& r : rs) names += (names.empty() ? "" : ", ") + r;
    LOG_WARN(kComp, "%s each set %s numbered from the container's first GPU: a container that requests more "
             "than one of them gets only one plugin's list (the kubelet keeps one value per variable), "
             "numbered without the other's devices -- request one of them per container", names.c_str(), what);
  };
  warn(masks, "HSA_CU_MASK");
  warn(grants, "AMD_GPU_MEMORY_LIMIT_MIB/_FRACTION/_DEVICES");
}

void ArmTimer(int tfd, int ms) {
  itimerspec its{};
  its.it_value.tv_sec = ms / 1000;
  its.it_value.tv_nsec = (ms % 1000) * 1000000L;
  timerfd_settime(tfd, 0, &its, nullptr);
}

}  // namespace

int RunDaemon(const Config& startup_cfg, std::function<Result<Config>()> reload) {
  Config cfg = startup_cfg;  // replaced on a successful reload
  auto validated = Validate(cfg);
  if (!validated.ok()) {
    LOG_ERROR(kComp, "unable to validate flags: %s", validated.status().message().c_str());
    return 1;
  }
  Validated v = std::move(*validated);
  // The relay's liveness probe runs every 30 s: no config dump, no amdsmi.
  if (cfg.flags.relay_ping) return health::PingRelay(cfg.flags.health_event_socket, 5000);
  LOG_INFO(kComp, "running with config:\n%s", cfg.ToJson().c_str());
  LOG_INFO(kComp, "running with resource config: %s", v.rc.ToJson().c_str());

  if (cfg.flags.list_grants) return ListGrants(PathJoin(cfg.flags.plugin_dir, "amdgpu-dp/usage"));

  // Signals are consumed through a signalfd; block them before any thread starts.
  sigset_t sigs;
  sigemptyset(&sigs);
  for (int s : {SIGHUP, SIGINT, SIGTERM, SIGQUIT, SIGUSR1}) sigaddset(&sigs, s);
  pthread_sigmask(SIG_BLOCK, &sigs, nullptr);
  int sfd = signalfd(-1, &sigs, SFD_CLOEXEC | SFD_NONBLOCK);

  LOG_INFO(kComp, "loading amdsmi");
  auto lib = smi::Library::Open(cfg.flags.amdsmi_lib);
  if (!lib.ok() && cfg.flags.doctor) {
    DoctorReport d;
    d.Line("FAIL", "amdsmi: " + lib.status().message() + " -- is ROCm's libamd_smi.so in the image (--amdsmi-lib)?");
    return d.Finish();
  }
  if (!lib.ok()) {
    LOG_ERROR(kComp, "failed to initialize amdsmi: %s", lib.status().message().c_str());
    LOG_ERROR(kComp, "if this is a GPU node, check that the amdgpu driver is loaded and ROCm's "
                     "libamd_smi.so is available (or pass --amdsmi-lib)");
    LOG_ERROR(kComp, "if this is not a GPU node, use a nodeSelector or toleration so the plugin "
                     "only runs on GPU nodes");
    if (cfg.flags.fail_on_init_error) return 1;
    LOG_INFO(kComp, "failOnInitError=false: blocking until terminated");
    while (true) {
      signalfd_siginfo si;
      pollfd p{sfd, POLLIN, 0};
      poll(&p, 1, -1);
      if (read(sfd, &si, sizeof(si)) == sizeof(si) && si.ssi_signo != SIGHUP && si.ssi_signo != SIGUSR1)
        return 0;
    }
  }
  LOG_INFO(kComp, "amdsmi %s loaded from %s", (*lib)->Version().c_str(), (*lib)->path().c_str());
  if (cfg.flags.dry_run) return DryRun(lib->get(), v, cfg);
  if (cfg.flags.smi_report) return SmiReport(lib->get(), v, cfg);
  if (cfg.flags.doctor) {
    DoctorReport d;
    return Doctor(lib->get(), v, cfg, d);
  }
  if (!cfg.flags.drain.empty() || !cfg.flags.undrain.empty()) return DrainCommand(lib->get(), v, cfg);
  if (cfg.flags.event_relay) return health::RunEventRelay(lib->get(), cfg.flags.health_event_socket, sfd,
                                                      {cfg.flags.driver_root, cfg.flags.host_proc,
                                                       cfg.flags.kfd_proc_dir});

  std::string kubelet_sock =
      v.popts.kubelet_socket.empty() ? PathJoin(v.popts.plugin_dir, "kubelet.sock") : v.popts.kubelet_socket;
  std::string watch_dir = kubelet_sock.substr(0, kubelet_sock.rfind('/'));
  if (watch_dir.empty()) watch_dir = "/";
  std::string kubelet_name = BaseName(kubelet_sock);
  LOG_INFO(kComp, "starting FS watcher on %s", watch_dir.c_str());
  int ifd = inotify_init1(IN_NONBLOCK | IN_CLOEXEC);
  if (ifd < 0 || inotify_add_watch(ifd, watch_dir.c_str(), IN_CREATE | IN_MOVED_TO | IN_DELETE) < 0) {
    LOG_ERROR(kComp, "failed to create FS watcher on %s: %s", watch_dir.c_str(), strerror(errno));
    return 1;
  }
  if (PathJoin(v.popts.plugin_dir, "") != PathJoin(watch_dir, ""))
    inotify_add_watch(ifd, v.popts.plugin_dir.c_str(), IN_DELETE);
  // Config file: watch its directory (editors and ConfigMap updates replace the
  // file rather than writing it in place).
  int config_wd = -1;
  std::string config_name;
  if (reload && !cfg.config_file.empty()) {
    std::string dir = cfg.config_file.substr(0, cfg.config_file.rfind('/') + 1);
    if (dir.empty()) dir = ".";
    config_name = BaseName(cfg.config_file);
    config_wd = inotify_add_watch(ifd, dir.c_str(), IN_CLOSE_WRITE | IN_MOVED_TO | IN_CREATE);
    if (config_wd < 0) LOG_WARN(kComp, "cannot watch config file %s: %s", cfg.config_file.c_str(), strerror(errno));
  }
  int tfd = timerfd_create(CLOCK_MONOTONIC, TFD_CLOEXEC | TFD_NONBLOCK);
  int efd = eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);
  int lfd = eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);  // health monitor: partition layout changed
  // One-shot: look again at plugin sockets deleted from under us (recheck_sockets).
  int rfd = timerfd_create(CLOCK_MONOTONIC, TFD_CLOEXEC | TFD_NONBLOCK);
  int ep = epoll_create1(EPOLL_CLOEXEC);
  for (int fd : {sfd, ifd, tfd, efd, lfd, rfd}) {
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.fd = fd;
    epoll_ctl(ep, EPOLL_CTL_ADD, fd, &ev);
  }
  // Plugin sockets found deleted, looked at again when rfd fires.
  std::set<std::string> recheck_sockets;
  const int kSocketRecheckMs = [] {  // test hook: widens the window (default 20 ms)
    const char* e = getenv("ADP_DEBUG_SOCKET_RECHECK_MS");
    return e && atoi(e) > 0 ? atoi(e) : 20;
  }();
  auto stand_by = [](const plugin::Plugin& pl) {
    // Another instance (a rollout with maxSurge) unlinked ours and bound the
    // path: binding it back would start a tug of war. The kubelet now talks to
    // that instance; this one stands by until the kubelet restarts or the file
    // disappears again.
    LOG_WARN(kComp, "inotify: %s now belongs to another process; '%s' stands by", pl.socket_path().c_str(),
             pl.resource_name().c_str());
  };


  std::vector<std::unique_ptr<plugin::Plugin>> plugins;
  // The metrics thread reads `plugins`; the vector is only changed under this
  // lock (plugin objects themselves are safe to read while they start/stop).
  std::mutex plugins_mu;
  std::atomic<uint64_t> restarts{0};
  std::atomic<bool> serving{false};
  std::unique_ptr<health::Monitor> monitor;
  // Health verdicts outlive every plugin generation (and, with a state file,
  // the process): a restart must not re-advertise a failed GPU as Healthy.
  health::Ledger ledger(cfg.flags.health_state_file);
  health::HealthCounters health_counters;
  int backoff_ms = 1000;
  int exit_code = 0;
  bool quit = false;
  // Re-initialise amdsmi before the next enumeration (SIGHUP, a detected
  // re-partition, or a retry): a re-partitioned GPU gets new processor handles.
  bool reinit = false;
  // The running generation's node snapshot and plugin specs: a kubelet restart
  // re-registers the same plugins without re-enumerating or restarting the
  // health monitor (whose amdsmi event wait cannot be interrupted).
  std::shared_ptr<const inventory::Snapshot> cur_snap;
  std::vector<strategy::PluginSpec> cur_specs;

  // Driver-side check of enforced HBM grants (--driver-hbm-poll-ms): started
  // with the first generation that enforces grants into an accounting dir.
  std::unique_ptr<memcap::DriverHbmMonitor> driver_hbm;
  std::mutex access_mu;  // node_access, metrics_gpus: written by restart, read by /metrics
  std::vector<inventory::NodeAccess> node_access;
  std::vector<std::pair<std::string, std::string>> metrics_gpus;  // (ledger key, bdf) of the served GPUs
  const std::string usage_dir = PathJoin(cfg.flags.plugin_dir, "amdgpu-dp/usage");  // startup-only flag
  std::unique_ptr<metrics::HttpServer> http;
  std::unique_ptr<podresources::CachedLister> pod_lister;
  if (!cfg.flags.metrics_addr.empty() && !cfg.flags.pod_resources_socket.empty())
    pod_lister = std::make_unique<podresources::CachedLister>(cfg.flags.pod_resources_socket,
                                                              std::chrono::milliseconds(2000));
  // (env only: how long the health loop may go without an iteration before /healthz fails)
  const int64_t stall_ms = [] {
    const char* e = getenv("ADP_HEALTH_STALL_MS");
    return e && atoll(e) > 0 ? static_cast<int64_t>(atoll(e)) : int64_t{60000};
  }();
  std::atomic<bool> stall_logged{false};
  if (!cfg.flags.metrics_addr.empty()) {
    std::string smi_version = (*lib)->Version();
    http = std::make_unique<metrics::HttpServer>(
        [&, smi_version] {
          std::string out =
              "# HELP amdgpu_dp_build_info Plugin and amdsmi versions.\n"
              "# TYPE amdgpu_dp_build_info gauge\n"
              "amdgpu_dp_build_info{version=\"" ADP_VERSION "\",amdsmi=\"" +
              metrics::LabelValue(smi_version) +
              "\"} 1\n"
              "# HELP amdgpu_dp_restarts_total Plugin (re)starts: kubelet restart, SIGHUP, retries.\n"
              "# TYPE amdgpu_dp_restarts_total counter\n"
              "amdgpu_dp_restarts_total " + std::to_string(restarts.load()) + "\n"
              "# HELP amdgpu_dp_health_events_enabled 1 if amdsmi event notification is registered (-1 not started).\n"
              "# TYPE amdgpu_dp_health_events_enabled gauge\n"
              "amdgpu_dp_health_events_enabled " + std::to_string(health_counters.events_enabled.load()) + "\n"
              "# HELP amdgpu_dp_health_loop_age_seconds Time since the health monitor loop last iterated (0 when "
              "none runs; /healthz fails past ADP_HEALTH_STALL_MS).\n"
              "# TYPE amdgpu_dp_health_loop_age_seconds gauge\n"
              "amdgpu_dp_health_loop_age_seconds " + std::to_string(health_counters.HealthLoopAgeMs() / 1e3) + "\n"
              "# HELP amdgpu_dp_health_polls_total Health polls (liveness + uncorrectable ECC) run.\n"
              "# TYPE amdgpu_dp_health_polls_total counter\n"
              "amdgpu_dp_health_polls_total " + std::to_string(health_counters.polls.load()) + "\n"
              "# HELP amdgpu_dp_health_ecc_reads_total Uncorrectable-ECC reads by result.\n"
              "# TYPE amdgpu_dp_health_ecc_reads_total counter\n"
              "amdgpu_dp_health_ecc_reads_total{result=\"ok\"} " + std::to_string(health_counters.ecc_reads_ok.load()) + "\n"
              "amdgpu_dp_health_ecc_reads_total{result=\"error\"} " + std::to_string(health_counters.ecc_read_errors.load()) + "\n"
              "# HELP amdgpu_dp_health_events_total amdsmi events received.\n"
              "# TYPE amdgpu_dp_health_events_total counter\n"
              "amdgpu_dp_health_events_total " + std::to_string(health_counters.events_received.load()) + "\n"
              "# HELP amdgpu_dp_health_retired_page_reads_total Retired-HBM-page reads by result.\n"
              "# TYPE amdgpu_dp_health_retired_page_reads_total counter\n"
              "amdgpu_dp_health_retired_page_reads_total{result=\"ok\"} " +
              std::to_string(health_counters.retired_reads_ok.load()) + "\n"
              "amdgpu_dp_health_retired_page_reads_total{result=\"error\"} " +
              std::to_string(health_counters.retired_read_errors.load()) + "\n";
          {
            std::lock_guard<std::mutex> lk(access_mu);
            // Why a GPU is Unhealthy, one series per failure cause (the ledger's bits).
            static const std::pair<uint32_t, const char*> kCauses[] = {
                {health::kFailEcc, "ecc"},           {health::kFailUnresponsive, "unresponsive"},
                {health::kFailResetPending, "reset_pending"}, {health::kFailEvent, "event"},
                {health::kFailRetiredPages, "retired_pages"}, {health::kFailDrained, "drained"}};
            if (!metrics_gpus.empty())
              out += "# HELP amdgpu_dp_gpu_failure 1 while the GPU is Unhealthy for this cause (drained: the "
                     "operator's drain file, not a fault).\n"
                     "# TYPE amdgpu_dp_gpu_failure gauge\n";
            for (const auto& [key, bdf] : metrics_gpus) {
              uint32_t bits = ledger.Get(key).fail;
              for (const auto& [bit, cause] : kCauses)
                out += "amdgpu_dp_gpu_failure{bdf=\"" + metrics::LabelValue(bdf) + "\",cause=\"" + cause + "\"} " +
                       ((bits & bit) ? "1" : "0") + "\n";
            }
            if (!node_access.empty())
              out += "# HELP amdgpu_dp_device_node_openable 1 if the plugin can open the device node (0: denied, "
                     "e.g. by the container's device cgroup).\n"
                     "# TYPE amdgpu_dp_device_node_openable gauge\n";
            for (const auto& a : node_access)
              out += "amdgpu_dp_device_node_openable{node=\"" + metrics::LabelValue(a.path) + "\"} " +
                     (a.err ? "0" : "1") + "\n";
          }
          if (auto events = health_counters.EventCounts(); !events.empty()) {
            out += "# HELP amdgpu_dp_gpu_events_total amdsmi events per GPU and type, ignored ones included "
                   "(VMFAULT: an application's GPU page fault; THERMAL_THROTTLE; GPU_PRE_RESET / GPU_POST_RESET).\n"
                   "# TYPE amdgpu_dp_gpu_events_total counter\n";
            for (const auto& [k, n] : events)
              out += "amdgpu_dp_gpu_events_total{bdf=\"" + metrics::LabelValue(k.first) + "\",type=\"" +
                     metrics::LabelValue(k.second) + "\"} " + std::to_string(n) + "\n";
          }
          if (auto retired = health_counters.RetiredPages(); !retired.empty()) {
            out += "# HELP amdgpu_dp_retired_pages HBM pages the driver retired (last health poll).\n"
                   "# TYPE amdgpu_dp_retired_pages gauge\n";
            for (const auto& [bdf, n] : retired)
              out += "amdgpu_dp_retired_pages{bdf=\"" + metrics::LabelValue(bdf) + "\"} " + std::to_string(n) + "\n";
          }
          if (auto total = health_counters.VramTotal(); !total.empty()) {
            out += "# HELP amdgpu_dp_gpu_hbm_total_bytes HBM of the GPU.\n"
                   "# TYPE amdgpu_dp_gpu_hbm_total_bytes gauge\n";
            for (const auto& [bdf, n] : total)
              out += "amdgpu_dp_gpu_hbm_total_bytes{bdf=\"" + metrics::LabelValue(bdf) + "\"} " + std::to_string(n) + "\n";
          }
          if (auto used = health_counters.VramUsed(); !used.empty()) {
            out += "# HELP amdgpu_dp_gpu_hbm_used_bytes HBM in use on the GPU, all processes (last health poll).\n"
                   "# TYPE amdgpu_dp_gpu_hbm_used_bytes gauge\n";
            for (const auto& [bdf, n] : used)
              out += "amdgpu_dp_gpu_hbm_used_bytes{bdf=\"" + metrics::LabelValue(bdf) + "\"} " + std::to_string(n) + "\n";
          }
          // Ask the kubelet who holds which device (cached; outside the plugins lock).
          Result<std::vector<podresources::Assignment>> assigned = Unavailable("off");
          if (pod_lister) {
            assigned = pod_lister->Get();
            out += "# HELP amdgpu_dp_pod_resources_up 1 if the kubelet PodResources API answered.\n"
                   "# TYPE amdgpu_dp_pod_resources_up gauge\n"
                   "amdgpu_dp_pod_resources_up " + std::string(assigned.ok() ? "1" : "0") + "\n";
          }
          // Grant accounting files: read (and old ones collected) here, before
          // the plugins lock the health listener also takes -- a slow
          // filesystem must not hold up health verdicts.
          std::vector<memcap::Usage> grant_files;
          bool have_grants = false;
          {
            struct stat st;
            if (stat(usage_dir.c_str(), &st) == 0 && S_ISDIR(st.st_mode)) {
              have_grants = true;
              grant_files = memcap::ReadAll(usage_dir);
              std::set<std::string> live;
              if (assigned.ok()) {
                std::map<std::tuple<std::string, std::string, std::string, std::string>,
                         std::vector<std::string_view>> ctrs;
                for (const auto& a : *assigned) ctrs[{a.ns, a.pod, a.container, a.resource}].push_back(a.device_id);
                for (const auto& [k, ids] : ctrs) live.insert(memcap::AllocationKey(ids));
              }
              memcap::Collect(usage_dir, assigned.ok() ? &live : nullptr, 120, 4096);
            }
          }
          std::unique_ptr<memcap::DriverHbmMonitor::Snapshot> dsnap;
          if (driver_hbm) {
            dsnap = std::make_unique<memcap::DriverHbmMonitor::Snapshot>(driver_hbm->Get());
            out += "# HELP amdgpu_dp_driver_hbm_polls_total Driver-side HBM scans run (DRM fdinfo of every process).\n"
                   "# TYPE amdgpu_dp_driver_hbm_polls_total counter\n"
                   "amdgpu_dp_driver_hbm_polls_total " + std::to_string(dsnap->polls) + "\n"
                   "# HELP amdgpu_dp_driver_hbm_unreadable_processes Processes whose file descriptors the plugin "
                   "may not read (their HBM is not seen).\n"
                   "# TYPE amdgpu_dp_driver_hbm_unreadable_processes gauge\n"
                   "amdgpu_dp_driver_hbm_unreadable_processes " + std::to_string(dsnap->scan.fd_dirs_unreadable) + "\n"
                   "# HELP amdgpu_dp_driver_hbm_scan_processes Processes the last driver-side scan read (the GPU "
                   "processes KFD lists, or every process without that list).\n"
                   "# TYPE amdgpu_dp_driver_hbm_scan_processes gauge\n"
                   "amdgpu_dp_driver_hbm_scan_processes{source=\"" + dsnap->scan.pid_source + "\"} " +
                   std::to_string(dsnap->scan.pids_scanned) + "\n"
                   "# HELP amdgpu_dp_driver_hbm_scan_descriptors File descriptors the last driver-side scan examined.\n"
                   "# TYPE amdgpu_dp_driver_hbm_scan_descriptors gauge\n"
                   "amdgpu_dp_driver_hbm_scan_descriptors " + std::to_string(dsnap->scan.fd_entries) + "\n"
                   "# HELP amdgpu_dp_driver_hbm_scan_seconds Wall time of the last driver-side scan.\n"
                   "# TYPE amdgpu_dp_driver_hbm_scan_seconds gauge\n"
                   "amdgpu_dp_driver_hbm_scan_seconds " + std::to_string(dsnap->last_scan_ns / 1e9) + "\n"
                   "# HELP amdgpu_dp_driver_hbm_scan_failures_total Driver-side scans the event relay could not "
                   "run (the previous scan stays in effect).\n"
                   "# TYPE amdgpu_dp_driver_hbm_scan_failures_total counter\n"
                   "amdgpu_dp_driver_hbm_scan_failures_total " + std::to_string(dsnap->scan_failures) + "\n"
                   "# HELP amdgpu_dp_hbm_over_grant_events_total Transitions of any grant to over its HBM by the "
                   "driver's count.\n"
                   "# TYPE amdgpu_dp_hbm_over_grant_events_total counter\n"
                   "amdgpu_dp_hbm_over_grant_events_total " + std::to_string(dsnap->over_total) + "\n";
            out += "# HELP amdgpu_dp_gpu_hbm_driver_bytes HBM every process holds on the GPU by the driver's count.\n"
                   "# TYPE amdgpu_dp_gpu_hbm_driver_bytes gauge\n";
            for (const auto& [bdf, n] : dsnap->scan.total)
              out += "amdgpu_dp_gpu_hbm_driver_bytes{bdf=\"" + metrics::LabelValue(bdf) + "\"} " + std::to_string(n) + "\n";
            out += "# HELP amdgpu_dp_gpu_hbm_unattributed_bytes HBM on the GPU held by processes outside every "
                   "enforced grant (no grant file mapped, no grant in their cgroup).\n"
                   "# TYPE amdgpu_dp_gpu_hbm_unattributed_bytes gauge\n";
            for (const auto& [bdf, n] : dsnap->scan.unattributed)
              out += "amdgpu_dp_gpu_hbm_unattributed_bytes{bdf=\"" + metrics::LabelValue(bdf) + "\"} " +
                     std::to_string(n) + "\n";
          }
          std::lock_guard<std::mutex> lk(plugins_mu);
          std::vector<const plugin::Plugin*> ps;
          for (auto& p : plugins)
            if (p->device_count() > 0) ps.push_back(p.get());
          plugin::Plugin::AppendPrometheus(ps, &out, assigned.ok() ? &*assigned : nullptr, dsnap.get(),
                                           have_grants ? &grant_files : nullptr);
          return out;
        },
        [&, stall_ms] {
          if (!serving.load()) return false;
          // A health loop stuck in a call that never returns (an amdsmi event
          // wait or query) stops advancing: the liveness probe restarts us.
          if (int64_t age = health_counters.HealthLoopAgeMs(); age > stall_ms) {
            if (!stall_logged.exchange(true))
              LOG_ERROR(kComp, "the health monitor has not advanced for %lld ms: /healthz fails",
                        static_cast<long long>(age));
            return false;
          }
          stall_logged.store(false);
          std::lock_guard<std::mutex> lk(plugins_mu);
          for (auto& p : plugins)
            if (p->device_count() > 0 && !p->running()) return false;
          return true;
        },
        [&] {  // GET /stats: what SIGUSR1 logs, as one JSON document
          std::string out = "{\"plugins\": [";
          {
            std::lock_guard<std::mutex> lk(plugins_mu);
            for (size_t i = 0; i < plugins.size(); ++i) out += (i ? ", " : "") + plugins[i]->StatsJson();
          }
          return out + "], \"health\": " + health_counters.Json() + ", \"restarts\": " +
                 std::to_string(restarts.load()) + "}\n";
        });
    Status ms = http->Start(cfg.flags.metrics_addr);
    if (!ms.ok()) {
      LOG_ERROR(kComp, "%s", ms.ToString().c_str());
      return 1;
    }
  }

  auto stop_all = [&] {
    serving.store(false);
    if (monitor) monitor->Stop();
    monitor.reset();
    for (auto& p : plugins) p->Stop();
    std::lock_guard<std::mutex> lk(plugins_mu);
    plugins.clear();
  };

  auto schedule_retry = [&](const char* why) {
    LOG_WARN(kComp, "%s; retrying in %d ms", why, backoff_ms);
    ArmTimer(tfd, backoff_ms);
    backoff_ms = std::min(kMaxBackoffMs, backoff_ms * 2);
  };

  // Starts (serves + registers) every plugin with devices; the number started,
  // or -1 after scheduling a retry because the kubelet could not be reached.
  auto start_plugins = [&]() -> int {
    int started = 0;
    for (auto& p : plugins) {
      if (p->device_count() == 0) continue;
      Status st = p->Start([efd] {
        uint64_t one = 1;
        ssize_t w = write(efd, &one, sizeof(one));
        (void)w;
      });
      if (!st.ok()) {
        LOG_ERROR(kComp, "could not contact kubelet, retrying (is the device-plugin feature "
                         "enabled and is %s present?)", kubelet_sock.c_str());
        schedule_retry("plugin start failed");
        return -1;
      }
      ++started;
    }
    backoff_ms = 1000;
    serving.store(true);
    return started;
  };

  // Creates this generation's plugins and applies the failures recorded by
  // earlier generations, in ONE critical section with the health listener
  // (plugins_mu): the monitor writes the ledger before it notifies, so a
  // verdict that changes concurrently is either in the ledger read here or
  // notified to the new plugins afterwards -- a GPU_POST_RESET racing a
  // re-registration can never leave a recovered GPU advertised Unhealthy.
  const int reregister_delay_ms = [] {  // test hook: widens the window the lock closes
    const char* e = getenv("ADP_DEBUG_PUBLISH_DELAY_MS");
    return e ? atoi(e) : 0;
  }();
  auto publish_plugins = [&](const std::shared_ptr<const inventory::Snapshot>& snap,
                             const std::vector<strategy::PluginSpec>& specs, bool apply_ledger) {
    std::lock_guard<std::mutex> lk(plugins_mu);
    for (const auto& s : specs) plugins.push_back(std::make_unique<plugin::Plugin>(snap, s, v.popts));
    WarnSharedDeviceLists(plugins);
    if (!apply_ledger) return;
    auto failed = ledger.Failed(*snap);
    if (reregister_delay_ms > 0) usleep(static_cast<useconds_t>(reregister_delay_ms) * 1000);
    for (const auto& [gpu, why] : failed) {
      LOG_WARN(kComp, "GPU %s is unhealthy since an earlier plugin generation: %s", snap->gpus[gpu].bdf.c_str(),
               why.c_str());
      for (auto& p : plugins) p->SetGpuHealth(gpu, false, why);
    }
  };

  auto restart = [&] {
    stop_all();
    ArmTimer(tfd, 0);  // disarm
    ArmTimer(rfd, 0);
    recheck_sockets.clear();
    if (reinit) {
      Status rs = (*lib)->Reinit();
      if (!rs.ok()) {
        LOG_ERROR(kComp, "amdsmi re-initialisation failed: %s", rs.ToString().c_str());
        schedule_retry("amdsmi re-init failed");
        return;
      }
      reinit = false;
      LOG_INFO(kComp, "amdsmi re-initialised");
    }
    LOG_INFO(kComp, "retrieving plugins");
    auto snap = inventory::BuildSnapshot(lib->get(), v.bopts);
    if (!snap.ok()) {
      LOG_ERROR(kComp, "device enumeration failed: %s", snap.status().ToString().c_str());
      reinit = true;
      schedule_retry("enumeration failed");
      return;
    }
    if (!cfg.flags.node_labels_file.empty()) WriteLabels(cfg.flags.node_labels_file, **snap);
    {
      auto access = inventory::ProbeDeviceAccess(**snap, cfg.flags.driver_root);
      std::string what = inventory::DescribeAccess(access);
      if (what == "ok") LOG_INFO(kComp, "device access: %zu node(s) openable", access.size());
      else LOG_WARN(kComp, "device access: %s", what.c_str());
      std::lock_guard<std::mutex> lk(access_mu);
      node_access = std::move(access);
      metrics_gpus.clear();
      for (const auto& g : (*snap)->gpus) metrics_gpus.emplace_back(health::Ledger::KeyOf(g), g.bdf);
    }
    auto specs = strategy::BuildPluginSpecs(**snap, v.partition, v.rc, cfg.flags.resource_prefix);
    if (!specs.ok()) {
      LOG_ERROR(kComp, "error creating partition strategy: %s", specs.status().message().c_str());
      exit_code = 1;
      quit = true;
      return;
    }
    restarts.fetch_add(1);
    cur_snap = *snap;
    cur_specs = *specs;
    for (const auto& g : cur_snap->gpus) health_counters.SetVramTotal(g.bdf, g.vram_mib << 20);
    v.popts.memcap_host_path = cfg.flags.enforce_memory_units ? InstallMemcap(cfg.flags) : "";
    v.popts.memcap_preload_list = !v.popts.memcap_host_path.empty() && cfg.flags.memcap_ld_so_preload
                                      ? InstallPreloadList(cfg.flags)
                                      : "";
    v.popts.memcap_usage_dir = !v.popts.memcap_host_path.empty() && cfg.flags.container_hbm_metrics &&
                                       !cfg.flags.metrics_addr.empty()
                                   ? PathJoin(cfg.flags.plugin_dir, "amdgpu-dp/usage")
                                   : "";
    if (!driver_hbm && !v.popts.memcap_usage_dir.empty() && cfg.flags.driver_hbm_poll_ms > 0) {
      memcap::DriverHbmMonitor::Options dopt;
      dopt.proc_root = cfg.flags.host_proc;
      dopt.kfd_proc_dir = cfg.flags.kfd_proc_dir;
      // With an event relay the scan runs there (it holds the privilege to
      // read other containers' descriptors; this daemon then needs none).
      dopt.relay_socket = cfg.flags.health_event_socket;
      dopt.usage_dir = v.popts.memcap_usage_dir;
      dopt.poll_ms = static_cast<int>(std::min<uint64_t>(cfg.flags.driver_hbm_poll_ms, 3600000));
      dopt.slack_bytes = cfg.flags.driver_hbm_slack_mib << 20;
      std::string dir = v.popts.memcap_usage_dir;
      driver_hbm = std::make_unique<memcap::DriverHbmMonitor>(dopt, [&plugins, &plugins_mu, dir] {
        // The accounting files are read before taking the lock the health
        // listener needs (as /metrics does): only ID lookups run under it.
        std::vector<memcap::Usage> files = memcap::ReadAll(dir);
        std::lock_guard<std::mutex> lk(plugins_mu);
        std::vector<const plugin::Plugin*> ps;
        for (auto& p : plugins) ps.push_back(p.get());
        return plugin::Plugin::GrantedByKey(ps, files);
      });
      driver_hbm->Start();
    }
    health::HealthConfig hcfg = health::HealthConfig::FromEnv();
    hcfg.events = cfg.flags.health_events;
    hcfg.drain_file = cfg.flags.drain_file;
    hcfg.driver_root = cfg.flags.driver_root;
    hcfg.event_relay = cfg.flags.health_event_socket;
    publish_plugins(*snap, *specs, !hcfg.disabled);
    int started = start_plugins();
    if (started < 0) return;
    if (started == 0) LOG_INFO(kComp, "no devices found; waiting indefinitely");
    monitor = std::make_unique<health::Monitor>(lib->get(), *snap, hcfg, &ledger, &health_counters);
    monitor->SetLayoutListener([lfd](const std::string&) {
      uint64_t one = 1;
      ssize_t w = write(lfd, &one, sizeof(one));
      (void)w;
    });
    // Verdicts go to whichever plugins are serving (re-registration replaces them).
    monitor->AddListener([&plugins, &plugins_mu](int gpu, bool ok, const std::string& why) {
      std::lock_guard<std::mutex> lk(plugins_mu);
      for (auto& p : plugins) p->SetGpuHealth(gpu, ok, why);
    });
    Status hs = monitor->Start();
    if (!hs.ok()) LOG_WARN(kComp, "health monitor: %s", hs.ToString().c_str());
  };

  // Kubelet restarted (or our socket vanished): same devices, same health
  // monitor; only the plugins are replaced and register again.
  auto reregister = [&] {
    if (!monitor || !cur_snap) {
      restart();
      return;
    }
    serving.store(false);
    ArmTimer(tfd, 0);
    ArmTimer(rfd, 0);
    recheck_sockets.clear();
    for (auto& p : plugins) p->Stop();
    {
      std::lock_guard<std::mutex> lk(plugins_mu);
      plugins.clear();
    }
    restarts.fetch_add(1);
    LOG_INFO(kComp, "re-registering plugins (devices and health monitor unchanged)");
    if (cfg.flags.enforce_memory_units) v.popts.memcap_host_path = InstallMemcap(cfg.flags);
    if (!v.popts.memcap_preload_list.empty()) v.popts.memcap_preload_list = InstallPreloadList(cfg.flags);
    publish_plugins(cur_snap, cur_specs, !health::HealthConfig::FromEnv().disabled);
    start_plugins();
  };

  // Re-reads flags/env/file; on success adopts the new config (startup-bound
  // settings excepted). Returns false when the new config is invalid.
  auto reload_config = [&](const char* why) -> bool {
    if (!reload) return true;
    auto next = reload();
    if (!next.ok()) {
      LOG_ERROR(kComp, "%s: config not reloaded: %s", why, next.status().message().c_str());
      return false;
    }
    for (const auto& w : next->warnings) LOG_WARN(kComp, "%s: %s", why, w.c_str());
    auto nv = Validate(*next);
    if (!nv.ok()) {
      LOG_ERROR(kComp, "%s: config not reloaded: %s", why, nv.status().message().c_str());
      return false;
    }
    const Flags& was = cfg.flags;
    const Flags& now = next->flags;
    if (now.amdsmi_lib != was.amdsmi_lib || now.metrics_addr != was.metrics_addr ||
        now.pod_resources_socket != was.pod_resources_socket || now.node_labels_file != was.node_labels_file ||
        now.plugin_dir != was.plugin_dir || now.kubelet_socket != was.kubelet_socket ||
        now.health_state_file != was.health_state_file)
      LOG_WARN(kComp, "%s: amdsmiLib, metricsAddr, podResourcesSocket, nodeLabelsFile, devicePluginPath, "
                      "kubeletSocket and healthStateFile apply at startup only", why);
    std::string old_json = cfg.ToJson();
    Config merged = *next;
    merged.flags.amdsmi_lib = was.amdsmi_lib;
    merged.flags.metrics_addr = was.metrics_addr;
    merged.flags.pod_resources_socket = was.pod_resources_socket;
    merged.flags.node_labels_file = was.node_labels_file;
    merged.flags.plugin_dir = was.plugin_dir;
    merged.flags.kubelet_socket = was.kubelet_socket;
    merged.flags.health_state_file = was.health_state_file;
    auto mv = Validate(merged);
    if (!mv.ok()) return false;
    if (merged.ToJson() != old_json) {
      cfg = std::move(merged);
      v = std::move(*mv);
      LOG_INFO(kComp, "%s: reloaded config:\n%s", why, cfg.ToJson().c_str());
      LOG_INFO(kComp, "running with resource config: %s", v.rc.ToJson().c_str());
    }
    return true;
  };

  restart();
  while (!quit) {
    epoll_event events[8];
    int n = epoll_wait(ep, events, 8, -1);
    if (n < 0) {
      if (errno == EINTR) continue;
      LOG_ERROR(kComp, "epoll_wait: %s", strerror(errno));
      exit_code = 1;
      break;
    }
    bool do_restart = false;
    bool do_reregister = false;  // a lighter restart: see reregister
    for (int i = 0; i < n && !quit; ++i) {
      int fd = events[i].data.fd;
      if (fd == tfd) {
        uint64_t exp;
        ssize_t r = read(tfd, &exp, sizeof(exp));
        (void)r;
        do_restart = true;
      } else if (fd == rfd) {
        uint64_t exp;
        ssize_t r = read(rfd, &exp, sizeof(exp));
        (void)r;
        for (auto& pl : plugins) {
          if (!recheck_sockets.count(pl->socket_path()) || !pl->running()) continue;
          struct stat st;
          if (stat(pl->socket_path().c_str(), &st) != 0) {
            LOG_WARN(kComp, "inotify: %s was removed, restarting", pl->socket_path().c_str());
            do_reregister = true;
          } else if (!pl->owns_socket()) {
            stand_by(*pl);
          }
        }
        recheck_sockets.clear();
      } else if (fd == efd) {
        uint64_t x;
        ssize_t r = read(efd, &x, sizeof(x));
        (void)r;
        LOG_ERROR(kComp, "a gRPC server exhausted its crash budget; exiting");
        exit_code = 1;
        quit = true;
      } else if (fd == lfd) {
        uint64_t x;
        ssize_t r = read(lfd, &x, sizeof(x));
        (void)r;
        LOG_INFO(kComp, "partition layout changed, re-enumerating");
        reinit = true;
        do_restart = true;
      } else if (fd == ifd) {
        char buf[4096] __attribute__((aligned(__alignof__(inotify_event))));
        ssize_t len;
        while ((len = read(ifd, buf, sizeof(buf))) > 0) {
          for (char* p = buf; p < buf + len;) {
            auto* e = reinterpret_cast<inotify_event*>(p);
            if (config_wd >= 0 && e->wd == config_wd && e->len &&
                (config_name == e->name || std::string(e->name) == "..data")) {
              LOG_INFO(kComp, "inotify: config file %s changed", cfg.config_file.c_str());
              std::string before = cfg.ToJson();
              if (reload_config("config file changed") && cfg.ToJson() != before) {
                reinit = true;
                do_restart = true;
              }
              p += sizeof(inotify_event) + e->len;
              continue;
            }
            if (e->len && kubelet_name == e->name && (e->mask & (IN_CREATE | IN_MOVED_TO))) {
              LOG_INFO(kComp, "inotify: %s created, restarting", kubelet_sock.c_str());
              backoff_ms = 1000;
              do_reregister = true;
            }
            // One of our own sockets removed from under us (not by our own Stop():
            // those are re-created before this event is read, so stat finds them).
            if (e->len && (e->mask & IN_DELETE)) {
              // The HBM-cap shim's directory wiped (a kubelet cleaning its
              // plugin directory): put it back for the next memory-unit pod.
              if (!v.popts.memcap_host_path.empty() && std::string(e->name) == "amdgpu-dp") {
                LOG_WARN(kComp, "inotify: %s was removed; reinstalling", v.popts.memcap_host_path.c_str());
                InstallMemcap(cfg.flags);
                if (!v.popts.memcap_preload_list.empty()) InstallPreloadList(cfg.flags);
                for (auto& pl : plugins)
                  if (Status gs = pl->InstallGrantFiles(); !gs.ok())
                    LOG_ERROR(kComp, "%s", gs.ToString().c_str());
              }
              for (auto& pl : plugins) {
                struct stat st;
                if (!pl->running() || BaseName(pl->socket_path()) != e->name) continue;
                if (stat(pl->socket_path().c_str(), &st) != 0) {
                  // Another instance unlinks the path and binds it microseconds
                  // later: look again after a moment (rfd) before taking it back
                  // -- without sleeping here, so signals and kubelet events
                  // are not held up meanwhile.
                  recheck_sockets.insert(pl->socket_path());
                  ArmTimer(rfd, kSocketRecheckMs);
                } else if (!pl->owns_socket()) {
                  stand_by(*pl);
                }
              }
            }
            p += sizeof(inotify_event) + e->len;
          }
        }
      } else if (fd == sfd) {
        signalfd_siginfo si;
        while (read(sfd, &si, sizeof(si)) == sizeof(si)) {
          if (si.ssi_signo == SIGHUP) {
            LOG_INFO(kComp, "received SIGHUP, restarting");
            reload_config("SIGHUP");
            // The monitor is stopped first so it cannot write the old verdicts back.
            if (monitor) monitor->Stop();
            ledger.Reload();
            reinit = true;
            do_restart = true;
          } else if (si.ssi_signo == SIGUSR1) {
            // Explicitly requested: printed whatever the log level.
            for (auto& p : plugins) Logf(LogLevel::kInfo, kComp, "stats: %s", p->StatsJson().c_str());
            Logf(LogLevel::kInfo, kComp, "health: %s", health_counters.Json().c_str());
          } else {
            LOG_INFO(kComp, "received signal %s, shutting down", strsignal(static_cast<int>(si.ssi_signo)));
            quit = true;
          }
        }
      }
    }
    if (do_restart && !quit) restart();
    else if (do_reregister && !quit) reregister();
  }
  stop_all();
  if (driver_hbm) driver_hbm->Stop();
  if (http) http->Stop();
  // Grant files of containers allocated just before the signal: the runtime mounts them next.
  if (!v.popts.memcap_usage_dir.empty() && !memcap::Flush(2000))
    LOG_WARN(kComp, "grant accounting files still being written at exit");
  // Labels describe a node this daemon is serving; do not leave them behind.
  if (!cfg.flags.node_labels_file.empty()) unlink(cfg.flags.node_labels_file.c_str());
  for (int fd : {ep, sfd, ifd, tfd, efd, lfd, rfd}) close(fd);
  LOG_INFO(kComp, "shutdown complete (exit %d)", exit_code);
  return exit_code;
}

}  // namespace adp::daemon

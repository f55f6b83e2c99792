#include "daemon/supervisor.h"

#include "daemon/daemon_metrics.h"
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

// A fault-injection delay from the environment: only in builds with
// ADP_TEST_HOOKS (the development tree); shipped binaries read nothing.
int TestHookMs(const char* name, int dflt) {
#ifdef ADP_TEST_HOOKS
  const char* e = getenv(name);
  return e && atoi(e) > 0 ? atoi(e) : dflt;
#else
  (void)name;
  return dflt;
#endif
}

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

// Atomically replaces `path` with one `key=value` line per label: the node's
// (inventory::NodeLabels) and `extra` (the served resources').
void WriteLabels(const std::string& path, const inventory::Snapshot& snap,
                 const std::vector<std::pair<std::string, std::string>>& extra) {
  std::string body;
  for (const auto& [k, v] : inventory::NodeLabels(snap)) body += k + "=" + v + "\n";
  for (const auto& [k, v] : extra) body += k + "=" + v + "\n";
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

// One daemon: the running generation (node snapshot, plugins, health
// monitor), the state that outlives generations (health ledger and counters,
// the driver-side HBM check, /metrics), and the epoll loop that restarts,
// re-registers or stops them (main.go:205-326).
class Supervisor {
 public:
  Supervisor(Config cfg, Validated v, std::function<Result<Config>()> reload, smi::Library* lib, int sfd)
      : cfg_(std::move(cfg)), v_(std::move(v)), reload_(std::move(reload)), lib_(lib), sfd_(sfd),
        ledger_(cfg_.flags.health_state_file),
        usage_dir_(PathJoin(cfg_.flags.plugin_dir, "amdgpu-dp/usage")) {
    // Where this daemon is in the event relay's stream survives the container
    // with the verdicts it goes with (health.h HealthCounters::PersistRelayCursor).
    if (!cfg_.flags.health_state_file.empty() && !cfg_.flags.health_event_socket.empty())
      health_counters_.PersistRelayCursor(cfg_.flags.health_state_file + ".relay");
  }
  ~Supervisor() {
    for (int fd : {ep_, ifd_, tfd_, efd_, lfd_, rfd_, dfd_})
      if (fd >= 0) close(fd);
  }

  int Run() {
    if (Status st = SetupWatches(); !st.ok()) {
      LOG_ERROR(kComp, "%s", st.message().c_str());
      return 1;
    }
    if (Status st = StartHttp(); !st.ok()) {
      LOG_ERROR(kComp, "%s", st.ToString().c_str());
      return 1;
    }
    Restart();
    while (!quit_) {
      epoll_event events[8];
      int n = epoll_wait(ep_, events, 8, -1);
      if (n < 0) {
        if (errno == EINTR) continue;
        LOG_ERROR(kComp, "epoll_wait: %s", strerror(errno));
        exit_code_ = 1;
        break;
      }
      bool do_restart = false;
      bool do_reregister = false;  // a lighter restart: see Reregister
      for (int i = 0; i < n && !quit_; ++i) {
        int fd = events[i].data.fd;
        uint64_t x;
        if (fd == tfd_) {
          Drain(tfd_, &x);
          do_restart = true;
        } else if (fd == rfd_) {
          Drain(rfd_, &x);
          OnSocketRecheck(&do_reregister);
        } else if (fd == dfd_) {
          Drain(dfd_, &x);
          const std::string before = cfg_.ToJson();
          if (ReloadConfig("deferred config change") && cfg_.ToJson() != before) do_restart = true;
        } else if (fd == efd_) {
          Drain(efd_, &x);
          LOG_ERROR(kComp, "a gRPC server exhausted its crash budget; exiting");
          exit_code_ = 1;
          quit_ = true;
        } else if (fd == lfd_) {
          Drain(lfd_, &x);
          LOG_INFO(kComp, "partition layout changed, re-enumerating");
          reinit_ = true;
          do_restart = true;
        } else if (fd == ifd_) {
          OnInotify(&do_restart, &do_reregister);
        } else if (fd == sfd_) {
          OnSignals(&do_restart);
        }
      }
      if (do_restart && !quit_) Restart();
      else if (do_reregister && !quit_) Reregister();
    }
    StopAll();
    if (driver_hbm_) driver_hbm_->Stop();
    if (http_) http_->Stop();
    // Grant files of containers allocated just before the signal: the runtime mounts them next.
    if (!v_.popts.memcap_usage_dir.empty() && !memcap::Flush(2000))
      LOG_WARN(kComp, "grant accounting files still being written at exit");
    // Labels describe a node this daemon is serving; do not leave them behind.
    if (!cfg_.flags.node_labels_file.empty()) unlink(cfg_.flags.node_labels_file.c_str());
    return exit_code_;
  }

 private:
  static void Drain(int fd, uint64_t* x) {
    ssize_t r = read(fd, x, sizeof(*x));
    (void)r;
  }

  // inotify on the kubelet socket's directory (and the plugin directory, and
  // the config file's), timers and eventfds, all in one epoll set.
  Status SetupWatches() {
    kubelet_sock_ = v_.popts.kubelet_socket.empty() ? PathJoin(v_.popts.plugin_dir, "kubelet.sock")
                                                    : v_.popts.kubelet_socket;
    std::string watch_dir = kubelet_sock_.substr(0, kubelet_sock_.rfind('/'));
    if (watch_dir.empty()) watch_dir = "/";
    kubelet_name_ = BaseName(kubelet_sock_);
    LOG_INFO(kComp, "starting FS watcher on %s", watch_dir.c_str());
    ifd_ = inotify_init1(IN_NONBLOCK | IN_CLOEXEC);
    if (ifd_ < 0 || inotify_add_watch(ifd_, watch_dir.c_str(), IN_CREATE | IN_MOVED_TO | IN_DELETE) < 0)
      return Internal("failed to create FS watcher on " + watch_dir + ": " + strerror(errno));
    if (PathJoin(v_.popts.plugin_dir, "") != PathJoin(watch_dir, ""))
      inotify_add_watch(ifd_, v_.popts.plugin_dir.c_str(), IN_DELETE);
    // Config file: watch its directory (editors and ConfigMap updates replace the
    // file rather than writing it in place).
    if (reload_ && !cfg_.config_file.empty()) {
      std::string dir = cfg_.config_file.substr(0, cfg_.config_file.rfind('/') + 1);
      if (dir.empty()) dir = ".";
      config_name_ = BaseName(cfg_.config_file);
      config_wd_ = inotify_add_watch(ifd_, dir.c_str(), IN_CLOSE_WRITE | IN_MOVED_TO | IN_CREATE);
      if (config_wd_ < 0)
        LOG_WARN(kComp, "cannot watch config file %s: %s", cfg_.config_file.c_str(), strerror(errno));
    }
    tfd_ = timerfd_create(CLOCK_MONOTONIC, TFD_CLOEXEC | TFD_NONBLOCK);  // retry backoff
    efd_ = eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);  // a gRPC server exhausted its crash budget
    lfd_ = eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);  // health monitor: partition layout changed
    // One-shot: look again at plugin sockets deleted from under us (recheck_sockets_).
    rfd_ = timerfd_create(CLOCK_MONOTONIC, TFD_CLOEXEC | TFD_NONBLOCK);
    // One-shot: look again at a config change deferred for live grants.
    dfd_ = timerfd_create(CLOCK_MONOTONIC, TFD_CLOEXEC | TFD_NONBLOCK);
    ep_ = epoll_create1(EPOLL_CLOEXEC);
    for (int fd : {sfd_, ifd_, tfd_, efd_, lfd_, rfd_, dfd_}) {
      epoll_event ev{};
      ev.events = EPOLLIN;
      ev.data.fd = fd;
      epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &ev);
    }
    return Status::Ok();
  }

  Status StartHttp() {
    if (cfg_.flags.metrics_addr.empty()) return Status::Ok();
    if (!cfg_.flags.pod_resources_socket.empty())
      pod_lister_ = std::make_unique<podresources::CachedLister>(cfg_.flags.pod_resources_socket,
                                                                 std::chrono::milliseconds(2000));
    smi_version_ = lib_->Version();
    // (env only: how long the health loop may go without an iteration before /healthz fails)
    if (const char* e = getenv("ADP_HEALTH_STALL_MS"); e && atoll(e) > 0) stall_ms_ = atoll(e);
    http_ = std::make_unique<metrics::HttpServer>([this] { return MetricsText(); }, [this] { return Healthy(); },
                                                  [this] { return StatsJson(); });
    return http_->Start(cfg_.flags.metrics_addr);
  }

  // GET /metrics: the daemon's families, then the plugins'.
  std::string MetricsText() {
    DaemonMetricsInput in;
    in.smi_version = smi_version_;
    in.restarts = restarts_.load();
    in.health = &health_counters_;
    {
      std::lock_guard<std::mutex> lk(access_mu_);
      in.node_access = node_access_;
      in.layout_changes_live = layout_changes_live_;
      in.deferred_layouts.assign(deferred_layouts_.begin(), deferred_layouts_.end());
      for (const auto& [key, bdf] : metrics_gpus_) {
        uint32_t fail = ledger_.Get(key).fail;
        health::GapMark m;
        bool gap = (fail & health::kFailResetPending) && ledger_.Gap(key, &m) && !m.tentative;
        in.gpus.push_back({bdf, fail, gap});
      }
    }
    // Ask the kubelet who holds which device (cached; outside the plugins lock).
    Result<std::vector<podresources::Assignment>> assigned = Unavailable("off");
    if (pod_lister_) {
      assigned = pod_lister_->Get();
      in.pod_resources_up = assigned.ok() ? 1 : 0;
    }
    // Grant accounting files: read (and old ones collected) here, before the
    // plugins lock the health listener also takes -- a slow filesystem must
    // not hold up health verdicts.
    std::vector<memcap::Usage> grant_files;
    bool have_grants = false;
    struct stat st;
    if (stat(usage_dir_.c_str(), &st) == 0 && S_ISDIR(st.st_mode)) {
      have_grants = true;
      grant_files = memcap::ReadAll(usage_dir_);
      std::set<std::string> live;
      if (assigned.ok()) {
        std::map<std::tuple<std::string, std::string, std::string, std::string>, std::vector<std::string_view>> ctrs;
        for (const auto& a : *assigned) ctrs[{a.ns, a.pod, a.container, a.resource}].push_back(a.device_id);
        for (const auto& [k, ids] : ctrs) live.insert(memcap::AllocationKey(ids));
      }
      memcap::Collect(usage_dir_, assigned.ok() ? &live : nullptr, 120, 4096);
    }
    std::unique_ptr<memcap::DriverHbmMonitor::Snapshot> dsnap;
    if (driver_hbm_) dsnap = std::make_unique<memcap::DriverHbmMonitor::Snapshot>(driver_hbm_->Get());
    in.driver_hbm = dsnap.get();
    std::string out;
    AppendDaemonMetrics(in, &out);
    std::lock_guard<std::mutex> lk(plugins_mu_);
    std::vector<const plugin::Plugin*> ps;
    for (auto& p : plugins_)
      if (p->device_count() > 0) ps.push_back(p.get());
    plugin::Plugin::AppendPrometheus(ps, &out, assigned.ok() ? &*assigned : nullptr, dsnap.get(),
                                     have_grants ? &grant_files : nullptr);
    return out;
  }

  // GET /healthz
  bool Healthy() {
    if (!serving_.load()) return false;
    // A health loop stuck in a call that never returns (an amdsmi event wait
    // or query) stops advancing: the liveness probe restarts us.
    if (int64_t age = health_counters_.HealthLoopAgeMs(); age > stall_ms_) {
      if (!stall_logged_.exchange(true))
        LOG_ERROR(kComp, "the health monitor has not advanced for %lld ms: /healthz fails", static_cast<long long>(age));
      return false;
    }
    stall_logged_.store(false);
    std::lock_guard<std::mutex> lk(plugins_mu_);
    for (auto& p : plugins_)
      if (p->device_count() > 0 && !p->running()) return false;
    return true;
  }

  // GET /stats: what SIGUSR1 logs, as one JSON document
  std::string StatsJson() {
    std::string out = "{\"plugins\": [";
    {
      std::lock_guard<std::mutex> lk(plugins_mu_);
      for (size_t i = 0; i < plugins_.size(); ++i) out += (i ? ", " : "") + plugins_[i]->StatsJson();
    }
    return out + "], \"health\": " + health_counters_.Json() + ", \"restarts\": " + std::to_string(restarts_.load()) +
           "}\n";
  }

  void StopAll() {
    serving_.store(false);
    if (monitor_) monitor_->Stop();
    monitor_.reset();
    for (auto& p : plugins_) p->Stop();
    std::lock_guard<std::mutex> lk(plugins_mu_);
    plugins_.clear();
  }

  void ScheduleRetry(const char* why) {
    LOG_WARN(kComp, "%s; retrying in %d ms", why, backoff_ms_);
    ArmTimer(tfd_, backoff_ms_);
    backoff_ms_ = std::min(kMaxBackoffMs, backoff_ms_ * 2);
  }

  // Starts (serves + registers) every plugin with devices; the number started,
  // or -1 after scheduling a retry because the kubelet could not be reached.
  int StartPlugins() {
    int started = 0;
    const int efd = efd_;
    for (auto& p : plugins_) {
      if (p->device_count() == 0) continue;
      Status st = p->Start([efd] {
        uint64_t one = 1;
        ssize_t w = write(efd, &one, sizeof(one));
        (void)w;
      });
      if (!st.ok()) {
        LOG_ERROR(kComp, "could not contact kubelet, retrying (is the device-plugin feature "
                         "enabled and is %s present?)", kubelet_sock_.c_str());
        ScheduleRetry("plugin start failed");
        return -1;
      }
      ++started;
    }
    backoff_ms_ = 1000;
    serving_.store(true);
    return started;
  }

  // Creates this generation's plugins and applies the failures recorded by
  // earlier generations, in ONE critical section with the health listener
  // (plugins_mu_): the monitor writes the ledger before it notifies, so a
  // verdict that changes concurrently is either in the ledger read here or
  // notified to the new plugins afterwards -- a GPU_POST_RESET racing a
  // re-registration can never leave a recovered GPU advertised Unhealthy.
  void PublishPlugins(const std::shared_ptr<const inventory::Snapshot>& snap,
                      const std::vector<strategy::PluginSpec>& specs, bool apply_ledger) {
    // Test hook (ADP_TEST_HOOKS builds only): widens the window the lock closes.
    static const int reregister_delay_ms = TestHookMs("ADP_DEBUG_PUBLISH_DELAY_MS", 0);
    std::lock_guard<std::mutex> lk(plugins_mu_);
    for (const auto& s : specs) plugins_.push_back(std::make_unique<plugin::Plugin>(snap, s, v_.popts));
    WarnSharedDeviceLists(plugins_);
    if (!apply_ledger) return;
    auto failed = ledger_.Failed(*snap);
    if (reregister_delay_ms > 0) usleep(static_cast<useconds_t>(reregister_delay_ms) * 1000);
    for (const auto& [gpu, why] : failed) {
      LOG_WARN(kComp, "GPU %s is unhealthy since an earlier plugin generation: %s", snap->gpus[gpu].bdf.c_str(),
               why.c_str());
      for (auto& p : plugins_) p->SetGpuHealth(gpu, false, why);
    }
  }

  // Where the HBM-cap shim, its preload list and the grant accounting files
  // go this generation (--enforce-memory-units).
  void InstallMemcapFiles() {
    const Flags& f = cfg_.flags;
    v_.popts.memcap_host_path = f.enforce_memory_units ? InstallMemcap(f) : "";
    v_.popts.memcap_preload_list =
        !v_.popts.memcap_host_path.empty() && f.memcap_ld_so_preload ? InstallPreloadList(f) : "";
    v_.popts.memcap_usage_dir =
        !v_.popts.memcap_host_path.empty() && f.container_hbm_metrics && !f.metrics_addr.empty() ? usage_dir_ : "";
  }

  // Driver-side check of enforced HBM grants (--driver-hbm-poll-ms): started
  // with the first generation that enforces grants into an accounting dir.
  void StartDriverHbm() {
    if (driver_hbm_ || v_.popts.memcap_usage_dir.empty() || cfg_.flags.driver_hbm_poll_ms == 0) return;
    memcap::DriverHbmMonitor::Options dopt;
    dopt.proc_root = cfg_.flags.host_proc;
    dopt.kfd_proc_dir = cfg_.flags.kfd_proc_dir;
    // With an event relay the scan runs there (it holds the privilege to
    // read other containers' descriptors; this daemon then needs none).
    dopt.relay_socket = cfg_.flags.health_event_socket;
    dopt.usage_dir = v_.popts.memcap_usage_dir;
    dopt.poll_ms = static_cast<int>(std::min<uint64_t>(cfg_.flags.driver_hbm_poll_ms, 3600000));
    dopt.slack_bytes = cfg_.flags.driver_hbm_slack_mib << 20;
    std::string dir = v_.popts.memcap_usage_dir;
    driver_hbm_ = std::make_unique<memcap::DriverHbmMonitor>(dopt, [this, dir] {
      // The accounting files are read before taking the lock the health
      // listener needs (as /metrics does): only ID lookups run under it.
      std::vector<memcap::Usage> files = memcap::ReadAll(dir);
      std::lock_guard<std::mutex> lk(plugins_mu_);
      std::vector<const plugin::Plugin*> ps;
      for (auto& p : plugins_) ps.push_back(p.get());
      return plugin::Plugin::GrantedByKey(ps, files);
    });
    driver_hbm_->Start();
  }

  health::HealthConfig HealthConfigNow() const {
    health::HealthConfig h = health::HealthConfig::FromEnv();
    h.events = cfg_.flags.health_events;
    h.drain_file = cfg_.flags.drain_file;
    h.driver_root = cfg_.flags.driver_root;
    h.event_relay = cfg_.flags.health_event_socket;
    h.extra_types = v_.extra_event_types;
    h.reset_recovery_hold_ms = static_cast<int64_t>(std::min<uint64_t>(cfg_.flags.reset_recovery_hold_ms, 86400000));
    h.reset_flap_limit = static_cast<int>(std::min<uint64_t>(cfg_.flags.reset_flap_limit, 1000));
    h.reset_flap_window_ms = static_cast<int64_t>(std::min<uint64_t>(cfg_.flags.reset_flap_window_ms, 86400000));
    return h;
  }

  void StartMonitor(const std::shared_ptr<const inventory::Snapshot>& snap, const health::HealthConfig& hcfg) {
    monitor_ = std::make_unique<health::Monitor>(lib_, snap, hcfg, &ledger_, &health_counters_);
    const int lfd = lfd_;
    monitor_->SetLayoutListener([lfd](const std::string&) {
      uint64_t one = 1;
      ssize_t w = write(lfd, &one, sizeof(one));
      (void)w;
    });
    // Verdicts go to whichever plugins are serving (re-registration replaces them).
    monitor_->AddListener([this](int gpu, bool ok, const std::string& why) {
      std::lock_guard<std::mutex> lk(plugins_mu_);
      for (auto& p : plugins_) p->SetGpuHealth(gpu, ok, why);
    });
    Status hs = monitor_->Start();
    if (!hs.ok()) LOG_WARN(kComp, "health monitor: %s", hs.ToString().c_str());
  }

  // A new generation: re-enumerate (after amdsmi re-init when asked), rebuild
  // the plugins from the strategy, start them and a new health monitor.
  void Restart() {
    StopAll();
    if (standby_) {
      // Back from standing by: the instance that served meanwhile wrote the
      // verdicts; start from its file.
      standby_ = false;
      ledger_.Reload();
    }
    ArmTimer(tfd_, 0);  // disarm
    ArmTimer(rfd_, 0);
    recheck_sockets_.clear();
    if (reinit_) {
      Status rs = lib_->Reinit();
      if (!rs.ok()) {
        LOG_ERROR(kComp, "amdsmi re-initialisation failed: %s", rs.ToString().c_str());
        ScheduleRetry("amdsmi re-init failed");
        return;
      }
      reinit_ = false;
      LOG_INFO(kComp, "amdsmi re-initialised");
    }
    LOG_INFO(kComp, "retrieving plugins");
    auto snap = inventory::BuildSnapshot(lib_, v_.bopts);
    if (!snap.ok()) {
      LOG_ERROR(kComp, "device enumeration failed: %s", snap.status().ToString().c_str());
      reinit_ = true;
      ScheduleRetry("enumeration failed");
      return;
    }
    {
      auto access = inventory::ProbeDeviceAccess(**snap, cfg_.flags.driver_root);
      std::string what = inventory::DescribeAccess(access);
      if (what == "ok") LOG_INFO(kComp, "device access: %zu node(s) openable", access.size());
      else LOG_WARN(kComp, "device access: %s", what.c_str());
      std::lock_guard<std::mutex> lk(access_mu_);
      node_access_ = std::move(access);
      metrics_gpus_.clear();
      for (const auto& g : (*snap)->gpus) metrics_gpus_.emplace_back(health::Ledger::KeyOf(g), g.bdf);
    }
    auto specs = strategy::BuildPluginSpecs(**snap, v_.partition, v_.rc, cfg_.flags.resource_prefix);
    if (!specs.ok()) {
      LOG_ERROR(kComp, "error creating partition strategy: %s", specs.status().message().c_str());
      exit_code_ = 1;
      quit_ = true;
      return;
    }
    restarts_.fetch_add(1);
    cur_snap_ = *snap;
    cur_specs_ = *specs;
    for (const auto& g : cur_snap_->gpus) health_counters_.SetVramTotal(g.bdf, g.vram_mib << 20);
    InstallMemcapFiles();
    StartDriverHbm();
    health::HealthConfig hcfg = HealthConfigNow();
    PublishPlugins(*snap, *specs, !hcfg.disabled);
    if (!cfg_.flags.node_labels_file.empty()) WriteLabels(cfg_.flags.node_labels_file, **snap, ResourceLabels());
    CheckReplicaLayouts();
    int started = StartPlugins();
    if (started < 0) return;
    if (started == 0) LOG_INFO(kComp, "no devices found; waiting indefinitely");
    StartMonitor(*snap, hcfg);
  }

  // Per memory-unit resource: what one unit is, where pod authors (and
  // schedulers) can read it -- amd.com/<resource>.memory-unit-mib and
  // .memory-unit (cu-slot or mib).
  std::vector<std::pair<std::string, std::string>> ResourceLabels() {
    std::vector<std::pair<std::string, std::string>> out;
    std::lock_guard<std::mutex> lk(plugins_mu_);
    for (const auto& p : plugins_) {
      if (!p->memory_units() || p->device_count() == 0) continue;
      const std::string key = p->resource_name();  // "<prefix>/<name>"
      out.emplace_back(key + ".memory-unit", p->memory_unit_kind());
      if (p->memory_unit_mib()) out.emplace_back(key + ".memory-unit-mib", std::to_string(p->memory_unit_mib()));
      else out.emplace_back(key + ".memory-unit-mib", "mixed");
    }
    return out;
  }

  // What each replicated resource's IDs mean (Plugin::ReplicaLayout), kept
  // across generations and -- in <plugin dir>/amdgpu-dp/replica-layout --
  // across processes. A resource whose layout changes (autoReplicaUnit,
  // replicaCuMask, a resourceConfig replica count, a re-partition) while the
  // kubelet says running containers hold its IDs: those IDs now mean other
  // devices or other amounts of HBM than the containers were given, and the
  // node can be over-committed until they end. Logged as an error and counted.
  void CheckReplicaLayouts() {
    std::map<std::string, std::string> now;
    {
      std::lock_guard<std::mutex> lk(plugins_mu_);
      for (const auto& p : plugins_)
        if (p->device_count() > 0) now[p->resource_name()] = p->ReplicaLayout();
    }
    const std::string path = PathJoin(cfg_.flags.plugin_dir, "amdgpu-dp/replica-layout");
    if (!layouts_loaded_) {
      layouts_loaded_ = true;
      if (FILE* f = fopen(path.c_str(), "r")) {
        char line[8192];
        while (fgets(line, sizeof(line), f)) {
          std::string l(line);
          while (!l.empty() && l.back() == '\n') l.pop_back();
          size_t tab = l.find('\t');
          if (tab != std::string::npos) layouts_[l.substr(0, tab)] = l.substr(tab + 1);
        }
        fclose(f);
      }
    }
    std::vector<std::string> changed;
    for (const auto& [res, before] : layouts_) {
      auto it = now.find(res);
      if (it != now.end() && it->second != before) changed.push_back(res);
    }
    // A resource absent this time (no device left, a config without it) keeps
    // its last layout: if it comes back changed, that is still a change.
    for (const auto& [res, lay] : now) layouts_[res] = lay;
    std::string body;
    for (const auto& [res, lay] : layouts_) body += res + "\t" + lay + "\n";
    if (body != layouts_written_) WriteLayoutFile(path, body);  // (each restart would rewrite it otherwise)
    if (changed.empty()) return;

    Result<std::vector<podresources::Assignment>> live = Unavailable("no --pod-resources-socket");
    if (!cfg_.flags.pod_resources_socket.empty()) live = podresources::List(cfg_.flags.pod_resources_socket, 1000);
    for (const auto& res : changed) {
      const std::string& after = now[res];
      if (!live.ok()) {
        LOG_WARN(kComp, "'%s': what its IDs mean changed (now: %s); whether running containers hold some is unknown "
                 "(kubelet PodResources: %s)", res.c_str(), after.c_str(), live.status().ToString().c_str());
        continue;
      }
      size_t held = 0, pods = 0;
      std::set<std::string> seen;
      for (const auto& a : *live)
        if (a.resource == res) {
          ++held;
          if (seen.insert(a.ns + "/" + a.pod).second) ++pods;
        }
      if (held == 0) {
        LOG_INFO(kComp, "'%s': what its IDs mean changed (now: %s); no running container holds any", res.c_str(),
                 after.c_str());
        continue;
      }
      {
        std::lock_guard<std::mutex> lk(access_mu_);
        ++layout_changes_live_[res];
      }
      LOG_ERROR(kComp, "'%s': what its IDs mean changed while %zu of them are held by %zu running pod(s) (now: %s): "
                "those pods keep what they were given, new pods are granted by the new layout, and the node can be "
                "over-committed until the old pods end. Drain the node before changing autoReplicaUnit, "
                "replicaCuMask or a resourceConfig replica count (amdgpu_dp_stale_allocated_ids counts their IDs "
                "that no longer exist)", res.c_str(), held, pods, after.c_str());
    }
  }

  void WriteLayoutFile(const std::string& path, const std::string& body) {
    mkdir(PathJoin(cfg_.flags.plugin_dir, "amdgpu-dp").c_str(), 0755);
    std::string tmp = path + ".tmp";
    FILE* f = fopen(tmp.c_str(), "w");
    bool ok = f && fwrite(body.data(), 1, body.size(), f) == body.size();
    if (f) ok = (fclose(f) == 0) && ok;
    if (!ok || rename(tmp.c_str(), path.c_str()) != 0) {
      unlink(tmp.c_str());
      return;
    }
    layouts_written_ = body;
  }

  // Kubelet restarted (or our socket vanished): same devices, same health
  // monitor; only the plugins are replaced and register again.
  void Reregister() {
    if (!monitor_ || !cur_snap_) {
      Restart();
      return;
    }
    serving_.store(false);
    ArmTimer(tfd_, 0);
    ArmTimer(rfd_, 0);
    recheck_sockets_.clear();
    for (auto& p : plugins_) p->Stop();
    {
      std::lock_guard<std::mutex> lk(plugins_mu_);
      plugins_.clear();
    }
    restarts_.fetch_add(1);
    LOG_INFO(kComp, "re-registering plugins (devices and health monitor unchanged)");
    if (cfg_.flags.enforce_memory_units) v_.popts.memcap_host_path = InstallMemcap(cfg_.flags);
    if (!v_.popts.memcap_preload_list.empty()) v_.popts.memcap_preload_list = InstallPreloadList(cfg_.flags);
    PublishPlugins(cur_snap_, cur_specs_, !health::HealthConfig::FromEnv().disabled);
    StartPlugins();
  }

  // Re-reads flags/env/file; on success adopts the new config (startup-bound
  // settings excepted). Returns false when the new config is invalid.
  bool ReloadConfig(const char* why) {
    if (!reload_) return true;
    auto next = reload_();
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
    const Flags& was = cfg_.flags;
    const Flags& now = next->flags;
    if (now.amdsmi_lib != was.amdsmi_lib || now.metrics_addr != was.metrics_addr ||
        now.pod_resources_socket != was.pod_resources_socket || now.node_labels_file != was.node_labels_file ||
        now.plugin_dir != was.plugin_dir || now.kubelet_socket != was.kubelet_socket ||
        now.health_state_file != was.health_state_file)
      LOG_WARN(kComp, "%s: amdsmiLib, metricsAddr, podResourcesSocket, nodeLabelsFile, devicePluginPath, "
                      "kubeletSocket and healthStateFile apply at startup only", why);
    std::string old_json = cfg_.ToJson();
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
    if (merged.ToJson() == old_json) {
      ForgetDeferral();  // (an edit undone while deferred)
      return true;
    }
    if (merged.flags.defer_layout_changes && DeferLayoutChange(merged, *mv, why)) return false;
    ForgetDeferral();
    {
      cfg_ = std::move(merged);
      v_ = std::move(*mv);
      LOG_INFO(kComp, "%s: reloaded config:\n%s", why, cfg_.ToJson().c_str());
      LOG_INFO(kComp, "running with resource config: %s", v_.rc.ToJson().c_str());
    }
    return true;
  }

  void ForgetDeferral() {
    ArmTimer(dfd_, 0);
    std::lock_guard<std::mutex> lk(access_mu_);
    deferred_layouts_.clear();
  }

  // --defer-layout-changes: true (and the timer armed) when `next` would change
  // what a resource's IDs mean while running pods hold some of them. The
  // layouts are those of plugins built from the current devices, not started.
  bool DeferLayoutChange(const Config& next, const Validated& nv, const char* why) {
    static const int recheck_ms = [] {  // test hook (default: every 30 s)
      const char* e = getenv("ADP_DEFER_RECHECK_MS");
      return e && atoi(e) > 0 ? atoi(e) : 30000;
    }();
    if (!cur_snap_) return false;
    auto specs = strategy::BuildPluginSpecs(*cur_snap_, nv.partition, nv.rc, next.flags.resource_prefix);
    if (!specs.ok()) return false;  // the restart says why
    plugin::PluginOptions po = nv.popts;
    po.quiet = true;
    std::map<std::string, std::string> after, now;
    for (const auto& sp : *specs) {
      plugin::Plugin p(cur_snap_, sp, po);
      if (p.device_count() > 0) after[p.resource_name()] = p.ReplicaLayout();
    }
    {
      std::lock_guard<std::mutex> lk(plugins_mu_);
      for (const auto& p : plugins_)
        if (p->device_count() > 0) now[p->resource_name()] = p->ReplicaLayout();
    }
    // IDs that would mean something else, or vanish -- as CheckReplicaLayouts
    // counts it: a whole-GPU resource ("" layout) turned into replicas or
    // memory units re-means the exclusive IDs running pods hold just as well.
    std::set<std::string> changed;
    for (const auto& [res, lay] : now) {
      auto it = after.find(res);
      if (it == after.end() || it->second != lay) changed.insert(res);
    }
    if (changed.empty()) return false;
    if (cfg_.flags.pod_resources_socket.empty()) {
      LOG_WARN(kComp, "%s: --defer-layout-changes needs the kubelet's PodResources socket; applying", why);
      return false;
    }
    auto live = podresources::List(cfg_.flags.pod_resources_socket, 1000);
    if (!live.ok()) {
      LOG_WARN(kComp, "%s: whether running pods hold IDs of the resources this change re-means is unknown (%s); "
               "applying", why, live.status().ToString().c_str());
      return false;
    }
    std::set<std::string> held;
    for (const auto& a : *live)
      if (changed.count(a.resource)) held.insert(a.resource);
    if (held.empty()) return false;
    std::string names;
    for (const auto& r : held) names += (names.empty() ? "'" : ", '") + r + "'";
    bool first;
    {
      std::lock_guard<std::mutex> lk(access_mu_);
      first = deferred_layouts_ != held;
      deferred_layouts_ = held;
    }
    if (first)
      LOG_WARN(kComp, "%s: config change deferred: running pods hold IDs of %s, which it would re-mean; the "
               "current layout is served until they end (looked at every %d s; --defer-layout-changes)", why,
               names.c_str(), recheck_ms / 1000);
    ArmTimer(dfd_, recheck_ms);
    return true;
  }

  void StandBy(const plugin::Plugin& pl) {
    // Another instance (a rollout with maxSurge) unlinked ours and bound the
    // path: binding it back would start a tug of war. The kubelet now talks to
    // that instance; this one stands by until the kubelet restarts or the file
    // disappears again.
    LOG_WARN(kComp, "inotify: %s now belongs to another process; '%s' stands by", pl.socket_path().c_str(),
             pl.resource_name().c_str());
    // No plugin of this instance serves any more: its health monitor pauses.
    // The serving instance owns the verdicts now -- the state file both would
    // write, the operator's return-to-service requests both would take.
    for (const auto& p : plugins_)
      if (p->running() && p->owns_socket()) return;
    if (monitor_) {
      monitor_->Stop();  // (its last poll may still be running: the log line follows it)
      monitor_.reset();
      standby_ = true;
      LOG_WARN(kComp, "no plugin of this instance serves: its health monitor pauses (the serving instance keeps "
               "the health verdicts)");
    }
  }

  void OnSocketRecheck(bool* do_reregister) {
    for (auto& pl : plugins_) {
      if (!recheck_sockets_.count(pl->socket_path()) || !pl->running()) continue;
      struct stat st;
      if (stat(pl->socket_path().c_str(), &st) != 0) {
        LOG_WARN(kComp, "inotify: %s was removed, restarting", pl->socket_path().c_str());
        *do_reregister = true;
      } else if (!pl->owns_socket()) {
        StandBy(*pl);
      }
    }
    recheck_sockets_.clear();
  }

  void OnInotify(bool* do_restart, bool* do_reregister) {
    // Test hook (ADP_TEST_HOOKS builds only): widens the window (default 20 ms).
    static const int kSocketRecheckMs = TestHookMs("ADP_DEBUG_SOCKET_RECHECK_MS", 20);
    char buf[4096] __attribute__((aligned(__alignof__(inotify_event))));
    ssize_t len;
    while ((len = read(ifd_, buf, sizeof(buf))) > 0) {
      for (char* p = buf; p < buf + len;) {
        auto* e = reinterpret_cast<inotify_event*>(p);
        p += sizeof(inotify_event) + e->len;
        if (config_wd_ >= 0 && e->wd == config_wd_ && e->len &&
            (config_name_ == e->name || std::string(e->name) == "..data")) {
          LOG_INFO(kComp, "inotify: config file %s changed", cfg_.config_file.c_str());
          std::string before = cfg_.ToJson();
          if (ReloadConfig("config file changed") && cfg_.ToJson() != before) {
            reinit_ = true;
            *do_restart = true;
          }
          continue;
        }
        if (e->len && kubelet_name_ == e->name && (e->mask & (IN_CREATE | IN_MOVED_TO))) {
          LOG_INFO(kComp, "inotify: %s created, restarting", kubelet_sock_.c_str());
          backoff_ms_ = 1000;
          *do_reregister = true;
        }
        // One of our own sockets removed from under us (not by our own Stop():
        // those are re-created before this event is read, so stat finds them).
        if (!e->len || !(e->mask & IN_DELETE)) continue;
        // (the replica-layout file went with it: written again at the next restart)
        if (std::string(e->name) == "amdgpu-dp") layouts_written_.clear();
        // The HBM-cap shim's directory wiped (a kubelet cleaning its plugin
        // directory): put it back for the next memory-unit pod.
        if (!v_.popts.memcap_host_path.empty() && std::string(e->name) == "amdgpu-dp") {
          LOG_WARN(kComp, "inotify: %s was removed; reinstalling", v_.popts.memcap_host_path.c_str());
          InstallMemcap(cfg_.flags);
          if (!v_.popts.memcap_preload_list.empty()) InstallPreloadList(cfg_.flags);
          for (auto& pl : plugins_)
            if (Status gs = pl->InstallGrantFiles(); !gs.ok()) LOG_ERROR(kComp, "%s", gs.ToString().c_str());
        }
        for (auto& pl : plugins_) {
          struct stat st;
          if (!pl->running() || BaseName(pl->socket_path()) != e->name) continue;
          if (stat(pl->socket_path().c_str(), &st) != 0) {
            // Another instance unlinks the path and binds it microseconds
            // later: look again after a moment (rfd_) before taking it back
            // -- without sleeping here, so signals and kubelet events are
            // not held up meanwhile.
            recheck_sockets_.insert(pl->socket_path());
            ArmTimer(rfd_, kSocketRecheckMs);
          } else if (!pl->owns_socket()) {
            StandBy(*pl);
          }
        }
      }
    }
  }

  void OnSignals(bool* do_restart) {
    signalfd_siginfo si;
    while (read(sfd_, &si, sizeof(si)) == sizeof(si)) {
      if (si.ssi_signo == SIGHUP) {
        LOG_INFO(kComp, "received SIGHUP, restarting");
        ReloadConfig("SIGHUP");
        // The monitor is stopped first so it cannot write the old verdicts back.
        if (monitor_) monitor_->Stop();
        ledger_.Reload();
        reinit_ = true;
        *do_restart = true;
      } else if (si.ssi_signo == SIGUSR1) {
        // Explicitly requested: printed whatever the log level.
        for (auto& p : plugins_) Logf(LogLevel::kInfo, kComp, "stats: %s", p->StatsJson().c_str());
        Logf(LogLevel::kInfo, kComp, "health: %s", health_counters_.Json().c_str());
      } else {
        LOG_INFO(kComp, "received signal %s, shutting down", strsignal(static_cast<int>(si.ssi_signo)));
        quit_ = true;
      }
    }
  }

  Config cfg_;  // replaced on a successful reload
  Validated v_;
  std::function<Result<Config>()> reload_;
  smi::Library* lib_;
  const int sfd_;
  int ep_ = -1, ifd_ = -1, tfd_ = -1, efd_ = -1, lfd_ = -1, rfd_ = -1;
  std::string kubelet_sock_, kubelet_name_;
  int config_wd_ = -1;
  std::string config_name_;
  // Plugin sockets found deleted, looked at again when rfd_ fires.
  std::set<std::string> recheck_sockets_;

  std::vector<std::unique_ptr<plugin::Plugin>> plugins_;
  // The metrics thread reads plugins_; the vector is only changed under this
  // lock (plugin objects themselves are safe to read while they start/stop).
  std::mutex plugins_mu_;
  std::atomic<uint64_t> restarts_{0};
  std::atomic<bool> serving_{false};
  std::unique_ptr<health::Monitor> monitor_;
  bool standby_ = false;  // another instance took every socket: the monitor is paused
  // Health verdicts outlive every plugin generation (and, with a state file,
  // the process): a restart must not re-advertise a failed GPU as Healthy.
  health::Ledger ledger_;
  health::HealthCounters health_counters_;
  int backoff_ms_ = 1000;
  int exit_code_ = 0;
  bool quit_ = false;
  // Re-initialise amdsmi before the next enumeration (SIGHUP, a detected
  // re-partition, or a retry): a re-partitioned GPU gets new processor handles.
  bool reinit_ = false;
  // The running generation's node snapshot and plugin specs: a kubelet restart
  // re-registers the same plugins without re-enumerating or restarting the
  // health monitor (whose amdsmi event wait cannot be interrupted).
  std::shared_ptr<const inventory::Snapshot> cur_snap_;
  std::vector<strategy::PluginSpec> cur_specs_;
  std::unique_ptr<memcap::DriverHbmMonitor> driver_hbm_;
  std::mutex access_mu_;  // node_access_, metrics_gpus_: written by Restart, read by /metrics
  std::vector<inventory::NodeAccess> node_access_;
  std::vector<std::pair<std::string, std::string>> metrics_gpus_;  // (ledger key, bdf) of the served GPUs
  std::map<std::string, uint64_t> layout_changes_live_;  // per resource (CheckReplicaLayouts)
  // --defer-layout-changes: resources whose layout change waits for the pods
  // holding their IDs (under access_mu_), and the timer that looks again.
  std::set<std::string> deferred_layouts_;
  int dfd_ = -1;
  std::map<std::string, std::string> layouts_;  // resource -> Plugin::ReplicaLayout of the running generation
  bool layouts_loaded_ = false;
  std::string layouts_written_;  // the replica-layout file's body as last written
  const std::string usage_dir_;  // grant accounting files (the plugin directory is a startup-only flag)
  std::string smi_version_;
  std::unique_ptr<metrics::HttpServer> http_;
  std::unique_ptr<podresources::CachedLister> pod_lister_;
  int64_t stall_ms_ = 60000;
  std::atomic<bool> stall_logged_{false};
};

}  // namespace

int RunDaemon(const Config& startup_cfg, std::function<Result<Config>()> reload) {
  auto validated = Validate(startup_cfg);
  if (!validated.ok()) {
    LOG_ERROR(kComp, "unable to validate flags: %s", validated.status().message().c_str());
    return 1;
  }
  Validated v = std::move(*validated);
  const Config& cfg = startup_cfg;
  // The relay's liveness probe runs every 30 s: no config dump, no amdsmi.
  if (cfg.flags.relay_ping) return health::PingRelay(cfg.flags.health_event_socket, 5000);
  // An operator's command (kubectl exec): its printed answer, not the startup log.
  const bool operator_command =
      !cfg.flags.drain.empty() || !cfg.flags.undrain.empty() || !cfg.flags.return_to_service.empty();
  if (operator_command && !getenv("ADP_LOG_LEVEL")) SetLogLevel(LogLevel::kWarn);
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
      if (read(sfd, &si, sizeof(si)) == sizeof(si) && si.ssi_signo != SIGHUP && si.ssi_signo != SIGUSR1) return 0;
    }
  }
  LOG_INFO(kComp, "amdsmi %s loaded from %s", (*lib)->Version().c_str(), (*lib)->path().c_str());
  if (cfg.flags.dry_run) return DryRun(lib->get(), v, cfg);
  if (cfg.flags.smi_report) return SmiReport(lib->get(), v, cfg);
  if (cfg.flags.doctor) {
    DoctorReport d;
    return Doctor(lib->get(), v, cfg, d);
  }
  if (operator_command) return DrainCommand(lib->get(), v, cfg);
  if (cfg.flags.event_relay) {
    health::RelayOptions ro{cfg.flags.driver_root, cfg.flags.host_proc, cfg.flags.kfd_proc_dir};
    for (uint32_t t : v.extra_event_types) ro.extra_mask |= smi::EventMask(t);
    return health::RunEventRelay(lib->get(), cfg.flags.health_event_socket, sfd, ro);
  }
  int rc;
  {
    Supervisor s(cfg, std::move(v), std::move(reload), lib->get(), sfd);
    rc = s.Run();
  }
  close(sfd);
  LOG_INFO(kComp, "shutdown complete (exit %d)", rc);
  return rc;
}

}  // namespace adp::daemon

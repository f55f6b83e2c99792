#include "health/health.h"

#include <fcntl.h>
#include <poll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <optional>
#include <set>

#include "common/log.h"
#include "common/strings.h"
#include "health/relay.h"

namespace adp::health {
namespace {
constexpr const char* kComp = "health";
// Housekeeping period when liveness polls are off (DP_HEALTH_POLL_MS=0).
constexpr int kHousekeepingMs = 1000;
}  // namespace

int64_t Clock::SteadyMs() const {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// For what is persisted (the reset history): a steady clock restarts with the node.
int64_t Clock::WallMs() const {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}

const Clock* Clock::System() {
  static const Clock c;
  return &c;
}

std::string DescribeFailures(uint32_t bits) {
  static const std::pair<uint32_t, const char*> kNames[] = {
      {kFailResetPending, "waiting for GPU_POST_RESET"}, {kFailFlapping, "resetting too often"},
      {kFailEcc, "uncorrectable ECC errors"},            {kFailRetiredPages, "retired HBM pages"},
      {kFailUnresponsive, "not responding"},             {kFailEvent, "an amdsmi event"},
      {kFailDrained, "drained by the operator"}};
  std::string out;
  for (const auto& [bit, name] : kNames)
    if (bits & bit) out += (out.empty() ? "" : ", ") + std::string(name);
  return out;
}

std::vector<uint64_t> ParseAdditionalIds(std::string_view input) {
  std::vector<uint64_t> out;
  if (input.empty()) return out;
  for (const auto& part : Split(input, ',')) {
    std::string t = Trim(part);
    if (t.empty()) continue;
    auto v = ParseUint(t);
    if (!v) {
      LOG_DEBUG(kComp, "ignoring malformed event ID value %s", t.c_str());
      continue;
    }
    out.push_back(*v);
  }
  return out;
}

Result<std::set<uint32_t>> ParseEventTypes(std::string_view input) {
  std::set<uint32_t> out;
  for (const auto& part : Split(input, ',')) {
    std::string t = Trim(part);
    if (t.empty()) continue;
    std::optional<uint64_t> v = ParseUint(t);
    if (!v) {
      std::string up = t;
      for (auto& c : up) c = static_cast<char>(toupper(static_cast<unsigned char>(c)));
      if (up.rfind("AMDSMI_EVT_NOTIF_", 0) == 0) up = up.substr(17);
      for (uint32_t i = 1; i <= smi::kEvtLast && !v; ++i)
        if (smi::EventTypeName(i) == up) v = i;
    }
    if (!v || *v < 1 || *v > smi::kEvtLast)
      return InvalidArgument("unknown amdsmi event type '" + t + "' (1.." + std::to_string(smi::kEvtLast) +
                             " or a name such as PROCESS_START)");
    out.insert(static_cast<uint32_t>(*v));
  }
  return out;
}

uint64_t HealthConfig::EventMask() const {
  uint64_t mask = smi::EventMask(smi::kEvtGpuPreReset) | smi::EventMask(smi::kEvtGpuPostReset) |
                  smi::EventMask(smi::kEvtVmFault) | smi::EventMask(smi::kEvtThermalThrottle);
  for (uint32_t t : extra_types) mask |= smi::EventMask(t);
  return mask;
}

HealthConfig HealthConfig::FromValues(const char* disable_value, const char* poll_ms_value) {
  HealthConfig c;
  std::string v = ToLower(disable_value ? disable_value : "");
  if (v == "all") v = "xids";
  if (v.find("xids") != std::string::npos || v.find("events") != std::string::npos) {
    c.disabled = true;
    return c;
  }
  for (uint64_t id : ParseAdditionalIds(v)) c.ignored.insert(static_cast<uint32_t>(id));
  if (poll_ms_value && *poll_ms_value) {
    auto p = ParseInt(poll_ms_value);
    if (p && *p >= 0) c.poll_interval_ms = static_cast<int>(*p);
  }
  return c;
}

HealthConfig HealthConfig::FromEnv() {
  HealthConfig c = FromValues(std::getenv("DP_DISABLE_HEALTHCHECKS"), std::getenv("DP_HEALTH_POLL_MS"));
  if (const char* v = std::getenv("DP_MAX_RETIRED_PAGES"); v && *v) {
    auto n = ParseInt(v);
    if (n && *n >= -1) c.max_retired_pages = *n;
    else LOG_WARN(kComp, "ignoring DP_MAX_RETIRED_PAGES=%s (want -1, 0 or a page count)", v);
  }
  if (const char* v = std::getenv("ADP_EVENT_FAIL_MS"); v && *v) {
    auto n = ParseInt(v);
    if (n && *n > 0 && *n < 86400000) c.event_fail_ms = static_cast<int>(*n);
  }
  return c;
}

int Monitor::Classify(const HealthConfig& cfg, uint32_t type) {
  if (cfg.ignored.count(type)) return 0;
  if (type == smi::kEvtGpuPostReset) return +1;
  if (type >= smi::kEvtVmFault && type <= smi::kEvtGpuPreReset) return -1;
  // KFD's informational events (5..13: migration, page faults, queue
  // eviction, process start/end), registered only by --health-event-extra-types:
  // counted, never a verdict.
  return 0;
}

Monitor::Monitor(smi::Library* lib, std::shared_ptr<const inventory::Snapshot> snap, HealthConfig cfg,
                 Ledger* ledger, HealthCounters* counters)
    : lib_(lib), snap_(std::move(snap)), cfg_(std::move(cfg)), ledger_(ledger ? ledger : &own_ledger_),
      counters_(counters ? counters : &own_counters_) {
  for (const auto& p : snap_->procs) handles_.push_back(p.handle);
  size_t n = snap_->gpus.size();
  keys_.resize(n);
  for (const auto& g : snap_->gpus) keys_[g.index] = Ledger::KeyOf(g);
  ecc_baseline_.assign(n, 0);
  fail_.assign(n, 0);
  link_change_polls_.assign(n, 0);
  retired_threshold_.assign(n, 0);
  fingerprint_ = ProcessorFingerprint(snap_->procs);
}

Monitor::~Monitor() { Stop(); }

void Monitor::AddListener(Listener l) { listeners_.push_back(std::move(l)); }

void Monitor::Notify(int gpu, bool healthy, const std::string& reason) {
  for (auto& l : listeners_) l(gpu, healthy, reason);
}

Status Monitor::Start() {
  if (cfg_.disabled) {
    LOG_INFO(kComp, "health checks disabled by DP_DISABLE_HEALTHCHECKS");
    if (!cfg_.drain_file.empty())
      LOG_WARN(kComp, "--drain-file %s is not applied: health checks are disabled", cfg_.drain_file.c_str());
    return Status::Ok();
  }
  // Only the handles of GPUs in this snapshot are watched.
  std::vector<void*> watched;
  for (const auto& g : snap_->gpus)
    for (const auto& p : g.partitions) watched.push_back(snap_->procs[p.handle].handle);
  handles_ = watched;
  const uint64_t mask = cfg_.EventMask();
  if (!cfg_.events) {
    events_ok_ = false;
    events_reason_ = "off by configuration (--health-events=false)";
    LOG_INFO(kComp, "amdsmi event notification %s; GPU resets are seen by polling only", events_reason_.c_str());
  } else if (!cfg_.event_relay.empty()) {
    // Privilege separation: the relay holds the registration; this process
    // needs no /dev/kfd. It asks the relay to re-enumerate (a new generation
    // may follow a re-partition) and takes its hello as the event state.
    // The monitor thread reads its answer: the supervisor is not held up here.
    RelayConnect();
    if (relay_fd_ < 0)
      LOG_WARN(kComp, "events via relay %s: %s; polling meanwhile, reconnecting (every second at most)",
               cfg_.event_relay.c_str(), events_reason_.c_str());
  } else {
    Status st = lib_->EventsInit(handles_, mask);
    events_ok_ = st.ok();
    events_reason_ = events_ok_ ? "" : st.ToString();
    if (!events_ok_) {
      // Say why: the usual cause in a pod is a device cgroup that denies /dev/kfd.
      int kerr = inventory::KfdAccessErrno(cfg_.driver_root);
      if (kerr == EPERM)
        events_reason_ += "; /dev/kfd not openable (EPERM): the container's device cgroup denies it -- run the "
                          "event relay privileged (--event-relay + --health-event-socket; helm healthEvents: true) for "
                          "GPU_PRE_RESET/POST_RESET events";
      else if (kerr)
        events_reason_ += std::string("; /dev/kfd not openable (") + strerror(kerr) + ")";
      LOG_WARN(kComp, "events off: amdsmi event notification unavailable (%s); using polling only",
               events_reason_.c_str());
    }
  }
  counters_->events_enabled.store(events_ok_ ? 1 : 0);
  LoadVerdicts();
  // A confirmed gap from before this process (the state file): this process's
  // own link to the events may miss nothing, and the wait still has to end.
  for (const auto& g : snap_->gpus) {
    const std::string gap = ledger_->Get(keys_[g.index]).gap;
    if (gap.empty() || !(fail_[g.index] & kFailResetPending)) continue;
    if (ledger_->MarkGap(keys_[g.index], gap, false, SteadyNow()))
      LOG_WARN(kComp, "GPU %s waits for GPU_POST_RESET across an event gap from before this process (%s): back in "
               "service once amdsmi has answered every poll for %g s", g.bdf.c_str(), gap.c_str(),
               static_cast<double>(cfg_.reset_recovery_hold_ms) / 1000.0);
  }
  // GPUs still waiting for GPU_POST_RESET from an earlier generation (or
  // process): a new in-process registration cannot receive what was sent
  // before it existed; events off receive nothing. In relay mode the relay's
  // answer to this generation's reinit says whether anything was missed.
  if (!events_ok_ && (!cfg_.events || cfg_.event_relay.empty()))
    MarkGap("events off: " + events_reason_, false);
  else if (cfg_.event_relay.empty())
    MarkGap("amdsmi event registration renewed by a new monitor generation", false);
  else if (relay_fd_ < 0)
    MarkGap(events_reason_, true);
  if (!cfg_.drain_file.empty()) ApplyDrain();  // at once, not a poll interval later
  LOG_INFO(kComp, "health monitor watching %zu GPU(s) (events %s, poll every %d ms)", snap_->gpus.size(),
           events_ok_ ? "on" : relay_fd_ >= 0 ? "through the relay, once it answers" : "off", cfg_.poll_interval_ms);
  if (cfg_.poll_interval_ms == 0 && cfg_.reset_recovery_hold_ms > 0)
    LOG_WARN(kComp, "DP_HEALTH_POLL_MS=0: no liveness polls, so a GPU waiting for GPU_POST_RESET across an event gap "
             "is not brought back by --reset-recovery-hold-ms (only the event or --return-to-service does); "
             "quarantines, drains and return-to-service requests are still applied every %d ms", kHousekeepingMs);
  // The thread runs even without events and polls: quarantines end, drains
  // and return-to-service requests apply (Housekeeping).
  if (!cfg_.run_thread) return Status::Ok();
  stop_.store(false);
  if (wake_fd_ < 0) wake_fd_ = eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);
  thread_ = std::thread([this] { Run(); });
  return Status::Ok();
}

// Each GPU's verdict and ECC baseline from the ledger: the baseline is the
// one recorded at the first observation of the GPU, not the current count, so
// errors that accrued across a restart still count.
void Monitor::LoadVerdicts() {
  for (const auto& g : snap_->gpus) {
    void* h = snap_->procs[g.partitions.front().handle].handle;
    auto ecc = lib_->UncorrectableErrors(h);
    GpuRecord r = ledger_->Get(keys_[g.index]);
    const uint32_t was = r.fail;
    if (!r.has_baseline && ecc.ok()) {
      r.has_baseline = true;
      r.ecc_baseline = r.ecc_seen = *ecc;
    } else if (ecc.ok() && *ecc < r.ecc_seen) {
      LOG_INFO(kComp, "GPU %s: uncorrectable ECC count %llu below the %llu seen before (counters reset); "
               "re-baselined", g.bdf.c_str(), static_cast<unsigned long long>(*ecc),
               static_cast<unsigned long long>(r.ecc_seen));
      r.ecc_baseline = r.ecc_seen = *ecc;
      if (r.fail & kFailEcc) {
        r.fail &= ~kFailEcc;
        r.reason = r.fail ? "still: " + DescribeFailures(r.fail) : "";
      }
    }
    ecc_baseline_[g.index] = r.ecc_baseline;
    // Retired-page threshold: explicit, else the driver's when readable (root).
    if (cfg_.max_retired_pages > 0) {
      retired_threshold_[g.index] = static_cast<uint32_t>(cfg_.max_retired_pages);
    } else if (cfg_.max_retired_pages < 0) {
      auto t = lib_->RetiredPageThreshold(h);
      retired_threshold_[g.index] = t.ok() ? *t : 0;
    }
    fail_[g.index] = r.fail;
    ledger_->Put(keys_[g.index], r);
    if (r.fail) {
      LOG_WARN(kComp, "GPU %s stays unhealthy from an earlier generation: %s", g.bdf.c_str(), r.reason.c_str());
      Notify(g.index, false, r.reason);
    } else if (was) {
      // The plugins applied the ledger's verdict before this monitor started
      // (Supervisor::PublishPlugins); no poll would change it back.
      LOG_INFO(kComp, "GPU %s healthy again: uncorrectable ECC counters reset since an earlier generation",
               g.bdf.c_str());
      Notify(g.index, true, "uncorrectable ECC counters reset");
    }
  }
}

void Monitor::Sleep(int ms) {
  pollfd p{wake_fd_, POLLIN, 0};
  poll(&p, 1, ms);
}

void Monitor::Stop() {
  if (thread_.joinable()) {
    stop_.store(true);
    uint64_t one = 1;
    ssize_t w = write(wake_fd_, &one, sizeof(one));
    (void)w;
    thread_.join();
  }
  if (wake_fd_ >= 0) {
    close(wake_fd_);
    wake_fd_ = -1;
  }
  if (!cfg_.event_relay.empty()) {
    // Connected or not: where this daemon is in the relay's stream goes to
    // the state file, so a restart is not replayed what it already handled.
    if (relay_fd_ >= 0) close(relay_fd_);
    relay_fd_ = -1;
    events_ok_ = false;
    counters_->FlushRelayCursor();
  } else if (lib_) {
    // Whatever is registered, events on or not (the library undoes a partial
    // registration itself, and stops only what it holds).
    lib_->EventsStop(handles_);
    events_ok_ = false;
  }
}


void Monitor::RelayConnect() {
  relay_tried_ms_ = SteadyNow();
  int fd = ConnectRelay(cfg_.event_relay);
  if (fd < 0) {
    events_reason_ = "event relay " + cfg_.event_relay + " not reachable (" + strerror(errno) + ")";
    if (relay_lost_ms_ == 0) relay_lost_ms_ = SteadyNow();
    counters_->relay_connected.store(0);
    relay_retry_ms_ = std::min(1000, relay_retry_ms_ * 2);
    return;
  }
  RelayAttach(fd);
}

void Monitor::RelayAttach(int fd) {
  relay_fd_ = fd;
  relay_tried_ms_ = SteadyNow();
  relay_retry_ms_ = 100;
  relay_lost_ms_ = 0;
  relay_lost_confirmed_ = false;
  counters_->relay_connected.store(1);
  // Our processors (the relay re-enumerates only if they differ from its
  // registration) and where we are in its event stream (it replays what this
  // daemon missed since, e.g. across a SIGHUP).
  HealthCounters::RelayCursor cur = counters_->GetRelayCursor();
  std::string req = "reinit fp=" + fingerprint_ + " since=" +
                    (cur.valid ? cur.relay + ":" + std::to_string(cur.seq) + ":" + std::to_string(cur.gen)
                               : std::string("-")) + "\n";
  if (send(relay_fd_, req.data(), req.size(), MSG_NOSIGNAL) != static_cast<ssize_t>(req.size())) {
    RelayClose("cannot write to the event relay");
    return;
  }
  relay_buf_.clear();
  relay_synced_ = false;
  relay_cursor_sent_ = cur.valid;
  relay_connected_ms_ = SteadyNow();
  relay_overdue_ = false;
  events_reason_ = "waiting for the event relay's hello";
}

void Monitor::RelayClose(const std::string& why) {
  if (relay_fd_ >= 0) {
    close(relay_fd_);
    counters_->relay_disconnects.fetch_add(1);
  }
  counters_->relay_connected.store(0);
  relay_fd_ = -1;
  if (events_ok_) LOG_WARN(kComp, "event relay: %s; polling only until it is back", why.c_str());
  events_ok_ = false;
  events_reason_ = why;
  counters_->events_enabled.store(0);
  relay_lost_ms_ = SteadyNow();
  relay_lost_confirmed_ = false;
  relay_tried_ms_ = relay_lost_ms_;  // the next try in relay_retry_ms_
  // Events sent meanwhile are replayed if the relay comes back holding them.
  MarkGap("event relay: " + why, true);
}

void Monitor::RelayWait(int ms) {
  pollfd p[2] = {{relay_fd_, POLLIN, 0}, {wake_fd_, POLLIN, 0}};
  if (poll(p, wake_fd_ >= 0 ? 2 : 1, ms) <= 0 || !(p[0].revents & (POLLIN | POLLHUP | POLLERR))) return;
  char buf[4096];
  // Lines are handled as they arrive, at most 1 MiB per wake-up: a relay that
  // kept writing (a bug) can neither hold this thread nor grow the buffer past
  // one over-long line (64 KiB, then dropped).
  size_t budget = size_t{1} << 20;
  bool closed = false;
  while (budget > 0) {
    const ssize_t n = recv(relay_fd_, buf, sizeof(buf), 0);
    if (n < 0 && errno == EINTR) continue;
    if (n <= 0) {
      closed = n == 0 || errno != EAGAIN;
      break;
    }
    budget -= std::min(budget, static_cast<size_t>(n));
    relay_buf_.append(buf, static_cast<size_t>(n));
    size_t nl;
    while ((nl = relay_buf_.find('\n')) != std::string::npos) {
      RelayLine l = ParseRelayLine(std::string_view(relay_buf_).substr(0, nl));
      relay_buf_.erase(0, nl + 1);
      HandleRelayLine(l);
    }
    if (relay_buf_.size() > 65536) relay_buf_.clear();
  }
  if (closed) RelayClose("the event relay closed the connection");
}

void Monitor::HandleRelayLine(const RelayLine& l) {
  if (l.kind == "hello" && !l.after_reinit && !relay_synced_) {
    // The connect hello predates the re-enumeration this monitor asked for.
  } else if (l.kind == "hello") {
    relay_synced_ = true;
    bool was = events_ok_;
    events_ok_ = l.events_ok;
    events_reason_ = l.events_ok ? "" : "relay: " + l.reason;
    counters_->events_enabled.store(events_ok_ ? 1 : 0);
    if (events_ok_ && !was) LOG_INFO(kComp, "events on through the relay at %s", cfg_.event_relay.c_str());
    if (!events_ok_) LOG_WARN(kComp, "event relay reports %s; using polling only", events_reason_.c_str());
    if (!l.relay.empty()) counters_->SetRelayCursor({true, l.relay, l.seq, l.gen});
    if (!events_ok_) {
      MarkGap("the event relay reports events off (" + l.reason + ")", false);
    } else if (l.gap != 0) {
      MarkGap(l.gap != 1             ? "the event relay cannot replay missed events (an older relay)"
              : !relay_cursor_sent_ ? "a first connection to the event relay: what was sent before it is unknown"
                                    : "the event relay renewed its registration or no longer holds the events missed",
              false);
    } else {
      for (const auto& key : ledger_->CancelTentativeGaps())
        LOG_INFO(kComp, "GPU %s: the event relay replayed what was missed; waiting for GPU_POST_RESET again",
                 key.c_str());
    }
  } else if (l.kind == "event") {
    counters_->AdvanceRelaySeq(l.seq);
    // The relay's processor -> this snapshot's handle: by KFD node when both
    // know it, else by PCI address and partition. "node=- bdf=-": the relay
    // could not place it either (amdsmi named a processor it never enumerated).
    void* handle = nullptr;
    const bool placed = l.node != 0xffffffffu || (!l.bdf.empty() && l.bdf != "-");
    for (const auto& pr : snap_->procs) {
      bool hit = l.node != 0xffffffffu && pr.kfd_node != 0xffffffffu ? pr.kfd_node == l.node
                                                                     : pr.bdf == l.bdf && pr.partition_id == l.part;
      if (placed && hit) {
        handle = pr.handle;
        break;
      }
    }
    std::string unplaced;
    if (!handle && placed)
      unplaced = "the relay's processor (node " + (l.node == 0xffffffffu ? std::string("-") : std::to_string(l.node)) +
                 ", " + l.bdf + " partition " + std::to_string(l.part) + ") is none of this daemon's";
    else if (!handle)
      unplaced = "the event relay could not place it either";
    // In order with the hellos around it; a replayed event is known by its
    // relay and sequence number.
    const HealthCounters::RelayCursor cur = counters_->GetRelayCursor();
    HandleEvent({handle, l.type, l.message}, unplaced,
                cur.valid && l.seq ? cur.relay + ":" + std::to_string(l.seq) : std::string());
    // An event that changed a verdict is saved as handled at once (others at
    // most once a second): a restart replaying a GPU_PRE_RESET the operator
    // has since returned, or a GPU_POST_RESET older than an ECC verdict,
    // would undo what came after it.
    if (Classify(cfg_, l.type) != 0) counters_->FlushRelayCursor();
  } else if (l.kind.empty()) {
    LOG_WARN(kComp, "event relay: malformed line ignored");
  }
}

void Monitor::ApplyDrain() {
  std::string text;
  int fd = open(cfg_.drain_file.c_str(), O_RDONLY | O_CLOEXEC | O_NONBLOCK);
  if (fd >= 0) {
    char buf[4096];
    ssize_t n;
    while ((n = read(fd, buf, sizeof(buf))) > 0 && text.size() < 65536) text.append(buf, static_cast<size_t>(n));
    close(fd);
  }  // absent or unreadable: nothing drained
  const std::set<std::string> names = DrainTokens(text);
  for (const auto& g : snap_->gpus) {
    bool drained = false;
    for (const auto& n : DrainNames(g)) drained = drained || names.count(n);
    bool was = fail_[g.index] & kFailDrained;
    if (drained && !was) Update(g.index, kFailDrained, 0, "drained by the operator (" + cfg_.drain_file + ")");
    if (!drained && was) Update(g.index, 0, kFailDrained, "removed from the drain file");
  }
}

void Monitor::ApplyReturnRequests() {
  // Taken by rename first: a request written meanwhile is a new file, read at
  // the next poll, never lost to our unlink.
  const std::string req = cfg_.drain_file + ".return", taken = req + ".taken";
  if (rename(req.c_str(), taken.c_str()) != 0) {
    if (errno != ENOENT && !return_request_warned_) {  // e.g. a read-only directory: say so once
      return_request_warned_ = true;
      LOG_WARN(kComp, "cannot take the return-to-service request %s: %s", req.c_str(), strerror(errno));
    }
    return;
  }
  std::string text;
  int fd = open(taken.c_str(), O_RDONLY | O_CLOEXEC | O_NONBLOCK);
  if (fd >= 0) {
    char buf[4096];
    ssize_t n;
    while ((n = read(fd, buf, sizeof(buf))) > 0 && text.size() < 65536) text.append(buf, static_cast<size_t>(n));
    close(fd);
  }
  unlink(taken.c_str());
  const std::set<std::string> names = DrainTokens(text);
  for (const auto& g : snap_->gpus) {
    bool named = false;
    for (const auto& n : DrainNames(g)) named = named || names.count(n);
    if (!named) continue;
    const std::string& key = keys_[g.index];
    // As if the GPU's line were deleted from the state file: the current ECC
    // count is the new baseline, no reset history, no gap.
    GpuRecord r = ledger_->Get(key);
    const std::string was = r.reason;
    auto ecc = lib_->UncorrectableErrors(snap_->procs[g.partitions.front().handle].handle);
    if (ecc.ok()) {
      ecc_baseline_[g.index] = *ecc;
      r.has_baseline = true;
      r.ecc_baseline = r.ecc_seen = *ecc;
      ledger_->Put(key, r);
    }
    ledger_->ClearGap(key);
    ledger_->ClearResets(key);
    if (!(fail_[g.index] & ~kFailDrained)) {
      LOG_INFO(kComp, "GPU %s: return-to-service asked: %s", g.bdf.c_str(),
               fail_[g.index] ? "drained -- the drain file keeps it out (--undrain)" : "nothing held against it");
      continue;
    }
    LOG_WARN(kComp, "GPU %s returned to service by the operator (was: %s)", g.bdf.c_str(), was.c_str());
    Update(g.index, 0, ~static_cast<uint32_t>(kFailDrained), "returned to service by the operator");
  }
}

void Monitor::Housekeeping() {
  if (!cfg_.drain_file.empty()) {
    ApplyDrain();
    ApplyReturnRequests();
  }
  for (const auto& g : snap_->gpus) EndQuarantine(g.index);
}

void Monitor::EndQuarantine(int gpu) {
  if (!(fail_[gpu] & kFailFlapping)) return;
  // Quarantine ends after a whole window without a GPU_PRE_RESET (or with
  // damping turned off).
  const int64_t now = clock_->WallMs();
  const int64_t quiet = now - ledger_->LastReset(keys_[gpu], now);
  if (cfg_.reset_flap_limit <= 0 || quiet >= cfg_.reset_flap_window_ms)
    Update(gpu, 0, kFailFlapping,
           cfg_.reset_flap_limit <= 0 ? "reset-flap damping off"
                                      : "no reset for " + std::to_string(quiet / 1000) + " s: quarantine over");
}

void Monitor::PollOnce() {
  uint64_t poll = counters_->polls.fetch_add(1) + 1;
  Housekeeping();
  size_t answered = 0, ecc_ok = 0, retired_ok = 0;
  std::string counts;
  for (const auto& g : snap_->gpus) {
    void* h = snap_->procs[g.partitions.front().handle].handle;
    if (layout_listener_ && !layout_changed_ && PollLayout(g, h))
      return;  // handles are about to be re-created; no health verdicts from them
    if (!PollLiveness(g, h, poll)) continue;
    ++answered;
    counters_->responsive.fetch_add(1);
    retired_ok += PollRetiredPages(g, h);
    if (auto ecc = PollEcc(g, h, poll)) {
      ++ecc_ok;
      counts += (counts.empty() ? "" : ",") + std::to_string(*ecc);
    }
  }
  if (poll == 1) {
    size_t thresholds = 0;
    for (uint32_t t : retired_threshold_) thresholds += t != 0;
    LOG_INFO(kComp, "health poll #1: %zu/%zu GPU(s) responding, uncorrectable ECC readable on %zu (counts [%s]), "
             "retired pages readable on %zu (threshold on %zu); events %s%s%s", answered, snap_->gpus.size(), ecc_ok,
             counts.c_str(), retired_ok, thresholds, events_ok_ ? "on" : "off", events_ok_ ? "" : ": ",
             events_reason_.c_str());
  }
}

bool Monitor::PollLayout(const inventory::PhysicalGpu& g, void* h) {
  auto [compute, memory] = lib_->PartitionModes(h);
  for (auto& c : compute) c = static_cast<char>(toupper(static_cast<unsigned char>(c)));
  for (auto& c : memory) c = static_cast<char>(toupper(static_cast<unsigned char>(c)));
  std::string why;
  if ((!compute.empty() && compute != g.reported_compute) || (!memory.empty() && memory != g.reported_memory)) {
    why = "GPU " + g.bdf + " partition mode changed " + g.reported_compute + "/" + g.reported_memory + " -> " +
          compute + "/" + memory;
  } else {
    // xGMI links that went down (or came back) change the topology scores
    // GetPreferredAllocation uses; re-enumerate once the new count has held for
    // two consecutive polls (a flapping link does not cause restart storms).
    int down = lib_->XgmiLinksDown(h);
    if (down == g.xgmi_links_down) {
      link_change_polls_[g.index] = 0;
      return false;
    }
    if (++link_change_polls_[g.index] < 2) return false;
    why = "GPU " + g.bdf + " xGMI links down " + std::to_string(g.xgmi_links_down) + " -> " + std::to_string(down);
  }
  layout_changed_ = true;
  LOG_WARN(kComp, "%s", why.c_str());
  layout_listener_(why);
  return true;
}

bool Monitor::PollLiveness(const inventory::PhysicalGpu& g, void* h, uint64_t poll) {
  const bool alive = lib_->Responsive(h);
  if (!alive && !(fail_[g.index] & kFailUnresponsive))
    Update(g.index, kFailUnresponsive, 0, "device not responding to amdsmi");
  else if (alive && (fail_[g.index] & kFailUnresponsive))
    Update(g.index, 0, kFailUnresponsive, "device responding again");
  // The polled recovery wants the driver answering about the device's memory
  // too (it fails while a reset is under way), not just the UUID amdsmi
  // keeps; on a platform where that query never works, liveness alone.
  Result<uint64_t> used = alive ? lib_->VramUsed(h) : Result<uint64_t>(Unavailable("not responding"));
  if (used.ok()) counters_->SetVramUsed(g.bdf, *used);
  // The SMU's metrics (graphics activity) are refused while the GPU is in
  // reset, which makes them the better sign that a reset is over; asked only
  // of a GPU waiting across a gap.
  bool activity_ok = true;
  if (alive && (fail_[g.index] & kFailResetPending) && ledger_->Gap(keys_[g.index], nullptr)) {
    auto act = lib_->Activity(h);
    if (act.ok()) counters_->MarkQueryOk(g.bdf, "activity");
    activity_ok = act.ok() || !counters_->QueryEverOk(g.bdf, "activity");
  } else if (alive && poll == 1) {
    if (lib_->Activity(h).ok()) counters_->MarkQueryOk(g.bdf, "activity");  // learn whether it works here
  }
  // (the counters outlive monitor generations: "ever readable" does too)
  CheckGapRecovery(g.index, alive && activity_ok && (used.ok() || !counters_->HasVramUsed(g.bdf)));
  return alive;
}

// Retired HBM pages: the driver takes a page out of service after an
// uncorrectable error in it; past the threshold the GPU is not trusted with
// new work (the reference has no such check).
bool Monitor::PollRetiredPages(const inventory::PhysicalGpu& g, void* h) {
  auto bp = lib_->RetiredPages(h);
  if (!bp.ok()) {
    counters_->retired_read_errors.fetch_add(1);
    return false;
  }
  counters_->retired_reads_ok.fetch_add(1);
  counters_->SetRetiredPages(g.bdf, *bp);
  const uint32_t thr = retired_threshold_[g.index];
  const bool failed = fail_[g.index] & kFailRetiredPages;
  if (thr && *bp >= thr && !failed)
    Update(g.index, kFailRetiredPages, 0,
           std::to_string(*bp) + " retired HBM pages (threshold " + std::to_string(thr) + ")");
  else if (failed && (!thr || *bp < thr))
    Update(g.index, 0, kFailRetiredPages, "retired HBM pages below the threshold");
  return true;
}

std::optional<uint64_t> Monitor::PollEcc(const inventory::PhysicalGpu& g, void* h, uint64_t poll) {
  auto ecc = lib_->UncorrectableErrors(h);
  if (!ecc.ok()) {
    counters_->ecc_read_errors.fetch_add(1);
    if (poll == 1)
      LOG_WARN(kComp, "GPU %s: uncorrectable ECC count unreadable (%s); read again every poll", g.bdf.c_str(),
               ecc.status().ToString().c_str());
    return std::nullopt;
  }
  counters_->ecc_reads_ok.fetch_add(1);
  GpuRecord r = ledger_->Get(keys_[g.index]);
  if (!r.has_baseline) {  // unreadable when the monitor started: the first read is the baseline
    r.has_baseline = true;
    r.ecc_baseline = r.ecc_seen = *ecc;
    ecc_baseline_[g.index] = *ecc;
    ledger_->Put(keys_[g.index], r);
    return *ecc;
  }
  if (*ecc < r.ecc_seen) {
    // The driver reset its RAS counters (GPU reset / driver reload): the
    // errors that failed the GPU are gone with the state they described.
    LOG_INFO(kComp, "GPU %s: uncorrectable ECC count fell %llu -> %llu (counters reset); re-baselined",
             g.bdf.c_str(), static_cast<unsigned long long>(r.ecc_seen), static_cast<unsigned long long>(*ecc));
    ecc_baseline_[g.index] = *ecc;
    r.has_baseline = true;
    r.ecc_baseline = r.ecc_seen = *ecc;
    ledger_->Put(keys_[g.index], r);
    if (fail_[g.index] & kFailEcc) Update(g.index, 0, kFailEcc, "uncorrectable ECC counters reset");
    return *ecc;
  }
  if (*ecc > r.ecc_seen) {
    r.ecc_seen = *ecc;
    ledger_->Put(keys_[g.index], r);
  }
  if (*ecc > ecc_baseline_[g.index] && !(fail_[g.index] & kFailEcc))
    Update(g.index, kFailEcc, 0,
           "uncorrectable ECC errors rose to " + std::to_string(*ecc) + " (baseline " +
               std::to_string(ecc_baseline_[g.index]) + ")");
  return *ecc;
}

void Monitor::MarkGap(const std::string& why, bool tentative) {
  if (!tentative) counters_->event_gaps.fetch_add(1);
  const int64_t now = SteadyNow();
  for (const auto& g : snap_->gpus) {
    if (!(fail_[g.index] & kFailResetPending)) continue;
    if (!ledger_->MarkGap(keys_[g.index], why, tentative, now)) continue;
    if (cfg_.reset_recovery_hold_ms > 0 && tentative)
      LOG_WARN(kComp, "GPU %s waits for GPU_POST_RESET; events may have been missed (%s): unless the event relay "
               "replays them, it is back in service once amdsmi has answered every poll for %g s",
               g.bdf.c_str(), why.c_str(), static_cast<double>(cfg_.reset_recovery_hold_ms) / 1000.0);
    else if (cfg_.reset_recovery_hold_ms > 0)
      LOG_WARN(kComp, "GPU %s waits for GPU_POST_RESET across an event gap (%s): back in service once amdsmi has "
               "answered every poll for %g s, unless a GPU_PRE_RESET arrives", g.bdf.c_str(), why.c_str(),
               static_cast<double>(cfg_.reset_recovery_hold_ms) / 1000.0);
    else
      LOG_WARN(kComp, "GPU %s waits for GPU_POST_RESET across an event gap (%s); --reset-recovery-hold-ms=0: only "
               "the event (or the operator) brings it back", g.bdf.c_str(), why.c_str());
  }
}

void Monitor::CheckGapRecovery(int gpu, bool alive) {
  const std::string& key = keys_[gpu];
  GapMark m;
  if (!ledger_->Gap(key, &m)) return;
  if (!(fail_[gpu] & kFailResetPending)) {  // the event came after all, or the operator cleared it
    ledger_->ClearGap(key);
    return;
  }
  const int64_t now = SteadyNow();
  if (!alive) {
    ledger_->SetResponsiveSince(key, 0);
    return;
  }
  if (m.responsive_since_ms == 0) {
    m.responsive_since_ms = now;
    ledger_->SetResponsiveSince(key, now);
  }
  // A tentative gap (the relay connection dropped) may be replayed whole:
  // only a confirmed one lets polling end the wait.
  if (cfg_.reset_recovery_hold_ms <= 0 || m.tentative) return;
  const int64_t from = std::max(m.since_ms, m.responsive_since_ms);
  if (now - from < cfg_.reset_recovery_hold_ms) return;
  const auto& g = snap_->gpus[gpu];
  char held[32];
  snprintf(held, sizeof(held), "%.1f", static_cast<double>(now - from) / 1000.0);
  std::string why = "no GPU_POST_RESET after an event gap (" + m.why + "); amdsmi answered every poll for " + held +
                    " s";
  LOG_WARN(kComp, "GPU %s recovered without GPU_POST_RESET: %s", g.bdf.c_str(), why.c_str());
  counters_->CountRecovered(g.bdf);
  ledger_->ClearGap(key);
  Update(gpu, 0, kFailResetPending, why);
}

void Monitor::Update(int gpu, uint32_t set, uint32_t clear, const std::string& reason) {
  uint32_t before = fail_[gpu];
  uint32_t after = (before | set) & ~clear;
  fail_[gpu] = after;
  GpuRecord r = ledger_->Get(keys_[gpu]);
  r.fail = after;
  if (!after) r.reason.clear();
  else if (set & ~before) r.reason = reason;
  else if (clear & before) r.reason = "still: " + DescribeFailures(after);  // the old reason may be the cleared one
  ledger_->Put(keys_[gpu], r);
  if ((before == 0) != (after == 0)) {
    Notify(gpu, after == 0, reason);
  } else if (after) {
    LOG_INFO(kComp, "GPU %s stays unhealthy (%s; failure bits %u -> %u)", snap_->gpus[gpu].bdf.c_str(),
             reason.c_str(), before, after);
  }
}

void Monitor::HandleEvent(const smi::Event& e, const std::string& unplaced, const std::string& event_id) {
  counters_->events_received.fetch_add(1);
  int proc = -1;
  if (e.handle)
    for (size_t i = 0; i < snap_->procs.size(); ++i)
      if (snap_->procs[i].handle == e.handle) proc = static_cast<int>(i);
  const int gpu = proc >= 0 ? snap_->GpuOfHandle(proc) : -1;
  const int verdict = Classify(cfg_, e.type);
  const std::string name = smi::EventTypeName(e.type);
  if (proc >= 0 && gpu < 0) {
    // A GPU of the node this daemon does not serve (--devices): the relay
    // forwards every GPU's events.
    LOG_DEBUG(kComp, "event %s(%u) on %s, which this daemon does not serve", name.c_str(), e.type,
              snap_->procs[proc].bdf.c_str());
    return;
  }
  if (gpu < 0) {
    HandleUnmatched(e, verdict, unplaced.empty() ? "amdsmi named a processor handle it never enumerated" : unplaced);
    return;
  }
  const std::string& bdf = snap_->gpus[gpu].bdf;
  // KFD's informational events come with every HIP process: not worth a line
  // each. Ignored ones (a workload's VM faults, throttling) can come in storms:
  // the first ten of each type, then every thousandth (all are counted).
  if (e.type > smi::kEvtGpuPostReset && verdict == 0) {
    LOG_DEBUG(kComp, "event %s(%u) on GPU %d (%s): %s (counted)", name.c_str(), e.type, gpu, bdf.c_str(),
              e.message.c_str());
  } else if (verdict == 0) {
    const uint64_t n = ++ignored_seen_[e.type];
    if (n <= 10 || n % 1000 == 0)
      LOG_INFO(kComp, "event %s(%u) on GPU %d (%s): %s (ignored; %llu of this type so far)", name.c_str(), e.type,
               gpu, bdf.c_str(), e.message.c_str(), static_cast<unsigned long long>(n));
  } else {
    LOG_INFO(kComp, "event %s(%u) on GPU %d (%s): %s", name.c_str(), e.type, gpu, bdf.c_str(), e.message.c_str());
  }
  counters_->CountEvent(bdf, name);
  if (verdict == 0) return;
  std::string why = name + ": " + e.message;
  if (verdict > 0) {
    // A completed reset clears every failure, poll-detected ones included,
    // and the ECC count after the reset is the new baseline.
    void* h = snap_->procs[snap_->gpus[gpu].partitions.front().handle].handle;
    auto ecc = lib_->UncorrectableErrors(h);
    if (ecc.ok()) {
      ecc_baseline_[gpu] = *ecc;
      GpuRecord r = ledger_->Get(keys_[gpu]);
      r.has_baseline = true;
      r.ecc_baseline = r.ecc_seen = *ecc;
      ledger_->Put(keys_[gpu], r);
    }
    if (fail_[gpu] == 0) Notify(gpu, true, why);  // keep the reference's idempotent notify
    // A drain outlives a reset, and so does a flapping GPU's quarantine.
    Update(gpu, 0, ~static_cast<uint32_t>(kFailDrained | kFailFlapping), why);
    ledger_->ClearGap(keys_[gpu]);
  } else {
    // KFD reports a reset on every KFD node of the GPU -- each compute
    // partition (DPX/QPX/CPX) -- so one reset is a GPU_PRE_RESET per partition,
    // then a GPU_POST_RESET per partition. Only the first, the one that finds
    // the GPU not waiting yet, starts a reset; the others belong to it.
    const bool same_reset = e.type == smi::kEvtGpuPreReset && (fail_[gpu] & kFailResetPending);
    Update(gpu, e.type == smi::kEvtGpuPreReset ? kFailResetPending : kFailEvent, 0, why);
    if (e.type == smi::kEvtGpuPreReset) {
      // Only a gap after it lets polling end the wait (the GPU_POST_RESETs come
      // after every partition's GPU_PRE_RESET: one seen now is not missed yet).
      ledger_->ClearGap(keys_[gpu]);
      if (cfg_.reset_flap_limit > 0 && !same_reset) {
        int n = ledger_->RecordReset(keys_[gpu], clock_->WallMs(), cfg_.reset_flap_window_ms, event_id);
        if (n >= cfg_.reset_flap_limit && !(fail_[gpu] & kFailFlapping)) {
          std::string w = std::to_string(cfg_.reset_flap_window_ms / 1000);
          LOG_WARN(kComp, "GPU %s reset %d times within %s s: quarantined until %s s pass without a reset",
                   bdf.c_str(), n, w.c_str(), w.c_str());
          Update(gpu, kFailFlapping, 0, std::to_string(n) + " resets within " + w + " s (flapping)");
        }
      }
    }
  }
}

void Monitor::HandleUnmatched(const smi::Event& e, int verdict, const std::string& why) {
  const std::string name = smi::EventTypeName(e.type);
  counters_->CountUnmatched(name);
  const bool reset = e.type == smi::kEvtGpuPreReset && verdict < 0;
  // Logged every time for a reset; otherwise the first ten, then every thousandth.
  if (reset || ++unmatched_seen_ <= 10 || unmatched_seen_ % 1000 == 0)
    LOG_ERROR(kComp, "event %s(%u) on a processor that matches no GPU of this node (%s): %s%s", name.c_str(), e.type,
              why.c_str(), e.message.c_str(),
              reset ? "; every GPU is held until the polled check (--reset-recovery-hold-ms) or the operator returns it"
                    : "; counted in amdgpu_dp_unmatched_events_total");
  if (!reset) return;
  // The reference's rule for an event that names no device: every device goes
  // Unhealthy (nvidia.go:244-251). Here every GPU waits for a GPU_POST_RESET,
  // which cannot be placed either: each gets a confirmed event gap too, so the
  // polled recovery check brings it back after the hold. A GPU already waiting
  // for its own GPU_POST_RESET keeps waiting for that (no gap is added to it).
  const std::string reason = "GPU_PRE_RESET on an unknown processor (" + why + "): " + e.message;
  const int64_t now = SteadyNow();
  counters_->event_gaps.fetch_add(1);
  for (const auto& g : snap_->gpus) {
    const bool waiting = fail_[g.index] & kFailResetPending;
    Update(g.index, kFailResetPending, 0, reason);
    if (!waiting) ledger_->MarkGap(keys_[g.index], "a GPU_PRE_RESET that could not be placed", false, now);
  }
}

void Monitor::InProcessWait(int ms, std::vector<smi::Event>* events) {
  events->clear();
  Status st = lib_->EventsWait(ms, events);
  if (!st.ok()) {
    if (wait_failures_++ == 0) wait_failing_since_ms_ = SteadyNow();
    if (wait_failures_ == 1 || wait_failures_ % 600 == 0)  // the first, then about one a minute
      LOG_WARN(kComp, "event wait failed (%llu in a row): %s", static_cast<unsigned long long>(wait_failures_),
               st.ToString().c_str());
    // Waits that keep failing deliver no events: say so (the metric, the
    // relay-less equivalent of the relay's watchdog) and keep trying.
    if (!events_failing_ && SteadyNow() - wait_failing_since_ms_ > cfg_.event_fail_ms) {
      events_failing_ = true;
      counters_->events_enabled.store(0);
      LOG_ERROR(kComp, "amdsmi event waits have failed for %lld ms: events off, polling only until they succeed",
                static_cast<long long>(SteadyNow() - wait_failing_since_ms_));
      MarkGap("amdsmi event waits failing", false);
    }
    if (ms > 0) Sleep(ms);
  } else if (wait_failures_) {
    wait_failures_ = 0;
    if (events_failing_) {
      events_failing_ = false;
      counters_->events_enabled.store(1);
      LOG_INFO(kComp, "amdsmi event waits succeed again: events on");
    }
  }
  for (const auto& e : *events) HandleEvent(e);
}

void Monitor::RelayDeadlines() {
  // A relay that accepted the reinit but never answers it (its registrar
  // stuck in amdsmi): events cannot be trusted to arrive.
  if (relay_fd_ >= 0 && !relay_synced_ && !relay_overdue_ && SteadyNow() - relay_connected_ms_ > cfg_.event_fail_ms) {
    relay_overdue_ = true;
    LOG_WARN(kComp, "the event relay has not answered this daemon's reinit for %d ms; polling only until it does",
             cfg_.event_fail_ms);
    MarkGap("the event relay did not answer", false);
  }
  // A relay away for good cannot replay anything: the tentative gap holds.
  if (relay_fd_ < 0 && relay_lost_ms_ != 0 && !relay_lost_confirmed_ &&
      SteadyNow() - relay_lost_ms_ > cfg_.event_fail_ms) {
    relay_lost_confirmed_ = true;
    char secs[32];
    snprintf(secs, sizeof(secs), "%g", cfg_.event_fail_ms / 1000.0);
    MarkGap(std::string("the event relay has been unreachable for ") + secs + " s", false);
  }
}

void Monitor::Run() {
  using SteadyClock = std::chrono::steady_clock;
  // Polls, or -- with polls off -- the housekeeping they include.
  const int period = cfg_.poll_interval_ms > 0 ? cfg_.poll_interval_ms : kHousekeepingMs;
  auto next_poll = SteadyClock::now() + std::chrono::milliseconds(period);
  std::vector<smi::Event> events;
  while (!stop_.load()) {
    counters_->loop_beat_ms.store(Clock::System()->SteadyMs());  // /healthz compares it with the real clock
    // An amdsmi event wait cannot be interrupted: bounded so Stop() (SIGHUP,
    // config, re-partition, exit) is prompt -- the reference waits 5000 ms.
    // Every other wait here also ends on the wake eventfd, so it sleeps until
    // the next thing due (a poll, a relay reconnection or deadline): an idle
    // daemon wakes a few times a second at most, not ten.
    const bool in_process_wait = events_ok_ && (cfg_.event_relay.empty() || !cfg_.events);
    int slice = in_process_wait ? 100 : 5000;
    if (in_process_wait && cfg_.wait_ms > 0 && cfg_.wait_ms < slice) slice = cfg_.wait_ms;
    {  // wake for the next poll, not a slice later
      auto until = std::chrono::duration_cast<std::chrono::milliseconds>(next_poll - SteadyClock::now()).count();
      slice = static_cast<int>(std::max<long long>(1, std::min<long long>(slice, until)));
    }
    if (!cfg_.event_relay.empty() && cfg_.events) {
      const int64_t now = SteadyNow();
      auto due = [&](int64_t at) { slice = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(slice, at - now))); };
      if (relay_fd_ < 0) due(relay_tried_ms_ + relay_retry_ms_);
      if (relay_fd_ >= 0 && !relay_synced_ && !relay_overdue_) due(relay_connected_ms_ + cfg_.event_fail_ms + 1);
      if (relay_fd_ < 0 && relay_lost_ms_ != 0 && !relay_lost_confirmed_) due(relay_lost_ms_ + cfg_.event_fail_ms + 1);
      if (relay_fd_ < 0 && SteadyNow() - relay_tried_ms_ >= relay_retry_ms_) {
        RelayConnect();
        if (relay_fd_ >= 0) LOG_INFO(kComp, "connected to the event relay at %s", cfg_.event_relay.c_str());
      }
      if (relay_fd_ >= 0) RelayWait(slice);
      else Sleep(slice);
      RelayDeadlines();
    } else if (events_ok_) {
      InProcessWait(slice, &events);
    } else {
      Sleep(slice);
    }
    if (SteadyClock::now() >= next_poll) {
      if (cfg_.poll_interval_ms > 0) PollOnce();
      else Housekeeping();
      next_poll = SteadyClock::now() + std::chrono::milliseconds(period);
    }
  }
  counters_->loop_beat_ms.store(0);
}

}  // namespace adp::health

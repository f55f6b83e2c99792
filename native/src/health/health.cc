#include "health/health.h"

#include <poll.h>
#include <sys/eventfd.h>
#include <unistd.h>

#include <cctype>
#include <chrono>
#include <cstdlib>

#include "common/log.h"
#include "common/strings.h"

namespace adp::health {
namespace {
constexpr const char* kComp = "health";

const char* EventName(uint32_t t) {
  switch (t) {
    case 1: return "VMFAULT";
    case 2: return "THERMAL_THROTTLE";
    case 3: return "GPU_PRE_RESET";
    case 4: return "GPU_POST_RESET";
    default: return "EVENT";
  }
}
}  // namespace

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
  return FromValues(std::getenv("DP_DISABLE_HEALTHCHECKS"), std::getenv("DP_HEALTH_POLL_MS"));
}

int Monitor::Classify(const HealthConfig& cfg, uint32_t type) {
  if (cfg.ignored.count(type)) return 0;
  if (type == smi::kEvtGpuPostReset) return +1;
  return -1;
}

Monitor::Monitor(smi::Library* lib, std::shared_ptr<const inventory::Snapshot> snap, HealthConfig cfg)
    : lib_(lib), snap_(std::move(snap)), cfg_(std::move(cfg)) {
  for (const auto& p : snap_->procs) handles_.push_back(p.handle);
  size_t n = snap_->gpus.size();
  ecc_baseline_.assign(n, 0);
  unresponsive_.assign(n, 0);
  ecc_failed_.assign(n, 0);
  link_change_polls_.assign(n, 0);
}

Monitor::~Monitor() { Stop(); }

void Monitor::AddListener(Listener l) { listeners_.push_back(std::move(l)); }

void Monitor::Notify(int gpu, bool healthy, const std::string& reason) {
  for (auto& l : listeners_) l(gpu, healthy, reason);
}

Status Monitor::Start() {
  if (cfg_.disabled) {
    LOG_INFO(kComp, "health checks disabled by DP_DISABLE_HEALTHCHECKS");
    return Status::Ok();
  }
  // Only the handles of GPUs in this snapshot are watched.
  std::vector<void*> watched;
  for (const auto& g : snap_->gpus)
    for (const auto& p : g.partitions) watched.push_back(snap_->procs[p.handle].handle);
  handles_ = watched;
  uint64_t mask = smi::EventMask(smi::kEvtGpuPreReset) | smi::EventMask(smi::kEvtGpuPostReset) |
                  smi::EventMask(smi::kEvtVmFault) | smi::EventMask(smi::kEvtThermalThrottle);
  Status st = lib_->EventsInit(handles_, mask);
  events_ok_ = st.ok();
  if (!events_ok_)
    LOG_WARN(kComp, "amdsmi event notification unavailable (%s); using polling only",
             st.ToString().c_str());
  for (const auto& g : snap_->gpus) {
    void* h = snap_->procs[g.partitions.front().handle].handle;
    auto ecc = lib_->UncorrectableErrors(h);
    ecc_baseline_[g.index] = ecc.ok() ? *ecc : 0;
  }
  LOG_INFO(kComp, "health monitor watching %zu GPU(s) (events %s, poll every %d ms)", snap_->gpus.size(),
           events_ok_ ? "on" : "off", cfg_.poll_interval_ms);
  if (!events_ok_ && cfg_.poll_interval_ms == 0) return Status::Ok();
  stop_.store(false);
  if (wake_fd_ < 0) wake_fd_ = eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);
  thread_ = std::thread([this] { Run(); });
  return Status::Ok();
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
  if (events_ok_) {
    lib_->EventsStop(handles_);
    events_ok_ = false;
  }
}

void Monitor::PollOnce() {
  for (const auto& g : snap_->gpus) {
    void* h = snap_->procs[g.partitions.front().handle].handle;
    if (layout_listener_ && !layout_changed_) {
      auto [compute, memory] = lib_->PartitionModes(h);
      for (auto& c : compute) c = static_cast<char>(toupper(static_cast<unsigned char>(c)));
      for (auto& c : memory) c = static_cast<char>(toupper(static_cast<unsigned char>(c)));
      bool changed = (!compute.empty() && compute != g.reported_compute) ||
                     (!memory.empty() && memory != g.reported_memory);
      if (changed) {
        layout_changed_ = true;
        std::string why = "GPU " + g.bdf + " partition mode changed " + g.reported_compute + "/" +
                          g.reported_memory + " -> " + compute + "/" + memory;
        LOG_WARN(kComp, "%s", why.c_str());
        layout_listener_(why);
        return;  // handles are about to be re-created; no health verdicts from them
      }
      // xGMI links that went down (or came back) change the topology scores
      // GetPreferredAllocation uses; re-enumerate once the new count has held for
      // two consecutive polls (a flapping link does not cause restart storms).
      int down = lib_->XgmiLinksDown(h);
      if (down != g.xgmi_links_down) {
        if (++link_change_polls_[g.index] >= 2) {
          layout_changed_ = true;
          std::string why = "GPU " + g.bdf + " xGMI links down " + std::to_string(g.xgmi_links_down) +
                            " -> " + std::to_string(down);
          LOG_WARN(kComp, "%s", why.c_str());
          layout_listener_(why);
          return;
        }
      } else {
        link_change_polls_[g.index] = 0;
      }
    }
    bool alive = lib_->Responsive(h);
    if (!alive && !unresponsive_[g.index]) {
      unresponsive_[g.index] = 1;
      Notify(g.index, false, "device not responding to amdsmi");
    } else if (alive && unresponsive_[g.index]) {
      unresponsive_[g.index] = 0;
      if (!ecc_failed_[g.index]) Notify(g.index, true, "device responding again");
    }
    if (!alive) continue;
    auto ecc = lib_->UncorrectableErrors(h);
    if (ecc.ok() && *ecc > ecc_baseline_[g.index] && !ecc_failed_[g.index]) {
      ecc_failed_[g.index] = 1;
      Notify(g.index, false,
             "uncorrectable ECC errors rose to " + std::to_string(*ecc) + " (baseline " +
                 std::to_string(ecc_baseline_[g.index]) + ")");
    }
  }
}

void Monitor::Run() {
  using Clock = std::chrono::steady_clock;
  auto next_poll = Clock::now() + std::chrono::milliseconds(cfg_.poll_interval_ms);
  std::vector<smi::Event> events;
  while (!stop_.load()) {
    int slice = 500;  // bounded so Stop() is prompt; the reference waits 5000 ms per call
    if (cfg_.wait_ms > 0 && cfg_.wait_ms < slice) slice = cfg_.wait_ms;
    if (events_ok_) {
      events.clear();
      Status st = lib_->EventsWait(slice, &events);
      if (!st.ok()) {
        LOG_WARN(kComp, "event wait failed: %s", st.ToString().c_str());
        Sleep(slice);
      }
      for (const auto& e : events) {
        int gpu = -1;
        for (size_t i = 0; i < snap_->procs.size(); ++i)
          if (snap_->procs[i].handle == e.handle) gpu = snap_->GpuOfHandle(static_cast<int>(i));
        int verdict = Classify(cfg_, e.type);
        LOG_INFO(kComp, "event %s(%u) on GPU %d: %s%s", EventName(e.type), e.type, gpu,
                 e.message.c_str(), verdict == 0 ? " (ignored)" : "");
        if (gpu < 0 || verdict == 0) continue;
        if (verdict > 0) {
          // A completed reset clears poll-detected failures as well.
          unresponsive_[gpu] = 0;
          ecc_failed_[gpu] = 0;
          void* h = snap_->procs[snap_->gpus[gpu].partitions.front().handle].handle;
          auto ecc = lib_->UncorrectableErrors(h);
          if (ecc.ok()) ecc_baseline_[gpu] = *ecc;
        }
        Notify(gpu, verdict > 0, std::string(EventName(e.type)) + ": " + e.message);
      }
    } else {
      Sleep(slice);
    }
    if (cfg_.poll_interval_ms > 0 && Clock::now() >= next_poll) {
      PollOnce();
      next_poll = Clock::now() + std::chrono::milliseconds(cfg_.poll_interval_ms);
    }
  }
}

}  // namespace adp::health

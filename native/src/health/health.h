// Device health: amdsmi event pump + RAS polling, with recovery.
//
// Parity: reference cmd/nvidia-device-plugin/nvidia.go:181-294 (checkHealth):
//  * DP_DISABLE_HEALTHCHECKS: "all" or anything containing "xids" disables health
//    checking; otherwise a comma-separated list of extra IDs to ignore
//    (getAdditionalXids, nvidia.go:274-294 -- its 10 test vectors are pinned).
//  * Application errors are ignored by default (Xids 13,31,43,45,68, nvidia.go:193-199).
//  * Event wait with a 5000 ms timeout (nvidia.go:235).
//
// MI355X-native mapping (amdsmi_evt_notification_type_t):
//  * GPU_PRE_RESET (3)  -> every device of that GPU goes Unhealthy.
//  * GPU_POST_RESET (4) -> the GPU's devices go Healthy again. The reference has
//    no recovery path at all (FIXME at server.go:259, defect B15).
//  * VMFAULT (1) and THERMAL_THROTTLE (2) are application/environment events,
//    the analogue of Xid 31/43 -> ignored by default.
//  * The extra IDs in DP_DISABLE_HEALTHCHECKS are amdsmi event type numbers.
//  * If event notification is unavailable (e.g. missing permissions) the device
//    is NOT marked unhealthy (the reference does, nvidia.go:218-223, because on
//    NVIDIA that meant an ancient GPU); health falls back to polling only.
//  * Polling (every DP_HEALTH_POLL_MS, default 5000, 0 = off): a GPU that stops
//    answering amdsmi or whose uncorrectable ECC count rises goes Unhealthy; an
//    unresponsive GPU that answers again recovers.
// One Monitor per daemon generation serves all plugins (amdsmi event delivery
// is process-wide, so per-plugin pumps as in the reference would steal each
// other's events).
//
// Failure state outlives a Monitor: every restart (SIGHUP, kubelet.sock
// re-creation, config reload, re-partition, xGMI link change) builds a new
// Monitor and new Plugin objects, so the per-GPU verdicts live in a Ledger
// owned by the supervisor, keyed by GPU UUID (BDF when there is none), and --
// with --health-state-file -- in a small file that also survives a container
// restart. A new generation starts its plugins with the ledger's failures
// already applied, keeps the ECC baseline of the FIRST observation, and only a
// GPU_POST_RESET event (or a device that answers again, for "unresponsive")
// clears a failure. The reference keeps Device health only for one
// ListAndWatch lifetime (server.go:95-116,251-265) and never recovers it.
//
// Event gaps: a GPU_POST_RESET that nobody was registered to receive is lost
// for good, and a GPU whose GPU_PRE_RESET was seen would stay Unhealthy. The
// monitor therefore records every stretch in which events may have been missed
// -- a new in-process registration (each monitor generation), event waits that
// keep failing, events off, a relay that says it re-registered or could not
// replay what this daemon missed (relay.h), a first connection, or a reinit
// it leaves unanswered -- on each GPU that is waiting for its GPU_POST_RESET.
// A dropped relay connection is a tentative gap: the relay's replay on
// reconnection cancels it, and it is confirmed when the relay cannot replay or
// stays away for event_fail_ms. A GPU with a confirmed gap gets a polled
// recovery check: once amdsmi has answered at every poll for
// --reset-recovery-hold-ms since the gap -- liveness, the device's VRAM usage
// and the SMU's activity metrics, which the driver refuses mid-reset -- with no
// new GPU_PRE_RESET, it is back in service (logged,
// amdgpu_dp_gpu_recovered_without_event_total). A GPU with no gap since its
// GPU_PRE_RESET keeps waiting for the event -- or for the operator
// (--return-to-service, ApplyReturnRequests).
#pragma once

#include <atomic>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <set>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

#include "inventory/inventory.h"
#include "smi/smi.h"

namespace adp::health {

// getAdditionalXids semantics: split on ',', trim, keep valid unsigned values in order.
std::vector<uint64_t> ParseAdditionalIds(std::string_view input);
// --health-event-extra-types: comma-separated amdsmi event type numbers
// (1..13) or names ("PROCESS_START"); an error names the first bad entry.
Result<std::set<uint32_t>> ParseEventTypes(std::string_view input);
// What failure bits (FailBits) hold a GPU out, in words: "drained by the operator, ...".
std::string DescribeFailures(uint32_t bits);

struct HealthConfig {
  bool disabled = false;
  std::set<uint32_t> ignored{smi::kEvtVmFault, smi::kEvtThermalThrottle};
  int wait_ms = 5000;
  int poll_interval_ms = 5000;
  // Retired HBM pages at which a GPU is Unhealthy (DP_MAX_RETIRED_PAGES):
  // -1 = the driver's own threshold when amdsmi can read it (root), else off;
  // 0 = off; N = N pages.
  int64_t max_retired_pages = -1;
  // In-process events: how long amdsmi event waits may keep failing before
  // events count as off (ADP_EVENT_FAIL_MS; the event relay's watchdog is
  // ADP_RELAY_STUCK_MS).
  int event_fail_ms = 10000;
  // amdsmi event notification (--health-events); off = polling only.
  bool events = true;
  // --health-event-extra-types: amdsmi event types registered on top of the
  // four the monitor acts on (e.g. 12,13 = KFD PROCESS_START / PROCESS_END,
  // which any HIP process causes): counted per GPU, never a health verdict.
  std::set<uint32_t> extra_types;
  // The registration mask: GPU_PRE/POST_RESET, VMFAULT, THERMAL_THROTTLE and the extra types.
  uint64_t EventMask() const;
  // Where /dev/kfd is (--driver-root): why event registration failed.
  std::string driver_root = "/";
  // --health-event-socket: events come from the privileged relay (relay.h) at
  // this Unix socket instead of an in-process amdsmi registration ("" = in-process).
  std::string event_relay;
  // Operator drain list (--drain-file): GPUs named in it (PCI address, UUID,
  // partition UUID or node index; one or more per line, '#' comments) are
  // advertised Unhealthy until removed. Read at every poll.
  std::string drain_file;
  // A GPU waiting for GPU_POST_RESET across an event gap is back in service
  // once amdsmi has answered at every poll for this long (--reset-recovery-hold-ms;
  // 0 = never without the event).
  int64_t reset_recovery_hold_ms = 120000;
  // Reset-flap damping (--reset-flap-limit / --reset-flap-window-ms): a GPU
  // that sees this many GPU_PRE_RESETs within the window is kept out of
  // service -- its GPU_POST_RESETs notwithstanding -- until a whole window
  // passes without one. 0 = off.
  int reset_flap_limit = 3;
  int64_t reset_flap_window_ms = 600000;
  // Tests (native/tests/health_model.cc): Start() starts no thread; the
  // harness steps the monitor itself.
  bool run_thread = true;
  static HealthConfig FromEnv();
  static HealthConfig FromValues(const char* disable_value, const char* poll_ms_value);
};

using Listener = std::function<void(int gpu, bool healthy, const std::string& reason)>;

// Why a GPU is Unhealthy; a GPU is Healthy iff no bit is set.
enum FailBits : uint32_t {
  kFailEcc = 1u << 0,           // uncorrectable ECC count rose above the baseline
  kFailUnresponsive = 1u << 1,  // amdsmi stopped answering (clears when it answers)
  kFailResetPending = 1u << 2,  // GPU_PRE_RESET without a GPU_POST_RESET yet
  kFailEvent = 1u << 3,         // any other non-ignored amdsmi event
  kFailRetiredPages = 1u << 4,  // retired HBM pages reached the threshold
  kFailDrained = 1u << 5,       // listed in the operator's drain file (not a fault; cleared by removal only)
  kFailFlapping = 1u << 6,      // reset too often: quarantined until a quiet window passes (a POST_RESET does not clear it)
};

struct GpuRecord {
  bool has_baseline = false;
  uint64_t ecc_baseline = 0;  // uncorrectable count at the first observation (or last reset)
  uint64_t ecc_seen = 0;      // highest count observed since; a lower count means a counter reset
  uint32_t fail = 0;
  std::string reason;  // last failure reason (empty when healthy)
  // GPU_PRE_RESETs within the flap window (wall clock, ms since the epoch):
  // kept with the verdict, so a plugin container restart does not reset the
  // count or shorten a quarantine.
  std::vector<int64_t> resets;
  // A confirmed event gap this GPU is waiting across (why; "" = none): kept
  // with the verdict, so a process started after it -- whose own connection
  // to the relay may miss nothing -- still lets the polled check end the wait.
  std::string gap;
  // The relayed GPU_PRE_RESET last counted in `resets` ("<relay>:<seq>"; ""
  // = none or in-process): a replay of it after a restart -- the persisted
  // relay cursor lags by up to a second -- is not counted twice.
  std::string last_reset_event;
};

// The monitor's time (a test harness drives a fake one): steady for holds,
// gaps and deadlines; wall for what is persisted (the reset history).
class Clock {
 public:
  virtual ~Clock() = default;
  virtual int64_t SteadyMs() const;
  virtual int64_t WallMs() const;
  static const Clock* System();
};

// Liveness of the health machinery itself, shared by all Monitor generations
// (the metrics thread reads it while monitors come and go): whether event
// notification is registered, and how many polls / ECC reads succeeded.
struct HealthCounters {
  std::atomic<int> events_enabled{-1};  // -1 not started, 0 off, 1 on
  std::atomic<uint64_t> polls{0};
  std::atomic<uint64_t> responsive{0};       // GPU answered amdsmi in a poll
  std::atomic<uint64_t> ecc_reads_ok{0};
  std::atomic<uint64_t> ecc_read_errors{0};
  std::atomic<uint64_t> events_received{0};
  std::atomic<uint64_t> retired_reads_ok{0};
  std::atomic<uint64_t> retired_read_errors{0};
  // Steady-clock ms of the monitor loop's last iteration (0 = no monitor
  // running): a wait or amdsmi query that never returns stops it advancing,
  // which /healthz reports (HealthLoopAgeMs).
  std::atomic<int64_t> loop_beat_ms{0};
  // How long the running monitor loop has not iterated (0 when none runs).
  int64_t HealthLoopAgeMs() const;
  // Last retired-page count per GPU (by PCI address), for /metrics.
  void SetRetiredPages(const std::string& bdf, uint32_t n);
  std::map<std::string, uint32_t> RetiredPages() const;
  // Last HBM-in-use reading per GPU (bytes, all processes), for /metrics.
  void SetVramUsed(const std::string& bdf, uint64_t bytes);
  std::map<std::string, uint64_t> VramUsed() const;
  bool HasVramUsed(const std::string& bdf) const;  // readable at least once (any generation)
  // Other amdsmi queries that have answered at least once for a GPU (any generation).
  void MarkQueryOk(const std::string& bdf, const std::string& query);
  bool QueryEverOk(const std::string& bdf, const std::string& query) const;
  // HBM of each GPU (bytes, from the snapshot; set by the supervisor), next to VramUsed().
  void SetVramTotal(const std::string& bdf, uint64_t bytes);
  std::map<std::string, uint64_t> VramTotal() const;
  // amdsmi events per GPU (by PCI address) and type name, ignored ones too:
  // application VM faults and thermal throttling never change health but are
  // worth watching.
  void CountEvent(const std::string& bdf, const std::string& type);
  std::map<std::pair<std::string, std::string>, uint64_t> EventCounts() const;
  // Events on a processor that matches no enumerated one (amdsmi handed back
  // a handle it never enumerated, or the relay could not place it), by type.
  void CountUnmatched(const std::string& type);
  std::map<std::string, uint64_t> Unmatched() const;
  // Event gaps the monitor recorded (any GPU waiting for GPU_POST_RESET or not).
  std::atomic<uint64_t> event_gaps{0};
  // Relay mode: connections to the event relay that broke (it restarted, or
  // dropped a daemon that fell behind), and whether one is up now.
  std::atomic<uint64_t> relay_disconnects{0};
  std::atomic<int> relay_connected{-1};  // -1: not in relay mode
  // GPUs put back in service by the polled check after an event gap, per PCI address.
  void CountRecovered(const std::string& bdf);
  std::map<std::string, uint64_t> Recovered() const;
  // Where this daemon is in the relay's event stream, across monitor
  // generations: the relay instance, the last event sequence number handled
  // and the relay's registration generation (relay.h). Not valid until a relay
  // has answered a reinit; a new process starts without one.
  struct RelayCursor {
    bool valid = false;
    std::string relay;
    uint64_t seq = 0;
    uint64_t gen = 0;
  };
  RelayCursor GetRelayCursor() const;
  void SetRelayCursor(const RelayCursor& c);
  void AdvanceRelaySeq(uint64_t seq);
  // With --health-state-file the cursor also outlives the process (<state>.relay):
  // a restarted plugin container resumes the relay's stream where it left it,
  // and the relay replays what it missed instead of reporting a gap. Loaded
  // here; written on every hello, at once after an event that changed a
  // verdict (GPU_PRE/POST_RESET), at most once a second for the others, and
  // by FlushRelayCursor (monitor stop, connected or not). A replay of events
  // already handled would re-apply them out of turn -- a GPU_PRE_RESET the
  // operator has since returned would hold the GPU again, a GPU_POST_RESET
  // would erase a later ECC verdict (found by native/tests/health_model.cc).
  void PersistRelayCursor(const std::string& path);
  void FlushRelayCursor();
  std::string Json() const;
  // Where the cursor's save throttle reads the time (tests; default the system's).
  void SetClock(const Clock* c) { clock_ = c; }

 private:
  mutable std::mutex mu_;
  std::map<std::string, uint32_t> retired_;
  std::map<std::string, uint64_t> vram_used_, vram_total_;
  std::map<std::pair<std::string, std::string>, uint64_t> events_;
  std::map<std::string, uint64_t> recovered_, unmatched_;
  std::set<std::pair<std::string, std::string>> queries_ok_;
  RelayCursor cursor_;
  std::string cursor_path_;
  int64_t cursor_saved_ms_ = 0;
  bool cursor_dirty_ = false;
  const Clock* clock_ = Clock::System();
  void SaveCursorLocked();
};

// An event gap recorded on a GPU waiting for GPU_POST_RESET (Ledger, in memory
// only: a new process starts a gap of its own).
struct GapMark {
  int64_t since_ms = 0;  // steady clock
  std::string why;
  // The relay connection dropped: confirmed if the relay cannot replay what
  // was missed, dropped if it can.
  bool tentative = false;
  int64_t responsive_since_ms = 0;  // first poll of the current run of answered polls (0 = none yet)
};

// Per-GPU health verdicts shared by all Monitor generations of a daemon.
// Thread-safe. With a path, every change is written through (atomic rename)
// and the file is loaded at construction; a missing or unreadable file starts
// empty (logged), a malformed line is skipped.
class Ledger {
 public:
  explicit Ledger(std::string path = "");
  static std::string KeyOf(const inventory::PhysicalGpu& g) { return g.uuid.empty() ? g.bdf : g.uuid; }
  GpuRecord Get(const std::string& key) const;
  void Put(const std::string& key, const GpuRecord& r);
  std::map<std::string, GpuRecord> All() const;
  // (gpu index, reason) of every GPU of `snap` the ledger holds as failed.
  std::vector<std::pair<int, std::string>> Failed(const inventory::Snapshot& snap) const;
  const std::string& path() const { return path_; }
  // Re-reads the state file (SIGHUP): records an operator removed from it are
  // forgotten, i.e. those GPUs are Healthy again with a fresh ECC baseline.
  // No-op without a file; an unreadable file keeps the in-memory state.
  void Reload();
  // File format, exposed for tests: "adp-health v1" header, then one
  // tab-separated line per GPU: key, ecc baseline ("-" = none), highest ECC
  // count seen, fail bits, reason, and -- when there are any -- the recent
  // resets as "resets=<ms>,<ms>,..." and a confirmed event gap as "gap=<why>"
  // (fields older versions ignore).
  static std::string Serialize(const std::map<std::string, GpuRecord>& m);
  static std::map<std::string, GpuRecord> Parse(const std::string& body);

  // Event gaps (GapMark). MarkGap returns true when it created a mark or
  // confirmed a tentative one (worth a log line).
  bool MarkGap(const std::string& key, const std::string& why, bool tentative, int64_t now_ms);
  std::vector<std::string> CancelTentativeGaps();
  void ClearGap(const std::string& key);
  bool Gap(const std::string& key, GapMark* out) const;
  void SetResponsiveSince(const std::string& key, int64_t ms);
  // Reset history for flap damping (GpuRecord::resets; wall clock, so it
  // survives a restart): records a GPU_PRE_RESET at `now_ms` and returns how
  // many fall within `window_ms`. `event_id` ("<relay>:<seq>" of a relayed
  // event, "" otherwise): an event of the same relay at or before the last one
  // recorded is a replay, not recorded again. At most kMaxResetHistory are
  // kept (the newest): the count only has to reach the limit.
  static constexpr size_t kMaxResetHistory = 64;
  int RecordReset(const std::string& key, int64_t now_ms, int64_t window_ms, const std::string& event_id = "");
  // The last recorded reset (none known, e.g. a state file from an older
  // version: `now_ms` is recorded, so its quarantine lasts one more window).
  int64_t LastReset(const std::string& key, int64_t now_ms);
  void ClearResets(const std::string& key);

 private:
  void SaveLocked() const;
  mutable std::mutex mu_;
  std::map<std::string, GpuRecord> recs_;
  std::map<std::string, GapMark> gaps_;
  std::string path_;
};

// The drain file's syntax (--drain-file), shared by the monitor and the
// --drain / --undrain commands: the names in `text` (whitespace or comma
// separated, '#' starts a comment), and the names a GPU answers to there (its
// UUID, PCI address with or without the function, node index, partition UUIDs).
std::set<std::string> DrainTokens(std::string_view text);
std::set<std::string> DrainNames(const inventory::PhysicalGpu& g);
// One drain-file line without the tokens in `names`: the other names on it and
// its comment stay (a line "0,1 # maintenance" undrained of GPU 0 becomes
// "1 # maintenance"). "" when no name is left on it (the line goes).
std::string RemoveDrainNames(std::string_view line, const std::set<std::string>& names);

struct RelayLine;  // relay.h

class Monitor {
 public:
  // `ledger` / `counters` may be null: the Monitor then keeps its own.
  Monitor(smi::Library* lib, std::shared_ptr<const inventory::Snapshot> snap, HealthConfig cfg,
          Ledger* ledger = nullptr, HealthCounters* counters = nullptr);
  ~Monitor();
  void AddListener(Listener l);
  // Called once (from the monitor thread) when polling sees a GPU whose compute
  // or memory partition mode differs from the snapshot: the node was
  // re-partitioned and must be re-enumerated.
  void SetLayoutListener(std::function<void(const std::string& why)> l) { layout_listener_ = std::move(l); }
  Status Start();
  void Stop();
  bool events_enabled() const { return events_ok_.load(); }
  // Before Start(): where the monitor reads the time (tests; default the system's).
  void SetClock(const Clock* c) { clock_ = c; }

  // Decision function, exposed for tests: how an event changes a GPU's health.
  // Returns +1 (healthy), -1 (unhealthy), 0 (no change).
  static int Classify(const HealthConfig& cfg, uint32_t event_type);

 private:
  friend class MonitorTestPeer;  // native/tests/health_model.cc steps a monitor without its thread
  void Run();
  void Notify(int gpu, bool healthy, const std::string& reason);
  void PollOnce();
  // What must run whether or not polls do (DP_HEALTH_POLL_MS=0): the drain
  // file, return-to-service requests and the end of reset-flap quarantines.
  // Part of every poll, and on a timer of its own when polling is off.
  void Housekeeping();
  void EndQuarantine(int gpu);
  void LoadVerdicts();  // Start(): the verdicts, ECC baselines and retired-page thresholds of the GPUs
  // PollOnce's parts, per GPU (h: its first processor's handle). PollLayout:
  // true when the partition modes or xGMI links changed (the supervisor
  // re-enumerates); PollLiveness: whether amdsmi answers (and the polled
  // recovery and the end of a quarantine); PollRetiredPages: whether readable;
  // PollEcc: the uncorrectable count when readable.
  bool PollLayout(const inventory::PhysicalGpu& g, void* h);
  bool PollLiveness(const inventory::PhysicalGpu& g, void* h, uint64_t poll);
  bool PollRetiredPages(const inventory::PhysicalGpu& g, void* h);
  std::optional<uint64_t> PollEcc(const inventory::PhysicalGpu& g, void* h, uint64_t poll);
  // Sets/clears failure bits of a GPU, records them in the ledger and notifies
  // listeners when the GPU's overall health flips.
  void Update(int gpu, uint32_t set, uint32_t clear, const std::string& reason);
  // Applies the drain file to every GPU (PollOnce).
  void ApplyDrain();
  // Consumes the operator's return-to-service request (<drain file>.return,
  // --return-to-service): clears every failure but a drain of the GPUs named.
  void ApplyReturnRequests();
  // Records an event gap on every GPU waiting for GPU_POST_RESET.
  void MarkGap(const std::string& why, bool tentative);
  // The polled recovery check of a GPU waiting across a gap (PollOnce).
  void CheckGapRecovery(int gpu, bool alive);

  smi::Library* lib_;
  std::shared_ptr<const inventory::Snapshot> snap_;
  HealthConfig cfg_;
  std::vector<Listener> listeners_;
  std::vector<void*> handles_;
  std::atomic<bool> events_ok_{false};
  // Relay mode: the connection to the event relay (-1 = not connected), its
  // partial input line, and when a connection was last tried.
  int relay_fd_ = -1;
  std::string relay_buf_;
  bool relay_synced_ = false;  // the relay answered this connection's "reinit"
  bool relay_cursor_sent_ = false;  // the reinit named where this daemon was in the relay's events
  int64_t relay_connected_ms_ = 0;  // when this connection's reinit was sent
  bool relay_overdue_ = false;      // no answer for event_fail_ms: counted as a gap
  // Since when the relay has been out of reach (0 = connected): a tentative
  // gap is confirmed once that lasts event_fail_ms.
  int64_t relay_lost_ms_ = 0;
  bool relay_lost_confirmed_ = false;
  bool return_request_warned_ = false;
  int64_t relay_tried_ms_ = -1000000;
  // Reconnection backoff: 100 ms after a drop (a relay restart takes about that
  // long, and events it holds meanwhile die with it if it restarts again),
  // doubling to 1 s while the relay stays away.
  int relay_retry_ms_ = 100;
  std::string fingerprint_;  // ProcessorFingerprint of the snapshot, sent with "reinit"
  // In-process event waits that keep failing: since when, how many, and
  // whether events are reported off because of it.
  int64_t wait_failing_since_ms_ = 0;
  uint64_t wait_failures_ = 0;
  bool events_failing_ = false;
  void RelayConnect();
  // A connection to the relay (non-blocking socket) is this monitor's: asks
  // for the events it missed (the "reinit" line) and waits for the answer.
  void RelayAttach(int fd);
  void RelayClose(const std::string& why);
  // Reads relay lines for up to `ms`: hellos update events_ok_ and the event
  // gaps, events are mapped to this snapshot's handles and handled, in order.
  void RelayWait(int ms);
  void HandleRelayLine(const RelayLine& l);
  // The relay's deadlines: an unanswered reinit, a relay away for event_fail_ms.
  void RelayDeadlines();
  // One in-process amdsmi event wait of up to `ms` (its failures tracked as a
  // gap once they last event_fail_ms), and the events it returned.
  void InProcessWait(int ms, std::vector<smi::Event>* events);
  // One amdsmi event (in-process or relayed): counts it and updates health.
  // A null/unknown handle is an unmatched event (`unplaced`: what the relay
  // said about it); `event_id`: "<relay>:<seq>" of a relayed event.
  void HandleEvent(const smi::Event& e, const std::string& unplaced = "", const std::string& event_id = "");
  // An event on no enumerated processor: ERROR + amdgpu_dp_unmatched_events_total;
  // a GPU_PRE_RESET holds every GPU (reference nvidia.go:244-251).
  void HandleUnmatched(const smi::Event& e, int verdict, const std::string& why);
  uint64_t unmatched_seen_ = 0;  // log rate limit
  std::map<uint32_t, uint64_t> ignored_seen_;  // ignored events per type (log rate limit)
  const Clock* clock_ = Clock::System();
  int64_t SteadyNow() const { return clock_->SteadyMs(); }
  std::thread thread_;
  std::atomic<bool> stop_{false};
  std::function<void(const std::string&)> layout_listener_;
  bool layout_changed_ = false;
  int wake_fd_ = -1;  // eventfd: Stop() wakes the idle wait at once
  void Sleep(int ms);
  // Per-GPU state (mirrored into the ledger).
  Ledger own_ledger_;
  Ledger* ledger_;
  HealthCounters own_counters_;
  HealthCounters* counters_;
  std::string events_reason_;  // why event notification is off ("" when on)
  std::vector<std::string> keys_;
  std::vector<uint64_t> ecc_baseline_;
  std::vector<uint32_t> fail_;
  std::vector<int> link_change_polls_;
  std::vector<uint32_t> retired_threshold_;  // 0 = not checked
};

}  // namespace adp::health

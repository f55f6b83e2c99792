// Bounded exhaustive model check of the health state machine (round-6 review
// item 2). Run: build/native/adp_health_model [--depth N] [--mode in-process|relay|both]
//   [--extended] [--replay STEP,STEP,...] [--random WALKS --length STEPS --seed S]
//
// The reference's whole health loop is ~120 lines (nvidia.go:181-269,
// server.go:251-265): a device goes Unhealthy on an Xid and never comes back.
// Here the monitor tracks seven failure bits, tentative and confirmed event
// gaps, relay generations and cursors, flap history, drains and
// return-to-service requests, ECC baselines, persisted in four files -- too
// much state for example-based tests. This harness drives a real
// health::Monitor, without its thread, through EVERY sequence of up to
// --depth steps over a 16-symbol alphabet, in both event layouts:
//
//   PRE POST VMFAULT          an amdsmi event on GPU 0 (in-process: the fake
//                             library's queue; relay: an event line of the
//                             modelled relay, held for replay while the
//                             daemon is away)
//   POLL_OK POLL_FAIL         200 ms pass, GPU 0 answers / stops answering, a poll
//   ECC_UP ECC_RESET          GPU 0's uncorrectable count +1 / back to 0, a poll
//   RELAY_DROP                relay: the relay drops the daemon's connection
//                             (it reconnects at the next step that lets time
//                             pass); in-process: amdsmi event waits start failing
//   RELAY_RESTART             relay: a new relay instance (new ID, empty ring);
//                             in-process: event waits succeed again
//   LOST_EVENT                relay: the relay loses a GPU_POST_RESET of GPU 0 and
//                             says so (gap=1); in-process: a GPU_PRE_RESET on a
//                             processor handle amdsmi never enumerated
//   SIGHUP                    monitor stopped, ledger re-read, a new generation
//   RESTART                   container restart: monitor, ledger and counters
//                             gone, everything re-read from the state files
//   DRAIN UNDRAIN RETURN      the operator's drain file / --return-to-service for GPU 0
//   CLOCK_HOLD                --reset-recovery-hold-ms (+1) pass
//
// --extended adds (24 symbols in-process, 25 with the relay):
//   PRE1 POST1                an amdsmi event on GPU 1, which then resets too
//   UNPLACED                  relay: a GPU_PRE_RESET the relay could not place
//                             (node=- bdf=-); in-process: a GPU_POST_RESET on an
//                             unknown handle (counted, no verdict)
//   RELAY_RENEW               relay: the relay renews its registration (events
//                             keep flowing); in-process: one failing wait
//   RELAY_STUCK               relay only: the watchdog turns events off and on
//   HALF_HOLD                 half of --reset-recovery-hold-ms passes
//   ECC_UNREADABLE            GPU 0's ECC count turns unreadable / readable again
//   PRE_P1 POST_P1            the event reported by GPU 0's second compute
//                             partition (GPU 0 is DPX; KFD reports a reset on
//                             every KFD node of the GPU)
//
// against a small reference model of what the monitor must believe, given the
// events it was delivered. Invariants checked after every step:
//   I1  what the plugins advertise (the listener) = the monitor's failure bits
//       = the ledger's, for every GPU (no Unhealthy with an empty failure set,
//       no Healthy with one);
//   I2  a GPU is reset-pending exactly while the model says a delivered
//       GPU_PRE_RESET awaits its GPU_POST_RESET; it may leave that state
//       without the event only by the polled recovery, only after a confirmed
//       gap and a full hold of answered polls, and only by a poll;
//   I3  liveness: a reset-pending GPU with a confirmed gap that then answers a
//       poll, a hold, and another poll is back (lookahead run per state);
//   I4  the state file re-read (Ledger::Parse) equals the ledger in memory;
//   I5  drained exactly while the drain file names the GPU;
//   I6  GPU 1 (never the target) stays healthy, but for an unplaceable reset
//       (--extended: it may wait for its own GPU_POST_RESET and be quarantined);
//   I7  (per GPU) a reset-flap quarantine begins only with a delivered GPU_PRE_RESET and
//       ends only after a quiet window (or the operator), and does end then;
//   I8  (per GPU) the reset history never counts more resets than were
//       delivered: a GPU_PRE_RESET that finds the GPU already waiting is the
//       same reset (every partition of a GPU reports it), and a relay replay
//       counts once;
//   I9  the ECC verdict = the count rose above the baseline of the first
//       observation / the last completed reset / counter reset / operator,
//       whenever the count could be read;
//   I10 (per GPU) a new reset that makes --reset-flap-limit resets within the
//       window quarantines the GPU.
// States are deduplicated by a canonical hash (times relative to the clock,
// clamped past every threshold), so each distinct state is expanded once per
// remaining depth: every sequence up to --depth is covered. Each node is
// rebuilt by replaying its sequence from scratch (deterministic: fake clock,
// fake library, a relay modelled on relay.cc's Subscribe behind a real Unix
// socket, its ring 3 events long so that replays overflow within the bound --
// the contract tests/test_relay_protocol.py pins on the real relay).
// --random instead walks N random sequences of L steps (far past the bound),
// every step checked, each walk probed for liveness at its end.
#include <fcntl.h>
#include <poll.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <new>
#include <random>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <functional>
#include <map>
#include <memory>
#include <set>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "common/log.h"
#include "common/strings.h"
#include "health/health.h"
#include "health/relay.h"
#include "inventory/inventory.h"
#include "smi/smi.h"

namespace adp::health {

// Steps a Monitor without its thread (health.h: friend).
class MonitorTestPeer {
 public:
  static void Poll(Monitor& m) { m.PollOnce(); }
  static void Housekeeping(Monitor& m) { m.Housekeeping(); }
  static void Wait(Monitor& m) {
    std::vector<smi::Event> ev;
    if (m.events_ok_ && m.cfg_.event_relay.empty()) m.InProcessWait(0, &ev);
  }
  static void RelayRead(Monitor& m) {
    if (m.relay_fd_ >= 0) m.RelayWait(0);
  }
  static void Reconnect(Monitor& m) {
    if (m.relay_fd_ < 0) m.RelayConnect();
  }
  static void Deadlines(Monitor& m) { m.RelayDeadlines(); }
  static bool Connected(const Monitor& m) { return m.relay_fd_ >= 0; }
  static uint32_t Fail(const Monitor& m, int gpu) { return m.fail_[gpu]; }
  static uint64_t EccBaseline(const Monitor& m, int gpu) { return m.ecc_baseline_[gpu]; }
  // The monitor's own state that decides what happens next (for the state hash).
  static std::string Key(const Monitor& m, int64_t now) {
    auto rel = [&](int64_t t) { return t == 0 ? std::string("0") : std::to_string(std::min<int64_t>(4000, now - t)); };
    std::string k;
    k += m.events_ok_ ? 'E' : 'e';
    k += m.relay_fd_ >= 0 ? 'C' : 'c';
    k += m.relay_synced_ ? 'S' : 's';
    k += m.relay_cursor_sent_ ? 'U' : 'u';
    k += m.relay_overdue_ ? 'O' : 'o';
    k += m.relay_lost_confirmed_ ? 'L' : 'l';
    k += m.events_failing_ ? 'F' : 'f';
    k += "|lost=" + rel(m.relay_lost_ms_) + "|wf=" + std::to_string(std::min<uint64_t>(m.wait_failures_, 1)) + ":" +
         (m.wait_failures_ ? rel(m.wait_failing_since_ms_) : std::string("-"));
    for (size_t g = 0; g < m.fail_.size(); ++g)
      k += "|g" + std::to_string(g) + "=" + std::to_string(m.fail_[g]) + "/" + std::to_string(m.ecc_baseline_[g]);
    return k;
  }
};

}  // namespace adp::health

using namespace adp;
using health::MonitorTestPeer;

namespace {

enum Sym : int {
  A_PRE, A_POST, A_VMFAULT, A_POLL_OK, A_POLL_FAIL, A_ECC_UP, A_ECC_RESET, A_RELAY_DROP, A_RELAY_RESTART, A_LOST_EVENT, A_SIGHUP,
  A_RESTART, A_DRAIN, A_UNDRAIN, A_RETURN, A_CLOCK_HOLD, kBaseSymbols,
  // --extended: GPU 1 resets too; an unplaceable GPU_PRE_RESET from the relay
  // (in-process: an unplaceable GPU_POST_RESET); the relay renewing its
  // registration (in-process: one failing wait); the relay's watchdog turning
  // events off and on again (relay only); half a hold passing; GPU 0's ECC
  // count becoming unreadable and readable again; a reset event reported by
  // GPU 0's second compute partition (GPU 0 is DPX: KFD reports a reset on
  // each of its nodes).
  A_PRE1 = kBaseSymbols, A_POST1, A_UNPLACED, A_RELAY_RENEW, A_RELAY_STUCK, A_HALF_HOLD, A_ECC_UNREADABLE,
  A_PRE_P1, A_POST_P1, kSymbols
};
const char* kSymNames[] = {"PRE",         "POST",          "VMFAULT",      "POLL_OK",     "POLL_FAIL",
                           "ECC_UP",      "ECC_RESET",     "RELAY_DROP",   "RELAY_RESTART", "LOST_EVENT",
                           "SIGHUP",      "RESTART",       "DRAIN",        "UNDRAIN",     "RETURN",
                           "CLOCK_HOLD",  "PRE1",          "POST1",        "UNPLACED",    "RELAY_RENEW",
                           "RELAY_STUCK", "HALF_HOLD",     "ECC_UNREADABLE", "PRE_P1",      "POST_P1"};
static_assert(sizeof(kSymNames) / sizeof(kSymNames[0]) == kSymbols, "symbol names");

bool g_extended = false;  // --extended: set before the workers fork

// The symbols explored in a layout.
std::vector<int> Alphabet(bool relay, bool extended) {
  std::vector<int> a;
  for (int s = 0; s < (extended ? static_cast<int>(kSymbols) : static_cast<int>(kBaseSymbols)); ++s)
    if (relay || s != A_RELAY_STUCK) a.push_back(s);
  return a;
}

constexpr int64_t kHoldMs = 1000, kWindowMs = 2500, kEventFailMs = 500, kPollMs = 200;
constexpr int kFlapLimit = 2;
const char* kBdf[2] = {"0000:0c:00.0", "0000:2c:00.0"};

class FakeClock : public health::Clock {
 public:
  int64_t steady = 1000000, wall = 1700000000000;
  int64_t SteadyMs() const override { return steady; }
  int64_t WallMs() const override { return wall; }
  void Advance(int64_t ms) {
    steady += ms;
    wall += ms;
  }
};

// The amdsmi the monitor sees: two SPX GPUs, scripted.
class FakeSmi : public smi::Library {
 public:
  struct Gpu {
    bool alive = true;
    uint64_t ecc = 0;
  };
  Gpu gpu[2];
  char handle[3] = {0, 0, 0};  // GPU 0 partition 0, GPU 1, GPU 0 partition 1
  char foreign = 0;  // a handle amdsmi never enumerated
  bool waits_failing = false;
  bool ecc_ok = true;  // GPU 0's uncorrectable count readable
  std::set<void*> registered;
  std::deque<smi::Event> queue;        // events the kernel holds for the registration
  std::vector<smi::Event> delivered;   // what EventsWait handed out (for the model)

  int Index(void* h) const { return h == &handle[0] || h == &handle[2] ? 0 : h == &handle[1] ? 1 : -1; }
  Status EventsInit(const std::vector<void*>& hs, uint64_t) override {
    for (void* h : hs) registered.insert(h);
    return Status::Ok();
  }
  Status EventsWait(int, std::vector<smi::Event>* out) override {
    if (waits_failing) return Unavailable("amdsmi_get_gpu_event_notification failed (fake)");
    while (!queue.empty()) {
      smi::Event e = queue.front();
      queue.pop_front();
      out->push_back(e);
      delivered.push_back(e);
    }
    return Status::Ok();
  }
  void EventsStop(const std::vector<void*>& hs) override {
    for (void* h : hs) registered.erase(h);
    if (registered.empty()) queue.clear();  // the kernel's queue goes with the registration
  }
  void EventsStopAll() override {
    registered.clear();
    queue.clear();
  }
  // An event the hardware raises: held only while a registration exists.
  void Raise(void* h, uint32_t type) {
    if (!registered.empty()) queue.push_back({h, type, "fake"});
  }
  Result<uint64_t> UncorrectableErrors(void* h) override {
    int i = Index(h);
    if (i < 0 || !gpu[i].alive) return Unavailable("not answering");
    if (i == 0 && !ecc_ok) return Unavailable("ecc query failed");
    return gpu[i].ecc;
  }
  Result<uint32_t> RetiredPages(void* h) override {
    int i = Index(h);
    if (i < 0 || !gpu[i].alive) return Unavailable("not answering");
    return 0u;
  }
  Result<uint32_t> RetiredPageThreshold(void*) override { return NotSupported("needs root"); }
  Result<uint64_t> VramUsed(void* h) override {
    int i = Index(h);
    if (i < 0 || !gpu[i].alive) return Unavailable("not answering");
    return uint64_t{1} << 30;
  }
  Result<uint32_t> Activity(void* h) override {
    int i = Index(h);
    if (i < 0 || !gpu[i].alive) return Unavailable("in reset");
    return 0u;
  }
  bool Responsive(void* h) override {
    int i = Index(h);
    return i >= 0 && gpu[i].alive;
  }
  std::pair<std::string, std::string> PartitionModes(void*) override { return {"SPX", "NPS1"}; }
  int XgmiLinksDown(void*) override { return 0; }
  Status Reinit() override { return Status::Ok(); }
};

std::shared_ptr<const inventory::Snapshot> MakeSnapshot(FakeSmi* smi) {
  // GPU 0 in DPX (two compute partitions, KFD nodes 2 and 3), GPU 1 in SPX.
  std::vector<smi::ProcessorInfo> procs(3);
  for (int i = 0; i < 3; ++i) {
    const int gpu = i == 2 ? 1 : 0, part = i == 1 ? 1 : 0;
    auto& p = procs[i];
    p.handle = &smi->handle[i == 0 ? 0 : i == 1 ? 2 : 1];
    p.uuid = "75a3000" + std::to_string(gpu) + "-0000-1000-80c0-bf990789000" + std::to_string(part);
    p.bdf = std::string(kBdf[gpu]).substr(0, 11) + std::to_string(part);
    p.bdf_id = ((gpu == 0 ? 0x0cull : 0x2cull) << 8) | static_cast<uint64_t>(part);
    p.render_minor = 128 + 8 * gpu + part;
    p.numa_node = 0;
    p.vram_mib = gpu == 0 ? 294896 / 2 : 294896;
    p.compute_partition = gpu == 0 ? "DPX" : "SPX";
    p.memory_partition = "NPS1";
    p.partition_id = static_cast<uint32_t>(part);
    p.kfd_node = 2 + 8 * gpu + part;
    p.num_cu = gpu == 0 ? 128 : 256;
    p.xcd_count = gpu == 0 ? 4 : 8;
    p.market_name = "AMD Instinct MI355X";
    p.asic_serial = "0x09C0BF990789730" + std::to_string(gpu);
  }
  inventory::BuildOptions o;
  o.sysfs_root = "";
  auto s = inventory::GroupProcessors(procs, o);
  if (!s.ok()) {
    fprintf(stderr, "snapshot: %s\n", s.status().ToString().c_str());
    exit(2);
  }
  return *s;
}

std::string ReadFile(const std::string& path) {
  std::ifstream in(path, std::ios::binary);
  std::stringstream ss;
  ss << in.rdbuf();
  return ss.str();
}

void WriteFile(const std::string& path, const std::string& body) {
  FILE* f = fopen(path.c_str(), "w");
  if (f) {
    fwrite(body.data(), 1, body.size(), f);
    fclose(f);
  }
}

// The relay as relay.cc serves a daemon: numbered events held in its ring,
// the connect hello, the replay and the reinit hello of Subscribe, and the
// loss report of OnDropped.
// The relay keeps the last kRelayRingSize (1,024) events for replays; the model
// keeps 3, so that sequences within the depth bound overflow it too.
constexpr size_t kModelRing = 3;

struct RelayModel {
  int instance = 1;
  uint64_t gen = 1, seq = 0;
  std::vector<std::pair<uint64_t, std::string>> ring;
  bool lost = false;
  uint64_t lost_seq = 0;
  bool stuck = false;  // the watchdog says the amdsmi event wait hangs: events=off
  int fd = -1;  // the daemon's connection (relay side), -1: none
  std::string Id() const {
    char b[8];
    snprintf(b, sizeof(b), "a%x", instance);
    return b;
  }
  std::string Hello(bool reinit, int gap) const {
    std::string h = std::string("hello v1 ") + (reinit ? "reinit " : "") +
                    (stuck ? std::string("events=off") : std::string("events=ok processors=2")) + " relay=" + Id() +
                    " gen=" + std::to_string(gen) + " seq=" + std::to_string(seq) + " fp=- renew_ms=0";
    if (gap >= 0) h += " gap=" + std::to_string(gap);
    if (stuck) h += " reason=the amdsmi event wait has not returned for 10001 ms";
    return h + "\n";
  }
  void Send(const std::string& s) {
    if (fd < 0) return;
    if (send(fd, s.data(), s.size(), MSG_NOSIGNAL) != static_cast<ssize_t>(s.size())) {
      fprintf(stderr, "relay model: short send\n");
      exit(2);
    }
  }
  void Close() {
    if (fd >= 0) close(fd);
    fd = -1;
  }
};

struct Model {
  bool pending[2] = {false, false};      // a delivered GPU_PRE_RESET awaits its GPU_POST_RESET
  bool gap_since_pre[2] = {false, false};  // the monitor recorded a confirmed gap since it
  bool drained = false;
  // Resets since the operator's last return: the GPU_PRE_RESETs that found the
  // GPU not waiting (on a partitioned GPU every partition reports the same
  // reset: one per KFD node), with the time each was delivered.
  std::set<std::string> pre_ids[2];
  std::vector<int64_t> pre_times[2];
  bool has_baseline = false;
  uint64_t baseline = 0, seen = 0;       // GPU 0's ECC reference
};

struct Violation {
  std::string what;
};

class World {
 public:
  World(bool relay_mode, const std::string& dir) : relay_mode_(relay_mode), dir_(dir) {
    snap_ = MakeSnapshot(&smi_);
    for (int g = 0; g < 2; ++g) key_[g] = health::Ledger::KeyOf(snap_->gpus[g]);
    state_ = dir_ + "/health.state";
    drain_ = dir_ + "/drain";
    sock_ = dir_ + "/relay.sock";
    for (const auto& f : {state_, state_ + ".relay", state_ + ".tmp", state_ + ".relay.tmp", drain_,
                          drain_ + ".return", drain_ + ".return.taken"})
      unlink(f.c_str());
    if (relay_mode_) {
      unlink(sock_.c_str());
      lfd_ = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC | SOCK_NONBLOCK, 0);
      sockaddr_un a{};
      a.sun_family = AF_UNIX;
      memcpy(a.sun_path, sock_.c_str(), sock_.size());
      if (bind(lfd_, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || listen(lfd_, 8) != 0) {
        perror("relay model listen");
        exit(2);
      }
    }
    ledger_ = std::make_unique<health::Ledger>(state_);
    counters_ = std::make_unique<health::HealthCounters>();
    counters_->SetClock(&clock_);
    counters_->PersistRelayCursor(state_ + ".relay");
    StartMonitor();
    Settle();
    model_.has_baseline = true;  // LoadVerdicts' first observation
    model_.baseline = model_.seen = smi_.gpu[0].ecc;
  }
  ~World() {
    mon_.reset();
    relay_.Close();
    if (lfd_ >= 0) close(lfd_);
  }

  // One symbol; the violation text if an invariant breaks ("" = none).
  std::string Step(int sym) {
    Before before = Observe();
    smi_.delivered.clear();
    sent_.clear();
    pres_delivered_[0] = pres_delivered_[1] = 0;
    bool housekept = false, polled = false;
    const bool in_proc = !relay_mode_;
    switch (sym) {
      case A_PRE: case A_POST: case A_VMFAULT: {
        uint32_t type = sym == A_PRE ? 3 : sym == A_POST ? 4 : 1;
        if (in_proc) {
          smi_.Raise(&smi_.handle[0], type);
          MonitorTestPeer::Wait(*mon_);
        } else {
          Emit(type);
        }
        break;
      }
      case A_POLL_OK: case A_POLL_FAIL: case A_ECC_UP: case A_ECC_RESET:
        if (sym == A_POLL_OK) smi_.gpu[0].alive = true;
        if (sym == A_POLL_FAIL) smi_.gpu[0].alive = false;
        if (sym == A_ECC_UP) ++smi_.gpu[0].ecc;
        if (sym == A_ECC_RESET) smi_.gpu[0].ecc = 0;
        clock_.Advance(kPollMs);
        TimePasses();
        MonitorTestPeer::Poll(*mon_);
        polled = housekept = true;
        break;
      case A_RELAY_DROP:
        if (in_proc) {
          smi_.waits_failing = true;
          MonitorTestPeer::Wait(*mon_);
        } else if (relay_.fd >= 0) {
          relay_.Close();
          MonitorTestPeer::RelayRead(*mon_);  // EOF: the connection is gone
        }
        break;
      case A_RELAY_RESTART:
        if (in_proc) {
          smi_.waits_failing = false;
          MonitorTestPeer::Wait(*mon_);
        } else {
          relay_.Close();
          MonitorTestPeer::RelayRead(*mon_);
          const int next = relay_.instance + 1;
          relay_ = RelayModel();
          relay_.instance = next;
        }
        break;
      case A_LOST_EVENT:
        if (in_proc) {
          smi_.Raise(&smi_.foreign, 3);
          MonitorTestPeer::Wait(*mon_);
        } else {
          // The waiter could not hand the GPU_POST_RESET to the loop: no
          // number, no replay; every connected daemon is told.
          relay_.lost = true;
          relay_.lost_seq = relay_.seq;
          if (relay_.fd >= 0) {
            relay_.Send(relay_.Hello(true, 1));
            MonitorTestPeer::RelayRead(*mon_);
          }
        }
        break;
      case A_SIGHUP:
        mon_->Stop();
        DropConnection();
        ledger_->Reload();
        mon_.reset();
        StartMonitor();
        break;
      case A_RESTART:
        mon_.reset();
        DropConnection();
        counters_.reset();
        ledger_.reset();
        ledger_ = std::make_unique<health::Ledger>(state_);
        counters_ = std::make_unique<health::HealthCounters>();
        counters_->SetClock(&clock_);
        counters_->PersistRelayCursor(state_ + ".relay");
        StartMonitor();
        break;
      case A_DRAIN: case A_UNDRAIN: case A_RETURN:
        if (sym == A_DRAIN) WriteFile(drain_, std::string(kBdf[0]) + "\n");
        if (sym == A_UNDRAIN) WriteFile(drain_, "");
        if (sym == A_RETURN) WriteFile(drain_ + ".return", std::string(kBdf[0]) + "\n");
        MonitorTestPeer::Housekeeping(*mon_);
        housekept = true;
        break;
      case A_CLOCK_HOLD: case A_HALF_HOLD:
        clock_.Advance(sym == A_CLOCK_HOLD ? kHoldMs + 1 : kHoldMs / 2);
        if (relay_mode_) MonitorTestPeer::Deadlines(*mon_);
        TimePasses();
        break;
      case A_PRE1: case A_POST1:
        if (in_proc) {
          smi_.Raise(&smi_.handle[1], sym == A_PRE1 ? 3 : 4);
          MonitorTestPeer::Wait(*mon_);
        } else {
          Emit(sym == A_PRE1 ? 3 : 4, 1);
        }
        break;
      case A_PRE_P1: case A_POST_P1:
        if (in_proc) {
          smi_.Raise(&smi_.handle[2], sym == A_PRE_P1 ? 3 : 4);
          MonitorTestPeer::Wait(*mon_);
        } else {
          Emit(sym == A_PRE_P1 ? 3 : 4, 0, 1);
        }
        break;
      case A_UNPLACED:
        if (in_proc) {
          smi_.Raise(&smi_.foreign, 4);  // (the unplaceable PRE is LOST_EVENT here)
          MonitorTestPeer::Wait(*mon_);
        } else {
          Emit(3, -1);  // "node=- bdf=-"
        }
        break;
      case A_RELAY_RENEW:
        if (in_proc) {  // one wait fails, the next succeeds: no gap
          const bool was = smi_.waits_failing;
          smi_.waits_failing = true;
          MonitorTestPeer::Wait(*mon_);
          smi_.waits_failing = was;
          MonitorTestPeer::Wait(*mon_);
        } else {  // relay.cc OnRenewals "1": every subscribed daemon went without a registration
          ++relay_.gen;
          if (relay_.fd >= 0) {
            relay_.Send(relay_.Hello(true, 1));
            MonitorTestPeer::RelayRead(*mon_);
          }
        }
        break;
      case A_RELAY_STUCK:  // relay.cc Watchdog: events off (and on again), told to every daemon
        relay_.stuck = !relay_.stuck;
        if (relay_.fd >= 0) {
          relay_.Send(relay_.Hello(true, 1));
          MonitorTestPeer::RelayRead(*mon_);
        }
        break;
      case A_ECC_UNREADABLE:
        smi_.ecc_ok = !smi_.ecc_ok;
        clock_.Advance(kPollMs);
        TimePasses();
        MonitorTestPeer::Poll(*mon_);
        polled = housekept = true;
        break;
    }
    Settle();
    return Check(sym, before, polled, housekept);
  }

  // The state hash: everything that decides what happens next.
  std::string Key() const {
    const int64_t now = clock_.steady, wall = clock_.wall;
    auto relw = [&](int64_t t) { return std::to_string(std::min<int64_t>(4000, wall - t)); };
    auto rels = [&](int64_t t) { return t == 0 ? std::string("0") : std::to_string(std::min<int64_t>(4000, now - t)); };
    std::string k = MonitorTestPeer::Key(*mon_, now);
    for (int g = 0; g < 2; ++g) {
      health::GpuRecord r = ledger_->Get(key_[g]);
      k += "|r" + std::to_string(g) + ":" + (r.has_baseline ? std::to_string(r.ecc_baseline) : "-") + "/" +
           std::to_string(r.ecc_seen) + "/" + std::to_string(r.fail) + "/" + r.gap + "/" + r.last_reset_event + "/";
      std::vector<int64_t> rs = r.resets;
      std::sort(rs.begin(), rs.end());
      for (int64_t t : rs) k += relw(t) + ",";
      health::GapMark m;
      if (ledger_->Gap(key_[g], &m))
        k += "|gap" + std::to_string(g) + ":" + rels(m.since_ms) + "/" + (m.tentative ? "t" : "c") + "/" +
             rels(m.responsive_since_ms);
      k += std::string("|h") + (healthy_[g] ? "1" : "0");
      k += std::string("|m") + (model_.pending[g] ? "P" : "p") + (model_.gap_since_pre[g] ? "G" : "g");
      for (int64_t t : model_.pre_times[g]) k += "," + std::to_string(std::min<int64_t>(clock_.wall - t, kWindowMs));
    }
    k += "|smi:" + std::to_string(smi_.gpu[0].alive) + "/" + std::to_string(smi_.gpu[0].ecc) + "/" +
         std::to_string(smi_.ecc_ok) + "/" + std::to_string(smi_.waits_failing) + "/r" +
         std::to_string(smi_.registered.size()) + "/q";
    for (const auto& e : smi_.queue) k += std::to_string(smi_.Index(e.handle)) + ":" + std::to_string(e.type) + ",";
    k += "|model:" + std::to_string(model_.drained) + "/" +
         std::to_string(model_.has_baseline) + "/" + std::to_string(model_.baseline) + "/" +
         std::to_string(model_.seen);
    if (relay_mode_) {
      auto cur = counters_->GetRelayCursor();
      std::string file = ReadFile(state_ + ".relay");
      health::HealthCounters::RelayCursor fc;  // the persisted cursor (a container restart resumes from it)
      {
        auto lines = Split(file, '\n');
        auto f = lines.size() >= 2 ? Split(lines[1], '\t') : std::vector<std::string>{};
        if (f.size() == 3) fc = {true, f[0], std::stoull(f[1]), std::stoull(f[2])};
      }
      auto cursor = [&](const health::HealthCounters::RelayCursor& c) {
        if (!c.valid) return std::string("none");
        if (c.relay != relay_.Id()) return std::string("other");
        return "lag" + std::to_string(relay_.seq - c.seq) + (c.gen == relay_.gen ? "" : "g") +
               (relay_.lost && c.seq <= relay_.lost_seq ? "L" : "");
      };
      k += "|relay:" + std::to_string(relay_.fd >= 0) + (relay_.stuck ? "S" : "s") + "/mem:" + cursor(cur) +
           "/file:" + cursor(fc);
      // The events either cursor could still have replayed, and whether the
      // daemon already had each.
      uint64_t base = UINT64_MAX;
      for (const auto* c : {&cur, &fc})
        if (c->valid && c->relay == relay_.Id()) base = std::min(base, c->seq);
      for (const auto& [q, l] : relay_.ring)
        if (q > base)
          k += std::to_string(GpuOf(l)) + ":" + std::to_string(TypeOf(l)) +
               (delivered_ids_.count(relay_.Id() + ":" + std::to_string(q)) ? "d" : "n");
    }
    for (int g = 0; g < 2; ++g) {
      // resets recorded vs distinct resets delivered (I8), clamped
      const size_t rs = ledger_->Get(key_[g]).resets.size(), ids = model_.pre_ids[g].size();
      k += "|i8:" + std::to_string(std::min<size_t>(3, ids - std::min(rs, ids)));
    }
    return k;
  }

  // A reset-pending GPU with a confirmed gap, and no event still to come
  // that could legitimately start a new reset (queued in the fake library,
  // or held by the relay for a replay).
  // The GPUs (bit g) that must be back after the probe; 0 = no probe.
  int NeedsLivenessProbe() const {
    if (!smi_.queue.empty()) return 0;
    if (relay_mode_) {
      auto cur = counters_->GetRelayCursor();
      if (cur.valid && cur.relay == relay_.Id())
        for (const auto& [q, l] : relay_.ring)
          if (q > cur.seq && !delivered_ids_.count(relay_.Id() + ":" + std::to_string(q))) return 0;
    }
    int gpus = 0;
    for (int g = 0; g < 2; ++g) {
      health::GapMark m;
      // a confirmed gap in the ledger, or one the model knows there must be
      // (an unplaceable GPU_PRE_RESET)
      const bool gap = (ledger_->Gap(key_[g], &m) && !m.tentative) || (model_.pending[g] && model_.gap_since_pre[g]);
      if ((MonitorTestPeer::Fail(*mon_, g) & health::kFailResetPending) && gap) gpus |= 1 << g;
    }
    return gpus;
  }
  int ResetPending() const {
    int gpus = 0;
    for (int g = 0; g < 2; ++g)
      if (MonitorTestPeer::Fail(*mon_, g) & health::kFailResetPending) gpus |= 1 << g;
    return gpus;
  }

 private:
  struct Before {
    uint32_t fail[2];
    std::vector<int64_t> resets[2];
    bool gap_confirmed[2];
    health::GapMark gap[2];
    uint64_t recovered[2];
    int64_t steady, wall;
  };

  Before Observe() const {
    Before s{};
    auto rec = counters_->Recovered();
    for (int g = 0; g < 2; ++g) {
      s.fail[g] = ledger_->Get(key_[g]).fail | (mon_ ? MonitorTestPeer::Fail(*mon_, g) & health::kFailDrained : 0);
      s.gap_confirmed[g] = ledger_->Gap(key_[g], &s.gap[g]) && !s.gap[g].tentative;
      s.recovered[g] = rec.count(kBdf[g]) ? rec[kBdf[g]] : 0;
      s.resets[g] = ledger_->Get(key_[g]).resets;
    }
    s.steady = clock_.steady;
    s.wall = clock_.wall;
    return s;
  }

  void StartMonitor() {
    health::HealthConfig c;
    c.run_thread = false;
    c.poll_interval_ms = kPollMs;
    c.wait_ms = 0;
    c.event_fail_ms = kEventFailMs;
    c.reset_recovery_hold_ms = kHoldMs;
    c.reset_flap_limit = kFlapLimit;
    c.reset_flap_window_ms = kWindowMs;
    c.max_retired_pages = 0;
    c.drain_file = drain_;
    if (relay_mode_) c.event_relay = sock_;
    mon_ = std::make_unique<health::Monitor>(&smi_, snap_, c, ledger_.get(), counters_.get());
    mon_->SetClock(&clock_);
    // What the supervisor does before the monitor starts (PublishPlugins):
    // the plugins advertise the ledger's verdicts.
    for (int g = 0; g < 2; ++g) healthy_[g] = ledger_->Get(key_[g]).fail == 0;
    mon_->AddListener([this](int g, bool ok, const std::string&) { healthy_[g] = ok; });
    mon_->Start();
    Accept();
  }

  // The relay's side of a daemon connection: accept, greet, answer the reinit
  // (relay.cc Subscribe, with a ring that never overflows).
  void Accept() {
    if (!relay_mode_) return;
    int fd = accept4(lfd_, nullptr, nullptr, SOCK_CLOEXEC);
    if (fd < 0) return;  // the monitor did not connect
    relay_.Close();
    relay_.fd = fd;
    relay_.Send(relay_.Hello(false, -1));
    std::string line;
    char c;
    while (read(fd, &c, 1) == 1 && c != '\n') line += c;
    health::RelayRequest rq = health::ParseRelayRequest(line);
    if (rq.kind != "reinit") {
      fprintf(stderr, "relay model: expected a reinit, got '%s'\n", line.c_str());
      exit(2);
    }
    int gap = 1;
    if (rq.has_since && rq.since_relay == relay_.Id() && rq.since_seq <= relay_.seq) {
      // relay.cc Subscribe: the cursor's next event still held, and none lost after it
      bool held = rq.since_seq == relay_.seq ||
                  (!relay_.ring.empty() && relay_.ring.front().first <= rq.since_seq + 1);
      if (relay_.lost && rq.since_seq <= relay_.lost_seq) held = false;
      std::string replay;
      for (const auto& [q, l] : relay_.ring)
        if (q > rq.since_seq) {
          replay += l;
          sent_.push_back({relay_.Id() + ":" + std::to_string(q), TypeOf(l), GpuOf(l)});
        }
      relay_.Send(replay);
      gap = held && rq.since_gen == relay_.gen ? 0 : 1;
    }
    if (relay_.stuck) relay_.Send(relay_.Hello(true, 1));
    relay_.Send(relay_.Hello(true, gap));
    MonitorTestPeer::RelayRead(*mon_);
  }

  void DropConnection() {
    if (relay_mode_) relay_.Close();
  }

  // An event line of GPU `gpu`'s partition `part` (-1: unplaceable, "node=- bdf=-").
  void Emit(uint32_t type, int gpu = 0, int part = 0) {
    const uint64_t seq = ++relay_.seq;
    std::string where = gpu < 0 ? std::string("node=- bdf=-")
                                : "node=" + std::to_string(2 + 8 * gpu + part) + " bdf=" +
                                      std::string(kBdf[gpu]).substr(0, 11) + std::to_string(part);
    std::string line = "event seq=" + std::to_string(seq) + " " + where + " part=" + std::to_string(part) +
                       " type=" + std::to_string(type) + " fake\n";
    relay_.ring.emplace_back(seq, line);
    if (relay_.ring.size() > kModelRing) relay_.ring.erase(relay_.ring.begin());
    if (relay_.fd >= 0) {
      sent_.push_back({relay_.Id() + ":" + std::to_string(seq), type, gpu});
      relay_.Send(line);
      MonitorTestPeer::RelayRead(*mon_);
    }
  }

  // Time has passed: the monitor's thread would have waited for events,
  // reconnected to the relay, read it.
  void TimePasses() {
    if (relay_mode_) {
      if (!MonitorTestPeer::Connected(*mon_)) {
        MonitorTestPeer::Reconnect(*mon_);
        Accept();
      }
      MonitorTestPeer::RelayRead(*mon_);
    } else {
      MonitorTestPeer::Wait(*mon_);
    }
  }

  static uint32_t TypeOf(const std::string& line) {
    return static_cast<uint32_t>(std::stoul(line.substr(line.find("type=") + 5)));
  }
  static int GpuOf(const std::string& line) {
    return line.find(std::string("bdf=") + kBdf[1]) != std::string::npos ? 1
           : line.find("bdf=-") != std::string::npos                    ? -1
                                                                         : 0;
  }

  // Everything the monitor was handed this step, into the model, in order
  // (the relay's lines are read as soon as they are written).
  void Settle() {
    if (relay_mode_) {
      for (const auto& e : sent_) Deliver(e.gpu, e.type, e.id);
      for (const auto& e : sent_) delivered_ids_.insert(e.id);
    } else {
      for (const auto& e : smi_.delivered) {
        int g = smi_.Index(e.handle);
        Deliver(g, e.type, "local:" + std::to_string(++local_events_));
      }
    }
  }

  void Deliver(int g, uint32_t type, const std::string& id) {
    if (g < 0) {  // unplaceable: a GPU_PRE_RESET holds every GPU, each with a gap unless already waiting
      if (type != 3) return;
      for (int i = 0; i < 2; ++i)
        if (!model_.pending[i]) model_.pending[i] = model_.gap_since_pre[i] = true;
      return;
    }
    if (type == 3) {
      // A replayed event the daemon already handled is no new reset.
      if (replayed_.count(id)) return;
      replayed_.insert(id);
      if (!model_.pending[g]) {  // a new reset (not another partition's report of the one pending)
        ++pres_delivered_[g];
        model_.pre_ids[g].insert(id);
        model_.pre_times[g].push_back(clock_.wall);
      }
      model_.pending[g] = true;
      model_.gap_since_pre[g] = false;
    } else if (type == 4) {
      if (replayed_.count(id)) return;
      replayed_.insert(id);
      model_.pending[g] = false;
      model_.gap_since_pre[g] = false;
      if (smi_.gpu[g].alive && g == 0 && smi_.ecc_ok) {
        model_.has_baseline = true;
        model_.baseline = model_.seen = smi_.gpu[0].ecc;
      }
    }
  }

  std::string Check(int sym, const Before& before, bool polled, bool housekept) {
    std::string v;
    auto fail = [&](const std::string& s) {
      if (v.empty()) v = s;
    };
    // The model learns of confirmed gaps and of GPU 0's ECC observations.
    for (int g = 0; g < 2; ++g) {
      health::GapMark m;
      bool confirmed = ledger_->Gap(key_[g], &m) && !m.tentative;
      if (confirmed && model_.pending[g]) model_.gap_since_pre[g] = true;
    }
    if (sym == A_RETURN) {
      for (int g = 0; g < 1; ++g) model_.pending[g] = model_.gap_since_pre[g] = false;
      model_.pre_ids[0].clear();
      model_.pre_times[0].clear();
      if (smi_.gpu[0].alive && smi_.ecc_ok) {
        model_.has_baseline = true;
        model_.baseline = model_.seen = smi_.gpu[0].ecc;
      }
    }
    if (sym == A_DRAIN) model_.drained = true;
    if (sym == A_UNDRAIN) model_.drained = false;
    if ((polled || sym == A_SIGHUP || sym == A_RESTART) && smi_.gpu[0].alive && smi_.ecc_ok) {
      const uint64_t c = smi_.gpu[0].ecc;
      if (!model_.has_baseline) {
        model_.has_baseline = true;
        model_.baseline = model_.seen = c;
      } else if (c < model_.seen) {
        model_.baseline = model_.seen = c;
      } else if (c > model_.seen) {
        model_.seen = c;
      }
    }
    for (int g = 0; g < 2; ++g) {
      const uint32_t f = MonitorTestPeer::Fail(*mon_, g);
      const health::GpuRecord r = ledger_->Get(key_[g]);
      // I1
      if (healthy_[g] != (f == 0))
        fail("I1: GPU " + std::to_string(g) + " advertised " + (healthy_[g] ? "Healthy" : "Unhealthy") +
             " with failure bits " + std::to_string(f) + " (" + health::DescribeFailures(f) + ")");
      if ((r.fail & ~health::kFailDrained) != (f & ~health::kFailDrained))
        fail("I1: GPU " + std::to_string(g) + " ledger bits " + std::to_string(r.fail) + " != monitor bits " +
             std::to_string(f));
      // I2
      const bool pending = f & health::kFailResetPending;
      const bool was_pending = before.fail[g] & health::kFailResetPending;
      if (pending && !model_.pending[g])
        fail("I2: GPU " + std::to_string(g) + " reset-pending without a delivered GPU_PRE_RESET awaiting its POST");
      if (!pending && model_.pending[g]) {
        // Only the polled recovery may end it: a poll, after a confirmed gap
        // and a full hold of answered polls.
        const bool recovered = counters_->Recovered()[kBdf[g]] > before.recovered[g];
        if (!was_pending)
          fail("I2: GPU " + std::to_string(g) + " awaits GPU_POST_RESET (model) but was never held");
        else if (!recovered || !polled)
          fail("I2: GPU " + std::to_string(g) + " left reset-pending without GPU_POST_RESET, recovery or operator");
        else if (!model_.gap_since_pre[g] || !before.gap_confirmed[g])
          fail("I2: GPU " + std::to_string(g) + " recovered by polling with no confirmed gap since its GPU_PRE_RESET");
        else if (before.gap[g].responsive_since_ms == 0 ||
                 clock_.steady - std::max(before.gap[g].since_ms, before.gap[g].responsive_since_ms) < kHoldMs)
          fail("I2: GPU " + std::to_string(g) + " recovered before a full hold of answered polls");
        model_.pending[g] = model_.gap_since_pre[g] = false;
      }
      // I4: the state file re-read equals memory
      auto parsed = health::Ledger::Parse(ReadFile(state_));
      const auto it = parsed.find(key_[g]);
      const health::GpuRecord fr = it == parsed.end() ? health::GpuRecord{} : it->second;
      std::string reason = r.reason;
      for (auto& c : reason)
        if (c == '\t' || c == '\n' || c == '\r') c = ' ';
      std::vector<int64_t> a = r.resets, b = fr.resets;
      std::sort(a.begin(), a.end());
      std::sort(b.begin(), b.end());
      if (it == parsed.end() ? (r.fail || r.has_baseline || !r.resets.empty())
                             : (fr.fail != (r.fail & ~health::kFailDrained) || fr.has_baseline != r.has_baseline ||
                                fr.ecc_baseline != r.ecc_baseline || fr.ecc_seen != r.ecc_seen || a != b ||
                                fr.gap != r.gap || fr.last_reset_event != r.last_reset_event || fr.reason != reason))
        fail("I4: GPU " + std::to_string(g) + " state file != ledger in memory (file: " +
             health::Ledger::Serialize(parsed) + ")");
    }
    const uint32_t f0 = MonitorTestPeer::Fail(*mon_, 0), f1 = MonitorTestPeer::Fail(*mon_, 1);
    // I5
    if (model_.drained != static_cast<bool>(f0 & health::kFailDrained))
      fail(std::string("I5: drain file ") + (model_.drained ? "names" : "does not name") + " GPU 0, bits " +
           std::to_string(f0));
    // I6: the bystander GPU 1 (in --extended it resets too, so it may wait
    // for a GPU_POST_RESET and be quarantined)
    const uint32_t allowed1 = health::kFailResetPending | (g_extended ? uint32_t{health::kFailFlapping} : 0u);
    if ((f1 & ~allowed1) != 0) fail("I6: bystander GPU 1 has failure bits " + std::to_string(f1));
    // I7, per GPU
    for (int g = 0; g < 2; ++g) {
      const std::string G = "I7: GPU " + std::to_string(g) + " ";
      const uint32_t f = MonitorTestPeer::Fail(*mon_, g);
      const std::vector<int64_t>& was = before.resets[g];
      const bool flap = f & health::kFailFlapping, was_flap = before.fail[g] & health::kFailFlapping;
      const bool returned = sym == A_RETURN && g == 0;
      const int64_t last = was.empty() ? INT64_MIN : *std::max_element(was.begin(), was.end());
      const std::vector<int64_t> now = ledger_->Get(key_[g]).resets;
      if (flap && !was_flap) {
        if (pres_delivered_[g] == 0) fail(G + "quarantine began without a new GPU_PRE_RESET delivered");
        int in_window = 0;
        for (int64_t t : now) in_window += clock_.wall - t < kWindowMs;
        if (in_window < kFlapLimit) fail(G + "quarantined with " + std::to_string(in_window) + " resets in the window");
      }
      if (!flap && was_flap && !returned && !was.empty() && clock_.wall - last < kWindowMs)
        fail(G + "quarantine ended " + std::to_string(clock_.wall - last) + " ms after the last reset");
      if (flap && housekept && !returned && !was.empty()) {
        const int64_t last_now = now.empty() ? INT64_MIN : *std::max_element(now.begin(), now.end());
        if (clock_.wall - last_now >= kWindowMs) fail(G + "still quarantined after a quiet window");
      }
      // I8
      if (now.size() > model_.pre_ids[g].size())
        fail("I8: GPU " + std::to_string(g) + " " + std::to_string(now.size()) + " resets recorded for " +
             std::to_string(model_.pre_ids[g].size()) + " resets delivered");
      // I10: a new reset that makes --reset-flap-limit resets within the window
      // quarantines the GPU (counted with a step's worth of slack: the monitor
      // timestamps an event when it handles it, within the step).
      if (pres_delivered_[g] > 0) {
        int recent = 0;
        for (int64_t t : model_.pre_times[g]) recent += clock_.wall - t < kWindowMs - kHoldMs - 100;
        if (recent >= kFlapLimit && !flap)
          fail("I10: GPU " + std::to_string(g) + " had " + std::to_string(recent) +
               " resets within the window and is not quarantined");
      }
    }
    // I9 (after a poll that read the count)
    if (polled && smi_.gpu[0].alive && smi_.ecc_ok && model_.has_baseline &&
        static_cast<bool>(f0 & health::kFailEcc) != (smi_.gpu[0].ecc > model_.baseline))
      fail("I9: ECC verdict " + std::to_string(static_cast<bool>(f0 & health::kFailEcc)) + " for count " +
           std::to_string(smi_.gpu[0].ecc) + " against baseline " + std::to_string(model_.baseline));
    return v;
  }

  const bool relay_mode_;
  const std::string dir_;
  std::string state_, drain_, sock_;
  FakeSmi smi_;
  FakeClock clock_;
  std::shared_ptr<const inventory::Snapshot> snap_;
  std::string key_[2];
  std::unique_ptr<health::Ledger> ledger_;
  std::unique_ptr<health::HealthCounters> counters_;
  std::unique_ptr<health::Monitor> mon_;
  bool healthy_[2] = {true, true};
  int lfd_ = -1;
  RelayModel relay_;
  Model model_;
  struct Sent {
    std::string id;  // "<relay>:<seq>"
    uint32_t type;
    int gpu;         // -1: unplaceable
  };
  std::vector<Sent> sent_;  // relay event lines written this step
  std::set<std::string> delivered_ids_;  // every relay event the daemon was sent
  std::set<std::string> replayed_;
  int pres_delivered_[2] = {0, 0};  // new GPU_PRE_RESETs this step
  uint64_t local_events_ = 0;
};

// Shared by the worker processes (MAP_SHARED, before fork): the visited set
// -- 64-bit state hashes with the largest remaining depth each was expanded
// with -- and the counters.
struct Shared {
  std::atomic<uint64_t> next_task{0};
  std::atomic<uint64_t> distinct{0}, transitions{0}, pruned{0}, probes{0}, steps{0}, violations{0}, printed{0};
  static constexpr size_t kSlots = size_t{1} << 24;  // 128 MiB: ~5x the states of extended depth 7
  std::atomic<uint64_t> table[kSlots];
};

uint64_t Hash(const std::string& s) {
  uint64_t h = 0xcbf29ce484222325ull;  // FNV-1a, then a final mix
  for (unsigned char c : s) h = (h ^ c) * 0x100000001b3ull;
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  return h;
}

// True when the state is to be expanded: never seen, or seen with less depth left.
bool Claim(Shared* sh, const std::string& key, int remaining, bool* fresh) {
  const uint64_t h = Hash(key);
  uint64_t tag = h & ~uint64_t{0xff};
  if (!tag) tag = 0x100;
  const uint64_t want = tag | static_cast<uint64_t>(remaining + 1);
  size_t probes = 0;
  for (size_t i = (h >> 8) & (Shared::kSlots - 1);; i = (i + 1) & (Shared::kSlots - 1)) {
    if (++probes > Shared::kSlots) {
      fprintf(stderr, "health model: the state table is full (%zu slots)\n", Shared::kSlots);
      abort();
    }
    uint64_t e = sh->table[i].load();
    while (true) {
      if (e == 0) {
        if (sh->table[i].compare_exchange_weak(e, want)) {
          *fresh = true;
          return true;
        }
        continue;  // e reloaded
      }
      if ((e & ~uint64_t{0xff}) != tag) break;  // another state: next slot
      if ((e & 0xff) >= static_cast<uint64_t>(remaining + 1)) return false;
      if (sh->table[i].compare_exchange_weak(e, want)) {
        *fresh = false;
        return true;
      }
    }
  }
}

std::string Trace(const std::vector<int>& seq) {
  std::string s;
  for (int x : seq) s += std::string(s.empty() ? "" : " ") + kSymNames[x];
  return s;
}

// Replays `seq`; the violation (with the step it happened at) or "".
std::string Replay(bool relay, const std::string& dir, const std::vector<int>& seq, std::string* key, int* probe,
                   Shared* sh) {
  World w(relay, dir);
  for (size_t i = 0; i < seq.size(); ++i) {
    sh->steps.fetch_add(1, std::memory_order_relaxed);
    std::string v = w.Step(seq[i]);
    if (!v.empty()) return v + " -- after " + Trace(std::vector<int>(seq.begin(), seq.begin() + i + 1));
  }
  if (key) *key = w.Key();
  if (probe) *probe = w.NeedsLivenessProbe();
  return "";
}

void Report(Shared* sh, bool relay, const std::string& v) {
  sh->violations.fetch_add(1);
  if (sh->printed.fetch_add(1) < 20) printf("VIOLATION [%s] %s\n", relay ? "relay" : "in-process", v.c_str());
}

// I3: an answered poll, a hold, an answered poll -> the GPUs in `probe` back in service.
void Lookahead(bool relay, const std::string& dir, const std::vector<int>& seq, int probe, Shared* sh) {
  sh->probes.fetch_add(1, std::memory_order_relaxed);
  std::vector<int> look = seq;
  look.insert(look.end(), {A_POLL_OK, A_CLOCK_HOLD, A_POLL_OK});
  World w(relay, dir);
  std::string pv;
  for (size_t i = 0; i < look.size() && pv.empty(); ++i) pv = w.Step(look[i]);
  if (pv.empty() && (w.ResetPending() & probe))
    pv = "I3: a reset-pending GPU with a confirmed gap is still held after POLL_OK CLOCK_HOLD POLL_OK";
  if (!pv.empty()) Report(sh, relay, pv + " -- after " + Trace(look));
}

// --random: walks far deeper than the exhaustive bound, each checked at every
// step and probed for liveness at its end.
void RandomWalks(bool relay, const std::string& dir, uint64_t seed, int walks, int length, Shared* sh) {
  std::mt19937_64 rng(seed);
  const std::vector<int> alpha = Alphabet(relay, g_extended);
  for (int i = 0; i < walks; ++i) {
    std::vector<int> seq(static_cast<size_t>(length));
    for (auto& x : seq) x = alpha[rng() % alpha.size()];
    sh->transitions.fetch_add(1, std::memory_order_relaxed);
    int probe = 0;
    std::string v = Replay(relay, dir, seq, nullptr, &probe, sh);
    if (!v.empty()) {
      Report(sh, relay, v);
      continue;
    }
    if (probe) Lookahead(relay, dir, seq, probe, sh);
  }
}

// One node: checked, claimed, probed for liveness; true when it is to be expanded.
bool Visit(bool relay, const std::string& dir, int depth, const std::vector<int>& seq, Shared* sh) {
  sh->transitions.fetch_add(1, std::memory_order_relaxed);
  std::string key;
  int probe = 0;
  std::string v = Replay(relay, dir, seq, &key, &probe, sh);
  if (!v.empty()) {
    Report(sh, relay, v);
    return false;
  }
  const int remaining = depth - static_cast<int>(seq.size());
  bool fresh = false;
  if (!Claim(sh, std::string(relay ? "R" : "I") + key, remaining, &fresh)) {
    sh->pruned.fetch_add(1, std::memory_order_relaxed);
    return false;
  }
  if (fresh) sh->distinct.fetch_add(1, std::memory_order_relaxed);
  if (probe) Lookahead(relay, dir, seq, probe, sh);
  return remaining > 0;
}

// Depth-first below `root` (already visited and to be expanded).
void Expand(bool relay, const std::string& dir, int depth, const std::vector<int>& root, Shared* sh) {
  std::vector<std::vector<int>> stack = {root};
  while (!stack.empty()) {
    std::vector<int> seq = std::move(stack.back());
    stack.pop_back();
    for (int s : Alphabet(relay, g_extended)) {
      std::vector<int> next = seq;
      next.push_back(s);
      if (Visit(relay, dir, depth, next, sh)) stack.push_back(std::move(next));
    }
  }
}

}  // namespace

int main(int argc, char** argv) {
  int depth = 6;
  int jobs = static_cast<int>(std::min<long>(8, std::max<long>(1, sysconf(_SC_NPROCESSORS_ONLN))));
  std::string mode = "both";
  std::vector<std::string> replay;
  int walks = 0, length = 40;
  uint64_t seed = 1;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--depth") && i + 1 < argc) depth = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--jobs") && i + 1 < argc) jobs = std::max(1, atoi(argv[++i]));
    else if (!strcmp(argv[i], "--mode") && i + 1 < argc) mode = argv[++i];
    else if (!strcmp(argv[i], "--replay") && i + 1 < argc) replay = Split(argv[++i], ',');
    else if (!strcmp(argv[i], "--extended")) g_extended = true;
    else if (!strcmp(argv[i], "--random") && i + 1 < argc) walks = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--length") && i + 1 < argc) length = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--seed") && i + 1 < argc) seed = strtoull(argv[++i], nullptr, 10);
  }
  SetLogLevel(getenv("ADP_LOG_LEVEL") ? LogLevel::kInfo : LogLevel::kError);
  setvbuf(stdout, nullptr, _IOLBF, 0);
  if (!getenv("ADP_LOG_LEVEL") && replay.empty()) {  // the monitor's ERROR lines: thousands of them
    int devnull = open("/dev/null", O_WRONLY | O_CLOEXEC);
    if (devnull >= 0) dup2(devnull, 2);
  }
  char tmpl[] = "/dev/shm/adp-health-model-XXXXXX";
  const char* root = mkdtemp(tmpl);
  if (!root) {
    perror("mkdtemp");
    return 2;
  }
  const std::string dir = root;
  std::vector<bool> modes;
  if (mode != "relay") modes.push_back(false);
  if (mode != "in-process") modes.push_back(true);
  int rc = 0;
  auto* sh = static_cast<Shared*>(
      mmap(nullptr, sizeof(Shared), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0));
  if (sh == MAP_FAILED) {
    perror("mmap");
    return 2;
  }
  new (sh) Shared();
  if (!replay.empty()) {  // one sequence, logged: --replay PRE,SIGHUP,...
    std::vector<int> seq;
    for (const auto& n : replay) {
      int sym = -1;
      for (int s = 0; s < kSymbols; ++s)
        if (n == kSymNames[s]) sym = s;
      if (sym < 0) {
        fprintf(stderr, "unknown step '%s'\n", n.c_str());
        rmdir(dir.c_str());
        return 2;
      }
      if (sym >= kBaseSymbols) g_extended = true;  // a step of the extended alphabet: its invariants
      seq.push_back(sym);
    }
    for (bool relay : modes) {
      std::string v = Replay(relay, dir, seq, nullptr, nullptr, sh);
      printf("%s: %s\n", relay ? "relay" : "in-process", v.empty() ? "ok" : v.c_str());
      rc |= !v.empty();
    }
  } else if (walks > 0) {  // --random N --length L [--seed S]
    auto t0 = std::chrono::steady_clock::now();
    std::vector<pid_t> kids;
    for (int j = 0; j < jobs; ++j) {
      pid_t pid = fork();
      if (pid == 0) {
        const std::string wdir = dir + "/w" + std::to_string(j);
        mkdir(wdir.c_str(), 0700);
        const int mine = walks / jobs + (j < walks % jobs ? 1 : 0);
        for (size_t m = 0; m < modes.size(); ++m)
          RandomWalks(modes[m], wdir, seed * 1000003 + static_cast<uint64_t>(j) * 17 + m, mine, length, sh);
        for (const char* f : {"health.state", "health.state.relay", "health.state.tmp", "health.state.relay.tmp",
                              "drain", "drain.return", "drain.return.taken", "relay.sock"})
          unlink((wdir + "/" + f).c_str());
        rmdir(wdir.c_str());
#ifdef ADP_COVERAGE
        exit(0);
#else
        _exit(0);
#endif
      }
      if (pid > 0) kids.push_back(pid);
    }
    for (pid_t k : kids) {
      int status = 0;
      waitpid(k, &status, 0);
      if (!WIFEXITED(status) || WEXITSTATUS(status) != 0) {
        printf("worker %d failed (status %d)\n", static_cast<int>(k), status);
        rc = 1;
      }
    }
    double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("health model: %s%s, %d random walks of %d steps per layout (seed %llu), %d workers: %llu monitor steps, "
           "%llu liveness probes in %.1f s: %llu violation(s)\n",
           mode.c_str(), g_extended ? " (extended)" : "", walks, length, static_cast<unsigned long long>(seed), jobs,
           static_cast<unsigned long long>(sh->steps.load()), static_cast<unsigned long long>(sh->probes.load()), secs,
           static_cast<unsigned long long>(sh->violations.load()));
    rc |= sh->violations.load() != 0;
  } else {
    auto t0 = std::chrono::steady_clock::now();
    // Depth 1 here; every (first, second) pair below it is a task the workers
    // pull from a shared counter, each expanding its subtree depth first.
    std::vector<std::pair<bool, std::vector<int>>> tasks;
    for (bool relay : modes)
      for (int s : Alphabet(relay, g_extended))
        if (Visit(relay, dir, depth, {s}, sh))
          for (int s2 : Alphabet(relay, g_extended)) tasks.push_back({relay, {s, s2}});
    std::vector<pid_t> kids;
    for (int j = 0; j < jobs; ++j) {
      pid_t pid = fork();
      if (pid == 0) {
        const std::string wdir = dir + "/w" + std::to_string(j);
        mkdir(wdir.c_str(), 0700);
        for (uint64_t t; (t = sh->next_task.fetch_add(1)) < tasks.size();) {
          const auto& [relay, seq] = tasks[t];
          if (Visit(relay, wdir, depth, seq, sh)) Expand(relay, wdir, depth, seq, sh);
        }
        for (const char* f : {"health.state", "health.state.relay", "health.state.tmp", "health.state.relay.tmp",
                              "drain", "drain.return", "drain.return.taken", "relay.sock"})
          unlink((wdir + "/" + f).c_str());
        rmdir(wdir.c_str());
#ifdef ADP_COVERAGE
        exit(0);  // gcov writes this worker's counts at exit
#else
        _exit(0);
#endif
      }
      if (pid > 0) kids.push_back(pid);
    }
    for (pid_t k : kids) {
      int status = 0;
      waitpid(k, &status, 0);
      if (!WIFEXITED(status) || WEXITSTATUS(status) != 0) {
        printf("worker %d failed (status %d)\n", static_cast<int>(k), status);
        rc = 1;
      }
    }
    double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    double all = 0;
    std::string sizes;
    for (bool relay : modes) {
      const size_t k = Alphabet(relay, g_extended).size();
      double n = 1;
      for (int i = 0; i < depth; ++i) all += (n *= static_cast<double>(k));
      sizes += (sizes.empty() ? "" : "/") + std::to_string(k);
    }
    printf("health model: %s%s, depth %d, %s symbols, %d workers: all %.0f sequences of 1..%d steps covered by %llu "
           "distinct states (%llu transitions, %llu pruned as seen, %llu liveness probes, %llu monitor steps) in "
           "%.1f s: %llu violation(s)\n",
           mode.c_str(), g_extended ? " (extended)" : "", depth, sizes.c_str(), jobs, all, depth, static_cast<unsigned long long>(sh->distinct.load()),
           static_cast<unsigned long long>(sh->transitions.load()), static_cast<unsigned long long>(sh->pruned.load()),
           static_cast<unsigned long long>(sh->probes.load()), static_cast<unsigned long long>(sh->steps.load()), secs,
           static_cast<unsigned long long>(sh->violations.load()));
    rc |= sh->violations.load() != 0;
  }
  for (const char* f : {"health.state", "health.state.relay", "health.state.tmp", "health.state.relay.tmp", "drain",
                        "drain.return", "drain.return.taken", "relay.sock"})
    unlink((dir + "/" + f).c_str());
  rmdir(dir.c_str());
  munmap(sh, sizeof(Shared));
  return rc;
}

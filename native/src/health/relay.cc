// The event relay process (--event-relay): the amdsmi registration and its
// waiter, the registrar, the scan worker and the loop serving daemons. The
// protocol and the client side are relay_protocol.cc.
#include "health/relay.h"

#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <sys/signalfd.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "common/log.h"
#include "common/strings.h"
#include "inventory/inventory.h"
#include "memcap/driver_usage.h"

namespace adp::health {
namespace {

constexpr const char* kComp = "event-relay";

// Every event type the daemon classifies (health.cc Classify), and the
// relay's --health-event-extra-types.
uint64_t RelayMask(uint64_t extra) {
  return smi::EventMask(smi::kEvtGpuPreReset) | smi::EventMask(smi::kEvtGpuPostReset) |
         smi::EventMask(smi::kEvtVmFault) | smi::EventMask(smi::kEvtThermalThrottle) | extra;
}

std::string OneLine(std::string s) {
  for (char& c : s)
    if (c == '\n' || c == '\r') c = ' ';
  return s;
}

int64_t NowMs() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

bool SendAll(int fd, const std::string& s) {
  size_t off = 0;
  while (off < s.size()) {
    ssize_t n = send(fd, s.data() + off, s.size() - off, MSG_NOSIGNAL);
    if (n < 0 && errno == EINTR) continue;
    if (n <= 0) return false;  // a daemon that does not read is dropped, never waited for
    off += static_cast<size_t>(n);
  }
  return true;
}

// 16 hex digits from /dev/urandom (time and PID if it cannot be read).
std::string RandomId() {
  uint64_t v = 0;
  int fd = open("/dev/urandom", O_RDONLY | O_CLOEXEC);
  if (fd < 0 || read(fd, &v, sizeof(v)) != static_cast<ssize_t>(sizeof(v)))
    v = static_cast<uint64_t>(NowMs()) * 0x9e3779b97f4a7c15ull ^ static_cast<uint64_t>(getpid());
  if (fd >= 0) close(fd);
  char buf[17];
  snprintf(buf, sizeof(buf), "%016llx", static_cast<unsigned long long>(v));
  return buf;
}

// Scans run on their own thread: a walk of every /proc/<pid>/fd can take
// seconds on a busy node, and events must not wait for it. Requests beyond a
// few queued ones are refused (the connection closes; the daemon retries on
// its next poll).
class ScanWorker {
 public:
  explicit ScanWorker(const RelayOptions& o) : opts_(o), thread_([this] { Run(); }) {
    state_.full_walk_ms = memcap::FullWalkMsFromEnv();
  }
  ~ScanWorker() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    thread_.join();
    for (auto& r : queue_) close(r.fd);
  }
  // Takes ownership of `fd`.
  void Submit(int fd, std::string usage_dir, std::string cgroup) {
    std::lock_guard<std::mutex> lk(mu_);
    if (queue_.size() >= 4) {
      LOG_WARN(kComp, "scan request refused: %zu already queued", queue_.size());
      close(fd);
      return;
    }
    queue_.push_back({fd, std::move(usage_dir), std::move(cgroup)});
    cv_.notify_one();
  }

 private:
  struct Request {
    int fd;
    std::string usage_dir, cgroup;
  };
  void Run() {
    for (;;) {
      Request r;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !queue_.empty(); });
        if (stop_) return;
        r = std::move(queue_.front());
        queue_.pop_front();
      }
      // One ScanState for every daemon's requests: the periodic full walk and
      // the render-only holders it found are the node's, not a connection's.
      memcap::DriverScan s = memcap::ScanDriverHbm(opts_.proc_root, memcap::ListGrantFiles(r.usage_dir), r.cgroup,
                                                   opts_.kfd_proc_dir, &state_);
      if (s.pid_source == "proc" && s.render_only && !render_only_logged_) {
        render_only_logged_ = true;
        LOG_WARN(kComp, "%zu process(es) hold HBM through a render node without /dev/kfd (not in KFD's process "
                 "list): read on every scan from now on, and a full walk every %lld ms finds new ones",
                 s.render_only, static_cast<long long>(state_.full_walk_ms));
      }
      if (!logged_) {
        logged_ = true;
        LOG_INFO(kComp, "first HBM scan for a daemon: %zu process(es) from %s, %zu descriptor(s), %zu unreadable",
                 s.pids_scanned, s.pid_source == "kfd" ? opts_.kfd_proc_dir.c_str() : opts_.proc_root.c_str(),
                 s.fd_entries, s.fd_dirs_unreadable);
        // A node has hundreds of processes; a handful means this /proc is the
        // relay container's own PID namespace, where no pod's process is seen.
        if (s.pid_source == "proc" && s.pids_scanned < 5)
          LOG_WARN(kComp, "only %zu process(es) under %s: is the host's /proc mounted there (--host-proc)? Other "
                   "pods' HBM is not seen", s.pids_scanned, opts_.proc_root.c_str());
      }
      // The reply is written blocking, bounded: a daemon that stops reading loses it.
      fcntl(r.fd, F_SETFL, fcntl(r.fd, F_GETFL) & ~O_NONBLOCK);
      timeval tv{5, 0};
      setsockopt(r.fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
      SendAll(r.fd, memcap::SerializeScan(s));
      close(r.fd);
    }
  }
  RelayOptions opts_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Request> queue_;
  bool stop_ = false;
  bool logged_ = false;
  bool render_only_logged_ = false;
  memcap::ScanState state_;  // only the scan thread touches it
  std::thread thread_;
};

// The amdsmi side of the relay: the processors, their event registration, the
// thread that waits for events (writing each as a line to `event_fd`), and
// the registrar thread that renews the registration when a daemon's view of
// the processors differs from it. None of it runs on the poll loop: a
// re-enumeration (amdsmi shut_down + init) takes as long as the driver makes
// it, and greetings, scans and event forwarding do not wait for it. Renewals
// end with a "done <client> <renewed 0|1>" line on `done_fd`.
class Registration {
 public:
  struct State {
    bool ok = false;
    std::string reason;     // events off: why
    size_t processors = 0;
    uint64_t gen = 0;       // renewals so far (each one a stretch without a registration)
    std::string fp;         // ProcessorFingerprint of the registered processors ("" = none)
    int64_t renew_ms = 0;   // how long the last renewal took
  };

  Registration(smi::Library* lib, std::string driver_root, uint64_t mask, int event_fd, int done_fd, int64_t stuck_ms)
      : lib_(lib), driver_root_(std::move(driver_root)), mask_(mask), event_fd_(event_fd), done_fd_(done_fd),
        stuck_ms_(stuck_ms),
        // The wait's slice (an event ends the wait at once): short, because a
        // renewal must wait for the slice to end before it can stop the waiter;
        // and well under the watchdog's threshold. Idle, that is ~10 wake-ups/s
        // at 0.02% of a core (profiles/r4/idle/).
        slice_ms_(static_cast<int>(std::max<int64_t>(10, std::min<int64_t>(100, stuck_ms / 4)))) {}

  State Get() const {
    std::lock_guard<std::mutex> lk(mu_);
    return state_;
  }
  bool running() const { return running_.load(); }
  // How long the running waiter has been inside one amdsmi wait.
  int64_t SilentMs() const { return running_.load() ? NowMs() - beat_ms_.load() : 0; }
  // How long waits have kept failing (each failure is followed by 100 ms of rest).
  int64_t FailingMs() const { return running_.load() ? static_cast<int64_t>(wait_failures_.load()) * 100 : 0; }
  bool Hung() const { return SilentMs() > stuck_ms_; }
  // Events the waiter could not hand to the poll loop (its pipe full) since
  // the last call: they are in no daemon's stream and in no replay.
  uint64_t TakeDropped() { return dropped_.exchange(0); }

  // Enumerates (after amdsmi shut_down + init when `reinit`), registers every
  // processor and starts the waiter. Only the registrar thread calls it.
  void Renew(bool reinit) {
    const int64_t t0 = NowMs();
    StopWaiter();
    // Every registration the library holds, whether the last renewal
    // completed or not (it undoes a partial one itself).
    lib_->EventsStopAll();
    registered_ = false;
    handles_.clear();
    procs_.clear();
    State s = Get();
    ++s.gen;
    s.ok = false;
    s.processors = 0;
    s.fp.clear();
    Status st = reinit ? lib_->Reinit() : Status::Ok();
    if (!st.ok()) {
      s.reason = "amdsmi re-initialisation failed: " + OneLine(st.ToString());
    } else if (auto en = lib_->Enumerate(); !en.ok()) {
      s.reason = "enumeration failed: " + OneLine(en.status().ToString());
    } else {
      procs_ = std::move(*en);
      for (const auto& p : procs_) handles_.push_back(p.handle);
      s.processors = procs_.size();
      s.fp = ProcessorFingerprint(procs_);
      st = lib_->EventsInit(handles_, mask_);
      registered_ = st.ok();
      s.ok = st.ok();
      s.reason.clear();
      if (!st.ok()) {
        s.reason = OneLine(st.ToString());
        if (inventory::KfdAccessErrno(driver_root_) == EPERM)
          s.reason += "; /dev/kfd not openable (EPERM) in the relay's container: run the relay privileged";
      }
    }
    s.renew_ms = NowMs() - t0;
    {
      std::lock_guard<std::mutex> lk(mu_);
      state_ = s;
    }
    if (s.ok)
      LOG_INFO(kComp, "event notification registered on %zu processor(s) (generation %llu, %s%lld ms)", s.processors,
               static_cast<unsigned long long>(s.gen), reinit ? "amdsmi re-initialised, " : "",
               static_cast<long long>(s.renew_ms));
    else if (s.processors)
      LOG_ERROR(kComp, "event notification unavailable: %s", s.reason.c_str());
    else
      LOG_ERROR(kComp, "events=off reason=%s", s.reason.c_str());
    StartWaiter();
  }

  // Starts the registrar thread: the first registration, then Request()s.
  // The poll loop runs meanwhile -- a scan or a greeting does not wait for
  // amdsmi (~100 ms on the MI355X); a daemon's reinit is answered after it.
  void StartRegistrar() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      state_.reason = "registering event notification";
    }
    registrar_ = std::thread([this] {
      Renew(false);
      RegistrarLoop();
      registrar_exited_.store(true);
    });
  }
  // A daemon (client `id`) subscribed with its fingerprint ("" = none given).
  void Request(uint64_t id, std::string fp) {
    std::lock_guard<std::mutex> lk(req_mu_);
    requests_.push_back({id, std::move(fp)});
    req_cv_.notify_one();
  }

  // Ends the registrar (after the renewal it may be in) and the registration.
  // Returns false when the waiter is stuck in amdsmi: it is left running and
  // this object must outlive it (the process is about to exit).
  bool Shutdown() {
    {
      std::lock_guard<std::mutex> lk(req_mu_);
      req_stop_ = true;
    }
    req_cv_.notify_all();
    // A renewal stopping a waiter that is stuck in amdsmi never ends: exit
    // without it rather than hang the container's shutdown. (Polled: no timed
    // condition-variable wait, which this toolchain's TSan cannot follow.)
    const int64_t deadline = NowMs() + stuck_ms_ + slice_ms_ + 1000;
    while (registrar_.joinable() && !registrar_exited_.load() && NowMs() < deadline) usleep(10000);
    if (registrar_.joinable() && !registrar_exited_.load()) {
      LOG_WARN(kComp, "exiting with a registration renewal stuck in amdsmi");
      registrar_.detach();
      return false;
    }
    if (registrar_.joinable()) registrar_.join();
    if (Hung()) {
      LOG_WARN(kComp, "exiting with the event wait still stuck");
      waiter_.detach();
      return false;
    }
    StopWaiter();
    lib_->EventsStopAll();
    registered_ = false;
    return true;
  }

 private:
  void RegistrarLoop() {
    for (;;) {
      std::pair<uint64_t, std::string> r;
      {
        std::unique_lock<std::mutex> lk(req_mu_);
        req_cv_.wait(lk, [&] { return req_stop_ || !requests_.empty(); });
        if (req_stop_) return;
        r = std::move(requests_.front());
        requests_.pop_front();
      }
      State cur = Get();
      bool renewed = false;
      if (Hung()) {
        // amdsmi cannot be re-initialised under a wait that does not return:
        // the daemon gets the current (events off) state instead.
        LOG_WARN(kComp, "re-enumeration a daemon asked for skipped: the event wait is stuck");
      } else if (r.second.empty() || r.second != cur.fp || !cur.ok || wait_failures_.load() > 0) {
        LOG_INFO(kComp, "re-enumerating (a daemon asked: %s)",
                 r.second.empty()        ? "no processor fingerprint given"
                 : r.second != cur.fp    ? ("its processors " + r.second + " differ from the registration's " +
                                         (cur.fp.empty() ? std::string("(none)") : cur.fp)).c_str()
                 : !cur.ok               ? "events are off"
                                         : "the event wait is failing");
        Renew(true);
        renewed = true;
      } else {
        LOG_INFO(kComp, "registration kept (a daemon's processors match it: %s, generation %llu)", cur.fp.c_str(),
                 static_cast<unsigned long long>(cur.gen));
      }
      std::string line = "done " + std::to_string(r.first) + (renewed ? " 1\n" : " 0\n");
      if (write(done_fd_, line.data(), line.size()) != static_cast<ssize_t>(line.size()))
        LOG_WARN(kComp, "renewal result not delivered to the poll loop");
    }
  }

  void StartWaiter() {
    if (!registered_) return;
    wait_failures_.store(0);  // a fresh registration: earlier failures say nothing about it
    beat_ms_.store(NowMs());
    waiter_stop_.store(false);
    running_.store(true);
    waiter_ = std::thread([this] {
      std::vector<smi::Event> events;
      while (!waiter_stop_.load()) {
        events.clear();
        beat_ms_.store(NowMs());
        Status st = lib_->EventsWait(slice_ms_, &events);
        beat_ms_.store(NowMs());
        if (!st.ok()) {
          int n = wait_failures_.fetch_add(1) + 1;
          if (n == 1 || n % 600 == 0)  // the first, then one a minute
            LOG_WARN(kComp, "event wait failed (%d in a row): %s", n, st.ToString().c_str());
          usleep(100000);
          continue;
        }
        wait_failures_.store(0);
        for (const auto& e : events) {
          const smi::ProcessorInfo* p = nullptr;
          for (const auto& q : procs_)
            if (q.handle == e.handle) p = &q;
          if (!p) {
            // A handle amdsmi never enumerated: forwarded unplaced ("node=-
            // bdf=-"), and each daemon applies its rule for those (a
            // GPU_PRE_RESET holds every GPU); never dropped silently.
            const uint64_t n = unmatched_.fetch_add(1) + 1;
            if (e.type == smi::kEvtGpuPreReset || n <= 10 || n % 1000 == 0)
              LOG_ERROR(kComp, "event %s(%u) on a processor handle amdsmi did not enumerate (%llu so far): forwarded "
                        "unplaced", smi::EventTypeName(e.type).c_str(), e.type, static_cast<unsigned long long>(n));
          }
          std::string line = p ? FormatRelayEvent(*p, e.type, e.message) : FormatUnplacedRelayEvent(e.type, e.message);
          bool refused = false;
#ifdef ADP_TEST_HOOKS
          refused = !drop_event_.empty() && line.find(drop_event_) != std::string::npos;
#endif
          if (refused || write(event_fd_, line.data(), line.size()) != static_cast<ssize_t>(line.size())) {
            LOG_ERROR(kComp, "event dropped (relay loop behind): %s", OneLine(line).c_str());
            dropped_.fetch_add(1);  // the poll loop tells the daemons (within a second)
          }
        }
      }
    });
  }
  void StopWaiter() {
    if (!waiter_.joinable()) return;
    waiter_stop_.store(true);
    waiter_.join();
    running_.store(false);
  }

  smi::Library* lib_;
  const std::string driver_root_;
  const uint64_t mask_;
  const int event_fd_, done_fd_;
  const int64_t stuck_ms_;
  const int slice_ms_;
  // Owned by whichever thread runs Renew (never two at once); the waiter
  // reads procs_ and only runs while they do not change.
  std::vector<smi::ProcessorInfo> procs_;
  std::vector<void*> handles_;
  bool registered_ = false;
  std::thread waiter_;
  std::atomic<bool> waiter_stop_{false};
  std::atomic<bool> running_{false};
  std::atomic<int64_t> beat_ms_{0};    // the waiter's last sign of life
  std::atomic<int> wait_failures_{0};  // consecutive failed waits
  std::atomic<uint64_t> dropped_{0};    // events the pipe refused (TakeDropped)
  std::atomic<uint64_t> unmatched_{0};  // events on handles amdsmi never enumerated
#ifdef ADP_TEST_HOOKS
  const std::string drop_event_ = [] {  // test hook: refuse event lines containing it
    const char* e = getenv("ADP_DEBUG_RELAY_REFUSE_EVENT");
    return std::string(e ? e : "");
  }();
#endif
  mutable std::mutex mu_;
  State state_;
  std::thread registrar_;
  std::mutex req_mu_;
  std::condition_variable req_cv_;
  std::deque<std::pair<uint64_t, std::string>> requests_;
  bool req_stop_ = false;
  std::atomic<bool> registrar_exited_{false};
};

// A Registration a stuck thread still uses at exit: deliberately kept, and
// reachable (not a leak to LeakSanitizer).
Registration* volatile g_abandoned = nullptr;

// The relay's socket server: one poll() loop over the signals, the listening
// socket, the two pipes (event lines from the waiter, renewal results from
// the registrar) and the connected daemons. It answers a daemon at once;
// nothing it does waits for amdsmi.
class RelayServer {
 public:
  RelayServer(smi::Library* lib, const RelayOptions& opts)
      : lib_(lib), opts_(opts), stuck_ms_(EnvMs("ADP_RELAY_STUCK_MS", 10000)), relay_id_(RandomId()),
#ifdef ADP_TEST_HOOKS
        drop_on_(Env("ADP_DEBUG_RELAY_DROP_ON")),
#endif
        scans_(opts) {}
  ~RelayServer() {
    for (auto& c : clients_)
      if (c.fd >= 0) close(c.fd);
    for (int fd : {ev_pipe_[0], done_pipe_[0], lfd_})
      if (fd >= 0) close(fd);
  }

  // Binds the socket (owner-only) and starts the registration; false: logged.
  bool Open(const std::string& socket_path) {
    sockaddr_un addr{};
    socket_path_ = socket_path;
    lfd_ = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC | SOCK_NONBLOCK, 0);
    addr.sun_family = AF_UNIX;
    memcpy(addr.sun_path, socket_path.c_str(), socket_path.size());
    unlink(socket_path.c_str());
    mode_t old = umask(0077);  // owner-only: only the daemon's uid (root, same pod) may connect
    int rc = lfd_ < 0 ? -1 : bind(lfd_, reinterpret_cast<sockaddr*>(&addr), sizeof(addr));
    umask(old);
    if (rc != 0 || listen(lfd_, 8) != 0) {
      LOG_ERROR(kComp, "cannot listen on %s: %s", socket_path.c_str(), strerror(errno));
      return false;
    }
    if (pipe2(ev_pipe_, O_CLOEXEC | O_NONBLOCK) != 0 || pipe2(done_pipe_, O_CLOEXEC | O_NONBLOCK) != 0) {
      LOG_ERROR(kComp, "pipe: %s", strerror(errno));
      for (int* p : {ev_pipe_, done_pipe_})
        for (int i : {0, 1})
          if (p[i] >= 0) close(p[i]), p[i] = -1;
      return false;
    }
    // Heap-held: a waiter stuck in amdsmi at exit keeps using it (Shutdown).
    reg_ = new Registration(lib_, opts_.driver_root, RelayMask(opts_.extra_mask), ev_pipe_[1], done_pipe_[1], stuck_ms_);
    reg_->StartRegistrar();
    LOG_INFO(kComp, "relaying amdsmi events on %s (relay %s)", socket_path.c_str(), relay_id_.c_str());
    return true;
  }

  // Serves until a terminating signal; then ends the registration.
  int Run(int signal_fd) {
    bool quit = false;
    while (!quit) {
      std::vector<pollfd> pfds = {
          {signal_fd, POLLIN, 0}, {lfd_, POLLIN, 0}, {ev_pipe_[0], POLLIN, 0}, {done_pipe_[0], POLLIN, 0}};
      constexpr size_t kFixed = 4;  // signals, listener, event pipe, renewal pipe
      for (const auto& c : clients_) pfds.push_back({c.fd, POLLIN, 0});
      int timeout = static_cast<int>(std::min<int64_t>(1000, stuck_ms_ / 2 + 1));
      if (poll(pfds.data(), pfds.size(), timeout) < 0 && errno != EINTR) break;
      Watchdog();
      if (pfds[2].revents & POLLIN) OnEvents();
      OnDropped();
      if (pfds[3].revents & POLLIN) OnRenewals();
      if (pfds[0].revents & POLLIN) {
        signalfd_siginfo si;
        while (read(signal_fd, &si, sizeof(si)) == sizeof(si))
          if (si.ssi_signo != SIGHUP && si.ssi_signo != SIGUSR1) quit = true;
      }
      // Only the clients polled above (accept below appends new ones).
      for (size_t i = 0; i + kFixed < pfds.size(); ++i)
        if (clients_[i].fd >= 0 && (pfds[kFixed + i].revents & (POLLIN | POLLHUP | POLLERR))) OnClient(clients_[i]);
      if (pfds[1].revents & POLLIN) Accept();
      clients_.erase(std::remove_if(clients_.begin(), clients_.end(), [](const Client& c) { return c.fd < 0; }),
                     clients_.end());
    }
    if (reg_->Shutdown()) {
      delete reg_;
      close(ev_pipe_[1]);
      close(done_pipe_[1]);
    } else {
      // A thread stuck in amdsmi still uses it and the pipes' write ends; the
      // process exits next.
      g_abandoned = reg_;
    }
    unlink(socket_path_.c_str());
    LOG_INFO(kComp, "event relay stopped");
    return 0;
  }

 private:
  struct Client {
    int fd;
    std::string in;
    uint64_t id;
    bool subscribed = false;  // sent its reinit: gets events and reinit hellos
    int gap = 1;              // what its reinit hello says, unless the registration is renewed
  };

  static std::string Env(const char* name) {
    const char* e = getenv(name);
    return e ? e : "";
  }
  static int64_t EnvMs(const char* name, int64_t dflt) {
    const char* e = getenv(name);
    return e && atoll(e) > 0 ? static_cast<int64_t>(atoll(e)) : dflt;
  }

  std::string Hello(bool reinit, int gap) const {
    Registration::State s = reg_->Get();
    bool ok = s.ok && !stuck_;
    std::string h = std::string("hello v1 ") + (reinit ? "reinit " : "") +
                    (ok ? "events=ok processors=" + std::to_string(s.processors) : std::string("events=off")) +
                    " relay=" + relay_id_ + " gen=" + std::to_string(s.gen) + " seq=" + std::to_string(seq_) +
                    " fp=" + (s.fp.empty() ? std::string("-") : s.fp) + " renew_ms=" + std::to_string(s.renew_ms);
    if (gap >= 0) h += " gap=" + std::to_string(gap);
    if (!ok) h += " reason=" + (stuck_ ? stuck_reason_ : s.reason);
    return h + "\n";
  }
  static void SendTo(Client& c, const std::string& s) {
    if (c.fd >= 0 && !SendAll(c.fd, s)) {
      close(c.fd);
      c.fd = -1;
    }
  }
  void Broadcast(const std::string& s) {
    for (auto& c : clients_)
      if (c.subscribed) SendTo(c, s);
  }

  // Watchdog: an amdsmi wait that has not returned (or has kept failing) for
  // stuck_ms_ means events are not being delivered; the daemons are told (a
  // "reinit" hello with events=off, so they poll) and told again when the
  // wait returns.
  void Watchdog() {
    if (!reg_->running()) return;
    int64_t silent = reg_->SilentMs();
    // A wait that keeps failing delivers no more events than one that hangs.
    int64_t failing_ms = reg_->FailingMs();
    if (!stuck_ && (silent > stuck_ms_ || failing_ms > stuck_ms_)) {
      stuck_ = true;
      stuck_reason_ = silent > stuck_ms_
                          ? "the amdsmi event wait has not returned for " + std::to_string(silent) + " ms"
                          : "the amdsmi event wait has failed for " + std::to_string(failing_ms) + " ms";
      LOG_ERROR(kComp, "events=off reason=%s: daemons fall back to polling", stuck_reason_.c_str());
      Broadcast(Hello(true, 1));
    } else if (stuck_ && silent <= stuck_ms_ && failing_ms <= stuck_ms_) {
      stuck_ = false;
      LOG_INFO(kComp, "the amdsmi event wait returned again: events back on");
      Broadcast(Hello(true, 1));
    }
  }

  // Event lines from the waiter: numbered, held for replays, forwarded.
  void OnEvents() {
    char buf[4096];
    ssize_t n;
    while ((n = read(ev_pipe_[0], buf, sizeof(buf))) > 0) pending_.append(buf, static_cast<size_t>(n));
    std::string out;
    size_t nl;
    while ((nl = pending_.find('\n')) != std::string::npos) {
      // "event node=..." -> "event seq=<n> node=...", held for replays
      std::string line = "event seq=" + std::to_string(++seq_) + pending_.substr(5, nl - 4);
      pending_.erase(0, nl + 1);
      ring_.emplace_back(seq_, line);
      if (ring_.size() > kRelayRingSize) ring_.pop_front();
      out += line;
    }
    if (out.empty()) return;
    // Every reset line is logged; other events (a workload's VM-fault storm,
    // KFD's per-process events) the first hundred batches, then every
    // thousandth -- the daemons count each.
    const bool resets = out.find(" type=3 ") != std::string::npos || out.find(" type=4 ") != std::string::npos;
    if (resets || ++batches_logged_ <= 100 || batches_logged_ % 1000 == 0)
      LOG_INFO(kComp, "%s", OneLine(out).c_str());
#ifdef ADP_TEST_HOOKS
    if (!drop_on_.empty() && out.find(drop_on_) != std::string::npos) {
      // Tests: what a daemon whose socket buffer is full sees -- dropped,
      // the events it missed held in the ring for its reconnection.
      for (auto& c : clients_)
        if (c.subscribed && c.fd >= 0) {
          close(c.fd);
          c.fd = -1;
        }
      LOG_WARN(kComp, "every daemon connection dropped (ADP_DEBUG_RELAY_DROP_ON)");
      return;
    }
#endif
    Broadcast(out);
  }

  // Events the waiter dropped are in no daemon's stream and no replay: every
  // subscribed daemon is told it may have missed events (a confirmed gap: it
  // polls its waiting GPUs back), and so is one that reconnects later with a
  // cursor from before the loss.
  void OnDropped() {
    const uint64_t n = reg_->TakeDropped();
    if (!n) return;
    lost_ = true;
    lost_seq_ = seq_;
    LOG_ERROR(kComp, "%llu event(s) lost after #%llu: daemons are told they may have missed events",
              static_cast<unsigned long long>(n), static_cast<unsigned long long>(seq_));
    Broadcast(Hello(true, 1));
  }

  // "done <client> <renewed 0|1>" from the registrar.
  void OnRenewals() {
    char buf[512];
    ssize_t n;
    while ((n = read(done_pipe_[0], buf, sizeof(buf))) > 0) done_pending_.append(buf, static_cast<size_t>(n));
    size_t nl;
    while ((nl = done_pending_.find('\n')) != std::string::npos) {
      auto f = Split(std::string_view(done_pending_).substr(0, nl), ' ');
      done_pending_.erase(0, nl + 1);
      if (f.size() != 3) continue;
      if (f[2] == "1") {
        // Renewed: every subscribed daemon went without a registration meanwhile.
        Broadcast(Hello(true, 1));
      } else {
        auto id = ParseUint(f[1]);
        for (auto& c : clients_)
          if (id && c.id == *id) SendTo(c, Hello(true, c.gap));
      }
    }
  }

  // "reinit fp=<fp> since=<relay>:<seq>:<gen>": replay what the daemon missed,
  // decide whether it can have missed anything, and pass the fingerprint on.
  void Subscribe(Client& c, RelayRequest& rq) {
    int gap = 1;
    if (rq.has_since && rq.since_relay == relay_id_ && rq.since_seq <= seq_) {
      const uint64_t s = rq.since_seq;
      bool held = s == seq_ || (!ring_.empty() && ring_.front().first <= s + 1);
      if (lost_ && s <= lost_seq_) held = false;  // it was away when events were lost
      std::string replay;
      size_t n = 0;
      for (const auto& [q, l] : ring_)
        if (q > s) {
          replay += l;
          ++n;
        }
      if (n) {
        LOG_INFO(kComp, "replaying %zu event(s) after #%llu to a reconnected daemon%s", n,
                 static_cast<unsigned long long>(s), held ? "" : " (older ones are no longer held)");
        SendTo(c, replay);
      }
      gap = held && rq.since_gen == reg_->Get().gen ? 0 : 1;
    }
    c.subscribed = true;
    c.gap = gap;
    LOG_INFO(kComp, "daemon connected for events (%s)",
             rq.has_since ? (gap ? "it may have missed events" : "nothing missed") : "a new daemon");
    // The watchdog's events=off stands whatever the registrar answers (and a
    // registrar renewing under a stuck wait may never answer): say so now.
    if (stuck_) SendTo(c, Hello(true, 1));
    reg_->Request(c.id, std::move(rq.fp));
  }

  // A daemon's request lines: a reinit subscribes it; a scan takes the
  // connection over.
  void OnClient(Client& c) {
    char buf[256];
    ssize_t n = recv(c.fd, buf, sizeof(buf), 0);
    if (n <= 0) {
      if (n < 0 && (errno == EAGAIN || errno == EINTR)) return;
      close(c.fd);
      c.fd = -1;
      return;
    }
    c.in.append(buf, static_cast<size_t>(n));
    if (c.in.size() > 4096) {  // nothing legitimate is that long
      close(c.fd);
      c.fd = -1;
      return;
    }
    size_t nl;
    while (c.fd >= 0 && (nl = c.in.find('\n')) != std::string::npos) {
      RelayRequest rq = ParseRelayRequest(std::string_view(c.in.data(), nl));
      if (rq.kind == "reinit") Subscribe(c, rq);
      if (rq.kind == "scan") {
        // The connection becomes the scan's.
        if (rq.malformed) {
          LOG_WARN(kComp, "malformed scan request dropped");
          close(c.fd);
        } else {
          scans_.Submit(c.fd, std::move(rq.usage_dir), std::move(rq.cgroup));
        }
        c.fd = -1;
        return;
      }
      c.in.erase(0, nl + 1);
    }
  }

  void Accept() {
    int cfd;
    while ((cfd = accept4(lfd_, nullptr, nullptr, SOCK_CLOEXEC | SOCK_NONBLOCK)) >= 0) {
      // Only this relay's own uid (the plugin container runs as the same
      // root) -- the socket's mode says so already; the kernel's peer
      // credentials make sure.
      ucred cred{};
      socklen_t clen = sizeof(cred);
      if (getsockopt(cfd, SOL_SOCKET, SO_PEERCRED, &cred, &clen) != 0 || cred.uid != geteuid()) {
        LOG_WARN(kComp, "connection from uid %u refused", static_cast<unsigned>(cred.uid));
        close(cfd);
        continue;
      }
      if (!SendAll(cfd, Hello(false, -1))) {
        close(cfd);
        continue;
      }
      clients_.push_back({cfd, "", next_id_++});
      // (a scan connection every poll: not worth an info line each)
      LOG_DEBUG(kComp, "connection accepted (%zu client(s))", clients_.size());
    }
  }

  smi::Library* lib_;
  const RelayOptions opts_;
  const int64_t stuck_ms_;
  const std::string relay_id_;
#ifdef ADP_TEST_HOOKS
  const std::string drop_on_;  // test hook (ADP_DEBUG_RELAY_DROP_ON)
#endif
  std::string socket_path_;
  int lfd_ = -1;
  int ev_pipe_[2] = {-1, -1}, done_pipe_[2] = {-1, -1};
  Registration* reg_ = nullptr;
  ScanWorker scans_;
  std::vector<Client> clients_;
  uint64_t next_id_ = 1;
  // The last kRelayRingSize events forwarded, for daemons that reconnect.
  std::deque<std::pair<uint64_t, std::string>> ring_;
  uint64_t seq_ = 0;
  bool lost_ = false;      // events were dropped (OnDropped) ...
  uint64_t lost_seq_ = 0;  // ... after this one: a cursor at or before it missed them
  bool stuck_ = false;
  std::string stuck_reason_;
  std::string pending_, done_pending_;  // bytes read from the pipes, up to the last full line
  uint64_t batches_logged_ = 0;          // event batches without a reset (log rate limit)
};

}  // namespace

int RunEventRelay(smi::Library* lib, const std::string& socket_path, int signal_fd, const RelayOptions& opts) {
  if (socket_path.empty() || socket_path.size() >= sizeof(sockaddr_un{}.sun_path)) {
    LOG_ERROR(kComp, "--event-relay needs --health-event-socket (a path shorter than %zu bytes)",
              sizeof(sockaddr_un{}.sun_path));
    return 1;
  }
  RelayServer server(lib, opts);
  if (!server.Open(socket_path)) return 1;
  return server.Run(signal_fd);
}

}  // namespace adp::health

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

// Every event type the daemon classifies (health.cc Classify).
uint64_t RelayMask() {
  return smi::EventMask(smi::kEvtGpuPreReset) | smi::EventMask(smi::kEvtGpuPostReset) |
         smi::EventMask(smi::kEvtVmFault) | smi::EventMask(smi::kEvtThermalThrottle);
}

std::string OneLine(std::string s) {
  for (char& c : s)
    if (c == '\n' || c == '\r') c = ' ';
  return s;
}

// Value of "key=value" (up to the next space) in `line`, "" if absent.
std::string_view Kv(std::string_view line, std::string_view key, size_t* end = nullptr) {
  for (size_t b = 0; b < line.size();) {
    size_t e = line.find(' ', b);
    if (e == std::string_view::npos) e = line.size();
    std::string_view tok = line.substr(b, e - b);
    if (tok.size() > key.size() && tok.compare(0, key.size(), key) == 0 && tok[key.size()] == '=') {
      if (end) *end = e;
      return tok.substr(key.size() + 1);
    }
    b = e + 1;
  }
  return {};
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

// Scans run on their own thread: a walk of every /proc/<pid>/fd can take
// seconds on a busy node, and events must not wait for it. Requests beyond a
// few queued ones are refused (the connection closes; the daemon retries on
// its next poll).
class ScanWorker {
 public:
  explicit ScanWorker(const RelayOptions& o) : opts_(o), thread_([this] { Run(); }) {}
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
      memcap::DriverScan s = memcap::ScanDriverHbm(opts_.proc_root, memcap::ListGrantFiles(r.usage_dir), r.cgroup,
                                                   opts_.kfd_proc_dir);
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
  std::thread thread_;
};

}  // namespace

RelayLine ParseRelayLine(std::string_view line) {
  RelayLine r;
  while (!line.empty() && (line.back() == '\n' || line.back() == '\r')) line.remove_suffix(1);
  if (line.rfind("hello ", 0) == 0) {
    r.kind = "hello";
    r.events_ok = Kv(line, "events") == "ok";
    r.after_reinit = line.rfind("hello v1 reinit ", 0) == 0;
    size_t at = line.find(" reason=");
    if (at != std::string_view::npos) r.reason = std::string(line.substr(at + 8));
    return r;
  }
  if (line.rfind("event ", 0) != 0) return r;
  size_t end = 0, last = 0;
  std::string_view node = Kv(line, "node", &end);
  last = std::max(last, end);
  r.bdf = std::string(Kv(line, "bdf", &end));
  last = std::max(last, end);
  auto part = ParseUint(std::string(Kv(line, "part", &end)));
  last = std::max(last, end);
  auto type = ParseUint(std::string(Kv(line, "type", &end)));
  last = std::max(last, end);
  if (!part || !type || *type > 0xffffffffu || *part > 0xffffffffu) return r;
  if (node != "-") {
    auto n = ParseUint(std::string(node));
    if (!n || *n >= 0xffffffffu) return r;
    r.node = static_cast<uint32_t>(*n);
  }
  r.part = static_cast<uint32_t>(*part);
  r.type = static_cast<uint32_t>(*type);
  if (last < line.size()) r.message = std::string(line.substr(last + 1));
  r.kind = "event";
  return r;
}

std::string FormatRelayEvent(const smi::ProcessorInfo& p, uint32_t type, const std::string& message) {
  return "event node=" + (p.kfd_node == 0xffffffffu ? std::string("-") : std::to_string(p.kfd_node)) +
         " bdf=" + (p.bdf.empty() ? std::string("-") : p.bdf) + " part=" + std::to_string(p.partition_id) +
         " type=" + std::to_string(type) + " " + OneLine(message) + "\n";
}

int ConnectRelay(const std::string& socket_path) {
  sockaddr_un addr{};
  if (socket_path.empty() || socket_path.size() >= sizeof(addr.sun_path)) return -1;
  int fd = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) return -1;
  addr.sun_family = AF_UNIX;
  memcpy(addr.sun_path, socket_path.c_str(), socket_path.size());
  if (connect(fd, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0) {
    close(fd);
    return -1;
  }
  fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK);
  return fd;
}

int PingRelay(const std::string& socket_path, int timeout_ms) {
  int fd = ConnectRelay(socket_path);
  if (fd < 0) {
    printf("event relay at %s not reachable: %s\n", socket_path.c_str(), strerror(errno));
    return 1;
  }
  std::string in;
  auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  size_t nl;
  while ((nl = in.find('\n')) == std::string::npos) {
    int left = static_cast<int>(
        std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now()).count());
    pollfd p{fd, POLLIN, 0};
    if (left <= 0 || poll(&p, 1, left) <= 0) break;
    char buf[512];
    ssize_t n = recv(fd, buf, sizeof(buf), 0);
    if (n <= 0) break;
    in.append(buf, static_cast<size_t>(n));
  }
  close(fd);
  if (nl == std::string::npos) {
    printf("event relay at %s did not greet within %d ms\n", socket_path.c_str(), timeout_ms);
    return 1;
  }
  RelayLine l = ParseRelayLine(std::string_view(in).substr(0, nl));
  printf("%s\n", in.substr(0, nl).c_str());
  if (l.kind != "hello") return 1;
  // a hung or failing event wait: a restart (amdsmi initialised afresh) is the fix
  return l.reason.find("has not returned") != std::string::npos || l.reason.find("has failed for") != std::string::npos
             ? 1
             : 0;
}

int RunEventRelay(smi::Library* lib, const std::string& socket_path, int signal_fd, const RelayOptions& opts) {
  const std::string& driver_root = opts.driver_root;
  sockaddr_un addr{};
  if (socket_path.empty() || socket_path.size() >= sizeof(addr.sun_path)) {
    LOG_ERROR(kComp, "--event-relay needs --health-event-socket (a path shorter than %zu bytes)",
              sizeof(addr.sun_path));
    return 1;
  }
  int lfd = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC | SOCK_NONBLOCK, 0);
  addr.sun_family = AF_UNIX;
  memcpy(addr.sun_path, socket_path.c_str(), socket_path.size());
  unlink(socket_path.c_str());
  mode_t old = umask(0077);  // owner-only: only the daemon's uid (root, same pod) may connect
  int rc = lfd < 0 ? -1 : bind(lfd, reinterpret_cast<sockaddr*>(&addr), sizeof(addr));
  umask(old);
  if (rc != 0 || listen(lfd, 8) != 0) {
    LOG_ERROR(kComp, "cannot listen on %s: %s", socket_path.c_str(), strerror(errno));
    if (lfd >= 0) close(lfd);
    return 1;
  }

  std::vector<smi::ProcessorInfo> procs;
  std::vector<void*> handles;
  std::string events_state;  // the hello line's tail
  bool registered = false;   // event notification is registered on `handles`
  auto enumerate_and_register = [&](bool reinit) {
    if (registered) lib->EventsStop(handles);
    registered = false;
    handles.clear();
    procs.clear();
    if (reinit) {
      if (Status st = lib->Reinit(); !st.ok()) {
        events_state = "events=off reason=amdsmi re-initialisation failed: " + OneLine(st.ToString());
        LOG_ERROR(kComp, "%s", events_state.c_str());
        return;
      }
    }
    auto en = lib->Enumerate();
    if (!en.ok()) {
      events_state = "events=off reason=enumeration failed: " + OneLine(en.status().ToString());
      LOG_ERROR(kComp, "%s", events_state.c_str());
      return;
    }
    procs = std::move(*en);
    for (const auto& p : procs) handles.push_back(p.handle);
    Status st = lib->EventsInit(handles, RelayMask());
    registered = st.ok();
    std::string why = st.ok() ? "" : OneLine(st.ToString());
    if (int kerr = st.ok() ? 0 : inventory::KfdAccessErrno(driver_root); kerr == EPERM)
      why += "; /dev/kfd not openable (EPERM) in the relay's container: run the relay privileged";
    events_state = st.ok() ? "events=ok processors=" + std::to_string(procs.size()) : "events=off reason=" + why;
    if (st.ok()) LOG_INFO(kComp, "event notification registered on %zu processor(s)", procs.size());
    else LOG_ERROR(kComp, "event notification unavailable: %s", st.ToString().c_str());
  };
  // The amdsmi wait blocks (≤100 ms slices), so it runs on a thread of its
  // own and hands formatted lines to the main loop through a pipe: the main
  // loop sleeps in poll() on sockets, signals and that pipe, and answers a
  // daemon's request at once. Re-enumeration stops the thread first (it reads
  // `procs`, which only the main thread changes, and only then).
  int pipefd[2];
  if (pipe2(pipefd, O_CLOEXEC | O_NONBLOCK) != 0) {
    LOG_ERROR(kComp, "pipe: %s", strerror(errno));
    close(lfd);
    return 1;
  }
  // Watchdog: an amdsmi wait that has not returned for kStuckMs means events
  // are not being delivered; the daemons are told (a "reinit" hello with
  // events=off, so they poll) and told again when the wait returns.
  const int64_t kStuckMs = [] {
    const char* e = getenv("ADP_RELAY_STUCK_MS");
    return e && atoll(e) > 0 ? static_cast<int64_t>(atoll(e)) : int64_t{10000};
  }();
  // The wait's slice (an event ends the wait at once): short, because
  // re-enumeration -- every daemon (re)start asks for one -- must wait for the
  // slice to end before it can stop the waiter; and well under the watchdog's
  // threshold. Idle, that is ~10 wake-ups/s at 0.02% of a core (profiles/r4/idle/).
  const int wait_slice_ms = static_cast<int>(std::max<int64_t>(10, std::min<int64_t>(100, kStuckMs / 4)));
  std::atomic<bool> waiter_stop{false};
  std::atomic<int64_t> beat_ms{0};  // the waiter's last sign of life (steady clock)
  std::atomic<int> wait_failures{0};  // consecutive failed waits
  auto now_ms = [] {
    return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
  };
  std::thread waiter;
  auto start_waiter = [&] {
    if (!registered) return;
    waiter_stop.store(false);
    wait_failures.store(0);  // a fresh registration: earlier failures say nothing about it
    beat_ms.store(now_ms());
    waiter = std::thread([&] {
      std::vector<smi::Event> events;
      while (!waiter_stop.load()) {
        events.clear();
        beat_ms.store(now_ms());
        Status st = lib->EventsWait(wait_slice_ms, &events);
        beat_ms.store(now_ms());
        if (!st.ok()) {
          int n = wait_failures.fetch_add(1) + 1;
          if (n == 1 || n % 600 == 0)  // the first, then one a minute
            LOG_WARN(kComp, "event wait failed (%d in a row): %s", n, st.ToString().c_str());
          usleep(100000);
          continue;
        }
        wait_failures.store(0);
        for (const auto& e : events) {
          const smi::ProcessorInfo* p = nullptr;
          for (const auto& q : procs)
            if (q.handle == e.handle) p = &q;
          if (!p) continue;
          std::string line = FormatRelayEvent(*p, e.type, e.message);
          if (write(pipefd[1], line.data(), line.size()) != static_cast<ssize_t>(line.size()))
            LOG_WARN(kComp, "event dropped (relay loop behind): %s", OneLine(line).c_str());
        }
      }
    });
  };
  auto stop_waiter = [&] {
    if (!waiter.joinable()) return;
    waiter_stop.store(true);
    waiter.join();
  };
  enumerate_and_register(false);
  start_waiter();
  LOG_INFO(kComp, "relaying amdsmi events on %s", socket_path.c_str());

  struct Client {
    int fd;
    std::string in;
  };
  std::vector<Client> clients;
  ScanWorker scans(opts);
  auto hello = [&]() { return "hello v1 " + events_state + "\n"; };
  int exit_code = 0;
  bool quit = false;
  std::string pending;  // event bytes read from the pipe, up to the last full line

  bool stuck = false;
  std::string state_before_stuck;
  auto broadcast = [&](const std::string& line) {
    for (auto& c : clients)
      if (c.fd >= 0 && !SendAll(c.fd, line)) {
        close(c.fd);
        c.fd = -1;
      }
  };
  while (!quit) {
    std::vector<pollfd> pfds = {{signal_fd, POLLIN, 0}, {lfd, POLLIN, 0}, {pipefd[0], POLLIN, 0}};
    for (const auto& c : clients) pfds.push_back({c.fd, POLLIN, 0});
    int timeout = waiter.joinable() ? static_cast<int>(std::min<int64_t>(1000, kStuckMs / 2 + 1)) : -1;
    if (poll(pfds.data(), pfds.size(), timeout) < 0 && errno != EINTR) break;
    if (waiter.joinable()) {
      int64_t silent = now_ms() - beat_ms.load();
      // A wait that keeps failing delivers no more events than one that hangs.
      int64_t failing_ms = static_cast<int64_t>(wait_failures.load()) * 100;
      if (!stuck && (silent > kStuckMs || failing_ms > kStuckMs)) {
        stuck = true;
        state_before_stuck = events_state;
        events_state = silent > kStuckMs
                           ? "events=off reason=the amdsmi event wait has not returned for " + std::to_string(silent) +
                                 " ms"
                           : "events=off reason=the amdsmi event wait has failed for " + std::to_string(failing_ms) +
                                 " ms";
        LOG_ERROR(kComp, "%s: daemons fall back to polling", events_state.c_str());
        broadcast("hello v1 reinit " + events_state + "\n");
      } else if (stuck && silent <= kStuckMs && failing_ms <= kStuckMs) {
        stuck = false;
        events_state = state_before_stuck;
        LOG_INFO(kComp, "the amdsmi event wait returned again: events back on");
        broadcast("hello v1 reinit " + events_state + "\n");
      }
    }
    if (pfds[2].revents & POLLIN) {
      char buf[4096];
      ssize_t n;
      while ((n = read(pipefd[0], buf, sizeof(buf))) > 0) pending.append(buf, static_cast<size_t>(n));
      size_t cut = pending.rfind('\n');
      if (cut != std::string::npos) {
        std::string lines = pending.substr(0, cut + 1);
        pending.erase(0, cut + 1);
        LOG_INFO(kComp, "%s", OneLine(lines).c_str());
        broadcast(lines);
      }
    }
    if (pfds[0].revents & POLLIN) {
      signalfd_siginfo si;
      while (read(signal_fd, &si, sizeof(si)) == sizeof(si))
        if (si.ssi_signo != SIGHUP && si.ssi_signo != SIGUSR1) quit = true;
    }
    if (pfds[1].revents & POLLIN) {
      int cfd;
      while ((cfd = accept4(lfd, nullptr, nullptr, SOCK_CLOEXEC | SOCK_NONBLOCK)) >= 0) {
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
        if (!SendAll(cfd, hello())) {
          close(cfd);
          continue;
        }
        clients.push_back({cfd, ""});
        // (a scan connection every poll: not worth an info line each)
        LOG_DEBUG(kComp, "connection accepted (%zu client(s))", clients.size());
      }
    }
    bool do_reinit = false;
    // Only the clients polled above (accept may have appended new ones).
    constexpr size_t kFixed = 3;  // signals, listener, event pipe
    const size_t polled = pfds.size() - kFixed;
    for (size_t i = 0; i < polled; ++i) {
      auto& c = clients[i];
      if (c.fd < 0 || !(pfds[kFixed + i].revents & (POLLIN | POLLHUP | POLLERR))) continue;
      char buf[256];
      ssize_t n = recv(c.fd, buf, sizeof(buf), 0);
      if (n <= 0) {
        if (n < 0 && (errno == EAGAIN || errno == EINTR)) continue;
        close(c.fd);
        c.fd = -1;
        continue;
      }
      c.in.append(buf, static_cast<size_t>(n));
      if (c.in.size() > 4096) {  // nothing legitimate is that long
        close(c.fd);
        c.fd = -1;
        continue;
      }
      size_t nl;
      while (c.fd >= 0 && (nl = c.in.find('\n')) != std::string::npos) {
        std::string_view line(c.in.data(), nl);
        if (line == "reinit") {
          do_reinit = true;
          LOG_INFO(kComp, "daemon connected for events");
        }
        if (line.rfind("scan\t", 0) == 0) {
          // "scan\t<usage dir>\t<cgroup>": the connection becomes the scan's.
          size_t tab = line.find('\t', 5);
          std::string_view dir = tab == std::string_view::npos ? std::string_view() : line.substr(5, tab - 5);
          // An absolute directory without "..": the relay stats its entries, nothing more.
          if (dir.empty() || dir[0] != '/' || dir.find("/..") != std::string_view::npos) {
            LOG_WARN(kComp, "malformed scan request dropped");
            close(c.fd);
          } else {
            scans.Submit(c.fd, std::string(line.substr(5, tab - 5)), std::string(line.substr(tab + 1)));
          }
          c.fd = -1;
          break;
        }
        c.in.erase(0, nl + 1);
      }
    }
    clients.erase(std::remove_if(clients.begin(), clients.end(), [](const Client& c) { return c.fd < 0; }),
                  clients.end());
    const bool hung = waiter.joinable() && now_ms() - beat_ms.load() > kStuckMs;
    if (do_reinit) {
      if (hung) {
        // amdsmi cannot be re-initialised under a wait that does not return:
        // the daemon gets the current (events off) state instead.
        LOG_WARN(kComp, "re-enumeration a daemon asked for skipped: the event wait is stuck");
      } else {
        LOG_INFO(kComp, "re-enumerating (a daemon asked)");
        stop_waiter();
        enumerate_and_register(true);
        start_waiter();
      }
      // Marked, so a daemon tells the state after its own request from the
      // hello every connection gets first (sent before the request was read).
      broadcast("hello v1 reinit " + events_state + "\n");
    }
  }
  if (waiter.joinable() && now_ms() - beat_ms.load() > kStuckMs) {
    // Joining would wait on the hung call; the process is about to exit.
    LOG_WARN(kComp, "exiting with the event wait still stuck");
    waiter.detach();
  } else {
    stop_waiter();
    if (!handles.empty() && registered) lib->EventsStop(handles);
  }
  for (auto& c : clients)
    if (c.fd >= 0) close(c.fd);
  close(pipefd[0]);
  close(pipefd[1]);
  close(lfd);
  unlink(socket_path.c_str());
  LOG_INFO(kComp, "event relay stopped");
  return exit_code;
}

}  // namespace adp::health

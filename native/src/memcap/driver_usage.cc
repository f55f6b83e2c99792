#include "memcap/driver_usage.h"

#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/sysmacros.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <set>
#include <tuple>

#include "common/log.h"

namespace adp::memcap {
namespace {

constexpr const char* kComp = "driver-hbm";

bool IsPid(const char* name) {
  if (!*name) return false;
  for (const char* p = name; *p; ++p)
    if (*p < '0' || *p > '9') return false;
  return true;
}

// Small bounded read of a /proc file (fdinfo, cgroup): never blocks, never
// follows a link out of /proc.
std::string ReadSmall(const std::string& path, size_t max = 16384) {
  int fd = open(path.c_str(), O_RDONLY | O_CLOEXEC | O_NONBLOCK);
  if (fd < 0) return "";
  std::string out;
  char buf[4096];
  ssize_t n;
  while (out.size() < max && (n = read(fd, buf, sizeof(buf))) > 0) out.append(buf, static_cast<size_t>(n));
  close(fd);
  return out;
}

std::string Field(const std::string& text, const char* key) {
  size_t klen = strlen(key);
  for (size_t b = 0; b < text.size();) {
    size_t e = text.find('\n', b);
    if (e == std::string::npos) e = text.size();
    if (e - b > klen && text.compare(b, klen, key) == 0 && text[b + klen] == ':') {
      size_t v = b + klen + 1;
      while (v < e && (text[v] == ' ' || text[v] == '\t')) ++v;
      return text.substr(v, e - v);
    }
    b = e + 1;
  }
  return "";
}

// The grant whose accounting file this process maps ("" if none).
std::string GrantFromMaps(const std::string& maps_path, const std::vector<GrantFile>& grants) {
  if (grants.empty()) return "";
  FILE* f = fopen(maps_path.c_str(), "re");
  if (!f) return "";
  std::string found;
  char line[1024];
  while (found.empty() && fgets(line, sizeof(line), f)) {
    // "start-end perms offset MAJ:MIN inode path"
    unsigned maj = 0, mn = 0;
    unsigned long long ino = 0;
    int path_at = 0;
    if (sscanf(line, "%*s %*s %*s %x:%x %llu %n", &maj, &mn, &ino, &path_at) != 3 || ino == 0) continue;
    std::string path = path_at > 0 ? std::string(line + path_at) : "";
    while (!path.empty() && (path.back() == '\n' || path.back() == ' ')) path.pop_back();
    auto ends = [&path](const std::string& suffix) {
      return path.size() >= suffix.size() && path.compare(path.size() - suffix.size(), suffix.size(), suffix) == 0;
    };
    for (const auto& g : grants) {
      if (g.ino != ino) continue;
      // Same device and inode; or, where the daemon's path is on an overlay
      // (maps names the underlying device), the same inode under a grant file's
      // name: the pod's mount point or the file itself.
      if ((g.dev_major == maj && g.dev_minor == mn) || ends("/amdgpu-dp/memcap") || ends("/" + g.key + ".memcap")) {
        found = g.key;
        break;
      }
    }
    // A line longer than the buffer: skip its remainder.
    size_t len = strlen(line);
    while (len && line[len - 1] != '\n' && fgets(line, sizeof(line), f)) len = strlen(line);
  }
  fclose(f);
  return found;
}

std::string FirstLine(const std::string& s) { return s.substr(0, s.find('\n')); }

}  // namespace

uint64_t ParseFdinfoSize(const std::string& value) {
  char* end = nullptr;
  unsigned long long n = strtoull(value.c_str(), &end, 10);
  if (end == value.c_str()) return 0;
  while (*end == ' ' || *end == '\t') ++end;
  uint64_t mul = 1;
  if (!strncmp(end, "KiB", 3)) mul = 1ull << 10;
  else if (!strncmp(end, "MiB", 3)) mul = 1ull << 20;
  else if (!strncmp(end, "GiB", 3)) mul = 1ull << 30;
  if (n > UINT64_MAX / mul) return UINT64_MAX;  // saturate: never wrap a huge claim to a small one
  return static_cast<uint64_t>(n) * mul;
}

std::vector<GrantFile> ListGrantFiles(const std::string& usage_dir) {
  std::vector<GrantFile> out;
  DIR* d = opendir(usage_dir.c_str());
  if (!d) return out;
  int dfd = dirfd(d);
  if (dfd < 0) {
    closedir(d);
    return out;
  }
  while (dirent* e = readdir(d)) {
    std::string name = e->d_name;
    if (name.size() != 16 + 7 || name.compare(16, 7, ".memcap") != 0) continue;
    struct stat st;
    if (fstatat(dfd, name.c_str(), &st, AT_SYMLINK_NOFOLLOW) != 0 || !S_ISREG(st.st_mode)) continue;
    out.push_back({name.substr(0, 16), major(st.st_dev), minor(st.st_dev), static_cast<uint64_t>(st.st_ino)});
  }
  closedir(d);
  return out;
}

std::string SelfCgroup() { return FirstLine(ReadSmall("/proc/self/cgroup", 4096)); }

namespace {

// Numeric entries of a directory (PIDs), in readdir order.
std::vector<std::string> PidEntries(const std::string& dir, bool* opened) {
  std::vector<std::string> out;
  DIR* d = opendir(dir.c_str());
  *opened = d != nullptr;
  if (!d) return out;
  while (dirent* e = readdir(d))
    if (IsPid(e->d_name)) out.emplace_back(e->d_name);
  closedir(d);
  return out;
}

}  // namespace

namespace {

struct PidHbm {
  int pid;
  std::map<std::string, uint64_t> by_bdf;
  bool kfd = false;  // also holds /dev/kfd open
};

// Reads the descriptors of `pids`: render-node fds with DRM fdinfo become
// per-GPU bytes. `kfd_holders` counts the processes with /dev/kfd open.
void ReadPids(const std::string& proc_root, const std::vector<std::string>& pids, DriverScan* out,
              std::vector<PidHbm>* holders, size_t* present, size_t* kfd_holders) {
  // (pdev, drm-client-id): a descriptor shared with another process counts once.
  std::set<std::pair<std::string, uint64_t>> clients;
  // Without a drm-client-id (older kernels) a descriptor cannot be matched to
  // another process's: each (pid, fd) counts on its own.
  std::set<std::tuple<std::string, int, std::string>> anonymous;
  for (const auto& pid : pids) {
    ++out->pids_scanned;
    std::string base = proc_root + "/" + pid;
    DIR* fds = opendir((base + "/fd").c_str());
    if (!fds) {
      if (errno == EACCES || errno == EPERM) {
        ++out->fd_dirs_unreadable;
        ++*present;
      }
      continue;
    }
    int fdd = dirfd(fds);
    if (fdd < 0) {
      closedir(fds);
      continue;
    }
    ++*present;
    PidHbm ph{atoi(pid.c_str()), {}, false};
    bool kfd = false;
    while (dirent* f = readdir(fds)) {
      if (!IsPid(f->d_name)) continue;
      ++out->fd_entries;
      char target[256];
      ssize_t n = readlinkat(fdd, f->d_name, target, sizeof(target) - 1);
      if (n <= 0) continue;
      target[n] = 0;
      if (strcmp(target, "/dev/kfd") == 0) kfd = true;
      if (strncmp(target, "/dev/dri/renderD", 16) != 0) continue;
      std::string info = ReadSmall(base + "/fdinfo/" + f->d_name);
      std::string pdev = Field(info, "drm-pdev");
      if (pdev.empty()) continue;
      std::string client_id = Field(info, "drm-client-id");
      char* end = nullptr;
      uint64_t client = strtoull(client_id.c_str(), &end, 10);
      bool has_client = !client_id.empty() && end && *end == 0;
      // A descriptor shared with another process (fork, SCM_RIGHTS) is one
      // client: its memory counts once, but both processes stay GPU holders
      // (either may be the one that maps the grant's file).
      uint64_t bytes = 0;
      bool first = has_client ? clients.insert({pdev, client}).second
                              : anonymous.insert({pdev, ph.pid, f->d_name}).second;
      if (first) {
        std::string v = Field(info, "drm-resident-vram");
        if (v.empty()) v = Field(info, "drm-memory-vram");
        if (v.empty()) v = Field(info, "drm-total-vram");
        bytes = ParseFdinfoSize(v);
      }
      ph.by_bdf[pdev] += bytes;
    }
    closedir(fds);
    *kfd_holders += kfd;
    ph.kfd = kfd;
    if (!ph.by_bdf.empty()) holders->push_back(std::move(ph));
  }
}

}  // namespace

int64_t FullWalkMsFromEnv() {
  const char* e = getenv("ADP_DRIVER_FULL_WALK_MS");
  if (e && *e) {
    char* end = nullptr;
    long long v = strtoll(e, &end, 10);
    if (end && *end == 0 && v >= 0) return v;
  }
  return 60000;
}

DriverScan ScanDriverHbm(const std::string& proc_root, const std::vector<GrantFile>& grants,
                         const std::string& self_cgroup, const std::string& kfd_proc_dir, ScanState* state) {
  DriverScan out;
  std::vector<PidHbm> holders;
  bool opened = false;
  const int64_t now = std::chrono::duration_cast<std::chrono::milliseconds>(
                          std::chrono::steady_clock::now().time_since_epoch()).count();
  // A full walk: the first scan, then one every full_walk_ms (ScanState).
  const bool walk_all = state && (state->last_full_ms < 0 ||
                                  (state->full_walk_ms > 0 && now - state->last_full_ms >= state->full_walk_ms));
  if (!kfd_proc_dir.empty() && !walk_all) {
    // The driver's own list of GPU processes. It names host PIDs: it is used
    // when they are the PIDs of proc_root -- every listed process found there
    // holds /dev/kfd open -- else (a /proc of another PID namespace, whose
    // numbers mean other processes) the scan falls back to the full walk.
    std::vector<std::string> pids = PidEntries(kfd_proc_dir, &opened);
    if (opened) {
      DriverScan kfd;
      kfd.pid_source = "kfd";
      size_t present = 0, kfd_holders = 0;
      std::vector<PidHbm> h;
      ReadPids(proc_root, pids, &kfd, &h, &present, &kfd_holders);
      if (pids.empty() || (present > 0 && kfd_holders + kfd.fd_dirs_unreadable >= present)) {
        // ... plus the render-only holders the last full walk found (not in
        // KFD's list, still read every scan).
        if (state && !state->render_only_pids.empty()) {
          std::set<std::string> listed(pids.begin(), pids.end());
          std::vector<std::string> extra;
          for (const auto& pid : state->render_only_pids)
            if (!listed.count(pid)) extra.push_back(pid);
          size_t p2 = 0, k2 = 0;
          ReadPids(proc_root, extra, &kfd, &h, &p2, &k2);
        }
        out = std::move(kfd);
        holders = std::move(h);
      } else {
        out.fd_entries = kfd.fd_entries;  // the wasted look counts as cost
      }
    }
  }
  if (out.pid_source != "kfd") {
    std::vector<std::string> pids = PidEntries(proc_root, &opened);
    if (!opened) return out;
    size_t present = 0, kfd_holders = 0;
    ReadPids(proc_root, pids, &out, &holders, &present, &kfd_holders);
    if (state) {
      state->last_full_ms = now;
      ++state->full_walks;
      state->render_only_pids.clear();
      for (const auto& h : holders) {
        uint64_t bytes = 0;
        for (const auto& [_, b] : h.by_bdf) bytes += b;
        if (!h.kfd && bytes) state->render_only_pids.push_back(std::to_string(h.pid));
      }
    }
  }
  for (const auto& h : holders) {
    uint64_t bytes = 0;
    for (const auto& [_, b] : h.by_bdf) bytes += b;
    out.render_only += !h.kfd && bytes;
  }

  // Attribution: own mapping first, then the cgroup of an attributed process
  // -- a container's own cgroup, never the root one ("0::/", "N:ctrl:/") that
  // every process outside a container shares.
  auto is_root = [](const std::string& cg) { return cg.size() >= 2 && cg.compare(cg.size() - 2, 2, ":/") == 0; };
  std::map<std::string, std::string> grant_of_cgroup;
  for (auto& h : holders) {
    std::string base = proc_root + "/" + std::to_string(h.pid);
    std::string cg = FirstLine(ReadSmall(base + "/cgroup", 4096));
    std::string grant = GrantFromMaps(base + "/maps", grants);
    if (!grant.empty() && !cg.empty() && cg != self_cgroup && !is_root(cg)) grant_of_cgroup.emplace(cg, grant);
    for (auto& [bdf, bytes] : h.by_bdf) out.procs.push_back({h.pid, bdf, bytes, cg, grant, false});
  }
  for (auto& p : out.procs) {
    if (p.grant.empty() && !p.cgroup.empty() && p.cgroup != self_cgroup) {
      auto it = grant_of_cgroup.find(p.cgroup);
      if (it != grant_of_cgroup.end()) {
        p.grant = it->second;
        p.via_cgroup = true;
      }
    }
  }
  Aggregate(&out);
  return out;
}

void Aggregate(DriverScan* s) {
  s->total.clear();
  s->unattributed.clear();
  s->by_grant.clear();
  s->grant_procs.clear();
  for (const auto& p : s->procs) {
    s->total[p.bdf] += p.bytes;
    if (p.grant.empty()) {
      s->unattributed[p.bdf] += p.bytes;
    } else {
      s->by_grant[{p.grant, p.bdf}] += p.bytes;
      if (p.bytes) ++s->grant_procs[{p.grant, p.bdf}];
    }
  }
}

namespace {

// Fields are tab separated; none may hold a tab or a newline (a cgroup path or
// BDF with one is rewritten: those come from /proc, not from the daemon).
std::string Clean(std::string v) {
  for (char& c : v)
    if (c == '\t' || c == '\n' || c == '\r') c = ' ';
  return v;
}

std::vector<std::string_view> Fields(std::string_view line) {
  std::vector<std::string_view> f;
  for (size_t b = 0; b <= line.size();) {
    size_t e = line.find('\t', b);
    if (e == std::string_view::npos) e = line.size();
    f.push_back(line.substr(b, e - b));
    b = e + 1;
  }
  return f;
}

// Canonical decimal only (no sign, no leading zero): what std::to_string writes.
bool ToU64(std::string_view v, uint64_t* out) {
  if (v.empty() || v.size() > 20 || (v.size() > 1 && v[0] == '0')) return false;
  uint64_t n = 0;
  for (char c : v) {
    if (c < '0' || c > '9') return false;
    uint64_t d = static_cast<uint64_t>(c - '0');
    if (n > (UINT64_MAX - d) / 10) return false;
    n = n * 10 + d;
  }
  *out = n;
  return true;
}

}  // namespace

std::string SerializeScan(const DriverScan& s) {
  std::string out = "scan\t" + Clean(s.pid_source) + "\t" + std::to_string(s.pids_scanned) + "\t" +
                    std::to_string(s.fd_entries) + "\t" + std::to_string(s.fd_dirs_unreadable) + "\t" +
                    std::to_string(s.procs.size()) + "\t" + std::to_string(s.render_only) + "\n";
  for (const auto& p : s.procs)
    out += "p\t" + std::to_string(p.pid) + "\t" + Clean(p.bdf) + "\t" + std::to_string(p.bytes) + "\t" +
           Clean(p.grant) + "\t" + (p.via_cgroup ? "1" : "0") + "\t" + Clean(p.cgroup) + "\n";
  return out;
}

ParseResult ParseScanReply(std::string_view text, DriverScan* out, size_t* consumed) {
  // A header, then exactly as many process lines as it announces. Until a
  // line is complete it can only be judged as far as it goes: "scan\t" and a
  // run of digits can still become a reply, "scab" or a letter in a number
  // cannot -- a reply that is not one fails at once instead of at the timeout.
  constexpr std::string_view kHead = "scan\t";
  size_t nl = text.find('\n');
  if (nl == std::string_view::npos) {
    size_t n = std::min(text.size(), kHead.size());
    if (text.substr(0, n) != kHead.substr(0, n)) return ParseResult::kMalformed;
    return text.find('\r') != std::string_view::npos || text.size() > 4096 ? ParseResult::kMalformed
                                                                             : ParseResult::kIncomplete;
  }
  // (SerializeScan never writes a carriage return: a reply holding one is not its)
  if (text.substr(0, nl).find('\r') != std::string_view::npos) return ParseResult::kMalformed;
  auto h = Fields(text.substr(0, nl));
  uint64_t pids = 0, fds = 0, unreadable = 0, n = 0, render_only = 0;
  if ((h.size() != 6 && h.size() != 7) || h[0] != "scan" || !ToU64(h[2], &pids) || !ToU64(h[3], &fds) ||
      !ToU64(h[4], &unreadable) || !ToU64(h[5], &n) || n > 1000000 || (h.size() == 7 && !ToU64(h[6], &render_only)))
    return ParseResult::kMalformed;
  DriverScan s;
  s.pid_source = std::string(h[1]);
  s.pids_scanned = pids;
  s.fd_entries = fds;
  s.fd_dirs_unreadable = unreadable;
  s.render_only = render_only;
  size_t pos = nl + 1;
  for (uint64_t i = 0; i < n; ++i) {
    size_t e = text.find('\n', pos);
    if (e == std::string_view::npos) {
      std::string_view part = text.substr(pos);
      if (part.find('\r') != std::string_view::npos || (!part.empty() && part[0] != 'p'))
        return ParseResult::kMalformed;
      return ParseResult::kIncomplete;
    }
    if (text.substr(pos, e - pos).find('\r') != std::string_view::npos) return ParseResult::kMalformed;
    auto f = Fields(text.substr(pos, e - pos));
    uint64_t pid = 0, bytes = 0;
    if (f.size() != 7 || f[0] != "p" || !ToU64(f[1], &pid) || pid > INT32_MAX || !ToU64(f[3], &bytes) ||
        (f[5] != "0" && f[5] != "1"))
      return ParseResult::kMalformed;
    s.procs.push_back({static_cast<int>(pid), std::string(f[2]), bytes, std::string(f[6]), std::string(f[4]),
                       f[5] == "1"});
    pos = e + 1;
  }
  Aggregate(&s);
  *out = std::move(s);
  if (consumed) *consumed = pos;
  return ParseResult::kOk;
}

bool ParseScan(std::string_view text, DriverScan* out, size_t* consumed) {
  return ParseScanReply(text, out, consumed) == ParseResult::kOk;
}

Result<DriverScan> RemoteScan(int fd, const std::string& usage_dir, const std::string& self_cgroup, int timeout_ms,
                              int cancel_fd) {
  if (usage_dir.find_first_of("\t\n") != std::string::npos || self_cgroup.find_first_of("\t\n") != std::string::npos)
    return InvalidArgument("usage directory or cgroup with a tab or newline");
  std::string req = "scan\t" + usage_dir + "\t" + self_cgroup + "\n";
  if (send(fd, req.data(), req.size(), MSG_NOSIGNAL) != static_cast<ssize_t>(req.size()))
    return Unavailable(std::string("event relay: ") + strerror(errno));
  std::string in;
  auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  for (;;) {
    // The relay greets every connection ("hello v1 ..."): lines before the reply are skipped.
    for (size_t nl; in.compare(0, 5, "scan\t") != 0 && (nl = in.find('\n')) != std::string::npos;)
      in.erase(0, nl + 1);
    DriverScan s;
    if (in.compare(0, 5, "scan\t") == 0) {  // (a partial line before it may still be a greeting)
      ParseResult pr = ParseScanReply(in, &s, nullptr);
      if (pr == ParseResult::kOk) return s;
      if (pr == ParseResult::kMalformed) return Internal("event relay: malformed scan reply");
    }
    if (in.size() > (64u << 20)) return Internal("event relay: scan reply too large");
    int left = static_cast<int>(
        std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now()).count());
    if (left <= 0) return Unavailable("event relay: no scan reply in time");
    pollfd p[2] = {{fd, POLLIN, 0}, {cancel_fd, POLLIN, 0}};
    if (poll(p, cancel_fd >= 0 ? 2 : 1, left) <= 0) continue;
    if (cancel_fd >= 0 && (p[1].revents & POLLIN)) return Unavailable("scan cancelled");
    char buf[65536];
    ssize_t n = recv(fd, buf, sizeof(buf), 0);
    if (n == 0) return Unavailable("event relay closed the connection");
    if (n < 0) {
      if (errno == EINTR || errno == EAGAIN) continue;
      return Unavailable(std::string("event relay: ") + strerror(errno));
    }
    in.append(buf, static_cast<size_t>(n));
  }
}

DriverHbmMonitor::DriverHbmMonitor(Options opts, GrantFn grants)
    : opts_(std::move(opts)), grants_(std::move(grants)), self_cgroup_(SelfCgroup()) {
  snap_.slack_bytes = opts_.slack_bytes;
  scan_state_.full_walk_ms = FullWalkMsFromEnv();
}

DriverHbmMonitor::~DriverHbmMonitor() { Stop(); }

namespace {

int ConnectUnix(const std::string& path) {
  sockaddr_un addr{};
  if (path.empty() || path.size() >= sizeof(addr.sun_path)) return -1;
  int fd = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) return -1;
  addr.sun_family = AF_UNIX;
  memcpy(addr.sun_path, path.c_str(), path.size());
  if (connect(fd, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0) {
    close(fd);
    return -1;
  }
  return fd;
}

}  // namespace

void DriverHbmMonitor::PollOnce() {
  auto t0 = std::chrono::steady_clock::now();
  DriverScan scan;
  if (!opts_.relay_socket.empty()) {
    // A poll that cannot reach the relay keeps the previous scan and grant states.
    int fd = ConnectUnix(opts_.relay_socket);
    Result<DriverScan> r = fd < 0 ? Result<DriverScan>(Unavailable("event relay " + opts_.relay_socket + ": " +
                                                                   strerror(errno)))
                                  : RemoteScan(fd, opts_.usage_dir, self_cgroup_, std::max(opts_.poll_ms, 30000),
                                               wake_fd_);
    if (fd >= 0) close(fd);
    if (!r.ok()) {
      if (stop_.load()) return;  // cancelled by Stop()
      std::lock_guard<std::mutex> lk(mu_);
      // The pod's two containers start together: a relay not listening yet is
      // expected for the first polls, a warning only after that.
      constexpr uint64_t kStartupGrace = 5;  // failed polls before a relay that never answered is a warning
      if (snap_.polls == 0 && snap_.scan_failures < kStartupGrace) {
        if (snap_.scan_failures == 0)
          LOG_INFO(kComp, "driver-side scan: waiting for the event relay (%s)", r.status().ToString().c_str());
      } else if (snap_.polls == 0 ? snap_.scan_failures == kStartupGrace : snap_.scan_error.empty()) {
        LOG_WARN(kComp, "driver-side scan through the relay failed: %s", r.status().ToString().c_str());
      }
      snap_.scan_error = r.status().ToString();
      snap_.remote = true;
      ++snap_.scan_failures;
      return;
    }
    scan = std::move(*r);
  } else {
    scan = ScanDriverHbm(opts_.proc_root, ListGrantFiles(opts_.usage_dir), self_cgroup_, opts_.kfd_proc_dir,
                         &scan_state_);
  }
  uint64_t scan_ns = static_cast<uint64_t>(
      std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count());
  auto granted = grants_ ? grants_() : std::map<std::string, std::map<std::string, uint64_t>>{};
  std::map<std::pair<std::string, std::string>, GrantState> states;
  for (const auto& [key, per_bdf] : granted)
    for (const auto& [bdf, bytes] : per_bdf) states[{key, bdf}].granted_bytes = bytes;
  for (const auto& [kb, bytes] : scan.by_grant) {
    auto& st = states[kb];
    st.driver_bytes = bytes;
    st.processes = scan.grant_procs[kb];
  }
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& [kb, st] : states) {
    // Not a grant of ours (no granted bytes on that GPU): everything held there is over.
    uint64_t allowed = st.granted_bytes + static_cast<uint64_t>(st.processes) * opts_.slack_bytes;
    st.over = st.driver_bytes > allowed;
    bool was = false;
    auto prev = snap_.grants.find(kb);
    if (prev != snap_.grants.end()) was = prev->second.over;
    if (st.over && !was) {
      ++transitions_[kb];
      ++snap_.over_total;
      LOG_WARN(kComp, "grant %s holds %.1f MiB on GPU %s by the driver's count, granted %.1f MiB (+%.0f MiB "
               "runtime allowance x %d process(es)): over its grant", kb.first.c_str(), st.driver_bytes / 1048576.0,
               kb.second.c_str(), st.granted_bytes / 1048576.0, opts_.slack_bytes / 1048576.0, st.processes);
    }
    st.over_transitions = transitions_[kb];
  }
  const bool remote = !opts_.relay_socket.empty();
  if (snap_.polls == 0 && scan.fd_dirs_unreadable)
    LOG_WARN(kComp, "%zu of %zu processes' file descriptors are not readable: HBM they hold is not seen (run %s "
             "privileged, with the host's PID namespace or /proc at --host-proc)",
             scan.fd_dirs_unreadable, scan.pids_scanned, remote ? "the event relay" : "the plugin");
  if (snap_.polls == 0) {
    std::string from = remote                      ? "the event relay's " + scan.pid_source + " list"
                       : scan.pid_source == "kfd" ? opts_.kfd_proc_dir
                                                  : opts_.proc_root;
    LOG_INFO(kComp, "first scan: %zu candidate process(es) from %s, %zu descriptor(s), %.2f ms", scan.pids_scanned,
             from.c_str(), scan.fd_entries, scan_ns / 1e6);
  }
  if (!snap_.scan_error.empty())
    LOG_INFO(kComp, "%s", snap_.polls == 0 ? "driver-side scan: the event relay answers"
                                           : "driver-side scan through the relay works again");
  snap_.scan_error.clear();
  if (scan.pid_source == "proc") {
    snap_.render_only = scan.render_only;
    if (scan.render_only && !snap_.render_only_logged) {
      snap_.render_only_logged = true;
      LOG_WARN(kComp, "%zu process(es) hold HBM through a render node without /dev/kfd (not in KFD's process list): "
               "read on every scan from now on, and a full walk every %lld ms finds new ones",
               scan.render_only, static_cast<long long>(scan_state_.full_walk_ms));
    }
  }
  snap_.full_walks = remote ? snap_.full_walks : scan_state_.full_walks;
  snap_.remote = remote;
  snap_.scan = std::move(scan);
  snap_.grants = std::move(states);
  snap_.last_scan_ns = scan_ns;
  snap_.scan_ns_total += scan_ns;
  ++snap_.polls;
}

DriverHbmMonitor::Snapshot DriverHbmMonitor::Get() const {
  std::lock_guard<std::mutex> lk(mu_);
  return snap_;
}

void DriverHbmMonitor::Start() {
  if (thread_.joinable() || opts_.poll_ms <= 0) return;
  stop_.store(false);
  wake_fd_ = eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);
  thread_ = std::thread([this] {
    while (!stop_.load()) {
      PollOnce();
      pollfd p{wake_fd_, POLLIN, 0};
      poll(&p, 1, opts_.poll_ms);
    }
  });
  LOG_INFO(kComp, "checking HBM grants against the driver every %d ms (%s, runtime allowance %.0f MiB/process)",
           opts_.poll_ms,
           opts_.relay_socket.empty() ? opts_.proc_root.c_str() : ("scans by the event relay at " + opts_.relay_socket).c_str(),
           opts_.slack_bytes / 1048576.0);
}

void DriverHbmMonitor::Stop() {
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
}

}  // namespace adp::memcap

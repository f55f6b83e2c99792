// The relay protocol both ends speak (relay.h): the lines the relay sends
// (hello, event) and the requests it reads (reinit, scan), the processor
// fingerprint, and the client side -- connecting, and the liveness probe
// (--relay-ping). The relay process itself is relay.cc.
#include <fcntl.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstring>

#include "common/strings.h"
#include "health/relay.h"

namespace adp::health {
namespace {

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

}  // namespace

RelayLine ParseRelayLine(std::string_view line) {
  RelayLine r;
  while (!line.empty() && (line.back() == '\n' || line.back() == '\r')) line.remove_suffix(1);
  if (line.rfind("hello ", 0) == 0) {
    r.kind = "hello";
    size_t at = line.find(" reason=");
    if (at != std::string_view::npos) r.reason = std::string(line.substr(at + 8));
    std::string_view head = line.substr(0, at);  // key=value tokens never come from the reason
    r.events_ok = Kv(head, "events") == "ok";
    r.after_reinit = line.rfind("hello v1 reinit ", 0) == 0;
    r.relay = std::string(Kv(head, "relay"));
    if (auto v = ParseUint(std::string(Kv(head, "gen")))) r.gen = *v;
    if (auto v = ParseUint(std::string(Kv(head, "seq")))) r.seq = *v;
    std::string_view gap = Kv(head, "gap");
    r.gap = gap == "0" ? 0 : gap == "1" ? 1 : -1;
    return r;
  }
  if (line.rfind("event ", 0) != 0) return r;
  size_t end = 0, last = 0;
  std::string_view seq = Kv(line, "seq", &end);
  if (!seq.empty()) last = std::max(last, end);
  std::string_view node = Kv(line, "node", &end);
  last = std::max(last, end);
  r.bdf = std::string(Kv(line, "bdf", &end));
  last = std::max(last, end);
  auto part = ParseUint(std::string(Kv(line, "part", &end)));
  last = std::max(last, end);
  auto type = ParseUint(std::string(Kv(line, "type", &end)));
  last = std::max(last, end);
  if (!part || !type || *type > 0xffffffffu || *part > 0xffffffffu) return r;
  if (!seq.empty()) {
    auto s = ParseUint(std::string(seq));
    if (!s) return r;
    r.seq = *s;
  }
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

RelayRequest ParseRelayRequest(std::string_view line) {
  RelayRequest r;
  while (!line.empty() && (line.back() == '\n' || line.back() == '\r')) line.remove_suffix(1);
  auto hex = [](std::string_view v, size_t min, size_t max) {
    if (v.size() < min || v.size() > max) return false;
    for (char c : v)
      if (!((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f'))) return false;
    return true;
  };
  if (line == "reinit" || line.rfind("reinit ", 0) == 0) {
    r.kind = "reinit";
    std::string_view fp = Kv(line, "fp");
    if (hex(fp, 16, 16)) r.fp = std::string(fp);
    auto since = Split(Kv(line, "since"), ':');
    if (since.size() == 3 && hex(since[0], 1, 32)) {
      auto seq = ParseUint(since[1]);
      auto gen = ParseUint(since[2]);
      if (seq && gen) {
        r.has_since = true;
        r.since_relay = since[0];
        r.since_seq = *seq;
        r.since_gen = *gen;
      }
    }
    return r;
  }
  if (line.rfind("scan\t", 0) == 0) {
    // "scan\t<usage dir>\t<cgroup>": an absolute directory without "..": the
    // relay stats its entries, nothing more.
    r.kind = "scan";
    size_t tab = line.find('\t', 5);
    if (tab == std::string_view::npos) {
      r.malformed = true;
      return r;
    }
    std::string_view dir = line.substr(5, tab - 5);
    r.usage_dir = std::string(dir);
    r.cgroup = std::string(line.substr(tab + 1));
    r.malformed = dir.empty() || dir[0] != '/' || dir.find("/..") != std::string_view::npos;
  }
  return r;
}

std::string FormatRelayEvent(const smi::ProcessorInfo& p, uint32_t type, const std::string& message) {
  return "event node=" + (p.kfd_node == 0xffffffffu ? std::string("-") : std::to_string(p.kfd_node)) +
         " bdf=" + (p.bdf.empty() ? std::string("-") : p.bdf) + " part=" + std::to_string(p.partition_id) +
         " type=" + std::to_string(type) + " " + OneLine(message) + "\n";
}

std::string FormatUnplacedRelayEvent(uint32_t type, const std::string& message) {
  return "event node=- bdf=- part=0 type=" + std::to_string(type) + " " + OneLine(message) + "\n";
}

std::string ProcessorFingerprint(const std::vector<smi::ProcessorInfo>& procs) {
  std::vector<std::string> keys;
  keys.reserve(procs.size());
  for (const auto& p : procs)
    keys.push_back(p.bdf + "/" + std::to_string(p.partition_id) + "/" + std::to_string(p.kfd_node) + "/" +
                   p.compute_partition + "/" + p.memory_partition);
  std::sort(keys.begin(), keys.end());
  uint64_t h = 0xcbf29ce484222325ull;  // FNV-1a
  for (const auto& k : keys) {
    for (unsigned char c : k) h = (h ^ c) * 0x100000001b3ull;
    h = (h ^ ';') * 0x100000001b3ull;
  }
  char buf[17];
  snprintf(buf, sizeof(buf), "%016llx", static_cast<unsigned long long>(h));
  return buf;
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
}  // namespace adp::health

#include "metrics/metrics.h"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "common/log.h"
#include "common/strings.h"

namespace adp::metrics {
namespace {
constexpr const char* kComp = "metrics";
}

const double Histogram::kBoundsSec[kBuckets] = {
    250e-9, 500e-9, 1e-6, 2e-6, 5e-6, 10e-6, 20e-6, 50e-6, 100e-6, 200e-6,
    500e-6, 1e-3,   2e-3, 5e-3, 10e-3, 20e-3, 50e-3, 100e-3, 500e-3, 1.0};

int ShardIndex() {
  static std::atomic<int> next{0};
  thread_local int idx = next.fetch_add(1, std::memory_order_relaxed) % kShards;
  return idx;
}

uint64_t Counter::Value() const {
  uint64_t t = 0;
  for (const auto& s : s_) t += s.v.load(std::memory_order_relaxed);
  return t;
}

void MaxGauge::Observe(uint64_t v) {
  auto& a = s_[ShardIndex()].v;
  uint64_t prev = a.load(std::memory_order_relaxed);
  while (v > prev && !a.compare_exchange_weak(prev, v, std::memory_order_relaxed)) {}
}

uint64_t MaxGauge::Value() const {
  uint64_t m = 0;
  for (const auto& s : s_) m = std::max(m, s.v.load(std::memory_order_relaxed));
  return m;
}

void Histogram::Observe(uint64_t ns) {
  int b = 0;
  while (b < kBuckets && ns > static_cast<uint64_t>(kBoundsSec[b] * 1e9 + 0.5)) ++b;
  Shard& s = shards_[ShardIndex()];
  s.buckets[b].fetch_add(1, std::memory_order_relaxed);
  s.sum_ns.fetch_add(ns, std::memory_order_relaxed);
}

void Histogram::Totals(uint64_t counts[kBuckets + 1]) const {
  for (int b = 0; b <= kBuckets; ++b) {
    counts[b] = 0;
    for (const auto& s : shards_) counts[b] += s.buckets[b].load(std::memory_order_relaxed);
  }
}

uint64_t Histogram::count() const {
  uint64_t counts[kBuckets + 1], t = 0;
  Totals(counts);
  for (uint64_t c : counts) t += c;
  return t;
}

double Histogram::sum_seconds() const {
  uint64_t t = 0;
  for (const auto& s : shards_) t += s.sum_ns.load(std::memory_order_relaxed);
  return t / 1e9;
}

double Histogram::QuantileUs(double q) const {
  uint64_t counts[kBuckets + 1];
  Totals(counts);
  uint64_t total = 0;
  for (uint64_t c : counts) total += c;
  if (total == 0) return 0.0;
  uint64_t rank = static_cast<uint64_t>(q * static_cast<double>(total - 1)) + 1;
  uint64_t seen = 0;
  for (int b = 0; b <= kBuckets; ++b) {
    seen += counts[b];
    if (seen >= rank) return (b < kBuckets ? kBoundsSec[b] : kBoundsSec[kBuckets - 1] * 10) * 1e6;
  }
  return kBoundsSec[kBuckets - 1] * 1e6;
}

void Histogram::AppendPrometheus(const std::string& name, const std::string& labels,
                                 std::string* out) const {
  // Appended whole (no fixed line buffer: a truncated line breaks the scrape).
  uint64_t counts[kBuckets + 1];
  Totals(counts);
  uint64_t cum = 0;
  std::string head = name + "_bucket{" + labels + (labels.empty() ? "" : ",") + "le=\"";
  char num[48];
  for (int b = 0; b <= kBuckets; ++b) {
    cum += counts[b];
    *out += head;
    if (b < kBuckets) {
      snprintf(num, sizeof(num), "%g", kBoundsSec[b]);
      *out += num;
    } else {
      *out += "+Inf";
    }
    *out += "\"} " + std::to_string(cum) + "\n";
  }
  snprintf(num, sizeof(num), "%.9f", sum_seconds());
  *out += name + "_sum{" + labels + "} " + num + "\n" + name + "_count{" + labels + "} " + std::to_string(cum) + "\n";
}

FineHistogram::FineHistogram() : shards_(new Shard[kShards]) {}

void FineHistogram::Observe(uint64_t ns) {
  uint64_t b = ns / kBinNs;
  Shard& s = shards_[ShardIndex()];
  s.bins[b < kBins ? b : kBins].fetch_add(1, std::memory_order_relaxed);
  s.sum_ns.fetch_add(ns, std::memory_order_relaxed);
}

std::vector<uint64_t> FineHistogram::Counts() const {
  std::vector<uint64_t> c(kBins + 1, 0);
  for (int i = 0; i < kShards; ++i)
    for (int b = 0; b <= kBins; ++b) c[b] += shards_[i].bins[b].load(std::memory_order_relaxed);
  return c;
}

uint64_t FineHistogram::sum_ns() const {
  uint64_t t = 0;
  for (int i = 0; i < kShards; ++i) t += shards_[i].sum_ns.load(std::memory_order_relaxed);
  return t;
}

double FineHistogram::QuantileUs(const std::vector<uint64_t>& counts, double q) {
  uint64_t total = 0;
  for (uint64_t c : counts) total += c;
  if (total == 0) return 0.0;
  uint64_t rank = static_cast<uint64_t>(q * static_cast<double>(total - 1)) + 1, seen = 0;
  for (size_t b = 0; b < counts.size(); ++b) {
    seen += counts[b];
    if (seen >= rank) return static_cast<double>((b + 1) * kBinNs) / 1e3;
  }
  return static_cast<double>(counts.size() * kBinNs) / 1e3;
}

std::string FineHistogram::SparseJson() const {
  std::vector<uint64_t> c = Counts();
  std::string out = "[";
  for (size_t b = 0; b < c.size(); ++b) {
    if (!c[b]) continue;
    if (out.size() > 1) out += ", ";
    out += "[" + std::to_string(b) + ", " + std::to_string(c[b]) + "]";
  }
  return out + "]";
}

void FineHistogram::AppendPrometheus(const std::string& name, const std::string& labels, std::string* out) const {
  std::vector<uint64_t> c = Counts();
  static const double kLe[] = {1e-6, 2e-6, 5e-6, 10e-6, 20e-6, 50e-6, 100e-6};
  std::string head = name + "_bucket{" + labels + (labels.empty() ? "" : ",") + "le=\"";
  uint64_t cum = 0;
  size_t b = 0;
  char num[48];
  for (double le : kLe) {
    // bins entirely below the bound (bin b ends at (b+1) x 100 ns)
    for (; b < kBins && (b + 1) * kBinNs <= static_cast<uint64_t>(le * 1e9 + 0.5); ++b) cum += c[b];
    snprintf(num, sizeof(num), "%g", le);
    *out += head + num + "\"} " + std::to_string(cum) + "\n";
  }
  for (; b <= kBins; ++b) cum += c[b];
  *out += head + "+Inf\"} " + std::to_string(cum) + "\n";
  snprintf(num, sizeof(num), "%.9f", sum_ns() / 1e9);
  *out += name + "_sum{" + labels + "} " + num + "\n" + name + "_count{" + labels + "} " + std::to_string(cum) + "\n";
}

std::string LabelValue(const std::string& v) {
  std::string o;
  o.reserve(v.size());
  for (char c : v) {
    if (c == '\\') o += "\\\\";
    else if (c == '"') o += "\\\"";
    else if (c == '\n') o += "\\n";
    else o += c;
  }
  return o;
}

HttpServer::HttpServer(Render render, Healthy healthy, Render stats)
    : render_(std::move(render)), healthy_(std::move(healthy)), stats_(std::move(stats)) {}

HttpServer::~HttpServer() { Stop(); }

Status HttpServer::Listen(const std::string& addr) {
  std::string host, port = addr;
  size_t colon = addr.rfind(':');
  if (colon != std::string::npos) {
    host = addr.substr(0, colon);
    port = addr.substr(colon + 1);
  }
  if (!host.empty() && host.front() == '[' && host.back() == ']') host = host.substr(1, host.size() - 2);
  auto p = ParseUint(port);
  if (!p || *p > 65535) return InvalidArgument("invalid --metrics-addr '" + addr + "'");
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  hints.ai_flags = AI_PASSIVE | AI_NUMERICSERV;
  int rc = getaddrinfo(host.empty() ? nullptr : host.c_str(), port.c_str(), &hints, &res);
  if (rc != 0) return InvalidArgument("invalid --metrics-addr '" + addr + "': " + gai_strerror(rc));
  Status st = Unavailable("no usable address for " + addr);
  bool bound = false;
  for (addrinfo* ai = res; ai && !bound; ai = ai->ai_next) {
    int fd = socket(ai->ai_family, ai->ai_socktype | SOCK_CLOEXEC | SOCK_NONBLOCK, ai->ai_protocol);
    if (fd < 0) continue;
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    if (bind(fd, ai->ai_addr, ai->ai_addrlen) == 0 && listen(fd, 16) == 0) {
      if (listen_fds_.empty()) {
        sockaddr_storage ss{};
        socklen_t len = sizeof(ss);
        getsockname(fd, reinterpret_cast<sockaddr*>(&ss), &len);
        port_ = ntohs(ss.ss_family == AF_INET6 ? reinterpret_cast<sockaddr_in6*>(&ss)->sin6_port
                                               : reinterpret_cast<sockaddr_in*>(&ss)->sin_port);
      }
      listen_fds_.push_back(fd);
      bound = true;
      break;
    }
    st = Unavailable("metrics listen on " + addr + ": " + strerror(errno));
    close(fd);
  }
  freeaddrinfo(res);
  return bound ? Status::Ok() : st;
}

Status HttpServer::Start(const std::string& addr) {
  for (const auto& one : Split(addr, ',')) {
    std::string a = Trim(one);
    if (a.empty()) continue;
    if (Status st = Listen(a); !st.ok()) {
      for (int fd : listen_fds_) close(fd);
      listen_fds_.clear();
      return st;
    }
  }
  if (listen_fds_.empty()) return InvalidArgument("invalid --metrics-addr '" + addr + "'");
  stop_fd_ = eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);
  spare_fd_ = open("/dev/null", O_RDONLY | O_CLOEXEC);
  thread_ = std::thread([this] { Run(); });
  LOG_INFO(kComp, "serving /metrics and /healthz on port %d (and /stats) at %s", port_, addr.c_str());
  return Status::Ok();
}

void HttpServer::Stop() {
  if (thread_.joinable()) {
    uint64_t one = 1;
    ssize_t w = write(stop_fd_, &one, sizeof(one));
    (void)w;
    thread_.join();
  }
  for (int fd : listen_fds_) close(fd);
  listen_fds_.clear();
  if (stop_fd_ >= 0) close(stop_fd_);
  if (spare_fd_ >= 0) close(spare_fd_);
  stop_fd_ = spare_fd_ = -1;
}

// Connections are served concurrently from one poll loop, each with a 2 s
// budget for the whole exchange: a slow or idle client (or many) cannot hold
// up the kubelet-side liveness probe on /healthz. One request per connection
// (a scraper on the node, not a general web server).
void HttpServer::Run() {
  using Clock = std::chrono::steady_clock;
  constexpr size_t kMaxClients = 64;
  struct Client {
    int fd;
    Clock::time_point deadline;
    std::string in, out;
    size_t off = 0;
    bool responding = false;
  };
  std::vector<Client> cs;
  std::vector<pollfd> p;
  auto drop = [&](size_t i) {
    close(cs[i].fd);
    cs[i] = std::move(cs.back());
    cs.pop_back();
  };
  while (true) {
    p.clear();
    p.push_back({stop_fd_, POLLIN, 0});
    for (int lfd : listen_fds_)
      p.push_back({cs.size() < kMaxClients ? lfd : -1, POLLIN, 0});  // full: leave them in the backlog
    const size_t fixed = 1 + listen_fds_.size();
    int timeout = -1;
    auto now = Clock::now();
    for (const auto& c : cs) {
      p.push_back({c.fd, static_cast<short>(c.responding ? POLLOUT : POLLIN), 0});
      int ms = static_cast<int>(
          std::max<long long>(0, std::chrono::duration_cast<std::chrono::milliseconds>(c.deadline - now).count()) + 1);
      timeout = timeout < 0 ? ms : std::min(timeout, ms);
    }
    if (poll(p.data(), p.size(), timeout) < 0) {
      if (errno == EINTR) continue;
      break;
    }
    if (p[0].revents) break;
    // Clients first (their pollfds follow the fixed entries, in order).
    now = Clock::now();
    for (size_t i = cs.size(); i-- > 0;) {
      Client& c = cs[i];
      short re = p[fixed + i].revents;
      bool done = false;
      if (re && !c.responding) {
        char buf[2048];
        ssize_t n = read(c.fd, buf, sizeof(buf));
        if (n > 0) c.in.append(buf, static_cast<size_t>(n));
        if (n == 0 || (n < 0 && errno != EAGAIN && errno != EINTR)) {
          done = true;
        } else if (c.in.find("\r\n\r\n") != std::string::npos || c.in.size() >= 8192) {
          c.out = Respond(c.in);
          c.responding = true;
        }
      }
      if (!done && c.responding && c.off < c.out.size()) {
        ssize_t n = send(c.fd, c.out.data() + c.off, c.out.size() - c.off, MSG_NOSIGNAL);
        if (n > 0) c.off += static_cast<size_t>(n);
        else if (n < 0 && errno != EAGAIN && errno != EINTR) done = true;
        if (c.off == c.out.size()) done = true;
      }
      if (done || now >= c.deadline) drop(i);
    }
    for (size_t l = 0; l < listen_fds_.size(); ++l) {
      if (!p[1 + l].revents) continue;
      const int listen_fd = listen_fds_[l];
      while (cs.size() < kMaxClients) {
        int fd = accept4(listen_fd, nullptr, nullptr, SOCK_CLOEXEC | SOCK_NONBLOCK);
        if (fd >= 0) {
          cs.push_back({fd, Clock::now() + std::chrono::seconds(2), {}, {}, 0, false});
          continue;
        }
        if (errno == EINTR) continue;
        if ((errno == EMFILE || errno == ENFILE) && spare_fd_ >= 0) {
          close(spare_fd_);
          int shed = accept4(listen_fd, nullptr, nullptr, SOCK_CLOEXEC);
          if (shed >= 0) close(shed);
          spare_fd_ = open("/dev/null", O_RDONLY | O_CLOEXEC);
          if (shed >= 0) continue;
        }
        break;
      }
    }
  }
  for (auto& c : cs) close(c.fd);
}

std::string HttpServer::Respond(const std::string& req) {
  std::string line = req.substr(0, req.find("\r\n"));
  auto parts = Split(line, ' ');
  std::string status = "200 OK", type = "text/plain; version=0.0.4; charset=utf-8", body;
  std::string path = parts.size() >= 2 ? parts[1] : "";
  if (size_t q = path.find('?'); q != std::string::npos) path.resize(q);
  if (parts.size() < 3 || (parts[0] != "GET" && parts[0] != "HEAD")) {
    status = "405 Method Not Allowed";
    body = "only GET\n";
  } else if (path == "/metrics") {
    body = render_();
  } else if (path == "/stats" && stats_) {
    type = "application/json";
    body = stats_();
  } else if (path == "/healthz") {
    bool ok = healthy_();
    status = ok ? "200 OK" : "503 Service Unavailable";
    body = ok ? "ok\n" : "plugins not serving\n";
  } else {
    status = "404 Not Found";
    body = "try /metrics, /healthz or /stats\n";
  }
  std::string resp = "HTTP/1.1 " + status + "\r\nContent-Type: " + type +
                     "\r\nContent-Length: " + std::to_string(body.size()) + "\r\nConnection: close\r\n\r\n";
  if (parts.empty() || parts[0] != "HEAD") resp += body;
  return resp;
}

}  // namespace adp::metrics

// UDS round-trip floor: what a request/response over a Unix socket costs with
// no HTTP/2, no gRPC and no handler -- the lower bound for the plugin's
// Allocate() latency on the same host. The server side mirrors the daemon's
// loop (epoll, optional adaptive busy-poll); the client mirrors the benchmark
// client (send, poll, read). Payload sizes default to the bench's Allocate
// request/response frame sizes.
//
//   amdgpu-dp-uds-floor [--iters N] [--busy-poll-us U] [--req B] [--resp B]
#include <poll.h>
#include <sys/epoll.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

using Clock = std::chrono::steady_clock;

double ThreadCpuUs() {
  rusage ru{};
  getrusage(RUSAGE_THREAD, &ru);
  return (ru.ru_utime.tv_sec + ru.ru_stime.tv_sec) * 1e6 + ru.ru_utime.tv_usec + ru.ru_stime.tv_usec;
}

std::atomic<double> g_server_cpu_us{0};

void Server(int fd, int busy_poll_us, size_t resp_bytes, std::atomic<bool>* stop) {
  int ep = epoll_create1(0);
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = fd;
  epoll_ctl(ep, EPOLL_CTL_ADD, fd, &ev);
  std::vector<char> buf(1 << 16), resp(resp_bytes, 'r');
  bool spinning = false;
  Clock::time_point until{};
  while (!stop->load(std::memory_order_relaxed)) {
    epoll_event out[4];
    int n = epoll_wait(ep, out, 4, spinning ? 0 : 100);
    if (n <= 0) {
      if (spinning && Clock::now() >= until) spinning = false;
      continue;
    }
    ssize_t r = read(fd, buf.data(), buf.size());
    if (r <= 0) break;
    if (send(fd, resp.data(), resp.size(), MSG_NOSIGNAL) < 0) break;
    if (busy_poll_us > 0) {
      spinning = true;
      until = Clock::now() + std::chrono::microseconds(busy_poll_us);
    }
  }
  close(ep);
  g_server_cpu_us.store(ThreadCpuUs());
}

}  // namespace

int main(int argc, char** argv) {
  int iters = 100000, busy = 50;
  size_t req = 120, resp = 200;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&] { return i + 1 < argc ? argv[++i] : "0"; };
    if (a == "--iters") iters = atoi(next());
    else if (a == "--busy-poll-us") busy = atoi(next());
    else if (a == "--req") req = strtoul(next(), nullptr, 10);
    else if (a == "--resp") resp = strtoul(next(), nullptr, 10);
    else {
      fprintf(stderr, "usage: %s [--iters N] [--busy-poll-us U] [--req B] [--resp B]\n", argv[0]);
      return 2;
    }
  }
  int sv[2];
  if (socketpair(AF_UNIX, SOCK_STREAM | SOCK_NONBLOCK, 0, sv) != 0) return 1;
  std::atomic<bool> stop{false};
  std::thread t(Server, sv[1], busy, resp, &stop);
  std::vector<char> q(req, 'q'), buf(1 << 16);
  std::vector<double> us;
  us.reserve(iters);
  for (int i = 0; i < iters + 1000; ++i) {
    auto t0 = Clock::now();
    if (send(sv[0], q.data(), q.size(), MSG_NOSIGNAL) < 0) return 1;
    size_t got = 0;
    while (got < resp) {
      pollfd p{sv[0], POLLIN, 0};
      poll(&p, 1, 1000);
      ssize_t r = read(sv[0], buf.data(), buf.size());
      if (r > 0) got += static_cast<size_t>(r);
    }
    if (i >= 1000) us.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
  }
  stop.store(true);
  shutdown(sv[0], SHUT_RDWR);
  t.join();
  double client_cpu_us = ThreadCpuUs();
  std::sort(us.begin(), us.end());
  auto pct = [&](double p) { return us[static_cast<size_t>(p / 100.0 * (us.size() - 1))]; };
  printf("{\"iters\": %d, \"busy_poll_us\": %d, \"req_bytes\": %zu, \"resp_bytes\": %zu, \"p50_us\": %.2f, "
         "\"p99_us\": %.2f, \"min_us\": %.2f, \"server_cpu_us_per_req\": %.3f, \"client_cpu_us_per_req\": %.3f}\n",
         iters, busy, req, resp, pct(50), pct(99), us.front(), g_server_cpu_us.load() / (iters + 1000),
         client_cpu_us / (iters + 1000));
  return 0;
}

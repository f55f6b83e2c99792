// amdgpu-dp-kubelet: a native stand-in for the kubelet's device-manager side.
//
//   serve  --kubelet-socket PATH [--plugin-dir DIR]
//          Serves /v1beta1.Registration/Register. For every registration it dials
//          the plugin endpoint, calls GetDevicePluginOptions, opens ListAndWatch
//          and prints one JSON line per event on stdout:
//            {"event":"register", "resource":..., "endpoint":..., "preferred":bool}
//            {"event":"devices", "resource":..., "total":n, "healthy":h, "unhealthy":u}
//            {"event":"stream_end", "resource":..., "status":"..."}
//
//   bench  --socket PATH [--pods N] [--warmup W] [--pod-size K] [--rank R --world W]
//          Synthetic pod churn against a running plugin, the way kubelet drives it
//          at pod admission: GetPreferredAllocation(free devices, K) then
//          Allocate(chosen); pods are retired FIFO once the node is full. Prints
//          one JSON object with client-side latency percentiles.
//
// The reference has no such harness (no fake kubelet, no gRPC
// tests); BASELINE.md §4 defines the metrics this measures.
#include <signal.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "bench/churn.h"
#include "common/strings.h"
#include "grpc/grpc.h"
#include "proto/messages.h"

using namespace adp;

namespace {

std::mutex g_out_mu;
// One JSON object per line, stamped with CLOCK_MONOTONIC microseconds ("t_us").
void Emit(const std::string& line) {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  std::string stamped = "{\"t_us\": " + std::to_string(int64_t(ts.tv_sec) * 1000000 + ts.tv_nsec / 1000) +
                        (line.size() > 2 ? ", " : "") + line.substr(1);
  std::lock_guard<std::mutex> lk(g_out_mu);
  fputs(stamped.c_str(), stdout);
  fputc('\n', stdout);
  fflush(stdout);
}

std::map<std::string, std::string> ParseArgs(int argc, char** argv, int first) {
  std::map<std::string, std::string> m;
  for (int i = first; i < argc; ++i) {
    std::string a = argv[i];
    if (!StartsWith(a, "--")) continue;
    a = a.substr(2);
    size_t eq = a.find('=');
    if (eq != std::string::npos) m[a.substr(0, eq)] = a.substr(eq + 1);
    else if (i + 1 < argc && !StartsWith(argv[i + 1], "--")) m[a] = argv[++i];
    else m[a] = "true";
  }
  return m;
}

std::atomic<bool> g_stop{false};
void OnSignal(int) { g_stop.store(true); }

void WatchPlugin(std::string resource, std::string endpoint_path) {
  auto ch = grpc::Channel::Dial(endpoint_path, 5000);
  if (!ch.ok()) {
    Emit("{\"event\": \"error\", \"resource\": \"" + JsonEscape(resource) + "\", \"message\": \"" +
         JsonEscape(ch.status().ToString()) + "\"}");
    return;
  }
  std::string resp;
  Status st = (*ch)->Unary("/v1beta1.DevicePlugin/GetDevicePluginOptions", "", &resp, 5000);
  pb::DevicePluginOptions opts;
  if (st.ok()) st = pb::Decode(resp, &opts);
  Emit("{\"event\": \"options\", \"resource\": \"" + JsonEscape(resource) + "\", \"ok\": " +
       (st.ok() ? "true" : "false") + ", \"preferred\": " +
       (opts.get_preferred_allocation_available ? "true" : "false") + "}");
  auto sid = (*ch)->StartStream("/v1beta1.DevicePlugin/ListAndWatch", "");
  if (!sid.ok()) return;
  while (!g_stop.load()) {
    std::string msg;
    Status rs = (*ch)->Recv(*sid, &msg, 200);
    if (rs.code() == Code::kDeadlineExceeded) continue;
    if (!rs.ok()) {
      Emit("{\"event\": \"stream_end\", \"resource\": \"" + JsonEscape(resource) + "\", \"status\": \"" +
           JsonEscape(rs.ToString()) + "\"}");
      return;
    }
    pb::ListAndWatchResponse law;
    if (!pb::Decode(msg, &law).ok()) continue;
    size_t healthy = 0;
    std::string numa;
    std::map<int64_t, int> per_numa;
    for (const auto& d : law.devices) {
      if (d.health == pb::kHealthy) ++healthy;
      for (auto n : d.numa_nodes) per_numa[n]++;
    }
    for (const auto& [n, c] : per_numa) numa += (numa.empty() ? "" : ", ") + ("\"" + std::to_string(n) + "\": " + std::to_string(c));
    std::string first = law.devices.empty() ? "" : law.devices.front().id;
    Emit("{\"event\": \"devices\", \"resource\": \"" + JsonEscape(resource) + "\", \"total\": " +
         std::to_string(law.devices.size()) + ", \"healthy\": " + std::to_string(healthy) +
         ", \"unhealthy\": " + std::to_string(law.devices.size() - healthy) + ", \"numa\": {" + numa +
         "}, \"first_id\": \"" + JsonEscape(first) + "\", \"bytes\": " + std::to_string(msg.size()) + "}");
  }
}

int Serve(std::map<std::string, std::string> args) {
  std::string sock = args.count("kubelet-socket") ? args["kubelet-socket"] : "/var/lib/kubelet/device-plugins/kubelet.sock";
  std::string dir = args.count("plugin-dir") ? args["plugin-dir"] : sock.substr(0, sock.rfind('/'));
  signal(SIGINT, OnSignal);
  signal(SIGTERM, OnSignal);
  grpc::Server srv("kubelet-stub");
  std::vector<std::thread> watchers;
  std::mutex mu;
  srv.AddUnary("/v1beta1.Registration/Register", [&](std::string_view req, std::string* resp) {
    pb::RegisterRequest r;
    ADP_RETURN_IF_ERROR(pb::Decode(req, &r));
    if (r.version != pb::kApiVersion)
      return InvalidArgument("Unsupported version: " + r.version);
    Emit("{\"event\": \"register\", \"resource\": \"" + JsonEscape(r.resource_name) + "\", \"endpoint\": \"" +
         JsonEscape(r.endpoint) + "\", \"version\": \"" + JsonEscape(r.version) + "\", \"preferred\": " +
         (r.options.get_preferred_allocation_available ? "true" : "false") + "}");
    std::lock_guard<std::mutex> lk(mu);
    watchers.emplace_back(WatchPlugin, r.resource_name, PathJoin(dir, r.endpoint));
    return Status::Ok();
  });
  Status st = srv.Listen(sock);
  if (st.ok()) st = srv.Start();
  if (!st.ok()) {
    fprintf(stderr, "kubelet-stub: %s\n", st.ToString().c_str());
    return 1;
  }
  Emit("{\"event\": \"listening\", \"socket\": \"" + JsonEscape(sock) + "\"}");
  while (!g_stop.load()) usleep(50 * 1000);
  srv.Stop();
  std::lock_guard<std::mutex> lk(mu);
  for (auto& t : watchers) t.join();
  return 0;
}

int Bench(std::map<std::string, std::string> args) {
  bench::ChurnOptions opt;
  opt.pod_size = args.count("pod-size") ? atoi(args["pod-size"].c_str()) : 1;
  opt.rank = args.count("rank") ? atoi(args["rank"].c_str()) : 0;
  opt.world = args.count("world") ? atoi(args["world"].c_str()) : 1;
  opt.preferred = !args.count("no-preferred");
  int pods = args.count("pods") ? atoi(args["pods"].c_str()) : 2000;
  int warmup = args.count("warmup") ? atoi(args["warmup"].c_str()) : 200;
  auto c = bench::ChurnClient::Open(args["socket"], opt);
  if (!c.ok()) {
    fprintf(stderr, "bench: %s\n", c.status().ToString().c_str());
    return 1;
  }
  Status st = (*c)->Run(warmup, false);
  if (st.ok()) st = (*c)->Run(pods, true);
  if (!st.ok()) {
    fprintf(stderr, "bench: %s\n", st.ToString().c_str());
    return 1;
  }
  Emit((*c)->StatsJson());
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s serve|bench [--flags]\n", argv[0]);
    return 2;
  }
  signal(SIGPIPE, SIG_IGN);
  std::string mode = argv[1];
  auto args = ParseArgs(argc, argv, 2);
  if (mode == "serve") return Serve(args);
  if (mode == "bench") return Bench(args);
  fprintf(stderr, "unknown mode %s\n", mode.c_str());
  return 2;
}

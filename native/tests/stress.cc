// Concurrency stress test for TSan/ASan builds (make tsan / make asan).
//
// One plugin serving 8 mock MI355X GPUs x 4 replicas while, concurrently:
//   * 4 kubelet clients churn GetPreferredAllocation + Allocate,
//   * 1 client keeps a ListAndWatch stream open and reconnects when it drops,
//   * 1 thread flips device health (the monitor's path into the plugin),
//   * 1 thread stops and restarts the plugin (SIGHUP / kubelet-restart path).
// The reference never ran its Go tests with -race and has known races between
// cleanup() and RPC goroutines (server.go:118-125); this is the
// regression test that ours has none.
//
// usage: adp_stress [path/to/libamdsmi_mock.so] [seconds]
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <random>
#include <thread>
#include <vector>

#include "bench/churn.h"
#include "grpc/grpc.h"
#include "inventory/inventory.h"
#include "plugin/plugin.h"
#include "smi/smi.h"
#include "strategy/strategy.h"

using namespace adp;

int main(int argc, char** argv) {
  std::string mock = argc > 1 ? argv[1] : "";
  if (mock.empty()) {
    std::string self = argv[0];
    mock = self.substr(0, self.rfind('/') + 1) + "libamdsmi_mock.so";
  }
  double seconds = argc > 2 ? atof(argv[2]) : 3.0;
  std::string dir = "/tmp/adp-stress-" + std::to_string(getpid());
  mkdir(dir.c_str(), 0755);
  {
    std::ofstream f(dir + "/fx.json");
    f << "{\"gpus\": [";
    for (int i = 0; i < 8; ++i) f << (i ? "," : "") << "{\"numa\": " << (i < 4 ? 0 : 1) << "}";
    f << "]}";
  }
  setenv("AMDSMI_MOCK_FIXTURE", (dir + "/fx.json").c_str(), 1);
  auto lib = smi::Library::Open(mock);
  if (!lib.ok()) {
    fprintf(stderr, "stress: %s\n", lib.status().ToString().c_str());
    return 2;
  }
  auto snap = inventory::BuildSnapshot(lib->get(), {});
  auto rc = strategy::ResourceConfig::Parse("gpu:gpu:4");
  auto specs = strategy::BuildPluginSpecs(**snap, strategy::PartitionStrategy::kNone, *rc);
  plugin::PluginOptions po;
  po.plugin_dir = dir;
  po.register_with_kubelet = false;
  po.dial_timeout_ms = 2000;
  plugin::Plugin p(*snap, (*specs)[0], po);
  if (!p.Start().ok()) return 3;
  std::string sock = p.socket_path();

  std::atomic<bool> stop{false};
  std::atomic<uint64_t> pods{0}, law_msgs{0}, flips{0}, restarts{0}, reconnects{0};
  std::vector<std::thread> ts;
  for (int r = 0; r < 4; ++r) {
    ts.emplace_back([&, r] {
      bench::ChurnOptions o;
      o.rank = r;
      o.world = 4;
      o.timeout_ms = 2000;
      while (!stop.load()) {
        auto c = bench::ChurnClient::Open(sock, o);
        if (!c.ok()) { std::this_thread::sleep_for(std::chrono::milliseconds(5)); continue; }
        while (!stop.load() && (*c)->Run(10, false).ok()) pods += 10;
        ++reconnects;
      }
    });
  }
  ts.emplace_back([&] {
    while (!stop.load()) {
      auto ch = grpc::Channel::Dial(sock, 500);
      if (!ch.ok()) { std::this_thread::sleep_for(std::chrono::milliseconds(5)); continue; }
      auto sid = (*ch)->StartStream("/v1beta1.DevicePlugin/ListAndWatch", "");
      if (!sid.ok()) continue;
      std::string m;
      while (!stop.load()) {
        Status st = (*ch)->Recv(*sid, &m, 50);
        if (st.code() == Code::kDeadlineExceeded) continue;
        if (!st.ok()) break;
        ++law_msgs;
      }
    }
  });
  ts.emplace_back([&] {
    std::mt19937 rng(1);
    while (!stop.load()) {
      p.SetGpuHealth(static_cast<int>(rng() % 8), rng() % 2, "stress");
      ++flips;
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
  });
  ts.emplace_back([&] {
    while (!stop.load()) {
      std::this_thread::sleep_for(std::chrono::milliseconds(150));
      p.Stop();
      if (p.Start().ok()) ++restarts;
    }
  });
  std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
  stop.store(true);
  for (auto& t : ts) t.join();
  p.Stop();
  printf("stress: pods=%llu law_msgs=%llu health_flips=%llu restarts=%llu reconnects=%llu\n",
         (unsigned long long)pods.load(), (unsigned long long)law_msgs.load(),
         (unsigned long long)flips.load(), (unsigned long long)restarts.load(),
         (unsigned long long)reconnects.load());
  unlink((dir + "/fx.json").c_str());
  rmdir(dir.c_str());
  return (pods.load() > 0 && law_msgs.load() > 0 && restarts.load() > 0) ? 0 : 1;
}

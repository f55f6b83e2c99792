// Synthetic pod churn against a running device plugin -- the Allocate() latency
// benchmark of BASELINE.md §4.
//
// A pod admission is what kubelet's device manager does for a container that
// requests K devices: GetPreferredAllocation(free devices, K) when the plugin
// offers it, then Allocate(chosen). Pods are retired FIFO when the node is
// full, so the free set keeps changing (churn). Latencies are client-side wall
// times of each unary RPC on one persistent HTTP/2 connection, which is how
// kubelet talks to a plugin.
#pragma once

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "common/status.h"
#include "grpc/grpc.h"

namespace adp::bench {

struct ChurnOptions {
  int pod_size = 1;
  bool preferred = true;
  int rank = 0;   // this client churns devices i with i % world == rank ...
  int world = 1;
  // ... unless `owned` is set: then exactly the advertised devices whose
  // physical ID (replica suffix stripped) is listed -- the rank's own GPU.
  std::vector<std::string> owned;
  int timeout_ms = 5000;
  bool grpc_go = false;  // kubelet (grpc-go) client frame pattern, grpc::Channel::EmulateGrpcGo
};

struct LatencyStats {
  size_t n = 0;
  double p50 = 0, p90 = 0, p99 = 0, mean = 0, min = 0, max = 0;  // microseconds
};
LatencyStats Summarize(std::vector<double> us);
std::string ToJson(const char* name, const LatencyStats& s);

class ChurnClient {
 public:
  static Result<std::unique_ptr<ChurnClient>> Open(const std::string& socket, const ChurnOptions& opt);

  size_t advertised() const { return advertised_; }
  size_t allocatable() const { return allocatable_; }
  size_t rank_devices() const { return mine_; }

  // Admits `pods` pods; latencies are kept when `record` is true.
  Status Run(int pods, bool record);
  void ResetStats();
  std::string StatsJson() const;
  const std::vector<double>& allocate_us() const { return alloc_us_; }

 private:
  ChurnClient() = default;
  std::unique_ptr<grpc::Channel> ch_;
  ChurnOptions opt_;
  size_t advertised_ = 0, allocatable_ = 0, mine_ = 0;
  std::vector<std::string> free_;
  std::vector<std::string> mine_ids_;  // physical device IDs this rank churns (replica suffix stripped)
  std::vector<std::vector<std::string>> live_;  // FIFO of admitted pods
  size_t live_head_ = 0;
  std::vector<double> alloc_us_, pref_us_, pod_us_;
  double run_seconds_ = 0;
  size_t run_pods_ = 0;
  std::map<int, int> cpus_;  // CPU this client ran on, sampled every 64 recorded pods
};

}  // namespace adp::bench

// Observability: lock-free latency histograms and a Prometheus text endpoint.
//
// The reference has no metrics (Go `log` lines only). Here every
// plugin keeps per-RPC handler-time histograms (atomic bucket counters, one
// relaxed increment per call -- nothing on the Allocate path blocks), dumped by
// SIGUSR1 and, when --metrics-addr is set, served as Prometheus text on
// GET /metrics together with per-device health and build info. GET /healthz
// answers 200 while every plugin that has devices is serving (a DaemonSet
// liveness probe).
#pragma once

#include <atomic>
#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "common/status.h"

namespace adp::metrics {

// Counters written on the RPC path are sharded per thread: with N server loops
// serving concurrent clients, one shared cache line per counter would bounce
// between cores on every call. A thread gets a shard index round-robin on first
// use; readers sum the shards.
constexpr int kShards = 16;
int ShardIndex();

class Counter {
 public:
  void Add(uint64_t n) { s_[ShardIndex()].v.fetch_add(n, std::memory_order_relaxed); }
  uint64_t Value() const;

 private:
  struct alignas(64) Slot { std::atomic<uint64_t> v{0}; };
  Slot s_[kShards];
};

class MaxGauge {
 public:
  void Observe(uint64_t v);
  uint64_t Value() const;

 private:
  struct alignas(64) Slot { std::atomic<uint64_t> v{0}; };
  Slot s_[kShards];
};

// Fixed 1-2-5 buckets from 250 ns to 1 s (upper bounds, seconds); sharded.
class Histogram {
 public:
  static constexpr int kBuckets = 20;
  static const double kBoundsSec[kBuckets];

  void Observe(uint64_t ns);
  uint64_t count() const;
  double sum_seconds() const;
  // Upper bound of the bucket holding quantile q (0 if empty), in microseconds.
  double QuantileUs(double q) const;
  // Appends `name_bucket{labels,le=..}`, `name_sum`, `name_count` lines.
  void AppendPrometheus(const std::string& name, const std::string& labels, std::string* out) const;

 private:
  struct alignas(64) Shard {
    std::atomic<uint64_t> buckets[kBuckets + 1] = {};  // last = +Inf
    std::atomic<uint64_t> sum_ns{0};
  };
  void Totals(uint64_t counts[kBuckets + 1]) const;
  Shard shards_[kShards];
};

// The microsecond regime at full resolution: 100 ns bins up to 102.4 us plus
// one overflow bin, sharded like Histogram (each loop thread writes its own
// shard). Holds the gRPC server's per-call residency, whose interesting range
// (1-10 us) the 1-2-5 buckets above would cover with three buckets.
class FineHistogram {
 public:
  static constexpr int kBins = 1024;
  static constexpr uint64_t kBinNs = 100;

  FineHistogram();
  void Observe(uint64_t ns);
  // Merged counts, kBins + 1 entries (the last is >= 102.4 us).
  std::vector<uint64_t> Counts() const;
  uint64_t sum_ns() const;
  // Upper edge (us) of the bin holding quantile q of `counts` (0 if empty).
  static double QuantileUs(const std::vector<uint64_t>& counts, double q);
  // `[[bin, count], ...]` over the nonzero bins (bin b covers [b, b+1) x 100 ns).
  std::string SparseJson() const;
  // Prometheus histogram with Histogram's bucket bounds from 1 us to 100 us.
  void AppendPrometheus(const std::string& name, const std::string& labels, std::string* out) const;

 private:
  struct Shard {
    std::atomic<uint64_t> bins[kBins + 1] = {};
    std::atomic<uint64_t> sum_ns{0};
  };
  std::unique_ptr<Shard[]> shards_;
};

// Escapes a Prometheus label value (backslash, quote, newline).
std::string LabelValue(const std::string& v);

// Minimal HTTP/1.1 server for /metrics and /healthz on one TCP address.
class HttpServer {
 public:
  using Render = std::function<std::string()>;
  using Healthy = std::function<bool()>;
  // `stats` (optional) answers GET /stats with JSON: the SIGUSR1 counters for
  // tools that would otherwise parse the log.
  HttpServer(Render render, Healthy healthy, Render stats = nullptr);
  ~HttpServer();
  // addr: "host:port", ":port" (all interfaces) or "port", or several of them
  // comma separated (e.g. the pod IP and loopback: kubectl port-forward and
  // in-pod tools dial 127.0.0.1). Port 0 picks a free port. port() is the
  // first address's.
  Status Start(const std::string& addr);
  void Stop();
  int port() const { return port_; }

 private:
  void Run();
  std::string Respond(const std::string& request);
  Render render_;
  Healthy healthy_;
  Render stats_;
  Status Listen(const std::string& addr);
  std::vector<int> listen_fds_;
  int stop_fd_ = -1;
  int spare_fd_ = -1;  // reserve descriptor: shed connections at EMFILE instead of spinning
  int port_ = 0;
  std::thread thread_;
};

}  // namespace adp::metrics

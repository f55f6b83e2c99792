#include "bench/churn.h"

#include <sched.h>

#include "alloc/replicas.h"
#include "common/strings.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>

#include "proto/messages.h"

namespace adp::bench {
namespace {
using Clock = std::chrono::steady_clock;
double Us(Clock::time_point a, Clock::time_point b) {
  return std::chrono::duration<double, std::micro>(b - a).count();
}
double Pct(const std::vector<double>& v, double p) {
  double idx = p / 100.0 * (v.size() - 1);
  size_t lo = static_cast<size_t>(std::floor(idx)), hi = static_cast<size_t>(std::ceil(idx));
  return v[lo] + (v[hi] - v[lo]) * (idx - lo);
}
}  // namespace

LatencyStats Summarize(std::vector<double> us) {
  LatencyStats s;
  s.n = us.size();
  if (us.empty()) return s;
  std::sort(us.begin(), us.end());
  double sum = 0;
  for (double x : us) sum += x;
  s.p50 = Pct(us, 50);
  s.p90 = Pct(us, 90);
  s.p99 = Pct(us, 99);
  s.mean = sum / us.size();
  s.min = us.front();
  s.max = us.back();
  return s;
}

std::string ToJson(const char* name, const LatencyStats& s) {
  char buf[320];
  snprintf(buf, sizeof(buf),
           "\"%s\": {\"n\": %zu, \"p50_us\": %.2f, \"p90_us\": %.2f, \"p99_us\": %.2f, \"mean_us\": %.2f, "
           "\"min_us\": %.2f, \"max_us\": %.2f}",
           name, s.n, s.p50, s.p90, s.p99, s.mean, s.min, s.max);
  return buf;
}

Result<std::unique_ptr<ChurnClient>> ChurnClient::Open(const std::string& socket, const ChurnOptions& opt) {
  std::unique_ptr<ChurnClient> c(new ChurnClient());
  c->opt_ = opt;
  auto ch = grpc::Channel::Dial(socket, opt.timeout_ms);
  if (!ch.ok()) return ch.status();
  c->ch_ = std::move(*ch);
  c->ch_->EmulateGrpcGo(opt.grpc_go);
  auto sid = c->ch_->StartStream("/v1beta1.DevicePlugin/ListAndWatch", "");
  if (!sid.ok()) return sid.status();
  std::string msg;
  ADP_RETURN_IF_ERROR(c->ch_->Recv(*sid, &msg, opt.timeout_ms));
  pb::ListAndWatchResponse law;
  ADP_RETURN_IF_ERROR(pb::Decode(msg, &law));
  c->advertised_ = law.devices.size();
  for (size_t i = 0; i < law.devices.size(); ++i) {
    if (law.devices[i].health == pb::kHealthy) ++c->allocatable_;
    bool mine = opt.owned.empty()
                    ? static_cast<int>(i % opt.world) == opt.rank
                    : std::find(opt.owned.begin(), opt.owned.end(), alloc::StripReplica(law.devices[i].id)) !=
                          opt.owned.end();
    if (mine && law.devices[i].health == pb::kHealthy) c->free_.push_back(law.devices[i].id);
  }
  c->mine_ = c->free_.size();
  c->mine_ids_ = alloc::StripReplicas(c->free_);
  if (c->mine_ < static_cast<size_t>(opt.pod_size))
    return FailedPrecondition("only " + std::to_string(c->mine_) + " healthy devices for rank " +
                              std::to_string(opt.rank) + ", pod size " + std::to_string(opt.pod_size));
  return c;
}

void ChurnClient::ResetStats() {
  alloc_us_.clear();
  pref_us_.clear();
  pod_us_.clear();
  run_seconds_ = 0;
  run_pods_ = 0;
  cpus_.clear();
}

Status ChurnClient::Run(int pods, bool record) {
  const size_t k = static_cast<size_t>(opt_.pod_size);
  std::string req, resp;
  auto t_run = Clock::now();
  for (int i = 0; i < pods; ++i) {
    if (free_.size() < k) {  // node full: retire the oldest pod
      for (auto& id : live_[live_head_]) free_.push_back(std::move(id));
      ++live_head_;
      if (live_head_ > 4096) {
        live_.erase(live_.begin(), live_.begin() + live_head_);
        live_head_ = 0;
      }
    }
    auto p0 = Clock::now();
    std::vector<std::string> chosen;
    if (opt_.preferred) {
      pb::PreferredAllocationRequest pr;
      pr.container_requests.emplace_back();
      pr.container_requests[0].available = free_;
      pr.container_requests[0].allocation_size = static_cast<int32_t>(k);
      req.clear();
      pb::Encode(pr, &req);
      auto a0 = Clock::now();
      ADP_RETURN_IF_ERROR(ch_->Unary("/v1beta1.DevicePlugin/GetPreferredAllocation", req, &resp, opt_.timeout_ms));
      auto a1 = Clock::now();
      ADP_RETURN_IF_ERROR(ch_->SendBdpPing());
      pb::PreferredAllocationResponse prr;
      ADP_RETURN_IF_ERROR(pb::Decode(resp, &prr));
      if (!prr.container_responses.empty()) chosen = std::move(prr.container_responses[0]);
      if (record) pref_us_.push_back(Us(a0, a1));
    }
    if (chosen.size() != k) chosen.assign(free_.begin(), free_.begin() + k);
    for (const auto& id : chosen) {
      auto it = std::find(free_.begin(), free_.end(), id);
      if (it == free_.end()) return Internal("preferred allocation returned a non-free device " + id);
      free_.erase(it);
    }
    pb::AllocateRequest ar;
    ar.container_requests.push_back(chosen);
    req.clear();
    pb::Encode(ar, &req);
    auto a0 = Clock::now();
    ADP_RETURN_IF_ERROR(ch_->Unary("/v1beta1.DevicePlugin/Allocate", req, &resp, opt_.timeout_ms));
    auto a1 = Clock::now();
    ADP_RETURN_IF_ERROR(ch_->SendBdpPing());
    pb::AllocateResponse arr;
    ADP_RETURN_IF_ERROR(pb::Decode(resp, &arr));
    if (arr.container_responses.size() != 1 || arr.container_responses[0].devices.empty())
      return Internal("Allocate response without device specs");
    if (record) {
      alloc_us_.push_back(Us(a0, a1));
      pod_us_.push_back(Us(p0, a1));
    }
    live_.push_back(std::move(chosen));
    if (record && (i & 63) == 0) ++cpus_[sched_getcpu()];
  }
  if (record) {
    run_seconds_ += std::chrono::duration<double>(Clock::now() - t_run).count();
    run_pods_ += pods;
  }
  return Status::Ok();
}

std::string ChurnClient::StatsJson() const {
  char head[400];
  snprintf(head, sizeof(head),
           "{\"rank\": %d, \"world\": %d, \"advertised\": %zu, \"allocatable\": %zu, \"rank_devices\": %zu, "
           "\"pod_size\": %d, \"pods\": %zu, \"seconds\": %.6f, \"pods_per_s\": %.1f, "
           "\"client\": \"%s\", \"bdp_pings\": %llu, ",
           opt_.rank, opt_.world, advertised_, allocatable_, mine_, opt_.pod_size, run_pods_, run_seconds_,
           run_seconds_ > 0 ? run_pods_ / run_seconds_ : 0.0, opt_.grpc_go ? "grpc-go" : "native",
           static_cast<unsigned long long>(ch_->bdp_pings_sent()));
  std::string ids = "\"device_ids\": [";
  for (size_t i = 0; i < mine_ids_.size() && i < 64; ++i)
    ids += (i ? ", \"" : "\"") + JsonEscape(mine_ids_[i]) + "\"";
  ids += "], ";
  std::string cpus = "\"cpus\": {";
  for (const auto& [cpu, n] : cpus_) cpus += (cpus.size() > 9 ? ", \"" : "\"") + std::to_string(cpu) + "\": " + std::to_string(n);
  cpus += "}, ";
  return std::string(head) + ids + cpus + ToJson("allocate", Summarize(alloc_us_)) + ", " +
         ToJson("preferred", Summarize(pref_us_)) + ", " + ToJson("pod", Summarize(pod_us_)) + "}";
}

}  // namespace adp::bench

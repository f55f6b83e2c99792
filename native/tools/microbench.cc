// In-process microbenchmarks of the RPC handlers (no transport): how long the
// daemon spends inside Allocate / GetPreferredAllocation / a ListAndWatch
// rebuild for the node shapes of BASELINE.json. Prints one JSON object.
//
// usage: adp_microbench [iterations]
#include <stdlib.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "inventory/inventory.h"
#include "node_model.h"
#include "plugin/plugin.h"
#include "proto/messages.h"
#include "strategy/strategy.h"

using namespace adp;
using Clock = std::chrono::steady_clock;

namespace {

template <typename Fn>
double TimeUs(int iters, Fn fn) {
  auto t0 = Clock::now();
  for (int i = 0; i < iters; ++i) fn();
  return std::chrono::duration<double, std::micro>(Clock::now() - t0).count() / iters;
}

}  // namespace

int main(int argc, char** argv) {
  int iters = argc > 1 ? atoi(argv[1]) : 2000;
  struct Case {
    const char* name;
    int gpus, parts;
    strategy::PartitionStrategy ps;
    const char* rc;
    alloc::ReplicaPolicy pol;
    int k;
    bool enforce = false;  // --enforce-memory-units (the shim mount + read-only grant files)
    bool usage_files = false;  // ... + grant accounting files (written to a scratch dir)
  };
  std::vector<Case> cases = {
      {"spx8_none", 8, 1, strategy::PartitionStrategy::kNone, "", alloc::ReplicaPolicy::kSpread, 1},
      {"spx8_none_k4", 8, 1, strategy::PartitionStrategy::kNone, "", alloc::ReplicaPolicy::kSpread, 4},
      {"spx8_timeslice4", 8, 1, strategy::PartitionStrategy::kNone, "gpu:sharedgpu:4", alloc::ReplicaPolicy::kSpread, 1},
      {"cpx64_single_k4", 8, 8, strategy::PartitionStrategy::kSingle, "", alloc::ReplicaPolicy::kSpread, 4},
      {"automem2352_spread_k1", 8, 1, strategy::PartitionStrategy::kNone, "gpu:gpu-mem-gb:-1", alloc::ReplicaPolicy::kSpread, 1},
      {"automem2352_pack_k36", 8, 1, strategy::PartitionStrategy::kNone, "gpu:gpu-mem-gb:-1", alloc::ReplicaPolicy::kPack, 36},
      {"automem2352_enforced_k1", 8, 1, strategy::PartitionStrategy::kNone, "gpu:gpu-mem-gb:-1", alloc::ReplicaPolicy::kPack, 1,
       true},
      {"automem2352_enforced_usage_k1", 8, 1, strategy::PartitionStrategy::kNone, "gpu:gpu-mem-gb:-1",
       alloc::ReplicaPolicy::kPack, 1, true, true},
  };
  char scratch[] = "/tmp/adp-microbench-XXXXXX";
  const char* root = mkdtemp(scratch);
  if (!root) {
    perror("mkdtemp");
    return 2;
  }
  std::string usage_dir = std::string(root) + "/usage";
  printf("{");
  bool first = true;
  for (const auto& c : cases) {
    auto snap = testing::NodeModel(c.gpus, c.parts);
    auto rc = strategy::ResourceConfig::Parse(c.rc);
    auto specs = strategy::BuildPluginSpecs(*snap, c.ps, *rc);
    plugin::PluginOptions po;
    po.register_with_kubelet = false;
    po.replica_policy = c.pol;
    if (c.enforce) {
      po.memcap_host_path = "/nonexistent/libadp_memcap.so";  // only named in the responses
      if (c.usage_files) po.memcap_usage_dir = usage_dir;
    }
    plugin::Plugin p(snap, (*specs)[0], po);
    const auto& ids = p.advertised_ids();
    // GetPreferredAllocation with every advertised device free (a fresh node).
    pb::PreferredAllocationRequest pr;
    pr.container_requests.push_back({ids, {}, c.k});
    std::string preq = pb::Encode(pr), presp;
    double pref_us = TimeUs(iters / 4 + 1, [&] { presp.clear(); p.HandlePreferred(preq, &presp); });
    pb::PreferredAllocationResponse prr;
    pb::Decode(presp, &prr);
    // Allocate the preferred set.
    pb::AllocateRequest ar;
    ar.container_requests.push_back(prr.container_responses.at(0));
    std::string areq = pb::Encode(ar), aresp;
    double alloc_us = TimeUs(iters, [&] { aresp.clear(); p.HandleAllocate(areq, &aresp); });
    std::vector<pb::ContainerPreferredAllocationRequestView> x;  // reused, as the handler does
    double decode_us = TimeUs(iters / 4 + 1, [&] { pb::DecodeView(preq, &x); });
    double prio_us = 0;
    if (p.replicated()) {
      std::vector<std::string_view> views(ids.begin(), ids.end());
      prio_us = TimeUs(iters / 4 + 1, [&] { alloc::PrioritizeDeviceViews(views, {}, c.k, c.pol); });
    }
    printf("%s\n \"%s_parts\": {\"decode_view_us\": %.3f, \"prioritize_us\": %.3f}", first ? "" : ",", c.name,
           decode_us, prio_us);
    first = false;
    printf("%s\n \"%s\": {\"advertised\": %zu, \"k\": %d, \"preferred_us\": %.3f, \"preferred_request_bytes\": %zu, "
           "\"preferred_decode_us\": %.3f, \"allocate_us\": %.3f, \"allocate_response_bytes\": %zu}",
           first ? "" : ",", c.name, ids.size(), c.k, pref_us, preq.size(), decode_us, alloc_us, aresp.size());
    first = false;
  }
  printf("\n}\n");
  return 0;
}

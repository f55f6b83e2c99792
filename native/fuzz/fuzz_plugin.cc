// Coverage-guided fuzzing (libFuzzer) of the kubelet-facing RPC handlers:
// Allocate, GetPreferredAllocation and PreStartContainer of the plugins the
// daemon builds for BASELINE.json's node shapes (8 x SPX; 4 time-slice
// replicas per GPU; 64 CPX partitions; 2,352 memory units, spread and pack;
// CU shares of time-slice replicas and of memory units, proportional and whole).
//
// Two kinds of input: raw request bytes (the protobuf decoder and every error
// path), and a request built from the input over the plugin's own advertised
// IDs, whose answer is checked:
//   * GetPreferredAllocation: every returned ID is advertised, available and
//     returned once; must-include IDs are all in it; its size is the requested
//     one; the same request answered again (a best-effort cache hit for up to
//     8 devices) gives the same answer.
//   * Allocate: OK exactly when every ID is advertised, one container response
//     per container request, /dev/kfd in every response; an HSA_CU_MASK names
//     each agent once, in order, with ascending, disjoint, XCD-aligned ranges
//     inside the device's CUs.
// The reference's equivalents panic on a required list longer than the
// request (B12) and answer bare UUIDs for replicated resources (B6).
#include <fuzzer/FuzzedDataProvider.h>

#include <algorithm>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "../tools/node_model.h"
#include "common/log.h"
#include "plugin/plugin.h"
#include "proto/messages.h"
#include "strategy/strategy.h"

using namespace adp;

namespace {

struct Shape {
  int gpus, parts;
  strategy::PartitionStrategy ps;
  const char* rc;
  alloc::ReplicaPolicy pol;
  bool cu_mask = false, whole = false;
};

std::vector<std::unique_ptr<plugin::Plugin>>& Plugins() {
  static auto* all = [] {
    SetLogLevel(LogLevel::kError);
    auto* v = new std::vector<std::unique_ptr<plugin::Plugin>>();
    const Shape shapes[] = {
        {8, 1, strategy::PartitionStrategy::kNone, "", alloc::ReplicaPolicy::kSpread},
        {8, 1, strategy::PartitionStrategy::kNone, "gpu:sharedgpu:4", alloc::ReplicaPolicy::kSpread},
        {8, 8, strategy::PartitionStrategy::kSingle, "", alloc::ReplicaPolicy::kSpread},
        {8, 1, strategy::PartitionStrategy::kNone, "gpu:gpu-mem-gb:-1", alloc::ReplicaPolicy::kSpread},
        {8, 1, strategy::PartitionStrategy::kNone, "gpu:gpu-mem-gb:-1", alloc::ReplicaPolicy::kPack},
        {2, 1, strategy::PartitionStrategy::kNone, "gpu:gpu:3", alloc::ReplicaPolicy::kPack},
        {8, 1, strategy::PartitionStrategy::kNone, "gpu:sharedgpu:4", alloc::ReplicaPolicy::kSpread, true},
        {8, 1, strategy::PartitionStrategy::kNone, "gpu:gpu-mem-gb:-1", alloc::ReplicaPolicy::kPack, true},
        {8, 1, strategy::PartitionStrategy::kNone, "gpu:gpu-mem-gb:-1", alloc::ReplicaPolicy::kPack, true, true},
    };
    for (const auto& s : shapes) {
      auto snap = testing::NodeModel(s.gpus, s.parts);
      auto rc = strategy::ResourceConfig::Parse(s.rc);
      auto specs = strategy::BuildPluginSpecs(*snap, s.ps, *rc);
      plugin::PluginOptions po;
      po.register_with_kubelet = false;
      po.replica_policy = s.pol;
      po.replica_cu_mask = s.cu_mask;
      po.whole_cu_slots = s.whole;
      v->push_back(std::make_unique<plugin::Plugin>(snap, (*specs)[0], po));
    }
    return v;
  }();
  return *all;
}

std::string g_context;  // the request and answer under check, printed on failure

[[noreturn]] void Fail(const char* what) {
  fprintf(stderr, "invariant violated: %s\n%s\n", what, g_context.c_str());
  abort();
}

std::string Join(const std::vector<std::string>& v) {
  std::string s;
  for (const auto& x : v) s += (s.empty() ? "" : " ") + x;
  return s;
}

// Picks IDs: mostly advertised ones, sometimes an unknown or a mangled one.
std::string PickId(FuzzedDataProvider& in, const std::vector<std::string>& ids, bool* unknown) {
  uint8_t kind = in.ConsumeIntegral<uint8_t>();
  const std::string& base = ids[in.ConsumeIntegralInRange<size_t>(0, ids.size() - 1)];
  if (kind < 240) return base;
  std::string id = kind < 248 ? base + "x" : in.ConsumeRandomLengthString(80);
  // (a random string may still be one of ours)
  if (std::find(ids.begin(), ids.end(), id) == ids.end())
    *unknown = true;
  return id;
}

void CheckPreferred(plugin::Plugin& p, FuzzedDataProvider& in) {
  const auto& ids = p.advertised_ids();
  pb::PreferredAllocationRequest req;
  int containers = in.ConsumeIntegralInRange<int>(1, 3);
  bool unknown = false;
  for (int c = 0; c < containers; ++c) {
    pb::ContainerPreferredAllocationRequest cr;
    size_t navail = in.ConsumeIntegralInRange<size_t>(0, std::min<size_t>(ids.size(), 96));
    if (in.ConsumeBool() && ids.size() <= 96) {
      cr.available = ids;  // a fresh node: everything free
    } else {
      for (size_t i = 0; i < navail; ++i) cr.available.push_back(PickId(in, ids, &unknown));
    }
    size_t nmust = in.ConsumeIntegralInRange<size_t>(0, 4);
    for (size_t i = 0; i < nmust && !cr.available.empty(); ++i)
      cr.must_include.push_back(
          cr.available[in.ConsumeIntegralInRange<size_t>(0, cr.available.size() - 1)]);
    cr.allocation_size = in.ConsumeIntegralInRange<int32_t>(-1, 12);
    req.container_requests.push_back(std::move(cr));
  }
  std::string wire = pb::Encode(req), resp, again;
  Status st = p.HandlePreferred(wire, &resp);
  if (!st.ok()) return;  // refusals are fine; crashes and wrong answers are not
  pb::PreferredAllocationResponse out;
  if (!pb::Decode(resp, &out).ok()) Fail("preferred response does not decode");
  g_context.clear();
  for (size_t c = 0; c < req.container_requests.size() && c < out.container_responses.size(); ++c) {
    const auto& cr = req.container_requests[c];
    g_context += "available: " + Join(cr.available) + "\nmust: " + Join(cr.must_include) + "\nsize: " +
                 std::to_string(cr.allocation_size) + "\nanswer: " + Join(out.container_responses[c]) + "\n";
  }
  if (out.container_responses.size() != req.container_requests.size()) Fail("one response per container");
  std::set<std::string> advertised(ids.begin(), ids.end());
  for (size_t c = 0; c < out.container_responses.size(); ++c) {
    const auto& got = out.container_responses[c];
    const auto& cr = req.container_requests[c];
    std::set<std::string> avail(cr.available.begin(), cr.available.end());
    std::set<std::string> uniq(got.begin(), got.end());
    if (uniq.size() != got.size()) Fail("an ID returned twice");
    for (const auto& id : got) {
      if (!advertised.count(id)) Fail("returned an ID the plugin never advertised");
      if (!avail.count(id)) Fail("returned an ID that is not available");
    }
    if (!got.empty()) {
      if (static_cast<int32_t>(got.size()) != cr.allocation_size) Fail("wrong number of IDs");
      for (const auto& m : cr.must_include)
        if (!uniq.count(m)) Fail("a must-include ID is missing");
    }
  }
  if (!p.HandlePreferred(wire, &again).ok() || again != resp) Fail("same request, different answer");
}

// HSA_CU_MASK="<agent>:<lo>-<hi>,...;...": agents ascending, each once;
// ranges ascending, disjoint, non-adjacent (adjacent ones merge), whole slots
// (one CU per XCD) inside the device.
void CheckCuMask(const plugin::Plugin& p, const pb::ContainerAllocateResponse& cr) {
  auto it = std::find_if(cr.envs.begin(), cr.envs.end(), [](const auto& kv) { return kv.first == "HSA_CU_MASK"; });
  if (it == cr.envs.end()) return;
  const std::string& m = it->second;
  const auto& u0 = p.units().front();
  long last_agent = -1;
  for (size_t b = 0; b < m.size();) {
    size_t e = std::min(m.find(';', b), m.size());
    std::string part = m.substr(b, e - b);
    b = e + 1;
    size_t colon = part.find(':');
    if (colon == std::string::npos || colon == 0) Fail("HSA_CU_MASK agent without ':'");
    long agent = strtol(part.substr(0, colon).c_str(), nullptr, 10);
    if (agent <= last_agent) Fail("HSA_CU_MASK agents not ascending");
    last_agent = agent;
    long prev_hi = -2;
    for (size_t rb = colon + 1; rb <= part.size();) {
      size_t re = std::min(part.find(',', rb), part.size());
      std::string r = part.substr(rb, re - rb);
      rb = re + 1;
      size_t dash = r.find('-');
      if (dash == std::string::npos) Fail("HSA_CU_MASK range without '-'");
      long lo = strtol(r.substr(0, dash).c_str(), nullptr, 10), hi = strtol(r.substr(dash + 1).c_str(), nullptr, 10);
      if (lo > hi || lo <= prev_hi + 1) Fail("HSA_CU_MASK ranges not ascending and disjoint");
      if (lo % u0.xcds != 0 || (hi + 1) % u0.xcds != 0) Fail("HSA_CU_MASK range not XCD-aligned");
      if (hi >= static_cast<long>(u0.cus)) Fail("HSA_CU_MASK range past the device's CUs");
      prev_hi = hi;
    }
  }
}

void CheckAllocate(plugin::Plugin& p, FuzzedDataProvider& in) {
  const auto& ids = p.advertised_ids();
  pb::AllocateRequest req;
  int containers = in.ConsumeIntegralInRange<int>(1, 3);
  bool unknown = false;
  for (int c = 0; c < containers; ++c) {
    std::vector<std::string> cids;
    size_t n = in.ConsumeIntegralInRange<size_t>(0, 40);
    for (size_t i = 0; i < n; ++i) cids.push_back(PickId(in, ids, &unknown));
    req.container_requests.push_back(std::move(cids));
  }
  std::string resp;
  g_context.clear();
  for (const auto& c : req.container_requests) g_context += "container: " + Join(c) + "\n";
  Status st = p.HandleAllocate(pb::Encode(req), &resp);
  bool any_empty = false;
  for (const auto& c : req.container_requests) any_empty = any_empty || c.empty();
  if (!unknown && !any_empty && !st.ok()) Fail("Allocate of advertised IDs refused");
  if (unknown && st.ok()) Fail("Allocate of an unknown ID accepted");
  if (!st.ok()) return;
  pb::AllocateResponse out;
  if (!pb::Decode(resp, &out).ok()) Fail("allocate response does not decode");
  if (out.container_responses.size() != req.container_requests.size()) Fail("one response per container");
  for (size_t c = 0; c < out.container_responses.size(); ++c) {
    const auto& cr = out.container_responses[c];
    bool kfd = std::any_of(cr.devices.begin(), cr.devices.end(),
                           [](const pb::DeviceSpec& d) { return d.container_path == "/dev/kfd"; });
    if (!kfd) Fail("no /dev/kfd in an Allocate response");
    CheckCuMask(p, cr);
    // Memory units: the grant is 1000 MiB per distinct ID, whatever is repeated.
    auto mib = std::find_if(cr.envs.begin(), cr.envs.end(),
                            [](const auto& kv) { return kv.first == "AMD_GPU_MEMORY_LIMIT_MIB"; });
    if (p.resource_name().find("gpu-mem-gb") != std::string::npos && !req.container_requests[c].empty()) {
      if (mib == cr.envs.end()) Fail("memory units without AMD_GPU_MEMORY_LIMIT_MIB");
      std::set<std::string> distinct(req.container_requests[c].begin(), req.container_requests[c].end());
      uint64_t total = 0;
      for (size_t b = 0; b <= mib->second.size();) {
        size_t e = std::min(mib->second.find(',', b), mib->second.size());
        total += strtoull(mib->second.substr(b, e - b).c_str(), nullptr, 10);
        b = e + 1;
      }
      if (total != 1000 * distinct.size()) Fail("granted MiB != 1000 x distinct memory units");
    }
  }
}

}  // namespace

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  if (size < 2) return 0;
  auto& plugins = Plugins();
  plugin::Plugin& p = *plugins[data[0] % plugins.size()];
  uint8_t mode = data[1] % 5;
  std::string_view raw(reinterpret_cast<const char*>(data + 2), size - 2);
  std::string resp;
  FuzzedDataProvider in(data + 2, size - 2);
  switch (mode) {
    case 0: (void)p.HandleAllocate(raw, &resp); break;
    case 1: (void)p.HandlePreferred(raw, &resp); break;
    case 2: (void)p.HandlePreStart(raw, &resp); break;
    case 3: CheckPreferred(p, in); break;
    default: CheckAllocate(p, in); break;
  }
  return 0;
}

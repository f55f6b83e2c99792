// Coverage-guided fuzzing (libFuzzer) of the kubelet-facing RPC handlers --
// Allocate, GetPreferredAllocation, PreStartContainer -- over the plugin's
// option space, not a fixed list of shapes (round-6 review item 5). The first
// five input bytes choose the plugin:
//   node       1/2/4/8 GPUs, SPX or CPX (2 or 8 partitions), KFD nodes
//              unreported / in enumeration order / reversed
//   strategy   partition strategy none/single/mixed, and which of its plugins
//              (mixed: one per partition profile plus the whole GPUs)
//   resources  resource-config: whole devices, time-slice replicas (2, 3, 4;
//              with a per-entry policy), memory units (spread / pack)
//   options    --device-id-strategy uuid/index, --device-list-strategy
//              envvar/volume-mounts/cdi-annotations/cdi-cri,
//              --pass-device-specs, --replica-cu-mask, --memory-unit-cu-slots
//              whole, --auto-replica-unit cu-slot, --replica-hbm-share,
//              --replica-policy, --enforce-memory-units, --reject-unhealthy
//   health     which GPUs are Unhealthy
// (plugins built once per option set, kept in a bounded cache). The rest of
// the input is raw request bytes (the protobuf decoder and every error path)
// or a request built over the plugin's own advertised IDs, whose answer is
// checked:
//   * GetPreferredAllocation: every returned ID advertised, available, once;
//     must-include IDs in it; the requested size; the same answer again.
//   * Allocate: OK exactly when every ID is advertised -- and, with
//     --reject-unhealthy, none names an Unhealthy device; one response per
//     container; the device specs (/dev/kfd + every device's node) exactly
//     with --pass-device-specs; under the index strategy AMD_VISIBLE_DEVICES
//     in KFD order; one volume mount per device (volume-mounts), one CDI name
//     per device (cdi-*); AMD_GPU_MEMORY_{LIMIT_MIB,FRACTION,DEVICES} one
//     entry per device in KFD order, the limit = distinct IDs x unit grant,
//     at most the device's HBM, the fraction at most 1; with the HBM-cap shim
//     its preload and one grant mount per device; an HSA_CU_MASK naming each
//     agent once, in order, with ascending, disjoint, XCD-aligned ranges.
// Reference: server.go:316-353 (Allocate), :268-313 (GetPreferredAllocation);
// it panics on a required list longer than the request (B12) and answers
// bare UUIDs for replicated resources (B6).
#include <fuzzer/FuzzedDataProvider.h>

#include <algorithm>
#include <cstring>
#include <map>
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

struct Built {
  std::unique_ptr<plugin::Plugin> plugin;
  plugin::PluginOptions opts;
  std::shared_ptr<const inventory::Snapshot> snap;
  bool kfd_known = false;
};

const char* const kResourceConfigs[] = {"",
                                        "gpu:sharedgpu:2",
                                        "gpu:sharedgpu:3:pack",
                                        "gpu:sharedgpu:4",
                                        "gpu:gpu-mem-gb:-1",
                                        "gpu:gpu-mem-gb:-1:spread",
                                        "gpu:gpu:1,cpx-1xcd.36gb:small:2,cpx-4xcd.144gb:half:-1",
                                        "cpx-1xcd.36gb:small:-1:pack"};

// The plugin of option bytes b[0..3], built on first use.
Built* PluginFor(const uint8_t* b) {
  static auto* cache = new std::map<uint32_t, std::unique_ptr<Built>>();
  const uint32_t key = b[0] | b[1] << 8 | b[2] << 16 | static_cast<uint32_t>(b[3]) << 24;
  if (auto it = cache->find(key); it != cache->end()) return it->second.get();
  if (cache->size() >= 512) cache->clear();  // bounded: a long run touches many option sets
  SetLogLevel(LogLevel::kError);
  static const int kGpus[] = {1, 2, 4, 8}, kParts[] = {1, 1, 2, 8};
  const int gpus = kGpus[b[0] & 3], parts = kParts[(b[0] >> 2) & 3], kfd = (b[0] >> 4) % 3;
  auto snap = testing::NodeModel(gpus, parts, kfd);
  const auto ps = static_cast<strategy::PartitionStrategy>(b[1] % 3);
  auto rc = strategy::ResourceConfig::Parse(kResourceConfigs[(b[1] >> 2) % 8]);
  if (!rc.ok()) return nullptr;
  auto specs = strategy::BuildPluginSpecs(*snap, ps, *rc);
  if (!specs.ok() || specs->empty()) return nullptr;
  auto built = std::make_unique<Built>();
  plugin::PluginOptions& po = built->opts;
  po.register_with_kubelet = false;
  po.quiet = true;
  po.id_strategy = b[2] & 1 ? plugin::DeviceIdStrategy::kIndex : plugin::DeviceIdStrategy::kUuid;
  po.list_strategy = static_cast<plugin::DeviceListStrategy>((b[2] >> 1) & 3);
  po.pass_device_specs = !(b[2] & 8);
  po.replica_cu_mask = b[2] & 16;
  po.whole_cu_slots = b[2] & 32;
  po.cu_slot_units = b[2] & 64;
  po.replica_hbm_share = b[2] & 128;
  static const alloc::ReplicaPolicy kPolicies[] = {alloc::ReplicaPolicy::kAuto, alloc::ReplicaPolicy::kSpread,
                                                   alloc::ReplicaPolicy::kPack};
  po.replica_policy = kPolicies[b[3] % 3];
  if (b[3] & 4) po.memcap_host_path = "/var/lib/kubelet/device-plugins/amdgpu-dp/libadp_memcap.so";
  po.reject_unhealthy = b[3] & 8;
  po.cdi_spec_dir = "/nonexistent-cdi";  // (Allocate never writes it)
  const auto& spec = (*specs)[(b[3] >> 4) % specs->size()];
  built->plugin = std::make_unique<plugin::Plugin>(snap, spec, po);
  built->snap = snap;
  built->kfd_known = kfd != 0;
  if (built->plugin->advertised_ids().empty()) return nullptr;
  return (*cache)[key] = std::move(built), (*cache)[key].get();
}

std::string g_context;  // the plugin, the request and the answer under check, printed on failure

[[noreturn]] void Fail(const char* what) {
  fprintf(stderr, "invariant violated: %s\n%s\n", what, g_context.c_str());
  abort();
}

std::string Join(const std::vector<std::string>& v, const char* sep = " ") {
  std::string s;
  for (const auto& x : v) s += (s.empty() ? "" : sep) + x;
  return s;
}

std::vector<std::string> SplitList(const std::string& s) {
  std::vector<std::string> out;
  for (size_t b = 0; b <= s.size();) {
    size_t e = std::min(s.find(',', b), s.size());
    out.push_back(s.substr(b, e - b));
    b = e + 1;
  }
  return out;
}

const std::string* Env(const pb::ContainerAllocateResponse& cr, const std::string& name) {
  for (const auto& kv : cr.envs)
    if (kv.first == name) return &kv.second;
  return nullptr;
}

// Picks IDs: mostly advertised ones, sometimes an unknown or a mangled one.
std::string PickId(FuzzedDataProvider& in, const std::vector<std::string>& ids, bool* unknown) {
  uint8_t kind = in.ConsumeIntegral<uint8_t>();
  const std::string& base = ids[in.ConsumeIntegralInRange<size_t>(0, ids.size() - 1)];
  if (kind < 240) return base;
  std::string id = kind < 248 ? base + "x" : in.ConsumeRandomLengthString(80);
  if (std::find(ids.begin(), ids.end(), id) == ids.end()) *unknown = true;  // (a random string may be one of ours)
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
      cr.must_include.push_back(cr.available[in.ConsumeIntegralInRange<size_t>(0, cr.available.size() - 1)]);
    cr.allocation_size = in.ConsumeIntegralInRange<int32_t>(-1, 12);
    req.container_requests.push_back(std::move(cr));
  }
  std::string wire = pb::Encode(req), resp, again;
  Status st = p.HandlePreferred(wire, &resp);
  if (!st.ok()) return;  // refusals are fine; crashes and wrong answers are not
  pb::PreferredAllocationResponse out;
  if (!pb::Decode(resp, &out).ok()) Fail("preferred response does not decode");
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
void CheckCuMask(const plugin::Plugin& p, const pb::ContainerAllocateResponse& cr, size_t devices) {
  const std::string* mask = Env(cr, "HSA_CU_MASK");
  if (!mask) return;
  const std::string& m = *mask;
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
    if (agent >= static_cast<long>(devices)) Fail("HSA_CU_MASK names an agent the container does not have");
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

// The units a request names (advertised IDs only), and distinct IDs per unit.
struct Named {
  std::vector<int> units;      // unique, ascending (= KFD / HIP order)
  std::map<int, size_t> distinct_ids;
};

Named Resolve(const plugin::Plugin& p, const std::vector<std::string>& ids) {
  Named n;
  const auto& adv = p.advertised_ids();
  std::set<std::string> seen;
  std::set<int> us;
  for (const auto& id : ids) {
    auto it = std::find(adv.begin(), adv.end(), id);
    if (it == adv.end()) continue;
    // The advertised ID's unit: its physical ID is the unit whose id is a prefix.
    int unit = -1;
    const std::string_view join = alloc::kReplicaJoin;
    for (size_t u = 0; u < p.units().size(); ++u) {
      const std::string& uid = p.units()[u].id;
      if (id == uid || (id.size() > uid.size() + join.size() && id.compare(0, uid.size(), uid) == 0 &&
                        std::string_view(id).substr(uid.size(), join.size()) == join))
        unit = static_cast<int>(u);
    }
    if (unit < 0) Fail("an advertised ID maps to no unit");
    us.insert(unit);
    if (seen.insert(id).second) ++n.distinct_ids[unit];
  }
  n.units.assign(us.begin(), us.end());
  return n;
}

void CheckAllocate(Built& b, const std::vector<bool>& unhealthy_gpu, FuzzedDataProvider& in) {
  plugin::Plugin& p = *b.plugin;
  const auto& po = b.opts;
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
  for (const auto& c : req.container_requests) g_context += "container: " + Join(c) + "\n";
  Status st = p.HandleAllocate(pb::Encode(req), &resp);
  bool any_empty = false, names_unhealthy = false;
  std::vector<Named> named;
  for (const auto& c : req.container_requests) {
    any_empty = any_empty || c.empty();
    named.push_back(Resolve(p, c));
    for (int u : named.back().units) names_unhealthy = names_unhealthy || unhealthy_gpu[p.units()[u].gpu];
  }
  const bool refuse_health = po.reject_unhealthy && names_unhealthy;
  if (unknown && st.ok()) Fail("Allocate of an unknown ID accepted");
  if (!unknown && !any_empty && refuse_health != !st.ok()) {
    g_context += "status: " + st.ToString() + "\n";
    Fail(refuse_health ? "--reject-unhealthy: an Unhealthy device allocated" : "Allocate of advertised IDs refused");
  }
  if (!st.ok()) return;
  pb::AllocateResponse out;
  if (!pb::Decode(resp, &out).ok()) Fail("allocate response does not decode");
  if (out.container_responses.size() != req.container_requests.size()) Fail("one response per container");
  const auto& units = p.units();
  for (size_t c = 0; c < out.container_responses.size(); ++c) {
    const auto& cr = out.container_responses[c];
    const Named& nm = named[c];
    const size_t devices = nm.units.size();
    // Device specs: /dev/kfd and every device's node, exactly with --pass-device-specs.
    std::set<std::string> spec_paths;
    for (const auto& d : cr.devices) spec_paths.insert(d.container_path);
    if (po.pass_device_specs) {
      if (!spec_paths.count("/dev/kfd")) Fail("no /dev/kfd in an Allocate response");
      for (int u : nm.units)
        for (const auto& path : units[u].paths)
          if (!spec_paths.count(path)) Fail("an allocated device's node is not in the device specs");
    } else if (!cr.devices.empty()) {
      Fail("device specs without --pass-device-specs");
    }
    // The device list, in the strategy's form.
    std::vector<std::string> want;  // visible IDs, in the strategy's order
    std::vector<int> order = nm.units;
    if (po.id_strategy == plugin::DeviceIdStrategy::kUuid)
      std::sort(order.begin(), order.end(), [&](int a, int b2) { return units[a].id < units[b2].id; });
    for (int u : order) want.push_back(units[u].visible_id);
    const std::string* visible = Env(cr, plugin::kVisibleDevicesEnv);
    switch (po.list_strategy) {
      case plugin::DeviceListStrategy::kEnvvar:
        if (!visible || *visible != Join(want, ",")) Fail("AMD_VISIBLE_DEVICES is not the device list");
        if (po.id_strategy == plugin::DeviceIdStrategy::kIndex && b.kfd_known) {
          // index: KFD-node order, how HIP numbers the container's devices
          uint32_t last = 0;
          for (size_t i = 0; i < nm.units.size(); ++i) {
            const auto& g = b.snap->gpus[units[nm.units[i]].gpu];
            uint32_t node = g.partitions.empty() ? 0 : g.kfd_node;
            if (i && node < last) Fail("index strategy: AMD_VISIBLE_DEVICES not in KFD order");
            last = node;
          }
        }
        break;
      case plugin::DeviceListStrategy::kVolumeMounts: {
        if (!visible || *visible != plugin::kVolumeMountRoot) Fail("volume-mounts: the env var is not the root");
        std::vector<std::string> mounted;
        for (const auto& m : cr.mounts)
          if (m.container_path.rfind(std::string(plugin::kVolumeMountRoot) + "/", 0) == 0)
            mounted.push_back(m.container_path.substr(strlen(plugin::kVolumeMountRoot) + 1));
        if (mounted.size() != devices) Fail("volume-mounts: not one mount per device");
        std::vector<std::string> a = mounted, w = want;
        std::sort(a.begin(), a.end());
        std::sort(w.begin(), w.end());
        if (a != w) Fail("volume-mounts: the mounts do not name the devices");
        break;
      }
      case plugin::DeviceListStrategy::kCdiAnnotations: {
        size_t names = 0;
        for (const auto& kv : cr.annotations)
          if (kv.first.rfind("cdi.k8s.io/", 0) == 0) names += SplitList(kv.second).size();
        if (names != devices) Fail("cdi-annotations: not one CDI name per device");
        break;
      }
      case plugin::DeviceListStrategy::kCdiCri:
        if (cr.cdi_devices.size() != devices) Fail("cdi-cri: not one CDI device per device");
        break;
    }
    // HBM grants.
    const std::string* lim = Env(cr, plugin::kMemoryLimitEnv);
    if (p.grants_hbm() && devices > 0) {
      const std::string* frac = Env(cr, plugin::kMemoryFractionEnv);
      const std::string* devs = Env(cr, plugin::kMemoryDevicesEnv);
      if (!lim || !frac || !devs) Fail("a grant without AMD_GPU_MEMORY_LIMIT_MIB/FRACTION/DEVICES");
      auto l = SplitList(*lim), f = SplitList(*frac), d = SplitList(*devs);
      if (l.size() != devices || f.size() != devices || d.size() != devices)
        Fail("AMD_GPU_MEMORY_*: not one entry per device");
      for (size_t i = 0; i < devices; ++i) {
        const auto& u = units[nm.units[i]];  // KFD order
        if (d[i] != u.visible_id) Fail("AMD_GPU_MEMORY_DEVICES not in KFD order");
        uint64_t mib = strtoull(l[i].c_str(), nullptr, 10);
        if (mib != nm.distinct_ids.at(nm.units[i]) * u.grant_mib) Fail("granted MiB != distinct IDs x unit grant");
        if (mib > u.vram_mib) Fail("a grant exceeds the device's HBM");
        if (strtod(f[i].c_str(), nullptr) > 1.00001) Fail("a grant fraction above 1");
      }
      if (!po.memcap_host_path.empty()) {
        size_t grant_mounts = 0;
        bool shim = false;
        for (const auto& m : cr.mounts) {
          grant_mounts += m.container_path.rfind("/run/amdgpu-dp/grant/", 0) == 0 ||
                          m.host_path.find("/grants/") != std::string::npos;
          shim = shim || m.container_path == plugin::kMemcapContainerPath;
        }
        const std::string* preload = Env(cr, "LD_PRELOAD");
        if (!shim || !preload || preload->find("libadp_memcap.so") == std::string::npos)
          Fail("--enforce-memory-units: no HBM-cap shim on a grant");
        if (grant_mounts != devices) Fail("--enforce-memory-units: not one grant file per device");
      }
    } else if (lim) {
      Fail("AMD_GPU_MEMORY_LIMIT_MIB without a grant");
    }
    CheckCuMask(p, cr, devices);
  }
}

}  // namespace

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  if (size < 7) return 0;
  Built* b = PluginFor(data);
  if (!b) return 0;
  plugin::Plugin& p = *b->plugin;
  // Health: the GPUs of data[4]'s bits are Unhealthy, the rest Healthy.
  std::vector<bool> unhealthy(b->snap->gpus.size());
  for (size_t g = 0; g < unhealthy.size(); ++g) {
    unhealthy[g] = data[4] >> (g % 8) & 1;
    p.SetGpuHealth(static_cast<int>(g), !unhealthy[g], "fuzz");
  }
  const uint8_t mode = data[5] % 6;
  g_context = "plugin " + p.resource_name() + " options " + std::to_string(data[0]) + "," + std::to_string(data[1]) +
              "," + std::to_string(data[2]) + "," + std::to_string(data[3]) + " unhealthy " + std::to_string(data[4]) +
              "\n";
  std::string_view raw(reinterpret_cast<const char*>(data + 6), size - 6);
  std::string resp;
  FuzzedDataProvider in(data + 6, size - 6);
  switch (mode) {
    case 0: (void)p.HandleAllocate(raw, &resp); break;
    case 1: (void)p.HandlePreferred(raw, &resp); break;
    case 2: (void)p.HandlePreStart(raw, &resp); break;
    case 3: CheckPreferred(p, in); break;
    default: CheckAllocate(*b, unhealthy, in); break;
  }
  return 0;
}

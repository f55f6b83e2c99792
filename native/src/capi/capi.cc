// C ABI over the native core, for the Python test-suite and benchmark harness
// (loaded with ctypes from k8s_gpu_sharing_plugin_amd/native.py). Every function
// takes and returns JSON strings; returned strings are freed with adp_free().
// This is a test/tooling surface -- the daemon itself never goes through it.
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <json.hpp>
#include <memory>
#include <mutex>
#include <string>

#include "alloc/replicas.h"
#include "alloc/topology.h"
#include "health/health.h"
#include "memcap/driver_usage.h"
#include "inventory/inventory.h"
#include "plugin/plugin.h"
#include "proto/messages.h"
#include "smi/smi.h"
#include "strategy/strategy.h"

using nlohmann::json;

namespace {

char* Dup(const std::string& s) {
  char* p = static_cast<char*>(malloc(s.size() + 1));
  memcpy(p, s.data(), s.size());
  p[s.size()] = 0;
  return p;
}

char* Err(const std::string& msg) { return Dup(json{{"error", msg}}.dump()); }

template <typename Fn>
char* Guard(Fn fn) {
  try {
    return fn();
  } catch (const std::exception& e) {
    return Err(std::string("exception: ") + e.what());
  }
}

json SnapshotJson(const adp::inventory::Snapshot& s) {
  json gpus = json::array();
  for (const auto& g : s.gpus) {
    json parts = json::array();
    for (const auto& p : g.partitions) {
      const auto& raw = s.procs[p.handle];
      parts.push_back({{"uuid", p.uuid}, {"partition_id", p.partition_id}, {"render", p.render_path},
                       {"card", p.card_path}, {"numa", p.numa}, {"vram_mib", p.vram_mib},
                       {"xcds", p.xcds}, {"cus", p.cus},
                       {"kfd_node", p.kfd_node == adp::inventory::kNoKfdNode ? json(nullptr) : json(p.kfd_node)},
                       {"hip_id", raw.hip_id == 0xffffffffu ? json(nullptr) : json(raw.hip_id)},
                       // what amdsmi itself reported for this handle
                       {"reported", {{"vram_mib", raw.vram_mib}, {"xcd_count", raw.xcd_count},
                                     {"profile_type", raw.profile_type},
                                     {"profile_partitions", raw.profile_partitions},
                                     {"profile_xccs", raw.profile_xccs}, {"mem_ranges", raw.mem_ranges},
                                     {"mem_ranges_mib", raw.mem_ranges_mib},
                                     {"asic_serial", raw.asic_serial}, {"bdf", raw.bdf}}}});
    }
    gpus.push_back({{"index", g.index}, {"node_index", g.node_index}, {"uuid", g.uuid}, {"bdf", g.bdf},
                    {"numa", g.numa}, {"vram_mib", g.vram_mib}, {"xcds", g.xcds}, {"cus", g.cus},
                    {"kfd_node", g.kfd_node == adp::inventory::kNoKfdNode ? json(nullptr) : json(g.kfd_node)},
                    {"compute_mode", g.compute_mode}, {"memory_mode", g.memory_mode},
                    {"market_name", g.market_name}, {"profile", g.PartitionProfile()},
                    {"partitioned", g.partitioned()}, {"xgmi_links_down", g.xgmi_links_down},
                    {"vram_source", g.vram_source}, {"driver_profile", g.driver_profile},
                    {"model_hbm_mib", adp::inventory::ModelHbmMib(g.market_name)}, {"partitions", parts}});
  }
  // N x N matrices: the link class the allocator scores (inventory::LinkClass),
  // and what amdsmi reported per pair (link type name, hops, weight).
  static const char* kTypeNames[] = {"internal", "pcie", "xgmi", "n/a", "unknown"};
  json links = json::array(), types = json::array(), hops = json::array(), weights = json::array();
  const size_t n = s.gpus.size();
  for (size_t a = 0; a < n; ++a) {
    json row = json::array(), trow = json::array(), hrow = json::array(), wrow = json::array();
    for (size_t b = 0; b < n; ++b) {
      row.push_back(static_cast<int>(s.Link(a, b)));
      int t = s.gpu_link_types[a * n + b];
      trow.push_back(a == b ? "self" : (t >= 0 && t <= 4 ? kTypeNames[t] : "error"));
      hrow.push_back(s.Hops(a, b));
      wrow.push_back(s.gpu_weights[a * n + b]);
    }
    links.push_back(row);
    types.push_back(trow);
    hops.push_back(hrow);
    weights.push_back(wrow);
  }
  return {{"gpus", gpus}, {"links", links}, {"link_types", types}, {"hops", hops}, {"weights", weights},
          {"smi_path", s.smi_path}, {"smi_version", s.smi_version}};
}

}  // namespace

extern "C" {

void adp_free(char* p) { free(p); }

const char* adp_version() { return ADP_VERSION; }

// {"available": [...], "must_include": [...], "size": n, "policy": "spread"|"pack"}
char* adp_prioritize(const char* in) {
  return Guard([&] {
    json j = json::parse(in);
    adp::alloc::ReplicaPolicy pol = adp::alloc::ReplicaPolicy::kSpread;
    if (j.count("policy")) adp::alloc::ParseReplicaPolicy(j["policy"].get<std::string>(), &pol);
    auto r = adp::alloc::PrioritizeDevices(j["available"].get<std::vector<std::string>>(),
                                           j["must_include"].get<std::vector<std::string>>(),
                                           j["size"].get<int>(), pol);
    if (!r.ok()) return Err(r.status().message());
    return Dup(json{{"ids", r->ids}, {"non_unique", r->non_unique}}.dump());
  });
}

// One driver-side HBM scan: {"proc_root", "kfd_proc_dir", "usage_dir", "self_cgroup"} ->
// {pid_source, pids_scanned, fd_entries, fd_dirs_unreadable, render_only, scan_us, procs: [{pid, bdf, bytes, grant}],
//  total: {bdf: bytes}, unattributed: {bdf: bytes}}
char* adp_driver_scan(const char* in) {
  return Guard([&] {
    json j = json::parse(in);
    auto t0 = std::chrono::steady_clock::now();
    auto s = adp::memcap::ScanDriverHbm(j.value("proc_root", std::string("/proc")),
                                        adp::memcap::ListGrantFiles(j.value("usage_dir", std::string())),
                                        j.value("self_cgroup", std::string()), j.value("kfd_proc_dir", std::string()));
    double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    json procs = json::array();
    for (const auto& p : s.procs)
      procs.push_back({{"pid", p.pid}, {"bdf", p.bdf}, {"bytes", p.bytes}, {"grant", p.grant}});
    return Dup(json{{"pid_source", s.pid_source}, {"pids_scanned", s.pids_scanned}, {"fd_entries", s.fd_entries},
                    {"fd_dirs_unreadable", s.fd_dirs_unreadable}, {"render_only", s.render_only},
                    {"scan_us", us}, {"procs", procs},
                    {"total", s.total}, {"unattributed", s.unattributed}}
                   .dump());
  });
}

char* adp_strip_replicas(const char* in) {
  return Guard([&] {
    json j = json::parse(in);
    return Dup(json(adp::alloc::StripReplicas(j.get<std::vector<std::string>>())).dump());
  });
}

char* adp_parse_additional_ids(const char* in) {
  return Guard([&] { return Dup(json(adp::health::ParseAdditionalIds(in)).dump()); });
}

// Health config from (DP_DISABLE_HEALTHCHECKS, DP_HEALTH_POLL_MS) + event classification table.
char* adp_health_config(const char* disable_value, const char* poll_value) {
  return Guard([&] {
    auto c = adp::health::HealthConfig::FromValues(disable_value, poll_value);
    json verdicts = json::object();
    for (uint32_t t = 1; t <= 13; ++t)
      verdicts[std::to_string(t)] = adp::health::Monitor::Classify(c, t);
    return Dup(json{{"disabled", c.disabled}, {"ignored", c.ignored}, {"poll_ms", c.poll_interval_ms},
                    {"verdicts", verdicts}}
                   .dump());
  });
}

char* adp_parse_resource_config(const char* in) {
  return Guard([&] {
    auto rc = adp::strategy::ResourceConfig::Parse(in);
    if (!rc.ok()) return Err(rc.status().message());
    json out = json::object();
    for (const auto& [k, v] : rc->entries())
      out[k] = {{"name", v.name}, {"replicas", v.replicas}, {"auto", v.auto_replicas}};
    return Dup(out.dump());
  });
}

// {"parent": [...], "scores": [n*n], "available": [...], "required": [...], "size": k}
char* adp_best_effort(const char* in) {
  return Guard([&] {
    json j = json::parse(in);
    adp::alloc::DeviceGraph g(j["parent"].get<std::vector<int>>(), j["scores"].get<std::vector<int>>());
    auto r = adp::alloc::BestEffortAllocate(g, j["available"].get<std::vector<int>>(),
                                            j["required"].get<std::vector<int>>(), j["size"].get<int>());
    return Dup(json(r).dump());
  });
}

// Loads libamd_smi (path "" = default search), enumerates, returns the snapshot.
// {"lib": "...", "devices": [0, 1] | ["0000:0c:00.0", "<uuid>", ...]} (as --devices)
// {"dir", "node"} -> {"cus": n}: inventory::KfdTopologyCus.
char* adp_kfd_topology_cus(const char* in) {
  return Guard([&] {
    json j = json::parse(in);
    return Dup(json{{"cus", adp::inventory::KfdTopologyCus(j.value("dir", std::string()), j.value("node", 0u))}}.dump());
  });
}

char* adp_snapshot(const char* in) {
  return Guard([&] {
    json j = json::parse(in);
    auto lib = adp::smi::Library::Open(j.value("lib", std::string()));
    if (!lib.ok()) return Err(lib.status().ToString());
    adp::inventory::BuildOptions opt;
    if (j.count("devices"))
      for (const auto& d : j["devices"]) {
        if (d.is_number_integer()) opt.only_gpus.push_back(d.get<int>());
        else opt.only_ids.push_back(d.get<std::string>());
      }
    opt.include_card_nodes = j.value("include_card_nodes", false);
    opt.sysfs_root = j.value("sysfs_root", opt.sysfs_root);
    auto snap = adp::inventory::BuildSnapshot(lib->get(), opt);
    if (!snap.ok()) return Err(snap.status().ToString());
    return Dup(SnapshotJson(**snap).dump());
  });
}

// Plugin set for a strategy: {"lib", "strategy", "resource_config", "devices",
//  "auto_unit_mib", "id_strategy"} -> [{resource, socket, original, devices:[{id,index,paths,replicas,vram_mib,numa}], advertised}]
char* adp_plugin_specs(const char* in) {
  return Guard([&] {
    json j = json::parse(in);
    auto lib = adp::smi::Library::Open(j.value("lib", std::string()));
    if (!lib.ok()) return Err(lib.status().ToString());
    adp::inventory::BuildOptions opt;
    if (j.count("devices")) opt.only_gpus = j["devices"].get<std::vector<int>>();
    auto snap = adp::inventory::BuildSnapshot(lib->get(), opt);
    if (!snap.ok()) return Err(snap.status().ToString());
    adp::strategy::PartitionStrategy ps;
    if (!adp::strategy::ParsePartitionStrategy(j.value("strategy", std::string("none")), &ps))
      return Err("bad strategy");
    auto rc = adp::strategy::ResourceConfig::Parse(j.value("resource_config", std::string()));
    if (!rc.ok()) return Err(rc.status().message());
    auto specs = adp::strategy::BuildPluginSpecs(**snap, ps, *rc);
    if (!specs.ok()) return Err(specs.status().message());
    adp::plugin::PluginOptions po;
    po.auto_replica_unit_mib = j.value("auto_unit_mib", 1000);
    if (j.count("id_strategy"))
      adp::plugin::ParseDeviceIdStrategy(j["id_strategy"].get<std::string>(), &po.id_strategy);
    json out = json::array();
    for (const auto& s : *specs) {
      adp::plugin::Plugin p(*snap, s, po);
      json devs = json::array();
      for (const auto& u : p.units())
        devs.push_back({{"id", u.id}, {"index", u.index}, {"paths", u.paths}, {"replicas", u.replicas},
                        {"vram_mib", u.vram_mib}, {"numa", u.numa}, {"gpu", u.gpu}});
      out.push_back({{"resource", s.resource_name}, {"socket", s.socket_name}, {"original", s.original},
                     {"devices", devs}, {"advertised", p.advertised_count()},
                     {"advertised_ids", p.advertised_ids()}, {"replicated", p.replicated()},
                     {"hip_order_known", p.hip_order_known()}});
    }
    return Dup(out.dump());
  });
}

// Proto codec round trip: decode `len` bytes as message `type` with the native
// codec, re-encode, return hex. Types: allocate_request, allocate_response,
// preferred_request, preferred_response, law_response, register_request, options.
char* adp_proto_roundtrip(const char* type, const unsigned char* bytes, size_t len) {
  return Guard([&] {
    std::string_view in(reinterpret_cast<const char*>(bytes), len);
    std::string out;
    adp::Status st;
    std::string t = type;
    auto rt = [&](auto msg) {
      st = adp::pb::Decode(in, &msg);
      if (st.ok()) adp::pb::Encode(msg, &out);
    };
    if (t == "allocate_request") rt(adp::pb::AllocateRequest{});
    else if (t == "allocate_response") rt(adp::pb::AllocateResponse{});
    else if (t == "preferred_request") rt(adp::pb::PreferredAllocationRequest{});
    else if (t == "preferred_response") rt(adp::pb::PreferredAllocationResponse{});
    else if (t == "law_response") rt(adp::pb::ListAndWatchResponse{});
    else if (t == "register_request") rt(adp::pb::RegisterRequest{});
    else if (t == "options") rt(adp::pb::DevicePluginOptions{});
    else if (t == "prestart_request") rt(adp::pb::PreStartContainerRequest{});
    else return Err("unknown type");
    if (!st.ok()) return Err(st.message());
    static const char* hx = "0123456789abcdef";
    std::string h;
    for (unsigned char c : out) { h += hx[c >> 4]; h += hx[c & 15]; }
    return Dup(json{{"hex", h}}.dump());
  });
}

}  // extern "C"

// ---- in-process churn benchmark client (bench.py times exactly the K steps) ----
#include "bench/churn.h"

extern "C" {

// {"socket": "...", "pod_size": 1, "rank": 0, "world": 1, "preferred": true, "grpc_go": false,
//  "owned": ["<device id>", ...] (optional)} -> handle or null
void* adp_bench_open(const char* in, char** err) {
  try {
    json j = json::parse(in);
    adp::bench::ChurnOptions o;
    o.pod_size = j.value("pod_size", 1);
    o.rank = j.value("rank", 0);
    o.world = j.value("world", 1);
    o.preferred = j.value("preferred", true);
    o.grpc_go = j.value("grpc_go", false);
    if (j.count("owned")) o.owned = j["owned"].get<std::vector<std::string>>();
    auto c = adp::bench::ChurnClient::Open(j["socket"].get<std::string>(), o);
    if (!c.ok()) {
      *err = Dup(c.status().ToString());
      return nullptr;
    }
    return c->release();
  } catch (const std::exception& e) {
    *err = Dup(e.what());
    return nullptr;
  }
}

// Runs `pods` admissions; returns null on success or an error string.
char* adp_bench_run(void* h, int pods, int record) {
  auto* c = static_cast<adp::bench::ChurnClient*>(h);
  adp::Status st = c->Run(pods, record != 0);
  return st.ok() ? nullptr : Dup(st.ToString());
}

char* adp_bench_stats(void* h) { return Dup(static_cast<adp::bench::ChurnClient*>(h)->StatsJson()); }
void adp_bench_reset(void* h) { static_cast<adp::bench::ChurnClient*>(h)->ResetStats(); }
void adp_bench_close(void* h) { delete static_cast<adp::bench::ChurnClient*>(h); }

}  // extern "C"

// ---- the health monitor and the event relay, hosted in the calling process ----
// KFD hands an unprivileged event registration only the per-process events of
// its own process (PROCESS_START and the like; resets are device-wide), so to
// see real events flow through the monitor or the relay on a box without root
// the process that registers must be the one that then opens the GPU: a
// Python process hosting them here and running HIP (tests/test_gpu_events.py,
// utils/hosted_events.py).
#include <fcntl.h>
#include <signal.h>
#include <sys/signalfd.h>
#include <unistd.h>

#include <thread>

#include "health/relay.h"

namespace {

struct HostedMonitor {
  std::unique_ptr<adp::smi::Library> lib;
  std::shared_ptr<const adp::inventory::Snapshot> snap;
  adp::health::HealthCounters counters;
  adp::health::Ledger ledger;
  std::unique_ptr<adp::health::Monitor> mon;
  std::mutex mu;
  std::vector<std::pair<int, bool>> transitions;  // (gpu, healthy) notified
};

struct HostedRelay {
  std::unique_ptr<adp::smi::Library> lib;
  int sig[2] = {-1, -1};  // what RunEventRelay reads as its signalfd
  std::thread thread;
  int rc = -1;
};

adp::Result<std::unique_ptr<adp::smi::Library>> OpenLib(const json& j) {
  return adp::smi::Library::Open(j.value("lib", std::string()));
}

}  // namespace

extern "C" {

// {"lib", "devices": [0], "extra_types": "12,13", "poll_ms": 200} -> handle (null: *err says why)
void* adp_monitor_open(const char* in, char** err) {
  try {
    json j = json::parse(in);
    auto lib = OpenLib(j);
    if (!lib.ok()) {
      *err = Dup(lib.status().ToString());
      return nullptr;
    }
    adp::inventory::BuildOptions opt;
    if (j.count("devices")) opt.only_gpus = j["devices"].get<std::vector<int>>();
    auto snap = adp::inventory::BuildSnapshot(lib->get(), opt);
    if (!snap.ok()) {
      *err = Dup(snap.status().ToString());
      return nullptr;
    }
    auto extra = adp::health::ParseEventTypes(j.value("extra_types", std::string()));
    if (!extra.ok()) {
      *err = Dup(extra.status().ToString());
      return nullptr;
    }
    auto h = std::make_unique<HostedMonitor>();
    h->lib = std::move(*lib);
    h->snap = *snap;
    adp::health::HealthConfig c;
    c.poll_interval_ms = j.value("poll_ms", 200);
    c.extra_types = *extra;
    h->mon = std::make_unique<adp::health::Monitor>(h->lib.get(), h->snap, c, &h->ledger, &h->counters);
    HostedMonitor* raw = h.get();
    h->mon->AddListener([raw](int gpu, bool ok, const std::string&) {
      std::lock_guard<std::mutex> lk(raw->mu);
      raw->transitions.emplace_back(gpu, ok);
    });
    adp::Status st = h->mon->Start();
    if (!st.ok()) {
      *err = Dup(st.ToString());
      return nullptr;
    }
    return h.release();
  } catch (const std::exception& e) {
    *err = Dup(e.what());
    return nullptr;
  }
}

// -> {"events_enabled", "events": [{"bdf", "type", "n"}], "unmatched": {type: n}, "transitions": [[gpu, ok]],
//     "registrations": n, "gpus": [bdf]}
char* adp_monitor_state(void* hp) {
  return Guard([&] {
    auto* h = static_cast<HostedMonitor*>(hp);
    json events = json::array();
    for (const auto& [k, n] : h->counters.EventCounts()) events.push_back({{"bdf", k.first}, {"type", k.second}, {"n", n}});
    json tr = json::array();
    {
      std::lock_guard<std::mutex> lk(h->mu);
      for (const auto& [g, ok] : h->transitions) tr.push_back({g, ok});
    }
    json gpus = json::array();
    for (const auto& g : h->snap->gpus) gpus.push_back(g.bdf);
    return Dup(json{{"events_enabled", h->counters.events_enabled.load()}, {"events", events},
                    {"unmatched", h->counters.Unmatched()}, {"transitions", tr},
                    {"registrations", h->lib->EventsRegistered()}, {"gpus", gpus}}
                   .dump());
  });
}

void adp_monitor_close(void* hp) {
  auto* h = static_cast<HostedMonitor*>(hp);
  h->mon->Stop();
  delete h;
}

// {"lib", "socket", "extra_types": "12,13"} -> handle (null: *err says why); the relay serves on a thread.
void* adp_relay_open(const char* in, char** err) {
  try {
    json j = json::parse(in);
    auto lib = OpenLib(j);
    if (!lib.ok()) {
      *err = Dup(lib.status().ToString());
      return nullptr;
    }
    auto extra = adp::health::ParseEventTypes(j.value("extra_types", std::string()));
    if (!extra.ok()) {
      *err = Dup(extra.status().ToString());
      return nullptr;
    }
    auto h = std::make_unique<HostedRelay>();
    h->lib = std::move(*lib);
    if (pipe2(h->sig, O_CLOEXEC | O_NONBLOCK) != 0) {
      *err = Dup("pipe failed");
      return nullptr;
    }
    adp::health::RelayOptions ro;
    for (uint32_t t : *extra) ro.extra_mask |= adp::smi::EventMask(t);
    std::string sock = j.value("socket", std::string());
    HostedRelay* raw = h.get();
    h->thread = std::thread([raw, sock, ro] { raw->rc = adp::health::RunEventRelay(raw->lib.get(), sock, raw->sig[0], ro); });
    return h.release();
  } catch (const std::exception& e) {
    *err = Dup(e.what());
    return nullptr;
  }
}

// Stops the relay (as SIGTERM would) and returns its exit code.
int adp_relay_close(void* hp) {
  auto* h = static_cast<HostedRelay*>(hp);
  signalfd_siginfo si{};
  si.ssi_signo = SIGTERM;
  ssize_t w = write(h->sig[1], &si, sizeof(si));
  (void)w;
  h->thread.join();
  int rc = h->rc;
  close(h->sig[0]);
  close(h->sig[1]);
  delete h;
  return rc;
}

}  // extern "C"


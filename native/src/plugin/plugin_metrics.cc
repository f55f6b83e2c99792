// Plugin observability: the SIGUSR1 stats line, the Prometheus families of
// every plugin (/metrics), and the per-container HBM rows of enforced grants
// (the grant accounting files, matched to pods through PodResources and to the
// driver's own count). Split from plugin.cc; the same Plugin class.
#include "plugin/plugin.h"

#include <algorithm>
#include <cstdio>
#include <map>
#include <set>
#include <string>
#include <tuple>

#include "common/log.h"
#include "common/strings.h"
#include "memcap/usage.h"

namespace adp::plugin {

std::string Plugin::StatsJson() const {
  uint64_t n = stats_.allocate_calls.Value();
  double avg = n ? stats_.allocate_ns_total.Value() / 1e3 / n : 0.0;
  uint64_t np = stats_.preferred_calls.Value();
  double pavg = np ? stats_.preferred_ns_total.Value() / 1e3 / np : 0.0;
  int loops = 0;
  std::string placement = "[", residency = "[]";
  std::vector<uint64_t> res_counts;
  {
    std::lock_guard<std::mutex> lk(server_mu_);
    if (server_) {
      loops = server_->loops();
      for (const auto& [cpu, busy] : server_->LoopPlacement())
        placement += (placement.size() > 1 ? ", [" : "[") + std::to_string(cpu) + ", " + std::to_string(busy) + "]";
      res_counts = server_->stats().residency.Counts();
      residency = server_->stats().residency.SparseJson();
    }
  }
  placement += "]";
  // Only numbers go through the fixed buffer (bounded); the resource name is
  // appended as a string.
  char buf[1024];
  snprintf(buf, sizeof(buf),
           "\", \"devices\": %zu, \"advertised\": %zu, \"allocate_calls\": %llu, "
           "\"allocate_handler_avg_us\": %.3f, \"allocate_handler_max_us\": %.3f, "
           "\"preferred_calls\": %llu, \"preferred_handler_avg_us\": %.3f, "
           "\"preferred_handler_max_us\": %.3f, \"law_sends\": %llu, \"law_bytes\": %zu, "
           "\"server_threads\": %d, \"allocate_handler_p50_le_us\": %g, "
           "\"allocate_handler_p99_le_us\": %g, \"preferred_handler_p50_le_us\": %g, "
           "\"preferred_handler_p99_le_us\": %g, \"unhealthy_allocations\": %llu",
           units_.size(), advertised_.size(),
           static_cast<unsigned long long>(n), avg, stats_.allocate_ns_max.Value() / 1e3,
           static_cast<unsigned long long>(np), pavg, stats_.preferred_ns_max.Value() / 1e3,
           static_cast<unsigned long long>(stats_.law_sends.Value()), law_bytes_size_.load(), loops,
           stats_.allocate_hist.QuantileUs(0.5), stats_.allocate_hist.QuantileUs(0.99),
           stats_.preferred_hist.QuantileUs(0.5), stats_.preferred_hist.QuantileUs(0.99),
           static_cast<unsigned long long>(stats_.unhealthy_allocations.Value()));
  std::string out = "{\"resource\": \"" + JsonEscape(spec_.resource_name) + "\", \"replica_policy\": \"" +
                    (replicated_ ? alloc::ReplicaPolicyName(replica_policy_) : "none") + "\", \"hip_order\": \"" +
                    (hip_order_known_ ? "kfd" : "amdsmi");
  out += buf;
  snprintf(buf, sizeof(buf), ", \"residency_p50_us\": %.1f, \"residency_p99_us\": %.1f, \"residency_100ns\": ",
           metrics::FineHistogram::QuantileUs(res_counts, 0.5), metrics::FineHistogram::QuantileUs(res_counts, 0.99));
  return out + ", \"loop_cpus\": " + placement + buf + residency + "}";
}

size_t Plugin::healthy_count() const {
  auto law = CurrentLaw();
  size_t n = 0;
  for (uint8_t h : law->healthy) n += h;
  return n;
}

namespace {
// Exposition lines are appended whole: label values (pod names up to 253
// characters, ...) have no length bound a fixed buffer could hold, and one
// truncated line makes Prometheus reject the entire scrape.
void Family(std::string* out, const char* name, const char* type, const char* help) {
  *out += "# HELP ";
  *out += name;
  *out += ' ';
  *out += help;
  *out += "\n# TYPE ";
  *out += name;
  *out += ' ';
  *out += type;
  *out += '\n';
}
void Sample(std::string* out, const char* name, const std::string& labels, double v) {
  char num[40];
  snprintf(num, sizeof(num), "%.17g", v);
  *out += name;
  *out += '{';
  *out += labels;
  *out += "} ";
  *out += num;
  *out += '\n';
}
void Sample(std::string* out, const char* name, const std::string& labels, uint64_t v) {
  *out += name;
  *out += '{';
  *out += labels;
  *out += "} ";
  *out += std::to_string(v);
  *out += '\n';
}
}  // namespace

void Plugin::AppendPrometheus(const std::vector<const Plugin*>& plugins, std::string* out,
                              const std::vector<podresources::Assignment>* assignments,
                              const memcap::DriverHbmMonitor::Snapshot* driver,
                              const std::vector<memcap::Usage>* grant_files) {
  using metrics::LabelValue;
  auto family = [&](const char* name, const char* type, const char* help) { Family(out, name, type, help); };
  auto gauge = [&](const char* name, const std::string& labels, double v) { Sample(out, name, labels, v); };
  auto res = [](const Plugin* p) { return "resource=\"" + LabelValue(p->spec_.resource_name) + "\""; };

  family("amdgpu_dp_devices", "gauge", "Physical devices (GPUs or partitions) served by the plugin.");
  for (auto* p : plugins) gauge("amdgpu_dp_devices", res(p), static_cast<double>(p->units_.size()));
  family("amdgpu_dp_allocatable", "gauge", "Device IDs advertised to the kubelet (replicas included).");
  for (auto* p : plugins) gauge("amdgpu_dp_allocatable", res(p), static_cast<double>(p->advertised_.size()));
  family("amdgpu_dp_healthy_devices", "gauge", "Physical devices currently advertised Healthy.");
  for (auto* p : plugins) gauge("amdgpu_dp_healthy_devices", res(p), static_cast<double>(p->healthy_count()));
  {
    bool any = false;
    for (auto* p : plugins) any = any || p->memory_units_;
    if (any) {
      family("amdgpu_dp_memory_unit_mib", "gauge",
             "HBM one unit of a memory-unit resource (replicas -1) grants, per device: a pod requesting N units "
             "gets N times this (kind: cu-slot, a CU on every XCD and its share of the HBM, or mib).");
      for (auto* p : plugins) {
        if (!p->memory_units_) continue;
        for (const auto& u : p->units_)
          gauge("amdgpu_dp_memory_unit_mib",
                res(p) + ",device=\"" + LabelValue(u.id) + "\",kind=\"" + (p->UnitIsCuSlot(u) ? "cu-slot" : "mib") + "\"",
                static_cast<double>(u.grant_mib));
      }
    }
  }
  family("amdgpu_dp_registered", "gauge", "1 while the plugin is serving and registered with the kubelet.");
  for (auto* p : plugins) gauge("amdgpu_dp_registered", res(p), p->registered() ? 1 : 0);
  family("amdgpu_dp_device_healthy", "gauge", "Per-device health (1 Healthy, 0 Unhealthy).");
  for (auto* p : plugins) {
    auto law = p->CurrentLaw();
    for (size_t i = 0; i < p->units_.size(); ++i) {
      const Unit& u = p->units_[i];
      gauge("amdgpu_dp_device_healthy",
            res(p) + ",device=\"" + LabelValue(u.id) + "\",index=\"" + LabelValue(u.index) +
                "\",numa=\"" + std::to_string(u.numa) + "\"",
            i < law->healthy.size() ? law->healthy[i] : 0);
    }
  }
  family("amdgpu_dp_rpc_total", "counter", "Handled kubelet RPCs by method.");
  for (auto* p : plugins) {
    gauge("amdgpu_dp_rpc_total", res(p) + ",method=\"Allocate\"",
          static_cast<double>(p->stats_.allocate_calls.Value()));
    gauge("amdgpu_dp_rpc_total", res(p) + ",method=\"GetPreferredAllocation\"",
          static_cast<double>(p->stats_.preferred_calls.Value()));
    gauge("amdgpu_dp_rpc_total", res(p) + ",method=\"ListAndWatch\"",
          static_cast<double>(p->stats_.law_sends.Value()));
  }
  family("amdgpu_dp_unhealthy_allocations_total", "counter",
         "Allocate() calls that named a device advertised Unhealthy at the time.");
  for (auto* p : plugins)
    gauge("amdgpu_dp_unhealthy_allocations_total", res(p),
          static_cast<double>(p->stats_.unhealthy_allocations.Value()));
  family("amdgpu_dp_partial_cu_slot_allocations_total", "counter",
         "Container devices that filled no whole CU slot under --memory-unit-cu-slots whole and got their "
         "partial (shared) slots.");
  for (auto* p : plugins)
    gauge("amdgpu_dp_partial_cu_slot_allocations_total", res(p),
          static_cast<double>(p->stats_.partial_cu_slot_allocations.Value()));
  family("amdgpu_dp_prestart_refusals_total", "counter",
         "Container starts refused because a device was Unhealthy (--prestart-health-check).");
  for (auto* p : plugins)
    gauge("amdgpu_dp_prestart_refusals_total", res(p), static_cast<double>(p->stats_.prestart_refusals.Value()));
  family("amdgpu_dp_handler_seconds", "histogram",
         "In-daemon handler time per RPC (request decode, device lookup, response encode).");
  for (auto* p : plugins) {
    p->stats_.allocate_hist.AppendPrometheus("amdgpu_dp_handler_seconds", res(p) + ",method=\"Allocate\"", out);
    p->stats_.preferred_hist.AppendPrometheus("amdgpu_dp_handler_seconds",
                                              res(p) + ",method=\"GetPreferredAllocation\"", out);
  }
  family("amdgpu_dp_rpc_residency_seconds", "histogram",
         "Unary RPCs from the socket read that carried them to the reply written, in the gRPC loop "
         "(one sample per batch of calls answered together).");
  for (auto* p : plugins) {
    std::lock_guard<std::mutex> lk(p->server_mu_);
    if (p->server_) p->server_->stats().residency.AppendPrometheus("amdgpu_dp_rpc_residency_seconds", res(p), out);
  }
  if (assignments) {
    // Per physical device: advertised IDs held by running containers and the
    // number of distinct pods holding them (the sharing factor), plus one
    // series per (pod, container, device).
    struct Use { std::vector<uint64_t> ids; std::vector<std::set<std::string>> pods; };
    std::map<std::tuple<const Plugin*, int, std::string, std::string, std::string>, uint64_t> per_pod;
    std::vector<Use> uses(plugins.size());
    // IDs the kubelet says running containers hold that this plugin no longer
    // advertises: the replica count or memory unit changed under them.
    std::vector<uint64_t> stale(plugins.size(), 0);
    for (size_t i = 0; i < plugins.size(); ++i) {
      uses[i].ids.assign(plugins[i]->units_.size(), 0);
      uses[i].pods.resize(plugins[i]->units_.size());
    }
    for (const auto& a : *assignments) {
      for (size_t i = 0; i < plugins.size(); ++i) {
        const Plugin* p = plugins[i];
        if (a.resource != p->spec_.resource_name) continue;
        auto it = p->advertised_index_.find(a.device_id);
        if (it == p->advertised_index_.end()) {
          ++stale[i];
          continue;
        }
        ++uses[i].ids[it->second];
        uses[i].pods[it->second].insert(a.ns + "/" + a.pod);
        ++per_pod[{p, it->second, a.ns, a.pod, a.container}];
      }
    }
    auto dev = [&](const Plugin* p, int u) {
      return res(p) + ",device=\"" + LabelValue(p->units_[u].id) + "\"";
    };
    family("amdgpu_dp_device_allocated_ids", "gauge",
           "Advertised IDs (replicas / memory units) of the device held by running containers.");
    for (size_t i = 0; i < plugins.size(); ++i)
      for (size_t u = 0; u < uses[i].ids.size(); ++u)
        gauge("amdgpu_dp_device_allocated_ids", dev(plugins[i], static_cast<int>(u)),
              static_cast<double>(uses[i].ids[u]));
    family("amdgpu_dp_stale_allocated_ids", "gauge",
           "IDs of this resource that running containers hold (kubelet PodResources) but the plugin no longer "
           "advertises: the replica count or memory unit changed while they ran, so the node can be over-committed.");
    for (size_t i = 0; i < plugins.size(); ++i)
      gauge("amdgpu_dp_stale_allocated_ids", res(plugins[i]), static_cast<double>(stale[i]));
    family("amdgpu_dp_device_pods", "gauge", "Distinct pods sharing the device.");
    for (size_t i = 0; i < plugins.size(); ++i)
      for (size_t u = 0; u < uses[i].pods.size(); ++u)
        gauge("amdgpu_dp_device_pods", dev(plugins[i], static_cast<int>(u)),
              static_cast<double>(uses[i].pods[u].size()));
    family("amdgpu_dp_container_device_ids", "gauge", "Advertised IDs of a device held by one container.");
    for (const auto& [k, n] : per_pod) {
      const auto& [p, u, ns, pod, ctr] = k;
      gauge("amdgpu_dp_container_device_ids",
            dev(p, u) + ",namespace=\"" + LabelValue(ns) + "\",pod=\"" + LabelValue(pod) +
                "\",container=\"" + LabelValue(ctr) + "\"",
            static_cast<double>(n));
    }
  }
  for (auto* p : plugins) {
    if (p->memcap_bytes_.empty() || p->opts_.memcap_usage_dir.empty()) continue;
    AppendMemcapUsage(plugins, p->opts_.memcap_usage_dir, assignments, out, driver, grant_files);
    break;
  }
  struct Conn { const Plugin* p; uint64_t connections, shed, errors; };
  std::vector<Conn> conns;
  for (auto* p : plugins) {
    std::lock_guard<std::mutex> lk(p->server_mu_);
    if (p->server_)
      conns.push_back({p, p->server_->stats().connections.load(), p->server_->stats().shed_connections.load(),
                       p->server_->stats().errors.Value()});
  }
  family("amdgpu_dp_grpc_connections_total", "counter", "Accepted connections on the plugin socket.");
  for (auto& c : conns) gauge("amdgpu_dp_grpc_connections_total", res(c.p), static_cast<double>(c.connections));
  family("amdgpu_dp_grpc_connections_shed_total", "counter",
         "Connections closed on accept because the process was out of file descriptors.");
  for (auto& c : conns) gauge("amdgpu_dp_grpc_connections_shed_total", res(c.p), static_cast<double>(c.shed));
  family("amdgpu_dp_grpc_errors_total", "counter", "RPCs answered with a non-OK gRPC status.");
  for (auto& c : conns) gauge("amdgpu_dp_grpc_errors_total", res(c.p), static_cast<double>(c.errors));
}

std::vector<std::pair<int, uint64_t>> Plugin::GrantedUnits(const std::vector<std::string_view>& ids) const {
  std::vector<std::pair<int, uint64_t>> out;  // (unit, bytes), sorted by unit = the container's HIP order (OrderForHip)
  if (!hbm_grants_) return out;
  std::map<int, uint64_t> per;
  std::set<const void*> seen;  // an ID listed twice grants once (as Allocate counts it)
  for (auto id : ids) {
    auto it = advertised_index_.find(id);
    if (it == advertised_index_.end()) return {};
    if (seen.insert(&*it).second) per[it->second] += units_[it->second].grant_mib << 20;
  }
  out.assign(per.begin(), per.end());
  return out;
}

std::map<std::string, std::map<std::string, uint64_t>> Plugin::GrantedByKey(const std::vector<const Plugin*>& plugins,
                                                                            const std::string& dir) {
  return GrantedByKey(plugins, memcap::ReadAll(dir));
}

std::map<std::string, std::map<std::string, uint64_t>> Plugin::GrantedByKey(
    const std::vector<const Plugin*>& plugins, const std::vector<memcap::Usage>& files) {
  std::map<std::string, std::map<std::string, uint64_t>> out;
  for (auto& u : files) {
    if (u.ids.empty()) continue;  // IDs that do not hash to the file's name: not believed
    std::vector<std::string_view> ids;
    for (size_t b = 0; b <= u.ids.size();) {
      size_t e = std::min(u.ids.find(',', b), u.ids.size());
      ids.push_back(std::string_view(u.ids).substr(b, e - b));
      b = e + 1;
    }
    for (auto* p : plugins) {
      if (p->memcap_bytes_.empty()) continue;
      auto units = p->GrantedUnits(ids);
      if (units.empty()) continue;
      auto& per_bdf = out[u.key];
      for (const auto& [unit, bytes] : units) per_bdf[p->snap_->gpus[p->units_[unit].gpu].bdf] += bytes;
      break;
    }
  }
  return out;
}

// Per-container HBM use of enforced grants, from the shim's accounting files
// (memcap/usage.h): a container listed by PodResources is found by its device
// IDs; without PodResources every file is reported by its own (verified) IDs.
// Files of containers gone for two minutes are removed here. The granted
// bytes are this daemon's (from the container's IDs), never the file's cap[],
// which the container can rewrite; with `driver`, what the driver counts for
// the container's processes on each GPU is reported next to them.
void Plugin::AppendMemcapUsage(const std::vector<const Plugin*>& plugins, const std::string& dir,
                               const std::vector<podresources::Assignment>* assignments, std::string* out,
                               const memcap::DriverHbmMonitor::Snapshot* driver,
                               const std::vector<memcap::Usage>* grant_files) {
  using metrics::LabelValue;
  struct Row {
    const Plugin* p;
    std::string labels;
    std::vector<int> units;         // the container's devices in HIP order
    std::vector<uint64_t> granted;  // bytes granted on each, by this daemon
    memcap::Usage u;
  };
  auto enforced = [&](std::string_view resource) -> const Plugin* {
    for (auto* p : plugins)
      if (p->spec_.resource_name == resource && !p->memcap_bytes_.empty()) return p;
    return nullptr;
  };
  auto fill = [](const Plugin* p, const std::vector<std::string_view>& ids, Row* r) {
    for (const auto& [unit, bytes] : p->GrantedUnits(ids)) {
      r->units.push_back(unit);
      r->granted.push_back(bytes);
    }
    return !r->units.empty();
  };
  // The grant files, read by the caller before it took the plugins lock
  // (then Collect() ran there too), or here.
  std::vector<memcap::Usage> own;
  if (!grant_files) own = memcap::ReadAll(dir);
  const std::vector<memcap::Usage>& files = grant_files ? *grant_files : own;
  std::map<std::string, const memcap::Usage*> by_key;
  for (const auto& u : files) by_key[u.key] = &u;
  std::vector<Row> rows;
  std::set<std::string> live;
  if (assignments) {
    std::map<std::tuple<std::string, std::string, std::string, std::string>, std::vector<std::string_view>> ctrs;
    for (const auto& a : *assignments) ctrs[{a.ns, a.pod, a.container, a.resource}].push_back(a.device_id);
    for (const auto& [k, ids] : ctrs) {
      const auto& [ns, pod, ctr, resource] = k;
      const Plugin* p = enforced(resource);
      if (!p) continue;
      std::string key = memcap::AllocationKey(ids);
      live.insert(key);
      auto u = by_key.find(key);
      Row r{p, "", {}, {}, {}};
      if (u == by_key.end() || !fill(p, ids, &r)) continue;
      r.u = *u->second;
      r.labels = "resource=\"" + LabelValue(resource) + "\",namespace=\"" + LabelValue(ns) + "\",pod=\"" +
                 LabelValue(pod) + "\",container=\"" + LabelValue(ctr) + "\"";
      rows.push_back(std::move(r));
    }
  } else {
    for (const auto& u : files) {
      std::vector<std::string_view> ids;
      for (size_t b = 0; !u.ids.empty() && b <= u.ids.size();) {
        size_t e = std::min(u.ids.find(',', b), u.ids.size());
        ids.push_back(std::string_view(u.ids).substr(b, e - b));
        b = e + 1;
      }
      for (auto* p : plugins) {
        Row r{p, "", {}, {}, {}};
        if (ids.empty() || p->memcap_bytes_.empty() || !fill(p, ids, &r)) continue;
        r.labels = "resource=\"" + LabelValue(p->spec_.resource_name) + "\",allocation=\"" + u.key + "\"";
        r.u = u;
        rows.push_back(std::move(r));
        break;
      }
    }
  }
  if (!grant_files) memcap::Collect(dir, assignments ? &live : nullptr, 120, 4096);

  auto dev_label = [](const Row& r, size_t i) {
    return i < r.units.size() ? r.p->units_[r.units[i]].id : "hip" + std::to_string(i);
  };
  auto column = [&](const char* name, const char* type, const char* help,
                    std::vector<uint64_t> memcap::Usage::*col) {
    Family(out, name, type, help);
    for (const auto& r : rows) {
      const auto& v = r.u.*col;
      for (size_t i = 0; i < v.size(); ++i)
        Sample(out, name, r.labels + ",device=\"" + LabelValue(dev_label(r, i)) + "\"", v[i]);
    }
  };
  column("amdgpu_dp_container_hbm_used_bytes", "gauge",
         "HBM the container's processes hold on the device (HBM-cap shim).", &memcap::Usage::used);
  Family(out, "amdgpu_dp_container_hbm_granted_bytes", "gauge", "HBM granted to the container on the device.");
  for (const auto& r : rows)
    for (size_t i = 0; i < r.granted.size(); ++i)
      Sample(out, "amdgpu_dp_container_hbm_granted_bytes",
             r.labels + ",device=\"" + LabelValue(dev_label(r, i)) + "\"", r.granted[i]);
  column("amdgpu_dp_container_hbm_peak_bytes", "gauge", "Most HBM the container has held on the device.",
         &memcap::Usage::peak);
  column("amdgpu_dp_container_hbm_refusals_total", "counter",
         "HIP allocations refused because they would pass the container's grant.", &memcap::Usage::refused);
  Family(out, "amdgpu_dp_container_hbm_processes", "gauge", "Processes of the container using the HBM-cap shim.");
  for (const auto& r : rows) Sample(out, "amdgpu_dp_container_hbm_processes", r.labels, uint64_t{r.u.processes});
  if (!driver) return;

  // Driver-side truth, per GPU of the grant (partitions of one GPU share its
  // PCI address). Each family's samples form one group: a scrape that
  // interleaves families is refused by strict parsers.
  struct DriverRow {
    std::string labels;
    memcap::DriverHbmMonitor::GrantState st;
  };
  std::vector<DriverRow> drows;
  for (const auto& r : rows) {
    std::set<std::string> bdfs;
    for (int u : r.units) bdfs.insert(r.p->snap_->gpus[r.p->units_[u].gpu].bdf);
    for (const auto& bdf : bdfs) {
      DriverRow d{r.labels + ",bdf=\"" + LabelValue(bdf) + "\"", {}};
      if (auto it = driver->grants.find({r.u.key, bdf}); it != driver->grants.end()) d.st = it->second;
      drows.push_back(std::move(d));
    }
  }
  Family(out, "amdgpu_dp_container_hbm_driver_bytes", "gauge",
         "HBM the container's processes hold on the GPU by the driver's count (DRM fdinfo), whatever path "
         "allocated it.");
  for (const auto& d : drows) Sample(out, "amdgpu_dp_container_hbm_driver_bytes", d.labels, d.st.driver_bytes);
  Family(out, "amdgpu_dp_container_hbm_over_grant", "gauge",
         "1 while the driver counts more HBM for the container on the GPU than granted (+ the runtime allowance "
         "per process).");
  for (const auto& d : drows)
    Sample(out, "amdgpu_dp_container_hbm_over_grant", d.labels, uint64_t{d.st.over ? 1u : 0u});
  Family(out, "amdgpu_dp_container_hbm_over_grant_total", "counter",
         "Times the container went over its grant on the GPU by the driver's count.");
  for (const auto& d : drows) Sample(out, "amdgpu_dp_container_hbm_over_grant_total", d.labels, d.st.over_transitions);
}

}  // namespace adp::plugin

#include "daemon/daemon_metrics.h"

#include <cstdio>

#include "metrics/metrics.h"

namespace adp::daemon {
namespace {

void Family(std::string* out, const char* name, const char* type, const char* help) {
  *out += std::string("# HELP ") + name + " " + help + "\n# TYPE " + name + " " + type + "\n";
}

void Sample(std::string* out, const char* name, const std::string& labels, const std::string& value) {
  *out += name;
  if (!labels.empty()) *out += "{" + labels + "}";
  *out += " " + value + "\n";
}

std::string Bdf(const std::string& bdf) { return "bdf=\"" + metrics::LabelValue(bdf) + "\""; }

std::string Num(uint64_t v) { return std::to_string(v); }

std::string Seconds(double s) {
  char buf[32];
  snprintf(buf, sizeof(buf), "%.3f", s);
  return buf;
}

}  // namespace

void AppendDaemonMetrics(const DaemonMetricsInput& in, std::string* out) {
  const health::HealthCounters& h = *in.health;
  Family(out, "amdgpu_dp_build_info", "gauge", "Plugin and amdsmi versions.");
  Sample(out, "amdgpu_dp_build_info",
         "version=\"" ADP_VERSION "\",amdsmi=\"" + metrics::LabelValue(in.smi_version) + "\"", "1");
  Family(out, "amdgpu_dp_restarts_total", "counter", "Plugin (re)starts: kubelet restart, SIGHUP, retries.");
  Sample(out, "amdgpu_dp_restarts_total", "", Num(in.restarts));
  Family(out, "amdgpu_dp_health_events_enabled", "gauge",
         "1 if amdsmi event notification is registered (-1 not started).");
  Sample(out, "amdgpu_dp_health_events_enabled", "", std::to_string(h.events_enabled.load()));
  Family(out, "amdgpu_dp_health_loop_age_seconds", "gauge",
         "Time since the health monitor loop last iterated (0 when none runs; /healthz fails past "
         "ADP_HEALTH_STALL_MS).");
  Sample(out, "amdgpu_dp_health_loop_age_seconds", "", Seconds(h.HealthLoopAgeMs() / 1e3));
  Family(out, "amdgpu_dp_health_polls_total", "counter", "Health polls (liveness + uncorrectable ECC) run.");
  Sample(out, "amdgpu_dp_health_polls_total", "", Num(h.polls.load()));
  Family(out, "amdgpu_dp_health_ecc_reads_total", "counter", "Uncorrectable-ECC reads by result.");
  Sample(out, "amdgpu_dp_health_ecc_reads_total", "result=\"ok\"", Num(h.ecc_reads_ok.load()));
  Sample(out, "amdgpu_dp_health_ecc_reads_total", "result=\"error\"", Num(h.ecc_read_errors.load()));
  Family(out, "amdgpu_dp_health_events_total", "counter", "amdsmi events received.");
  Sample(out, "amdgpu_dp_health_events_total", "", Num(h.events_received.load()));
  Family(out, "amdgpu_dp_health_retired_page_reads_total", "counter", "Retired-HBM-page reads by result.");
  Sample(out, "amdgpu_dp_health_retired_page_reads_total", "result=\"ok\"", Num(h.retired_reads_ok.load()));
  Sample(out, "amdgpu_dp_health_retired_page_reads_total", "result=\"error\"", Num(h.retired_read_errors.load()));
  Family(out, "amdgpu_dp_health_event_gaps_total", "counter",
         "Stretches in which amdsmi events may have been lost: the event relay restarted, renewed its "
         "registration or could not replay what this daemon missed; events off; event waits failing; a new "
         "in-process registration.");
  Sample(out, "amdgpu_dp_health_event_gaps_total", "", Num(h.event_gaps.load()));
  {
    // Always exported (GPU_PRE_RESET at least, 0): an alert on it needs the series.
    Family(out, "amdgpu_dp_unmatched_events_total", "counter",
           "amdsmi events on a processor that matches no GPU of this node (a handle amdsmi never enumerated, or "
           "one the event relay could not place), by type. An unmatched GPU_PRE_RESET holds every GPU until the "
           "polled check or the operator returns it.");
    auto unmatched = h.Unmatched();
    unmatched.emplace("GPU_PRE_RESET", 0);
    for (const auto& [type, n] : unmatched)
      Sample(out, "amdgpu_dp_unmatched_events_total", "type=\"" + metrics::LabelValue(type) + "\"", Num(n));
  }
  if (h.relay_connected.load() >= 0) {
    // Relay mode: which relay this daemon follows and where it is in its stream.
    Family(out, "amdgpu_dp_event_relay_connected", "gauge", "1 while the daemon is connected to the event relay.");
    Sample(out, "amdgpu_dp_event_relay_connected", "", std::to_string(h.relay_connected.load()));
    Family(out, "amdgpu_dp_event_relay_disconnects_total", "counter",
           "Connections to the event relay that broke: the relay restarted, or dropped this daemon when it fell "
           "behind (events it held are replayed on reconnection).");
    Sample(out, "amdgpu_dp_event_relay_disconnects_total", "", Num(h.relay_disconnects.load()));
    auto cur = h.GetRelayCursor();
    if (cur.valid) {
      Family(out, "amdgpu_dp_event_relay_info", "gauge",
             "The event relay instance this daemon follows (relay: its random ID, new at every relay start), "
             "with the relay's registration generation (renewals so far) as the value.");
      Sample(out, "amdgpu_dp_event_relay_info", "relay=\"" + metrics::LabelValue(cur.relay) + "\"", Num(cur.gen));
      Family(out, "amdgpu_dp_event_relay_last_event_seq", "gauge",
             "Number of the last event this daemon received from the relay (the relay's count).");
      Sample(out, "amdgpu_dp_event_relay_last_event_seq", "", Num(cur.seq));
    }
  }

  if (!in.gpus.empty()) {
    // Why a GPU is Unhealthy, one series per failure cause (the ledger's bits).
    static const std::pair<uint32_t, const char*> kCauses[] = {
        {health::kFailEcc, "ecc"},           {health::kFailUnresponsive, "unresponsive"},
        {health::kFailResetPending, "reset_pending"}, {health::kFailEvent, "event"},
        {health::kFailRetiredPages, "retired_pages"}, {health::kFailDrained, "drained"},
        {health::kFailFlapping, "flapping"}};
    Family(out, "amdgpu_dp_gpu_failure", "gauge",
           "1 while the GPU is Unhealthy for this cause (drained: the operator's drain file, not a fault).");
    for (const auto& g : in.gpus)
      for (const auto& [bit, cause] : kCauses)
        Sample(out, "amdgpu_dp_gpu_failure", Bdf(g.bdf) + ",cause=\"" + cause + "\"", (g.fail & bit) ? "1" : "0");
    Family(out, "amdgpu_dp_gpu_awaiting_polled_recovery", "gauge",
           "1 while the GPU waits for GPU_POST_RESET across an event gap: back in service once amdsmi has "
           "answered every poll for --reset-recovery-hold-ms.");
    for (const auto& g : in.gpus)
      Sample(out, "amdgpu_dp_gpu_awaiting_polled_recovery", Bdf(g.bdf), g.awaiting_polled_recovery ? "1" : "0");
    Family(out, "amdgpu_dp_gpu_recovered_without_event_total", "counter",
           "GPUs put back in service by the polled check after a GPU_POST_RESET was lost in an event gap.");
    auto recovered = h.Recovered();
    for (const auto& g : in.gpus) {
      auto it = recovered.find(g.bdf);
      Sample(out, "amdgpu_dp_gpu_recovered_without_event_total", Bdf(g.bdf),
             Num(it == recovered.end() ? 0 : it->second));
    }
  }
  if (!in.node_access.empty()) {
    Family(out, "amdgpu_dp_device_node_openable", "gauge",
           "1 if the plugin can open the device node (0: denied, e.g. by the container's device cgroup).");
    for (const auto& a : in.node_access)
      Sample(out, "amdgpu_dp_device_node_openable", "node=\"" + metrics::LabelValue(a.path) + "\"",
             a.err ? "0" : "1");
  }
  if (auto events = h.EventCounts(); !events.empty()) {
    Family(out, "amdgpu_dp_gpu_events_total", "counter",
           "amdsmi events per GPU and type, ignored ones included (VMFAULT: an application's GPU page fault; "
           "THERMAL_THROTTLE; GPU_PRE_RESET / GPU_POST_RESET; --health-event-extra-types such as PROCESS_START).");
    for (const auto& [k, n] : events)
      Sample(out, "amdgpu_dp_gpu_events_total", Bdf(k.first) + ",type=\"" + metrics::LabelValue(k.second) + "\"",
             Num(n));
  }
  if (auto retired = h.RetiredPages(); !retired.empty()) {
    Family(out, "amdgpu_dp_retired_pages", "gauge", "HBM pages the driver retired (last health poll).");
    for (const auto& [bdf, n] : retired) Sample(out, "amdgpu_dp_retired_pages", Bdf(bdf), Num(n));
  }
  if (auto total = h.VramTotal(); !total.empty()) {
    Family(out, "amdgpu_dp_gpu_hbm_total_bytes", "gauge", "HBM of the GPU.");
    for (const auto& [bdf, n] : total) Sample(out, "amdgpu_dp_gpu_hbm_total_bytes", Bdf(bdf), Num(n));
  }
  if (auto used = h.VramUsed(); !used.empty()) {
    Family(out, "amdgpu_dp_gpu_hbm_used_bytes", "gauge", "HBM in use on the GPU, all processes (last health poll).");
    for (const auto& [bdf, n] : used) Sample(out, "amdgpu_dp_gpu_hbm_used_bytes", Bdf(bdf), Num(n));
  }
  if (!in.layout_changes_live.empty()) {
    Family(out, "amdgpu_dp_replica_layout_changes_with_live_allocations_total", "counter",
           "Plugin restarts that changed what a replicated resource's IDs mean (memory unit, replica count) while "
           "running pods held some of them (kubelet PodResources).");
    for (const auto& [res, n] : in.layout_changes_live)
      Sample(out, "amdgpu_dp_replica_layout_changes_with_live_allocations_total",
             "resource=\"" + metrics::LabelValue(res) + "\"", Num(n));
  }
  if (!in.deferred_layouts.empty()) {
    Family(out, "amdgpu_dp_deferred_layout_change", "gauge",
           "1 while a config change that would re-mean this resource's IDs waits for the running pods holding "
           "some (--defer-layout-changes).");
    for (const auto& res : in.deferred_layouts)
      Sample(out, "amdgpu_dp_deferred_layout_change", "resource=\"" + metrics::LabelValue(res) + "\"", "1");
  }
  if (in.pod_resources_up >= 0) {
    Family(out, "amdgpu_dp_pod_resources_up", "gauge", "1 if the kubelet PodResources API answered.");
    Sample(out, "amdgpu_dp_pod_resources_up", "", in.pod_resources_up ? "1" : "0");
  }
  if (const auto* d = in.driver_hbm) {
    Family(out, "amdgpu_dp_driver_hbm_polls_total", "counter",
           "Driver-side HBM scans run (DRM fdinfo of every process).");
    Sample(out, "amdgpu_dp_driver_hbm_polls_total", "", Num(d->polls));
    Family(out, "amdgpu_dp_driver_hbm_unreadable_processes", "gauge",
           "Processes whose file descriptors the plugin may not read (their HBM is not seen).");
    Sample(out, "amdgpu_dp_driver_hbm_unreadable_processes", "", Num(d->scan.fd_dirs_unreadable));
    Family(out, "amdgpu_dp_driver_hbm_scan_processes", "gauge",
           "Processes the last driver-side scan read (the GPU processes KFD lists, or every process without "
           "that list).");
    Sample(out, "amdgpu_dp_driver_hbm_scan_processes", "source=\"" + metrics::LabelValue(d->scan.pid_source) + "\"",
           Num(d->scan.pids_scanned));
    Family(out, "amdgpu_dp_driver_hbm_render_only_processes", "gauge",
           "Processes holding HBM through a render node without /dev/kfd (in no KFD process list), as the last "
           "full walk of every process found them (ADP_DRIVER_FULL_WALK_MS); they are read on every scan.");
    Sample(out, "amdgpu_dp_driver_hbm_render_only_processes", "", Num(d->render_only));
    Family(out, "amdgpu_dp_driver_hbm_scan_descriptors", "gauge", "File descriptors the last driver-side scan examined.");
    Sample(out, "amdgpu_dp_driver_hbm_scan_descriptors", "", Num(d->scan.fd_entries));
    Family(out, "amdgpu_dp_driver_hbm_scan_seconds", "gauge", "Wall time of the last driver-side scan.");
    Sample(out, "amdgpu_dp_driver_hbm_scan_seconds", "", std::to_string(d->last_scan_ns / 1e9));
    Family(out, "amdgpu_dp_driver_hbm_scan_failures_total", "counter",
           "Driver-side scans the event relay could not run (the previous scan stays in effect).");
    Sample(out, "amdgpu_dp_driver_hbm_scan_failures_total", "", Num(d->scan_failures));
    Family(out, "amdgpu_dp_hbm_over_grant_events_total", "counter",
           "Transitions of any grant to over its HBM by the driver's count.");
    Sample(out, "amdgpu_dp_hbm_over_grant_events_total", "", Num(d->over_total));
    Family(out, "amdgpu_dp_gpu_hbm_driver_bytes", "gauge", "HBM every process holds on the GPU by the driver's count.");
    for (const auto& [bdf, n] : d->scan.total) Sample(out, "amdgpu_dp_gpu_hbm_driver_bytes", Bdf(bdf), Num(n));
    Family(out, "amdgpu_dp_gpu_hbm_unattributed_bytes", "gauge",
           "HBM on the GPU held by processes outside every enforced grant (no grant file mapped, no grant in "
           "their cgroup).");
    for (const auto& [bdf, n] : d->scan.unattributed)
      Sample(out, "amdgpu_dp_gpu_hbm_unattributed_bytes", Bdf(bdf), Num(n));
  }
}

}  // namespace adp::daemon

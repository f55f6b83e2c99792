// amdgpu-dp-event-probe: what libamd_smi's event notification delivers on this
// node, without the daemon around it -- the raw evidence behind the health
// monitor's event path (round-6 review item 1).
//
// It enumerates the processors exactly as the daemon does (smi::Library),
// registers GPU_PRE_RESET / GPU_POST_RESET plus --types (e.g. 12,13: KFD
// PROCESS_START / PROCESS_END, which any HIP process causes, no privilege
// needed) on every processor, prints "registered" on a line of its own, then
// waits --wait-ms for events. The caller starts a HIP program meanwhile (this
// process never starts one: it holds amdsmi). It ends with one JSON object:
// the processors (bdf, KFD node, partition), the registration status, every
// wait's status (amdsmi_get_gpu_event_notification's, via EventsWait), and
// every event: type, message, and whether its handle is one amdsmi enumerated
// -- the pointer identity the daemon's in-process matching relies on.
//
// usage: amdgpu-dp-event-probe [--lib <libamd_smi.so>] [--types 12,13] [--wait-ms 8000]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "common/strings.h"
#include "health/health.h"
#include "smi/smi.h"

using namespace adp;

int main(int argc, char** argv) {
  std::string lib_path, types = "12,13";
  int wait_ms = 8000;
  for (int i = 1; i + 1 < argc; i += 2) {
    if (!strcmp(argv[i], "--lib")) lib_path = argv[i + 1];
    else if (!strcmp(argv[i], "--types")) types = argv[i + 1];
    else if (!strcmp(argv[i], "--wait-ms")) wait_ms = atoi(argv[i + 1]);
  }
  auto extra = health::ParseEventTypes(types);
  if (!extra.ok()) {
    fprintf(stderr, "%s\n", extra.status().ToString().c_str());
    return 2;
  }
  auto lib = smi::Library::Open(lib_path);
  if (!lib.ok()) {
    printf("{\"error\": \"%s\"}\n", JsonEscape(lib.status().ToString()).c_str());
    return 1;
  }
  auto procs = (*lib)->Enumerate();
  if (!procs.ok()) {
    printf("{\"error\": \"%s\"}\n", JsonEscape(procs.status().ToString()).c_str());
    return 1;
  }
  health::HealthConfig hc;
  hc.extra_types = *extra;
  std::vector<void*> handles;
  for (const auto& p : *procs) handles.push_back(p.handle);
  Status reg = (*lib)->EventsInit(handles, hc.EventMask());
  printf("%s\n", reg.ok() ? "registered" : "registration failed");
  fflush(stdout);

  std::map<std::string, int> wait_status;  // status text -> waits
  std::string events;
  size_t n_events = 0, unmatched = 0;
  auto t0 = std::chrono::steady_clock::now();
  auto elapsed = [&] {
    return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
  };
  while (reg.ok() && elapsed() < wait_ms) {
    std::vector<smi::Event> got;
    Status st = (*lib)->EventsWait(200, &got);
    ++wait_status[st.ok() ? (got.empty() ? "ok (no data)" : "ok") : st.ToString()];
    for (const auto& e : got) {
      int idx = -1;
      for (size_t i = 0; i < procs->size(); ++i)
        if ((*procs)[i].handle == e.handle) idx = static_cast<int>(i);
      unmatched += idx < 0;
      char head[160];
      snprintf(head, sizeof(head), "{\"ms\": %lld, \"type\": %u, \"name\": \"%s\", \"processor\": %d",
               static_cast<long long>(elapsed()), e.type, smi::EventTypeName(e.type).c_str(), idx);
      events += std::string(n_events++ ? ",\n   " : "") + head + ", \"bdf\": \"" +
                (idx >= 0 ? (*procs)[idx].bdf : std::string("?")) + "\", \"message\": \"" + JsonEscape(e.message) +
                "\"}";
    }
  }
  (*lib)->EventsStop(handles);

  std::string out = "{\"amdsmi\": \"" + (*lib)->Version() + "\", \"mask\": " + std::to_string(hc.EventMask()) +
                    ", \"registration\": \"" + JsonEscape(reg.ok() ? "ok" : reg.ToString()) + "\", \"processors\": [";
  for (size_t i = 0; i < procs->size(); ++i) {
    const auto& p = (*procs)[i];
    out += std::string(i ? ", " : "") + "{\"bdf\": \"" + p.bdf + "\", \"kfd_node\": " +
           (p.kfd_node == 0xffffffffu ? std::string("null") : std::to_string(p.kfd_node)) +
           ", \"partition_id\": " + std::to_string(p.partition_id) + "}";
  }
  out += "], \"waits\": {";
  bool first = true;
  for (const auto& [s, n] : wait_status) {
    out += std::string(first ? "" : ", ") + "\"" + JsonEscape(s) + "\": " + std::to_string(n);
    first = false;
  }
  out += "}, \"events_total\": " + std::to_string(n_events) + ", \"unmatched\": " + std::to_string(unmatched) +
         ", \"events\": [" + events + "]}";
  printf("%s\n", out.c_str());
  return 0;
}

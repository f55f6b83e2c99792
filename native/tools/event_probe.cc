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
// --self-hip: after registering, this process itself opens the GPU through
// HIP (dlopen'ed libamdhip64: hipInit, hipMalloc, hipFree) -- KFD delivers an
// unprivileged client only the per-process events of its own process, so this
// is how the decoding and the handle identity are seen on a box without root.
// The waits run on their own thread meanwhile, and every HIP step's start and
// end are recorded on the events' clock (ms since registration): an event's
// "ms" minus hipInit's start is KFD -> amdsmi -> this process's delivery
// latency.
//
// --cycles N: first N generations of what a SIGHUP does to the daemon's
// registration (EventsInit on every processor, then EventsStopAll), each
// status recorded, before the registration that waits -- whether the real
// library takes a registration again after a stop, in one process (review
// item 3; the rollback itself is exercised on the mock, which can fail one
// processor's init).
//
// usage: amdgpu-dp-event-probe [--lib <libamd_smi.so>] [--types 12,13] [--wait-ms 8000] [--self-hip]
//                              [--cycles N]
#include <dirent.h>
#include <dlfcn.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "common/strings.h"
#include "health/health.h"
#include "smi/smi.h"

using namespace adp;

namespace {
// Open descriptors of this process (a registration amdsmi does not release
// would keep a KFD event file open).
int OpenFds() {
  int n = 0;
  if (DIR* d = opendir("/proc/self/fd")) {
    while (readdir(d)) ++n;
    closedir(d);
  }
  return n - 3;  // ".", "..", and the directory's own descriptor
}
}  // namespace

int main(int argc, char** argv) {
  std::string lib_path, types = "12,13";
  int wait_ms = 8000, cycles = 0, cycles_ok = 0;
  bool self_hip = false;
  const char* usage =
      "usage: amdgpu-dp-event-probe [--lib <libamd_smi.so>] [--types 12,13] [--wait-ms 8000] [--self-hip] "
      "[--cycles N]\n";
  for (int i = 1; i < argc; ++i) {
    const bool has_value = i + 1 < argc;
    if (!strcmp(argv[i], "--self-hip")) self_hip = true;
    else if (!strcmp(argv[i], "--lib") && has_value) lib_path = argv[++i];
    else if (!strcmp(argv[i], "--types") && has_value) types = argv[++i];
    else if (!strcmp(argv[i], "--wait-ms") && has_value) wait_ms = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--cycles") && has_value) cycles = atoi(argv[++i]);
    else {
      fputs(usage, strcmp(argv[i], "--help") ? stderr : stdout);
      return strcmp(argv[i], "--help") ? 2 : 0;
    }
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
  std::string gens;
  const int fds_before = OpenFds();
  int fds_first = fds_before;  // after the first generation (what amdsmi keeps once is no leak)
  for (int c = 0; c < cycles; ++c) {
    Status st = (*lib)->EventsInit(handles, hc.EventMask());
    const size_t live = (*lib)->EventsRegistered();
    (*lib)->EventsStopAll();
    cycles_ok += st.ok() && live == handles.size() && (*lib)->EventsRegistered() == 0;
    if (c == 0) fds_first = OpenFds();
    gens += std::string(c ? ", " : "") + "{\"init\": \"" + JsonEscape(st.ok() ? "ok" : st.ToString()) +
            "\", \"registered\": " + std::to_string(live) +
            ", \"after_stop\": " + std::to_string((*lib)->EventsRegistered()) + "}";
  }
  const int fds_after = OpenFds();
  if (gens.size() > 4000) gens = gens.substr(0, gens.rfind("}, {", 2000) + 1) + ", \"...\"";  // the first ones
  Status reg = (*lib)->EventsInit(handles, hc.EventMask());
  printf("%s\n", reg.ok() ? "registered" : "registration failed");
  fflush(stdout);

  std::map<std::string, int> wait_status;  // status text -> waits
  std::string events;
  size_t n_events = 0, unmatched = 0;
  const auto t0 = std::chrono::steady_clock::now();
  auto elapsed = [&] {
    return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
  };
  auto elapsed_us = [&] {
    return std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
  };
  // The waits, on their own thread (amdsmi's wait returns as soon as KFD
  // queues an event), while the main thread opens the GPU.
  std::thread waiter([&] {
    while (reg.ok() && elapsed() < wait_ms) {
      std::vector<smi::Event> got;
      Status st = (*lib)->EventsWait(200, &got);
      const long long at_us = elapsed_us();
      ++wait_status[st.ok() ? (got.empty() ? "ok (no data)" : "ok") : st.ToString()];
      for (const auto& e : got) {
        int idx = -1;
        for (size_t i = 0; i < procs->size(); ++i)
          if ((*procs)[i].handle == e.handle) idx = static_cast<int>(i);
        unmatched += idx < 0;
        char head[200];
        snprintf(head, sizeof(head),
                 "{\"ms\": %lld, \"us\": %lld, \"type\": %u, \"name\": \"%s\", \"processor\": %d", at_us / 1000,
                 at_us, e.type, smi::EventTypeName(e.type).c_str(), idx);
        events += std::string(n_events++ ? ", " : "") + head + ", \"bdf\": \"" +
                  (idx >= 0 ? (*procs)[idx].bdf : std::string("?")) + "\", \"message\": \"" + JsonEscape(e.message) +
                  "\"}";
      }
    }
  });

  // This process opens the GPU itself (KFD process creation, VM acquire,
  // a queue): what KFD reports to its own registration.
  std::string hip = "\"not asked\"";
  if (self_hip && reg.ok()) {
    usleep(300000);  // the waiter is inside a wait by then
    void* dl = dlopen("libamdhip64.so", RTLD_NOW | RTLD_LOCAL);
    if (!dl) dl = dlopen("/opt/rocm/lib/libamdhip64.so", RTLD_NOW | RTLD_LOCAL);
    if (!dl) {
      hip = "\"" + JsonEscape(std::string("dlopen: ") + dlerror()) + "\"";
    } else {
      auto init = reinterpret_cast<int (*)(unsigned)>(dlsym(dl, "hipInit"));
      auto set = reinterpret_cast<int (*)(int)>(dlsym(dl, "hipSetDevice"));
      auto alloc = reinterpret_cast<int (*)(void**, size_t)>(dlsym(dl, "hipMalloc"));
      auto free_ = reinterpret_cast<int (*)(void*)>(dlsym(dl, "hipFree"));
      auto sync = reinterpret_cast<int (*)()>(dlsym(dl, "hipDeviceSynchronize"));
      int a = -1, b = -1, c = -1, d = -1, e = -1;
      void* p = nullptr;
      std::string steps;  // "name": [start_us, end_us] on the events' clock
      auto timed = [&](const char* name, auto&& fn) {
        const long long s0 = elapsed_us();
        int rc = fn();
        steps += std::string(steps.empty() ? "" : ", ") + "\"" + name + "\": [" + std::to_string(s0) + ", " +
                 std::to_string(elapsed_us()) + "]";
        return rc;
      };
      if (init && set && alloc && free_ && sync) {  // each step only after the one before succeeded
        if ((a = timed("hipInit", [&] { return init(0); })) == 0 &&
            (b = timed("hipSetDevice", [&] { return set(0); })) == 0 &&
            (c = timed("hipMalloc", [&] { return alloc(&p, 64 << 20); })) == 0 &&
            (d = timed("hipDeviceSynchronize", [&] { return sync(); })) == 0)
          e = timed("hipFree", [&] { return free_(p); });
      }
      hip = "{\"pid\": " + std::to_string(getpid()) + ", \"hipInit\": " + std::to_string(a) +
            ", \"hipSetDevice\": " + std::to_string(b) + ", \"hipMalloc\": " + std::to_string(c) +
            ", \"hipDeviceSynchronize\": " + std::to_string(d) + ", \"hipFree\": " + std::to_string(e) +
            ", \"steps_us\": {" + steps + "}}";
      // (not dlclose'd: the HIP runtime stays until exit)
    }
  }
  waiter.join();
  (*lib)->EventsStop(handles);

  std::string out = "{\"amdsmi\": \"" + (*lib)->Version() + "\", \"pid\": " + std::to_string(getpid()) +
                    ", \"self_hip\": " + hip + ", \"mask\": " + std::to_string(hc.EventMask()) +
                    ", \"cycles\": [" + gens + "], \"cycle_count\": " + std::to_string(cycles) +
                    ", \"cycles_ok\": " + std::to_string(cycles_ok) + ", \"fds_before_cycles\": " +
                    std::to_string(fds_before) + ", \"fds_after_first_cycle\": " + std::to_string(fds_first) +
                    ", \"fds_after_cycles\": " + std::to_string(fds_after) +
                    ", \"registration\": \"" +
                    JsonEscape(reg.ok() ? "ok" : reg.ToString()) + "\", \"processors\": [";
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

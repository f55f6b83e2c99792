// In-process CPU sampling profiler (no perf/strace on the build or GPU hosts).
//
// ADP_PROFILE_OUT=<file> makes the daemon sample its own program counter on a
// CPU-time timer (SIGPROF, ADP_PROFILE_HZ samples per CPU-second, default
// 1000) and write a flat profile -- samples per symbol and per shared object,
// symbolised with dladdr and demangled -- when it exits. Time spent in the
// kernel shows up at the libc syscall wrapper that entered it (read, send,
// epoll_wait, ...), so the report splits user work from syscall cost too.
#pragma once

#include <string>

namespace adp {

// Starts sampling if ADP_PROFILE_OUT is set. Returns true when active.
bool StartSamplerFromEnv();
// Stops sampling and writes the report (no-op when inactive).
void StopSamplerAndReport();

}  // namespace adp

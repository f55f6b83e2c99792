// One-shot modes of the daemon binary, each printing a report and exiting:
// --list-grants (enforced grants' accounting files), --dry-run (what this node
// would advertise), --smi-report (every amdsmi query's status and which device
// nodes open) and --doctor (one line per deployment prerequisite, with what to
// change). The reference has none of them; its only introspection is the JSON
// config it logs at start (cmd/nvidia-device-plugin/main.go:206-217).
#pragma once

#include <string>

#include "daemon/config.h"
#include "daemon/validate.h"
#include "smi/smi.h"

namespace adp::daemon {

int ListGrants(const std::string& dir);
int DryRun(smi::Library* lib, const Validated& v, const Config& cfg);
int SmiReport(smi::Library* lib, const Validated& v, const Config& cfg);

// --doctor: one line per check -- "ok", "warn" (works, with less) or "FAIL"
// (the plugin cannot serve) -- and what to change; exit 1 on a failure.
struct DoctorReport {
  int ok = 0, warn = 0, fail = 0;
  void Line(const char* level, const std::string& what);
  int Finish();
};
int Doctor(smi::Library* lib, const Validated& v, const Config& cfg, DoctorReport& d);
// --drain / --undrain: edits --drain-file (atomically) and prints it.
// --return-to-service: adds the GPUs to the request file next to it
// (<drain file>.return), which the running daemon's monitor consumes.
int DrainCommand(smi::Library* lib, const Validated& v, const Config& cfg);

}  // namespace adp::daemon

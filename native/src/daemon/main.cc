// amdgpu-device-plugin entry point (reference: cmd/nvidia-device-plugin/main.go:44-138).
#include <csignal>
#include <cstdio>

#include "common/log.h"
#include "common/sampler.h"
#include "daemon/config.h"
#include "daemon/supervisor.h"

#ifndef ADP_VERSION
#define ADP_VERSION "dev"
#endif

int main(int argc, char** argv) {
  // A kubelet that hangs up mid-response must not kill the daemon.
  signal(SIGPIPE, SIG_IGN);
  auto cfg = adp::daemon::LoadConfig(argc, argv);
  if (!cfg.ok()) {
    fprintf(stderr, "Error: %s\n", cfg.status().message().c_str());
    return 1;
  }
  if (cfg->show_help) {
    fputs(adp::daemon::UsageText().c_str(), stdout);
    return 0;
  }
  if (cfg->show_version) {
    printf("amdgpu-device-plugin version %s\n", ADP_VERSION);
    return 0;
  }
  LOG_INFO("main", "amdgpu-device-plugin %s", ADP_VERSION);
  for (const auto& d : cfg->deprecations) LOG_WARN("main", "%s", d.c_str());
  for (const auto& w : cfg->warnings) LOG_WARN("main", "%s", w.c_str());
  bool profiling = adp::StartSamplerFromEnv();
  int rc = adp::daemon::RunDaemon(*cfg, [argc, argv] { return adp::daemon::LoadConfig(argc, argv); });
  if (profiling) adp::StopSamplerAndReport();
  return rc;
}

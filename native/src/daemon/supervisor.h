// Process lifecycle: init, restart loop, kubelet-restart detection, signals.
//
// Parity: reference cmd/nvidia-device-plugin/main.go:205-326 (start): log the
// config as JSON, init the device library honouring failOnInitError (block
// forever when false), start an inotify watcher on the device-plugin directory
// and an OS-signal watcher, then `restart:` -- stop plugins, build them from the
// strategy, start those with devices -- and `events:` -- restart on a plugin
// start error, on kubelet.sock re-creation, on SIGHUP; stop and exit on
// SIGINT/SIGTERM/SIGQUIT. Watchers: watchers.go:9-31.
//
// Native design: one epoll loop over signalfd + inotify + timerfd + an eventfd
// that gRPC servers use to report an exhausted crash budget. Plugin start
// failures restart with exponential backoff (1 s .. 30 s) instead of
// immediately (defect B17). SIGUSR1 dumps per-plugin RPC counters.
//
// Config reload: on SIGHUP, and whenever the config file (--config-file; a
// ConfigMap mount's atomic `..data` swap included) changes, `reload` re-reads
// command line + environment + file. A valid new config replaces the running
// one (strategy, resourceConfig, list/ID strategies, replica policy, devices,
// ...) and the plugins restart with it; an invalid one is logged and ignored.
// Settings bound at startup (amdsmi library, metrics address, PodResources
// socket, node-labels file) keep their original values.
#pragma once

#include <functional>

#include "daemon/config.h"

namespace adp::daemon {

// Runs the daemon until a terminating signal. Returns the process exit code.
int RunDaemon(const Config& cfg, std::function<Result<Config>()> reload = nullptr);

}  // namespace adp::daemon

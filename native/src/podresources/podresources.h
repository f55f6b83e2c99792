// kubelet PodResources client: which pod/container holds which device IDs.
//
// The device-plugin API never tells a plugin when a pod goes away, so the
// plugin cannot know which replicas are in use (the reference does not try).
// The kubelet's PodResources service (proto/podresources/v1/api.proto, on
// /var/lib/kubelet/pod-resources/kubelet.sock) does; the metrics endpoint uses
// it to report per-device allocations -- e.g. how many pods share a GPU through
// time-slice or memory-unit replicas.
#pragma once

#include <chrono>
#include <mutex>
#include <string>
#include <vector>

#include "common/status.h"

namespace adp::podresources {

struct Assignment {
  std::string pod, ns, container, resource, device_id;
};

// Decodes a ListPodResourcesResponse into one Assignment per device ID.
Status DecodeList(std::string_view bytes, std::vector<Assignment>* out);

// One List() call over a fresh connection (the kubelet may restart any time).
Result<std::vector<Assignment>> List(const std::string& socket, int timeout_ms);

// List() with a time-based cache so a scrape storm costs one kubelet call per
// `max_age`. Thread-safe.
class CachedLister {
 public:
  CachedLister(std::string socket, std::chrono::milliseconds max_age) : socket_(std::move(socket)), max_age_(max_age) {}
  Result<std::vector<Assignment>> Get();
  const std::string& socket() const { return socket_; }

 private:
  std::string socket_;
  std::chrono::milliseconds max_age_;
  std::mutex mu_;
  std::chrono::steady_clock::time_point fetched_{};
  bool have_ = false;
  std::vector<Assignment> cached_;
};

}  // namespace adp::podresources

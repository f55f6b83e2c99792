// The kubelet device-plugin v1beta1 messages (proto/deviceplugin/v1beta1/api.proto)
// as plain structs with hand-written encode/decode.
//
// Parity: reference vendor/k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1/api.proto:27-211
// (17 message types) plus the later `cdi_devices` field (5) of
// ContainerAllocateResponse.
#pragma once

#include <cstdint>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

#include "common/status.h"

namespace adp::pb {

inline constexpr const char* kHealthy = "Healthy";
inline constexpr const char* kUnhealthy = "Unhealthy";
inline constexpr const char* kApiVersion = "v1beta1";

using StrMap = std::vector<std::pair<std::string, std::string>>;  // wire order kept

struct DevicePluginOptions {
  bool pre_start_required = false;
  bool get_preferred_allocation_available = false;
};

struct RegisterRequest {
  std::string version;
  std::string endpoint;
  std::string resource_name;
  bool has_options = false;
  DevicePluginOptions options;
};

struct Device {
  std::string id;
  std::string health;
  bool has_topology = false;
  std::vector<int64_t> numa_nodes;
};

struct ListAndWatchResponse {
  std::vector<Device> devices;
};

struct ContainerPreferredAllocationRequest {
  std::vector<std::string> available;
  std::vector<std::string> must_include;
  int32_t allocation_size = 0;
};
struct PreferredAllocationRequest {
  std::vector<ContainerPreferredAllocationRequest> container_requests;
};
struct PreferredAllocationResponse {
  std::vector<std::vector<std::string>> container_responses;  // deviceIDs per container
};

struct AllocateRequest {
  std::vector<std::vector<std::string>> container_requests;  // devicesIDs per container
};

struct Mount {
  std::string container_path;
  std::string host_path;
  bool read_only = false;
};
struct DeviceSpec {
  std::string container_path;
  std::string host_path;
  std::string permissions;
};
struct ContainerAllocateResponse {
  StrMap envs;
  std::vector<Mount> mounts;
  std::vector<DeviceSpec> devices;
  StrMap annotations;
  std::vector<std::string> cdi_devices;
};
struct AllocateResponse {
  std::vector<ContainerAllocateResponse> container_responses;
};

struct PreStartContainerRequest {
  std::vector<std::string> device_ids;
};

// --- zero-copy request views (string_views into the request buffer) ---
// The RPC handlers decode into these: a GetPreferredAllocation for a node with
// ~2.3k memory-unit replicas carries ~115 KB of IDs, and copying each into its
// own std::string dominated the handler.
struct ContainerPreferredAllocationRequestView {
  std::vector<std::string_view> available;
  std::vector<std::string_view> must_include;
  int32_t allocation_size = 0;
};
Status DecodeView(std::string_view b, std::vector<ContainerPreferredAllocationRequestView>* m);
// AllocateRequest: one ID list per container.
Status DecodeView(std::string_view b, std::vector<std::vector<std::string_view>>* m);

// --- encoders (append to *out) ---
void Encode(const DevicePluginOptions& m, std::string* out);
void Encode(const RegisterRequest& m, std::string* out);
void Encode(const Device& m, std::string* out);
void Encode(const ListAndWatchResponse& m, std::string* out);
void Encode(const ContainerPreferredAllocationRequest& m, std::string* out);
void Encode(const PreferredAllocationRequest& m, std::string* out);
void Encode(const PreferredAllocationResponse& m, std::string* out);
void Encode(const AllocateRequest& m, std::string* out);
void Encode(const Mount& m, std::string* out);
void Encode(const DeviceSpec& m, std::string* out);
void Encode(const ContainerAllocateResponse& m, std::string* out);
void Encode(const AllocateResponse& m, std::string* out);
void Encode(const PreStartContainerRequest& m, std::string* out);

template <typename M>
std::string Encode(const M& m) {
  std::string s;
  Encode(m, &s);
  return s;
}

// --- decoders ---
Status Decode(std::string_view b, DevicePluginOptions* m);
Status Decode(std::string_view b, RegisterRequest* m);
Status Decode(std::string_view b, Device* m);
Status Decode(std::string_view b, ListAndWatchResponse* m);
Status Decode(std::string_view b, ContainerPreferredAllocationRequest* m);
Status Decode(std::string_view b, PreferredAllocationRequest* m);
Status Decode(std::string_view b, PreferredAllocationResponse* m);
Status Decode(std::string_view b, AllocateRequest* m);
Status Decode(std::string_view b, Mount* m);
Status Decode(std::string_view b, DeviceSpec* m);
Status Decode(std::string_view b, ContainerAllocateResponse* m);
Status Decode(std::string_view b, AllocateResponse* m);
Status Decode(std::string_view b, PreStartContainerRequest* m);

}  // namespace adp::pb

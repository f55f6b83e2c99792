// Coverage-guided fuzzing (libFuzzer) of the protobuf codec (proto/wire.cc,
// proto/messages.cc) and the kubelet PodResources decoder: every v1beta1
// message the daemon decodes, the zero-copy request views the handlers use,
// and ListPodResourcesResponse. A message that decodes must re-encode to
// bytes that decode to the same message again (encode is canonical: a second
// round trip is byte-identical), and the view decoders must agree with the
// owning decoders on what they accept.
#include <string>
#include <vector>

#include "podresources/podresources.h"
#include "proto/messages.h"

using namespace adp;

namespace {

[[noreturn]] void Fail(const char* what) {
  fprintf(stderr, "invariant violated: %s\n", what);
  abort();
}

template <typename M>
void RoundTrip(std::string_view b) {
  M m;
  if (!pb::Decode(b, &m).ok()) return;
  std::string once = pb::Encode(m);
  M again;
  if (!pb::Decode(once, &again).ok()) Fail("re-encoded message does not decode");
  if (pb::Encode(again) != once) Fail("encoding is not stable");
}

}  // namespace

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  if (size < 1) return 0;
  std::string_view b(reinterpret_cast<const char*>(data + 1), size - 1);
  switch (data[0] % 14) {
    case 0: RoundTrip<pb::DevicePluginOptions>(b); break;
    case 1: RoundTrip<pb::RegisterRequest>(b); break;
    case 2: RoundTrip<pb::Device>(b); break;
    case 3: RoundTrip<pb::ListAndWatchResponse>(b); break;
    case 4: RoundTrip<pb::ContainerPreferredAllocationRequest>(b); break;
    case 5: RoundTrip<pb::PreferredAllocationResponse>(b); break;
    case 6: RoundTrip<pb::Mount>(b); break;
    case 7: RoundTrip<pb::DeviceSpec>(b); break;
    case 8: RoundTrip<pb::ContainerAllocateResponse>(b); break;
    case 9: RoundTrip<pb::AllocateResponse>(b); break;
    case 10: RoundTrip<pb::PreStartContainerRequest>(b); break;
    case 11: {
      RoundTrip<pb::PreferredAllocationRequest>(b);
      pb::PreferredAllocationRequest owned;
      std::vector<pb::ContainerPreferredAllocationRequestView> views;
      bool a = pb::Decode(b, &owned).ok(), v = pb::DecodeView(b, &views).ok();
      if (a != v) Fail("PreferredAllocationRequest: view and owning decoders disagree");
      if (a) {
        if (views.size() != owned.container_requests.size()) Fail("view: container count");
        for (size_t i = 0; i < views.size(); ++i) {
          const auto& o = owned.container_requests[i];
          if (views[i].available.size() != o.available.size() ||
              views[i].must_include.size() != o.must_include.size() ||
              views[i].allocation_size != o.allocation_size)
            Fail("view: container request differs");
          for (size_t k = 0; k < views[i].available.size(); ++k)
            if (views[i].available[k] != o.available[k]) Fail("view: available ID differs");
        }
      }
      break;
    }
    case 12: {
      RoundTrip<pb::AllocateRequest>(b);
      pb::AllocateRequest owned;
      std::vector<std::vector<std::string_view>> views;
      bool a = pb::Decode(b, &owned).ok(), v = pb::DecodeView(b, &views).ok();
      if (a != v) Fail("AllocateRequest: view and owning decoders disagree");
      if (a) {
        if (views.size() != owned.container_requests.size()) Fail("view: container count");
        for (size_t i = 0; i < views.size(); ++i) {
          if (views[i].size() != owned.container_requests[i].size()) Fail("view: ID count");
          for (size_t k = 0; k < views[i].size(); ++k)
            if (views[i][k] != owned.container_requests[i][k]) Fail("view: ID differs");
        }
      }
      break;
    }
    default: {
      std::vector<podresources::Assignment> out;
      (void)podresources::DecodeList(b, &out);
      break;
    }
  }
  return 0;
}

// Stand-in for libamdhip64 in the CPU tests of libadp_memcap.so: the HIP entry
// points the shim interposes or calls, with fake device pointers (no memory is
// allocated), 4 devices of 288 GiB, streams that carry their device, and a
// pitch rounded up to 256 bytes. Exported with libamdhip64's version nodes.
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <cstdint>
#include <cstring>

namespace {
constexpr int kDevices = 4;
constexpr size_t kTotal = size_t{288} << 30;
thread_local int current = 0;
std::atomic<uintptr_t> next_ptr{0x100000000ull};
std::atomic<size_t> used[kDevices];

void* Fake(size_t size) { return reinterpret_cast<void*>(next_ptr.fetch_add((size + 4095) & ~size_t{4095})); }
}  // namespace

extern "C" {
hipError_t hipGetDevice(int* d) { *d = current; return hipSuccess; }
hipError_t hipSetDevice(int d) {
  if (d < 0 || d >= kDevices) return hipErrorInvalidDevice;
  current = d;
  return hipSuccess;
}
// A stream handle of the mock is its device number + 1.
hipError_t hipStreamGetDevice(hipStream_t s, hipDevice_t* d) {
  *d = static_cast<int>(reinterpret_cast<uintptr_t>(s)) - 1;
  return hipSuccess;
}
hipError_t hipMalloc(void** p, size_t size) { *p = Fake(size); used[current] += size; return hipSuccess; }
hipError_t hipExtMallocWithFlags(void** p, size_t size, unsigned int) { return hipMalloc(p, size); }
hipError_t hipMallocManaged(void** p, size_t size, unsigned int) { return hipMalloc(p, size); }
hipError_t hipMallocPitch(void** p, size_t* pitch, size_t w, size_t h) {
  *pitch = (w + 255) & ~size_t{255};
  return hipMalloc(p, *pitch * h);
}
hipError_t hipMallocAsync(void** p, size_t size, hipStream_t) { return hipMalloc(p, size); }
hipError_t hipMallocFromPoolAsync(void** p, size_t size, hipMemPool_t, hipStream_t) { return hipMalloc(p, size); }
hipError_t hipFree(void*) { return hipSuccess; }
hipError_t hipFreeAsync(void*, hipStream_t) { return hipSuccess; }
hipError_t hipMemCreate(hipMemGenericAllocationHandle_t* h, size_t size, const hipMemAllocationProp*,
                        unsigned long long) {
  *h = reinterpret_cast<hipMemGenericAllocationHandle_t>(Fake(size));
  return hipSuccess;
}
hipError_t hipMemRelease(hipMemGenericAllocationHandle_t) { return hipSuccess; }
hipError_t hipMemGetInfo(size_t* free_b, size_t* total) {
  *total = kTotal;
  *free_b = kTotal - used[current];
  return hipSuccess;
}
hipError_t hipDeviceTotalMem(size_t* bytes, hipDevice_t) { *bytes = kTotal; return hipSuccess; }
hipError_t hipGetDevicePropertiesR0600(hipDeviceProp_tR0600* prop, int) {
  memset(prop, 0, sizeof(*prop));
  strcpy(prop->name, "mock MI355X");
  prop->totalGlobalMem = kTotal;
  return hipSuccess;
}
}

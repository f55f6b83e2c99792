// Stand-in for libamdhip64 in the CPU tests of libadp_memcap.so: the HIP entry
// points the shim interposes or calls, with fake device pointers (no memory is
// allocated), 4 devices of 288 GiB, streams that carry their device, a pitch
// rounded up to 256 bytes, and one stream-ordered pool per device that keeps
// freed blocks reserved until trimmed (release threshold "infinite"), like
// HIP's default pool. hip_mock_physical_bytes(dev) reports what the "device"
// holds: live allocations plus pool reserve -- what the cap must bound.
// Exported with libamdhip64's version nodes.
#include <hip/hip_runtime_api.h>
#include <hip/hip_deprecated.h>

#include <unistd.h>

#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_map>

namespace {
constexpr int kDevices = 4;
constexpr size_t kTotal = size_t{288} << 30;
thread_local int current = 0;
std::atomic<uintptr_t> next_ptr{0x100000000ull};

std::mutex mu;
struct Block {
  int dev;
  size_t size;
  bool pooled;
};
std::unordered_map<uintptr_t, Block> live;  // every live allocation
size_t direct[kDevices];                     // bytes of live non-pool allocations
size_t pool_used[kDevices];                  // bytes of live pool allocations
size_t pool_reserved[kDevices];              // what each device's pool holds (>= pool_used)

// Pool handles: device d's default pool is (d + 1) << 4.
hipMemPool_t PoolOf(int d) { return reinterpret_cast<hipMemPool_t>(static_cast<uintptr_t>(d + 1) << 4); }
int DevOfPool(hipMemPool_t p) { return static_cast<int>((reinterpret_cast<uintptr_t>(p) >> 4) - 1); }

void* Fake(size_t size) { return reinterpret_cast<void*>(next_ptr.fetch_add((size + 4095) & ~size_t{4095})); }

void* Alloc(int dev, size_t size, bool pooled) {
  void* p = Fake(size ? size : 1);
  std::lock_guard<std::mutex> lk(mu);
  live[reinterpret_cast<uintptr_t>(p)] = {dev, size, pooled};
  if (pooled) {
    pool_used[dev] += size;
    // Served from the pool's reserve when it has enough free, else the pool grows.
    if (pool_reserved[dev] < pool_used[dev]) pool_reserved[dev] = pool_used[dev];
  } else {
    direct[dev] += size;
  }
  return p;
}

hipError_t Free(const void* p) {
  if (!p) return hipSuccess;
  std::lock_guard<std::mutex> lk(mu);
  auto it = live.find(reinterpret_cast<uintptr_t>(p));
  if (it == live.end()) return hipErrorInvalidValue;
  Block b = it->second;
  live.erase(it);
  if (b.pooled) pool_used[b.dev] -= b.size;  // stays reserved by the pool
  else direct[b.dev] -= b.size;
  return hipSuccess;
}

int StreamDev(hipStream_t s) { return s ? static_cast<int>(reinterpret_cast<uintptr_t>(s)) - 1 : current; }
}  // namespace

extern "C" {
// Test hook: what device `dev` physically holds.
size_t hip_mock_physical_bytes(int dev) {
  std::lock_guard<std::mutex> lk(mu);
  return direct[dev] + pool_reserved[dev];
}

hipError_t hipGetDevice(int* d) { *d = current; return hipSuccess; }
hipError_t hipSetDevice(int d) {
  if (d < 0 || d >= kDevices) return hipErrorInvalidDevice;
  current = d;
  return hipSuccess;
}
// A stream handle of the mock is its device number + 1.
hipError_t hipStreamGetDevice(hipStream_t s, hipDevice_t* d) {
  *d = StreamDev(s);
  return hipSuccess;
}
hipError_t hipMalloc(void** p, size_t size) {
  if (size > kTotal) { *p = nullptr; return hipErrorOutOfMemory; }
  *p = Alloc(current, size, false);
  return hipSuccess;
}
hipError_t hipExtMallocWithFlags(void** p, size_t size, unsigned int) { return hipMalloc(p, size); }
hipError_t hipMallocManaged(void** p, size_t size, unsigned int) { return hipMalloc(p, size); }
hipError_t hipMallocPitch(void** p, size_t* pitch, size_t w, size_t h) {
  *pitch = (w + 255) & ~size_t{255};
  return hipMalloc(p, *pitch * h);
}
hipError_t hipMemAllocPitch(hipDeviceptr_t* p, size_t* pitch, size_t w, size_t h, unsigned int) {
  return hipMallocPitch(reinterpret_cast<void**>(p), pitch, w, h);
}
hipError_t hipMalloc3D(hipPitchedPtr* pp, hipExtent e) {
  size_t pitch = (e.width + 255) & ~size_t{255};
  pp->pitch = pitch;
  pp->xsize = e.width;
  pp->ysize = e.height;
  return hipMalloc(&pp->ptr, pitch * (e.height ? e.height : 1) * (e.depth ? e.depth : 1));
}
hipError_t hipMallocAsync(void** p, size_t size, hipStream_t s) {
  *p = Alloc(StreamDev(s), size, true);
  return hipSuccess;
}
hipError_t hipMallocFromPoolAsync(void** p, size_t size, hipMemPool_t pool, hipStream_t) {
  *p = Alloc(DevOfPool(pool), size, true);
  return hipSuccess;
}
hipError_t hipFree(void* p) { return Free(p); }
hipError_t hipFreeAsync(void* p, hipStream_t) { return Free(p); }
hipError_t hipDeviceGetDefaultMemPool(hipMemPool_t* pool, int dev) { *pool = PoolOf(dev); return hipSuccess; }
hipError_t hipDeviceGetMemPool(hipMemPool_t* pool, int dev) { *pool = PoolOf(dev); return hipSuccess; }
hipError_t hipMemPoolTrimTo(hipMemPool_t pool, size_t keep) {
  int d = DevOfPool(pool);
  std::lock_guard<std::mutex> lk(mu);
  size_t floor = pool_used[d] > keep ? pool_used[d] : keep;
  if (pool_reserved[d] > floor) pool_reserved[d] = floor;
  return hipSuccess;
}
hipError_t hipMemPoolGetAttribute(hipMemPool_t pool, hipMemPoolAttr attr, void* value) {
  int d = DevOfPool(pool);
  // Test hook: hold the answer back, so a caller's read races other threads' allocations.
  static const long delay_us = [] {
    const char* e = getenv("HIP_MOCK_POOL_ATTR_DELAY_US");
    return e ? atol(e) : 0L;
  }();
  std::unique_lock<std::mutex> lk(mu);
  if (delay_us > 0) {
    uint64_t v = attr == hipMemPoolAttrReservedMemCurrent ? pool_reserved[d] : pool_used[d];
    lk.unlock();
    usleep(static_cast<useconds_t>(delay_us));
    if (attr != hipMemPoolAttrReservedMemCurrent && attr != hipMemPoolAttrUsedMemCurrent) return hipErrorInvalidValue;
    *static_cast<uint64_t*>(value) = v;  // the value as it was when read
    return hipSuccess;
  }
  if (attr == hipMemPoolAttrReservedMemCurrent) *static_cast<uint64_t*>(value) = pool_reserved[d];
  else if (attr == hipMemPoolAttrUsedMemCurrent) *static_cast<uint64_t*>(value) = pool_used[d];
  else return hipErrorInvalidValue;
  return hipSuccess;
}
hipError_t hipMallocArray(hipArray_t* a, const hipChannelFormatDesc* d, size_t w, size_t h, unsigned int) {
  size_t elem = static_cast<size_t>((d->x + d->y + d->z + d->w) / 8);
  *a = static_cast<hipArray_t>(Alloc(current, elem * w * (h ? h : 1), false));
  return hipSuccess;
}
hipError_t hipMalloc3DArray(hipArray_t* a, const hipChannelFormatDesc* d, hipExtent e, unsigned int) {
  size_t elem = static_cast<size_t>((d->x + d->y + d->z + d->w) / 8);
  *a = static_cast<hipArray_t>(Alloc(current, elem * e.width * (e.height ? e.height : 1) * (e.depth ? e.depth : 1),
                                     false));
  return hipSuccess;
}
hipError_t hipArrayCreate(hipArray_t* a, const HIP_ARRAY_DESCRIPTOR* d) {
  *a = static_cast<hipArray_t>(Alloc(current, 4 * d->NumChannels * d->Width * (d->Height ? d->Height : 1), false));
  return hipSuccess;
}
hipError_t hipArray3DCreate(hipArray_t* a, const HIP_ARRAY3D_DESCRIPTOR* d) {
  *a = static_cast<hipArray_t>(Alloc(
      current, 4 * d->NumChannels * d->Width * (d->Height ? d->Height : 1) * (d->Depth ? d->Depth : 1), false));
  return hipSuccess;
}
hipError_t hipMallocMipmappedArray(hipMipmappedArray_t* m, const hipChannelFormatDesc* d, hipExtent e,
                                   unsigned int, unsigned int) {
  size_t elem = static_cast<size_t>((d->x + d->y + d->z + d->w) / 8);
  *m = static_cast<hipMipmappedArray_t>(Alloc(current, elem * e.width * (e.height ? e.height : 1), false));
  return hipSuccess;
}
hipError_t hipMipmappedArrayCreate(hipMipmappedArray_t* m, HIP_ARRAY3D_DESCRIPTOR* d, unsigned int) {
  *m = static_cast<hipMipmappedArray_t>(Alloc(current, 4 * d->NumChannels * d->Width, false));
  return hipSuccess;
}
hipError_t hipFreeArray(hipArray_t a) { return Free(a); }
hipError_t hipArrayDestroy(hipArray_t a) { return Free(a); }
hipError_t hipFreeMipmappedArray(hipMipmappedArray_t m) { return Free(m); }
hipError_t hipMipmappedArrayDestroy(hipMipmappedArray_t m) { return Free(m); }
hipError_t hipMemCreate(hipMemGenericAllocationHandle_t* h, size_t size, const hipMemAllocationProp*,
                        unsigned long long) {
  *h = reinterpret_cast<hipMemGenericAllocationHandle_t>(Alloc(current, size, false));
  return hipSuccess;
}
hipError_t hipMemRelease(hipMemGenericAllocationHandle_t h) { return Free(h); }
hipError_t hipMemGetInfo(size_t* free_b, size_t* total) {
  *total = kTotal;
  size_t used = hip_mock_physical_bytes(current);
  *free_b = used < kTotal ? kTotal - used : 0;
  return hipSuccess;
}
hipError_t hipDeviceTotalMem(size_t* bytes, hipDevice_t) { *bytes = kTotal; return hipSuccess; }
hipError_t hipGetDevicePropertiesR0600(hipDeviceProp_tR0600* prop, int) {
  memset(prop, 0, sizeof(*prop));
  strcpy(prop->name, "mock MI355X");
  prop->totalGlobalMem = kTotal;
  return hipSuccess;
}
// The pre-R0600 entry point (binaries built with HIP 5).
hipError_t LegacyProps(hipDeviceProp_tR0000* prop, int) __asm__("hipGetDeviceProperties");
hipError_t LegacyProps(hipDeviceProp_tR0000* prop, int) {
  memset(prop, 0, sizeof(*prop));
  strcpy(prop->name, "mock MI355X (R0000)");
  prop->totalGlobalMem = kTotal;
  return hipSuccess;
}
}

// libadp_memcap.so: HBM caps for memory-unit sharing, enforced in the container.
//
// With `gpu-mem-gb` style resources (resourceConfig replicas = -1) a pod is
// granted N memory units of a GPU; the reference only counts them (server.go:
// 99-111: replicas = MiB/1000) and nothing stops a pod from using the whole
// GPU. When the plugin runs with --enforce-memory-units, Allocate() mounts this
// library into the container and preloads it (LD_PRELOAD). It interposes the
// HIP allocation entry points the frameworks call through the PLT, keeps a
// per-device byte count, and refuses (hipErrorOutOfMemory) an allocation that
// would take a device past its cap. hipMemGetInfo / hipDeviceTotalMem /
// hipGetDeviceProperties report the cap as the device's memory, so frameworks
// that size themselves from free memory (PyTorch's mem_get_info, vLLM's
// gpu_memory_utilization) stay inside the grant.
//
// Caps: AMD_GPU_MEMORY_LIMIT_MIB="<mib>[,<mib>...]", one per device in the
// container's HIP order (the plugin writes it in that order); devices past the
// list are not capped. ADP_MEMCAP_VERBOSE=1 logs every decision to stderr.
//
// No link-time dependency on libamdhip64: the real entry points are resolved
// lazily (RTLD_NEXT, else the already-loaded libamdhip64). The exported
// symbols carry libamdhip64's version nodes (memcap.map).
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <pthread.h>

#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

constexpr int kMaxDevices = 64;

struct Alloc {
  int device;
  size_t bytes;
};

struct State {
  std::mutex mu;
  std::unordered_map<const void*, Alloc> allocs;  // device pointer or VMM handle -> owner
  size_t used[kMaxDevices] = {};
  size_t cap[kMaxDevices] = {};  // 0 = not capped
  bool verbose = false;
  std::atomic<bool> warned[kMaxDevices] = {};
};

State& S() {
  static State* s = [] {
    auto* st = new State();  // never destroyed: frees may run from atexit handlers
    const char* v = getenv("ADP_MEMCAP_VERBOSE");
    st->verbose = v && *v && *v != '0';
    const char* lim = getenv("AMD_GPU_MEMORY_LIMIT_MIB");
    int dev = 0;
    for (const char* p = lim; p && *p && dev < kMaxDevices; ++dev) {
      char* end = nullptr;
      unsigned long long mib = strtoull(p, &end, 10);
      if (end != p) st->cap[dev] = static_cast<size_t>(mib) << 20;
      p = strchr(p, ',');
      if (p) ++p;
    }
    return st;
  }();
  return *s;
}

void Log(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  fprintf(stderr, "amdgpu-dp memcap: %s\n", buf);
}

void* RealSym(const char* name) {
  if (void* f = dlsym(RTLD_NEXT, name)) return f;
  // libamdhip64 pulled in by a library dlopen'ed RTLD_LOCAL is not in the
  // global scope RTLD_NEXT searches: take it by name (already loaded).
  static void* lib = [] {
    const char* env = getenv("ADP_MEMCAP_HIP_LIB");
    const char* names[] = {env, "libamdhip64.so", "libamdhip64.so.7", "libamdhip64.so.6"};
    for (const char* n : names)
      if (n && *n)
        if (void* h = dlopen(n, RTLD_LAZY | RTLD_NOLOAD)) return h;
    for (const char* n : names)
      if (n && *n)
        if (void* h = dlopen(n, RTLD_LAZY)) return h;
    return static_cast<void*>(nullptr);
  }();
  return lib ? dlsym(lib, name) : nullptr;
}

template <typename F>
F Real(const char* name) {
  return reinterpret_cast<F>(RealSym(name));
}

// The header also declares C++ template overloads of several entry points, so
// the real function's type is spelled out at each use.
#define REAL(fn, type) static auto real = Real<type>(#fn)

int CurrentDevice() {
  static auto get = Real<hipError_t (*)(int*)>("hipGetDevice");
  int d = 0;
  if (!get || get(&d) != hipSuccess || d < 0 || d >= kMaxDevices) return 0;
  return d;
}

int StreamDevice(hipStream_t stream) {
  static auto get = Real<hipError_t (*)(hipStream_t, hipDevice_t*)>("hipStreamGetDevice");
  hipDevice_t d = 0;
  if (stream && get && get(stream, &d) == hipSuccess && d >= 0 && d < kMaxDevices) return d;
  return CurrentDevice();
}

// Reserves `bytes` on `dev`; false if that would pass the cap.
bool Reserve(int dev, size_t bytes) {
  State& s = S();
  if (!s.cap[dev]) return true;
  std::lock_guard<std::mutex> lk(s.mu);
  if (s.used[dev] + bytes > s.cap[dev]) {
    if (s.verbose || !s.warned[dev].exchange(true))
      Log("device %d: refused %.1f MiB (%.1f of %.1f MiB in use; AMD_GPU_MEMORY_LIMIT_MIB)", dev,
          bytes / 1048576.0, s.used[dev] / 1048576.0, s.cap[dev] / 1048576.0);
    return false;
  }
  s.used[dev] += bytes;
  return true;
}

void Unreserve(int dev, size_t bytes) {
  State& s = S();
  if (!s.cap[dev]) return;
  std::lock_guard<std::mutex> lk(s.mu);
  s.used[dev] -= std::min(bytes, s.used[dev]);
}

void Track(const void* key, int dev, size_t bytes) {
  State& s = S();
  if (!s.cap[dev] || !key) return;
  std::lock_guard<std::mutex> lk(s.mu);
  s.allocs[key] = {dev, bytes};
  if (s.verbose) Log("device %d: +%zu bytes (%zu in use)", dev, bytes, s.used[dev]);
}

void Untrack(const void* key) {
  State& s = S();
  if (!key) return;
  std::lock_guard<std::mutex> lk(s.mu);
  auto it = s.allocs.find(key);
  if (it == s.allocs.end()) return;  // not ours (uncapped device, or before a cap)
  s.used[it->second.device] -= std::min(it->second.bytes, s.used[it->second.device]);
  if (s.verbose) Log("device %d: -%zu bytes (%zu in use)", it->second.device, it->second.bytes,
                     s.used[it->second.device]);
  s.allocs.erase(it);
}

// Depth of interposed allocator calls on this thread: an entry point the HIP
// library implements by calling another exported one (hipMallocPitch ->
// hipMalloc, say) reaches this library again; only the outermost call counts.
thread_local int t_depth = 0;

// Common path of every allocator: reserve, call the real one, track or roll back.
template <typename Call>
hipError_t Capped(int dev, size_t bytes, void** out, Call call) {
  if (t_depth > 0) return call();
  if (!Reserve(dev, bytes)) {
    if (out) *out = nullptr;
    return hipErrorOutOfMemory;
  }
  ++t_depth;
  hipError_t e = call();
  --t_depth;
  if (e != hipSuccess || !out || !*out) {
    Unreserve(dev, bytes);
    return e;
  }
  Track(*out, dev, bytes);
  return e;
}

}  // namespace

extern "C" {

hipError_t hipMalloc(void** ptr, size_t size) {
  REAL(hipMalloc, hipError_t (*)(void**, size_t));
  if (!real) return hipErrorNotInitialized;
  return Capped(CurrentDevice(), size, ptr, [&] { return real(ptr, size); });
}

hipError_t hipExtMallocWithFlags(void** ptr, size_t size, unsigned int flags) {
  REAL(hipExtMallocWithFlags, hipError_t (*)(void**, size_t, unsigned int));
  if (!real) return hipErrorNotInitialized;
  return Capped(CurrentDevice(), size, ptr, [&] { return real(ptr, size, flags); });
}

hipError_t hipMallocManaged(void** ptr, size_t size, unsigned int flags) {
  REAL(hipMallocManaged, hipError_t (*)(void**, size_t, unsigned int));
  if (!real) return hipErrorNotInitialized;
  return Capped(CurrentDevice(), size, ptr, [&] { return real(ptr, size, flags); });
}

hipError_t hipMallocPitch(void** ptr, size_t* pitch, size_t width, size_t height) {
  REAL(hipMallocPitch, hipError_t (*)(void**, size_t*, size_t, size_t));
  if (!real) return hipErrorNotInitialized;
  // The pitch is only known afterwards: reserve the unpadded size, then track
  // what was really allocated.
  int dev = CurrentDevice();
  hipError_t e = Capped(dev, width * height, ptr, [&] { return real(ptr, pitch, width, height); });
  State& s = S();
  if (t_depth == 0 && e == hipSuccess && ptr && *ptr && pitch && *pitch > width && s.cap[dev]) {
    std::lock_guard<std::mutex> lk(s.mu);
    s.used[dev] += (*pitch - width) * height;
    s.allocs[*ptr].bytes = *pitch * height;
  }
  return e;
}

hipError_t hipMallocAsync(void** ptr, size_t size, hipStream_t stream) {
  REAL(hipMallocAsync, hipError_t (*)(void**, size_t, hipStream_t));
  if (!real) return hipErrorNotInitialized;
  return Capped(StreamDevice(stream), size, ptr, [&] { return real(ptr, size, stream); });
}

hipError_t hipMallocFromPoolAsync(void** ptr, size_t size, hipMemPool_t pool, hipStream_t stream) {
  REAL(hipMallocFromPoolAsync, hipError_t (*)(void**, size_t, hipMemPool_t, hipStream_t));
  if (!real) return hipErrorNotInitialized;
  return Capped(StreamDevice(stream), size, ptr, [&] { return real(ptr, size, pool, stream); });
}

hipError_t hipFree(void* ptr) {
  REAL(hipFree, hipError_t (*)(void*));
  if (!real) return hipErrorNotInitialized;
  hipError_t e = real(ptr);
  if (e == hipSuccess) Untrack(ptr);
  return e;
}

hipError_t hipFreeAsync(void* ptr, hipStream_t stream) {
  REAL(hipFreeAsync, hipError_t (*)(void*, hipStream_t));
  if (!real) return hipErrorNotInitialized;
  hipError_t e = real(ptr, stream);
  if (e == hipSuccess) Untrack(ptr);  // counted free once the free is enqueued
  return e;
}

// Virtual memory management (PyTorch's expandable segments): physical memory
// is created per handle.
hipError_t hipMemCreate(hipMemGenericAllocationHandle_t* handle, size_t size, const hipMemAllocationProp* prop,
                        unsigned long long flags) {
  REAL(hipMemCreate, hipError_t (*)(hipMemGenericAllocationHandle_t*, size_t, const hipMemAllocationProp*, unsigned long long));
  if (!real) return hipErrorNotInitialized;
  int dev = (prop && prop->location.type == hipMemLocationTypeDevice && prop->location.id >= 0 &&
             prop->location.id < kMaxDevices)
                ? prop->location.id
                : CurrentDevice();
  return Capped(dev, size, reinterpret_cast<void**>(handle), [&] { return real(handle, size, prop, flags); });
}

hipError_t hipMemRelease(hipMemGenericAllocationHandle_t handle) {
  REAL(hipMemRelease, hipError_t (*)(hipMemGenericAllocationHandle_t));
  if (!real) return hipErrorNotInitialized;
  hipError_t e = real(handle);
  if (e == hipSuccess) Untrack(handle);
  return e;
}

// What the device "has": the cap, and what is left of it.
hipError_t hipMemGetInfo(size_t* free_bytes, size_t* total_bytes) {
  REAL(hipMemGetInfo, hipError_t (*)(size_t*, size_t*));
  if (!real) return hipErrorNotInitialized;
  hipError_t e = real(free_bytes, total_bytes);
  int dev = CurrentDevice();
  State& s = S();
  if (e != hipSuccess || !s.cap[dev]) return e;
  std::lock_guard<std::mutex> lk(s.mu);
  size_t left = s.cap[dev] - std::min(s.used[dev], s.cap[dev]);
  if (free_bytes) *free_bytes = std::min(*free_bytes, left);
  if (total_bytes) *total_bytes = std::min(*total_bytes, s.cap[dev]);
  return e;
}

hipError_t hipDeviceTotalMem(size_t* bytes, hipDevice_t device) {
  REAL(hipDeviceTotalMem, hipError_t (*)(size_t*, hipDevice_t));
  if (!real) return hipErrorNotInitialized;
  hipError_t e = real(bytes, device);
  if (e == hipSuccess && bytes && device >= 0 && device < kMaxDevices && S().cap[device])
    *bytes = std::min(*bytes, S().cap[device]);
  return e;
}

hipError_t hipGetDevicePropertiesR0600(hipDeviceProp_tR0600* prop, int device) {
  REAL(hipGetDevicePropertiesR0600, hipError_t (*)(hipDeviceProp_tR0600*, int));
  if (!real) return hipErrorNotInitialized;
  hipError_t e = real(prop, device);
  if (e == hipSuccess && prop && device >= 0 && device < kMaxDevices && S().cap[device])
    prop->totalGlobalMem = std::min(prop->totalGlobalMem, S().cap[device]);
  return e;
}

}  // extern "C"

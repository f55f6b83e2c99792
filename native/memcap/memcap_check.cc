// Drives libadp_memcap.so the way a framework does -- HIP calls through the PLT
// of a binary linked against the HIP library (here the CPU mock) -- and prints
// one JSON line per step: {"step": ..., "rc": <hipError_t>, ...}. Run with
// LD_PRELOAD=libadp_memcap.so AMD_GPU_MEMORY_LIMIT_MIB=100,50 (tests/test_memcap.py).
#include <hip/hip_runtime_api.h>
#include <hip/hip_deprecated.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <cstdlib>
#include <thread>
#include <vector>

namespace {
constexpr size_t kMiB = size_t{1} << 20;
void Out(const char* step, hipError_t rc) { printf("{\"step\": \"%s\", \"rc\": %d}\n", step, static_cast<int>(rc)); }
void Info(const char* step) {
  size_t f = 0, t = 0;
  hipError_t rc = hipMemGetInfo(&f, &t);
  printf("{\"step\": \"%s\", \"rc\": %d, \"free_mib\": %zu, \"total_mib\": %zu}\n", step, static_cast<int>(rc),
         f / kMiB, t / kMiB);
}
}  // namespace

extern "C" size_t hip_mock_physical_bytes(int dev);  // the mock's test hook
extern "C" hipError_t LegacyProps(hipDeviceProp_tR0000* prop, int dev) __asm__("hipGetDeviceProperties");

void Phys(const char* step, int dev = 0) {
  printf("{\"step\": \"%s\", \"physical_mib\": %zu}\n", step, hip_mock_physical_bytes(dev) / kMiB);
}

// `pool`: stream-ordered allocations under a 100 MiB cap on device 0; the
// "device" (mock) must never hold more than the cap, pool reserve included.
int Pool() {
  (void)hipSetDevice(0);
  auto s0 = reinterpret_cast<hipStream_t>(uintptr_t{1});
  void *a = nullptr, *b = nullptr, *c = nullptr, *d = nullptr;
  Out("async 80", hipMallocAsync(&a, 80 * kMiB, s0));
  Out("freeasync 80", hipFreeAsync(a, s0));
  Phys("phys after freeasync");  // the pool keeps it reserved
  Info("info after freeasync");
  Out("malloc 50", hipMalloc(&b, 50 * kMiB));  // the pool is trimmed first
  Phys("phys after malloc 50");
  Out("free 50", hipFree(b));
  // A pool that cannot give everything back: 60 stays live.
  Out("async 60", hipMallocAsync(&a, 60 * kMiB, s0));
  Out("async 30", hipMallocAsync(&c, 30 * kMiB, s0));
  Out("freeasync 30", hipFreeAsync(c, s0));
  Out("malloc 40", hipMalloc(&b, 40 * kMiB));  // 60 live + 40: exactly the cap, after trimming the 30
  Phys("phys after malloc 40");
  Out("malloc 10", hipMalloc(&d, 10 * kMiB));  // past the cap
  Phys("phys after malloc 10");
  hipMemPool_t pool = nullptr;
  (void)hipDeviceGetDefaultMemPool(&pool, 0);
  Out("free 40", hipFree(b));
  Out("frompool 30", hipMallocFromPoolAsync(&c, 30 * kMiB, pool, s0));
  Out("free pool 30", hipFreeAsync(c, s0));
  Out("free async 60", hipFreeAsync(a, s0));
  Out("malloc 100", hipMalloc(&b, 100 * kMiB));  // every pool block trimmed away
  Phys("phys after malloc 100");
  Out("free 100", hipFree(b));
  Info("info end");
  return 0;
}

// `poolrace`: one thread churns stream-ordered allocations (their frees stay
// reserved by the pool) while others make synchronous allocations that only
// fit once the pools are trimmed (ReconcilePools). A monitor samples what the
// "device" physically holds: with the accounting right it never exceeds the
// cap, whatever the interleaving. Run with HIP_MOCK_POOL_ATTR_DELAY_US to widen
// the window between reading a pool's reserve and applying it.
int PoolRace() {
  std::atomic<bool> stop{false};
  std::atomic<size_t> max_phys{0};
  std::atomic<int> async_ok{0}, sync_ok{0}, refused{0};
  std::thread monitor([&] {
    while (!stop.load()) {
      size_t p = hip_mock_physical_bytes(0);
      size_t m = max_phys.load();
      while (p > m && !max_phys.compare_exchange_weak(m, p)) {
      }
    }
  });
  std::vector<std::thread> ts;
  ts.emplace_back([&] {
    (void)hipSetDevice(0);
    auto s0 = reinterpret_cast<hipStream_t>(uintptr_t{1});
    for (int i = 0; i < 4000; ++i) {
      void *a = nullptr, *b = nullptr;
      if (hipMallocAsync(&a, 20 * kMiB, s0) == hipSuccess) ++async_ok;
      else ++refused;
      if (hipMallocAsync(&b, 10 * kMiB, s0) == hipSuccess) ++async_ok;
      else ++refused;
      if (a) (void)hipFreeAsync(a, s0);
      if (b) (void)hipFreeAsync(b, s0);
    }
  });
  for (int t = 0; t < 3; ++t)
    ts.emplace_back([&, t] {
      (void)hipSetDevice(0);
      for (int i = 0; i < 1500; ++i) {
        void* p = nullptr;
        if (hipMalloc(&p, (30 + 10 * t) * kMiB) == hipSuccess) {
          ++sync_ok;
          (void)hipFree(p);
        } else {
          ++refused;
        }
      }
    });
  for (auto& t : ts) t.join();
  stop.store(true);
  monitor.join();
  printf("{\"step\": \"poolrace\", \"async_ok\": %d, \"sync_ok\": %d, \"refused\": %d, \"max_physical_mib\": %.3f}\n",
         async_ok.load(), sync_ok.load(), refused.load(), max_phys.load() / double(kMiB));
  Info("poolrace info");
  return 0;
}

// `arrays`: 3D, array, mipmap and pitched allocations and an overflowing size
// under a 100 MiB cap on device 0.
int Arrays() {
  (void)hipSetDevice(0);
  hipChannelFormatDesc f4{32, 32, 32, 32, hipChannelFormatKindFloat};
  hipChannelFormatDesc f1{32, 0, 0, 0, hipChannelFormatKindFloat};
  hipChannelFormatDesc u8{8, 0, 0, 0, hipChannelFormatKindUnsigned};
  hipArray_t a1 = nullptr, a2 = nullptr, a3 = nullptr, a4 = nullptr;
  Out("array 16", hipMallocArray(&a1, &f4, 1024, 1024, 0));
  Out("3darray 128", hipMalloc3DArray(&a2, &f1, make_hipExtent(1024, 1024, 32), 0));
  HIP_ARRAY_DESCRIPTOR d2{};
  d2.Format = HIP_AD_FORMAT_FLOAT;
  d2.NumChannels = 4;
  d2.Width = 1024;
  d2.Height = 1024;
  Out("arraycreate 16", hipArrayCreate(&a3, &d2));
  HIP_ARRAY3D_DESCRIPTOR d3{};
  d3.Format = HIP_AD_FORMAT_FLOAT;
  d3.NumChannels = 1;
  d3.Width = 1024;
  d3.Height = 1024;
  d3.Depth = 16;
  Out("array3dcreate 64", hipArray3DCreate(&a4, &d3));
  Info("info arrays");
  hipPitchedPtr pp{};
  Out("malloc3d 1000x1000x5", hipMalloc3D(&pp, make_hipExtent(1000, 1000, 5)));
  Out("freearray", hipFreeArray(a1));
  Out("arraydestroy", hipArrayDestroy(a3));
  Info("info freed");
  Out("malloc3d again", hipMalloc3D(&pp, make_hipExtent(1000, 1000, 5)));  // 1024 x 1000 x 5 bytes
  Info("info malloc3d");
  hipMipmappedArray_t mm = nullptr;
  Out("mipmap 64", hipMallocMipmappedArray(&mm, &u8, make_hipExtent(8192, 8192, 0), 14, 0));
  Out("free3d", hipFree(pp.ptr));
  Out("array3d free", hipFreeArray(a4));
  Info("info before overflow");
  void* p = nullptr;
  Out("malloc 1", hipMalloc(&p, 1 * kMiB));
  void* huge = nullptr;
  Out("malloc size_max", hipMalloc(&huge, SIZE_MAX));
  size_t pitch = 0;
  Out("pitch overflow", hipMallocPitch(&huge, &pitch, SIZE_MAX / 2, 4));
  Out("async size_max", hipMallocAsync(&huge, SIZE_MAX, reinterpret_cast<hipStream_t>(uintptr_t{1})));
  Info("info after overflow");
  Out("free 1", hipFree(p));
  hipDeviceProp_tR0000 legacy{};
  Out("legacy props", LegacyProps(&legacy, 0));
  printf("{\"step\": \"legacy props value\", \"mib\": %zu}\n", legacy.totalGlobalMem / kMiB);
  Info("info end");
  return 0;
}

// `stress`: 8 threads allocate and free random sizes on device 0 (sync and
// stream-ordered) against the cap; at the end every byte must be back.
int Stress() {
  std::vector<std::thread> ts;
  std::vector<int> refused(8, 0), granted(8, 0);
  for (int t = 0; t < 8; ++t)
    ts.emplace_back([t, &refused, &granted] {
      (void)hipSetDevice(0);
      std::mt19937 rng(t);
      std::vector<void*> held;
      auto s0 = reinterpret_cast<hipStream_t>(uintptr_t{1});
      for (int i = 0; i < 20000; ++i) {
        if (!held.empty() && (rng() % 2 || held.size() > 16)) {
          void* p = held.back();
          held.pop_back();
          (void)(rng() % 2 ? hipFree(p) : hipFreeAsync(p, s0));
          continue;
        }
        void* p = nullptr;
        size_t sz = (1 + rng() % 8) * kMiB;
        hipError_t rc = rng() % 2 ? hipMalloc(&p, sz) : hipMallocAsync(&p, sz, s0);
        if (rc == hipSuccess) { held.push_back(p); ++granted[t]; } else { ++refused[t]; }
      }
      for (void* p : held) (void)hipFree(p);
    });
  for (auto& t : ts) t.join();
  int r = 0, g = 0;
  for (int t = 0; t < 8; ++t) { r += refused[t]; g += granted[t]; }
  printf("{\"step\": \"stress\", \"granted\": %d, \"refused\": %d}\n", g, r);
  Info("stress info");
  return 0;
}

// Several processes of one container (tests/test_memcap.py):
//   hold <dev> <mib>  allocate, report, then hold it until stdin closes (normal exit)
//   try <dev> <mib>   allocate once, report rc and what is left, exit
//   fork <mib>        allocate, fork a child that tries <mib> and <mib>/2, report both
int Processes(int argc, char** argv) {
  const char* mode = argv[1];
  if (!strcmp(mode, "fork")) {
    size_t mib = strtoull(argv[2], nullptr, 10);
    void* p = nullptr;
    Out("parent malloc", hipMalloc(&p, mib * kMiB));
    fflush(stdout);
    pid_t c = fork();
    if (c == 0) {
      void *a = nullptr, *b = nullptr;
      Out("child malloc full", hipMalloc(&a, mib * kMiB));
      Out("child malloc half", hipMalloc(&b, mib / 2 * kMiB));
      fflush(stdout);
      _exit(0);
    }
    int st = 0;
    waitpid(c, &st, 0);
    Info("parent info after child");
    return 0;
  }
  if (argc < 4) return 2;
  int dev = atoi(argv[2]);
  size_t mib = strtoull(argv[3], nullptr, 10);
  (void)hipSetDevice(dev);
  void* p = nullptr;
  Out(mode, hipMalloc(&p, mib * kMiB));
  Info("info");
  fflush(stdout);
  if (!strcmp(mode, "hold")) {
    char buf[16];
    while (read(0, buf, sizeof(buf)) > 0) {
    }
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && strcmp(argv[1], "stress") == 0) return Stress();
  if (argc > 1 && strcmp(argv[1], "pool") == 0) return Pool();
  if (argc > 1 && strcmp(argv[1], "poolrace") == 0) return PoolRace();
  if (argc > 1 && strcmp(argv[1], "arrays") == 0) return Arrays();
  if (argc > 2) return Processes(argc, argv);
  void *a = nullptr, *b = nullptr, *c = nullptr;
  (void)hipSetDevice(0);
  Out("d0 malloc 60", hipMalloc(&a, 60 * kMiB));
  Out("d0 malloc 50", hipMalloc(&b, 50 * kMiB));
  printf("{\"step\": \"d0 refused ptr\", \"null\": %s}\n", b ? "false" : "true");
  Info("d0 info");
  Out("d0 free 60", hipFree(a));
  Out("d0 malloc 50 again", hipMalloc(&b, 50 * kMiB));
  Info("d0 info after");
  size_t pitch = 0;
  Out("d0 pitch 1000x1000", hipMallocPitch(&c, &pitch, 1000, 1000));  // 1024 x 1000 bytes really
  Info("d0 info pitch");
  Out("d0 free pitch", hipFree(c));
  hipMemGenericAllocationHandle_t h = nullptr;
  hipMemAllocationProp prop{};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  Out("d0 memcreate 60", hipMemCreate(&h, 60 * kMiB, &prop, 0));
  Out("d0 memcreate 40", hipMemCreate(&h, 40 * kMiB, &prop, 0));
  Out("d0 memrelease 40", hipMemRelease(h));
  Info("d0 info vmm");

  (void)hipSetDevice(1);
  auto s1 = reinterpret_cast<hipStream_t>(uintptr_t{2});  // mock stream of device 1
  Out("d1 malloc 60", hipMalloc(&a, 60 * kMiB));
  Out("d1 mallocasync 40", hipMallocAsync(&a, 40 * kMiB, s1));
  Out("d1 mallocasync 20", hipMallocAsync(&b, 20 * kMiB, s1));
  Out("d1 freeasync 40", hipFreeAsync(a, s1));
  Out("d1 mallocasync 20 again", hipMallocAsync(&b, 20 * kMiB, s1));
  Info("d1 info");
  size_t tot = 0;
  Out("d1 totalmem", hipDeviceTotalMem(&tot, 1));
  printf("{\"step\": \"d1 totalmem value\", \"mib\": %zu}\n", tot / kMiB);

  (void)hipSetDevice(2);
  Out("d2 malloc 100000", hipMalloc(&a, 100000 * kMiB));  // not capped
  Info("d2 info");
  hipDeviceProp_tR0600 p0{}, p2{};
  (void)hipGetDevicePropertiesR0600(&p0, 0);
  (void)hipGetDevicePropertiesR0600(&p2, 2);
  printf("{\"step\": \"props\", \"d0_mib\": %zu, \"d2_mib\": %zu}\n", p0.totalGlobalMem / kMiB,
         p2.totalGlobalMem / kMiB);
  return 0;
}

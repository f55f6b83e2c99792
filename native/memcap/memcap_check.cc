// Drives libadp_memcap.so the way a framework does -- HIP calls through the PLT
// of a binary linked against the HIP library (here the CPU mock) -- and prints
// one JSON line per step: {"step": ..., "rc": <hipError_t>, ...}. Run with
// LD_PRELOAD=libadp_memcap.so AMD_GPU_MEMORY_LIMIT_MIB=100,50 (tests/test_memcap.py).
#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <sys/wait.h>
#include <unistd.h>

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

// Cost of the HBM-cap shim on the allocation path, on real HIP:
//   amdgpu-dp-memcap-bench [n] [bytes]       (run with and without LD_PRELOAD)
// Times n hipMalloc + hipFree pairs and n hipMemGetInfo calls on device 0 and
// prints one JSON line (ns per call, median of 5 rounds).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

int main(int argc, char** argv) {
  int n = argc > 1 ? atoi(argv[1]) : 20000;
  size_t bytes = argc > 2 ? strtoull(argv[2], nullptr, 10) : (size_t{2} << 20);
  if (hipSetDevice(0) != hipSuccess) return 1;
  void* warm = nullptr;
  if (hipMalloc(&warm, bytes) != hipSuccess || hipFree(warm) != hipSuccess) return 1;
  using Clock = std::chrono::steady_clock;
  std::vector<double> pair_ns, info_ns;
  for (int round = 0; round < 5; ++round) {
    auto t0 = Clock::now();
    for (int i = 0; i < n; ++i) {
      void* p = nullptr;
      if (hipMalloc(&p, bytes) != hipSuccess || hipFree(p) != hipSuccess) return 2;
    }
    auto t1 = Clock::now();
    for (int i = 0; i < n; ++i) {
      size_t f = 0, t = 0;
      if (hipMemGetInfo(&f, &t) != hipSuccess) return 3;
    }
    auto t2 = Clock::now();
    pair_ns.push_back(std::chrono::duration<double, std::nano>(t1 - t0).count() / n);
    info_ns.push_back(std::chrono::duration<double, std::nano>(t2 - t1).count() / n);
  }
  std::sort(pair_ns.begin(), pair_ns.end());
  std::sort(info_ns.begin(), info_ns.end());
  const char* pre = getenv("LD_PRELOAD");
  const char* cap = getenv("AMD_GPU_MEMORY_LIMIT_MIB");
  printf("{\"n\": %d, \"bytes\": %zu, \"malloc_free_ns\": %.1f, \"memgetinfo_ns\": %.1f, \"shim\": %s, "
         "\"cap_mib\": \"%s\"}\n",
         n, bytes, pair_ns[2], info_ns[2], pre && strstr(pre, "libadp_memcap") ? "true" : "false", cap ? cap : "");
  return 0;
}

// HIP visibility / partition probe for gfx950 (MI355X).
//
// Run inside (or on behalf of) a container after Allocate() to prove that the
// device nodes the plugin handed out give a working GPU with the shape the
// plugin advertised -- the MI355X analogue of the reference's PyTorch smoke pod
// (examples/pods/pod1-shared-pytorch.yml) and SHARED_GPU_TUTORIAL.md's manual
// `nvidia-smi -L` check.
//
// What it measures, per HIP device:
//   * census: a launch of 8 workgroups per CU records each workgroup's
//     hardware placement -- XCC id (s_getreg HW_REG_XCC_ID) and SE/SH/CU id
//     (HW_REG_HW_ID) -- so the host counts the XCDs and CUs that actually run
//     work. SPX must show 8 XCDs / 256 CUs; a CPX partition 1 XCD / 32 CUs.
//   * HBM bandwidth: a 16-byte-per-lane streaming copy (grid-stride, 8
//     workgroups x 256 threads per CU, dwordx4 loads/stores) timed with events;
//     a partition should see its share of the ~6.3 TB/s a full MI355X sustains.
//   * correctness: the copied buffer is checksummed on the device (wave64
//     shuffle reduction + one 64-bit atomic per workgroup) against the closed
//     form, so a broken mapping cannot pass silently.
//
// C ABI (loaded with ctypes by k8s_gpu_sharing_plugin_amd/ops/probe.py):
//   int adp_probe_device_count(void);
//   int adp_probe_list(char* out, int len);                       // JSON array
//   int adp_probe_run(int device, unsigned long long bytes, int iters, char* out, int len);
// Return 0 on success, a hipError_t (>0) on failure; `out` holds JSON either way.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <set>
#include <string>
#include <vector>

#include "../memcap/memcap_area.h"

namespace {

__device__ __forceinline__ uint32_t ReadXccId() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xf;
}

__device__ __forceinline__ uint32_t ReadHwId() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(v));
  return v;
}

// One record per workgroup: xcc[3:0] << 16 | se/sh/cu bits of HW_ID [15:8].
__global__ void __launch_bounds__(64) CensusKernel(uint32_t* out) {
  if (threadIdx.x == 0) {
    uint32_t xcc = ReadXccId();
    uint32_t hw = ReadHwId();
    out[blockIdx.x] = (xcc << 16) | ((hw >> 8) & 0xff);
  }
}

// Placement census for CU masks: every workgroup records where it ran and then
// holds its CU for ~`hold_ticks` of the 100 MHz wall clock, so the dispatcher
// spreads the grid over every CU the queue may use (a bounded wait: each wave
// exits after at most hold_ticks).
__global__ void __launch_bounds__(64) HoldCensusKernel(uint32_t* out, uint64_t hold_ticks) {
  if (threadIdx.x == 0) {
    uint32_t xcc = ReadXccId();
    uint32_t hw = ReadHwId();
    out[blockIdx.x] = (xcc << 16) | ((hw >> 8) & 0xff);
    uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < hold_ticks) __builtin_amdgcn_s_sleep(2);
  }
}

// Sharing-interference pair (amdgpu-dp-probe --latency / --aggressor): what a
// latency-sensitive pod sees while a neighbour on the same GPU saturates it.
// Victim: a short fixed chain of FMAs per lane (one small launch, ~10 us solo).
__global__ void __launch_bounds__(256) VictimKernel(float* out, int iters) {
  float a = threadIdx.x * 1e-3f, b = 1.0001f;
  for (int i = 0; i < iters; ++i) a = __builtin_fmaf(a, b, 1e-7f);
  if (a == -1.0f) out[blockIdx.x] = a;  // never true: keeps the chain alive
}

// Aggressor: every workgroup keeps its SIMD busy with dependent FMAs until
// `ticks` of the 100 MHz wall clock have passed (a bounded spin: each wave exits
// on its own clock check).
__global__ void __launch_bounds__(256) AggressorKernel(float* out, uint64_t ticks) {
  float a = threadIdx.x * 1e-3f, b = 0.9999f;
  uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) {
#pragma unroll
    for (int i = 0; i < 64; ++i) a = __builtin_fmaf(a, b, 1e-7f);
  }
  if (a == -1.0f) out[blockIdx.x] = a;
}

__global__ void __launch_bounds__(256) FillKernel(uint4* p, size_t n) {
  size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint32_t b = static_cast<uint32_t>(i * 4);
    p[i] = make_uint4(b, b + 1, b + 2, b + 3);
  }
}

// Tunable streaming copy for the bandwidth sweep: UNROLL independent 16-byte
// loads in flight per lane, optional non-temporal (streaming) loads / stores.
template <bool NT>
__device__ __forceinline__ uint4 Load16(const uint4* p) {
  if (!NT) return *p;
  uint4 v;
  v.x = __builtin_nontemporal_load(&p->x);
  v.y = __builtin_nontemporal_load(&p->y);
  v.z = __builtin_nontemporal_load(&p->z);
  v.w = __builtin_nontemporal_load(&p->w);
  return v;
}

template <bool NT>
__device__ __forceinline__ void Store16(uint4* p, const uint4& v) {
  if (!NT) { *p = v; return; }
  __builtin_nontemporal_store(v.x, &p->x);
  __builtin_nontemporal_store(v.y, &p->y);
  __builtin_nontemporal_store(v.z, &p->z);
  __builtin_nontemporal_store(v.w, &p->w);
}

// Grid-stride form: consecutive workgroups touch adjacent 4 KiB slices.
template <int UNROLL, bool NT, bool NTL = false>
__global__ void __launch_bounds__(256) CopyKernelT(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                   size_t n) {
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
    uint4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) v[u] = Load16<NTL>(&src[i + u * stride]);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) Store16<NT>(&dst[i + u * stride], v[u]);
  }
  for (; i < n; i += stride) dst[i] = src[i];
}

// Chunked form: each workgroup streams one contiguous chunk of the buffer
// (long DRAM-page runs per workgroup instead of a chip-wide interleave).
template <int UNROLL, bool NT, bool NTL = false>
__global__ void __launch_bounds__(256) CopyChunkT(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                  size_t n) {
  const size_t step = static_cast<size_t>(blockDim.x) * UNROLL;
  const size_t per = ((n + gridDim.x - 1) / gridDim.x + step - 1) / step * step;
  const size_t begin = per * blockIdx.x;
  const size_t end = begin + per < n ? begin + per : n;
  size_t i = begin + threadIdx.x;
  for (; i + (UNROLL - 1) * blockDim.x < end; i += step) {
    uint4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) v[u] = Load16<NTL>(&src[i + u * blockDim.x]);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) Store16<NT>(&dst[i + u * blockDim.x], v[u]);
  }
  for (; i < end; i += blockDim.x) dst[i] = src[i];
}

// Matrix-core check: every wave keeps CHAINS independent 32x32 f32 accumulators
// and issues back-to-back v_mfma_f32_32x32x16_bf16 on them (two waves per SIMD,
// 8 per workgroup, one workgroup per CU), so the MFMA pipes never wait on a
// dependency. Shape from tools/hip/mfma_sweep.hip on the MI355X: 4 chains x 2
// waves/SIMD 2.35 PF/s vs 2.18 with one wave per SIMD; 8 chains spill. A = B = all ones (exact in bf16), so after n steps every
// accumulator element must be exactly 16 n -- a wrong element flags a bad
// matrix core. Rate = waves x iters x CHAINS x 32768 FLOP / time.
using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;
using f32x16 = __attribute__((ext_vector_type(16))) float;

template <int CHAINS>
__global__ void __launch_bounds__(512) MfmaKernel(float one, int iters, unsigned int* bad) {
  bf16x8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = static_cast<__bf16>(one);  // runtime value: nothing for the compiler to fold
    b[j] = static_cast<__bf16>(one);
  }
  f32x16 acc[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) acc[c] = f32x16{};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[c], 0, 0, 0);
  }
  const float want = 16.0f * static_cast<float>(iters) * one * one;
  unsigned int wrong = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) wrong += acc[c][r] != want;
  if (wrong) atomicAdd(bad, wrong);
}

__global__ void __launch_bounds__(256) SumKernel(const uint4* __restrict__ p, size_t n,
                                                 unsigned long long* total) {
  size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  unsigned long long acc = 0;
  for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint4 v = p[i];
    acc += static_cast<unsigned long long>(v.x) + v.y + v.z + v.w;
  }
  // wave64 reduction
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
  __shared__ unsigned long long partial[4];
  int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) partial[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long s = partial[0] + partial[1] + partial[2] + partial[3];
    atomicAdd(total, s);
  }
}

int Fail(char* out, int len, hipError_t e, const char* where) {
  snprintf(out, len, "{\"error\": \"%s: %s\"}", where, hipGetErrorString(e));
  return static_cast<int>(e) ? static_cast<int>(e) : 1;
}

// The probe runs inside other programs (the bench's torch.distributed ranks,
// where RCCL is bound to the rank's device): every entry point leaves the
// caller's current HIP device as it found it, on every return path.
struct DeviceGuard {
  int prev = -1;
  DeviceGuard() {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};

#define HIP_TRY(expr)                                   \
  do {                                                  \
    hipError_t _e = (expr);                             \
    if (_e != hipSuccess) return Fail(out, len, _e, #expr); \
  } while (0)

}  // namespace

// Bandwidth sweep over copy-kernel variants (unroll x store policy x grid size),
// used to pick the probe's default copy configuration on real hardware.
extern "C" int adp_probe_bw_sweep(int device, unsigned long long bytes, int iters, char* out, int len) {
  DeviceGuard device_guard;
  HIP_TRY(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  const int cus = prop.multiProcessorCount;
  size_t n = bytes / sizeof(uint4);
  uint4 *src = nullptr, *dst = nullptr;
  HIP_TRY(hipMalloc(&src, n * sizeof(uint4)));
  HIP_TRY(hipMalloc(&dst, n * sizeof(uint4)));
  hipLaunchKernelGGL(FillKernel, dim3(cus * 8), dim3(256), 0, 0, src, n);
  hipEvent_t e0, e1;
  HIP_TRY(hipEventCreate(&e0));
  HIP_TRY(hipEventCreate(&e1));
  using Launch = void (*)(dim3, const uint4*, uint4*, size_t);
  struct Variant { const char* name; Launch fn; };
#define V(K, U, NT, NTL) {#K "-" #U "x-st" #NT "-ld" #NTL, [](dim3 g, const uint4* s, uint4* d, size_t m) { \
    hipLaunchKernelGGL((K<U, NT, NTL>), g, dim3(256), 0, 0, s, d, m); }}
  Variant variants[] = {
      V(CopyKernelT, 1, false, false), V(CopyKernelT, 2, false, false), V(CopyKernelT, 4, false, false),
      V(CopyKernelT, 2, true, false),  V(CopyKernelT, 4, true, false),  V(CopyKernelT, 8, true, false),
      V(CopyKernelT, 2, true, true),   V(CopyKernelT, 4, true, true),
      V(CopyChunkT, 2, true, false),   V(CopyChunkT, 4, true, false),   V(CopyChunkT, 8, true, false),
      V(CopyChunkT, 4, true, true),    V(CopyChunkT, 4, false, false)};
#undef V
  std::string s = "[";
  bool first = true;
  for (int bpc : {1, 2, 4, 8}) {
    for (const auto& var : variants) {
      dim3 grid(cus * bpc);
      var.fn(grid, src, dst, n);  // warm-up
      HIP_TRY(hipEventRecord(e0, 0));
      for (int i = 0; i < iters; ++i) var.fn(grid, src, dst, n);
      HIP_TRY(hipEventRecord(e1, 0));
      HIP_TRY(hipEventSynchronize(e1));
      float ms = 0;
      HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
      double gbps = (2.0 * n * sizeof(uint4) * iters) / (ms * 1e-3) / 1e9;
      char buf[192];
      snprintf(buf, sizeof(buf), "%s{\"blocks_per_cu\": %d, \"variant\": \"%s\", \"gbps\": %.1f}",
               first ? "" : ", ", bpc, var.name, gbps);
      s += buf;
      first = false;
    }
  }
  s += "]";
  HIP_TRY(hipEventDestroy(e0));
  HIP_TRY(hipEventDestroy(e1));
  HIP_TRY(hipFree(src));
  HIP_TRY(hipFree(dst));
  snprintf(out, len, "%s", s.c_str());
  return 0;
}

// xGMI peer-read bandwidth between every ordered pair of visible devices: the
// kernel runs on device i and streams a buffer that lives on device j into local
// memory (the traffic a multi-GPU pod's collectives put on the link). A pair is
// only measured after hipDeviceEnablePeerAccess succeeded -- a kernel must never
// touch peer memory it has no mapping for. Output: {"devices": [...],
// "pairs": [{"dst": i, "src": j, "gbps": x | "no-peer-access": true}]}.
extern "C" int adp_probe_p2p(int ndev, unsigned long long bytes, int iters, char* out, int len) {
  DeviceGuard device_guard;
  int count = 0;
  HIP_TRY(hipGetDeviceCount(&count));
  if (ndev <= 0 || ndev > count) ndev = count;
  size_t n = bytes / sizeof(uint4);
  std::string s = "{\"devices\": " + std::to_string(ndev) + ", \"bytes\": " + std::to_string(n * sizeof(uint4)) +
                  ", \"pairs\": [";
  bool first = true;
  for (int i = 0; i < ndev; ++i) {
    for (int j = 0; j < ndev; ++j) {
      if (i == j) continue;
      char buf[160];
      int can = 0;
      HIP_TRY(hipDeviceCanAccessPeer(&can, i, j));
      if (can) {
        HIP_TRY(hipSetDevice(i));
        hipError_t e = hipDeviceEnablePeerAccess(j, 0);
        if (e == hipErrorPeerAccessAlreadyEnabled) {
          (void)hipGetLastError();  // clear the sticky "already enabled" status
          e = hipSuccess;
        }
        can = e == hipSuccess;
      }
      if (!can) {
        snprintf(buf, sizeof(buf), "%s{\"dst\": %d, \"src\": %d, \"no-peer-access\": true}", first ? "" : ", ", i, j);
        s += buf;
        first = false;
        continue;
      }
      uint4 *src = nullptr, *dst = nullptr;
      HIP_TRY(hipSetDevice(j));
      HIP_TRY(hipMalloc(&src, n * sizeof(uint4)));
      hipDeviceProp_t pj;
      HIP_TRY(hipGetDeviceProperties(&pj, j));
      hipLaunchKernelGGL(FillKernel, dim3(pj.multiProcessorCount * 4), dim3(256), 0, 0, src, n);
      HIP_TRY(hipDeviceSynchronize());
      HIP_TRY(hipSetDevice(i));
      HIP_TRY(hipMalloc(&dst, n * sizeof(uint4)));
      hipDeviceProp_t pi;
      HIP_TRY(hipGetDeviceProperties(&pi, i));
      dim3 grid(pi.multiProcessorCount);
      hipLaunchKernelGGL((CopyKernelT<4, true, true>), grid, dim3(256), 0, 0, src, dst, n);  // warm-up
      HIP_TRY(hipGetLastError());
      hipEvent_t e0, e1;
      HIP_TRY(hipEventCreate(&e0));
      HIP_TRY(hipEventCreate(&e1));
      HIP_TRY(hipEventRecord(e0, 0));
      for (int k = 0; k < iters; ++k)
        hipLaunchKernelGGL((CopyKernelT<4, true, true>), grid, dim3(256), 0, 0, src, dst, n);
      HIP_TRY(hipEventRecord(e1, 0));
      HIP_TRY(hipEventSynchronize(e1));
      float ms = 0;
      HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
      HIP_TRY(hipEventDestroy(e0));
      HIP_TRY(hipEventDestroy(e1));
      HIP_TRY(hipFree(dst));
      HIP_TRY(hipSetDevice(j));
      HIP_TRY(hipFree(src));
      double gbps = ms > 0 ? (static_cast<double>(n) * sizeof(uint4) * iters) / (ms * 1e-3) / 1e9 : 0.0;
      snprintf(buf, sizeof(buf), "%s{\"dst\": %d, \"src\": %d, \"gbps\": %.1f}", first ? "" : ", ", i, j, gbps);
      s += buf;
      first = false;
    }
  }
  s += "]}";
  snprintf(out, len, "%s", s.c_str());
  return 0;
}

// bf16 MFMA throughput + exactness on `device` (see MfmaKernel).
extern "C" int adp_probe_mfma(int device, int iters, char* out, int len) {
  DeviceGuard device_guard;
  HIP_TRY(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  if (iters <= 0 || iters > (1 << 20)) iters = 1 << 14;  // 16 n stays exact in f32 up to 2^20
  constexpr int kChains = 4;
  unsigned int* d_bad = nullptr;
  HIP_TRY(hipMalloc(&d_bad, sizeof(unsigned int)));
  HIP_TRY(hipMemset(d_bad, 0, sizeof(unsigned int)));
  const dim3 grid(prop.multiProcessorCount), block(512);
  hipLaunchKernelGGL(MfmaKernel<kChains>, grid, block, 0, 0, 1.0f, 64, d_bad);  // warm-up / clocks up
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemset(d_bad, 0, sizeof(unsigned int)));
  hipEvent_t e0, e1;
  HIP_TRY(hipEventCreate(&e0));
  HIP_TRY(hipEventCreate(&e1));
  HIP_TRY(hipEventRecord(e0, 0));
  hipLaunchKernelGGL(MfmaKernel<kChains>, grid, block, 0, 0, 1.0f, iters, d_bad);
  HIP_TRY(hipEventRecord(e1, 0));
  HIP_TRY(hipEventSynchronize(e1));
  float ms = 0;
  HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
  unsigned int bad = 0;
  HIP_TRY(hipMemcpy(&bad, d_bad, sizeof(bad), hipMemcpyDeviceToHost));
  HIP_TRY(hipEventDestroy(e0));
  HIP_TRY(hipEventDestroy(e1));
  HIP_TRY(hipFree(d_bad));
  const double waves = static_cast<double>(grid.x) * (block.x / 64);
  const double flops = waves * iters * kChains * (2.0 * 32 * 32 * 16);
  snprintf(out, len,
           "{\"device\": %d, \"instruction\": \"v_mfma_f32_32x32x16_bf16\", \"waves\": %.0f, "
           "\"iters\": %d, \"ms\": %.4f, \"bf16_tflops\": %.1f, \"wrong_elements\": %u, \"mfma_ok\": %s}",
           device, waves, iters, ms, ms > 0 ? flops / (ms * 1e-3) / 1e12 : 0.0, bad, bad == 0 ? "true" : "false");
  return bad == 0 ? 0 : 1;
}

extern "C" int adp_probe_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return -1;
  return n;
}

extern "C" int adp_probe_list(char* out, int len) {
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n));
  std::string s = "[";
  for (int d = 0; d < n; ++d) {
    hipDeviceProp_t p;
    HIP_TRY(hipGetDeviceProperties(&p, d));
    char buf[512];
    snprintf(buf, sizeof(buf),
             "%s{\"device\": %d, \"name\": \"%s\", \"arch\": \"%s\", \"pci\": \"%04x:%02x:%02x.0\", "
             "\"cus\": %d, \"total_mem_mib\": %zu}",
             d ? ", " : "", d, p.name, p.gcnArchName, p.pciDomainID, p.pciBusID, p.pciDeviceID,
             p.multiProcessorCount, static_cast<size_t>(p.totalGlobalMem >> 20));
    s += buf;
  }
  s += "]";
  snprintf(out, len, "%s", s.c_str());
  return 0;
}

// Which XCDs / CUs a queue of this process can use: under HSA_CU_MASK (e.g. a
// CU-partitioned time-slice replica, docs/SHARING_TUTORIAL.md) only the masked
// CUs show up. Returns {"xccs_seen", "cus_seen", "per_xcc": [...], "keys": [...]}
// with keys = xcc << 16 | HW_ID[15:8] (SE/SH/CU).
extern "C" int adp_probe_census(int device, char* out, int len) {
  DeviceGuard device_guard;
  HIP_TRY(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  const int blocks = prop.multiProcessorCount * 4;
  uint32_t* d = nullptr;
  HIP_TRY(hipMalloc(&d, blocks * sizeof(uint32_t)));
  HIP_TRY(hipMemset(d, 0xff, blocks * sizeof(uint32_t)));
  hipLaunchKernelGGL(HoldCensusKernel, dim3(blocks), dim3(64), 0, 0, d, 2000ull);  // 20 us per WG
  HIP_TRY(hipGetLastError());
  std::vector<uint32_t> rec(blocks);
  HIP_TRY(hipMemcpy(rec.data(), d, blocks * sizeof(uint32_t), hipMemcpyDeviceToHost));
  HIP_TRY(hipFree(d));
  std::set<uint32_t> keys, xccs;
  for (uint32_t r : rec) {
    if (r == 0xffffffffu) continue;
    keys.insert(r);
    xccs.insert(r >> 16);
  }
  std::vector<int> per_xcc(16, 0);
  for (uint32_t k : keys) ++per_xcc[(k >> 16) & 0xf];
  std::string s = "{\"device\": " + std::to_string(device) + ", \"cus\": " +
                  std::to_string(prop.multiProcessorCount) + ", \"xccs_seen\": " + std::to_string(xccs.size()) +
                  ", \"cus_seen\": " + std::to_string(keys.size()) + ", \"per_xcc\": [";
  int nx = xccs.empty() ? 0 : static_cast<int>(*xccs.rbegin()) + 1;
  for (int x = 0; x < nx; ++x) s += (x ? ", " : "") + std::to_string(per_xcc[x]);
  s += "], \"keys\": [";
  bool first = true;
  for (uint32_t k : keys) {
    s += (first ? "" : ", ") + std::to_string(k);
    first = false;
  }
  s += "]}";
  if (static_cast<int>(s.size()) >= len) return 3;
  snprintf(out, len, "%s", s.c_str());
  return 0;
}

// Launch-to-completion latency of a small kernel (VictimKernel, 2 workgroups per
// CU) timed on the host, `n` times after a warm-up: {"p50_us", "p99_us", ...}.
extern "C" int adp_probe_latency(int device, int n, char* out, int len) {
  DeviceGuard device_guard;
  HIP_TRY(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  if (n < 1) n = 1;
  float* d = nullptr;
  const int blocks = prop.multiProcessorCount * 2;
  HIP_TRY(hipMalloc(&d, blocks * sizeof(float)));
  hipStream_t st;
  HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  std::vector<double> us;
  us.reserve(n);
  for (int i = 0; i < n + 50; ++i) {
    auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(VictimKernel, dim3(blocks), dim3(256), 0, st, d, 2048);
    HIP_TRY(hipStreamSynchronize(st));
    if (i >= 50) us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  HIP_TRY(hipStreamDestroy(st));
  HIP_TRY(hipFree(d));
  std::sort(us.begin(), us.end());
  auto pct = [&](double p) { return us[static_cast<size_t>(p / 100.0 * (us.size() - 1))]; };
  snprintf(out, len,
           "{\"device\": %d, \"launches\": %d, \"p50_us\": %.1f, \"p90_us\": %.1f, \"p99_us\": %.1f, "
           "\"max_us\": %.1f}",
           device, n, pct(50), pct(90), pct(99), us.back());
  return 0;
}

// Saturates the device for `seconds`: back-to-back AggressorKernel launches of
// 8 workgroups x 256 lanes per CU, each holding its CUs for ~1 ms.
extern "C" int adp_probe_aggressor(int device, double seconds, char* out, int len) {
  DeviceGuard device_guard;
  HIP_TRY(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  float* d = nullptr;
  const int blocks = prop.multiProcessorCount * 8;
  HIP_TRY(hipMalloc(&d, blocks * sizeof(float)));
  auto t0 = std::chrono::steady_clock::now();
  long launches = 0;
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < seconds) {
    for (int k = 0; k < 4; ++k, ++launches)
      hipLaunchKernelGGL(AggressorKernel, dim3(blocks), dim3(256), 0, 0, d, 100000ull);  // 1 ms
    HIP_TRY(hipDeviceSynchronize());
  }
  HIP_TRY(hipFree(d));
  snprintf(out, len, "{\"device\": %d, \"aggressor_launches\": %ld, \"seconds\": %.2f}", device, launches,
           std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
  return 0;
}

extern "C" int adp_probe_run(int device, unsigned long long bytes, int iters, char* out, int len) {
  DeviceGuard device_guard;
  HIP_TRY(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  const int cus = prop.multiProcessorCount;

  // --- census ---
  const int census_blocks = cus * 8;
  uint32_t* d_census = nullptr;
  HIP_TRY(hipMalloc(&d_census, census_blocks * sizeof(uint32_t)));
  hipLaunchKernelGGL(CensusKernel, dim3(census_blocks), dim3(64), 0, 0, d_census);
  HIP_TRY(hipGetLastError());
  std::vector<uint32_t> census(census_blocks);
  HIP_TRY(hipMemcpy(census.data(), d_census, census_blocks * sizeof(uint32_t), hipMemcpyDeviceToHost));
  HIP_TRY(hipFree(d_census));
  std::set<uint32_t> xccs, cu_keys;
  for (uint32_t r : census) {
    xccs.insert(r >> 16);
    cu_keys.insert(r);
  }

  // --- bandwidth + checksum ---
  size_t n = bytes / sizeof(uint4);
  if (n < 1024) n = 1024;
  if (iters < 1) iters = 1;
  uint4 *src = nullptr, *dst = nullptr;
  unsigned long long* d_sum = nullptr;
  HIP_TRY(hipMalloc(&src, n * sizeof(uint4)));
  HIP_TRY(hipMalloc(&dst, n * sizeof(uint4)));
  HIP_TRY(hipMalloc(&d_sum, sizeof(unsigned long long)));
  const int blocks = cus * 8;
  // Copy shape picked by adp_probe_bw_sweep on MI355X (profiles/r1/session7/sweep_*.json):
  // 1 workgroup/CU, 4 x 16 B loads in flight per lane, non-temporal loads and
  // stores: 6.27 TB/s on 2 GiB (the ~6.3 TB/s achievable of an 8 TB/s part) vs
  // 5.90 TB/s for 2 WG/CU x2 with plain loads and 4.63 TB/s for the first cut.
  const int copy_blocks = cus;
  hipLaunchKernelGGL(FillKernel, dim3(blocks), dim3(256), 0, 0, src, n);
  hipLaunchKernelGGL((CopyKernelT<4, true, true>), dim3(copy_blocks), dim3(256), 0, 0, src, dst, n);  // warm-up
  HIP_TRY(hipGetLastError());
  hipEvent_t e0, e1;
  HIP_TRY(hipEventCreate(&e0));
  HIP_TRY(hipEventCreate(&e1));
  HIP_TRY(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL((CopyKernelT<4, true, true>), dim3(copy_blocks), dim3(256), 0, 0, src, dst, n);
  HIP_TRY(hipEventRecord(e1, 0));
  HIP_TRY(hipEventSynchronize(e1));
  float ms = 0;
  HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
  HIP_TRY(hipMemset(d_sum, 0, sizeof(unsigned long long)));
  hipLaunchKernelGGL(SumKernel, dim3(blocks), dim3(256), 0, 0, dst, n, d_sum);
  HIP_TRY(hipGetLastError());
  unsigned long long got = 0;
  HIP_TRY(hipMemcpy(&got, d_sum, sizeof(got), hipMemcpyDeviceToHost));
  // sum of the uint32 sequence 0..4n-1, each term taken mod 2^32
  unsigned long long want = 0;
  {
    unsigned long long m = 4ull * n;
    // terms are < 2^32 as long as 4n <= 2^32 (bytes <= 16 GiB); closed form otherwise too large
    want = (m % 2 == 0) ? (m / 2) * (m - 1) : m * ((m - 1) / 2);
  }
  HIP_TRY(hipEventDestroy(e0));
  HIP_TRY(hipEventDestroy(e1));
  HIP_TRY(hipFree(src));
  HIP_TRY(hipFree(dst));
  HIP_TRY(hipFree(d_sum));
  double gbps = ms > 0 ? (2.0 * n * sizeof(uint4) * iters) / (ms * 1e-3) / 1e9 : 0.0;
  snprintf(out, len,
           "{\"device\": %d, \"name\": \"%s\", \"arch\": \"%s\", \"pci\": \"%04x:%02x:%02x.0\", "
           "\"cus\": %d, \"total_mem_mib\": %zu, \"xccs_seen\": %zu, \"cus_seen\": %zu, "
           "\"copy_bytes\": %zu, \"copy_iters\": %d, \"copy_ms\": %.4f, \"hbm_copy_gbps\": %.1f, "
           "\"checksum_ok\": %s}",
           device, prop.name, prop.gcnArchName, prop.pciDomainID, prop.pciBusID, prop.pciDeviceID, cus,
           static_cast<size_t>(prop.totalGlobalMem >> 20), xccs.size(), cu_keys.size(),
           n * sizeof(uint4), iters, ms, gbps, got == want ? "true" : "false");
  return got == want ? 0 : 2;
}

// Memory-unit grant check (--enforce-memory-units): inside a pod the device
// must report the grant as its memory, refuse an allocation past it and allow
// one well inside it. Host-side HIP calls only.
extern "C" int adp_probe_grant(int device, unsigned long long grant_mib, char* out, int len) {
  DeviceGuard device_guard;
  HIP_TRY(hipSetDevice(device));
  size_t free_b = 0, total_b = 0;
  HIP_TRY(hipMemGetInfo(&free_b, &total_b));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  const size_t grant = static_cast<size_t>(grant_mib) << 20;
  void* p = nullptr;
  bool over_refused = hipMalloc(&p, grant + (size_t{64} << 20)) != hipSuccess;
  if (!over_refused) (void)hipFree(p);
  (void)hipGetLastError();  // the refusal is expected: clear it
  p = nullptr;
  bool half_ok = hipMalloc(&p, grant / 2) == hipSuccess;
  // While it is held: the grant's free memory went down by it, and -- when the
  // plugin mounted the grant's accounting file -- the file counts it (what
  // /metrics reports for this container).
  size_t free_held = 0, total_held = 0;
  bool accounted = half_ok && hipMemGetInfo(&free_held, &total_held) == hipSuccess && free_held + grant / 2 <= free_b;
  const char* file_state = "null";
  if (const char* f = getenv("ADP_MEMCAP_FILE"); f && half_ok) {
    uint64_t used = 0;
    int fd = open(f, O_RDONLY | O_CLOEXEC);
    bool got = fd >= 0 && device >= 0 && device < adp_memcap::kMaxDevices &&
               pread(fd, &used, sizeof(used), offsetof(adp_memcap::Area, used) + device * sizeof(uint64_t)) ==
                   static_cast<ssize_t>(sizeof(used));
    if (fd >= 0) close(fd);
    file_state = got && used >= grant / 2 ? "true" : "false";
  }
  if (half_ok) (void)hipFree(p);
  (void)hipGetLastError();
  bool ok = over_refused && half_ok && accounted && (total_b >> 20) == grant_mib &&
            (prop.totalGlobalMem >> 20) == grant_mib && strcmp(file_state, "false") != 0;
  snprintf(out, len,
           "{\"device\": %d, \"grant_mib\": %llu, \"total_mib\": %zu, \"free_mib\": %zu, \"props_mib\": %zu, "
           "\"over_grant_refused\": %s, \"half_grant_ok\": %s, \"accounted\": %s, \"grant_file_counts\": %s, "
           "\"enforced\": %s}",
           device, grant_mib, total_b >> 20, free_b >> 20, static_cast<size_t>(prop.totalGlobalMem >> 20),
           over_refused ? "true" : "false", half_ok ? "true" : "false", accounted ? "true" : "false", file_state,
           ok ? "true" : "false");
  return ok ? 0 : 3;
}

// Sweep of the MFMA probe's shape: accumulator chains per wave x waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -o build/mfma_sweep tools/hip/mfma_sweep.hip
#include <hip/hip_runtime.h>
#include <cstdio>

using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;
using f32x16 = __attribute__((ext_vector_type(16))) float;

template <int CHAINS>
__global__ void K(float one, int iters, unsigned* bad) {
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (__bf16)one; b[j] = (__bf16)one; }
  f32x16 acc[CHAINS];
  for (int c = 0; c < CHAINS; ++c) acc[c] = f32x16{};
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[c], 0, 0, 0);
  unsigned w = 0;
  for (int c = 0; c < CHAINS; ++c)
    for (int r = 0; r < 16; ++r) w += acc[c][r] != 16.0f * iters;
  if (w) atomicAdd(bad, w);
}

template <int CHAINS>
void Run(int cus, int threads, int iters, unsigned* bad) {
  hipLaunchKernelGGL(K<CHAINS>, dim3(cus), dim3(threads), 0, 0, 1.0f, 256, bad);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL(K<CHAINS>, dim3(cus), dim3(threads), 0, 0, 1.0f, iters, bad);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  double flops = double(cus) * (threads / 64) * iters * CHAINS * 32768.0;
  printf("{\"chains\": %d, \"waves_per_cu\": %d, \"tflops\": %.1f}\n", CHAINS, threads / 64, flops / (ms * 1e-3) / 1e12);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  unsigned* bad;
  hipMalloc(&bad, 4);
  hipMemset(bad, 0, 4);
  for (int threads : {256, 512}) {
    int iters = threads == 256 ? 1 << 15 : 1 << 14;
    Run<2>(p.multiProcessorCount, threads, iters * 2, bad);
    Run<4>(p.multiProcessorCount, threads, iters, bad);
    Run<8>(p.multiProcessorCount, threads, iters / 2, bad);
  }
  unsigned b = 0;
  hipMemcpy(&b, bad, 4, hipMemcpyDeviceToHost);
  printf("{\"wrong\": %u}\n", b);
  return b != 0;
}

// Probe: cost of one FNV-1a 64 step (flows.go:60-70) on gfx950, two forms:
//   mul: v_mad_u64_u32 + v_mul_lo_u32 (what the compiler makes of h * prime)
//   sha: x * (2^40 + 435) as four v_lshl_add_u64 (435x = 3x + 48x + 384x), inline asm
// 4 independent chains per lane, 8 waves per SIMD on every CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint64_t step_mul(uint64_t h, uint32_t b) {
  h ^= b;
  uint32_t lo = (uint32_t)h, hi = (uint32_t)(h >> 32);
  uint64_t m = (uint64_t)lo * 0x1b3u;
  uint32_t rhi = (uint32_t)(m >> 32) + hi * 0x1b3u + (lo << 8);
  return ((uint64_t)rhi << 32) | (uint32_t)m;
}
__device__ __forceinline__ uint64_t step_sha(uint64_t h, uint32_t b) {
  const uint64_t x = h ^ b;
  uint64_t a, r, o;
  asm volatile("v_lshl_add_u64 %0, %1, 1, %1" : "=v"(a) : "v"(x));
  asm volatile("v_lshl_add_u64 %0, %1, 4, %1" : "=v"(r) : "v"(a));
  asm volatile("v_lshl_add_u64 %0, %1, 7, %2" : "=v"(o) : "v"(a), "v"(r));
  asm volatile("v_lshl_add_u64 %0, %1, 40, %2" : "=v"(r) : "v"(x), "v"(o));
  return r;
}
template <int K>
__global__ void k(uint64_t* out, uint32_t n) {
  uint64_t h0 = threadIdx.x, h1 = h0 * 3, h2 = h0 * 5, h3 = h0 * 7;
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t b = i & 0xff;
    if (K == 0) {
      h0 = step_mul(h0, b); h1 = step_mul(h1, b); h2 = step_mul(h2, b); h3 = step_mul(h3, b);
    } else {
      h0 = step_sha(h0, b); h1 = step_sha(h1, b); h2 = step_sha(h2, b); h3 = step_sha(h3, b);
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = h0 ^ h1 ^ h2 ^ h3;
}
int main() {
  const int blocks = 256 * 8, threads = 256;
  uint64_t* d;
  (void)hipMalloc(&d, sizeof(uint64_t) * blocks * threads);
  uint64_t ref[2] = {0, 0};
  for (int kind = 0; kind < 2; kind++) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const uint32_t n = 4096;
    for (int rep = 0; rep < 2; rep++) {
      (void)hipEventRecord(e0);
      if (kind == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(threads), 0, 0, d, n);
      else hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(threads), 0, 0, d, n);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
    }
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    uint64_t h;
    (void)hipMemcpy(&h, d + 12345, 8, hipMemcpyDeviceToHost);
    ref[kind] = h;
    // steps per wave per SIMD-cycle at an assumed 2.4 GHz, 1024 SIMDs
    const double steps = (double)blocks * threads / 64 * 4 * n;
    printf("%s: %.3f ms, %.2f cycles per wave-step (2.4 GHz, 1024 SIMDs)\n", kind ? "shift-add" : "mul", ms,
           ms * 1e-3 * 2.4e9 * 1024 / steps);
  }
  printf("same hashes: %s\n", ref[0] == ref[1] ? "yes" : "NO");
  return 0;
}

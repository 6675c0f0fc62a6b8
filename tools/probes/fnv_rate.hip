// Probe: cost of one FNV-1a 64 step (flows.go:60-70) on gfx950, three forms:
//   0 mul: (h ^ b) * prime as the compiler makes it (v_mad_u64_u32 + v_mul_lo_u32 + adds)
//   1 mad: lo' : hi' = mad_u64(x, 0x1b3, (hi * 0x1b3 + (x << 8)) << 32), x = lo ^ b
//   2 sha: 435 x as v_lshl_add_u64 steps (shift <= 4: 3x, 51x, 27x, 408x + 27x), + x << 40
// 4 independent chains per lane, 8 waves per SIMD on every CU. Both forms must agree.
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
__device__ __forceinline__ uint64_t step_mad(uint64_t h, uint32_t b) {
  const uint32_t x = (uint32_t)h ^ b, hi = (uint32_t)(h >> 32);
  const uint32_t s = hi * 0x1b3u + (x << 8);
  return (uint64_t)x * 0x1b3u + ((uint64_t)s << 32);
}
__device__ __forceinline__ uint64_t step_sha(uint64_t h, uint32_t b) {
  const uint64_t x = h ^ b;
  uint64_t x3, x51, x27, r;
  asm("v_lshl_add_u64 %0, %1, 1, %1" : "=v"(x3) : "v"(x));
  asm("v_lshl_add_u64 %0, %1, 4, %1" : "=v"(x51) : "v"(x3));
  asm("v_lshl_add_u64 %0, %1, 3, %1" : "=v"(x27) : "v"(x3));
  asm("v_lshl_add_u64 %0, %1, 3, %2" : "=v"(r) : "v"(x51), "v"(x27));
  return r + ((uint64_t)(uint32_t)x << 40);
}
template <int K>
__global__ void k(uint64_t* out, uint32_t n) {
  uint64_t h0 = threadIdx.x, h1 = h0 * 3, h2 = h0 * 5, h3 = h0 * 7;
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t b = i & 0xff;
    if (K == 0) {
      h0 = step_mul(h0, b); h1 = step_mul(h1, b); h2 = step_mul(h2, b); h3 = step_mul(h3, b);
    } else if (K == 2) {
      h0 = step_sha(h0, b); h1 = step_sha(h1, b); h2 = step_sha(h2, b); h3 = step_sha(h3, b);
    } else {
      h0 = step_mad(h0, b); h1 = step_mad(h1, b); h2 = step_mad(h2, b); h3 = step_mad(h3, b);
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = h0 ^ h1 ^ h2 ^ h3;
}
int main() {
  const int blocks = 256 * 8, threads = 256;
  uint64_t* d;
  (void)hipMalloc(&d, sizeof(uint64_t) * blocks * threads);
  uint64_t ref[3] = {0, 0, 0};
  for (int kind = 0; kind < 3; kind++) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const uint32_t n = 4096;
    float ms = 0;
    for (int rep = 0; rep < 3; rep++) {
      (void)hipEventRecord(e0);
      if (kind == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(threads), 0, 0, d, n);
      else if (kind == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(threads), 0, 0, d, n);
      else hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(threads), 0, 0, d, n);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&ms, e0, e1);
    }
    uint64_t h = 0;
    (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    ref[kind] = h;
    // steps per SIMD: blocks*threads/64 waves * 4 chains * n over 1024 SIMDs
    const double waves = (double)blocks * threads / 64, steps = waves * 4 * n;
    const double cyc = ms * 1e-3 * 2.4e9 * 1024;  // SIMD-cycles at 2.4 GHz
    printf("kind %d (%s): %.3f ms, %.2f SIMD-cycles per wave-step\n", kind, kind == 0 ? "mul" : kind == 1 ? "mad" : "sha",
           ms, cyc / steps);
  }
  const bool ok = ref[0] == ref[1] && ref[0] == ref[2];
  printf("agree: %s\n", ok ? "yes" : "NO");
  return ok ? 0 : 1;
}

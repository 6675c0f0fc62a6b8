// Issue-rate probe: shader cycles per instruction per wave for a stream of
// independent scalar (s_movk_i32), vector (v_add_u32) or mixed (1:1)
// instructions, at 1..8 waves per SIMD (256-thread blocks, one wave per SIMD,
// k blocks per CU). Shows whether scalar issue is a per-CU or per-SIMD
// resource on gfx950, i.e. how much a wave's SALU count costs when the CU is
// full.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/probes/bin/issue_probe tools/probes/issue_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

template <int MODE>
__global__ __launch_bounds__(256) void issue_kernel(uint32_t iters, uint64_t* out) {
  uint32_t s0 = 1, s1 = 2, s2 = 3, s3 = 4, s4 = 5, s5 = 6, s6 = 7, s7 = 8;
  uint32_t v0 = threadIdx.x, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3, v4 = v0 + 4, v5 = v0 + 5, v6 = v0 + 6, v7 = v0 + 7;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t k = 0; k < iters; k++) {
    if (MODE == 0 || MODE == 2) {
      asm volatile(
          // s_movk_i32: no SCC write (an s_add here clobbered the loop's branch condition)
          "s_movk_i32 %0, 0x11\n\ts_movk_i32 %1, 0x12\n\ts_movk_i32 %2, 0x13\n\ts_movk_i32 %3, 0x14\n\t"
          "s_movk_i32 %4, 0x15\n\ts_movk_i32 %5, 0x16\n\ts_movk_i32 %6, 0x17\n\ts_movk_i32 %7, 0x18"
          : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7));
    }
    if (MODE == 1 || MODE == 2) {
      asm volatile(
          "v_add_u32 %0, %0, 1\n\tv_add_u32 %1, %1, 1\n\tv_add_u32 %2, %2, 1\n\tv_add_u32 %3, %3, 1\n\t"
          "v_add_u32 %4, %4, 1\n\tv_add_u32 %5, %5, 1\n\tv_add_u32 %6, %6, 1\n\tv_add_u32 %7, %7, 1"
          : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7));
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) {
    const uint64_t w = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
    out[2 * w] = t1 - t0;
    out[2 * w + 1] = (uint64_t)(s0 + s1 + s2 + s3 + s4 + s5 + s6 + s7) + v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7;
  }
}

int main() {
  int dev = 0, ncu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const uint32_t iters = 4096;
  uint64_t* out;
  CK(hipMalloc(&out, (size_t)ncu * 8 * 4 * 2 * 8));
  std::vector<uint64_t> h((size_t)ncu * 8 * 4 * 2);
  const char* names[3] = {"salu", "valu", "mixed"};
  printf("{\"iters\": %u, \"instr_per_iter\": 8, \"rows\": [\n", iters);
  bool first = true;
  for (int mode = 0; mode < 3; mode++) {
    for (int k = 1; k <= 8; k++) {
      const int grid = ncu * k;
      for (int rep = 0; rep < 2; rep++) {
        if (mode == 0) hipLaunchKernelGGL(issue_kernel<0>, dim3(grid), dim3(256), 0, 0, iters, out);
        if (mode == 1) hipLaunchKernelGGL(issue_kernel<1>, dim3(grid), dim3(256), 0, 0, iters, out);
        if (mode == 2) hipLaunchKernelGGL(issue_kernel<2>, dim3(grid), dim3(256), 0, 0, iters, out);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
      }
      CK(hipMemcpy(h.data(), out, (size_t)grid * 4 * 2 * 8, hipMemcpyDeviceToHost));
      double sum = 0;
      for (int w = 0; w < grid * 4; w++) sum += (double)h[2 * w];
      const double cyc = sum / (grid * 4) / (iters * 8.0);  // shader cycles per instruction (per kind) per wave
      printf("%s  {\"mode\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_instr_per_wave\": %.3f, "
             "\"instr_per_cycle_per_simd\": %.3f}",
             first ? "" : ",\n", names[mode], k, cyc, k / cyc);
      first = false;
      fflush(stdout);
    }
  }
  printf("\n]}\n");
  CK(hipFree(out));
  return 0;
}

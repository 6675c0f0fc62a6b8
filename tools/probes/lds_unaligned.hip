// Probe: are unaligned ds_read_b32 / ds_read_b64 byte-exact on this gfx950 setup?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(uint32_t* out) {
  __shared__ uint8_t s[256];
  for (int i = threadIdx.x; i < 256; i += 64) s[i] = (uint8_t)(i * 7 + 3);
  __syncthreads();
  const int a = threadIdx.x;  // byte address 0..63
  uint32_t v;
  asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((uint32_t)(uintptr_t)(s + a)));
  uint32_t w = s[a] | s[a + 1] << 8 | s[a + 2] << 16 | (uint32_t)s[a + 3] << 24;
  out[a] = v == w;
}
int main() {
  uint32_t* d; (void)hipMalloc(&d, 256);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  uint32_t h[64]; (void)hipMemcpy(h, d, 256, hipMemcpyDeviceToHost);
  int ok = 0; for (int i = 0; i < 64; i++) ok += h[i];
  printf("unaligned ds_read_b32 exact on %d/64 byte offsets\n", ok);
  return 0;
}

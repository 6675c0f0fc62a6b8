// Probe: LDS-DMA (global_load_lds_dwordx4) as the persistent decode kernel uses it.
// 4 waves; wave w issues 6 instructions k = 0..5 with M0 = its region + 1024 k and a
// per-lane source address that gathers (packet q, chunk c) = divmod(64 k + lane, 6) of
// 64 scattered "packets" at arbitrary 16-byte-aligned offsets (plus argv[1]
// bytes: 4, 8, 12 test dword-aligned sources). Expected: LDS byte
// 96 q + 16 c + b of the wave's region = source byte 16 c + b of packet q, i.e. the
// destination is M0 + 16 * lane whatever the source.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

extern __shared__ __attribute__((aligned(16))) uint32_t smem[];

__device__ __forceinline__ void dma16(const uint8_t* src, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
}

__global__ void k(const uint8_t* data, const uint64_t* pk_off, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // a different packet per lane and wave
  const uint64_t my = pk_off[wave * 64 + lane];
  const uint32_t region = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem + wave * 6144u);
  for (int i = threadIdx.x; i < 4 * 1536; i += 256) smem[i] = 0xdeadbeefu;
  __syncthreads();
#pragma unroll
  for (int kk = 0; kk < 6; kk++) {
    const uint32_t e = 64u * kk + lane, q = e / 6, c = e - q * 6;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(q * 4), (int)(uint32_t)my);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(q * 4), (int)(uint32_t)(my >> 32));
    const uint64_t o = ((uint64_t)hi << 32 | lo) + 16u * c;
    dma16(data + o, region + 1024u * kk);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 4 * 1536; i += 256) out[i] = smem[i];
}

int main(int argc, char** argv) {
  const int shift = argc > 1 ? atoi(argv[1]) : 0;
  const size_t nbytes = 1 << 22;
  std::vector<uint8_t> h(nbytes);
  for (size_t i = 0; i < nbytes; i++) h[i] = (uint8_t)(i * 2654435761u >> 13);
  std::vector<uint64_t> off(256);
  for (int i = 0; i < 256; i++) off[i] = ((uint64_t)(i * 7919 + 13) * 16) % (nbytes - 256) + shift;
  uint8_t* d;
  uint64_t* doff;
  uint32_t* dout;
  (void)hipMalloc(&d, nbytes);
  (void)hipMalloc(&doff, 256 * 8);
  (void)hipMalloc(&dout, 4 * 6144);
  (void)hipMemcpy(d, h.data(), nbytes, hipMemcpyHostToDevice);
  (void)hipMemcpy(doff, off.data(), 256 * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(256), 4 * 6144, 0, d, doff, dout);
  std::vector<uint8_t> got(4 * 6144);
  (void)hipMemcpy(got.data(), dout, got.size(), hipMemcpyDeviceToHost);
  size_t bad = 0;
  for (int w = 0; w < 4; w++)
    for (int q = 0; q < 64; q++)
      for (int b = 0; b < 96; b++)
        bad += got[w * 6144 + 96 * q + b] != h[off[w * 64 + q] + b];
  printf("LDS-DMA gather, source shift %d: %zu of %d bytes differ (%s)\n", shift, bad, 4 * 6144, bad ? "FAIL" : "ok");
  return bad != 0;
}

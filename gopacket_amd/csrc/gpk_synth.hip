// gpk_synth.hip — device and host generators of the synthetic benchmark
// batches (gpk_synth.h). Bench/test infrastructure, built as libgpk_synth.so,
// never linked into libgpk.so. Packets are generated in HBM directly (C3 is
// ~100 GB at 64 M packets, far more than is worth copying over PCIe).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstring>

#include "gpk_synth.h"

using namespace gpk_synth;

namespace {

// Byte sink that coalesces a packet's bytes into aligned dword stores; the
// first and last dword of a packet may be shared with a neighbour packet
// (written by another lane), so those are written bytewise.
struct DevSink {
  uint8_t* base;  // packet start
  uint32_t acc = 0, mask = 0;
  uintptr_t cur = ~uintptr_t(0);
  __device__ void flush() {
    if (cur == ~uintptr_t(0)) return;
    if (mask == 0xf) {
      *reinterpret_cast<uint32_t*>(cur) = acc;
    } else {
      for (int k = 0; k < 4; k++)
        if (mask & (1u << k)) reinterpret_cast<uint8_t*>(cur)[k] = (uint8_t)(acc >> (8 * k));
    }
    acc = mask = 0;
  }
  __device__ void operator()(uint32_t p, uint32_t b) {
    uintptr_t a = reinterpret_cast<uintptr_t>(base + p);
    uintptr_t w = a & ~uintptr_t(3);
    if (w != cur) {
      flush();
      cur = w;
    }
    uint32_t k = (uint32_t)(a & 3);
    acc |= b << (8 * k);
    mask |= 1u << k;
  }
};

struct Widen {
  __host__ __device__ uint64_t operator()(uint32_t x) const { return x; }
};

struct HostSink {
  uint8_t* base;
  void operator()(uint32_t p, uint32_t b) { base[p] = (uint8_t)b; }
};

__global__ void len_kernel(int cfg, uint64_t first, uint64_t n, uint32_t* caplens) {
  uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) caplens[k] = frame_len(cfg, first + k);
}

__global__ void fixed_off_kernel(uint64_t n, uint32_t len, uint64_t* offsets) {
  uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) offsets[k] = k * (uint64_t)len;
}

__global__ void fill_kernel(int cfg, uint64_t first, uint64_t n, uint8_t* data, const uint64_t* offsets) {
  uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  Desc d;
  describe(cfg, first + k, d);
  finish(d, first + k);
  DevSink s{data + offsets[k]};
  emit(d, first + k, s);
  s.flush();
}

}  // namespace

extern "C" {

uint32_t gpk_synth_len(int cfg, uint64_t i) { return frame_len(cfg, i); }

// Packet i of config cfg into out (>= gpk_synth_len bytes). Returns its length.
uint32_t gpk_synth_fill(int cfg, uint64_t i, uint8_t* out) {
  Desc d;
  describe(cfg, i, d);
  finish(d, i);
  HostSink s{out};
  emit(d, i, s);
  return d.len;
}

// Host batch of packets [first, first+n), packed contiguously.
// offsets/caplens: [n]; data: sum of lengths (query with data == NULL).
uint64_t gpk_synth_batch_host(int cfg, uint64_t first, uint64_t n, uint8_t* data, uint64_t* offsets,
                              uint32_t* caplens) {
  uint64_t off = 0;
  for (uint64_t k = 0; k < n; k++) {
    uint32_t l = frame_len(cfg, first + k);
    if (offsets) offsets[k] = off;
    if (caplens) caplens[k] = l;
    if (data) gpk_synth_fill(cfg, first + k, data + off);
    off += l;
  }
  return off;
}

// Device batch: caplens[n], offsets[n] (exclusive scan), then the bytes.
// data must hold gpk_synth_bytes(cfg, first, n) bytes (+16 slack).
int gpk_synth_device(int cfg, uint64_t first, uint64_t n, uint8_t* data, uint64_t* offsets, uint32_t* caplens,
                     void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (!n) return 0;
  dim3 b(256), g((unsigned)((n + 255) / 256));
  hipLaunchKernelGGL(len_kernel, g, b, 0, s, cfg, first, n, caplens);
  if (cfg == GPK_SYNTH_C2_UDP64 || cfg == GPK_SYNTH_C3_TCP1500) {
    hipLaunchKernelGGL(fixed_off_kernel, g, b, 0, s, n, frame_len(cfg, 0), offsets);
  } else {
    // 64-bit running sum (IMIX batches exceed 4 GiB)
    hipcub::TransformInputIterator<uint64_t, Widen, const uint32_t*> in(caplens, Widen());
    size_t tmp_bytes = 0;
    hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, in, offsets, (int)n, s);
    void* tmp = nullptr;
    if (hipMallocAsync(&tmp, tmp_bytes, s) != hipSuccess) return -2;
    hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, in, offsets, (int)n, s);
    (void)hipFreeAsync(tmp, s);
  }
  hipLaunchKernelGGL(fill_kernel, g, b, 0, s, cfg, first, n, data, offsets);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// Total bytes of packets [first, first+n) (host loop for IMIX; closed form otherwise).
uint64_t gpk_synth_bytes(int cfg, uint64_t first, uint64_t n) {
  if (cfg == GPK_SYNTH_C2_UDP64 || cfg == GPK_SYNTH_C3_TCP1500) return n * frame_len(cfg, 0);
  uint64_t t = 0;
  for (uint64_t k = 0; k < n; k++) t += frame_len(cfg, first + k);
  return t;
}

}  // extern "C"

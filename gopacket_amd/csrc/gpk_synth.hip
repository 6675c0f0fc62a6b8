// gpk_synth.hip — device and host generators of the synthetic benchmark
// batches (gpk_synth.h). Bench/test infrastructure, built as libgpk_synth.so,
// never linked into libgpk.so. Packets are generated in HBM directly (C3 is
// ~100 GB at 64 M packets, far more than is worth copying over PCIe).
#include <hip/hip_runtime.h>
#include <chrono>
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <atomic>
#include <thread>
#include <vector>
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

// Streaming-read probe: byte sum of data[0, nbytes) (nbytes % 16 == 0) with
// coalesced 16-byte non-temporal loads, 4 in flight per lane. It moves the
// same bytes as the decode kernel with none of its work, so its rate is the
// achievable HBM read rate of this box for that buffer (bench.py context
// for roofline.frac).
__global__ __launch_bounds__(256) void probe_read_kernel(const uint8_t* data, uint64_t nvec, uint32_t* out) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const u32x4* v = reinterpret_cast<const u32x4*>(data);
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t acc = 0;
  for (; k + 3 * stride < nvec; k += 4 * stride) {
    u32x4 a = __builtin_nontemporal_load(v + k);
    u32x4 b = __builtin_nontemporal_load(v + k + stride);
    u32x4 c = __builtin_nontemporal_load(v + k + 2 * stride);
    u32x4 d = __builtin_nontemporal_load(v + k + 3 * stride);
    acc = __builtin_amdgcn_udot4(a.x ^ b.y ^ c.z ^ d.w, 0x01010101u, acc, false);
    acc = __builtin_amdgcn_udot4(a.y ^ b.z ^ c.w ^ d.x, 0x01010101u, acc, false);
    acc = __builtin_amdgcn_udot4(a.z ^ b.w ^ c.x ^ d.y, 0x01010101u, acc, false);
    acc = __builtin_amdgcn_udot4(a.w ^ b.x ^ c.y ^ d.z, 0x01010101u, acc, false);
  }
  for (; k < nvec; k += stride) {
    u32x4 a = __builtin_nontemporal_load(v + k);
    acc = __builtin_amdgcn_udot4(a.x ^ a.y ^ a.z ^ a.w, 0x01010101u, acc, false);
  }
  if (acc == 0x9e3779b9u) out[0] = acc;  // keep the loads live; practically never stores
}

// Host-write probe: 16-byte vector stores from the CUs straight into pinned
// host memory (dst is a host pointer the device can address), grid-stride:
// results written over the link by the kernel instead of a DtoH copy
// (tools/duplex_probe.py).
__global__ __launch_bounds__(256) void probe_hostwrite_kernel(uint8_t* dst, uint64_t nvec) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  u32x4* v = reinterpret_cast<u32x4*>(dst);
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < nvec; k += stride) {
    const uint32_t x = (uint32_t)k;
    __builtin_nontemporal_store(u32x4{x, x ^ 1u, x ^ 2u, x ^ 3u}, v + k);
  }
}

// Mixed probe: the streaming read of probe_read_kernel over data[0, nbytes)
// and, at the same time, non-temporal 16-byte stores over wbuf[0, wbytes) (the
// records / flows / fields a decode writes): the first `writers` blocks store,
// the rest read, each side grid-strided over its own blocks. Its rate (read +
// written bytes over the time) is the box's achievable HBM rate for that mix.
__global__ __launch_bounds__(256) void probe_mixed_kernel(const uint8_t* data, uint64_t nvec, uint8_t* wbuf,
                                                          uint64_t wvec, uint32_t writers, uint32_t* out) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  if (blockIdx.x < writers) {
    u32x4* w = reinterpret_cast<u32x4*>(wbuf);
    const uint64_t stride = (uint64_t)writers * 256;
    const u32x4 x = {blockIdx.x, threadIdx.x, 0x9e3779b9u, 1u};
    for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < wvec; k += stride) __builtin_nontemporal_store(x, w + k);
    return;
  }
  const u32x4* v = reinterpret_cast<const u32x4*>(data);
  const uint64_t stride = (uint64_t)(gridDim.x - writers) * 256;
  uint64_t k = (uint64_t)(blockIdx.x - writers) * 256 + threadIdx.x;
  uint32_t acc = 0;
  for (; k + 3 * stride < nvec; k += 4 * stride) {
    u32x4 a = __builtin_nontemporal_load(v + k);
    u32x4 b = __builtin_nontemporal_load(v + k + stride);
    u32x4 c = __builtin_nontemporal_load(v + k + 2 * stride);
    u32x4 d = __builtin_nontemporal_load(v + k + 3 * stride);
    acc = __builtin_amdgcn_udot4(a.x ^ b.y ^ c.z ^ d.w, 0x01010101u, acc, false);
    acc = __builtin_amdgcn_udot4(a.y ^ b.z ^ c.w ^ d.x, 0x01010101u, acc, false);
    acc = __builtin_amdgcn_udot4(a.z ^ b.w ^ c.x ^ d.y, 0x01010101u, acc, false);
    acc = __builtin_amdgcn_udot4(a.w ^ b.x ^ c.y ^ d.z, 0x01010101u, acc, false);
  }
  for (; k < nvec; k += stride) {
    u32x4 a = __builtin_nontemporal_load(v + k);
    acc = __builtin_amdgcn_udot4(a.x ^ a.y ^ a.z ^ a.w, 0x01010101u, acc, false);
  }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

// Re-read probe (the traffic question): one wave per region of
// 64 "packets" of pkt bytes, the decode kernel's access pattern without its
// work. mode 0: the region streamed once (1 KiB per pass, 16 B per lane,
// non-temporal, 8 passes in flight); mode 1: first each lane's 6-chunk
// header window at its packet (temporal, as the decode kernel loads it), then
// the same stream, so the window's lines are fetched twice; mode 2: the
// header windows alone. If the second fetch of a window line costs DRAM
// bandwidth, mode 1 takes about mode 0 + the re-fetched share; if it is served
// on chip (L2 / Infinity Cache), mode 1 takes about mode 0. mode 3: the
// header windows, then a stream that skips the granules they hold (what a
// phase B taking those granules from the LDS windows would fetch). mode 4:
// the block's four waves stream its 256-packet region together, wave w taking
// the w-th KiB of every 4 KiB (the same bytes as mode 0 in 4 KiB passes per
// block instead of 1 KiB passes per wave: a quarter as many concurrent streams).
__global__ __launch_bounds__(256) void probe_reread_kernel(const uint8_t* data, uint64_t nbytes, uint32_t pkt,
                                                           int mode, uint32_t* out) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint64_t R = 64ull * pkt, base = wave * R;
  uint32_t acc = 0;
  if (mode == 4) {
    const uint64_t bb = (uint64_t)blockIdx.x * 4 * R;
    if (bb + 4 * R > nbytes) return;
    const u32x4* v = reinterpret_cast<const u32x4*>(data + bb);
    const uint32_t nv = (uint32_t)(4 * R / 16);
    uint32_t k = threadIdx.x;  // wave w's lanes: vectors 64 w .. 64 w + 63 of each 256
    for (; k + 7 * 256 < nv; k += 8 * 256) {
      u32x4 a[8];
#pragma unroll
      for (int j = 0; j < 8; j++) a[j] = __builtin_nontemporal_load(v + k + 256 * j);
#pragma unroll
      for (int j = 0; j < 8; j++) acc = __builtin_amdgcn_udot4(a[j].x ^ a[j].y ^ a[j].z ^ a[j].w, 0x01010101u, acc, false);
    }
    for (; k < nv; k += 256) {
      const u32x4 a = __builtin_nontemporal_load(v + k);
      acc = __builtin_amdgcn_udot4(a.x ^ a.y ^ a.z ^ a.w, 0x01010101u, acc, false);
    }
    if (acc == 0x9e3779b9u) out[0] = acc;
    return;
  }
  if (base + R > nbytes) return;
  if (mode >= 1) {  // 1, 2, 3
    const uint8_t* h = data + ((base + (uint64_t)lane * pkt) & ~15ull);
    u32x4 w[6];
#pragma unroll
    for (int k = 0; k < 6; k++) w[k] = *reinterpret_cast<const u32x4*>(h + 16 * k);
#pragma unroll
    for (int k = 0; k < 6; k++) acc = __builtin_amdgcn_udot4(w[k].x ^ w[k].y ^ w[k].z ^ w[k].w, 0x01010101u, acc, false);
  }
  if (mode <= 1 || mode == 3) {
    const u32x4* v = reinterpret_cast<const u32x4*>(data + base);
    const uint32_t nv = (uint32_t)(R / 16);
    // mode 3: the stream skips the 16-byte granules a header window holds
    // (range-checked loads out of range: zeros, no memory access)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(data + base), 0, (int)R, 0x00020000);
    const uint32_t inv = (uint32_t)((0x100000000ull + pkt - 1) / pkt);  // exact quotient below 2^17 bytes
    auto covered = [&](uint32_t g) {
      const uint32_t q = __umulhi(16u * g, inv);
      const uint32_t s0 = (q * pkt) & ~15u, s1 = q ? (((q - 1) * pkt) & ~15u) : 0xffffffffu;
      return 16u * g - s0 < 96u || (q && 16u * g - s1 < 96u);
    };
    uint32_t k = lane;
    for (; k + 7 * 64 < nv; k += 8 * 64) {
      u32x4 a[8];
      if (mode == 3) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
          const uint32_t g = k + 64 * j;
          a[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, covered(g) ? 0x7ffffff0u : 16u * g, 0, 2);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; j++) a[j] = __builtin_nontemporal_load(v + k + 64 * j);
      }
#pragma unroll
      for (int j = 0; j < 8; j++) acc = __builtin_amdgcn_udot4(a[j].x ^ a[j].y ^ a[j].z ^ a[j].w, 0x01010101u, acc, false);
    }
    for (; k < nv; k += 64) {
      const u32x4 a = __builtin_nontemporal_load(v + k);
      acc = __builtin_amdgcn_udot4(a.x ^ a.y ^ a.z ^ a.w, 0x01010101u, acc, false);
    }
  }
  if (acc == 0x9e3779b9u) out[0] = acc;  // keep the loads live; practically never stores
}

// Skeleton probe (DESIGN.md §5, C3's gap to its stream shape): the decode
// kernel's memory accesses per wave without its work, one wave per 64
// packets of pkt bytes. flags: 1 = first each lane's 12-byte index entry
// (offset + caplen, from idx[], the window addresses depend on it); 2 = its
// 6-chunk header window at the packet (temporal) into LDS; 4 = after the
// stream, the 16-byte record and three 8-byte flow hashes per lane
// (non-temporal, into wbuf); 8 = those stores with the default policy;
// 16 = the block's waves store together after a barrier. The stream itself:
// mode 0 of probe_reread.
__global__ __launch_bounds__(256) void probe_skeleton_kernel(const uint8_t* data, uint64_t nbytes, uint32_t pkt,
                                                             const uint32_t* idx, uint8_t* wbuf, int flags,
                                                             uint32_t* out) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  __shared__ u32x4 win[256 * 6];
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint64_t R = 64ull * pkt, base = wave * R;
  if (base + R > nbytes) return;
  const uint64_t pk = wave * 64 + lane;
  uint32_t acc = 0;
  uint64_t dep = 0;
  if (flags & 1) {  // the index entry: 8-byte offset + 4-byte caplen, as two coalesced loads
    const u32x2 o = *reinterpret_cast<const u32x2*>(idx + 2 * pk);
    const uint32_t c = idx[2 * (nbytes / pkt) + pk];
    dep = (uint64_t)((o.x ^ o.y ^ c) & 0u);  // zero, but the window addresses wait for it
    acc += o.x + c;
  }
  if (flags & 2) {
    const uint8_t* h = data + ((base + (uint64_t)lane * pkt + dep) & ~15ull);
    u32x4 w[6];
#pragma unroll
    for (int k = 0; k < 6; k++) w[k] = *reinterpret_cast<const u32x4*>(h + 16 * k);
#pragma unroll
    for (int k = 0; k < 6; k++) win[threadIdx.x * 6 + k] = w[k];
    __syncthreads();
    // (the interleaved-store form reuses the wave's own slots: no lane reads another wave's window)
    const u32x4 x = win[(flags & 512 ? threadIdx.x : (threadIdx.x + 1) & 255) * 6 + (lane & 3)];
    acc = __builtin_amdgcn_udot4(x.x ^ x.y ^ x.z ^ x.w, 0x01010101u, acc, false);
  }
  const u32x4* v = reinterpret_cast<const u32x4*>(data + base + dep);
  const uint32_t nv = (uint32_t)(R / 16);
  uint32_t k = lane;
  for (; k + 7 * 64 < nv; k += 8 * 64) {
    u32x4 a[8];
#pragma unroll
    for (int j = 0; j < 8; j++) a[j] = __builtin_nontemporal_load(v + k + 64 * j);
#pragma unroll
    for (int j = 0; j < 8; j++) acc = __builtin_amdgcn_udot4(a[j].x ^ a[j].y ^ a[j].z ^ a[j].w, 0x01010101u, acc, false);
  }
  for (; k < nv; k += 64) {
    const u32x4 a = __builtin_nontemporal_load(v + k);
    acc = __builtin_amdgcn_udot4(a.x ^ a.y ^ a.z ^ a.w, 0x01010101u, acc, false);
  }
  if (flags & 4) {
    const uint64_t n = nbytes / pkt;
    if (flags & 16) __syncthreads();  // the block's four waves store together (4 KiB of records at once)
    u32x4* r = reinterpret_cast<u32x4*>(wbuf) + pk;
    uint64_t* f = reinterpret_cast<uint64_t*>(wbuf + 16 * n);
    if (flags & 8) {  // default (temporal) policy: the stores go through L2
      *r = u32x4{acc, lane, 0u, 1u};
#pragma unroll
      for (int j = 0; j < 3; j++) f[j * n + pk] = (uint64_t)acc * (j + 1);
    } else {
      __builtin_nontemporal_store(u32x4{acc, lane, 0u, 1u}, r);
#pragma unroll
      for (int j = 0; j < 3; j++) __builtin_nontemporal_store((uint64_t)acc * (j + 1), f + j * n + pk);
    }
  } else if (acc == 0x9e3779b9u) {
    out[0] = acc;
  }
}

// The skeleton of any packed batch (offsets / caplens as the decode takes
// them): per wave of 64 packets, the index entries; the header windows
// (flags & 2: 6 chunks at each packet's 16-byte-aligned start, temporal);
// unless flags & 64, the stream over the wave's extent (first packet's chunk to last packet's
// end, 1 KiB passes, 8 in flight, non-temporal); then wbytes bytes per packet
// written (16: record; 40: record + flows; 168: + layer fields), non-temporal
// (flags & 8: default policy; flags & 16: the block's waves store together;
// flags & 32: before the stream instead of after it).
__global__ __launch_bounds__(256) void probe_skeleton_idx_kernel(const uint8_t* data, const uint64_t* offsets,
                                                                 const uint32_t* caplens, uint64_t n, uint8_t* wbuf,
                                                                 uint32_t wbytes, int flags, uint32_t* out) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  __shared__ u32x4 win[256 * 6];
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t w0 = ((uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64;
  if (w0 >= n) return;
  const uint64_t i = w0 + lane < n ? w0 + lane : n - 1;
  const uint64_t o = offsets[i];
  const uint32_t c = caplens[i];
  uint32_t acc = c;
  if (flags & 2) {
    const uint8_t* h = data + (o & ~15ull);
    u32x4 w[6];
#pragma unroll
    for (int k = 0; k < 6; k++) w[k] = *reinterpret_cast<const u32x4*>(h + 16 * k);
#pragma unroll
    for (int k = 0; k < 6; k++) win[threadIdx.x * 6 + k] = w[k];
    __syncthreads();
    // (the interleaved-store form reuses the wave's own slots: no lane reads another wave's window)
    const u32x4 x = win[(flags & 512 ? threadIdx.x : (threadIdx.x + 1) & 255) * 6 + (lane & 3)];
    acc = __builtin_amdgcn_udot4(x.x ^ x.y ^ x.z ^ x.w, 0x01010101u, acc, false);
  }
  auto store_out = [&]() {
    if (flags & 16) __syncthreads();  // the block's four waves store together
    if (w0 + lane < n) {
      // flags & 128: the outputs of packet i at i mod 2^20 (a 40 MiB ring that stays on chip) instead of i;
      // flags & 1024: at i mod 2^14 (640 KiB: a ring that stays in each XCD's L2)
      const uint64_t q = (flags & 1024)  ? ((w0 + lane) & ((1u << 14) - 1))
                         : (flags & 128) ? ((w0 + lane) & ((1u << 20) - 1))
                                         : w0 + lane;
      // wbytes 8 / 32: the 8-byte narrow record (gpk_record8), alone or with the flows
      const bool narrow = wbytes == 8 || wbytes == 32, flows = wbytes == 32 || wbytes >= 40;
      const uint32_t rb = narrow ? 8u : 16u;
      uint8_t* r = wbuf + q * rb;
      uint64_t* f = reinterpret_cast<uint64_t*>(wbuf + rb * n) + (q - (w0 + lane));
      if (flags & 8) {  // default (temporal) store policy
        if (narrow) *reinterpret_cast<uint64_t*>(r) = (uint64_t)lane << 32 | acc;
        else if (wbytes >= 16) *reinterpret_cast<u32x4*>(r) = u32x4{acc, lane, 0u, 1u};
        if (flows)
#pragma unroll
          for (int j = 0; j < 3; j++) f[j * n + w0 + lane] = (uint64_t)acc * (j + 1);
      } else {
        if (narrow) __builtin_nontemporal_store((uint64_t)lane << 32 | acc, reinterpret_cast<uint64_t*>(r));
        else if (wbytes >= 16) __builtin_nontemporal_store(u32x4{acc, lane, 0u, 1u}, reinterpret_cast<u32x4*>(r));
        if (flows)
#pragma unroll
          for (int j = 0; j < 3; j++) __builtin_nontemporal_store((uint64_t)acc * (j + 1), f + j * n + w0 + lane);
      }
      if (wbytes >= 168) {  // the wave's 64 128-byte records as eight coalesced 1 KiB runs (as the fused kernel stores)
        u32x4* fl = reinterpret_cast<u32x4*>(wbuf + 40 * n) + w0 * 8;
#pragma unroll
        for (int j = 0; j < 8; j++) __builtin_nontemporal_store(u32x4{acc, (uint32_t)j, lane, 0u}, fl + 64 * j + lane);
      }
    }
  };
  // flags & 512: the packet's 40 bytes (record + three flows) interleaved at wbuf + 40 i: each wave's outputs
  // as ONE contiguous 2560-byte run, staged through its own window slots (read above by its own lanes only)
  auto store_aos = [&]() {
    uint32_t* l = reinterpret_cast<uint32_t*>(win) + (threadIdx.x & ~63u) * 24;
    asm volatile("" ::: "memory");
    const uint64_t a = acc;
    *reinterpret_cast<uint64_t*>(l + 10 * lane) = (uint64_t)lane << 32 | acc;
    *reinterpret_cast<uint64_t*>(l + 10 * lane + 2) = 1ull << 32;
#pragma unroll
    for (int j = 0; j < 3; j++) *reinterpret_cast<uint64_t*>(l + 10 * lane + 4 + 2 * j) = a * (j + 1);
    asm volatile("" ::: "memory");
    const uint64_t lim = (n - w0 < 64 ? n - w0 : 64) * 40;  // bytes of this wave's run
    u32x4* r = reinterpret_cast<u32x4*>(wbuf + w0 * 40);
#pragma unroll
    for (uint32_t k = 0; k < 3; k++) {
      const uint32_t c = 64 * k + lane;
      // whole chunks inside the run; an odd packet count leaves an 8-byte tail
      if (c < 160 && 16ull * c + 16 <= lim) {
        __builtin_nontemporal_store(reinterpret_cast<const u32x4*>(l)[c], r + c);
      } else if (c < 160 && 16ull * c + 8 == lim) {
        __builtin_nontemporal_store(reinterpret_cast<const uint64_t*>(l)[2 * c], reinterpret_cast<uint64_t*>(r + c));
      }
    }
  };
  if (flags & 32) store_out();  // the outputs before the stream (their values are whatever acc holds then)
  // flags & 256: the block's outputs through LDS, stored by its first wave alone
  auto store_by_wave0 = [&]() {  // (records only when wbytes < 40; no fields)
    __syncthreads();  // every wave is past its window reads
    uint32_t* l = reinterpret_cast<uint32_t*>(win);
    const uint32_t t = threadIdx.x;
    l[4 * t + 0] = acc;
    l[4 * t + 1] = lane;
    l[4 * t + 2] = 0u;
    l[4 * t + 3] = 1u;
    uint64_t* lf = reinterpret_cast<uint64_t*>(l + 1024);
#pragma unroll
    for (int j = 0; j < 3; j++) lf[256 * j + t] = (uint64_t)acc * (j + 1);
    __syncthreads();
    if (threadIdx.x < 64) {
      const uint64_t b0 = (uint64_t)blockIdx.x * 256;
      u32x4* r = reinterpret_cast<u32x4*>(wbuf) + b0;
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (b0 + 64 * k + lane < n)
          __builtin_nontemporal_store(reinterpret_cast<const u32x4*>(l)[64 * k + lane], r + 64 * k + lane);
      if (wbytes >= 40) {  // the flows only where the buffer has them
        uint64_t* f = reinterpret_cast<uint64_t*>(wbuf + 16 * n) + b0;
#pragma unroll
        for (int j = 0; j < 3; j++)
#pragma unroll
          for (int k = 0; k < 4; k++)
            if (b0 + 64 * k + lane < n)
              __builtin_nontemporal_store(lf[256 * j + 64 * k + lane], f + j * n + 64 * k + lane);
      }
    }
  };
  const uint64_t lo = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)o) |
                      (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(o >> 32)) << 32;
  const uint64_t e = o + c;
  const uint64_t hi = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)e, 63) |
                      (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(e >> 32), 63) << 32;
  const uint64_t b = lo & ~15ull;
  const uint32_t nv = (flags & 64) || hi <= b ? 0u : (uint32_t)((hi - b + 15) / 16);  // 64: windows only
  const u32x4* v = reinterpret_cast<const u32x4*>(data + b);
  uint32_t k = lane;
  for (; k + 7 * 64 < nv; k += 8 * 64) {
    u32x4 a[8];
#pragma unroll
    for (int j = 0; j < 8; j++) a[j] = __builtin_nontemporal_load(v + k + 64 * j);
#pragma unroll
    for (int j = 0; j < 8; j++) acc = __builtin_amdgcn_udot4(a[j].x ^ a[j].y ^ a[j].z ^ a[j].w, 0x01010101u, acc, false);
  }
  for (; k < nv; k += 64) {
    const u32x4 a = __builtin_nontemporal_load(v + k);
    acc = __builtin_amdgcn_udot4(a.x ^ a.y ^ a.z ^ a.w, 0x01010101u, acc, false);
  }
  if (flags & 256) store_by_wave0();
  else if (flags & 512) store_aos();
  else if (!(flags & 32)) store_out();
  if (acc == 0x9e3779b9u) out[0] = acc;
}

// The skeleton with a fifth, storing wave per block: waves 0-3 do the
// skeleton's reads for the block's 256 packets (index, windows, stream) and
// put their records and flows into LDS; after a barrier wave 4, which reads
// nothing, stores the block's outputs (4 KiB of records, 3 x 2 KiB of flows,
// non-temporal). Whether stores cost less from a wave that does not stream.
__global__ __launch_bounds__(320) void probe_skeleton_storer_kernel(const uint8_t* data, const uint64_t* offsets,
                                                                   const uint32_t* caplens, uint64_t n, uint8_t* wbuf,
                                                                   uint32_t wbytes, uint32_t* out) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  __shared__ u32x4 win[256 * 6];
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t b0 = (uint64_t)blockIdx.x * 256;
  uint32_t acc = 0;
  if (wv < 4) {
    const uint64_t w0 = b0 + 64 * wv;
    const uint64_t i = w0 + lane < n ? w0 + lane : n - 1;
    const uint64_t o = offsets[i];
    const uint32_t c = caplens[i];
    acc = c;
    const uint8_t* h = data + (o & ~15ull);
    u32x4 w[6];
#pragma unroll
    for (int k = 0; k < 6; k++) w[k] = *reinterpret_cast<const u32x4*>(h + 16 * k);
#pragma unroll
    for (int k = 0; k < 6; k++) win[threadIdx.x * 6 + k] = w[k];
    const u32x4 x = win[threadIdx.x * 6 + (lane & 3)];
    acc = __builtin_amdgcn_udot4(x.x ^ x.y ^ x.z ^ x.w, 0x01010101u, acc, false);
    const uint64_t lo = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)o) |
                        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(o >> 32)) << 32;
    const uint64_t e = o + c;
    const uint64_t hi = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)e, 63) |
                        (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(e >> 32), 63) << 32;
    const uint64_t b = lo & ~15ull;
    const uint32_t nv = hi <= b ? 0u : (uint32_t)((hi - b + 15) / 16);
    const u32x4* v = reinterpret_cast<const u32x4*>(data + b);
    uint32_t k = lane;
    for (; k + 7 * 64 < nv; k += 8 * 64) {
      u32x4 a[8];
#pragma unroll
      for (int j = 0; j < 8; j++) a[j] = __builtin_nontemporal_load(v + k + 64 * j);
#pragma unroll
      for (int j = 0; j < 8; j++) acc = __builtin_amdgcn_udot4(a[j].x ^ a[j].y ^ a[j].z ^ a[j].w, 0x01010101u, acc, false);
    }
    for (; k < nv; k += 64) {
      const u32x4 a = __builtin_nontemporal_load(v + k);
      acc = __builtin_amdgcn_udot4(a.x ^ a.y ^ a.z ^ a.w, 0x01010101u, acc, false);
    }
  }
  __syncthreads();  // every wave is past its window reads
  uint32_t* l = reinterpret_cast<uint32_t*>(win);
  uint64_t* lf = reinterpret_cast<uint64_t*>(l + 1024);
  if (wv < 4) {
    const uint32_t t = threadIdx.x;
    l[4 * t + 0] = acc;
    l[4 * t + 1] = lane;
    l[4 * t + 2] = 0u;
    l[4 * t + 3] = 1u;
#pragma unroll
    for (int j = 0; j < 3; j++) lf[256 * j + t] = (uint64_t)acc * (j + 1);
  }
  __syncthreads();
  if (wv == 4) {
    u32x4* r = reinterpret_cast<u32x4*>(wbuf) + b0;
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (b0 + 64 * k + lane < n)
        __builtin_nontemporal_store(reinterpret_cast<const u32x4*>(l)[64 * k + lane], r + 64 * k + lane);
    if (wbytes >= 40) {
      uint64_t* f = reinterpret_cast<uint64_t*>(wbuf + 16 * n) + b0;
#pragma unroll
      for (int j = 0; j < 3; j++)
#pragma unroll
        for (int k = 0; k < 4; k++)
          if (b0 + 64 * k + lane < n)
            __builtin_nontemporal_store(lf[256 * j + 64 * k + lane], f + j * n + 64 * k + lane);
    }
  }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

extern "C" {

// wbuf_bytes: the size of wbuf. Every form stores at most wbytes bytes per
// packet inside [wbuf, wbuf + wbytes * n) (the ring form inside the first
// 2^20 packets' share); a call whose buffer is smaller, or whose wbytes is not
// one of the forms (0, 16, 40, 168), is rejected before launch (-1). Round 4's
// fault: the wave-0 form stored flows into a 16-byte-per-packet buffer.
static bool skeleton_args_ok(uint64_t n, uint32_t wbytes, int flags, uint64_t wbuf_bytes, bool storer) {
  if (wbytes != 0 && wbytes != 8 && wbytes != 16 && wbytes != 32 && wbytes != 40 && wbytes != 168) return false;
  if ((flags & 256) && wbytes != 16 && wbytes != 40) return false;  // the wave-0 form stores 16-byte records
  if (storer && wbytes != 16 && wbytes != 40) return false;
  if ((flags & 512) && wbytes != 40) return false;
  return wbuf_bytes >= (uint64_t)wbytes * n;
}

int gpk_probe_skeleton_storer(const uint8_t* data, const uint64_t* offsets, const uint32_t* caplens, uint64_t n,
                              uint8_t* wbuf, uint64_t wbuf_bytes, uint32_t wbytes, uint32_t* out, void* stream) {
  const uint64_t blocks = (n + 255) / 256;
  if (!n || blocks > 0xffffffffull || !skeleton_args_ok(n, wbytes, 0, wbuf_bytes, true)) return -1;
  hipLaunchKernelGGL(probe_skeleton_storer_kernel, dim3((unsigned)blocks), dim3(320), 0, (hipStream_t)stream, data,
                     offsets, caplens, n, wbuf, wbytes, out);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

int gpk_probe_skeleton_idx(const uint8_t* data, const uint64_t* offsets, const uint32_t* caplens, uint64_t n,
                           uint8_t* wbuf, uint64_t wbuf_bytes, uint32_t wbytes, int flags, uint32_t* out, void* stream) {
  const uint64_t blocks = (n + 255) / 256;
  if (!n || blocks > 0xffffffffull || !skeleton_args_ok(n, wbytes, flags, wbuf_bytes, false)) return -1;
  hipLaunchKernelGGL(probe_skeleton_idx_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, data,
                     offsets, caplens, n, wbuf, wbytes, flags, out);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// Launch the skeleton probe: idx holds 3 dwords per packet (nbytes / pkt
// packets: offsets as 2 dwords, then caplens), wbuf 40 bytes per packet.
int gpk_probe_skeleton(const uint8_t* data, uint64_t nbytes, uint32_t pkt, const uint32_t* idx, uint8_t* wbuf, int flags,
                       uint32_t* out, void* stream) {
  const uint64_t waves = nbytes / (64ull * pkt), blocks = (waves + 3) / 4;
  if (!pkt || !blocks) return -1;
  hipLaunchKernelGGL(probe_skeleton_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, data, nbytes,
                     pkt, idx, wbuf, flags, out);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

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
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, in, offsets, (int)n, s) != hipSuccess) return -2;
    void* tmp = nullptr;
    if (hipMallocAsync(&tmp, tmp_bytes, s) != hipSuccess) return -2;
    if (hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, in, offsets, (int)n, s) != hipSuccess) return -2;
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

// C5 capture file: SHB + one IDB (LinkType 1 = Ethernet, snaplen 65535,
// microsecond timestamps) + one EPB per packet [first, first+n) of config cfg
// (little endian; ts = 1.6e9 s + i microseconds). T threads generate disjoint
// ranges and pwrite them at offsets from a prefix sum of the record sizes.
// Returns the file size, or 0 on error.
uint64_t gpk_synth_write_pcapng(const char* path, int cfg, uint64_t first, uint64_t n, int T) {
  if (T < 1) T = 1;
  int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) return 0;
  uint8_t head[28 + 20];
  auto p32 = [](uint8_t* b, uint32_t v) { memcpy(b, &v, 4); };
  auto p16 = [](uint8_t* b, uint16_t v) { memcpy(b, &v, 2); };
  p32(head, 0x0A0D0D0A); p32(head + 4, 28); p32(head + 8, 0x1A2B3C4D); p16(head + 12, 1); p16(head + 14, 0);
  uint64_t minus1 = ~0ull;
  memcpy(head + 16, &minus1, 8);
  p32(head + 24, 28);
  p32(head + 28, 1); p32(head + 32, 20); p16(head + 36, 1); p16(head + 38, 0); p32(head + 40, 65535); p32(head + 44, 20);
  bool ok = pwrite(fd, head, sizeof(head), 0) == (ssize_t)sizeof(head);
  auto rec = [&](uint64_t i) { return 32ull + ((frame_len(cfg, i) + 3u) & ~3u); };
  std::vector<uint64_t> start(T + 1, 0);
  const uint64_t per = (n + T - 1) / T;
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++)  // bytes of each range
    th.emplace_back([&, t] {
      uint64_t a = first + std::min<uint64_t>(n, t * per), e = first + std::min<uint64_t>(n, (t + 1) * per), s = 0;
      for (uint64_t i = a; i < e; i++) s += rec(i);
      start[t + 1] = s;
    });
  for (auto& x : th) x.join();
  th.clear();
  start[0] = sizeof(head);
  for (int t = 0; t < T; t++) start[t + 1] += start[t];
  std::vector<int> good(T, 1);
  for (int t = 0; t < T; t++)
    th.emplace_back([&, t] {
      uint64_t a = first + std::min<uint64_t>(n, t * per), e = first + std::min<uint64_t>(n, (t + 1) * per);
      std::vector<uint8_t> buf(8u << 20);
      uint64_t fill = 0, at = start[t];
      for (uint64_t i = a; i <= e; i++) {
        const uint64_t r = i < e ? rec(i) : 0;
        if (i == e || fill + r > buf.size()) {
          if (fill && pwrite(fd, buf.data(), fill, (off_t)at) != (ssize_t)fill) good[t] = 0;
          at += fill;
          fill = 0;
          if (i == e) break;
        }
        uint8_t* b = buf.data() + fill;
        const uint32_t cl = frame_len(cfg, i);
        const uint64_t ts = 1600000000000000ull + i;
        memset(b + 28 + (cl & ~3u), 0, 4);
        p32(b, 6); p32(b + 4, (uint32_t)r); p32(b + 8, 0); p32(b + 12, (uint32_t)(ts >> 32)); p32(b + 16, (uint32_t)ts);
        p32(b + 20, cl); p32(b + 24, cl);
        gpk_synth_fill(cfg, i, b + 28);
        p32(b + r - 4, (uint32_t)r);
        fill += r;
      }
    });
  for (auto& x : th) x.join();
  for (int t = 0; t < T; t++) ok = ok && good[t];
  close(fd);
  return ok ? start[T] : 0;
}

// ---- AF_PACKET TPACKET_V3 rings (bench / test infrastructure) -------------
// Blocks laid out the way the Linux kernel fills them for a SOCK_RAW socket on
// an Ethernet device (measured on lo, tests/golden/afpacket/lo_v3.ring):
// tpacket_block_desc {version 2, offset_to_priv 48, hdr_v1 {block_status,
// num_pkts, offset_to_first_pkt 48, blk_len, seq_num, ts}}; packets chained
// from offset 48 with tp_mac 82, tp_net 96, tp_next_offset =
// TPACKET_ALIGN(82 + snaplen) (0 on the block's last packet), a sockaddr_ll at
// +48. Packet k of the ring is synth packet first+k of config cfg. Every
// vlan_every-th packet (0 = none) carries TP_STATUS_VLAN_VALID and a TCI.
// Returns the packet count; counts[b] (optional) = packets of block b.
static inline uint32_t tp_al(uint32_t x) { return (x + 15u) & ~15u; }

uint64_t gpk_synth_tpacket_v3(uint8_t* ring, uint32_t block_size, uint32_t nblocks, int cfg, uint64_t first,
                              int32_t ifindex, uint32_t vlan_every, uint64_t* counts) {
  std::vector<uint64_t> start(nblocks + 1, first);
  for (uint32_t b = 0; b < nblocks; b++) {  // packets per block from the lengths alone
    uint64_t i = start[b];
    uint32_t pos = 48;
    while (pos + tp_al(82 + frame_len(cfg, i)) <= block_size) pos += tp_al(82 + frame_len(cfg, i++));
    start[b + 1] = i;
  }
  const int T = (int)std::min<uint32_t>(16, std::max<uint32_t>(1, nblocks));
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++)
    th.emplace_back([&, t] {
      for (uint32_t b = (uint32_t)t; b < nblocks; b += (uint32_t)T) {
        uint8_t* B = ring + (uint64_t)b * block_size;
        memset(B, 0, 48);
        const uint64_t n = start[b + 1] - start[b];
        uint32_t pos = 48, last = 48;
        for (uint64_t k = 0; k < n; k++) {
          const uint64_t i = start[b] + k;
          uint8_t* P = B + pos;
          memset(P, 0, 82);
          const uint32_t snap = gpk_synth_fill(cfg, i, P + 82);
          const uint32_t step = tp_al(82 + snap);
          const bool vl = vlan_every && (i % vlan_every) == 0;
          const uint32_t sec = 1600000000u + (uint32_t)(i / 1000000u), nsec = (uint32_t)(i % 1000000u) * 1000u;
          const uint32_t status = 1u | (vl ? 0x10u : 0u), tci = vl ? (uint32_t)((i * 37u) & 0xfffu) | 0x2000u : 0u;
          const uint32_t nxt = k + 1 < n ? step : 0u;
          memcpy(P + 0, &nxt, 4);
          memcpy(P + 4, &sec, 4);
          memcpy(P + 8, &nsec, 4);
          memcpy(P + 12, &snap, 4);
          memcpy(P + 16, &snap, 4);
          memcpy(P + 20, &status, 4);
          const uint16_t mac = 82, net = 96;
          memcpy(P + 24, &mac, 2);
          memcpy(P + 26, &net, 2);
          memcpy(P + 32, &tci, 4);
          const uint16_t tpid = vl ? 0x8100 : 0;
          memcpy(P + 36, &tpid, 2);
          const uint16_t fam = 17, proto = 0x0008, hatype = 1;  // AF_PACKET, htons(ETH_P_IP), ARPHRD_ETHER
          memcpy(P + 48, &fam, 2);
          memcpy(P + 50, &proto, 2);
          memcpy(P + 52, &ifindex, 4);
          memcpy(P + 56, &hatype, 2);
          P[58] = 0;  // PACKET_HOST
          P[59] = 6;
          memcpy(P + 60, P + 82 + 6, 6);  // source MAC
          last = pos + 82 + snap;
          pos += step;
        }
        const uint32_t hdr[6] = {2u, 48u, 0u, (uint32_t)n, 48u, (last + 7u) & ~7u};
        memcpy(B, hdr, sizeof(hdr));
        const uint64_t seq = b + 1;
        memcpy(B + 24, &seq, 8);
        __atomic_store_n(reinterpret_cast<uint32_t*>(B + 8), 1u, __ATOMIC_RELEASE);  // TP_STATUS_USER: hand it over
        if (counts) counts[b] = n;
      }
    });
  for (auto& x : th) x.join();
  return start[nblocks] - first;
}

// Emulated kernel side of a ring for the capture benchmark: a thread that
// hands every released block (block_status == 0) straight back to user space
// (TP_STATUS_USER), in ring order, with its contents unchanged.
struct TpProducer {
  std::atomic<bool> stop{false};
  std::atomic<uint64_t> rearmed{0};
  std::thread th;
};

void* gpk_synth_tp_producer_start(uint8_t* ring, uint32_t block_size, uint32_t nblocks) {
  TpProducer* p = new TpProducer();
  p->th = std::thread([p, ring, block_size, nblocks] {
    uint32_t b = 0;
    while (!p->stop.load(std::memory_order_relaxed)) {
      uint32_t* st = reinterpret_cast<uint32_t*>(ring + (uint64_t)b * block_size + 8);
      if (__atomic_load_n(st, __ATOMIC_ACQUIRE) == 0) {
        __atomic_store_n(st, 1u, __ATOMIC_RELEASE);
        p->rearmed.fetch_add(1, std::memory_order_relaxed);
        b = (b + 1) % nblocks;
      } else {
        std::this_thread::yield();
      }
    }
  });
  return p;
}

uint64_t gpk_synth_tp_producer_stop(void* h) {
  TpProducer* p = static_cast<TpProducer*>(h);
  p->stop = true;
  p->th.join();
  uint64_t n = p->rearmed.load();
  delete p;
  return n;
}

// Launch the re-read probe over the whole regions of data[0, nbytes) on `stream`.
int gpk_probe_reread(const uint8_t* data, uint64_t nbytes, uint32_t pkt, int mode, uint32_t* out, void* stream) {
  const uint64_t waves = nbytes / (64ull * pkt), blocks = (waves + 3) / 4;
  if (!pkt || !blocks) return -1;
  hipLaunchKernelGGL(probe_reread_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, data, nbytes, pkt,
                     mode, out);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// The same with `lds` bytes of (unused) dynamic LDS per block: caps the
// blocks a CU holds at once (160 KiB / lds), the occupancy sweep of
// tools/stream_shape_probe.py --occ.
int gpk_probe_reread_lds(const uint8_t* data, uint64_t nbytes, uint32_t pkt, int mode, uint32_t lds, uint32_t* out,
                         void* stream) {
  const uint64_t waves = nbytes / (64ull * pkt), blocks = (waves + 3) / 4;
  if (!pkt || !blocks || lds > 160u * 1024u) return -1;
  hipLaunchKernelGGL(probe_reread_kernel, dim3((unsigned)blocks), dim3(256), lds, (hipStream_t)stream, data, nbytes,
                     pkt, mode, out);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// Launch the streaming-read probe over data[0, nbytes & ~15) on `stream`.
int gpk_probe_read(const uint8_t* data, uint64_t nbytes, uint32_t* out, int blocks, void* stream) {
  hipLaunchKernelGGL(probe_read_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, data, nbytes / 16, out);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// Launch the mixed read + write probe (blocks in all; writers of them store).
int gpk_probe_mixed(const uint8_t* data, uint64_t nbytes, uint8_t* wbuf, uint64_t wbytes, int blocks, int writers,
                    uint32_t* out, void* stream) {
  if (writers < 0 || writers >= blocks) return -1;
  hipLaunchKernelGGL(probe_mixed_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, data, nbytes / 16, wbuf,
                     wbytes / 16, (uint32_t)writers, out);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

int gpk_probe_hostwrite(uint8_t* dst, uint64_t nbytes, int blocks, void* stream) {
  hipLaunchKernelGGL(probe_hostwrite_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, dst, nbytes / 16);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// Host-to-device copy rate of `bytes` from host memory `src` (registered here
// with hipHostRegister unless it is already pinned: register = 0) in copies of
// `chunk` bytes over `streams` streams, `reps` rounds; returns GB/s or < 0
// (tools/duplex_probe.py: ring memory as the AF_PACKET pump copies it).
double gpk_probe_h2d_rate(const void* src, uint64_t bytes, uint64_t chunk, int streams, int reps, int register_) {
  if (!src || !bytes || !chunk || streams < 1 || streams > 16 || reps < 1) return -1;
  if (register_ && hipHostRegister(const_cast<void*>(src), bytes, hipHostRegisterDefault) != hipSuccess) return -2;
  void* dst = nullptr;
  double gbs = -3;
  hipStream_t st[16] = {};
  hipEvent_t e0 = nullptr, e1 = nullptr;
  bool ok = hipMalloc(&dst, bytes) == hipSuccess && hipEventCreate(&e0) == hipSuccess &&
            hipEventCreate(&e1) == hipSuccess;
  for (int k = 0; ok && k < streams; k++) ok = hipStreamCreateWithFlags(&st[k], hipStreamNonBlocking) == hipSuccess;
  if (ok) {
    auto round = [&]() {
      uint64_t i = 0;
      for (uint64_t o = 0; o < bytes; o += chunk, i++)
        (void)hipMemcpyAsync((char*)dst + o, (const char*)src + o, o + chunk <= bytes ? chunk : bytes - o,
                             hipMemcpyHostToDevice, st[i % streams]);
      for (int k = 0; k < streams; k++) (void)hipStreamSynchronize(st[k]);
    };
    round();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0, nullptr);
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; r++) round();
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    gbs = (double)bytes * reps / s / 1e9;
  }
  for (int k = 0; k < streams; k++)
    if (st[k]) (void)hipStreamDestroy(st[k]);
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (dst) (void)hipFree(dst);
  if (register_) (void)hipHostUnregister(const_cast<void*>(src));
  return gbs;
}

// Device memory of a given kind for placement experiments (tools/alloc_probe.py):
// hipExtMallocWithFlags flags (hipDeviceMallocDefault 0, Finegrained 1,
// Uncached 3, Contiguous 4).
int gpk_probe_malloc(void** p, uint64_t bytes, unsigned flags) {
  return hipExtMallocWithFlags(p, bytes, flags) == hipSuccess ? 0 : -1;
}
int gpk_probe_free(void* p) { return hipFree(p) == hipSuccess ? 0 : -1; }
int gpk_probe_d2d(void* dst, const void* src, uint64_t bytes) {
  return hipMemcpy(dst, src, bytes, hipMemcpyDeviceToDevice) == hipSuccess ? 0 : -1;
}

}  // extern "C"

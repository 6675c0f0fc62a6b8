// gpk_walk.hip — the pcapng record walk of a staging slot, on the device
// (gpk_walk.h has the scheme). One thread per segment: the walk is a chain of
// dependent 32-byte header reads, so the parallelism is across segments, and
// a slot of 256 MiB in 4 KiB segments is 64 Ki independent chains.
#include "gpk_walk.h"

namespace gpk {
namespace {

constexpr uint32_t kEPB = 6;
constexpr uint64_t kNone = ~0ull;

// Blocks sit at p = p0 (mod 4) from the 16-byte-aligned base (the slot's
// carry starts anywhere): byte loads.
__device__ __forceinline__ uint32_t ld32(const uint8_t* b, uint64_t p, uint32_t be) {
  uint32_t v;
  __builtin_memcpy(&v, b + p, 4);
  return be ? __builtin_bswap32(v) : v;
}

// What ReadPacketData does on a plain EPB at b[p] (ngread.go:494-514,
// 642-675; host twin: gpk_capture.cpp plain_epb): block type 6, total length
// == 32 + caplen + padding (no options), the block inside b[p, len), a known
// interface of an allowed link type. Returns the block length, 0 otherwise.
__device__ __forceinline__ uint32_t plain_epb(const WalkState& ws, const uint8_t* b, uint64_t p, uint64_t len,
                                              uint32_t* idx_out, uint32_t* cl_out) {
  if (p > len || len - p < 32) return 0;
  if (ld32(b, p, ws.be) != kEPB) return 0;
  const uint32_t L = ld32(b, p + 4, ws.be), idx = ld32(b, p + 8, ws.be), cl = ld32(b, p + 20, ws.be);
  if (idx >= ws.nif || !ws.ifc[idx].plain) return 0;
  if ((uint64_t)L != 32ull + cl + ((4u - (cl & 3u)) & 3u) || L > len - p) return 0;
  *idx_out = idx;
  *cl_out = cl;
  return L;
}

// First p in [from, to), p = ref (mod 4), where four plain EPBs with matching
// trailers follow each other (host twin: find_sync).
__device__ uint64_t find_sync(const WalkState& ws, const uint8_t* b, uint64_t from, uint64_t to, uint64_t len,
                              uint64_t ref) {
  for (uint64_t p = from + ((ref - from) & 3); p < to; p += 4) {
    uint64_t q = p;
    int k = 0;
    for (; k < 4; k++) {
      uint32_t idx, cl;
      const uint32_t L = plain_epb(ws, b, q, len, &idx, &cl);
      if (!L || ld32(b, q + L - 4, ws.be) != L) break;
      q += L;
    }
    if (k == 4) return p;
  }
  return kNone;
}

__global__ void walk_kernel(const uint8_t* b, uint64_t p0, uint64_t len, uint64_t seg, uint32_t nseg, WalkState ws,
                            WalkSegs out) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nseg) return;
  const uint64_t s0 = (uint64_t)k * seg, s1 = s0 + seg < len ? s0 + seg : len;
  // the segment holding p0 starts where the exact reader stands; the later
  // ones search (at most 1 MiB, as the host walk does), the earlier are empty
  const uint64_t k0 = p0 / seg;
  uint64_t p = k < k0 ? kNone : k == k0 ? p0 : find_sync(ws, b, s0, s1 < s0 + (1u << 20) ? s1 : s0 + (1u << 20), len, p0);
  out.sync[k] = p;
  uint32_t n = 0;
  if (p != kNone) {
    while (p < s1) {
      uint32_t idx, cl;
      const uint32_t L = plain_epb(ws, b, p, len, &idx, &cl);
      if (!L) break;
      n++;
      p += L;
    }
  }
  out.end[k] = p == kNone ? 0 : p;
  out.count[k] = n;
}

// convertTime (ngread.go:440-443) + time.Unix normalisation (host twin:
// gpk_capreader::iface_time, unix_norm)
__device__ void iface_time(const WalkIface& it, uint64_t ts, int64_t* s, uint32_t* ns) {
  const uint64_t m = it.second_mask;
  uint64_t q, r;
  if ((m & (m - 1)) == 0) {
    q = ts >> __builtin_ctzll(m);
    r = ts & (m - 1);
  } else {
    q = ts / m;
    r = ts - q * m;
  }
  uint64_t nsec = r * it.scale_up;
  if (it.scale_down != 1) nsec /= it.scale_down;
  int64_t sec = (int64_t)(q + it.tsoff), nn = (int64_t)nsec;
  if (nn < 0 || nn >= 1000000000LL) {
    const int64_t c = nn / 1000000000LL;
    sec = (int64_t)((uint64_t)sec + (uint64_t)c);
    nn -= c * 1000000000LL;
    if (nn < 0) {
      nn += 1000000000LL;
      sec = (int64_t)((uint64_t)sec - 1);
    }
  }
  *s = sec;
  *ns = (uint32_t)nn;
}

__global__ void emit_kernel(const uint8_t* b, uint64_t len, uint32_t nseg, WalkState ws, WalkSegs segs,
                            uint64_t* off, uint32_t* cap, gpk_capture_info* ci) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nseg) return;
  uint64_t j = segs.base[k];
  if (j == kNone) return;
  uint64_t p = segs.sync[k];
  const uint32_t n = segs.count[k];
  for (uint32_t i = 0; i < n; i++, j++) {
    uint32_t idx = 0, cl = 0;
    const uint32_t L = plain_epb(ws, b, p, len, &idx, &cl);
    if (!L) break;  // cannot happen: pass 1 walked the same blocks
    const WalkIface& it = ws.ifc[idx];
    gpk_capture_info c;
    iface_time(it, (uint64_t)ld32(b, p + 12, ws.be) << 32 | ld32(b, p + 16, ws.be), &c.ts_sec, &c.ts_nsec);
    c.length = ld32(b, p + 24, ws.be);
    c.iface = (int32_t)idx;
    c.link_type = ws.mixed ? it.link_type : -1;
    off[j] = p + 28;
    cap[j] = cl;
    ci[j] = c;
    p += L;
  }
}

}  // namespace
}  // namespace gpk

hipError_t gpk_walk_segments(const uint8_t* buf, uint64_t p0, uint64_t len, uint64_t seg, uint32_t nseg,
                             const gpk::WalkState& ws, const gpk::WalkSegs& out, hipStream_t stream) {
  if (!nseg) return hipSuccess;
  if (seg < 64 || (seg & 3) || (uint64_t)nseg * seg < len || p0 > len) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gpk::walk_kernel, dim3((nseg + 255) / 256), dim3(256), 0, stream, buf, p0, len, seg, nseg, ws,
                     out);
  return hipGetLastError();
}

hipError_t gpk_walk_emit(const uint8_t* buf, uint64_t len, uint32_t nseg, const gpk::WalkState& ws,
                         const gpk::WalkSegs& segs, uint64_t* offsets, uint32_t* caplens, gpk_capture_info* ci,
                         hipStream_t stream) {
  if (!nseg) return hipSuccess;
  hipLaunchKernelGGL(gpk::emit_kernel, dim3((nseg + 255) / 256), dim3(256), 0, stream, buf, len, nseg, ws, segs,
                     offsets, caplens, ci);
  return hipGetLastError();
}

// Load this module's code object on the device now and run its pass-1 kernel
// once over 128 zero bytes (no interface, so no block is plain and nothing is
// accepted): gpk_ctx_create calls it, so the first replay of a process does
// not pay the module's first use inside its own wall time.
extern "C" __attribute__((visibility("hidden"))) void gpk_walk_preload(void) {
  uint8_t* d = nullptr;
  if (hipMalloc(&d, 256) != hipSuccess) return;
  gpk::WalkState ws{};
  gpk::WalkSegs out{reinterpret_cast<uint64_t*>(d + 128), reinterpret_cast<uint64_t*>(d + 144),
                    reinterpret_cast<uint32_t*>(d + 160), reinterpret_cast<uint64_t*>(d + 176)};
  if (hipMemset(d, 0, 256) == hipSuccess && gpk_walk_segments(d, 0, 128, 128, 1, ws, out, nullptr) == hipSuccess)
    (void)hipDeviceSynchronize();
  (void)hipFree(d);
}

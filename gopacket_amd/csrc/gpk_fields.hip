// gpk_fields.hip — the scalar layer fields of every packet of a decoded batch
// (include/gpk.h gpk_fields, gpk_extract_fields), for consumers that read
// layer fields after DecodeLayers.
//
// A decoder's fields are a pure function of the slice its last successful
// DecodeFromBytes was handed, which the decode kernels report per packet as
// the layout ([start, end) per decoder slot). One lane per packet loads the
// 16-byte-aligned run of 6 chunks holding the packet's first bytes into its LDS
// slot, reads each present slice's header words from there (unaligned
// ds_read_b32; from memory past the run), and the wave writes its 64 records
// through LDS as eight coalesced 1 KiB stores.
// The field assignments are gpk_fields.h (shared with the decode kernel's
// fused-fields variant).
#include <hip/hip_runtime.h>

#include "../../include/gpk.h"
#include "gpk_fields.h"

namespace {

constexpr uint32_t kBlock = 256;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// n bytes at p in memory order (little-endian value), byte loads: exactly the
// field's bytes, never a byte past them (a field can end at the batch's last
// byte).
__device__ __forceinline__ uint32_t ldbytes(const uint8_t* p, int n) {
  uint32_t v = 0;
  for (int k = 0; k < n; k++) v |= (uint32_t)p[k] << (8 * k);
  return v;
}

// Header bytes of one packet: the 16-byte-aligned run of kWin chunks holding
// its first bytes sits in the lane's LDS slot (one round trip of wide loads
// instead of a dword pair per field); a field past the run (long IPv6
// extension chains) is read from memory.
constexpr uint32_t kWin = 6;               // chunks: 81..96 packet bytes
constexpr uint32_t kSlotDw = 4 * kWin + 1;  // odd stride: lanes at equal offsets on distinct banks
constexpr uint32_t kWaveDw = 64 * 32;       // LDS per wave: its 64 windows, later its 64 records (8 KiB)
static_assert(64 * kSlotDw <= kWaveDw, "the windows fit the record staging area");
extern __shared__ uint32_t fields_smem[];
typedef uint32_t u32_ua __attribute__((aligned(1)));

struct Hdr {
  const uint8_t* pk;  // packet byte 0 in memory
  uint32_t lb;        // byte offset of packet byte 0 in fields_smem
  uint32_t win;       // packet bytes [0, win) are in LDS
  __device__ __forceinline__ uint32_t u32(uint32_t p) const {  // 4 bytes at packet byte p, memory order
    if (p + 4 <= win)  // an unaligned ds_read_b32 (exact at any byte address on gfx950)
      return *reinterpret_cast<const u32_ua*>(reinterpret_cast<const uint8_t*>(fields_smem) + lb + p);
    return ldbytes(pk + p, 4);
  }
  // a 16-bit field reads its own 2 bytes only: from LDS as two byte reads when
  // it ends inside the window (a dword there could pass the window), else from
  // memory (the dword form read up to 7 bytes past the field)
  __device__ __forceinline__ uint32_t be16(uint32_t p) const {
    if (p + 4 <= win) {
      const uint32_t w = u32(p);
      return (w & 0xffu) << 8 | (w >> 8 & 0xffu);
    }
    if (p + 2 <= win) {
      const uint8_t* b = reinterpret_cast<const uint8_t*>(fields_smem) + lb + p;
      return (uint32_t)b[0] << 8 | b[1];
    }
    const uint32_t w = ldbytes(pk + p, 2);
    return (w & 0xffu) << 8 | w >> 8;
  }
  __device__ __forceinline__ uint32_t u8(uint32_t p) const {
    return p < win ? (uint32_t)reinterpret_cast<const uint8_t*>(fields_smem)[lb + p] : (uint32_t)pk[p];
  }
};

__global__ __launch_bounds__(kBlock) void fields_kernel(const uint8_t* data, const uint64_t* offsets,
                                                        const uint32_t* caplens, const gpk_layout* layouts, uint64_t n,
                                                        gpk_fields* out) {
  const uint64_t i0 = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool active = i0 < n;
  const uint64_t i = active ? i0 : n - 1;  // lanes past the batch redo the last packet, store nothing
  const uint64_t off = offsets[i];
  const uint32_t cl = caplens[i];
  const uint4* lp = reinterpret_cast<const uint4*>(layouts + i);
  const uint4 s0 = lp[0], s1 = lp[1], e0 = lp[2], e1 = lp[3];
  // the window: chunks past the packet re-read its last one (valid bytes)
  const uint32_t m = (uint32_t)(off & 15), win = cl < 16 * kWin - m ? cl : 16 * kWin - m;
  const uint32_t nch = (m + win + 15) >> 4, last = nch ? nch - 1 : 0;
  const uint8_t* wb = data + (off - m);
  const uint32_t lane = threadIdx.x & 63, wbase = (threadIdx.x >> 6) * kWaveDw;
  const uint32_t slot = wbase + lane * kSlotDw;
  u32x4 c[kWin];
#pragma unroll
  for (uint32_t k = 0; k < kWin; k++) c[k] = *reinterpret_cast<const u32x4*>(wb + 16 * (k < last ? k : last));
#pragma unroll
  for (uint32_t k = 0; k < kWin; k++) {
    fields_smem[slot + 4 * k + 0] = c[k].x;
    fields_smem[slot + 4 * k + 1] = c[k].y;
    fields_smem[slot + 4 * k + 2] = c[k].z;
    fields_smem[slot + 4 * k + 3] = c[k].w;
  }
  const Hdr h{data + off, slot * 4 + m, nch ? win : 0u};
  const uint32_t st[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
  const uint32_t en[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
  uint32_t w[32];
  uint32_t present = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) present |= (st[k] != GPK_LAYOUT_ABSENT ? 1u : 0u) << k;
  gpkf::fields_words(h, present, st, en[GPK_DEC_IPV4 - 1], w);
  // Records out through LDS: lane l's 128 bytes go to the wave's staging area
  // (chunk c at chunk position c ^ (l & 7), spreading the banks), then store
  // k of the wave writes its 1 KiB of records contiguously (coalesced), lane l
  // carrying chunk l & 7 of record 8k + l / 8. The wave's window reads above
  // precede these writes in its LDS instruction order.
  asm volatile("" ::: "memory");
#pragma unroll
  for (uint32_t c = 0; c < 8; c++)
    *reinterpret_cast<u32x4*>(fields_smem + wbase + lane * 32 + 4 * (c ^ (lane & 7))) =
        u32x4{w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]};
  asm volatile("" ::: "memory");
  const uint64_t first = (uint64_t)blockIdx.x * kBlock + (threadIdx.x & ~63u);  // the wave's first packet
  u32x4* o = reinterpret_cast<u32x4*>(out + first);
#pragma unroll
  for (uint32_t k = 0; k < 8; k++) {
    const uint32_t r = 8 * k + (lane >> 3), c = lane & 7;
    const u32x4 v = *reinterpret_cast<const u32x4*>(fields_smem + wbase + r * 32 + 4 * (c ^ (r & 7)));
    if (first + r < n) __builtin_nontemporal_store(v, o + 64 * k + lane);
  }
}

}  // namespace

static_assert(sizeof(gpk_fields) == 128, "gpk_fields is 128 bytes");
static_assert(offsetof(gpk_fields, tcp_seq) == 92 && offsetof(gpk_fields, udp_checksum) == 114 &&
                  offsetof(gpk_fields, ip4_start) == 116 && offsetof(gpk_fields, tcp_opt_map) == 123,
              "gpk_fields layout");

extern "C" int gpk_extract_fields(const gpk_batch* b, const gpk_layout* layouts, gpk_fields* fields, void* stream) {
  if (!b || (b->n && (!b->data || !b->offsets || !b->caplens || !layouts || !fields))) return GPK_EINVAL;
  if (!b->n) return GPK_OK;
  const uint64_t blocks = (b->n + kBlock - 1) / kBlock;
  if (blocks > 0x7fffffffull) return GPK_EINVAL;  // the grid's x dimension
  hipLaunchKernelGGL(fields_kernel, dim3((unsigned)blocks), dim3(kBlock), (kBlock / 64) * kWaveDw * 4, (hipStream_t)stream,
                     b->data, b->offsets, b->caplens, layouts, b->n, fields);
  return hipGetLastError() == hipSuccess ? GPK_OK : GPK_EHIP;
}

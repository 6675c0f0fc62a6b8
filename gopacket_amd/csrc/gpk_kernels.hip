// gpk_kernels.hip — batched DecodingLayerParser + Internet checksum + Flow
// hash for gfx950 (MI355X). Hand-written HIP; no MFMA (byte parse and integer
// reduction, HBM-bandwidth bound).
//
// One workgroup = 256 packets = 4 waves. Per packet the bytes are read once:
//
//  Phase A (lane per packet): the packet's first 128 B (16-byte aligned
//    chunks) are loaded with global_load_dwordx4 into the lane's LDS slot;
//    the lane runs DecodeLayers (gpk_device.h) out of LDS, computes the IPv4
//    header checksum (ip4.go:323-332), the three Flow.FastHash values
//    (flows.go:167-174) and, when the whole TCP/UDP segment sits inside the
//    window, the L4 checksum (tcpip.go:54-69) too.
//  Phase B (wave-cooperative): TCP/UDP segments that extend past the window
//    are summed by the whole wave. The wave's segments are cut into 16-byte
//    chunks laid end to end (exclusive scan of chunk counts); lane l takes
//    chunk t+l, so consecutive lanes load consecutive 16-byte chunks of the
//    same packet (coalesced dwordx4). Partial sums are combined with a
//    segmented scan keyed by packet and added into a per-packet LDS
//    accumulator. RFC1071 sums are position independent except for byte
//    parity, and ComputeChecksum wraps mod 2^32 (checksum.go:40-49), so
//    summing mod 2^32 in any order is bit-exact.
#include <hip/hip_runtime.h>

#include "gpk_device.h"

namespace gpk {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#ifndef GPK_NT_A
#define GPK_NT_A 0  // A/B (r01): temporal phase-A loads keep lines shared with phase B in L2: C3 +30%
#endif
#ifndef GPK_WAVES_PER_EU
#define GPK_WAVES_PER_EU 6  // <= 80 VGPRs: 6 waves/SIMD, matching the 6 blocks per CU the LDS allows
#endif
#ifndef GPK_LDS_FIT
#define GPK_LDS_FIT 1  // dynamic LDS sized to the parser's table blob (7 blocks/CU at 5 chunks)
#endif
#ifndef GPK_W4_WAVES
#define GPK_W4_WAVES 8  // 4-chunk window kernel: 64 VGPRs
#endif
#ifndef GPK_PB_G
#define GPK_PB_G 4  // phase B: pending packets per wave pass
#endif
#ifndef GPK_PREFETCH
#define GPK_PREFETCH 0  // 1: next tile's windows in flight (persistent only; A/B r01: no gain)
#endif
#ifndef GPK_PERSISTENT
#define GPK_PERSISTENT 0  // 1: blocks loop over tiles (A/B r01: +50 VGPRs from hoisting, no gain)
#endif
#ifndef GPK_PB_STREAM
#define GPK_PB_STREAM 1  // phase B as a continuous stream of 1 KiB wave loads
#endif
#ifndef GPK_PB_DEPTH
#define GPK_PB_DEPTH 8  // phase-B wave loads in flight
#endif
#ifndef GPK_PB_NULL
#define GPK_PB_NULL 0  // timing-only: phase-B loads read nothing (zero-record descriptors)
#endif
#ifndef GPK_PPL
#define GPK_PPL 1  // packets per lane (tiles per block)
#endif
#ifndef GPK_NT_B
#define GPK_NT_B 1
#endif

// 16-byte load; read-once packet bytes are non-temporal.
template <bool kNT>
__device__ __forceinline__ uint4 ld16t(const uint8_t* p) {
  u32x4 x = kNT ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p))
                : *reinterpret_cast<const u32x4*>(p);
  return make_uint4(x.x, x.y, x.z, x.w);
}
// header window and partial edge chunks (phase A) / full chunks (phase B)
__device__ __forceinline__ uint4 ld16(const uint8_t* p) { return ld16t<GPK_NT_A>(p); }
__device__ __forceinline__ uint4 ld16b(const uint8_t* p) { return ld16t<GPK_NT_B>(p); }

// Byte sums with v_dot4_u32_u8: bytes 0,2 (even addresses) and 1,3 (odd).
__device__ __forceinline__ uint32_t dot_even(uint32_t w, uint32_t acc) {
  return __builtin_amdgcn_udot4(w, 0x00010001u, acc, false);
}
__device__ __forceinline__ uint32_t dot_odd(uint32_t w, uint32_t acc) {
  return __builtin_amdgcn_udot4(w, 0x01000100u, acc, false);
}

// Sum of big-endian 16-bit words over LDS bytes [q, q+n) (ComputeChecksum
// with csum = 0, checksum.go:35-50; an odd tail byte counts <<8). Only the
// first and last dword are masked; interior dwords are two dot4s each.
__device__ __forceinline__ uint32_t sum_words_lds(uint32_t q, uint32_t n) {
  if (n == 0) return 0;
  const uint32_t last = q + n - 1;
  const uint32_t a0 = q & ~3u, a1 = last & ~3u;
  const uint32_t mhi = 0xffffffffu >> (8 * (3 - (last & 3)));
  uint32_t w = gpk_smem[a0 >> 2] & (0xffffffffu << (8 * (q & 3)));
  if (a0 == a1) w &= mhi;
  uint32_t E = dot_even(w, 0), O = dot_odd(w, 0);
  for (uint32_t a = a0 + 4; a < a1; a += 4) {
    w = gpk_smem[a >> 2];
    E = dot_even(w, E);
    O = dot_odd(w, O);
  }
  if (a1 != a0) {
    w = gpk_smem[a1 >> 2] & mhi;
    E = dot_even(w, E);
    O = dot_odd(w, O);
  }
  return (q & 1) ? (O << 8) + E : (E << 8) + O;
}

// Same over packet positions [p, p+n), from LDS when inside the window.
__device__ __forceinline__ uint32_t sum_words(const Rd& r, uint32_t p, uint32_t n) {
  if (p + n <= r.win) return sum_words_lds(r.lb + p, n);
  uint32_t s = 0;
  for (uint32_t k = 0; k + 1 < n; k += 2) s += rd16(r, p + k);
  if (n & 1) s += rd8(r, p + n - 1) << 8;
  return s;
}

// 16 bytes of a 16-aligned chunk at absolute address A, restricted to
// [s, e); a byte at address x counts <<8 when x has parity `par` (the parity
// of the segment's first byte: BE16 words start there). Used for the at most
// two partial chunks of a segment; full chunks go through chunk_eo.
__device__ __forceinline__ uint32_t chunk_sum(uint4 v, uint64_t A, uint64_t s, uint64_t e, uint32_t par) {
  uint32_t lo = s > A ? (uint32_t)(s - A) : 0u;        // 0..15
  uint32_t hi = e < A + 16 ? (uint32_t)(e - A) : 16u;  // 1..16
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t E = 0, O = 0;
#pragma unroll
  for (int d = 0; d < 4; d++) {
    int l = (int)lo - 4 * d, h = (int)hi - 4 * d;
    l = l < 0 ? 0 : (l > 4 ? 4 : l);
    h = h < 0 ? 0 : (h > 4 ? 4 : h);
    uint32_t m = h > l ? ((0xffffffffu >> (8 * (4 - (h - l)))) << (8 * l)) : 0u;
    E = dot_even(w[d] & m, E);
    O = dot_odd(w[d] & m, O);
  }
  return par ? (O << 8) + E : (E << 8) + O;
}

// Even/odd byte sums of a full chunk.
__device__ __forceinline__ void chunk_eo(uint4 v, uint32_t& E, uint32_t& O) {
  E = dot_even(v.x, E);
  O = dot_odd(v.x, O);
  E = dot_even(v.y, E);
  O = dot_odd(v.y, O);
  E = dot_even(v.z, E);
  O = dot_odd(v.z, O);
  E = dot_even(v.w, E);
  O = dot_odd(v.w, O);
}

// v_readlane_b32 returns int: widen through uint32_t, never through int
// (sign extension of an address's low word above 2 GiB corrupts it).
__device__ __forceinline__ uint32_t readlane32(uint32_t v, uint32_t lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t lane) {
  return ((uint64_t)readlane32((uint32_t)(v >> 32), lane) << 32) | (uint64_t)readlane32((uint32_t)v, lane);
}

// Sum over the 64 lanes (all active): rotations inside each 16-lane row
// (DPP row_ror 8,4,2,1), then the four row totals via readlane.
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x122, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x121, 0xf, 0xf, false);
  return readlane32(v, 0) + readlane32(v, 16) + readlane32(v, 32) + readlane32(v, 48);
}

// Header window of one packet in registers: chunks [0, nchunk) of the
// 16-byte-aligned run holding packet bytes [0, win).
template <int W>
struct WinT {
  uint4 v[W];
};
using Win = WinT<kWinChunks>;
// LDS dwords per lane for a window of W chunks (odd: see kSlotDw)
template <int W>
constexpr int slot_dw_of() {
  return W * 4 + (GPK_LINE_OWN ? 3 : 1);
}

struct Idx {
  uint64_t off;
  uint32_t cl;
};

__device__ __forceinline__ Idx load_index(const KParams& P, uint64_t i) {
  Idx x{0, 0};
  if (i < P.n) {
    x.off = P.offsets[i];
    x.cl = P.caplens[i];
  }
  return x;
}

template <int W = kWinChunks>
__device__ __forceinline__ uint32_t win_chunks(const Idx& x, bool active) {
  const uint32_t m = (uint32_t)(x.off & 15);
  uint32_t win = W * 16 - m;
  if (x.cl < win) win = x.cl;
  return active ? (m + win + 15) >> 4 : 0;
}

template <int W>
__device__ __forceinline__ void load_window(const KParams& P, const Idx& x, uint32_t nchunk, WinT<W>& w) {
  const uint8_t* src = P.data + (x.off & ~15ull);
#pragma unroll
  for (int k = 0; k < W; k++)
    if ((uint32_t)k < nchunk) w.v[k] = ld16(src + 16 * k);
}

template <int W>
__device__ __forceinline__ void store_window(uint32_t slot_dw, uint32_t nchunk, const WinT<W>& w) {
#pragma unroll
  for (int k = 0; k < W; k++)
    if ((uint32_t)k < nchunk) {
      gpk_smem[slot_dw + 4 * k + 0] = w.v[k].x;
      gpk_smem[slot_dw + 4 * k + 1] = w.v[k].y;
      gpk_smem[slot_dw + 4 * k + 2] = w.v[k].z;
      gpk_smem[slot_dw + 4 * k + 3] = w.v[k].w;
    }
}

// Line ownership (GPK_LINE_OWN). Phase B streams a packet's L4 bytes long
// after its header window was read, by which time L2 has evicted the window's
// lines: without care, the window's last 128-byte line and the packet's last
// line (which holds the next packet's header) are each fetched from HBM twice.
// So right after the window arrives (its lines are in L2) every lane also
// loads the other chunks of the lines the window touched:
//   head: [wend, he)  this packet's bytes after the window, up to the end of
//         the window's last line: even/odd byte sums (hE, hO);
//   tail: [L0, off)   the start of the window's first line, which is the END
//         of the previous packet when packets are contiguous: even/odd sums
//         (tE, tO) handed to lane-1, which then never touches that line.
// Phase B then streams whole lines [he, L0 of the next packet) only. Sums
// are by absolute byte parity, so the owner combines them with its segment
// parity like every other partial sum.
struct LineOwn {  // packed: three registers live across the parse
  uint32_t h;    // head sums: even | odd << 16 (<= 112 bytes: each < 2^16)
  uint32_t t;    // tail sums: even | odd << 16 (<= 127 bytes)
  uint32_t hx;   // (he - off) | tok << 8: head end relative to the packet, tail valid
};

__device__ __forceinline__ void chunk_eo_masked(uint4 v, uint32_t lo, uint32_t hi, uint32_t& E, uint32_t& O) {
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int d = 0; d < 4; d++) {
    int l = (int)lo - 4 * d, h = (int)hi - 4 * d;
    l = l < 0 ? 0 : (l > 4 ? 4 : l);
    h = h < 0 ? 0 : (h > 4 ? 4 : h);
    uint32_t m = h > l ? ((0xffffffffu >> (8 * (4 - (h - l)))) << (8 * l)) : 0u;
    E = dot_even(w[d] & m, E);
    O = dot_odd(w[d] & m, O);
  }
}

// Round 2 of the header loads: issued after the window chunks arrived, so
// these chunks (same lines) are L2 hits. prev_ok: the previous packet (lane-1)
// ends exactly at this packet's start and covers [off & ~127, off).
__device__ __forceinline__ LineOwn line_own(const KParams& P, uint64_t off, uint32_t cl, uint32_t nchunk,
                                            const uint4& chunk0, bool active, bool prev_ok) {
  const uint64_t A0 = off & ~15ull, wend = A0 + 16ull * nchunk, L0 = off & ~127ull;
  const uint64_t pend = (off + cl) & ~15ull;
  uint64_t he = (wend + 127) & ~127ull;
  if (he > pend) he = pend;
  if (he < wend || !active) he = wend;
  const uint32_t nh = (uint32_t)((he - wend) >> 4);
  const bool tok = active && prev_ok;
  const uint32_t nt = tok ? (uint32_t)((A0 - L0) >> 4) : 0u;
  uint32_t tE = 0, tO = 0, hE = 0, hO = 0;
  if (tok) chunk_eo_masked(chunk0, 0, (uint32_t)(off & 15), tE, tO);  // [A0, off) of chunk 0
  // the <= 11 non-window chunks of the <= 2 lines a window touches, in two
  // batches (7 + 4) so the loads in flight fit the 80-VGPR budget
#ifndef GPK_OWN_B2
#define GPK_OWN_B2 1  // two load batches (7 + 4) instead of one of 11
#endif
  constexpr int kB1 = GPK_OWN_B2 ? 7 : 11, kB2 = GPK_OWN_B2 ? 4 : 0;
#pragma unroll
  for (int b = 0; b < (kB2 ? 2 : 1); b++) {
    uint4 v[kB1];
    const int j0 = b ? kB1 : 0, nb = b ? kB2 : kB1;
    // batch 2 depends on batch 1's sums (an opaque zero): its loads cannot be
    // hoisted next to batch 1's, which would double the registers in flight
    uint32_t dep = 0;
    if (b) asm volatile("v_and_b32 %0, 0, %1" : "=v"(dep) : "v"(hE + tE));
#pragma unroll
    for (int k = 0; k < nb; k++) {
      const uint32_t j = (uint32_t)(j0 + k);
      const uint64_t a = (j < nt ? L0 + 16ull * j : wend + 16ull * (j - nt)) + dep;
      v[k] = j < nt + nh ? ld16(P.data + a) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < nb; k++) {
      uint32_t e = 0, od = 0;
      chunk_eo(v[k], e, od);
      if ((uint32_t)(j0 + k) < nt) {
        tE += e;
        tO += od;
      } else {
        hE += e;
        hO += od;
      }
    }
  }
  return LineOwn{hE | hO << 16, tE | tO << 16, (uint32_t)(he - off) | (tok ? 256u : 0u)};
}

__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, int d) {
  return ((uint64_t)(uint32_t)__shfl_up((int)(uint32_t)(v >> 32), d) << 32) | (uint32_t)__shfl_up((int)(uint32_t)v, d);
}
__device__ __forceinline__ uint64_t shfl_down64(uint64_t v, int d) {
  return ((uint64_t)(uint32_t)__shfl_down((int)(uint32_t)(v >> 32), d) << 32) | (uint32_t)__shfl_down((int)(uint32_t)v, d);
}

// The grouping key of gpk_flows.hip's key_kernel, derived here from the parse
// and the header bytes still in this lane's LDS window (include/gpk_flows.h:
// tcpassembly's key{netFlow, TransportFlow()}, ip4defrag's ipv4{NetworkFlow(),
// Id}), so the grouping needs no second pass over layouts and headers. Same
// words, same hash, same reason codes as key_kernel.
__device__ __forceinline__ uint32_t rd4raw(const Rd& r, uint32_t p) {
  return rd8(r, p) | rd8(r, p + 1) << 8 | rd8(r, p + 2) << 16 | rd8(r, p + 3) << 24;
}
__device__ __forceinline__ int derive_key(const KParams& P, const Rd& r, const Parse& q, uint32_t err, uint32_t* w) {
#pragma unroll
  for (int k = 0; k < 10; k++) w[k] = 0;
  if (P.key_kind == 1) {  // GPK_GROUP_CONNECTION
    if (!clean(q, GPK_DEC_TCP)) return -1;
    uint32_t net = 0;
    bool seen = false;
    const uint32_t m = q.nlayers < GPK_MAX_INLINE_LAYERS ? q.nlayers : GPK_MAX_INLINE_LAYERS;
    for (uint32_t k = 0; k < m && !seen; k++) {
      const uint32_t c = (uint32_t)(q.layers >> (4 * k)) & 15u;
      if (c == GPK_CODE_IPV4 || c == GPK_CODE_IPV6) net = c;
      seen = c == GPK_CODE_TCP;
    }
    if (!seen) return -6;
    if (!net) return -1;
    const uint32_t t0 = q.start(GPK_DEC_TCP);
    const uint32_t flags = rd8(r, t0 + 13), doff = rd8(r, t0 + 12) >> 4;
    if (!(flags & 7u) && (q.end(GPK_DEC_TCP) - t0) - doff * 4 == 0) return -2;
    if (net == GPK_CODE_IPV4) {
      const uint32_t ip = clean(q, GPK_DEC_IPV4) ? q.start(GPK_DEC_IPV4) : GPK_LAYOUT_ABSENT;
      w[0] = 1u | 1u << 8 | 4u << 16;
      w[1] = rd4raw(r, ip + 12);
      w[5] = rd4raw(r, ip + 16);
    } else {
      const uint32_t ip = clean(q, GPK_DEC_IPV6) ? q.start(GPK_DEC_IPV6) : GPK_LAYOUT_ABSENT;
      w[0] = 1u | 2u << 8 | 4u << 16;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        w[1 + k] = rd4raw(r, ip + 8 + 4 * k);
        w[5 + k] = rd4raw(r, ip + 24 + 4 * k);
      }
    }
    w[9] = rd4raw(r, t0);
    return 0;
  }
  // GPK_GROUP_DEFRAG
  if (!clean(q, GPK_DEC_IPV4) || (err >= GPK_ERR_IP4_HDR_SHORT && err <= GPK_ERR_IP4_OPT_BADLEN)) return -1;
  const uint32_t s = q.start(GPK_DEC_IPV4);
  const uint32_t ff = rd16(r, s + 6), flags = ff >> 13, fo = ff & 0x1FFF;
  if (flags & 2u) return -1;
  if (!(flags & 1u) && fo == 0) return -1;
  uint32_t len = rd16(r, s + 2);
  if (len == 0) len = (q.end(GPK_DEC_IPV4) - s) & 0xFFFF;
  if ((flags & 1u) && ((len - (rd8(r, s) & 15u) * 4) & 0xFFFF) < 8) return -3;
  if (fo > 8183) return -4;
  if (((fo * 8 + len) & 0xFFFF) > 65535u) return -5;
  w[0] = 2u | 1u << 8;
  w[1] = rd4raw(r, s + 12);
  w[5] = rd4raw(r, s + 16);
  w[9] = rd16(r, s + 4);
  return 0;
}

template <bool kL4, bool kLayout, class TT, bool kKeys = false, int W = kWinChunks>
__device__ __forceinline__ void decode_packet(const KParams& P, const TT& T, uint64_t i, bool active, uint64_t off,
                                              uint32_t cl, uint32_t slot_dw, uint32_t lane) {
  const uint32_t m = (uint32_t)(off & 15);
  uint32_t win = W * 16 - m;
  if (cl < win) win = cl;
  Rd r{P.data + off, slot_dw * 4 + m, win};

  // ---- Phase A: DecodeLayers ------------------------------------------------
  Parse q;
  q.init();
  Outcome s{0, 0, 0, 0};
#if GPK_FAST
  bool done = false;
  if (active && P.fast) done = fast_parser(P, T, r, cl, q, s);
  if (active && !done) s = run_parser<false>(P, T, r, cl, q);
#else
  if (active) s = run_parser<false>(P, T, r, cl, q);
#endif

  uint32_t st = (s.err & GPK_ST_ERR_MASK) | (s.trunc ? GPK_ST_TRUNCATED : 0u) |
                ((q.nlayers > GPK_ST_NLAYERS_MASK ? GPK_ST_NLAYERS_MASK : q.nlayers) << GPK_ST_NLAYERS_SHIFT);
  uint32_t ip4c = 0, l4c = 0;
  uint64_t lflow = 0, nflow = 0, tflow = 0;

  // L4 checksum: bytes of the segment inside the LDS window are summed here;
  // the rest, [ja, je) of data, is a job for the wave-cooperative phase B.
  uint64_t ja = 0, je = 0;
  uint32_t jsum = 0, jexist = 0, jpar = 0;
  bool job = false;

  if (active) {
    if ((P.outputs & GPK_OUT_IP4_CSUM) && clean(q, GPK_DEC_IPV4)) {  // ip4.go:323-332
      uint32_t s4 = q.start(GPK_DEC_IPV4);
      uint32_t hl = (rd8(r, s4) & 15) * 4;
      uint32_t existing = rd16(r, s4 + 10);
      ip4c = fold(sum_words(r, s4, hl) - existing);
      st |= GPK_ST_IP4_CSUM | (ip4c == existing ? GPK_ST_IP4_VALID : 0u);
    }
    const uint32_t tk = q.transport, nk = q.last_net;
    if ((P.outputs & GPK_OUT_L4_CSUM) && tk && clean(q, tk) && nk && clean(q, nk)) {
      // tcp.go:626-640 / udp.go:144-158 via tcpip.go:54-69
      uint32_t t0 = q.start(tk);
      uint32_t blen = tk == GPK_DEC_TCP ? q.end(tk) - t0 : q.udp_hlen;
      uint32_t ns = q.start(nk);
      uint32_t init = nk == GPK_DEC_IPV4 ? sum_words(r, ns + 12, 8) : sum_words(r, ns + 8, 32);
      init += (tk == GPK_DEC_TCP ? 6u : 17u) + (blen & 0xffff) + (blen >> 16);
      jexist = rd16(r, t0 + (tk == GPK_DEC_TCP ? 16 : 6));
      st |= GPK_ST_L4_CSUM | (tk == GPK_DEC_UDP ? GPK_ST_L4_UDP : 0u);
      uint32_t tend = t0 + blen;
      uint32_t in_end = tend < win ? tend : win;
      uint32_t part = t0 < in_end ? sum_words_lds(r.lb + t0, in_end - t0) : 0u;
      if (tend <= win) {
        l4c = fold(init + part - jexist);
      } else if (kL4) {
        // Remainder [ra, re) past the window: its partial first / last
        // 16-byte chunks are summed here, the full chunks in phase B.
        const uint64_t ra = off + (t0 > win ? t0 : win), re = off + tend;
        const uint32_t par = (uint32_t)((off + t0) & 1);
        const uint64_t fa = (ra + 15) & ~15ull, fe = re & ~15ull;
        uint32_t edge = 0;
#if GPK_LINE_OWN
        // head: the window's last line after the window, summed at load time
        // (LineOwn sums in this lane's LDS slot; the next packet's in lane+1's,
        // written by that lane of this wave before the parse)
        const uint32_t own_h = gpk_smem[slot_dw + kOwnDw], own_hx = gpk_smem[slot_dw + kOwnDw + 2];
        const uint32_t nx_t = gpk_smem[slot_dw + kSlotDw + kOwnDw + 1];
        const bool nx_tok = lane < 63 && (gpk_smem[slot_dw + kSlotDw + kOwnDw + 2] & 256u);
        const uint64_t he = off + (own_hx & 255u);
        const bool head_ok = t0 <= win && he > ra && he <= re;
        const uint64_t bs = head_ok ? he : fa;
        if (head_ok) edge += par ? ((own_h >> 16) << 8) + (own_h & 0xffff) : ((own_h & 0xffff) << 8) + (own_h >> 16);
        // tail: the next packet's line head, summed by lane+1 (which saw this
        // packet end exactly at its start)
        const uint64_t nl0 = re & ~127ull;
        const bool tail_ok = nx_tok && re == off + cl && nl0 >= bs && fa <= fe;
        const uint64_t be = tail_ok ? nl0 : fe;
        if (tail_ok) edge += par ? ((nx_t >> 16) << 8) + (nx_t & 0xffff) : ((nx_t & 0xffff) << 8) + (nx_t >> 16);
        if (fa > fe) {  // remainder inside a single chunk
          edge = chunk_sum(ld16(P.data + (ra & ~15ull)), ra & ~15ull, ra, re, par);
        } else {
          if (!head_ok && ra != fa) edge += chunk_sum(ld16(P.data + (ra & ~15ull)), ra & ~15ull, ra, re, par);
          if (!tail_ok && re != fe) edge += chunk_sum(ld16(P.data + fe), fe, ra, re, par);
        }
        jsum = init + part + edge;
        job = bs < be;
        ja = bs;
        je = be;
#else
        if (fa > fe) {  // remainder inside a single chunk
          edge = chunk_sum(ld16(P.data + (ra & ~15ull)), ra & ~15ull, ra, re, par);
        } else {
          if (ra != fa) edge += chunk_sum(ld16(P.data + (ra & ~15ull)), ra & ~15ull, ra, re, par);
          if (re != fe) edge += chunk_sum(ld16(P.data + fe), fe, ra, re, par);
        }
        jsum = init + part + edge;
        job = fa < fe;
        ja = fa;
        je = fe;
#endif
        jpar = par;
        if (!job) l4c = fold(jsum - jexist);
      }
    }
    if (P.outputs & GPK_OUT_FLOWS) {
      if (clean(q, GPK_DEC_ETHERNET)) {  // ethernet.go:38-40 (EndpointMAC = 3)
        uint32_t e0 = q.start(GPK_DEC_ETHERNET);
        lflow = flow_hash(fnv_range(r, e0 + 6, 6), fnv_range(r, e0, 6), 3);
        st |= GPK_ST_LINK_FLOW;
      }
      if (nk && clean(q, nk)) {
        uint32_t ns = q.start(nk);
        if (nk == GPK_DEC_IPV4) {  // ip4.go:63-65 (EndpointIPv4 = 1)
          nflow = flow_hash(fnv_range(r, ns + 12, 4), fnv_range(r, ns + 16, 4), 1);
        } else {  // ip6.go:49-51 (EndpointIPv6 = 2)
          nflow = flow_hash(fnv_range(r, ns + 8, 16), fnv_range(r, ns + 24, 16), 2);
          st |= GPK_ST_NET_IPV6;
        }
        st |= GPK_ST_NET_FLOW;
      }
      if (tk && clean(q, tk)) {  // tcp.go:614-616 (4), udp.go:132-134 (5)
        uint32_t t0 = q.start(tk);
        tflow = flow_hash(fnv_range(r, t0, 2), fnv_range(r, t0 + 2, 2), tk == GPK_DEC_TCP ? 4 : 5);
        st |= GPK_ST_TRANSPORT_FLOW;
      }
    }
  }

  // ---- Phase B: L4 segments past the window, one packet per wave pass ------
  // The wave takes up to four pending packets at a time; every lane loads
  // 16-byte chunks of each (consecutive lanes -> consecutive chunks: whole
  // cache lines per wave instruction), two 1 KiB rounds in flight per packet,
  // then each packet's partial sums are reduced across the wave (DPP row
  // rotations + four readlanes) into the owning lane. No LDS traffic.
  if (kL4) {
    uint32_t extra = 0;
    uint64_t pend = __ballot(job);
#if GPK_PB_STREAM
    // The wave's pending segments as one stream of 1 KiB wave loads (items),
    // packet after packet, GPK_PB_DEPTH items always in flight: a register
    // ring, refilled as each item is consumed. Item = one raw-buffer load of
    // 16 bytes per lane from the packet's remaining whole chunks; bytes past
    // the packet's end come back as zeros (range check), so no predicates.
    const uint32_t vo = lane * 16;
    constexpr int D = GPK_PB_DEPTH;
    uint32_t p_lane = 64, p_off = 0, p_len = 0;  // producer (wave-uniform)
    __amdgpu_buffer_rsrc_t p_rs = __builtin_amdgcn_make_buffer_rsrc((void*)P.data, 0, 0, 0x00020000);
    u32x4 ring[D];
    uint32_t r_lane[D], r_last[D];
#pragma unroll
    for (int k = 0; k < D; k++) {
      if (p_off >= p_len) {
        p_lane = 64;
        p_off = p_len = 0;
        uint64_t b0 = 0;
        if (pend) {
          p_lane = (uint32_t)__builtin_ctzll(pend);
          pend &= pend - 1;
          b0 = readlane64(ja, p_lane);
          p_len = (uint32_t)(readlane64(je, p_lane) - b0);
        }
        p_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(P.data + b0), 0, GPK_PB_NULL ? 0 : p_len, 0x00020000);
      }
      ring[k] = __builtin_amdgcn_raw_buffer_load_b128(p_rs, vo, p_off, GPK_NT_B ? 2 : 0);
      r_lane[k] = p_lane;
      r_last[k] = p_off + 1024 >= p_len;
      p_off += 1024;
    }
    uint32_t E = 0, O = 0;
    for (;;) {
      uint32_t live = 0;
#pragma unroll
      for (int k = 0; k < D; k++) {
        if (r_lane[k] < 64) {
          const u32x4 x = ring[k];
          chunk_eo(make_uint4(x.x, x.y, x.z, x.w), E, O);
          if (r_last[k]) {
            const uint32_t pr = readlane32(jpar, r_lane[k]);
            const uint32_t t = wave_sum(pr ? (O << 8) + E : (E << 8) + O);
            if (lane == r_lane[k]) extra += t;
            E = O = 0;
          }
        }
        if (p_off >= p_len) {
          p_lane = 64;
          p_off = p_len = 0;
          uint64_t b0 = 0;
          if (pend) {
            p_lane = (uint32_t)__builtin_ctzll(pend);
            pend &= pend - 1;
            b0 = readlane64(ja, p_lane);
            p_len = (uint32_t)(readlane64(je, p_lane) - b0);
          }
          p_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(P.data + b0), 0, GPK_PB_NULL ? 0 : p_len, 0x00020000);
        }
        ring[k] = __builtin_amdgcn_raw_buffer_load_b128(p_rs, vo, p_off, GPK_NT_B ? 2 : 0);
        r_lane[k] = p_lane;
        r_last[k] = p_off + 1024 >= p_len;
        p_off += 1024;
        live |= r_lane[k] < 64;
      }
      if (!live) break;
    }
#else
    const uint32_t vo = lane * 16;
    while (pend) {
      constexpr int G = GPK_PB_G;
      uint32_t jl[G];
      uint32_t len[G];
      __amdgpu_buffer_rsrc_t rs[G];
      uint32_t pr[G];
#pragma unroll
      for (int g = 0; g < G; g++) {
        jl[g] = 64;
        len[g] = 0;  // empty slot: a zero-record descriptor, every load returns 0
        pr[g] = 0;
        uint64_t b0 = 0;
        if (pend) {
          uint32_t j = (uint32_t)__builtin_ctzll(pend);
          pend &= pend - 1;
          jl[g] = j;
          b0 = readlane64(ja, j);
          len[g] = (uint32_t)(readlane64(je, j) - b0);
          pr[g] = readlane32(jpar, j);
        }
        // [b0, b0+len) as a raw buffer: loads past its end return zeros
        // (hardware range check), so no lane needs a predicate or a mask
        rs[g] = __builtin_amdgcn_make_buffer_rsrc((void*)(P.data + b0), 0, len[g], 0x00020000);
      }
      uint32_t E[G], O[G];
#pragma unroll
      for (int g = 0; g < G; g++) E[g] = O[g] = 0;
      uint32_t maxlen = 0;
#pragma unroll
      for (int g = 0; g < G; g++) maxlen = len[g] > maxlen ? len[g] : maxlen;
      for (uint32_t rr = 0; rr < maxlen; rr += 2048) {
        u32x4 v[G][2];
#pragma unroll
        for (int g = 0; g < G; g++)
#pragma unroll
          for (int h = 0; h < 2; h++)
            v[g][h] = __builtin_amdgcn_raw_buffer_load_b128(rs[g], vo + h * 1024, rr, GPK_NT_B ? 2 : 0);
#pragma unroll
        for (int g = 0; g < G; g++)
#pragma unroll
          for (int h = 0; h < 2; h++) chunk_eo(make_uint4(v[g][h].x, v[g][h].y, v[g][h].z, v[g][h].w), E[g], O[g]);
      }
#pragma unroll
      for (int g = 0; g < G; g++) {
        if (jl[g] < 64) {
          uint32_t t = wave_sum(pr[g] ? (O[g] << 8) + E[g] : (E[g] << 8) + O[g]);
          if (lane == jl[g]) extra += t;
        }
      }
    }
#endif
    if (job) l4c = fold(jsum + extra - jexist);
  }
  if (active && (st & GPK_ST_L4_CSUM)) {
    bool udp = (st & GPK_ST_L4_UDP) != 0;
    if (l4c == jexist || (udp && jexist == 0)) st |= GPK_ST_L4_VALID;
  }

  // ---- outputs ---------------------------------------------------------------
  if (active) {
    uint4 rec = make_uint4((uint32_t)q.layers, (uint32_t)(q.layers >> 32), st, ip4c | (l4c << 16));
    reinterpret_cast<uint4*>(P.records)[i] = rec;
    if (P.flows) {
      P.flows[i] = lflow;
      P.flows[P.n + i] = nflow;
      P.flows[2 * P.n + i] = tflow;
    }
    if (s.err && P.err_args) {
      P.err_args[2 * i] = s.a0;
      P.err_args[2 * i + 1] = s.a1;
    }
    if (kKeys) {  // fused grouping key (gpk_decode_group_batch)
      uint32_t w[10];
      const int c = derive_key(P, r, q, s.err & GPK_ST_ERR_MASK, w);
      P.kcode[i] = c;
      if (!c) {
        uint64_t h = 0x9E3779B97F4A7C15ull;
#pragma unroll
        for (int k = 0; k < 10; k++) {
          P.keys[i * 10 + k] = w[k];
          h = (h ^ w[k]) * 0xBF58476D1CE4E5B9ull;
          h ^= h >> 29;
        }
        h = (h ^ (h >> 30)) * 0xBF58476D1CE4E5B9ull;
        h = (h ^ (h >> 27)) * 0x94D049BB133111EBull;
        P.khash[i] = h ^ (h >> 31);
      }
    }
    if (kLayout) {
      const int slot_kind[8] = {GPK_DEC_ETHERNET, GPK_DEC_DOT1Q, GPK_DEC_IPV4, GPK_DEC_IPV6,
                                       GPK_DEC_IPV6_EXT, GPK_DEC_TCP,  GPK_DEC_UDP,  GPK_DEC_PAYLOAD};
      uint32_t so[8], eo[8];
#pragma unroll
      for (int k = 0; k < 8; k++) {
        int kd = slot_kind[k];
        if (k == 7 && !clean(q, GPK_DEC_PAYLOAD)) kd = GPK_DEC_FRAGMENT;
        bool c = clean(q, kd);
        so[k] = c ? q.start(kd) : GPK_LAYOUT_ABSENT;
        eo[k] = c ? q.end(kd) : GPK_LAYOUT_ABSENT;
      }
      uint4* L = reinterpret_cast<uint4*>(P.layouts + i);
      L[0] = make_uint4(so[0], so[1], so[2], so[3]);
      L[1] = make_uint4(so[4], so[5], so[6], so[7]);
      L[2] = make_uint4(eo[0], eo[1], eo[2], eo[3]);
      L[3] = make_uint4(eo[4], eo[5], eo[6], eo[7]);
    }
  }
}

// Persistent, software-pipelined over tiles of kBlock packets: block b takes
// tiles b, b+grid, b+2*grid, ... (grid = resident blocks, gpk_launch_decode).
// While tile t is decoded, the header windows of tile t+grid are in flight
// (registers) and the offsets/caplens of tile t+2*grid too, so the global
// load latency of the read-once header bytes is hidden behind decode work.
// The LDS slot is lane-private: no barrier between tiles.
template <bool kL4, bool kLayout, class TT, bool kKeys = false>
__device__ __forceinline__ void decode_tiles(const KParams& P, const TT& T) {
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63;
  const uint32_t slot_dw = tid * kSlotDw;
  const uint64_t ntiles = (P.n + kBlock - 1) / kBlock;
  [[maybe_unused]] const uint64_t stride = gridDim.x;
  uint64_t t = blockIdx.x;
  if (t >= ntiles) return;  // uniform over the block

  uint64_t i = t * kBlock + tid;
#if GPK_PREFETCH
  Idx cur = load_index(P, i);
  uint32_t nc = win_chunks(cur, i < P.n);
  Win w;
  load_window(P, cur, nc, w);
  Idx nxt = load_index(P, i + stride * kBlock);
  for (;;) {
    store_window(slot_dw, nc, w);
    const uint64_t i1 = i + stride * kBlock;
    const uint32_t nc1 = win_chunks(nxt, i1 < P.n);
    load_window(P, nxt, nc1, w);                         // tile t+grid, in flight
    const Idx nn = load_index(P, i1 + stride * kBlock);  // tile t+2*grid
    decode_packet<kL4, kLayout, TT, kKeys>(P, T, i, i < P.n, cur.off, cur.cl, slot_dw, lane);
    t += stride;
    if (t >= ntiles) break;
    i = i1;
    cur = nxt;
    nc = nc1;
    nxt = nn;
  }
#elif !GPK_PERSISTENT
  {  // one tile per block
    const Idx cur = load_index(P, i);
    const uint32_t nc = win_chunks(cur, i < P.n);
    Win w;
    load_window(P, cur, nc, w);
    store_window(slot_dw, nc, w);
    decode_packet<kL4, kLayout, TT, kKeys>(P, T, i, i < P.n, cur.off, cur.cl, slot_dw, lane);
  }
#else
  Idx nxt = load_index(P, i);
  for (;;) {
    const Idx cur = nxt;
    const uint32_t nc = win_chunks(cur, i < P.n);
    Win w;
    load_window(P, cur, nc, w);
    nxt = load_index(P, i + stride * kBlock);  // next tile's offsets/caplens
    store_window(slot_dw, nc, w);
    decode_packet<kL4, kLayout, TT, kKeys>(P, T, i, i < P.n, cur.off, cur.cl, slot_dw, lane);
    t += stride;
    if (t >= ntiles) break;
    i += stride * kBlock;
  }
#endif
}

// kCompact: the parser's lookup tables are copied into LDS once per block
// (after the header-window slots) and every NextLayerType lookup is an LDS
// read; otherwise they are read from the global DevTables. Either way the
// only vector-memory traffic of the decode is the packet bytes themselves,
// so waiting on a lookup never waits on the next tile's prefetch.
// W: header-window chunks. The 5-chunk default holds Ethernet + two tags +
// IPv6 + TCP; parsers with no Dot1Q/IPv6/TCP decoder and no L4 checksum (C2)
// run a 4-chunk window whose smaller LDS slot and 64-VGPR budget give 8 waves
// per SIMD (A/B: C2 -8.6 %, C4 and C3 no gain or worse with 4 chunks).
// O: waves per SIMD the register budget is cut for. Batches of small packets
// (mean < 1 KiB) are issue-bound in the header phase and run O = 7 (72 VGPRs;
// with the table blob sized to the parser, 7 blocks fit a CU's LDS); big
// packets keep O = 6 (A/B r02c: C4 -5.9 %, C1 -4.9 %, C3 +0.5 % at 7).
template <bool kL4, bool kLayout, bool kCompact, bool kKeys = false, int W = kWinChunks, int O = GPK_WAVES_PER_EU>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(W == 4 ? GPK_W4_WAVES : O, 8))) void decode_kernel(
    KParams P) {
  if ((uint64_t)blockIdx.x * kBlock * GPK_PPL >= P.n) return;  // uniform over the block
#if !GPK_PERSISTENT && !GPK_PREFETCH
  // GPK_PPL tiles per block, one packet of each per lane: every packet's
  // index, then every header window (the first in LDS, the others held in
  // registers) and the table blob are in flight together, so the two
  // dependent memory round trips are paid once for GPK_PPL packets.
  const uint32_t tid = threadIdx.x;
  const uint32_t slot_dw = tid * slot_dw_of<W>();
  const uint64_t i0 = (uint64_t)blockIdx.x * (kBlock * GPK_PPL) + tid, i1 = i0 + kBlock;
  static_assert(GPK_PPL == 1 || GPK_PPL == 2, "GPK_PPL is 1 or 2");
  const Idx c0 = load_index(P, i0);
  const Idx c1 = GPK_PPL == 2 ? load_index(P, i1) : Idx{0, 0};
  const uint32_t n0 = win_chunks<W>(c0, i0 < P.n);
  const uint32_t n1 = GPK_PPL == 2 ? win_chunks<W>(c1, i1 < P.n) : 0;
  WinT<W> w0, w1;
  load_window(P, c0, n0, w0);
  if (GPK_PPL == 2) load_window(P, c1, n1, w1);
  const uint32_t base = kBlock * slot_dw_of<W>();
  if (kCompact) {
    for (uint32_t k = tid; k < P.cg.words; k += kBlock) gpk_smem[base + k] = P.ctab[k];
    __syncthreads();
  }
#ifndef GPK_OWN_EARLY
#define GPK_OWN_EARLY 0  // 1: issue the line-ownership loads with the window loads
#endif
#if GPK_LINE_OWN && GPK_OWN_EARLY
  LineOwn own{0, 0, 0};
  if (kL4) {
    const uint64_t poff = shfl_up64(c0.off, 1);
    const uint32_t pcl = (uint32_t)__shfl_up((int)c0.cl, 1);
    const bool prev_ok = (tid & 63) > 0 && poff + pcl == c0.off && poff <= (c0.off & ~127ull);
    own = line_own(P, c0.off, c0.cl, n0, w0.v[0], i0 < P.n, prev_ok);
  }
#endif
  store_window(slot_dw, n0, w0);
#if GPK_LINE_OWN
  if (kL4) {
#if !GPK_OWN_EARLY
    const uint64_t poff = shfl_up64(c0.off, 1);
    const uint32_t pcl = (uint32_t)__shfl_up((int)c0.cl, 1);
    const bool prev_ok = (tid & 63) > 0 && poff + pcl == c0.off && poff <= (c0.off & ~127ull);
    const LineOwn own = line_own(P, c0.off, c0.cl, n0, w0.v[0], i0 < P.n, prev_ok);
#endif
    gpk_smem[slot_dw + kOwnDw] = own.h;
    gpk_smem[slot_dw + kOwnDw + 1] = own.t;
    gpk_smem[slot_dw + kOwnDw + 2] = own.hx;
  }
#endif
  if (kCompact)
    decode_packet<kL4, kLayout, LTab, kKeys, W>(P, LTab{P.cg, base}, i0, i0 < P.n, c0.off, c0.cl, slot_dw, tid & 63);
  else
    decode_packet<kL4, kLayout, GTab, kKeys, W>(P, GTab{P.tab}, i0, i0 < P.n, c0.off, c0.cl, slot_dw, tid & 63);
  if (GPK_PPL == 2) {
    store_window(slot_dw, n1, w1);  // lane-private slot, reused
    if (kCompact)
      decode_packet<kL4, kLayout, LTab, kKeys, W>(P, LTab{P.cg, base}, i1, i1 < P.n, c1.off, c1.cl, slot_dw, tid & 63);
    else
      decode_packet<kL4, kLayout, GTab, kKeys, W>(P, GTab{P.tab}, i1, i1 < P.n, c1.off, c1.cl, slot_dw, tid & 63);
  }
#else
  if (kCompact) {
    const uint32_t base = kBlock * kSlotDw;
    for (uint32_t w = threadIdx.x; w < P.cg.words; w += kBlock) gpk_smem[base + w] = P.ctab[w];
    __syncthreads();
    decode_tiles<kL4, kLayout, LTab, kKeys>(P, LTab{P.cg, base});
  } else {
    decode_tiles<kL4, kLayout, GTab, kKeys>(P, GTab{P.tab});
  }
#endif
}

// Full decoded list of one packet (lists longer than the 16 inline codes).
__global__ void list_kernel(KParams P, uint64_t index, int64_t* out, uint32_t cap, uint32_t* out_n) {
  if (threadIdx.x != 0) return;
  uint64_t off = P.offsets[index];
  uint32_t cl = P.caplens[index];
  Rd r{P.data + off, 0, 0};  // no LDS window: every byte from global memory
  Parse q;
  run_parser<true>(P, GTab{P.tab}, r, cl, q, out, cap);
  *out_n = q.nlayers;
}

}  // namespace gpk

namespace {

template <bool kL4, bool kLayout, bool kCompact, bool kKeys = false, int W = gpk::kWinChunks,
          int O = GPK_WAVES_PER_EU>
hipError_t launch(const gpk::KParams* P, hipStream_t stream) {
  using namespace gpk;
  constexpr int slot_lds = kBlock * slot_dw_of<W>() * 4;
#if GPK_LDS_FIT
  // the table blob takes only the words this parser's tables use (C3/C4: ~1.5 KB of 2.9)
  const int lds = kCompact ? slot_lds + (int)((P->cg.words + 127) & ~127u) * 4 : slot_lds;
#else
  constexpr int lds = kCompact ? slot_lds + kCtDwords * 4 : slot_lds;
#endif
  // Resident blocks per CU for this specialisation (cached per device).
  static int cached_bpc[64], cached_cus[64];  // per instantiation
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
  if (!cached_bpc[dev]) {
    int bpc = 0, cus = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, decode_kernel<kL4, kLayout, kCompact, kKeys, W, O>, kBlock,
                                                     lds);
    if (e != hipSuccess) return e;
    e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    cached_cus[dev] = cus > 0 ? cus : 1;
    cached_bpc[dev] = bpc > 0 ? bpc : 1;
  }
  // 8 rounds of resident blocks: if the occupancy figure is one block per CU
  // high, the static tile schedule loses ~3% instead of running a second
  // generation of late blocks; each block still pipelines >= 8 tiles.
  const uint64_t ntiles = (P->n + kBlock - 1) / kBlock;
  uint64_t grid = (uint64_t)cached_cus[dev] * cached_bpc[dev] * 8;
  if (ntiles < grid * 8) grid = (ntiles + 7) / 8;
  if (!GPK_PERSISTENT && !GPK_PREFETCH) grid = (ntiles + GPK_PPL - 1) / GPK_PPL;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL((decode_kernel<kL4, kLayout, kCompact, kKeys, W, O>), dim3((unsigned)grid), dim3(kBlock), lds,
                     stream, *P);
  return hipGetLastError();
}

template <bool kCompact>
hipError_t launch_outputs(const gpk::KParams* P, int with_l4, int with_layout, hipStream_t stream) {
  if (P->key_kind) {  // fused grouping keys: no layouts (gpk_decode_group_batch)
    if (with_layout) return hipErrorInvalidValue;
    return with_l4 ? launch<true, false, kCompact, true>(P, stream) : launch<false, false, kCompact, true>(P, stream);
  }
  if (!with_l4 && !with_layout && P->small_headers) return launch<false, false, kCompact, false, 4>(P, stream);
  constexpr int W = gpk::kWinChunks;
  if (with_l4 && with_layout) return launch<true, true, kCompact>(P, stream);
  if (with_l4)
    return P->big_packets ? launch<true, false, kCompact>(P, stream) : launch<true, false, kCompact, false, W, 7>(P, stream);
  if (!with_layout && !P->big_packets) return launch<false, false, kCompact, false, W, 7>(P, stream);
  if (with_layout) return launch<false, true, kCompact>(P, stream);
  return launch<false, false, kCompact>(P, stream);
}

}  // namespace

extern "C" hipError_t gpk_launch_decode(const gpk::KParams* P, int with_l4, int with_layout, hipStream_t stream) {
  if (P->n == 0) return hipSuccess;
  return P->ctab ? launch_outputs<true>(P, with_l4, with_layout, stream)
                 : launch_outputs<false>(P, with_l4, with_layout, stream);
}

extern "C" hipError_t gpk_launch_list(const gpk::KParams* P, uint64_t index, int64_t* out, uint32_t cap,
                                      uint32_t* out_n, hipStream_t stream) {
  hipLaunchKernelGGL(gpk::list_kernel, dim3(1), dim3(64), 0, stream, *P, index, out, cap, out_n);
  return hipGetLastError();
}

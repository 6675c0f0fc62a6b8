// gpk_kernels.hip — batched DecodingLayerParser + Internet checksum + Flow
// hash for gfx950 (MI355X). Hand-written HIP; no MFMA (byte parse and integer
// reduction, HBM-bandwidth bound).
//
// One workgroup = 256 packets = 4 waves, one lane per packet.
//
//  Phase A (lane per packet): the 16-byte-aligned run of W chunks holding
//    the packet's first bytes (W = 6: 96 bytes; 4 for header-only parsers)
//    is loaded into the lane's LDS slot; the lane runs DecodeLayers
//    (gpk_device.h: a straight-line common case, else the general state
//    machine) out of LDS, computes the IPv4 header checksum
//    (ip4.go:323-332), the three Flow.FastHash values (flows.go:167-174) and,
//    for the TCP/UDP checksum (tcpip.go:54-69), the pseudo-header sum and the
//    byte range [s, e) of the segment.
//  Phase B (wave-cooperative): the segments' byte sums. RFC1071 word sums are
//    position independent except for byte parity, and ComputeChecksum wraps
//    mod 2^32 (checksum.go:40-49), so the sum of [s, e) is assembled from
//    even-/odd-address byte sums mod 2^32 in any order, bit-exactly:
//    * dense waves (the usual packed batch: the wave's segments lie in one
//      region not much larger than their total): the wave streams the whole
//      region once, 1 KiB per pass (16 bytes per lane, one coalesced
//      raw-buffer load), keeps a running wave-wide prefix sum of one 32-bit
//      L-form sum per 16-byte granule (little-endian words at even addresses:
//      v_sad_u16; one DPP scan), and every lane picks the prefix at its
//      segment's first and last granule with ds_bpermute. Segment sum =
//      prefix difference - the head granule's bytes before s + the tail
//      granule's bytes before e, turned into the big-endian word sum of the
//      segment's alignment (exact mod 65535 for segments <= 64 KiB, which
//      is all the fold needs; see l_to_words). No per-packet reduction.
//    * sparse waves (scattered offsets): the segments are streamed one after
//      another as whole-wave 1 KiB loads and reduced per packet (DPP).
#include <hip/hip_runtime.h>

#include <cstdio>

#include "gpk_device.h"
#include "gpk_fields.h"

namespace gpk {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#ifndef GPK_WAVES_PER_EU
#define GPK_WAVES_PER_EU 6  // <= 80 VGPRs: 6 waves/SIMD, matching the 6 blocks per CU the LDS allows
#endif
#ifndef GPK_SMALL_WAVES
#define GPK_SMALL_WAVES 7  // register budget of batches with a mean packet under 1 KiB (waves per SIMD)
#endif
#ifndef GPK_W4_WAVES
#define GPK_W4_WAVES 8  // 4-chunk window kernel: 64 VGPRs
#endif
#ifndef GPK_MID_W5
#define GPK_MID_W5 1  // small-packet kernels of parsers without IPv6: dword-aligned 5-chunk window
#endif
#ifndef GPK_MID_MAXMEAN
#define GPK_MID_MAXMEAN 256  // ... for batches whose mean packet (batch bytes / packets) is under this
#endif
#ifndef GPK_MID_IP6
#define GPK_MID_IP6 0  // ... for parsers with IPv6 too
#endif
#ifndef GPK_PB_GRAN
#define GPK_PB_GRAN 1  // dense phase B: 16-byte chunks per lane per pass (A/B r03: 1 KiB passes, whole
                       // lines per load instruction, beat 2 KiB passes of two half-coalesced loads by 20 %)
#endif
#ifndef GPK_PB_DEPTH
#define GPK_PB_DEPTH 8  // dense phase B: passes in flight (80-VGPR kernels; A/B r04b: 8 vs 6 -0.4 % C3, 10 no better)
#endif
#ifndef GPK_PB_DEPTH7
#define GPK_PB_DEPTH7 8  // ... in the 72-VGPR kernels (7 waves per SIMD; A/B r04b: 6 vs 4 -0.9 % C4, -2.8 % C1; r14: 8 vs 6 C1 -3.9 %; 10 spills)
#endif
#ifndef GPK_PB_DEPTH7SB
#define GPK_PB_DEPTH7SB 5  // ... in the stream-before-parse kernel's phase B after the parse (the fallback of waves whose
                           // packets are not packed; 6: 20 B of scratch, 8: 40 B; 5 and below: none)
#endif
#ifndef GPK_PB_DEPTHF
#define GPK_PB_DEPTHF 4  // ... in its fused-fields variant
#endif
#ifndef GPK_PB_IDPERM
#define GPK_PB_IDPERM 1  // dense phase B: lanes outside their target pass pull their own prefix (no LDS bank conflicts)
#endif
#ifndef GPK_PB_LDS_HT
#define GPK_PB_LDS_HT 1  // segment head/tail chunks from the LDS header windows when they hold them
#endif
#ifndef GPK_BLOB_DMA
#define GPK_BLOB_DMA 0  // each wave copies the table blob into LDS by LDS-DMA itself, no block barrier (A/B r15:
                        // C4 +-0, C2 +1 %, C1 +5 %: the barrier was not what held the waves)
#endif
#ifndef GPK_BLOB_ROUND
#define GPK_BLOB_ROUND 128  // dwords: the table blob's LDS share is rounded to this
#endif
#ifndef GPK_PB_EARLY
#define GPK_PB_EARLY 1  // passes of the dense stream issued before DecodeLayers (0: none), 80-VGPR kernels (A/B r04k: C3 -2.4 %)
#endif
#ifndef GPK_PB_EARLY7
#define GPK_PB_EARLY7 0  // ... in the 72-VGPR kernels (A/B r04k: C4 +0.6 %, C1 +2 % with 1)
#endif
#ifndef GPK_PB_SDEPTH
#define GPK_PB_SDEPTH 4  // sparse phase B: 1 KiB wave loads in flight
#endif
#ifndef GPK_DIAG_NOPARSE
#define GPK_DIAG_NOPARSE 0  // timing only: skip DecodeLayers (fixed layout)
#endif
#ifndef GPK_SB
#define GPK_SB 1  // stream-before-parse small-packet L4 kernel (decode_sb_kernel; A/B r12: C4 -3.6..-4.7 %)
#endif
#ifndef GPK_SB_BIG
#define GPK_SB_BIG 0  // ... for big-packet batches too (C3: +1.2 %, not used)
#endif
#ifndef GPK_SB_WAVES
#define GPK_SB_WAVES GPK_SMALL_WAVES  // ... its register budget (waves per SIMD; LDS allows 6 blocks per CU)
#endif
#ifndef GPK_SBF_WAVES
#define GPK_SBF_WAVES 5  // ... its fused-fields variant (gpk_decode_batch_fields): 96 VGPRs, no scratch (A/B r15,
                         // C4 + fields: 80 VGPRs 44 B of scratch +7.5 %, 72 VGPRs 64 B +10 %)
#endif
#ifndef GPK_SB_DEPTH
#define GPK_SB_DEPTH 6  // ... its stream depth (passes in flight; 8 no better)
#endif
#ifndef GPK_DIAG_TIMES
#define GPK_DIAG_TIMES 0  // diagnostic builds: per-wave phase timestamps into KParams.diag (tools/wave_times.py)
#endif
#ifndef GPK_FIELDS_STAGE
#define GPK_FIELDS_STAGE 2  // fused fields: 1 = half records through LDS (64-byte runs), 2 = whole records (1 KiB runs;
                            // A/B r15 C4 + fields: 6.62 against 7.74 ms)
#endif
#ifndef GPK_FIELDS_TEMPORAL
#define GPK_FIELDS_TEMPORAL 0  // fused fields: record stores with the default policy instead of non-temporal (A/B r15:
                               // +3 % with whole records, -9 % with half records)
#endif
#ifndef GPK_DIAG_FIELDS
#define GPK_DIAG_FIELDS 0  // timing only: 1 = fused fields computed, not stored; 2 = stored, not read
#endif
#ifndef GPK_DIAG_NULLWIN
#define GPK_DIAG_NULLWIN 0  // timing only: the stream-before-parse windows read the L2-resident table copy
#endif
#ifndef GPK_PB_NULL
#define GPK_PB_NULL 0  // timing only: phase-B stream loads read nothing (zero-record descriptors)
#endif

constexpr int kGran = GPK_PB_GRAN;
constexpr uint32_t kGranBytes = 16u * kGran;
constexpr uint32_t kPassBytes = 64u * kGranBytes;
static_assert(kGran == 1 || kGran == 2 || kGran == 4, "granule of 1, 2 or 4 chunks");

// Header-window loads keep the default (temporal) policy: the window's last
// line is re-read by phase B (A/B r01: non-temporal window loads +11-23 %).
__device__ __forceinline__ uint4 ld16(const uint8_t* p) {
  const u32x4 x = *reinterpret_cast<const u32x4*>(p);
  return make_uint4(x.x, x.y, x.z, x.w);
}

// Byte sums with v_dot4_u32_u8: bytes 0,2 (even addresses) and 1,3 (odd).
__device__ __forceinline__ uint32_t dot_even(uint32_t w, uint32_t acc) {
  return __builtin_amdgcn_udot4(w, 0x00010001u, acc, false);
}
__device__ __forceinline__ uint32_t dot_odd(uint32_t w, uint32_t acc) {
  return __builtin_amdgcn_udot4(w, 0x01000100u, acc, false);
}

// Sum of big-endian 16-bit words over LDS bytes [q, q+n) (ComputeChecksum
// with csum = 0, checksum.go:35-50; an odd tail byte counts <<8): unaligned
// dword reads starting at q, so byte q+4k is always a word's high byte; only
// the last dword is masked.
__device__ __forceinline__ uint32_t sum_words_lds(uint32_t q, uint32_t n) {
  uint32_t E = 0, O = 0;
  const uint32_t nd = n >> 2, t = n & 3;
  for (uint32_t k = 0; k < nd; k++) {
    const uint32_t w = lds32u(q + 4 * k);
    E = dot_even(w, E);
    O = dot_odd(w, O);
  }
  if (t) {
    const uint32_t w = lds32u(q + 4 * nd) & (0xffffffffu >> (8 * (4 - t)));
    E = dot_even(w, E);
    O = dot_odd(w, O);
  }
  return (E << 8) + O;
}
// Fixed-length form (IPv4 header without options, pseudo-header addresses).
template <int N>
__device__ __forceinline__ uint32_t sum_words_lds(uint32_t q) {
  static_assert(N % 4 == 0, "whole dwords");
  uint32_t E = 0, O = 0;
#pragma unroll
  for (int k = 0; k < N; k += 4) {
    const uint32_t w = lds32u(q + k);
    E = dot_even(w, E);
    O = dot_odd(w, O);
  }
  return (E << 8) + O;
}

// Same over packet positions [p, p+n), from LDS when inside the window.
__device__ __forceinline__ uint32_t sum_words(const Rd& r, uint32_t p, uint32_t n) {
  if (p + n <= r.win) return sum_words_lds(r.lb + p, n);
  uint32_t s = 0;
  for (uint32_t k = 0; k + 1 < n; k += 2) s += rd16(r, p + k);
  if (n & 1) s += rd8(r, p + n - 1) << 8;
  return s;
}

// Even/odd byte sums of a 16-byte chunk (chunks are 16-byte aligned, so a
// byte's index parity is its address parity).
__device__ __forceinline__ void chunk_eo(const u32x4& v, uint32_t& E, uint32_t& O) {
  E = dot_even(v.x, E);
  O = dot_odd(v.x, O);
  E = dot_even(v.y, E);
  O = dot_odd(v.y, O);
  E = dot_even(v.z, E);
  O = dot_odd(v.z, O);
  E = dot_even(v.w, E);
  O = dot_odd(v.w, O);
}

// Even/odd byte sums of the chunk's bytes [0, n), n in 0..16.
__device__ __forceinline__ void chunk_eo_below(const u32x4& v, uint32_t n, uint32_t& E, uint32_t& O) {
  const uint32_t nl = n < 8 ? n : 8u, nh = n > 8 ? n - 8 : 0u;
  const uint64_t ml = nl >= 8 ? ~0ull : (1ull << (8 * nl)) - 1;
  const uint64_t mh = nh >= 8 ? ~0ull : (1ull << (8 * nh)) - 1;
  const uint32_t w0 = v.x & (uint32_t)ml, w1 = v.y & (uint32_t)(ml >> 32);
  const uint32_t w2 = v.z & (uint32_t)mh, w3 = v.w & (uint32_t)(mh >> 32);
  E = dot_even(w0, E);
  O = dot_odd(w0, O);
  E = dot_even(w1, E);
  O = dot_odd(w1, O);
  E = dot_even(w2, E);
  O = dot_odd(w2, O);
  E = dot_even(w3, E);
  O = dot_odd(w3, O);
}

// The same sums in one word ("L form"): little-endian 16-bit words at even
// addresses, i.e. even-address bytes + 256 * odd-address bytes (v_sad_u16
// against 0 adds a dword's two halves).
__device__ __forceinline__ uint32_t chunk_l(const u32x4& v, uint32_t acc) {
  acc = __builtin_amdgcn_sad_u16(v.x, 0u, acc);
  acc = __builtin_amdgcn_sad_u16(v.y, 0u, acc);
  acc = __builtin_amdgcn_sad_u16(v.z, 0u, acc);
  return __builtin_amdgcn_sad_u16(v.w, 0u, acc);
}
__device__ __forceinline__ uint32_t chunk_l_below(const u32x4& v, uint32_t n, uint32_t acc) {
  const uint32_t nl = n < 8 ? n : 8u, nh = n > 8 ? n - 8 : 0u;
  const uint64_t ml = nl >= 8 ? ~0ull : (1ull << (8 * nl)) - 1;
  const uint64_t mh = nh >= 8 ? ~0ull : (1ull << (8 * nh)) - 1;
  return chunk_l(u32x4{v.x & (uint32_t)ml, v.y & (uint32_t)(ml >> 32), v.z & (uint32_t)mh, v.w & (uint32_t)(mh >> 32)},
                 acc);
}
// An L-form segment sum L (mod 2^32) as ComputeChecksum's word sum of the
// segment (words start at its first byte, checksum.go:35-50):
//  * the segment starts at an odd address: its words are the little-endian
//    words at even addresses, so the word sum is L itself, exactly;
//  * it starts at an even address: the word sum is the byte-swapped sum,
//    congruent to 256 * L mod 65535 (2^16 = 1): swap16(fold(L)) + 65535, a
//    value congruent to the word sum and >= any one word. For segments of at
//    most 64 KiB the word sum does not wrap 2^32, so every later step the
//    caller takes (add the pseudo-header, subtract the checksum field, fold;
//    tcpip.go:54-69) yields the same 16 bits; segment_sums sends waves with a
//    longer segment to the exact per-segment stream.
__device__ __forceinline__ uint32_t l_to_words(uint32_t L, uint32_t odd) {
  if (odd) return L;
  uint32_t f = (L & 0xffffu) + (L >> 16);
  f = (f & 0xffffu) + (f >> 16);
  return ((f & 0xffu) << 8 | f >> 8) + 0xffffu;
}

// 16 bytes of an LDS window chunk (dword-aligned byte address; ~0 = none,
// reads zeros at 0 then).
__device__ __forceinline__ u32x4 lds_chunk(uint32_t a) {
  const uint32_t* p = gpk_smem + ((a == ~0u ? 0u : a) >> 2);
  return u32x4{p[0], p[1], p[2], p[3]};
}

// The parser's compact table blob (P.cg.words dwords) into LDS at byte
// address lds_base by THIS wave alone, by LDS-DMA (global_load_lds_dword:
// lane l's dword lands at M0 + 4 l; no registers held, completion counted by
// vmcnt). Every wave of the block writes the same words to the same
// addresses, so a wave needs only its own copy to have landed (s_waitcnt
// vmcnt) and the block needs no barrier: before, the block's waves waited for
// each other there (in the stream-before-parse kernel after their streams).
// Writes stay inside the blob's LDS share (rounded to GPK_BLOB_ROUND dwords >=
// 64); lanes past the blob re-read its last word.
__device__ __forceinline__ void blob_dma(const KParams& P, uint32_t lds_base, uint32_t lane) {
  const uint32_t words = P.cg.words, last = words - 1;
  const uint64_t src = (uint64_t)(uintptr_t)P.ctab;
  for (uint32_t k = 0; 64 * k < words; k++) {  // wave-uniform trip count
    const uint32_t j = 64 * k + lane;
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src + 4ull * (j < last ? j : last)), "s"(lds_base + 256u * k)
                 : "memory");
  }
}

// A granule: kGran consecutive 16-byte chunks.
struct Gran {
  u32x4 c[kGran];
};
__device__ __forceinline__ void gran_eo(const Gran& g, uint32_t& E, uint32_t& O) {
#pragma unroll
  for (int k = 0; k < kGran; k++) chunk_eo(g.c[k], E, O);
}
// The granule's bytes [0, n), n in 0..kGranBytes-1.
__device__ __forceinline__ void gran_eo_below(const Gran& g, uint32_t n, uint32_t& E, uint32_t& O) {
#pragma unroll
  for (int k = 0; k < kGran; k++) {
    const int m = (int)n - 16 * k;
    chunk_eo_below(g.c[k], m < 0 ? 0u : (m > 16 ? 16u : (uint32_t)m), E, O);
  }
}

// v_readlane_b32 returns int: widen through uint32_t, never through int
// (sign extension of an address's low word above 2 GiB corrupts it).
__device__ __forceinline__ uint32_t readlane32(uint32_t v, uint32_t lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t lane) {
  return ((uint64_t)readlane32((uint32_t)(v >> 32), lane) << 32) | (uint64_t)readlane32((uint32_t)v, lane);
}

// Inclusive prefix sum over the 64 lanes (all active): DPP row_shr 1,2,4,8
// inside each 16-lane row, then row_bcast 15 / 31 across rows.
__device__ __forceinline__ uint32_t wave_scan(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
  return v;
}
// Wave-wide min / max (all lanes active), same pattern; result in every lane
// via readlane 63 (an SGPR).
__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x111, 0xf, 0xf, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x112, 0xf, 0xf, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x114, 0xf, 0xf, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x118, 0xf, 0xf, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x142, 0xa, 0xf, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x143, 0xc, 0xf, false));
  return readlane32(v, 63);
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
  return readlane32(v, 63);
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) { return readlane32(wave_scan(v), 63); }

// Raw-buffer descriptor over [base, base + bytes): loads at offsets >= bytes
// return zeros without touching memory (hardware range check; a load that
// crosses `bytes` returns zeros too, so `bytes` is a multiple of 16).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const uint8_t* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, GPK_PB_NULL ? 0 : bytes, 0x00020000);
}
// streamed (read-once) bytes: non-temporal (A/B r01: -7 % on C3)
__device__ __forceinline__ u32x4 bload(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff) {
  return __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 2);
}

// Header window of one packet in registers: chunks [0, nchunk) of the
// 16-byte-aligned run holding packet bytes [0, win).
template <int W>
struct WinT {
  uint4 v[W];
  uint32_t x;  // AL = 4: the window's 4W+1-th dword (the slot's odd dword)
};
// LDS dwords per lane for a window of W chunks: W * 4 + 1 (the odd stride puts
// lanes reading equal packet positions on distinct banks; AL = 4 uses the odd
// dword as window bytes), except 6-chunk windows: 24 dwords, so a block with
// the table blob (<= 2 KiB) stays within the 26 KiB that 6 blocks per CU allow
// (25 dwords fit 5: tools/probes/occ_probe.hip; A/B r12 C4 -0.7..-3.6 %, C3
// -1 %, profiles/r12_ab_slot24.txt). The 4-chunk kernel fits 8 blocks either way
// and keeps the pad (C2 +4-7 % without it).
#ifndef GPK_SLOT_PAD6
#define GPK_SLOT_PAD6 0
#endif
template <int W, int AL>
constexpr int slot_dw_of() {
  return W * 4 + (AL == 4 ? 1 : (W >= 6 ? GPK_SLOT_PAD6 : 1));
}

struct Idx {
  uint64_t off;
  uint32_t cl;
};

// Branch-free prologue: every lane loads an index entry (lanes past the batch
// re-read the last one) and all W window chunks (chunks past the packet's
// window re-read its last window chunk, which holds a packet byte; a packet
// with no window chunk reads the parser's table copy instead, 16 valid bytes
// that are never used). No exec-mask juggling, one round trip each.
__device__ __forceinline__ Idx load_index(const KParams& P, uint64_t i) {
  const uint64_t j = i < P.n ? i : P.n - 1;
  return Idx{P.offsets[j], P.caplens[j]};
}

// AL: the window's alignment. 16: the run of 16-byte-aligned chunks holding
// the packet's first bytes (window = 16W - (off & 15) bytes, 16W - 15 at
// worst; the slot's odd dword is padding). 4: W 16-byte loads and one dword
// from the packet's own dword, off & ~3 (dword-aligned global_load_dwordx4;
// window = 16W + 4 - (off & 3) >= 16W + 1 bytes, so one chunk fewer covers
// the same headers and the slot shrinks by 16 bytes). A dword-aligned
// 16-byte load can reach into the 16-byte granule after the packet's last
// byte; a lane whose loads would pass the batch's readable end
// (P.data_end, from gpk_batch.data_bytes) takes the aligned run instead.
struct WinGeo {
  uint64_t wb;   // window base: batch offset of LDS slot byte 0 (off - m)
  uint32_t m;    // packet byte 0 at slot byte m
  uint32_t win;  // packet bytes in the window
  uint32_t nch;  // 16-byte loads that hold window bytes (0: inactive lane)
};
template <int W, int AL>
__device__ __forceinline__ WinGeo win_geo(const KParams& P, const Idx& x, bool active) {
  uint32_t m = (uint32_t)(x.off & (AL - 1)), cap = AL == 4 ? W * 16 + 4 : W * 16;
  uint32_t win = x.cl < cap - m ? x.cl : cap - m;
  if (AL == 4 && (x.off & ~3ull) + 16ull * ((m + win + 15) >> 4) > P.data_end) {
    m = (uint32_t)(x.off & 15);
    cap = W * 16;
    win = x.cl < cap - m ? x.cl : cap - m;
  }
  return WinGeo{x.off - m, m, win, active ? (m + win + 15) >> 4 : 0u};
}

typedef u32x4 u32x4_a4 __attribute__((aligned(4)));
template <int W, int AL>
__device__ __forceinline__ void load_window(const KParams& P, const WinGeo& g, WinT<W>& w) {
  const uint32_t nchunk = g.nch;
  const uint8_t* src = nchunk ? P.data + g.wb : reinterpret_cast<const uint8_t*>(P.tab);
  const uint32_t last = nchunk ? nchunk - 1 : 0;
#pragma unroll
  for (int k = 0; k < W; k++) {
    const uint8_t* p = src + 16 * ((uint32_t)k < last ? (uint32_t)k : last);
    if (AL == 16) {
      w.v[k] = ld16(p);
    } else {
      const u32x4 v = *reinterpret_cast<const u32x4_a4*>(p);
      w.v[k] = make_uint4(v.x, v.y, v.z, v.w);
    }
  }
  // the odd dword: bytes [16W, 16W + 4) of the window when it reaches them,
  // else a dword of the last chunk (valid memory, never used)
  if (AL == 4) w.x = *reinterpret_cast<const uint32_t*>(src + (nchunk > W ? 16u * W : 16u * last));
}

template <int W, int AL>
__device__ __forceinline__ void store_window(uint32_t slot_dw, const WinT<W>& w) {
#pragma unroll
  for (int k = 0; k < W; k++) {
    gpk_smem[slot_dw + 4 * k + 0] = w.v[k].x;
    gpk_smem[slot_dw + 4 * k + 1] = w.v[k].y;
    gpk_smem[slot_dw + 4 * k + 2] = w.v[k].z;
    gpk_smem[slot_dw + 4 * k + 3] = w.v[k].w;
  }
  if (AL == 4) gpk_smem[slot_dw + 4 * W] = w.x;
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

// ---- Phase B ---------------------------------------------------------------
// Each lane with a job holds its segment [s, e) as batch byte offsets; the
// result is the segment's word sum with words starting at s (mod 2^32).

// Dense: the wave's segments lie in [R0, R0 + R) (R0 16-byte aligned). The
// region is cut into granules (16 bytes), lane l of pass p holds granule
// 64p + l. P(g) = L-form sum (chunk_l) of granules [0, g], a wave-wide running
// prefix. Segment sum over granules [gs, ge) = P(ge-1) - P(gs-1), corrected by
// the head granule's bytes before s and the tail granule's bytes before e
// (from the LDS header windows, else loaded), then turned into the word sum
// of the segment's own alignment (l_to_words).
// One pass of the dense stream into a granule slot: kGran raw-buffer loads
// (16 bytes per lane each, consecutive lanes -> consecutive granules)
// written in place ("+v": the slot keeps its registers across the loop, so
// the stream needs no register rotation and no drain at the loop edge).
// Issued as inline asm, which the compiler's wait-count pass does not see:
// dense_segment_sums waits for the slots itself (slot_wait). The register
// allocator believes the asm wrote the slot at once and could copy or spill
// it while the load is in flight; every build's device code is therefore
// checked for that (tools/check_stream_isa.py, run by the Makefile).
#ifndef GPK_STREAM_NT
#define GPK_STREAM_NT 1  // phase-B stream loads non-temporal
#endif
#if GPK_STREAM_NT
#define GPK_SPOL " nt"
#else
#define GPK_SPOL ""
#endif
__device__ __forceinline__ void slot_load(u32x4 (&c)[kGran], __amdgpu_buffer_rsrc_t rs, uint32_t vo,
                                          uint32_t soff) {
  asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" GPK_SPOL : "+v"(c[0]) : "v"(vo), "s"(rs), "s"(soff) : "memory");
  if (kGran > 1)
    asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen offset:16" GPK_SPOL
                 : "+v"(c[kGran > 1 ? 1 : 0]) : "v"(vo), "s"(rs), "s"(soff) : "memory");
  if (kGran > 2) {
    asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen offset:32" GPK_SPOL
                 : "+v"(c[kGran > 2 ? 2 : 0]) : "v"(vo), "s"(rs), "s"(soff) : "memory");
    asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen offset:48" GPK_SPOL
                 : "+v"(c[kGran > 3 ? 3 : 0]) : "v"(vo), "s"(rs), "s"(soff) : "memory");
  }
}
// All but the youngest N vector-memory loads of this wave have completed.
// The slot's registers are operands, so no use of them moves above the wait.
template <int N>
__device__ __forceinline__ void slot_wait(u32x4 (&c)[kGran]) {
  if (kGran == 1)
    asm volatile("s_waitcnt vmcnt(%1)" : "+v"(c[0]) : "n"(N) : "memory");
  else if (kGran == 2)
    asm volatile("s_waitcnt vmcnt(%2)" : "+v"(c[0]), "+v"(c[kGran > 1 ? 1 : 0]) : "n"(N) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(%4)"
                 : "+v"(c[0]), "+v"(c[kGran > 1 ? 1 : 0]), "+v"(c[kGran > 2 ? 2 : 0]), "+v"(c[kGran > 3 ? 3 : 0])
                 : "n"(N)
                 : "memory");
}

// slot_wait with a count known after unrolling (the tail's per-slot counts)
__device__ __forceinline__ void slot_wait_n(u32x4 (&c)[kGran], int n) {
  static_assert(kGran == 1, "counts in loads");
  switch (n) {
    case 0: slot_wait<0>(c); break;
    case 1: slot_wait<1>(c); break;
    case 2: slot_wait<2>(c); break;
    case 3: slot_wait<3>(c); break;
    case 4: slot_wait<4>(c); break;
    case 5: slot_wait<5>(c); break;
    case 6: slot_wait<6>(c); break;
    case 7: slot_wait<7>(c); break;
    case 8: slot_wait<8>(c); break;
    case 9: slot_wait<9>(c); break;
    case 10: slot_wait<10>(c); break;
    default: slot_wait<0>(c); break;  // deeper rings: wait for everything
  }
}

// The dense stream of one wave: region [R0, R0 + R) (R0 16-byte aligned),
// D passes in flight in fixed slot registers. Started early (stream_start,
// before DecodeLayers, from the packet extents) when the wave's packets are
// packed, so the first D KiB arrive while the headers are parsed.
template <int D>
struct Stream {
  Gran ring[D];
  uint64_t R0;
  uint32_t R;
  bool on;
};

// Issue passes [d0, d1) of the stream over [R0, R0 + R) into their slots.
template <int D>
__device__ __forceinline__ void stream_issue(const KParams& P, Stream<D>& S, uint64_t R0, uint32_t R, uint32_t lane,
                                             int d0, int d1) {
  S.R0 = R0;
  S.R = R;
  // whole 16-byte chunks: the range check zeroes a 16-byte load that
  // crosses the record limit, not just its bytes past it
  const __amdgpu_buffer_rsrc_t rs = rsrc(P.data + R0, (R + 15) & ~15u);
#pragma unroll
  for (int d = 0; d < D; d++) {
    if (d < d0 || d >= d1) continue;
#pragma unroll
    for (int k = 0; k < kGran; k++) S.ring[d].c[k] = u32x4{0, 0, 0, 0};
    slot_load(S.ring[d].c, rs, lane * kGranBytes, d * kPassBytes);
  }
}

// Whether the byte ranges [s, e) of the lanes with `job` lie in one compact
// region (at most 4 x their total + 8 KiB, within +-2 GiB of a wave-uniform
// base, none over 64 KiB: l_to_words); returns it as R0 / R.
__device__ __forceinline__ bool dense_region(bool job, uint64_t s, uint64_t e, uint64_t& R0, uint32_t& R) {
  const uint64_t jobs = __ballot(job);
  if (!jobs) return false;
  // relative to a wave-uniform base (the first job lane's chunk), in 32-bit
  // biased coordinates
  const uint64_t B = readlane64(s, (uint32_t)__builtin_ctzll(jobs)) & ~15ull;
  constexpr uint64_t kBias = 0x80000000ull;
  const uint64_t bs = s + kBias - B, be = e + kBias - B;
  const bool far = job && (bs >> 32 || be >> 32 || e - s > 65536u);
  const uint32_t lo = wave_min(job ? (uint32_t)bs : 0xffffffffu);
  const uint32_t hi = wave_max(job ? (uint32_t)be : 0u);
  const uint32_t tot = wave_sum(job ? (uint32_t)(e - s) : 0u);
  const uint32_t lo16 = lo & ~15u;
  R0 = B + lo16 - kBias;
  R = hi - lo16;
  return !__ballot(far) && hi - lo16 <= 4u * tot + 8192u;
}

// Early start: the packets of the wave (not yet parsed) as the region; the
// first E passes are issued now (their slot registers stay live through
// DecodeLayers, so only a few: tools/check_stream_isa.py rejects a build
// whose register allocation touches them), the rest when phase B begins.
// The passes are issued on every path, over an empty region (range-checked
// zeros, no memory access) when the wave's packets are not packed, and
// segment_sums drains them first on every path: no later branch has to know
// whether they were issued.
template <int D, int E>
__device__ __forceinline__ void stream_start(const KParams& P, Stream<D>& S, bool active, uint64_t off, uint32_t cl,
                                             uint32_t lane) {
  uint64_t R0;
  uint32_t R;
  S.on = dense_region(active, off, off + cl, R0, R);
  if (!S.on) {
    R0 = 0;
    R = 0;
  }
  stream_issue(P, S, R0, R, lane, 0, E < D ? E : D);
}

// All stream loads of the wave have landed (the slot registers are free).
template <int D>
__device__ __forceinline__ void stream_drain(Stream<D>& S) {
#pragma unroll
  for (int d = 0; d < D; d++) slot_wait<0>(S.ring[d].c);
}

// tafter: tlds holds the bytes of the granule of e from e on (the next
// packet's first bytes, in the next lane's window; the bytes before e in that
// chunk are not the granule's): the segment then takes P(ge) minus them
// instead of P(ge - 1) plus the bytes before e.
// The head / tail part of a dense segment sum (issued before the stream: the
// head and tail chunks come from the LDS header windows when a window holds
// them, hlds / tlds = LDS byte address, else ~0, else from memory). Returns the
// correction L; ta: the granule of e is streamed and P(ge) is taken.
__device__ __forceinline__ uint32_t dense_head_tail(const KParams& P, uint64_t R0, uint32_t R, bool job, uint64_t s,
                                                    uint64_t e, uint32_t hlds, uint32_t tlds, bool tafter, bool& ta) {
  static_assert(kGran == 1, "head/tail chunks from the LDS window need 16-byte granules");
  const __amdgpu_buffer_rsrc_t rs = rsrc(P.data + R0, (R + 15) & ~15u);
  const uint32_t rsl = job ? (uint32_t)(s - R0) : 0u, rel = job ? (uint32_t)(e - R0) : 0u;
  ta = tafter && rel < R;  // the granule of e is streamed: P(ge) exists
  u32x4 hc = lds_chunk(hlds), tc = lds_chunk(tlds);
  if (hlds == ~0u) hc = __builtin_amdgcn_raw_buffer_load_b128(rs, rsl & ~15u, 0, 0);
  if (tlds == ~0u || (tafter && !ta)) tc = __builtin_amdgcn_raw_buffer_load_b128(rs, rel & ~15u, 0, 0);
  return chunk_l_below(tc, rel & 15u, 0u) - (ta ? chunk_l(tc, 0u) : 0u) - chunk_l_below(hc, rsl & 15u, 0u);
}

template <int D>
__device__ __forceinline__ uint32_t dense_segment_sums(const KParams& P, Stream<D>& S, bool job, uint64_t s,
                                                       uint64_t e, uint32_t lane, uint32_t L, bool ta) {
  const uint64_t R0 = S.R0;
  const uint32_t R = S.R;
  const __amdgpu_buffer_rsrc_t rs = rsrc(P.data + R0, (R + 15) & ~15u);
  const uint32_t rsl = job ? (uint32_t)(s - R0) : 0u, rel = job ? (uint32_t)(e - R0) : 0u;
  const uint32_t np = (R + kPassBytes - 1) / kPassBytes;  // wave-uniform
  const uint32_t vo = lane * kGranBytes;
  Gran (&ring)[D] = S.ring;
  const int32_t a = (int32_t)(rsl / kGranBytes) - 1, b = (int32_t)(rel / kGranBytes) - (ta ? 0 : 1);
  const int32_t pa = a >> 6, pb = b >> 6;  // -1 never matches
  const int32_t la = (a & 63) << 2, lb = (b & 63) << 2, ll = (int32_t)lane << 2;
  uint32_t xa = 0, xb = 0, c = 0;
  // One pass: slot d holds pass p; refill it with pass p + D when asked.
  auto pass = [&](const int d, const int32_t p, const bool refill) __attribute__((always_inline)) {
    const uint32_t g = chunk_l(ring[d].c[0], 0u);
    if (refill) slot_load(ring[d].c, rs, vo, (uint32_t)(p + D) * kPassBytes);
    const uint32_t sc = wave_scan(g);
    const uint32_t Pf = sc + c;
    const bool ma = pa == p, mb = pb == p;
    const uint32_t ya = (uint32_t)__builtin_amdgcn_ds_bpermute(GPK_PB_IDPERM ? (ma ? la : ll) : la, (int)Pf);
    const uint32_t yb = (uint32_t)__builtin_amdgcn_ds_bpermute(GPK_PB_IDPERM ? (mb ? lb : ll) : lb, (int)Pf);
    xa = ma ? ya : xa;
    xb = mb ? yb : xb;
    c += readlane32(sc, 63);
  };
  // Whole rounds of D passes, no branch inside; each slot is consumed, then
  // refilled at once (refills past the region read range-checked zeros).
  uint32_t p0 = 0;
  for (; p0 + D <= np; p0 += D) {
#pragma unroll
    for (int d = 0; d < D; d++) {
      slot_wait<(D - 1) * kGran>(ring[d].c);  // slot d's loads are the oldest in flight
      pass(d, (int32_t)(p0 + d), true);
    }
  }
  // The last np - p0 < D passes are in flight already: no refills, so slot
  // d waits for all but the D-1-d younger slots.
#pragma unroll
  for (int d = 0; d < D - 1; d++) {
    if (p0 + d >= np) break;
    slot_wait_n(ring[d].c, D - 1 - d);
    pass(d, (int32_t)(p0 + d), false);
  }
  L += xb - xa;
  stream_drain(S);  // the last refills land before the registers are reused
  return l_to_words(L, (uint32_t)s & 1u);
}

// Sparse: the segments one after another as whole-wave 1 KiB loads (16 bytes
// per lane, consecutive lanes -> consecutive chunks), GPK_PB_SDEPTH always in
// flight; at a segment's last load its even/odd sums are reduced across the
// wave into the owning lane. Each segment is streamed over whole chunks
// [s & ~15, e & ~15); its partial first and last chunks are the lane's own.
__device__ __forceinline__ uint32_t sparse_segment_sums(const KParams& P, bool job, uint64_t s, uint64_t e,
                                                        uint32_t lane) {
  const uint64_t fa = s & ~15ull, fe = e & ~15ull;
  u32x4 hc = {0, 0, 0, 0}, tc = {0, 0, 0, 0};
  if (job) hc = *reinterpret_cast<const u32x4*>(P.data + fa);
  if (job && (e & 15)) tc = *reinterpret_cast<const u32x4*>(P.data + fe);
  uint32_t E = 0, O = 0;
  chunk_eo_below(tc, (uint32_t)(e & 15), E, O);
  uint32_t hE = 0, hO = 0;
  chunk_eo_below(hc, (uint32_t)(s & 15), hE, hO);
  E -= hE;
  O -= hO;
  uint32_t own = (s & 1) ? (O << 8) + E : (E << 8) + O;
  uint64_t pend = __ballot(job && fe > fa);
  const uint32_t vo = lane * 16;
  constexpr int D = GPK_PB_SDEPTH;
  uint32_t p_lane = 64, p_off = 0, p_len = 0;  // producer (wave-uniform)
  __amdgpu_buffer_rsrc_t p_rs = rsrc(P.data, 0);
  u32x4 ring[D];
  uint32_t r_lane[D], r_last[D];
  const uint32_t par = (uint32_t)(s & 1);
#pragma unroll
  for (int k = 0; k < D; k++) {
    if (p_off >= p_len) {
      p_lane = 64;
      p_off = p_len = 0;
      uint64_t b0 = 0;
      if (pend) {
        p_lane = (uint32_t)__builtin_ctzll(pend);
        pend &= pend - 1;
        b0 = readlane64(fa, p_lane);
        p_len = (uint32_t)(readlane64(fe, p_lane) - b0);
      }
      p_rs = rsrc(P.data + b0, p_len);
    }
    ring[k] = bload(p_rs, vo, p_off);
    r_lane[k] = p_lane;
    r_last[k] = p_off + 1024 >= p_len;
    p_off += 1024;
  }
  uint32_t sE = 0, sO = 0;
  for (;;) {
    uint32_t live = 0;
#pragma unroll
    for (int k = 0; k < D; k++) {
      if (r_lane[k] < 64) {
        chunk_eo(ring[k], sE, sO);
        if (r_last[k]) {
          const uint32_t pr = readlane32(par, r_lane[k]);
          const uint32_t t = wave_sum(pr ? (sO << 8) + sE : (sE << 8) + sO);
          if (lane == r_lane[k]) own += t;
          sE = sO = 0;
        }
      }
      if (p_off >= p_len) {
        p_lane = 64;
        p_off = p_len = 0;
        uint64_t b0 = 0;
        if (pend) {
          p_lane = (uint32_t)__builtin_ctzll(pend);
          pend &= pend - 1;
          b0 = readlane64(fa, p_lane);
          p_len = (uint32_t)(readlane64(fe, p_lane) - b0);
        }
        p_rs = rsrc(P.data + b0, p_len);
      }
      ring[k] = bload(p_rs, vo, p_off);
      r_lane[k] = p_lane;
      r_last[k] = p_off + 1024 >= p_len;
      p_off += 1024;
      live |= r_lane[k] < 64;
    }
    if (!live) break;
  }
  return own;
}

// Word sums of every job lane's segment [s, e): the dense prefix stream (the
// one started early, else one over the segments' region when that is
// compact), else the per-segment stream.
template <int D, int E>
__device__ __forceinline__ uint32_t segment_sums(const KParams& P, Stream<D>& S, bool job, uint64_t s, uint64_t e,
                                                 uint32_t lane, uint32_t hlds, uint32_t tlds, bool tafter) {
  bool ta = false;
  // The early passes (E > 0: issued on every path) have landed during the
  // parse; waiting for them here (their registers as operands) puts any
  // register copy the allocator needs between the early slots and the loop's
  // after the data is in.
  if (E > 0) stream_drain(S);
  if (E > 0 && S.on) {
    if (!__ballot(job)) return 0;  // nothing to sum
    const uint32_t L = dense_head_tail(P, S.R0, S.R, job, s, e, hlds, tlds, tafter, ta);
    stream_issue(P, S, S.R0, S.R, lane, E < D ? E : D, D);
    return dense_segment_sums<D>(P, S, job, s, e, lane, L, ta);
  }
  // (with the early start on, a wave whose packets are not packed goes to
  // the per-segment stream: one call site keeps the slot registers in place)
  uint64_t R0;
  uint32_t R;
  if (E == 0 && dense_region(job, s, e, R0, R)) {
    const uint32_t L = dense_head_tail(P, R0, R, job, s, e, hlds, tlds, tafter, ta);
    stream_issue(P, S, R0, R, lane, 0, D);
    return dense_segment_sums<D>(P, S, job, s, e, lane, L, ta);
  }
  if (!__ballot(job)) return 0;
  return sparse_segment_sums(P, job, s, e, lane);
}

// ---- Stream before the parse (decode_sb_kernel) ---------------------------
// For waves of packed small packets phase B's stream runs before the parse,
// over the packets' extents, and captures per lane the L-form prefix just
// before its packet's first granule and at its last granule; after the parse
// the segment's sum is that packet sum minus the bytes before s and after e,
// which lie in the header windows (or come from memory).
struct SbPkt {
  uint32_t L;   // L-form sum of the packet's granules [a, b]
  uint64_t R0;  // region base (batch offset, 16-byte aligned)
  int32_t b;    // the packet's last granule (region-relative)
  bool on;      // wave-uniform: the wave ran stream-first (else windows loaded, phase B after the parse)
};

// The stream of a stream-before-parse wave: region [R0, R0 + R), D passes in
// flight (the dense stream's slots and waits); returns P(b) - P(a1) for the
// lane's packet (a1 = -1: none before it).
template <int D>
__device__ __forceinline__ uint32_t sb_stream(const KParams& P, Stream<D>& S, uint64_t R0, uint32_t R, uint32_t lane,
                                              int32_t a1, int32_t b) {
  static_assert(kGran == 1, "one 16-byte granule per lane per pass");
  stream_issue(P, S, R0, R, lane, 0, D);
  const __amdgpu_buffer_rsrc_t rs = rsrc(P.data + R0, (R + 15) & ~15u);
  const uint32_t np = (R + kPassBytes - 1) / kPassBytes;  // wave-uniform
  const uint32_t vo = lane * kGranBytes;
  Gran (&ring)[D] = S.ring;
  const int32_t pa = a1 >> 6, pb = b >> 6;  // -1 never matches
  const int32_t la = (a1 & 63) << 2, lb = (b & 63) << 2, ll = (int32_t)lane << 2;
  uint32_t xa = 0, xb = 0, c = 0;
  auto pass = [&](const int d, const int32_t p, const bool refill) __attribute__((always_inline)) {
    const uint32_t gl = chunk_l(ring[d].c[0], 0u);
    if (refill) slot_load(ring[d].c, rs, vo, (uint32_t)(p + D) * kPassBytes);
    const uint32_t sc = wave_scan(gl);
    const uint32_t Pf = sc + c;
    const bool ma = pa == p, mb = pb == p;
    const uint32_t ya = (uint32_t)__builtin_amdgcn_ds_bpermute(ma ? la : ll, (int)Pf);
    const uint32_t yb = (uint32_t)__builtin_amdgcn_ds_bpermute(mb ? lb : ll, (int)Pf);
    xa = ma ? ya : xa;
    xb = mb ? yb : xb;
    c += readlane32(sc, 63);
  };
  // The first round runs on every path (passes past the region read
  // range-checked zeros and add nothing): no edge bypasses the loop, so the slot registers the passes were
  // issued into are the loop's own (a bypass made the allocator copy them
  // while in flight: tools/check_stream_isa.py).
  uint32_t p0 = 0;
  do {
#pragma unroll
    for (int d = 0; d < D; d++) {
      slot_wait<(D - 1) * kGran>(ring[d].c);
      pass(d, (int32_t)(p0 + d), true);
    }
    p0 += D;
  } while (p0 + D <= np);
#pragma unroll
  for (int d = 0; d < D - 1; d++) {
    if (p0 + d >= np) break;
    slot_wait_n(ring[d].c, D - 1 - d);
    pass(d, (int32_t)(p0 + d), false);
  }
  stream_drain(S);
  return xb - xa;
}

// 16 bytes of the batch at granule address ga (16-byte aligned) for a
// stream-before-parse lane: its own window chunk, the next packet's first chunk, or
// memory.
__device__ __forceinline__ u32x4 sb_chunk(const KParams& P, uint64_t ga, uint64_t wb, uint32_t nch, uint32_t slot_dw,
                                          bool next_here, uint64_t nwb, uint32_t stride) {
  const uint64_t k = (ga - wb) >> 4;
  if (ga >= wb && k < nch) return lds_chunk(slot_dw * 4 + 16u * (uint32_t)k);
  if (next_here && ga == nwb) return lds_chunk((slot_dw + stride) * 4);
  return *reinterpret_cast<const u32x4*>(P.data + ga);
}

// ---- Fused layer fields (gpk_decode_batch_fields) ---------------------------
// The header reader gpk_fields.h expects, over the lane's LDS window (bytes
// past it from memory, byte by byte: a field never reads past its own bytes).
struct RdF {
  Rd r;
  __device__ __forceinline__ uint32_t u8(uint32_t p) const { return rd8(r, p); }
  __device__ __forceinline__ uint32_t be16(uint32_t p) const { return rd16(r, p); }
  __device__ __forceinline__ uint32_t u32(uint32_t p) const {
    if (p + 4 <= r.win) return lds32u(r.lb + p);
    return rd8(r, p) | rd8(r, p + 1) << 8 | rd8(r, p + 2) << 16 | rd8(r, p + 3) << 24;
  }
};

// The wave's 64 records of 128 bytes out as coalesced stores, staged through
// the wave's LDS window slots (>= 4 KiB) in two halves: lane l puts the 64
// bytes of its record's half into LDS (16-byte chunk c at chunk position
// c ^ (l & 3), spreading the banks), then store k of the half writes records
// 16k .. 16k+15, lane l carrying chunk l & 3 of record 16k + l / 4 (16 runs of
// 64 contiguous bytes per instruction; the halves meet in L2). Runs with the
// whole wave active, after every lane's last window read (LDS operations of a
// wave complete in order; the compiler barriers keep them in program order).
__device__ __forceinline__ void fields_store(const KParams& P, const uint32_t (&w)[32], uint32_t wave_dw, uint32_t lane,
                                             uint64_t first) {
  u32x4* out = reinterpret_cast<u32x4*>(P.fields + first);
#if GPK_FIELDS_STAGE == 2
  // whole records: lanes [48g, 48g + 48) put theirs into the 6 KiB (chunk c at
  // c ^ (l & 7)), then 1 KiB stores of 8 whole records each
#pragma unroll
  for (uint32_t g = 0; g < 2; g++) {
    const uint32_t l0 = 48 * g, nrec = g ? 16u : 48u;
    asm volatile("" ::: "memory");
    if (lane >= l0 && lane < l0 + nrec) {
      const uint32_t q = lane - l0;
#pragma unroll
      for (uint32_t c = 0; c < 8; c++)
        *reinterpret_cast<u32x4*>(gpk_smem + wave_dw + q * 32 + 4 * (c ^ (q & 7))) =
            u32x4{w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]};
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (uint32_t k = 0; k < 6; k++) {
      if (g && k >= 2) break;
      const uint32_t q = 8 * k + (lane >> 3), c = lane & 7, rr = l0 + q;
      const u32x4 v = *reinterpret_cast<const u32x4*>(gpk_smem + wave_dw + q * 32 + 4 * (c ^ (q & 7)));
      if (first + rr < P.n) {
        if (GPK_FIELDS_TEMPORAL)
          out[8 * rr + c] = v;
        else
          __builtin_nontemporal_store(v, out + 8 * rr + c);
      }
    }
  }
  asm volatile("" ::: "memory");
  return;
#endif
#pragma unroll
  for (int h = 0; h < 2; h++) {
    asm volatile("" ::: "memory");
#pragma unroll
    for (uint32_t c = 0; c < 4; c++)
      *reinterpret_cast<u32x4*>(gpk_smem + wave_dw + lane * 16 + 4 * (c ^ (lane & 3))) =
          u32x4{w[16 * h + 4 * c], w[16 * h + 4 * c + 1], w[16 * h + 4 * c + 2], w[16 * h + 4 * c + 3]};
    asm volatile("" ::: "memory");
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
      const uint32_t rr = 16 * k + (lane >> 2), c = lane & 3;
      const u32x4 v = *reinterpret_cast<const u32x4*>(gpk_smem + wave_dw + rr * 16 + 4 * (c ^ (rr & 3)));
      if (first + rr < P.n) {
        if (GPK_FIELDS_TEMPORAL)
          out[8 * rr + 4 * h + c] = v;
        else
          __builtin_nontemporal_store(v, out + 8 * rr + 4 * h + c);
      }
    }
  }
  asm volatile("" ::: "memory");
}

template <bool kL4, bool kLayout, class TT, bool kKeys, int W, int O, int AL, int kSlotStride = slot_dw_of<W, AL>(),
          int kEarly = -1, bool kSB = false, bool kFields = false>
__device__ __forceinline__ void decode_packet(const KParams& P, const TT& T, uint64_t i, bool active, uint64_t off,
                                              uint32_t cl, const WinGeo& g, uint32_t slot_dw, uint32_t lane,
                                              uint64_t* dt, const SbPkt sb = SbPkt{0, 0, -1, false}) {
  const uint32_t m = g.m, win = g.win;
  Rd r{P.data + off, slot_dw * 4 + m, win};

  // Phase B's stream over the wave's packets starts now when they are packed:
  // its first D KiB load while the headers are parsed.
  // (layouts: fewer registers left; the stream-before-parse kernel's phase B after the parse is its fallback)
  constexpr int D = kLayout ? 4 : (kSB ? (kFields ? GPK_PB_DEPTHF : GPK_PB_DEPTH7SB) : (O > 6 ? GPK_PB_DEPTH7 : GPK_PB_DEPTH));
  // early passes: as many as the kernel's register budget carries through
  // DecodeLayers untouched (tools/check_stream_isa.py)
  constexpr int E = kEarly >= 0 ? kEarly : ((kLayout || kKeys) ? 0 : (O > 6 ? GPK_PB_EARLY7 : GPK_PB_EARLY));
  Stream<D> S;
  S.on = false;
  if (kL4 && E > 0) stream_start<D, E>(P, S, active && (P.outputs & GPK_OUT_L4_CSUM), off, cl, lane);

  // ---- Phase A: DecodeLayers ------------------------------------------------
  Parse q;
  q.init();
  Outcome s{0, 0, 0, 0};
  bool done = false;
#if GPK_DIAG_NOPARSE  // timing only: a fixed Eth/IPv4/UDP|TCP layout, no decoding
  if (active) {
    q.s_eth = 0;
    q.e_eth = cl;
    q.s_ip4 = 14;
    q.e_ip4 = cl;
    q.last_net = GPK_DEC_IPV4;
    q.transport = lds8(r.lb + 23) == 6 ? GPK_DEC_TCP : GPK_DEC_UDP;
    q.s_tcp = q.s_udp = 34;
    q.e_tcp = q.e_udp = cl;
    q.udp_hlen = cl - 34;
    q.layers = 0x931;
    q.nlayers = 3;
  }
  (void)done;
#else
  if (active && P.fast) done = fast_parser(P, T, r, cl, q, s);
  if (active && !done) s = run_parser<false>(P, T, r, cl, q);
#endif

  // fused fields: the decoders' last slices in compact form (presence, the
  // starts the fields read, the IPv4 end), live to the fields epilogue instead
  // of the whole parse state
  uint32_t fpres = 0, fip4e = 0;
  uint32_t fst[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (kFields && active) {
    const int slot_kind[8] = {GPK_DEC_ETHERNET, GPK_DEC_DOT1Q, GPK_DEC_IPV4, GPK_DEC_IPV6,
                              GPK_DEC_IPV6_EXT, GPK_DEC_TCP,   GPK_DEC_UDP,  GPK_DEC_PAYLOAD};
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int kd = k == 7 && !clean(q, GPK_DEC_PAYLOAD) ? GPK_DEC_FRAGMENT : slot_kind[k];
      fpres |= clean(q, kd) ? 1u << k : 0u;
      if (k != 4 && k != 7) fst[k] = q.start(kd);
    }
    fip4e = q.end(GPK_DEC_IPV4);
  }
  uint32_t st = (s.err & GPK_ST_ERR_MASK) | (s.trunc ? GPK_ST_TRUNCATED : 0u) |
                ((q.nlayers > GPK_ST_NLAYERS_MASK ? GPK_ST_NLAYERS_MASK : q.nlayers) << GPK_ST_NLAYERS_SHIFT);
  uint32_t ip4c = 0, l4c = 0;

  // L4 checksum job: segment [js, je) of the batch, pseudo-header sum jinit
  uint64_t js = 0, je = 0;
  uint32_t jinit = 0, jexist = 0;
  bool job = false;

  if (active) {
    if ((P.outputs & GPK_OUT_IP4_CSUM) && clean(q, GPK_DEC_IPV4)) {  // ip4.go:323-332
      uint32_t s4 = q.start(GPK_DEC_IPV4);
      uint32_t hl = (rd8(r, s4) & 15) * 4;
      uint32_t existing = rd16(r, s4 + 10);
      const uint32_t sum = hl == 20 && s4 + 20 <= win ? sum_words_lds<20>(r.lb + s4) : sum_words(r, s4, hl);
      ip4c = fold(sum - existing);
      st |= GPK_ST_IP4_CSUM | (ip4c == existing ? GPK_ST_IP4_VALID : 0u);
    }
    const uint32_t tk = q.transport, nk = q.last_net;
    if (kL4 && (P.outputs & GPK_OUT_L4_CSUM) && tk && clean(q, tk) && nk && clean(q, nk)) {
      // tcp.go:626-640 / udp.go:144-158 via tcpip.go:54-69: bytes = Contents
      // + Payload as decoded, csum = pseudo-header + proto + length
      const uint32_t t0 = q.start(tk);
      const uint32_t blen = tk == GPK_DEC_TCP ? q.end(tk) - t0 : q.udp_hlen;
      const uint32_t ns = q.start(nk);
      uint32_t init;
      if (nk == GPK_DEC_IPV4)
        init = ns + 20 <= win ? sum_words_lds<8>(r.lb + ns + 12) : sum_words(r, ns + 12, 8);
      else
        init = ns + 40 <= win ? sum_words_lds<32>(r.lb + ns + 8) : sum_words(r, ns + 8, 32);
      init += (tk == GPK_DEC_TCP ? 6u : 17u) + (blen & 0xffff) + (blen >> 16);
      jinit = init;
      jexist = rd16(r, t0 + (tk == GPK_DEC_TCP ? 16 : 6));
      st |= GPK_ST_L4_CSUM | (tk == GPK_DEC_UDP ? GPK_ST_L4_UDP : 0u);
      js = off + t0;
      je = js + blen;
      job = true;
    }
    if (P.outputs & GPK_OUT_FLOWS) {
      const bool fl = clean(q, GPK_DEC_ETHERNET), fn = nk && clean(q, nk), ft = tk && clean(q, tk);
      uint64_t lflow, nflow, tflow;
      flow_hashes(r, fl, fl ? q.start(GPK_DEC_ETHERNET) : 0u, fn, fn ? q.start(nk) : 0u, nk == GPK_DEC_IPV6, ft,
                  ft ? q.start(tk) : 0u, tk == GPK_DEC_TCP ? 4u : 5u, lflow, nflow, tflow);
      lflow = fl ? lflow : 0;
      nflow = fn ? nflow : 0;
      tflow = ft ? tflow : 0;
      st |= (fl ? GPK_ST_LINK_FLOW : 0u) | (fn ? GPK_ST_NET_FLOW : 0u) |
            (fn && nk == GPK_DEC_IPV6 ? GPK_ST_NET_IPV6 : 0u) | (ft ? GPK_ST_TRANSPORT_FLOW : 0u);
      if (P.flows) {
        __builtin_nontemporal_store(lflow, P.flows + i);
        __builtin_nontemporal_store(nflow, P.flows + P.n + i);
        __builtin_nontemporal_store(tflow, P.flows + 2 * P.n + i);
      }
    }
  }

  // ---- outputs that do not wait for phase B (their registers die here) ------
  if (active) {
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
                                GPK_DEC_IPV6_EXT, GPK_DEC_TCP,   GPK_DEC_UDP,  GPK_DEC_PAYLOAD};
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
  const uint32_t lay_lo = (uint32_t)q.layers, lay_hi = (uint32_t)(q.layers >> 32);

  // Fused layer fields (gpk_decode_batch_fields): the fields of the decoders'
  // last slices (gpk_fields.h) read from this lane's header window, then the
  // wave's records staged through its window slots. Called once the windows
  // are no longer needed (after the stream-before-parse correction; before the
  // phase-B stream of a wave that takes it after the parse, whose head/tail
  // chunks then come from memory): the window reads and the stream's slots
  // never hold registers at the same time.
  auto emit_fields = [&]() __attribute__((always_inline)) {
    uint32_t fw[32];
#if GPK_DIAG_FIELDS == 2  // timing only: the stores without the field reads
#pragma unroll
    for (int k = 0; k < 32; k++) fw[k] = fst[k & 7] + fpres * k;
#else
    gpkf::fields_words(RdF{r}, fpres, fst, fip4e, fw);
#endif
#if GPK_DIAG_FIELDS == 1  // timing only: the field reads without the record stores
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 32; k++) x ^= fw[k];
    if (x == 0x9E3779B9u) P.fields[i].present = x;
#else
    fields_store(P, fw, slot_dw - lane * kSlotStride, lane, i - lane);
#endif
  };

  // ---- Phase B: segment sums ---------------------------------------------
#if GPK_DIAG_TIMES
  dt[3] = __builtin_amdgcn_s_memrealtime();
#endif
  if (kL4 && kSB && sb.on) {
    // stream before the parse: the packet's granule sum minus the bytes of its
    // granules before s (header bytes, in the window) and from e on (padding
    // and the next packet's first bytes)
    const uint32_t nch = active ? (m + win + 15) >> 4 : 0u;
    const uint32_t nwb_lo = (uint32_t)__shfl_down((int)(uint32_t)g.wb, 1);
    const uint32_t nwb_hi = (uint32_t)__shfl_down((int)(uint32_t)(g.wb >> 32), 1);
    const uint32_t nnch = (uint32_t)__shfl_down((int)nch, 1);
    const uint64_t nwb = (uint64_t)nwb_hi << 32 | nwb_lo;
    const bool next_here = lane < 63 && nnch != 0;
    uint32_t L = sb.L;
    if (job) {
      // header bytes [wb, js): whole window chunks below the chunk of js and
      // its bytes before js, from LDS; headers past the window (the general
      // decoder's long ones) from memory
      const uint32_t hl = (uint32_t)(js - g.wb), hk = hl >> 4;
      if (hl < 16u * nch) {
        for (uint32_t k = 0; k < hk; k++) L -= chunk_l(lds_chunk(slot_dw * 4 + 16u * k), 0u);
        L -= chunk_l_below(lds_chunk(slot_dw * 4 + 16u * hk), hl & 15u, 0u);
      } else {
        for (uint32_t k = 0; k < hk; k++) L -= chunk_l(*reinterpret_cast<const u32x4*>(P.data + g.wb + 16u * k), 0u);
        L -= chunk_l_below(*reinterpret_cast<const u32x4*>(P.data + g.wb + 16u * hk), hl & 15u, 0u);
      }
      // bytes [je, gend) of the packet's last granule(s): the granule of je is
      // in this packet's window or is the next packet's first window chunk
      // (else from memory); granules after it only with >= 16 padding bytes
      const uint64_t gend = sb.R0 + 16ull * (uint64_t)(sb.b + 1), gj = je & ~15ull;
      if (gj < gend) {
        const uint64_t kk = (gj - g.wb) >> 4;
        const bool own = kk < nch, nxt = !own && next_here && gj == nwb;
        u32x4 c = lds_chunk(own ? slot_dw * 4 + 16u * (uint32_t)kk : (slot_dw + kSlotStride) * 4);
        if (!own && !nxt) c = *reinterpret_cast<const u32x4*>(P.data + gj);
        L -= chunk_l(c, 0u) - chunk_l_below(c, (uint32_t)(je & 15), 0u);
        for (uint64_t ga = gj + 16; ga < gend; ga += 16)
          L -= chunk_l(sb_chunk(P, ga, g.wb, nch, slot_dw, next_here, nwb, kSlotStride), 0u);
      }
      const uint32_t sum = l_to_words(L, (uint32_t)js & 1u);
      l4c = fold(jinit + sum - jexist);
      const bool udp = (st & GPK_ST_L4_UDP) != 0;
      if (l4c == jexist || (udp && jexist == 0)) st |= GPK_ST_L4_VALID;
    }
    if (kFields) emit_fields();
#if GPK_DIAG_TIMES
    dt[4] = __builtin_amdgcn_s_memrealtime();
#endif
  } else if (kL4) {
    // the segment's first and last chunk in an LDS header window: its own,
    // or (the segment ending where the next packet starts) the next lane's
    const uint32_t nch = active ? (m + win + 15) >> 4 : 0u;
    const uint32_t noff_lo = (uint32_t)__shfl_down((int)(uint32_t)off, 1);
    const uint32_t noff_hi = (uint32_t)__shfl_down((int)(uint32_t)(off >> 32), 1);
    const uint32_t nnch = (uint32_t)__shfl_down((int)nch, 1);
    const uint64_t noff = (uint64_t)noff_hi << 32 | noff_lo;
    const uint64_t c0 = off >> 4;
    uint32_t hlds = ~0u, tlds = ~0u;
    bool tafter = false;
    if (AL == 16) {
      if (GPK_PB_LDS_HT && job && (js >> 4) - c0 < nch) hlds = slot_dw * 4 + 16 * (uint32_t)((js >> 4) - c0);
      if (GPK_PB_LDS_HT && job && (je >> 4) - c0 < nch)
        tlds = slot_dw * 4 + 16 * (uint32_t)((je >> 4) - c0);
      else if (GPK_PB_LDS_HT && job && lane < 63 && nnch && (noff >> 4) == (je >> 4))
        tlds = (slot_dw + kSlotStride) * 4;
    } else {
      // the window holds batch bytes [wb, wb + m + win): a head/tail chunk
      // (16-byte aligned in the batch, dword-aligned in the slot) is taken
      // from it when the bytes before s / e that it contributes are there
      const uint64_t wb = g.wb;
      const uint32_t vb = m + win;
      const uint32_t hb = (uint32_t)((js & ~15ull) - wb), tb = (uint32_t)((je & ~15ull) - wb);
      if (GPK_PB_LDS_HT && job && hb < vb && hb + (uint32_t)(js & 15) <= vb) hlds = slot_dw * 4 + hb;
      const uint32_t nm = (uint32_t)__shfl_down((int)m, 1);
      if (GPK_PB_LDS_HT && job && tb < vb && tb + (uint32_t)(je & 15) <= vb) {
        tlds = slot_dw * 4 + tb;
      } else if (GPK_PB_LDS_HT && job && lane < 63 && nnch && noff == je) {
        // the next packet starts at e: its window (packet byte 0 at slot byte
        // nm) holds the granule's bytes from e on, at a dword-aligned address
        tlds = (slot_dw + kSlotStride) * 4 + nm - (uint32_t)(je & 15);
        tafter = true;
      }
    }
    if (kFields) {  // the windows are staging space from here: head and tail chunks from memory
      emit_fields();
      hlds = tlds = ~0u;
      tafter = false;
    }
    const uint32_t sum = segment_sums<D, E>(P, S, job, js, je, lane, hlds, tlds, tafter);
#if GPK_DIAG_TIMES
    dt[4] = __builtin_amdgcn_s_memrealtime();
    dt[7] = (uint64_t)(S.on ? S.R : 0u) | (uint64_t)__popcll(__ballot(job)) << 32;
#endif
    if (job) {
      l4c = fold(jinit + sum - jexist);
      const bool udp = (st & GPK_ST_L4_UDP) != 0;
      if (l4c == jexist || (udp && jexist == 0)) st |= GPK_ST_L4_VALID;
    }
  }
  if (active && P.narrow) {
    // gpk_record8 (gpk.h): the full record only where Correct is not the
    // header's Checksum field (checksum.go:9-21; a UDP 0 is Valid unchecked,
    // udp.go:144-158) or the list has more than 8 entries
    const bool widen = q.nlayers > 8 || ((st & GPK_ST_IP4_CSUM) && !(st & GPK_ST_IP4_VALID)) ||
                       ((st & GPK_ST_L4_CSUM) && l4c != jexist);
    const uint32_t st8 = (st & ~(GPK_ST_NLAYERS_MASK << GPK_ST_NLAYERS_SHIFT)) |
                         ((q.nlayers > 8 ? GPK_ST8_NLAYERS_MASK : q.nlayers) << GPK_ST_NLAYERS_SHIFT) |
                         (widen ? GPK_ST8_WIDE : 0u);
    __builtin_nontemporal_store((uint64_t)st8 << 32 | lay_lo, reinterpret_cast<uint64_t*>(P.records) + i);
    if (widen)
      __builtin_nontemporal_store(u32x4{lay_lo, lay_hi, st, ip4c | (l4c << 16)}, reinterpret_cast<u32x4*>(P.wide) + i);
  } else if (active) {  // written once, never read back here: non-temporal
    __builtin_nontemporal_store(u32x4{lay_lo, lay_hi, st, ip4c | (l4c << 16)}, reinterpret_cast<u32x4*>(P.records) + i);
  }
}

// kCompact: the parser's lookup tables are copied into LDS once per block
// (after the header-window slots) and every NextLayerType lookup is an LDS
// read; otherwise they are read from the global DevTables. Either way the
// only vector-memory traffic of the decode is the packet bytes themselves.
// W: header-window chunks. The 6-chunk default holds Ethernet + two tags +
// IPv6 + TCP with timestamps at any packet alignment; parsers with no
// Dot1Q/IPv6/TCP decoder and no L4 checksum (C2) run a 4-chunk window whose
// smaller LDS slot and 64-VGPR budget give 8 waves per SIMD (A/B: C2 -8.6 %,
// C4 and C3 no gain or worse with 4 chunks).
// O: waves per SIMD the register budget is cut for. Batches of small packets
// (mean < 1 KiB) are issue-bound in the header phase and run O = 7 (72 VGPRs;
// with the table blob sized to the parser, 7 blocks fit a CU's LDS); big
// packets keep O = 6.
template <bool kL4, bool kLayout, bool kCompact, bool kKeys = false, int W = kWinChunks, int O = GPK_WAVES_PER_EU,
          int AL = 16>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(W == 4 ? GPK_W4_WAVES : O, 8))) void decode_kernel(
    KParams P) {
  const uint32_t tid = threadIdx.x;
  const uint32_t slot_dw = tid * slot_dw_of<W, AL>();
  const uint32_t base = kBlock * slot_dw_of<W, AL>();
  if ((uint64_t)blockIdx.x * kBlock >= P.n) return;  // uniform over the block
  // Every packet's index, then its header window and the table blob are in
  // flight together: two dependent memory round trips per packet.
  const uint64_t i0 = (uint64_t)blockIdx.x * kBlock + tid;
  uint64_t dt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#if GPK_DIAG_TIMES
  dt[0] = __builtin_amdgcn_s_memrealtime();
#endif
  const Idx c0 = load_index(P, i0);
#if GPK_DIAG_TIMES
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  dt[1] = __builtin_amdgcn_s_memrealtime();
#endif
  const WinGeo g0 = win_geo<W, AL>(P, c0, i0 < P.n);
  WinT<W> w0;
  load_window<W, AL>(P, g0, w0);
  if (kCompact && GPK_BLOB_DMA) {
    static_assert(GPK_BLOB_ROUND % 64 == 0, "the blob's LDS share holds whole 64-dword DMA rows");
    blob_dma(P, (uint32_t)(uintptr_t)gpk_smem + 4u * base, tid & 63);
  } else if (kCompact) {  // the table blob (<= kCtDwords): clamped indices, duplicate writes of equal values
    static_assert(kCtDwords <= 3 * kBlock, "three blob words per thread");
    const uint32_t last = P.cg.words - 1;
#pragma unroll
    for (uint32_t k = 0; k < 3; k++) {
      const uint32_t j = tid + k * kBlock < last ? tid + k * kBlock : last;
      gpk_smem[base + j] = P.ctab[j];
    }
    __syncthreads();
  }
  store_window<W, AL>(slot_dw, w0);
  // this wave's blob DMA has landed before the parse reads the tables (and
  // before decode_packet issues any stream load)
  if (kCompact && GPK_BLOB_DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if GPK_DIAG_TIMES
  dt[2] = __builtin_amdgcn_s_memrealtime();
#endif
  if (kCompact)
    decode_packet<kL4, kLayout, LTab, kKeys, W, O, AL>(P, LTab{P.cg, base}, i0, i0 < P.n, c0.off, c0.cl, g0, slot_dw,
                                                       tid & 63, dt);
  else
    decode_packet<kL4, kLayout, GTab, kKeys, W, O, AL>(P, GTab{P.tab}, i0, i0 < P.n, c0.off, c0.cl, g0, slot_dw,
                                                       tid & 63, dt);
#if GPK_DIAG_TIMES
  // timestamps (100 MHz realtime counter, one clock for all XCDs), HW_ID | XCC_ID << 32, the
  // phase-B region bytes | job lanes << 32
  dt[5] = __builtin_amdgcn_s_memrealtime();
  dt[6] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) | (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32;
  if (P.diag && (tid & 63) < 8) {
    uint64_t v = dt[0];
#pragma unroll
    for (int k = 1; k < 8; k++) v = (tid & 7) == (uint32_t)k ? dt[k] : v;
    P.diag[((uint64_t)blockIdx.x * kWaves + tid / 64) * 8 + (tid & 7)] = v;
  }
#endif
}

// Stream-before-parse L4 kernel (GPK_SB): the header windows go into LDS by
// LDS-DMA (no registers held) and phase B's stream over the wave's packets is
// issued right behind them, before DecodeLayers: the window's latency hides
// under the stream, the stream re-reads the window lines while they are still
// in L2, and the parse that follows has the whole register file. The stream
// keeps, per lane, the L-form sum of its packet's granules (sb_stream); after
// the parse decode_packet's stream-before-parse branch subtracts the header
// bytes before the segment (window) and the bytes after it. Waves whose
// packets are not packed run the ordinary phase B after the parse.

// 16 bytes per lane into LDS: lane l's bytes land at LDS byte `lds` + 16 l
// (wave-uniform destination, per-lane source; tools/probes/lds_dma.hip).
__device__ __forceinline__ void dma16(uint64_t src, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(lds)
               : "memory");
}
// The W-chunk windows of the wave's 64 packets into its slots (slot q at LDS
// byte `region` + 16 W q, no pad: instruction k writes cells 64 k .. 64 k + 63,
// cell e = chunk e mod W of packet e / W, the packet's window base and chunk
// count fetched from its lane). Chunks past a window re-read its last chunk, a
// packet with none reads the parser's table copy (as load_window).
template <int W>
__device__ __forceinline__ void window_dma(const KParams& P, const WinGeo& g, uint32_t region, uint32_t lane) {
#if GPK_DIAG_NULLWIN  // timing only: every window from the L2-resident table copy
  const uint64_t src = (uint64_t)(uintptr_t)P.tab;
#else
  const uint64_t src = g.nch ? (uint64_t)(uintptr_t)(P.data + g.wb) : (uint64_t)(uintptr_t)P.tab;
#endif
  const uint32_t last = g.nch ? g.nch - 1 : 0u;
#pragma unroll
  for (int k = 0; k < W; k++) {
    const uint32_t e = 64u * k + lane, q = e / W, c = e - q * W;
    const int qa = (int)(q << 2);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(qa, (int)(uint32_t)src);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(qa, (int)(uint32_t)(src >> 32));
    const uint32_t lq = (uint32_t)__builtin_amdgcn_ds_bpermute(qa, (int)last);
    dma16(((uint64_t)hi << 32 | lo) + 16u * (c < lq ? c : lq), region + 1024u * k);
  }
}

template <bool kCompact, int O, int W = 6, bool kFields = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(O, 8))) void decode_sb_kernel(KParams P) {
  // fields_store stages 48 whole 128-byte records (GPK_FIELDS_STAGE 2: 1536 dwords) or a half record per lane
  // (1: 1024 dwords) in the wave's window slots, 4 W dwords per lane
  static_assert(!kFields || 64 * 4 * W >= (GPK_FIELDS_STAGE == 2 ? 1536 : 1024),
                "the fused fields' staging does not fit the wave's window slots");
  constexpr int D = GPK_SB_DEPTH;
  constexpr int kSbStride = 4 * W;  // one 16-byte cell per window chunk, no pad
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t base = kBlock * kSbStride;  // table blob (dwords)
  if ((uint64_t)blockIdx.x * kBlock >= P.n) return;  // uniform over the block
  const uint64_t i0 = (uint64_t)blockIdx.x * kBlock + tid;
  const bool active = i0 < P.n;
  uint64_t dt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#if GPK_DIAG_TIMES
  dt[0] = __builtin_amdgcn_s_memrealtime();
#endif
  const Idx c0 = load_index(P, i0);
  const WinGeo g0 = win_geo<W, 16>(P, c0, active);
  window_dma<W>(P, g0, (uint32_t)(uintptr_t)gpk_smem + wave * (64u * kSbStride * 4u), lane);
  if (kCompact && GPK_BLOB_DMA) {  // this wave's own copy (the vmcnt(0) below waits for it)
    blob_dma(P, (uint32_t)(uintptr_t)gpk_smem + 4u * base, lane);
  } else if (kCompact) {  // the table blob (read after the barrier below)
    static_assert(kCtDwords <= 3 * kBlock, "three blob words per thread");
    const uint32_t last = P.cg.words - 1;
#pragma unroll
    for (uint32_t k = 0; k < 3; k++) {
      const uint32_t j = tid + k * kBlock < last ? tid + k * kBlock : last;
      gpk_smem[base + j] = P.ctab[j];
    }
  }
#if GPK_DIAG_TIMES
  dt[1] = __builtin_amdgcn_s_memrealtime();  // (diag phases: index | stream | parse | correction)
#endif
  // the stream over the packets' extents, when packed
  uint64_t R0 = 0;
  uint32_t R = 0;
  const bool ok = dense_region(active && (P.outputs & GPK_OUT_L4_CSUM) != 0, c0.off, c0.off + c0.cl, R0, R);
  uint32_t L = 0;
  int32_t b = -1;
  if (ok) {
    const int32_t a1 = active ? (int32_t)((g0.wb - R0) >> 4) - 1 : -1;
    b = active ? (int32_t)(((c0.off + c0.cl) - 1 - R0) >> 4) : -1;
    Stream<D> S;
    S.on = true;
    L = sb_stream<D>(P, S, R0, R, lane, a1, b);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the windows (and this wave's blob) have landed
  if (kCompact && !GPK_BLOB_DMA) __syncthreads();
#if GPK_DIAG_TIMES
  dt[2] = __builtin_amdgcn_s_memrealtime();
#endif
  // only the index entry crosses the stream: everything derived from it is formed again
  uint32_t off_lo = (uint32_t)c0.off, off_hi = (uint32_t)(c0.off >> 32), ccl = c0.cl;
  asm volatile("" : "+v"(off_lo), "+v"(off_hi), "+v"(ccl));
  const Idx c1{(uint64_t)off_hi << 32 | off_lo, ccl};
  const uint32_t tid1 = threadIdx.x;
  const uint64_t i1 = (uint64_t)blockIdx.x * kBlock + tid1;
  const WinGeo g1 = win_geo<W, 16>(P, c1, i1 < P.n);
  if (kCompact)
    decode_packet<true, false, LTab, false, W, O, 16, kSbStride, 0, true, kFields>(
        P, LTab{P.cg, base}, i1, i1 < P.n, c1.off, c1.cl, g1, tid1 * kSbStride, tid1 & 63, dt, SbPkt{L, R0, b, ok});
  else
    decode_packet<true, false, GTab, false, W, O, 16, kSbStride, 0, true, kFields>(
        P, GTab{P.tab}, i1, i1 < P.n, c1.off, c1.cl, g1, tid1 * kSbStride, tid1 & 63, dt, SbPkt{L, R0, b, ok});
#if GPK_DIAG_TIMES
  dt[5] = __builtin_amdgcn_s_memrealtime();
  dt[6] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) | (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32;
  dt[7] = ok ? (uint64_t)R | (uint64_t)__builtin_popcountll(__ballot(active)) << 32 : 0;
  if (P.diag && lane < 8) {
    uint64_t v = dt[0];
#pragma unroll
    for (int k = 1; k < 8; k++) v = lane == (uint32_t)k ? dt[k] : v;
    P.diag[((uint64_t)blockIdx.x * kWaves + wave) * 8 + lane] = v;
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

// Workgroups of `lds` bytes of LDS that are resident on one CU at once: the
// occupancy API's count, capped by what gfx950 places (measured,
// tools/probes/occ_probe.hip, profiles/r12_occupancy.json: 8 blocks up to
// 20480 bytes, 7 up to 23040, 6 up to 26624, 5 up to 31744; the API allows one
// more block above 27136 and 32256 bytes than are ever resident).
int lds_blocks_per_cu(int lds) {
  static const int lim[] = {0, 163840, 81920, 53248, 39936, 31744, 26624, 23040, 20480};
  int b = 8;
  while (b > 1 && lds > lim[b]) b--;
  return b;
}
template <class K>
hipError_t resident_blocks(K kernel, int lds, int* blocks) {
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, kernel, gpk::kBlock, lds);
  if (e == hipSuccess && *blocks > lds_blocks_per_cu(lds)) *blocks = lds_blocks_per_cu(lds);
  return e;
}

// Launch one specialisation on `stream`, or (occ != nullptr) report how many of
// its blocks fit a CU with this launch's LDS size instead.
template <bool kL4, bool kLayout, bool kCompact, bool kKeys = false, int W = gpk::kWinChunks,
          int O = GPK_WAVES_PER_EU, int AL = 16>
hipError_t launch(const gpk::KParams* P, hipStream_t stream, int* occ) {
  using namespace gpk;
  constexpr int slot_lds = kBlock * slot_dw_of<W, AL>() * 4;
  // the table blob takes only the words this parser's tables use
  const int lds = kCompact ? slot_lds + (int)((P->cg.words + GPK_BLOB_ROUND - 1) & ~(GPK_BLOB_ROUND - 1u)) * 4 : slot_lds;
  if (occ) return resident_blocks(decode_kernel<kL4, kLayout, kCompact, kKeys, W, O, AL>, lds, occ);
  const uint64_t grid = (P->n + kBlock - 1) / kBlock;
  if (grid > 0xffffffffull) return hipErrorInvalidValue;
  hipLaunchKernelGGL((decode_kernel<kL4, kLayout, kCompact, kKeys, W, O, AL>), dim3((unsigned)grid), dim3(kBlock), lds,
                     stream, *P);
  return hipGetLastError();
}

template <bool kCompact, int O, int W = 6, bool kFields = false>
hipError_t launch_sb(const gpk::KParams* P, hipStream_t stream, int* occ) {
  using namespace gpk;
  constexpr int fixed = kBlock * 4 * W * 4;
  const int lds = kCompact ? fixed + (int)((P->cg.words + GPK_BLOB_ROUND - 1) & ~(GPK_BLOB_ROUND - 1u)) * 4 : fixed;
  if (occ) return resident_blocks(decode_sb_kernel<kCompact, O, W, kFields>, lds, occ);
  const uint64_t grid = (P->n + kBlock - 1) / kBlock;
  if (grid > 0xffffffffull) return hipErrorInvalidValue;
  hipLaunchKernelGGL((decode_sb_kernel<kCompact, O, W, kFields>), dim3((unsigned)grid), dim3(kBlock), lds, stream, *P);
  return hipGetLastError();
}

// The specialisation a launch uses (gpk_launch_decode, gpk_launch_name).
struct Sel {
  bool l4, layout, compact, keys;
  int W, O, AL;
  bool sb;
};
Sel select(const gpk::KParams* P, int with_l4, int with_layout) {
  Sel s{with_l4 != 0, with_layout != 0, P->ctab != nullptr, P->key_kind != 0, gpk::kWinChunks, GPK_WAVES_PER_EU, 16,
        false};
  if (s.keys) {  // fused grouping keys: no layouts (gpk_decode_group_batch)
    s.layout = false;
  } else if (!s.l4 && !s.layout && P->small_headers) {
    s.W = 4;
  } else if (!s.layout && !P->big_packets) {
    s.O = GPK_SMALL_WAVES;
    // a dword-aligned 5-chunk window (7 blocks per CU) for the smallest packets; from a mean of
    // GPK_MID_MAXMEAN bytes on, the stream-before-parse kernel (A/B r15: C1, mean 113 B, +2.7 % with
    // it; C4's packets through a parser without IPv6, mean 362 B, -8 %)
    if (GPK_MID_W5 && (P->mid_headers || GPK_MID_IP6) && P->data_end && P->mean_bytes < GPK_MID_MAXMEAN) {
      s.W = 5;
      s.AL = 4;
    }
  }
  s.sb = GPK_SB && s.l4 && !s.layout && !s.keys && s.W == gpk::kWinChunks && s.AL == 16 &&
         (GPK_SB_BIG || s.O != GPK_WAVES_PER_EU);
  return s;
}

template <bool kCompact>
hipError_t launch_sel(const gpk::KParams* P, const Sel& s, hipStream_t stream, int* occ) {
  constexpr int W = gpk::kWinChunks;
  if (s.sb) {
#if GPK_SB_BIG
    if (s.O == GPK_WAVES_PER_EU) return launch_sb<kCompact, GPK_WAVES_PER_EU>(P, stream, occ);
#endif
    return launch_sb<kCompact, GPK_SB_WAVES>(P, stream, occ);
  }
  if (s.keys)
    return s.l4 ? launch<true, false, kCompact, true>(P, stream, occ) : launch<false, false, kCompact, true>(P, stream, occ);
  if (s.W == 4) return launch<false, false, kCompact, false, 4>(P, stream, occ);
  if (s.l4 && s.layout) return launch<true, true, kCompact>(P, stream, occ);
  if (s.l4)
    return s.O == GPK_WAVES_PER_EU ? launch<true, false, kCompact>(P, stream, occ)
           : s.AL == 4             ? launch<true, false, kCompact, false, 5, GPK_SMALL_WAVES, 4>(P, stream, occ)
                                   : launch<true, false, kCompact, false, W, GPK_SMALL_WAVES>(P, stream, occ);
  if (s.layout) return launch<false, true, kCompact>(P, stream, occ);
  return s.O == GPK_WAVES_PER_EU ? launch<false, false, kCompact>(P, stream, occ)
         : s.AL == 4             ? launch<false, false, kCompact, false, 5, GPK_SMALL_WAVES, 4>(P, stream, occ)
                                 : launch<false, false, kCompact, false, W, GPK_SMALL_WAVES>(P, stream, occ);
}

}  // namespace

extern "C" hipError_t gpk_launch_decode(const gpk::KParams* P, int with_l4, int with_layout, hipStream_t stream) {
  if (P->n == 0) return hipSuccess;
  if (P->key_kind && with_layout) return hipErrorInvalidValue;
  const Sel s = select(P, with_l4, with_layout);
  return s.compact ? launch_sel<true>(P, s, stream, nullptr) : launch_sel<false>(P, s, stream, nullptr);
}

// Blocks of that specialisation resident per CU (registers and this launch's LDS).
extern "C" hipError_t gpk_launch_occupancy(const gpk::KParams* P, int with_l4, int with_layout, int* blocks) {
  const Sel s = select(P, with_l4, with_layout);
  return s.compact ? launch_sel<true>(P, s, nullptr, blocks) : launch_sel<false>(P, s, nullptr, blocks);
}

// Name of the kernel specialisation gpk_launch_decode would launch.
extern "C" int gpk_launch_describe(const gpk::KParams* P, int with_l4, int with_layout, char* buf, size_t cap) {
  const Sel s = select(P, with_l4, with_layout);
  if (s.sb)
    return snprintf(buf, cap, "gpk::decode_sb_kernel<%s,%d,%d,false>", s.compact ? "true" : "false",
                    s.O == GPK_WAVES_PER_EU ? s.O : GPK_SB_WAVES, gpk::kWinChunks);
  return snprintf(buf, cap, "gpk::decode_kernel<%s,%s,%s,%s,%d,%d,%d>", s.l4 ? "true" : "false",
                  s.layout ? "true" : "false", s.compact ? "true" : "false", s.keys ? "true" : "false", s.W,
                  s.W == 4 ? 6 : s.O, s.AL);
}

// The fused decode + layer fields launch (gpk_decode_batch_fields without
// layouts): the stream-before-parse kernel with its fields epilogue, for every
// parser and batch (its 6-chunk window holds every header the fast path reads;
// the rest comes from memory). occ: report resident blocks instead; name:
// describe it instead.
extern "C" hipError_t gpk_launch_decode_fields(const gpk::KParams* P, hipStream_t stream, int* occ) {
  if (!occ && P->n == 0) return hipSuccess;
  if (P->key_kind || !P->fields) return hipErrorInvalidValue;
  return P->ctab ? launch_sb<true, GPK_SBF_WAVES, gpk::kWinChunks, true>(P, stream, occ)
                 : launch_sb<false, GPK_SBF_WAVES, gpk::kWinChunks, true>(P, stream, occ);
}
extern "C" int gpk_launch_describe_fields(const gpk::KParams* P, char* buf, size_t cap) {
  return snprintf(buf, cap, "gpk::decode_sb_kernel<%s,%d,%d,true>", P->ctab ? "true" : "false", GPK_SBF_WAVES,
                  gpk::kWinChunks);
}

extern "C" hipError_t gpk_launch_list(const gpk::KParams* P, uint64_t index, int64_t* out, uint32_t cap,
                                      uint32_t* out_n, hipStream_t stream) {
  hipLaunchKernelGGL(gpk::list_kernel, dim3(1), dim3(64), 0, stream, *P, index, out, cap, out_n);
  return hipGetLastError();
}

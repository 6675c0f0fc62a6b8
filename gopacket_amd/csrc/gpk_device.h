// gpk_device.h — per-packet DecodingLayerParser state machine for gfx950.
//
// One lane runs DecodingLayerParser.DecodeLayers (parser.go:303-317) for one
// packet, following LayersDecoder's loop (layers_decoder.go:60-79). The layer
// decoders below restate layers/{ethernet,dot1q,ip4,ip6,tcp,udp}.go; their
// results must be bit-identical to the reference (checked against oracle/).
//
// Bytes come from a per-lane LDS window holding the packet's first bytes (the
// 16-byte-aligned run of W chunks, filled by the kernel); positions past the
// window fall back to global byte loads (deep stacks, long options).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gpk.h"

namespace gpk {

// ---- configuration uploaded once per parser change ------------------------
struct DevTables {
  int32_t ethertype[65536];
  int32_t tcp_port[65536];
  int32_t udp_port[65536];
  int32_t ipprotocol[256];
  uint8_t dispatch[GPK_MAX_LAYER_TYPE];  // LayerType -> GPK_DEC_*
};

// Compact copy of a parser's lookup tables (LTab), built by the host when
// they fit (gpk_host.cpp build_compact) and copied into LDS by every block.
// Blob layout in dwords: LayerType per handle, kind|code<<4 per handle (u8),
// handle per IP protocol (u8), then the hash slots of the EtherType, TCP port
// and UDP port tables.
constexpr int kCtVal = 0;
constexpr int kCtKc = 128;
constexpr int kCtIpp = 160;
constexpr int kCtSlots = 224;
constexpr int kCtMaxHandles = 128;
constexpr int kCtMaxSlots = 512;
constexpr int kCtDwords = kCtSlots + kCtMaxSlots;
struct CompactGeom {
  uint32_t eth_off, eth_shift, eth_mask, eth_probe, eth_def;  // off: dwords from the blob base
  uint32_t tcp_off, tcp_shift, tcp_mask, tcp_probe, tcp_def;
  uint32_t udp_off, udp_shift, udp_mask, udp_probe, udp_def;
  uint32_t frag_h, zero_h, first_h, payload_h;
  uint32_t words;  // blob dwords to copy
};

struct KParams {
  const uint8_t* data;
  const uint64_t* offsets;
  const uint32_t* caplens;
  uint64_t n;
  uint64_t data_end;        // readable bytes of data: gpk_batch.data_bytes rounded up to 16 (0 = unknown)
  gpk_record* records;
  uint32_t* err_args;
  uint64_t* flows;
  gpk_layout* layouts;
  const DevTables* tab;
  int64_t first;
  uint32_t outputs;
  int32_t ignore_unsupported;
  int32_t first_kind;       // decoder registered for `first` (GPK_DEC_NONE if none)
  const uint32_t* ctab;     // compact blob in device memory, or null: global tables
  CompactGeom cg;
  uint32_t fast;            // GPK_FAST_* : which transitions the straight-line path may take
  // fused grouping keys (gpk_decode_group_batch): 0 = off, else GPK_GROUP_CONNECTION /
  // GPK_GROUP_DEFRAG; per packet 10 key words, a 64-bit hash and a reason code
  int32_t key_kind;
  uint32_t small_headers;   // no Dot1Q / IPv6 / IPv6-extension / TCP decoder: a 4-chunk window suffices
  uint32_t mid_headers;     // no IPv6 / IPv6-extension decoder: the small-packet kernel's 5-chunk window suffices
  uint32_t big_packets;     // batch bytes / packets >= 1 KiB: launch choice only (occupancy)
  uint32_t mean_bytes;      // batch bytes / packets (capped at 2^32 - 1): launch choice only
  uint32_t* keys;
  uint64_t* khash;
  int32_t* kcode;
  uint64_t* diag;           // GPK_DIAG_TIMES builds only: 8 u64 per wave (gpk_diag_set_buffer)
  gpk_fields* fields;       // fused layer fields (gpk_decode_batch_fields), the fields kernels only
  // narrow records (gpk_decode_batch_narrow): records holds gpk_record8[n], and a
  // packet whose record does not fit writes its full one to wide[i] (gpk.h)
  uint32_t narrow;
  gpk_record* wide;
};

// Straight-line common-case parse (fast_parser below). Each bit says the
// parser's container and tables make this transition go to the expected
// decoder, so the fast path may take it without the generic dispatch; the
// host derives them from the parser (gpk_host.cpp fast_flags).
#define GPK_FAST_ON 0x1u       // first decoder is Ethernet
#define GPK_FAST_IP4 0x2u      // EtherType 0x0800 -> IPv4 decoder
#define GPK_FAST_IP6 0x4u      // EtherType 0x86DD -> IPv6 decoder
#define GPK_FAST_D1Q 0x8u      // EtherType 0x8100 -> Dot1Q decoder
#define GPK_FAST_QINQ 0x10u    // EtherType 0x88A8 -> Dot1Q decoder
#define GPK_FAST_TCP 0x20u     // IPProtocol 6 -> TCP decoder
#define GPK_FAST_UDP 0x40u     // IPProtocol 17 -> UDP decoder

// LDS geometry: per lane a header window of WIN_CHUNKS 16-byte chunks.
// Slot stride is odd in dwords so byte/dword reads at equal packet positions
// from 32 lanes hit 32 different banks.
constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
#ifndef GPK_WIN_CHUNKS
#define GPK_WIN_CHUNKS 6  // 96-byte header window (A/B r03: C1 -25 %, C4 -1.5 %, C3 +-0 vs 5: Eth + tags +
                          // IPv6 + TCP headers fit, the general decoder stays off the common path)
#endif
constexpr int kWinChunks = GPK_WIN_CHUNKS;
// odd: lanes reading equal packet positions hit distinct banks
constexpr int kSlotDw = kWinChunks * 4 + 1;
constexpr int kLdsBytes = kBlock * kSlotDw * 4;

// Dynamic LDS of the decode kernels (one declaration, aliased everywhere).
extern __shared__ __attribute__((aligned(16))) uint32_t gpk_smem[];

__device__ __forceinline__ uint32_t lds8(uint32_t byte_addr) {
  return ((const uint8_t*)gpk_smem)[byte_addr];
}

// Packet byte readers. RdL: the bytes are in this lane's LDS window (the
// caller checked the whole header range), one ds_read_u8 per byte and no
// branch. Rd: LDS window first, global memory past it (deep stacks, long
// options, HopByHop TLVs).
struct RdL {
  uint32_t lb;  // LDS byte address of packet byte 0
};
struct Rd {
  const uint8_t* g;  // packet start (global)
  uint32_t lb;       // LDS byte address of packet byte 0
  uint32_t win;      // packet bytes present in LDS
};

// Four LDS bytes from any byte address: one ds_read_b32 (gfx950 serves
// unaligned LDS dword reads exactly: tools/probes/lds_unaligned.hip, 64/64
// byte offsets on MI355X). A read may run up to 3 bytes past the bytes a
// caller uses (into the next slot or the table blob; past the allocation the
// hardware returns zeros); those bytes are never used. Two aligned dwords +
// v_alignbyte instead, with or without the windows stored dword-rotated so
// packet byte 0 opens the slot, measured no faster and raised the LDS
// bank-conflict cycles 2-5x (profiles/r06_ab_lds_reads.txt).
typedef uint32_t u32_ua __attribute__((aligned(1)));
__device__ __forceinline__ uint32_t lds32u(uint32_t byte_addr) {
  return *reinterpret_cast<const u32_ua*>(reinterpret_cast<const uint8_t*>(gpk_smem) + byte_addr);
}
// big-endian 16 / 32 bits of the four bytes w = b0 | b1 << 8 | ... (v_perm_b32)
__device__ __forceinline__ uint32_t be16_of(uint32_t w) { return __builtin_amdgcn_perm(0u, w, 0x0c0c0001u); }
__device__ __forceinline__ uint32_t be32_of(uint32_t w) { return __builtin_amdgcn_perm(0u, w, 0x00010203u); }

__device__ __forceinline__ uint32_t rd8(const RdL& r, uint32_t p) { return lds8(r.lb + p); }
__device__ __forceinline__ uint32_t rd8(const Rd& r, uint32_t p) {
  return p < r.win ? lds8(r.lb + p) : (uint32_t)r.g[p];
}
__device__ __forceinline__ uint32_t rd16(const RdL& r, uint32_t p) { return be16_of(lds32u(r.lb + p)); }
__device__ __forceinline__ uint32_t rd32(const RdL& r, uint32_t p) { return be32_of(lds32u(r.lb + p)); }
__device__ __forceinline__ uint32_t rd16(const Rd& r, uint32_t p) {
  if (p + 2 <= r.win) return rd16(RdL{r.lb}, p);
  return (rd8(r, p) << 8) | rd8(r, p + 1);
}
__device__ __forceinline__ uint32_t rd32(const Rd& r, uint32_t p) {
  if (p + 4 <= r.win) return rd32(RdL{r.lb}, p);
  return (rd16(r, p) << 16) | rd16(r, p + 2);
}

// Outcome of one DecodeFromBytes + NextLayerType + LayerPayload, returned by
// value (a struct passed by reference through the inlined decoders ends up in
// scratch memory).
struct Res {
  uint32_t err, a0, a1;  // GPK_ERR_* and its arguments
  uint32_t trunc;        // DecodeFeedback.SetTruncated was called
  uint32_t off, len;     // LayerPayload()
  int32_t next;          // NextLayerType()
  uint32_t aux;          // UDP: len(Contents)+len(Payload)
};

__device__ __forceinline__ Res rerr(uint32_t trunc, uint32_t code, uint32_t a0 = 0, uint32_t a1 = 0) {
  Res x;
  x.err = code;
  x.a0 = a0;
  x.a1 = a1;
  x.trunc = trunc;
  x.off = x.len = 0;
  x.next = 0;
  x.aux = 0;
  return x;
}
__device__ __forceinline__ Res rok(uint32_t trunc, uint32_t off, uint32_t len, int32_t next, uint32_t aux = 0) {
  Res x;
  x.err = x.a0 = x.a1 = 0;
  x.trunc = trunc;
  x.off = off;
  x.len = len;
  x.next = next;
  x.aux = aux;
  return x;
}

// ---- layers/ethernet.go:42-63 (+ NextLayerType :111-113) ------------------
template <class TT, class R>
__device__ __forceinline__ Res dec_ethernet(const TT& T, const R& r, uint32_t off, uint32_t len) {
  if (len < 14) return rerr(0, GPK_ERR_ETH_TOO_SMALL);
  uint32_t et = rd16(r, off + 12);
  uint32_t plen = len - 14, trunc = 0;
  if (et < 0x0600) {  // 802.3 length field: EthernetTypeLLC, trim or flag
    if (plen < et) trunc = 1;
    else plen = et;
    et = 0;
  }
  return rok(trunc, off + 14, plen, T.eth(et));
}

// ---- layers/dot1q.go:30-41, :49-51 -----------------------------------------
template <class TT, class R>
__device__ __forceinline__ Res dec_dot1q(const TT& T, const R& r, uint32_t off, uint32_t len) {
  if (len < 4) return rerr(1, GPK_ERR_DOT1Q_SHORT, len);
  return rok(0, off + 4, len - 4, T.eth(rd16(r, off + 2)));
}

// ---- layers/ip4.go:178-271, :277-282 ---------------------------------------
template <class TT, class R>
__device__ __forceinline__ Res dec_ipv4(const TT& T, const R& r, uint32_t off, uint32_t len) {
  if (len < 20) return rerr(1, GPK_ERR_IP4_HDR_SHORT, len);
  uint32_t b0 = rd8(r, off);
  uint32_t length = rd16(r, off + 2);
  uint32_t ihl = b0 & 0xf;
  if (length == 0) length = len & 0xffff;  // TSO, uint16 wrap (ip4.go:189-193)
  if (length < 20) return rerr(0, GPK_ERR_IP4_LEN_SMALL, length);
  if (ihl < 5) return rerr(0, GPK_ERR_IP4_IHL_SMALL, ihl);
  uint32_t hl = ihl * 4;
  if (hl > length) return rerr(0, GPK_ERR_IP4_IHL_GT_LEN, ihl, length);
  uint32_t trunc = 0;
  if (len > length) {
    len = length;
  } else if (len < length) {
    trunc = 1;
    if (hl > len) return rerr(1, GPK_ERR_IP4_HDR_MISSING);
  }
  // options (ip4.go:217-256)
  uint32_t p = off + 20, rem = hl - 20;
  while (rem > 0) {
    uint32_t t = rd8(r, p);
    if (t == 0) break;
    uint32_t ol = 1;
    if (t != 1) {
      if (rem < 2) return rerr(1, GPK_ERR_IP4_OPT_SHORT, rem);
      ol = rd8(r, p + 1);
      if (rem < ol) return rerr(1, GPK_ERR_IP4_OPT_EXCEEDS, t, ol);
      if (ol <= 2) return rerr(trunc, GPK_ERR_IP4_OPT_BADLEN, t, ol);
    }
    p += ol;
    rem -= ol;
  }
  uint32_t ff = rd16(r, off + 6);
  int32_t next = ((ff & 0x2000u) || (ff & 0x1fffu)) ? T.frag() : T.ipp(rd8(r, off + 9));
  return rok(trunc, off + hl, len - hl, next);
}

// ---- IPv6: layers/ip6.go:221-278 with inline HopByHop :509-526,
//      decodeIPv6ExtensionBase :418-432, TLV :327-346, jumbogram :54-76,
//      NextLayerType :286-291 -------------------------------------------------
template <class TT, class R>
__device__ __forceinline__ Res dec_ipv6(const TT& T, const R& r, const Rd& rm, uint32_t off,
                                        uint32_t len) {
  if (len < 40) return rerr(1, GPK_ERR_IP6_HDR_SHORT, len);
  uint32_t length = rd16(r, off + 4);
  uint32_t nh = rd8(r, off + 6);
  uint32_t poff = off + 40, plen = len - 40;
  uint32_t next_nh = nh;
  if (nh == 0) {
    if (plen < 2) return rerr(1, GPK_ERR_IP6_EXT_SHORT, plen);
    uint32_t hnh = rd8(rm, poff);
    uint32_t actual = rd8(rm, poff + 1) * 8 + 8;
    if (plen < actual) return rerr(0, GPK_ERR_IP6_EXT_LEN, plen, actual);
    uint32_t have = 0, joff = 0, jlen = 0;
    for (uint32_t q = 2; q < actual;) {
      uint32_t rem = plen - q;
      if (rem < 2) return rerr(1, GPK_ERR_IP6_TLV_SHORT);
      uint32_t t = rd8(rm, poff + q);
      uint32_t al = 1;
      if (t != 0) {
        al = rd8(rm, poff + q + 1) + 2;
        if (rem < al) return rerr(1, GPK_ERR_IP6_TLV_TOO_SMALL);
        if (t == 0xC2 && !have) {
          have = 1;
          joff = poff + q + 2;
          jlen = al - 2;
        }
      }
      q += al;
    }
    next_nh = hnh;
    if (have) {
      if (jlen != 4) return rerr(0, GPK_ERR_IP6_JUMBO_TLV_LEN);
      uint32_t l = rd32(rm, joff);
      if (l <= 65535u) return rerr(0, GPK_ERR_IP6_JUMBO_SMALL);
      if (length != 0) return rerr(0, GPK_ERR_IP6_JUMBO_AND_LEN);
      uint32_t trunc = 0;
      if (l > plen) {  // payload stays at the HopByHop header (ip6.go:249-256)
        trunc = 1;
        l = plen;
      }
      return rok(trunc, poff, l, T.ipp(hnh));
    }
    if (length == 0) return rerr(0, GPK_ERR_IP6_LEN0_NO_JUMBO);
    poff += actual;  // ip6.go:262, then trimmed to the full Length below
    plen -= actual;
  }
  if (length == 0) return rerr(0, GPK_ERR_IP6_LEN0, nh);
  uint32_t trunc = 0;
  if (length > plen) {
    trunc = 1;
    length = plen;
  }
  return rok(trunc, poff, length, T.ipp(next_nh));
}

// ---- IPv6ExtensionSkipper ip6.go:443-461 (base :418-432) -------------------
template <class TT, class R>
__device__ __forceinline__ Res dec_ipv6_ext(const TT& T, const R& r, uint32_t off, uint32_t len) {
  if (len < 2) return rerr(1, GPK_ERR_IP6_EXT_SHORT, len);
  uint32_t nh = rd8(r, off);
  uint32_t actual = rd8(r, off + 1) * 8 + 8;
  if (len < actual) return rerr(0, GPK_ERR_IP6_EXT_LEN, len, actual);
  return rok(0, off + actual, len - actual, T.ipp(nh));
}

// ---- MPTCP option body tcp.go:347-533 with Go's bounds checks ---------------
// The option slice has len = bytes left in the TCP header and cap = bytes to
// the end of the packet. data[i] needs i < len; data[lo:hi] needs hi <= cap
// then lo <= hi; data[lo:] needs lo <= len. Returns err (0 = ok) and the
// option length in x.len.
#define GPK_IDX(i)                                                                  \
  do {                                                                              \
    if ((uint32_t)(i) >= slen) return rerr(0, GPK_ERR_PANIC_INDEX, (i), slen);      \
  } while (0)
#define GPK_SL(lo, hi)                                                                          \
  do {                                                                                          \
    if ((uint32_t)(hi) > scap) return rerr(0, GPK_ERR_PANIC_SLICE_ACAP, (hi), scap);            \
    if ((uint32_t)(lo) > (uint32_t)(hi)) return rerr(0, GPK_ERR_PANIC_SLICE_B, (lo), (hi));     \
  } while (0)

template <class R>
__device__ __forceinline__ Res mptcp_option(const R& r, uint32_t p, uint32_t slen, uint32_t scap) {
  GPK_IDX(1);
  uint32_t ol = rd8(r, p + 1);
  if (ol == 0) return rerr(0, GPK_ERR_MPTCP_LEN, ol);
  GPK_IDX(2);
  uint32_t b2 = rd8(r, p + 2);
  switch (b2 >> 4) {
    case 0:  // MP_CAPABLE
      if (ol != 4 && ol != 12 && ol != 20 && ol != 22 && ol != 24) return rerr(0, GPK_ERR_MP_CAPABLE_LEN, ol);
      GPK_IDX(3);
      if (ol >= 12) GPK_SL(4, 12);
      if (ol >= 20) GPK_SL(12, 20);
      if (ol >= 22) GPK_SL(20, 22);
      if (ol == 24) GPK_SL(22, 24);
      break;
    case 1:  // MP_JOIN
      if (ol != 12 && ol != 16 && ol != 24) return rerr(0, GPK_ERR_MP_JOIN_LEN, ol);
      if (ol == 12) {
        GPK_IDX(3);
        GPK_SL(4, 8);
        GPK_SL(8, 12);
      } else if (ol == 16) {
        GPK_IDX(3);
        GPK_SL(4, 12);
        GPK_SL(12, 16);
      } else {
        GPK_SL(4, 24);
      }
      break;
    case 2: {  // DSS, optionMptcpDsslen tcp.go:553-571
      GPK_IDX(3);
      uint32_t f = rd8(r, p + 3);
      uint32_t A = f & 1, a = f & 2, M = f & 4, m = f & 8;
      uint32_t l0 = 4 + (A ? (a ? 8 : 4) : 0) + (M ? (m ? 14 : 10) : 0);
      uint32_t l1 = l0 + (M ? 2 : 0);
      if (ol != l0 && ol != l1) return rerr(0, GPK_ERR_DSS_LEN, ol);
      uint32_t lo = 4;
      if (A) {
        uint32_t w = a ? 8 : 4;
        GPK_SL(lo, lo + w);
        lo += w;
      }
      if (M) {
        uint32_t w = m ? 8 : 4;
        GPK_SL(lo, lo + w);
        lo += w;
        GPK_SL(lo, lo + 4);
        lo += 4;
        GPK_SL(lo, lo + 2);
        lo += 2;
        if (((ol - lo) & 0xff) == 2) GPK_SL(lo, lo + 2);
      }
      break;
    }
    case 3: {  // ADD_ADDR, isValidOptionMptcpAddAddrlen tcp.go:573-585
      uint32_t ver1 = (b2 & 0xf) <= 1;
      uint32_t e = ver1 ? (b2 & 1) : 0;
      uint32_t chk = (ver1 && !e) ? ((ol - 8) & 0xff) : ol;
      if (!(chk == 8 || chk == 10 || chk == 20 || chk == 22)) return rerr(0, GPK_ERR_ADD_ADDR_LEN, ol);
      GPK_IDX(3);
      uint32_t lenopt = ol;
      if (ver1 && !e) {
        uint32_t lo = (ol - 8) & 0xff;
        if (lo > slen) return rerr(0, GPK_ERR_PANIC_SLICE_B, lo, slen);
        lenopt = lo;
      }
      if (lenopt == 8) {
        GPK_SL(4, 8);
      } else if (lenopt == 10) {
        GPK_SL(4, 8);
        GPK_SL(8, 10);
      } else if (lenopt == 20) {
        GPK_SL(4, 20);
      } else if (lenopt == 22) {
        GPK_SL(4, 20);
        GPK_SL(20, 22);
      }
      break;
    }
    case 4:  // REMOVE_ADDR: reads data[3+n] for n < len-3; first bad index is len(data)
      if (ol < 4) return rerr(0, GPK_ERR_REM_ADDR_LEN, ol);
      if (ol > slen) return rerr(0, GPK_ERR_PANIC_INDEX, slen, slen);
      break;
    case 5:  // MP_PRIO
      if (ol != 3 && ol != 4) return rerr(0, GPK_ERR_MP_PRIO_LEN, ol);
      if (ol == 4) GPK_IDX(3);
      break;
    case 6:  // MP_FAIL
      if (ol != 12) return rerr(0, GPK_ERR_MP_FAIL_LEN, ol);
      GPK_SL(4, 12);
      break;
    case 7:  // MP_FASTCLOSE
      if (ol != 12) return rerr(0, GPK_ERR_MP_FASTCLOSE_LEN, ol);
      GPK_SL(4, 12);
      break;
    case 8:  // MP_TCPRST
      if (ol != 4) return rerr(0, GPK_ERR_MP_TCPRST_LEN, ol);
      GPK_IDX(3);
      break;
    default:
      break;
  }
  return rok(0, 0, ol, 0);
}
#undef GPK_IDX
#undef GPK_SL

// ---- layers/tcp.go:291-551, NextLayerType :591-597 --------------------------
template <class TT, class R>
__device__ __forceinline__ Res dec_tcp(const TT& T, const R& r, uint32_t off, uint32_t len,
                                       uint32_t caplen) {
  if (len < 20) return rerr(1, GPK_ERR_TCP_HDR_SHORT, len);
  uint32_t ports = rd32(r, off);
  uint32_t doff = rd8(r, off + 12) >> 4;
  if (doff < 5) return rerr(0, GPK_ERR_TCP_DOFF_SMALL, doff);
  uint32_t ds = doff * 4;
  if (ds > len) return rerr(1, GPK_ERR_TCP_DOFF_GT_LEN);
  uint32_t p = off + 20, slen = ds - 20, scap = caplen - p;
  while (slen > 0) {
    uint32_t t = rd8(r, p);
    if (t == 0) break;  // EndList, Padding = rest
    uint32_t ol = 1;
    if (t == 30) {
      Res x = mptcp_option(r, p, slen, scap);
      if (x.err) return x;
      ol = x.len;
      if (ol > slen) return rerr(0, GPK_ERR_PANIC_SLICE_B, ol, slen);  // data[OptionLength:] (tcp.go:548)
    } else if (t != 1) {
      if (slen < 2) return rerr(1, GPK_ERR_TCP_OPT_SHORT, slen);
      ol = rd8(r, p + 1);
      if (ol < 2) return rerr(0, GPK_ERR_TCP_OPT_LEN_SMALL, ol);
      if (ol > slen) return rerr(1, GPK_ERR_TCP_OPT_EXCEEDS, ol, slen);
    }
    p += ol;
    slen -= ol;
    scap -= ol;
  }
  return rok(0, off + ds, len - ds, T.tcp(ports));
}

// ---- layers/udp.go:30-56, :114-119 -----------------------------------------
template <class TT, class R>
__device__ __forceinline__ Res dec_udp(const TT& T, const R& r, uint32_t off, uint32_t len) {
  if (len < 8) return rerr(1, GPK_ERR_UDP_HDR_SHORT, len);
  uint32_t ports = rd32(r, off);
  uint32_t length = rd16(r, off + 4);
  uint32_t hlen = len, trunc = 0;
  if (length >= 8) {
    if (length > len) trunc = 1;
    else hlen = length;
  } else if (length != 0) {
    return rerr(0, GPK_ERR_UDP_TOO_SMALL, length);
  }
  return rok(trunc, off + 8, hlen - 8, T.udp(ports), hlen);
}

__device__ __forceinline__ uint32_t code_of(int32_t typ) {
  switch (typ) {
    case GPK_LT_ETHERNET: return GPK_CODE_ETHERNET;
    case GPK_LT_DOT1Q: return GPK_CODE_DOT1Q;
    case GPK_LT_IPV4: return GPK_CODE_IPV4;
    case GPK_LT_IPV6: return GPK_CODE_IPV6;
    case GPK_LT_IPV6_HOPBYHOP: return GPK_CODE_IPV6_HOPBYHOP;
    case GPK_LT_IPV6_ROUTING: return GPK_CODE_IPV6_ROUTING;
    case GPK_LT_IPV6_FRAGMENT: return GPK_CODE_IPV6_FRAGMENT;
    case GPK_LT_IPV6_DESTINATION: return GPK_CODE_IPV6_DESTINATION;
    case GPK_LT_TCP: return GPK_CODE_TCP;
    case GPK_LT_UDP: return GPK_CODE_UDP;
    case GPK_LT_PAYLOAD: return GPK_CODE_PAYLOAD;
    case GPK_LT_FRAGMENT: return GPK_CODE_FRAGMENT;
    default: return GPK_CODE_NONE;
  }
}


// ---- next-layer lookups ------------------------------------------------------
// A decoder's NextLayerType() yields a "type handle": GTab (global tables,
// any configuration) uses the LayerType itself; LTab (the compact copy in
// LDS, used whenever the parser's tables fit, see CompactGeom) uses an index
// into the parser's dictionary of distinct LayerTypes. Either way kind(h) is
// the registered DecodingLayer (parser.go:177-183 decoders map), lt(h) the
// LayerType and code(h) its 4-bit record code.
// TCP/UDP: the destination port's type unless that is Payload, then the
// source port's (tcp.go:591-597, udp.go:114-119).
struct GTab {
  const DevTables* T;
  __device__ __forceinline__ int32_t eth(uint32_t k) const { return T->ethertype[k]; }
  __device__ __forceinline__ int32_t ipp(uint32_t k) const { return T->ipprotocol[k]; }
  __device__ __forceinline__ int32_t frag() const { return GPK_LT_FRAGMENT; }
  __device__ __forceinline__ int32_t zero() const { return GPK_LT_ZERO; }
  __device__ __forceinline__ int32_t first(int64_t lt) const { return (int32_t)lt; }
  __device__ __forceinline__ int32_t tcp(uint32_t ports) const {
    int32_t lt = T->tcp_port[ports & 0xffff];
    return lt == GPK_LT_PAYLOAD ? T->tcp_port[ports >> 16] : lt;
  }
  __device__ __forceinline__ int32_t udp(uint32_t ports) const {
    int32_t lt = T->udp_port[ports & 0xffff];
    return lt == GPK_LT_PAYLOAD ? T->udp_port[ports >> 16] : lt;
  }
  __device__ __forceinline__ int kind(int32_t h) const {
    return (h >= 0 && h < GPK_MAX_LAYER_TYPE) ? (int)T->dispatch[h] : GPK_DEC_NONE;
  }
  __device__ __forceinline__ int32_t lt(int32_t h) const { return h; }
  __device__ __forceinline__ uint32_t code(int32_t h) const { return code_of(h); }
};

// Compact tables in LDS (dword offsets from the blob base). Lookup of a
// 16-bit key in an open-addressed table: home slot (k * 0x9E3779B1) >> shift,
// linear probing; the host records the longest probe so an absent key stops
// after at most that many slots. Entry = key | handle << 16, empty =
// 0xFFFFFFFF.
struct LTab {
  CompactGeom g;  // from the kernel arguments: scalar registers
  uint32_t base;  // LDS dword index of the blob
  __device__ __forceinline__ int32_t probe(uint32_t k, uint32_t off, uint32_t shift, uint32_t mask,
                                           uint32_t maxp, uint32_t def) const {
    uint32_t h = (k * 0x9E3779B1u) >> shift;
    for (uint32_t i = 0; i <= maxp; i++) {
      uint32_t e = gpk_smem[base + off + ((h + i) & mask)];  // off: from the blob base
      if (e == 0xffffffffu) break;  // empty (before the key test: key 0xFFFF)
      if ((e & 0xffffu) == k) return (int32_t)(e >> 16);
    }
    return (int32_t)def;
  }
  __device__ __forceinline__ int32_t eth(uint32_t k) const {
    return probe(k, g.eth_off, g.eth_shift, g.eth_mask, g.eth_probe, g.eth_def);
  }
  __device__ __forceinline__ int32_t ipp(uint32_t k) const {
    return (int32_t)((gpk_smem[base + kCtIpp + (k >> 2)] >> (8 * (k & 3))) & 0xff);
  }
  __device__ __forceinline__ int32_t frag() const { return (int32_t)g.frag_h; }
  __device__ __forceinline__ int32_t zero() const { return (int32_t)g.zero_h; }
  __device__ __forceinline__ int32_t first(int64_t) const { return (int32_t)g.first_h; }
  __device__ __forceinline__ int32_t port(uint32_t k, uint32_t t) const {
    return t ? probe(k, g.udp_off, g.udp_shift, g.udp_mask, g.udp_probe, g.udp_def)
             : probe(k, g.tcp_off, g.tcp_shift, g.tcp_mask, g.tcp_probe, g.tcp_def);
  }
  __device__ __forceinline__ int32_t tcp(uint32_t ports) const {
    int32_t h = port(ports & 0xffff, 0);
    return h == (int32_t)g.payload_h ? port(ports >> 16, 0) : h;
  }
  __device__ __forceinline__ int32_t udp(uint32_t ports) const {
    int32_t h = port(ports & 0xffff, 1);
    return h == (int32_t)g.payload_h ? port(ports >> 16, 1) : h;
  }
  __device__ __forceinline__ uint32_t kc(int32_t h) const {
    return (gpk_smem[base + kCtKc + ((uint32_t)h >> 2)] >> (8 * (h & 3))) & 0xff;
  }
  __device__ __forceinline__ int kind(int32_t h) const { return (int)(kc(h) & 15); }
  __device__ __forceinline__ int32_t lt(int32_t h) const { return (int32_t)gpk_smem[base + kCtVal + h]; }
  __device__ __forceinline__ uint32_t code(int32_t h) const { return kc(h) >> 4; }
};

// Most packet bytes a decoder's DecodeFromBytes reads past its offset
// (IPv4/TCP: 15-word headers incl. options; IPv6: the fixed header, its
// HopByHop TLVs always go through the mixed reader).
__device__ __forceinline__ uint32_t max_header(int kind) {
  switch (kind) {
    case GPK_DEC_ETHERNET: return 14;
    case GPK_DEC_DOT1Q: return 4;
    case GPK_DEC_IPV4: return 60;
    case GPK_DEC_IPV6: return 40;
    case GPK_DEC_IPV6_EXT: return 2;
    case GPK_DEC_TCP: return 60;
    case GPK_DEC_UDP: return 8;
    default: return 0;
  }
}


// Result of running the parser on one packet.
// Per decoder instance (gopacket keeps one struct per DecodingLayer, so the
// last successful DecodeFromBytes wins): the [start, end) of the data slice it
// was handed. Named registers, not an array: a runtime-indexed per-lane array
// would live in scratch memory.
struct Parse {
  uint64_t layers;
  uint32_t nlayers;
  uint32_t s_eth, e_eth, s_d1q, e_d1q, s_ip4, e_ip4, s_ip6, e_ip6;
  uint32_t s_ext, e_ext, s_tcp, e_tcp, s_udp, e_udp, s_app, e_app;
  uint32_t app_kind;  // GPK_DEC_PAYLOAD / GPK_DEC_FRAGMENT of s_app/e_app
  uint32_t dirty;     // bit per decoder kind: its struct was left mid-decode
  uint32_t last_net;  // GPK_DEC_IPV4 / GPK_DEC_IPV6 / 0
  uint32_t transport; // GPK_DEC_TCP / GPK_DEC_UDP / 0
  uint32_t udp_hlen;

  __device__ __forceinline__ void init() {
    layers = 0;
    nlayers = 0;
    s_eth = e_eth = s_d1q = e_d1q = s_ip4 = e_ip4 = s_ip6 = e_ip6 = GPK_LAYOUT_ABSENT;
    s_ext = e_ext = s_tcp = e_tcp = s_udp = e_udp = s_app = e_app = GPK_LAYOUT_ABSENT;
    app_kind = 0;
    dirty = 0;
    last_net = 0;
    transport = 0;
    udp_hlen = 0;
  }
  __device__ __forceinline__ void set(int kind, uint32_t s, uint32_t e) {
    switch (kind) {
      case GPK_DEC_ETHERNET: s_eth = s; e_eth = e; break;
      case GPK_DEC_DOT1Q: s_d1q = s; e_d1q = e; break;
      case GPK_DEC_IPV4: s_ip4 = s; e_ip4 = e; break;
      case GPK_DEC_IPV6: s_ip6 = s; e_ip6 = e; break;
      case GPK_DEC_IPV6_EXT: s_ext = s; e_ext = e; break;
      case GPK_DEC_TCP: s_tcp = s; e_tcp = e; break;
      case GPK_DEC_UDP: s_udp = s; e_udp = e; break;
      default: s_app = s; e_app = e; app_kind = kind; break;
    }
  }
  __device__ __forceinline__ uint32_t start(uint32_t kind) const {
    switch (kind) {
      case GPK_DEC_ETHERNET: return s_eth;
      case GPK_DEC_DOT1Q: return s_d1q;
      case GPK_DEC_IPV4: return s_ip4;
      case GPK_DEC_IPV6: return s_ip6;
      case GPK_DEC_IPV6_EXT: return s_ext;
      case GPK_DEC_TCP: return s_tcp;
      case GPK_DEC_UDP: return s_udp;
      default: return kind == app_kind ? s_app : GPK_LAYOUT_ABSENT;
    }
  }
  __device__ __forceinline__ uint32_t end(uint32_t kind) const {
    switch (kind) {
      case GPK_DEC_ETHERNET: return e_eth;
      case GPK_DEC_DOT1Q: return e_d1q;
      case GPK_DEC_IPV4: return e_ip4;
      case GPK_DEC_IPV6: return e_ip6;
      case GPK_DEC_IPV6_EXT: return e_ext;
      case GPK_DEC_TCP: return e_tcp;
      case GPK_DEC_UDP: return e_udp;
      default: return kind == app_kind ? e_app : GPK_LAYOUT_ABSENT;
    }
  }
};

// DecodeLayers: parser.go:303-317 + layers_decoder.go:60-79.
// FULL: also writes every decoded LayerType to list[] (gpk_decoded_list).
struct Outcome {
  uint32_t err, a0, a1, trunc;
};

template <bool FULL, class TT>
__device__ __forceinline__ Outcome run_parser(const KParams& P, const TT& T, const Rd& r, uint32_t caplen, Parse& q,
                                              int64_t* list = nullptr, uint32_t list_cap = 0) {
  q.init();
  Outcome out{0, 0, 0, 0};
  int kind = P.first_kind;  // host: decoder registered for P.first
  if (kind == GPK_DEC_NONE) {  // LayersDecoder :12-16: (first, nil), decoded untouched
    if (!P.ignore_unsupported) out.err = GPK_ERR_UNSUPPORTED, out.a0 = (uint32_t)P.first;
    return out;
  }
  int32_t typ = T.first(P.first);
  uint32_t off = 0, len = caplen;
  for (;;) {
    Res x;
    // Whole header (the most bytes this decoder may read) inside the LDS
    // window: branch-free LDS reads; otherwise the mixed reader.
    // IPv4/TCP: the header length field bounds the bytes read (options
    // included), so only that much has to be in the window.
    uint32_t need = max_header(kind);
    if (kind == GPK_DEC_IPV4 && off < r.win) {
      const uint32_t h = 4 * (lds8(r.lb + off) & 15);
      need = h > 20 ? h : 20;
    } else if (kind == GPK_DEC_TCP && off + 12 < r.win) {
      const uint32_t h = 4 * (lds8(r.lb + off + 12) >> 4);
      need = h > 20 ? h : 20;
    }
    const bool fast = off + need <= r.win;
    const RdL rl{r.lb};
    switch (kind) {
      case GPK_DEC_ETHERNET: x = fast ? dec_ethernet(T, rl, off, len) : dec_ethernet(T, r, off, len); break;
      case GPK_DEC_DOT1Q: x = fast ? dec_dot1q(T, rl, off, len) : dec_dot1q(T, r, off, len); break;
      case GPK_DEC_IPV4: x = fast ? dec_ipv4(T, rl, off, len) : dec_ipv4(T, r, off, len); break;
      case GPK_DEC_IPV6: x = fast ? dec_ipv6(T, rl, r, off, len) : dec_ipv6(T, r, r, off, len); break;
      case GPK_DEC_IPV6_EXT: x = fast ? dec_ipv6_ext(T, rl, off, len) : dec_ipv6_ext(T, r, off, len); break;
      case GPK_DEC_TCP: x = fast ? dec_tcp(T, rl, off, len, caplen) : dec_tcp(T, r, off, len, caplen); break;
      case GPK_DEC_UDP: x = fast ? dec_udp(T, rl, off, len) : dec_udp(T, r, off, len); break;
      default:  // gopacket.Payload / gopacket.Fragment (base.go:61-70, :115-124)
        x = rok(0, off + len, 0, T.zero());
        break;
    }
    out.trunc |= x.trunc;
    if (x.err) {
      q.dirty |= 1u << kind;
      out.err = x.err;
      out.a0 = x.a0;
      out.a1 = x.a1;
      return out;
    }
    if (q.nlayers < GPK_MAX_INLINE_LAYERS) q.layers |= (uint64_t)T.code(typ) << (4 * q.nlayers);
    if (FULL && q.nlayers < list_cap) list[q.nlayers] = T.lt(typ);
    q.nlayers++;
    q.set(kind, off, off + len);
    if (kind == GPK_DEC_UDP) q.udp_hlen = x.aux;
    if (kind == GPK_DEC_IPV4 || kind == GPK_DEC_IPV6) q.last_net = kind;
    if (kind == GPK_DEC_TCP || kind == GPK_DEC_UDP) q.transport = kind;
    typ = x.next;
    off = x.off;
    len = x.len;
    if (len == 0) return out;  // LayerPayload() empty: success (layers_decoder.go:71-73)
    kind = T.kind(typ);
    if (kind == GPK_DEC_NONE) {  // (typ, nil): UnsupportedLayerType unless typ == 0
      const int32_t lt = T.lt(typ);
      if (lt != GPK_LT_ZERO && !P.ignore_unsupported) out.err = GPK_ERR_UNSUPPORTED, out.a0 = (uint32_t)lt;
      return out;
    }
  }
}

// The common case of DecodeLayers as straight-line code: Ethernet, up to two
// Dot1Q tags, IPv4 without options/fragmentation or IPv6 without HopByHop,
// TCP (options other than MPTCP) or UDP, then Payload or an unregistered
// port type. Every header byte must sit in the LDS window. It fills Parse and
// Outcome exactly as run_parser would (same layer list, slices, last
// writers); anything else (errors, truncation, options that need the general
// decoders, other types) returns false and the lane runs run_parser.
#ifndef GPK_FAST
#define GPK_FAST 1
#endif
#ifndef GPK_FAST_TCP_NEED
#define GPK_FAST_TCP_NEED 20
#endif
// TCP options of the straight-line path (tcp.go:336-549 for well-formed
// option lists without MPTCP): EOL ends the list, NOP, TLVs of length >= 2
// inside the header. False sends the packet to the general decoder.
#ifndef GPK_FAST_SYN_OPTS
#define GPK_FAST_SYN_OPTS 1  // the Linux SYN option block checked as a pattern (no TLV walk; A/B r12: C1 -4..-9 %)
#endif
template <class R>
__device__ __forceinline__ bool tcp_options_ok(const R& rd, uint32_t off, uint32_t ds) {
  if (ds == 20) return true;
  if (ds == 32 && rd32(rd, off + 20) == 0x0101080au) return true;  // NOP, NOP, Timestamps
#if GPK_FAST_SYN_OPTS
  // Linux SYN: MSS (4), SACK permitted (2), Timestamps (10), NOP, window scale (3)
  if (ds == 40 && (rd32(rd, off + 20) & 0xffff0000u) == 0x02040000u && rd32(rd, off + 24) == 0x0402080au &&
      (rd32(rd, off + 36) & 0xffffff00u) == 0x01030300u)
    return true;
#endif
  for (uint32_t p = off + 20, e = off + ds; p < e;) {
    const uint32_t t = rd8(rd, p);
    if (t == 0) break;
    if (t == 1) {
      p++;
      continue;
    }
    if (t == 30 || p + 2 > e) return false;  // MPTCP / short: the general decoder
    const uint32_t ol = rd8(rd, p + 1);
    if (ol < 2 || p + ol > e) return false;
    p += ol;
  }
  return true;
}

template <class TT>
__device__ __forceinline__ bool fast_parser(const KParams& P, const TT& T, const Rd& r, uint32_t caplen, Parse& q,
                                            Outcome& out) {
  const RdL rl{r.lb};
  const uint32_t W = r.win, F = P.fast;
  q.init();
  if (caplen < 15 || W < 14) return false;
  uint32_t et = rd16(rl, 12);
  uint32_t off = 14, len = caplen - 14, n = 1;
  uint64_t codes = GPK_CODE_ETHERNET;
  q.s_eth = 0;
  q.e_eth = caplen;
#pragma unroll
  for (int v = 0; v < 2; v++) {  // Dot1Q / QinQ tags (dot1q.go:30-41)
    const bool tag = (et == 0x8100 && (F & GPK_FAST_D1Q)) || (et == 0x88a8 && (F & GPK_FAST_QINQ));
    if (!tag) break;
    if (len < 5 || off + 4 > W) return false;
    codes |= (uint64_t)GPK_CODE_DOT1Q << (4 * n++);
    q.s_d1q = off;
    q.e_d1q = off + len;
    et = rd16(rl, off + 2);
    off += 4;
    len -= 4;
  }
  uint32_t proto;
  if (et == 0x0800 && (F & GPK_FAST_IP4)) {  // ip4.go:178-271, no options
    if (len < 20 || off + 20 > W) return false;
    const uint32_t b0 = rd8(rl, off), length = rd16(rl, off + 2), ff = rd16(rl, off + 6);
    if ((b0 & 15) != 5 || length < 20 || length > len || (ff & 0x3fff)) return false;
    proto = rd8(rl, off + 9);
    codes |= (uint64_t)GPK_CODE_IPV4 << (4 * n++);
    q.s_ip4 = off;
    q.e_ip4 = off + len;
    q.last_net = GPK_DEC_IPV4;
    off += 20;
    len = length - 20;
  } else if (et == 0x86dd && (F & GPK_FAST_IP6)) {  // ip6.go:221-278, no HopByHop
    if (len < 40 || off + 40 > W) return false;
    const uint32_t length = rd16(rl, off + 4);
    proto = rd8(rl, off + 6);
    if (proto == 0 || length == 0 || length > len - 40) return false;
    codes |= (uint64_t)GPK_CODE_IPV6 << (4 * n++);
    q.s_ip6 = off;
    q.e_ip6 = off + len;
    q.last_net = GPK_DEC_IPV6;
    off += 40;
    len = length;
  } else {
    return false;
  }
  if (len == 0) return false;
  int32_t h;
  uint32_t poff, plen;
  if (proto == 6 && (F & GPK_FAST_TCP)) {  // tcp.go:291-551
    // the header's first GPK_FAST_TCP_NEED bytes must be in the window: every
    // field an output reads (ports, data offset, flags; the checksum at 16-17
    // goes through the mixed reader) lies there, the urgent pointer (18-19) is
    // never read
    if (len < 20 || off + GPK_FAST_TCP_NEED > W) return false;
    const uint32_t ds = (rd8(rl, off + 12) >> 4) * 4;
    if (ds < 20 || ds > len) return false;
    // options: the block NOP, NOP, Timestamps (kind 8, length 10) is well
    // formed as it stands, anything else walks the TLVs; option bytes past
    // the window (tags + IPv6 push them there) come from global memory
    const bool opts_ok = off + ds <= W ? tcp_options_ok(rl, off, ds) : tcp_options_ok(r, off, ds);
    if (!opts_ok) return false;
    codes |= (uint64_t)GPK_CODE_TCP << (4 * n++);
    q.s_tcp = off;
    q.e_tcp = off + len;
    q.transport = GPK_DEC_TCP;
    h = T.tcp(rd32(rl, off));
    poff = off + ds;
    plen = len - ds;
  } else if (proto == 17 && (F & GPK_FAST_UDP)) {  // udp.go:30-56
    if (len < 8 || off + 8 > W) return false;
    const uint32_t length = rd16(rl, off + 4);
    uint32_t hlen = len;
    if (length >= 8) {
      if (length > len) return false;
      hlen = length;
    } else if (length != 0) {
      return false;
    }
    codes |= (uint64_t)GPK_CODE_UDP << (4 * n++);
    q.s_udp = off;
    q.e_udp = off + len;
    q.transport = GPK_DEC_UDP;
    q.udp_hlen = hlen;
    h = T.udp(rd32(rl, off));
    poff = off + 8;
    plen = hlen - 8;
  } else {
    return false;
  }
  if (plen != 0) {  // layers_decoder.go:71-79
    const int k = T.kind(h);
    if (k == GPK_DEC_PAYLOAD) {  // gopacket.Payload (base.go:61-70)
      codes |= (uint64_t)GPK_CODE_PAYLOAD << (4 * n++);
      q.s_app = poff;
      q.e_app = poff + plen;
      q.app_kind = GPK_DEC_PAYLOAD;
    } else if (k == GPK_DEC_NONE) {  // (typ, nil): UnsupportedLayerType unless typ == 0
      const int32_t lt = T.lt(h);
      if (lt != GPK_LT_ZERO && !P.ignore_unsupported) out.err = GPK_ERR_UNSUPPORTED, out.a0 = (uint32_t)lt;
    } else {
      return false;
    }
  }
  q.layers = codes;
  q.nlayers = n;
  return true;
}

__device__ __forceinline__ bool clean(const Parse& q, uint32_t kind) {
  return q.start(kind) != GPK_LAYOUT_ABSENT && !((q.dirty >> kind) & 1);
}

// FoldChecksum, checksum.go:53-58
__device__ __forceinline__ uint32_t fold(uint32_t c) {
  c = (c >> 16) + (c & 0xffff);
  c = (c >> 16) + (c & 0xffff);
  return (~c) & 0xffff;
}

// FNV-1a 64 step (flows.go:60-70): h = (h ^ b) * 0x100000001b3 mod 2^64.
// With x = lo ^ b: x * 0x1b3 + ((hi * 0x1b3 + (x << 8)) << 32), i.e. one
// v_mul_lo_u32, one v_lshl_add_u32 and one v_mad_u64_u32 whose 64-bit addend
// carries the high word (the b byte only reaches the low word).
__device__ __forceinline__ uint64_t fnv_step(uint64_t h, uint32_t b) {
  const uint32_t x = (uint32_t)h ^ b, hi = (uint32_t)(h >> 32);
  const uint32_t s = hi * 0x1b3u + (x << 8);
  return (uint64_t)x * 0x1b3u + ((uint64_t)s << 32);
}
template <class R>
__device__ __forceinline__ uint64_t fnv_bytes(const R& r, uint32_t p, uint32_t n) {
  uint64_t h = 14695981039346656037ull;
  for (uint32_t i = 0; i < n; i++) h = fnv_step(h, rd8(r, p + i));
  return h;
}
// Flow.FastHash flows.go:167-174
__device__ __forceinline__ uint64_t flow_hash(uint64_t hs, uint64_t hd, uint32_t typ) {
  return ((hs + hd) ^ (uint64_t)typ) * 1099511628211ull;
}
// The three Flow.FastHash values of a packet (flows.go:167-174):
//   LinkFlow       ethernet.go:38-40  source MAC at e0+6, destination at e0 (EndpointMAC = 3)
//   NetworkFlow    ip4.go:63-65 / ip6.go:49-51  addresses at ns+12 (4 bytes each, EndpointIPv4 = 1)
//                  or ns+8 (16 bytes each, EndpointIPv6 = 2)
//   TransportFlow  tcp.go:614-616 / udp.go:132-134  ports at t0, t0+2 (4 / 5)
// All six FNV chains are computed in one block of straight-line code so
// their multiplies interleave; the caller keeps the ones whose layer exists.
// Addresses are hashed one dword per step: 1 dword for IPv4, 4 for IPv6,
// with the count uniform over the active lanes (IPv4 lanes keep the state
// after their first dword), so a wave holding both runs 16 steps per address,
// not 4 + 16. Bytes past the LDS window (deep stacks) go through the mixed
// reader.
__device__ __forceinline__ void fnv_dword(uint64_t& h, uint32_t w, int j0, int j1) {
#pragma unroll
  for (int j = j0; j < j1; j++) h = fnv_step(h, (w >> (8 * j)) & 0xffu);
}
// fl / fn / ft: which of the three layers exist (their offsets are 0 otherwise
// and their chains hash window bytes that are then dropped).
__device__ __forceinline__ void flow_hashes(const Rd& r, bool fl, uint32_t e0, bool fn, uint32_t ns, bool v6, bool ft,
                                            uint32_t t0, uint32_t tcode, uint64_t& lflow, uint64_t& nflow,
                                            uint64_t& tflow) {
  constexpr uint64_t kBasis = 14695981039346656037ull;
  const uint32_t n = v6 ? 16u : 4u, a = ns + (v6 ? 8u : 12u);
  const bool inwin = (!fl || e0 + 12 <= r.win) && (!fn || a + 2 * n <= r.win) && (!ft || t0 + 4 <= r.win);
  uint64_t ls = kBasis, ld = kBasis, ts = kBasis, td = kBasis, hs = kBasis, hd = kBasis;
  if (__ballot(!inwin)) {  // rare: a field past the window; only the layers that exist are read
    if (!inwin && fl) {
      ls = fnv_bytes(r, e0 + 6, 6);
      ld = fnv_bytes(r, e0, 6);
    }
    if (!inwin && fn) {
      hs = fnv_bytes(r, a, n);
      hd = fnv_bytes(r, a + n, n);
    }
    if (!inwin && ft) {
      ts = fnv_bytes(r, t0, 2);
      td = fnv_bytes(r, t0 + 2, 2);
    }
  }
  if (inwin) {
    const uint32_t wl0 = lds32u(r.lb + e0), wl1 = lds32u(r.lb + e0 + 4), wl2 = lds32u(r.lb + e0 + 8);
    const uint32_t wt = lds32u(r.lb + t0);
    const uint32_t ws0 = lds32u(r.lb + a), wd0 = lds32u(r.lb + a + n);
    fnv_dword(ld, wl0, 0, 4);
    fnv_dword(ld, wl1, 0, 2);
    fnv_dword(ls, wl1, 2, 4);
    fnv_dword(ls, wl2, 0, 4);
    fnv_dword(ts, wt, 0, 2);
    fnv_dword(td, wt, 2, 4);
    fnv_dword(hs, ws0, 0, 4);
    fnv_dword(hd, wd0, 0, 4);
    if (__ballot(inwin && v6)) {
      const uint64_t hs4 = hs, hd4 = hd;
#pragma unroll
      for (uint32_t k = 1; k < 4; k++) {
        fnv_dword(hs, lds32u(r.lb + a + 4 * k), 0, 4);
        fnv_dword(hd, lds32u(r.lb + a + n + 4 * k), 0, 4);
      }
      if (!v6) {
        hs = hs4;
        hd = hd4;
      }
    }
  }
  lflow = flow_hash(ls, ld, 3);
  nflow = flow_hash(hs, hd, v6 ? 2u : 1u);
  tflow = flow_hash(ts, td, tcode);
}

}  // namespace gpk

// gpk_fields.h — the gpk_fields record of one packet (include/gpk.h) as 32
// dwords, from the header bytes of each decoder's last slice. Shared by the
// layout-driven extraction kernel (gpk_fields.hip, gpk_extract_fields) and the
// decode kernel's fused-fields variant (gpk_kernels.hip, gpk_decode_batch_fields),
// which reads the same bytes from its LDS header window during the decode.
//
// H: a header reader of one packet with
//   u8(p)    the byte at packet offset p
//   be16(p)  the big-endian 16 bits at p (reads bytes p, p+1 only)
//   u32(p)   the 4 bytes at p in memory order (little-endian value)
// Slot k = GPK_DEC_* - 1 of the layout (Payload and Fragment share slot 7).
//
// Field by field this restates:
//   Ethernet  layers/ethernet.go:42-55  (EthernetType < 0x0600: Length, LLC)
//   Dot1Q     layers/dot1q.go:28-41     (the tag control word, Type)
//   IPv4      layers/ip4.go:178-271     (Length 0 = the slice's length, TSO;
//                                       option starts, ip4.go:219-256)
//   IPv6      layers/ip6.go:221-278     (HopByHop option starts, ip6.go:509-526)
//   TCP       layers/tcp.go:292-313     (option starts, tcp.go:336-549)
//   UDP       layers/udp.go:30-43
#ifndef GPK_FIELDS_H
#define GPK_FIELDS_H

#include <hip/hip_runtime.h>

#include "../../include/gpk.h"

namespace gpkf {

// Where the options of a successfully decoded IPv4 or TCP header start:
// bit k set = an option starts at header byte 20 + k (k < 40), walked as the
// reference's loops walk them (End of options: stop; No-op: 1 byte; any other
// kind: its length byte, which the successful decode has checked to stay
// inside the header: ip4.go:219-256, tcp.go:336-549). hlen: the header length
// (IHL * 4 or DataOffset * 4).
template <class H>
__device__ __forceinline__ uint64_t option_map(const H& h, uint32_t s, uint32_t hlen) {
  uint64_t map = 0;
  const uint32_t n = hlen > 20 ? hlen - 20 : 0u;
  for (uint32_t k = 0; k < n;) {
    map |= 1ull << k;
    const uint32_t t = h.u8(s + 20 + k);
    if (t == 0) break;
    const uint32_t len = t == 1 ? 1u : h.u8(s + 21 + k);
    k += len ? len : n;  // (a zero length never decodes successfully)
  }
  return map;
}

// Where the options of the IPv6 layer's inline HopByHop header start (the
// header at IPv6 byte 40, ip6.go:244-246): bit k = an option at HopByHop byte
// 2 + k, walked as IPv6HopByHop.DecodeFromBytes walks them (ip6.go:509-526,
// TLVs :327-346: Pad1 is one byte, every other option its length byte + 2;
// the loop runs while the offset is below ActualLength = HeaderLength * 8 +
// 8). Only for HeaderLength <= 2 (ActualLength <= 24: every start, at byte
// 2 + k < 24, fits the 24 bits), else 0. s: the IPv6 start. The IPv6 decode succeeded, so every
// option it walked was inside the slice.
template <class H>
__device__ __forceinline__ uint32_t hbh_map(const H& h, uint32_t s) {
  const uint32_t hl = h.u8(s + 41);
  if (hl > 2) return 0;
  const uint32_t actual = hl * 8 + 8;
  uint32_t map = 0;
  for (uint32_t off = 2; off < actual;) {
    map |= 1u << (off - 2);
    const uint32_t t = h.u8(s + 40 + off);
    off += t == 0 ? 1u : h.u8(s + 41 + off) + 2u;
  }
  return map;
}

// present: bit k = layout slot k holds a slice; st[k]: its start (read only
// when present); ip4_end: the end of the IPv4 slice.
template <class H>
__device__ __forceinline__ void fields_words(const H& h, uint32_t present, const uint32_t (&st)[8], uint32_t ip4_end,
                                             uint32_t (&w)[32]) {
  // the HopByHop walk first, while no record word is live (no scratch in the fused kernel)
  uint32_t hmap = 0;
  if (present >> (GPK_DEC_IPV6 - 1) & 1u) {
    const uint32_t d = st[GPK_DEC_IPV6 - 1];
    if (h.u8(d + 6) == 0) hmap = hbh_map(h, d);  // NextHeader 0: the inline HopByHop, ip6.go:244-246
  }
#pragma unroll
  for (int k = 0; k < 32; k++) w[k] = 0;
  w[0] = present | hmap << 8;  // bytes 1-3: the HopByHop option map
  uint32_t ip4s = 0xFFu, tcps = 0xFFu;
  uint64_t ip4m = 0, tcpm = 0;
  if (present >> (GPK_DEC_ETHERNET - 1) & 1u) {  // ethernet.go:46-55
    const uint32_t d = st[GPK_DEC_ETHERNET - 1];
    uint32_t et = h.be16(d + 12), len = 0;
    if (et < 0x0600) {
      len = et;
      et = 0;  // EthernetTypeLLC
    }
    w[1] = et | len << 16;
    w[2] = h.u32(d);  // DstMAC, SrcMAC: bytes 8..19 of the record
    w[3] = h.u32(d + 4);
    w[4] = h.u32(d + 8);
  }
  if (present >> (GPK_DEC_DOT1Q - 1) & 1u) {  // dot1q.go:33-37
    const uint32_t d = st[GPK_DEC_DOT1Q - 1];
    w[5] = h.be16(d) | h.be16(d + 2) << 16;
  }
  if (present >> (GPK_DEC_IPV4 - 1) & 1u) {  // ip4.go:183-193, 257-267
    const uint32_t d = st[GPK_DEC_IPV4 - 1];
    const uint32_t b0 = h.u32(d);  // bytes 0..3
    uint32_t length = (b0 >> 16 & 0xffu) << 8 | b0 >> 24;
    if (length == 0) length = (ip4_end - d) & 0xffffu;
    const uint32_t b4 = h.u32(d + 4), b8 = h.u32(d + 8);  // Id, flags|frag; TTL, Protocol, Checksum
    w[6] = (b0 & 0xffu) >> 4 | (b0 & 0x0fu) << 8 | (b0 >> 8 & 0xffu) << 16 | (b8 & 0xffu) << 24;
    w[7] = length | ((b4 & 0xffu) << 8 | (b4 >> 8 & 0xffu)) << 16;
    w[8] = ((b4 >> 16 & 0xffu) << 8 | b4 >> 24) | (b8 >> 8 & 0xffu) << 16;
    w[9] = (b8 >> 16 & 0xffu) << 8 | b8 >> 24;
    w[12] = h.u32(d + 12);
    w[13] = h.u32(d + 16);
    ip4s = d < 0xFFu ? d : 0xFFu;
    ip4m = option_map(h, d, (b0 & 0x0fu) * 4);
  }
  if (present >> (GPK_DEC_IPV6 - 1) & 1u) {  // ip6.go:225-234
    const uint32_t d = st[GPK_DEC_IPV6 - 1];
    const uint32_t h0 = __builtin_bswap32(h.u32(d)), b4 = h.u32(d + 4);
    w[8] |= (h0 >> 28) << 24;                                          // Version
    w[9] |= (h0 >> 20 & 0xffu) << 16 | (b4 >> 16 & 0xffu) << 24;        // TrafficClass, NextHeader
    w[10] = h0 & 0x000fffffu;                                          // FlowLabel
    w[11] = ((b4 & 0xffu) << 8 | (b4 >> 8 & 0xffu)) | (b4 >> 24) << 16;  // Length, HopLimit
#pragma unroll
    for (int k = 0; k < 4; k++) {
      w[14 + k] = h.u32(d + 8 + 4 * k);
      w[18 + k] = h.u32(d + 24 + 4 * k);
    }
  }
  if (present >> (GPK_DEC_TCP - 1) & 1u) {  // tcp.go:296-313
    const uint32_t d = st[GPK_DEC_TCP - 1];
    const uint32_t b0 = h.u32(d), b12 = h.u32(d + 12);  // ports; DataOffset|NS, flags, Window
    w[11] |= (b12 & 0xffu) >> 4 << 24;
    w[22] = ((b0 & 0xffu) << 8 | (b0 >> 8 & 0xffu)) | ((b0 >> 16 & 0xffu) << 8 | b0 >> 24) << 16;
    w[23] = __builtin_bswap32(h.u32(d + 4));
    w[24] = __builtin_bswap32(h.u32(d + 8));
    w[25] = (b12 >> 8 & 0xffu) | (b12 & 1u) << 8 | ((b12 >> 16 & 0xffu) << 8 | b12 >> 24) << 16;
    w[26] = h.be16(d + 16) | h.be16(d + 18) << 16;
    tcps = d < 0xFFu ? d : 0xFFu;
    tcpm = option_map(h, d, (b12 & 0xffu) >> 4 << 2);
  }
  if (present >> (GPK_DEC_UDP - 1) & 1u) {  // udp.go:34-41
    const uint32_t d = st[GPK_DEC_UDP - 1];
    const uint32_t b0 = h.u32(d), b4 = h.u32(d + 4);
    w[27] = ((b0 & 0xffu) << 8 | (b0 >> 8 & 0xffu)) | ((b0 >> 16 & 0xffu) << 8 | b0 >> 24) << 16;
    w[28] = ((b4 & 0xffu) << 8 | (b4 >> 8 & 0xffu)) | ((b4 >> 16 & 0xffu) << 8 | b4 >> 24) << 16;
  }
  // bytes 116-127: ip4_start, tcp_start, the two 40-bit option maps
  w[29] = ip4s | tcps << 8 | (uint32_t)(ip4m & 0xffffu) << 16;
  w[30] = (uint32_t)(ip4m >> 16 & 0xffffffu) | (uint32_t)(tcpm & 0xffu) << 24;
  w[31] = (uint32_t)(tcpm >> 8);
}

}  // namespace gpkf

#endif  // GPK_FIELDS_H

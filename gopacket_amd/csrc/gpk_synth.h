// gpk_synth.h — deterministic synthetic packet batches for the benchmark
// configurations (BASELINE.json configs C2-C4).
//
// Bench/test infrastructure, not part of the decode path. Every packet is a
// pure function of (config, index): splitmix64 seeded with
// 0x9E3779B97F4A7C15 ^ i, so the device generator (gpk_synth.hip) and the
// host copy used for oracle sampling produce identical bytes.
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define GPK_HD __host__ __device__ __forceinline__
#else
#define GPK_HD static inline
#endif

#define GPK_SYNTH_C2_UDP64 2    /* 64 B Eth/IPv4/UDP, 10% zero UDP checksum      */
#define GPK_SYNTH_C3_TCP1500 3  /* 1500 B Eth/IPv4/TCP, 50% NOP,NOP,TS options    */
#define GPK_SYNTH_C4_IMIX 4     /* 64/594/1518 7:4:1, Dot1Q/QinQ, IPv4/IPv6(+HBH) */
#define GPK_SYNTH_C6_FLOWS 6    /* C4's frames with endpoints from 2^20 skewed flows in both
                                   directions, SYN/FIN/RST and empty-payload TCP, 5% IPv4
                                   fragments (row (f)3: flow-keyed grouping)               */

namespace gpk_synth {

GPK_HD uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Rng {
  uint64_t s;
  GPK_HD uint64_t next() {
    s += 0x9E3779B97F4A7C15ull;
    return mix64(s);
  }
};

GPK_HD uint64_t seed_of(uint64_t i) { return 0x9E3779B97F4A7C15ull ^ i; }

// Payload bytes: 8-byte group g of packet i (packet-relative positions 8g..8g+7).
GPK_HD uint64_t payload_group(uint64_t i, uint32_t g) {
  return mix64(seed_of(i) * 0xD1B54A32D192ED03ull + (uint64_t)g + 1);
}
GPK_HD uint32_t payload_byte(uint64_t i, uint32_t p) {
  return (uint32_t)(payload_group(i, p >> 3) >> ((p & 7) * 8)) & 0xff;
}

// Ports >= 1024 that map to an application LayerType (layers/ports.go): the
// generator avoids them so the next layer is gopacket.Payload.
GPK_HD bool tcp_port_taken(uint32_t p) {
  return p == 2222 || p == 3868 || p == 5061 || p == 5082 || p == 5083 || p == 44818;
}
GPK_HD bool udp_port_taken(uint32_t p) {
  return p == 1812 || p == 2123 || p == 2152 || p == 2222 || p == 3784 || p == 3868 || p == 4789 ||
         p == 5060 || p == 5082 || p == 5083 || p == 6081 || p == 6343 || p == 44818;
}
GPK_HD uint32_t pick_port(Rng& r, bool udp) {
  for (;;) {
    uint32_t p = 1024 + (uint32_t)(r.next() % (65536 - 1024));
    if (!(udp ? udp_port_taken(p) : tcp_port_taken(p))) return p;
  }
}

// Packet description: everything but the payload bytes.
struct Desc {
  uint32_t len;         // frame size (caplen)
  uint32_t ntags;       // 0, 1 (802.1Q) or 2 (QinQ 0x88a8 + 0x8100)
  uint32_t v6;          // IPv6 network layer
  uint32_t hbh;         // IPv6 with an 8-byte HopByHop PadN header
  uint32_t udp;         // UDP (else TCP)
  uint32_t doff;        // TCP data offset (words)
  uint32_t l4_zero;     // UDP checksum transmitted as 0
  uint32_t corrupt;     // 0 none, 1 IPv4 header checksum, 2 L4 checksum
  uint8_t hdr[128];     // header bytes (checksums filled in by build())
  uint32_t hlen;        // header bytes before the payload
  uint32_t l3;          // offset of the network header
  uint32_t l4;          // offset of the transport header
  uint32_t end;         // end of the IP datagram (< len: Ethernet padding follows)
};

GPK_HD void put16(uint8_t* b, uint32_t v) {
  b[0] = (uint8_t)(v >> 8);
  b[1] = (uint8_t)v;
}
GPK_HD void put32(uint8_t* b, uint32_t v) {
  put16(b, v >> 16);
  put16(b + 2, v & 0xffff);
}

GPK_HD uint32_t frame_len(int cfg, uint64_t i) {
  if (cfg == GPK_SYNTH_C2_UDP64) return 64;
  if (cfg == GPK_SYNTH_C3_TCP1500) return 1500;
  Rng r{seed_of(i)};
  uint32_t k = (uint32_t)(r.next() % 12);  // IMIX 7:4:1
  return k < 7 ? 64 : (k < 11 ? 594 : 1518);
}

// Header layout + field values (payload-independent part).
GPK_HD void describe(int cfg, uint64_t i, Desc& d) {
  Rng r{seed_of(i)};
  uint64_t r0 = r.next();
  d.len = frame_len(cfg, i);
  d.ntags = 0;
  d.v6 = 0;
  d.hbh = 0;
  d.udp = cfg == GPK_SYNTH_C2_UDP64;
  d.doff = 5;
  d.l4_zero = 0;
  d.corrupt = 0;
  d.end = d.len;
  uint64_t r1 = r.next(), r2 = r.next(), r3 = r.next();
  if (cfg == GPK_SYNTH_C2_UDP64) {
    d.l4_zero = (r1 % 10) == 0;
    d.corrupt = (r2 % 1024) == 0 ? 1 : 0;
  } else if (cfg == GPK_SYNTH_C3_TCP1500) {
    d.doff = (r1 & 1) ? 8 : 5;
    d.corrupt = (r2 % 1024) == 0 ? 2 : 0;
  } else {
    uint32_t t = (uint32_t)(r1 % 10);
    d.ntags = t < 6 ? 0 : (t < 9 ? 1 : 2);
    d.v6 = (r1 >> 8) % 5 == 0;
    d.hbh = d.v6 && ((r1 >> 16) % 100) == 0;
    d.udp = ((r1 >> 24) % 10) >= 7;
    uint32_t l3room = d.len - 14 - 4 * d.ntags;
    if (d.v6 && l3room < 40 + 8 * d.hbh + 8) d.v6 = d.hbh = 0;  // IPv6 + at least UDP must fit
    uint32_t l4room = l3room - (d.v6 ? 40 + 8 * d.hbh : 20);
    if (!d.udp && l4room < 20) d.udp = 1;
    uint32_t c = (uint32_t)(r2 % 1024);
    d.corrupt = c == 0 ? (d.v6 ? 2 : 1) : (c == 1 ? 2 : 0);
    d.l4_zero = d.udp && ((r2 >> 16) % 10) == 0;
  }
  (void)r0;
  uint8_t* h = d.hdr;
  for (int k = 0; k < 128; k++) h[k] = 0;
  // Ethernet: random unicast MACs
  uint64_t m = r.next();
  for (int k = 0; k < 6; k++) h[k] = (uint8_t)(m >> (8 * k));
  h[0] &= 0xfe;
  m = r.next();
  for (int k = 0; k < 6; k++) h[6 + k] = (uint8_t)(m >> (8 * k));
  h[6] &= 0xfe;
  uint32_t p = 12;
  if (d.ntags == 2) {
    put16(h + p, 0x88a8);
    put16(h + p + 2, (uint32_t)(r3 & 0x0fff));
    p += 4;
  }
  if (d.ntags >= 1) {
    put16(h + p, 0x8100);
    put16(h + p + 2, (uint32_t)((r3 >> 12) & 0xefff));
    p += 4;
  }
  put16(h + p, d.v6 ? 0x86dd : 0x0800);
  p += 2;
  d.l3 = p;
  uint32_t l3len = d.len - p;
  uint32_t proto = d.udp ? 17 : 6;
  if (!d.v6) {
    h[p] = 0x45;
    put16(h + p + 2, l3len);
    put16(h + p + 4, (uint32_t)(i & 0xffff));
    put16(h + p + 6, 0x4000);  // DF
    h[p + 8] = 64;
    h[p + 9] = (uint8_t)proto;
    uint64_t a = r.next();
    put32(h + p + 12, 0x0a000000u | (uint32_t)(a & 0xffffff));
    put32(h + p + 16, 0x0a000000u | (uint32_t)((a >> 24) & 0xffffff));
    d.l4 = p + 20;
  } else {
    uint64_t a = r.next();
    put32(h + p, 0x60000000u | (uint32_t)(a & 0x0fffffff));
    put16(h + p + 4, l3len - 40);
    h[p + 6] = d.hbh ? 0 : (uint8_t)proto;
    h[p + 7] = 64;
    for (int k = 0; k < 2; k++) {
      uint64_t b = r.next(), c = r.next();
      uint8_t* ip = h + p + 8 + 16 * k;
      put32(ip, 0x20010db8u);
      put32(ip + 4, (uint32_t)b);
      put32(ip + 8, (uint32_t)(b >> 32));
      put32(ip + 12, (uint32_t)c);
    }
    d.l4 = p + 40;
    if (d.hbh) {  // HopByHop: NextHeader, HdrExtLen 0, PadN(4)
      uint8_t* x = h + d.l4;
      x[0] = (uint8_t)proto;
      x[1] = 0;
      x[2] = 1;
      x[3] = 4;
      d.l4 += 8;
    }
  }
  uint32_t l4 = d.l4;
  put16(h + l4, pick_port(r, d.udp));
  put16(h + l4 + 2, pick_port(r, d.udp));
  if (d.udp) {
    put16(h + l4 + 4, d.len - l4);
    d.hlen = l4 + 8;
  } else {
    uint64_t a = r.next();
    put32(h + l4 + 4, (uint32_t)a);
    put32(h + l4 + 8, (uint32_t)(a >> 32));
    h[l4 + 12] = (uint8_t)(d.doff << 4);
    h[l4 + 13] = 0x18;  // ACK | PSH
    put16(h + l4 + 14, (uint32_t)(r.next() & 0xffff));
    if (d.doff == 8) {  // NOP, NOP, Timestamps (as testSimpleTCPPacket)
      uint64_t ts = r.next();
      h[l4 + 20] = 1;
      h[l4 + 21] = 1;
      h[l4 + 22] = 8;
      h[l4 + 23] = 10;
      put32(h + l4 + 24, (uint32_t)ts);
      put32(h + l4 + 28, (uint32_t)(ts >> 32));
    }
    d.hlen = l4 + 4 * d.doff;
  }
  if (cfg == GPK_SYNTH_C6_FLOWS) {  // endpoints from a flow pool, TCP flags, fragments
    const uint64_t fr = r.next();
    const uint64_t u = fr & 0xfffff;
    const uint64_t flow = (u * u * u) >> 40;  // heavy-tailed: a few elephant flows, many mice
    const uint64_t fh = mix64(flow * 0x9E3779B97F4A7C15ull + 0x51ED270B1F2A3C5Dull);
    const bool swap = (fr >> 20) & 1;
    uint32_t pa = 1024 + (uint32_t)((fh >> 32) % 64512), pb = 1024 + (uint32_t)((fh >> 48) % 64512);
    while (d.udp ? udp_port_taken(pa) : tcp_port_taken(pa)) pa++;
    while (d.udp ? udp_port_taken(pb) : tcp_port_taken(pb)) pb++;
    put16(h + l4, swap ? pb : pa);
    put16(h + l4 + 2, swap ? pa : pb);
    if (!d.v6) {
      const uint32_t a = 0x0a000000u | (uint32_t)(fh & 0xffffff), b = 0x0a000000u | (uint32_t)((fh >> 24) & 0xffffff);
      put32(h + d.l3 + 12, swap ? b : a);
      put32(h + d.l3 + 16, swap ? a : b);
      if (((fr >> 28) % 20) == 0) {  // a fragment: DF cleared, MF and/or an offset
        const uint32_t k = (uint32_t)(fr >> 33);
        const uint32_t off = (k & 1) ? 0u : 1u + ((k >> 1) % 180u);
        const uint32_t mf = (off == 0 || ((k >> 9) & 1)) ? 0x2000u : 0u;
        put16(h + d.l3 + 6, mf | off);
        put16(h + d.l3 + 4, (uint32_t)((fh >> 8) + ((k >> 10) & 3)) & 0xffff);
      }
    } else {
      const uint64_t g = mix64(fh);
      uint8_t* s6 = h + d.l3 + (swap ? 24 : 8);
      uint8_t* d6 = h + d.l3 + (swap ? 8 : 24);
      put32(s6, 0x20010db8u); put32(s6 + 4, (uint32_t)fh); put32(s6 + 8, (uint32_t)(fh >> 32)); put32(s6 + 12, (uint32_t)g);
      put32(d6, 0x20010db8u); put32(d6 + 4, (uint32_t)(g >> 32)); put32(d6 + 8, (uint32_t)flow); put32(d6 + 12, 0x1u);
    }
    if (!d.udp) {
      const uint32_t k = (uint32_t)((fr >> 40) % 100);
      h[l4 + 13] = k < 2 ? 0x02 : (k < 3 ? 0x11 : (k < 4 ? 0x04 : 0x18));  // SYN, FIN|ACK, RST, ACK|PSH
      if (k >= 4 && k < 14) {  // header-only segment, the rest of the frame is padding
        h[l4 + 13] = 0x10;  // ACK
        d.end = l4 + 4 * d.doff;
        if (!d.v6) put16(h + d.l3 + 2, d.end - d.l3);
        else put16(h + d.l3 + 4, d.end - d.l3 - 40);
      }
    }
  }
}

GPK_HD uint32_t byte_at(const Desc& d, uint64_t i, uint32_t p) {
  return p < d.hlen ? d.hdr[p] : payload_byte(i, p);
}

GPK_HD uint32_t fold16(uint32_t c) {
  while (c > 0xffff) c = (c >> 16) + (c & 0xffff);
  return (~c) & 0xffff;
}

// Fill in checksums (IPv4 header, TCP/UDP with pseudo-header) in d.hdr.
GPK_HD void finish(Desc& d, uint64_t i) {
  uint8_t* h = d.hdr;
  uint32_t proto = d.udp ? 17 : 6;
  if (!d.v6) {
    uint32_t s = 0;
    for (uint32_t k = 0; k < 20; k += 2) s += (uint32_t)h[d.l3 + k] << 8 | h[d.l3 + k + 1];
    uint32_t c = fold16(s);
    if (d.corrupt == 1) c ^= 0x0100;
    put16(h + d.l3 + 10, c);
  }
  uint32_t l4len = d.end - d.l4;
  uint32_t s = proto + l4len;
  if (!d.v6) {
    for (uint32_t k = 12; k < 20; k += 2) s += (uint32_t)h[d.l3 + k] << 8 | h[d.l3 + k + 1];
  } else {
    for (uint32_t k = 8; k < 40; k += 2) s += (uint32_t)h[d.l3 + k] << 8 | h[d.l3 + k + 1];
  }
  uint32_t p = d.l4;
  for (; p < d.hlen; p++) s += (uint32_t)h[p] << (((p - d.l4) & 1) ? 0 : 8);
  for (; p < d.end && (p & 7); p++) s += payload_byte(i, p) << (((p - d.l4) & 1) ? 0 : 8);
  for (; p + 8 <= d.end; p += 8) {
    uint64_t w = payload_group(i, p >> 3);
    uint32_t e = 0, o = 0;  // bytes at even / odd packet positions
    for (int k = 0; k < 8; k += 2) {
      e += (uint32_t)(w >> (8 * k)) & 0xff;
      o += (uint32_t)(w >> (8 * k + 8)) & 0xff;
    }
    s += ((p - d.l4) & 1) ? (o << 8) + e : (e << 8) + o;
  }
  for (; p < d.end; p++) s += payload_byte(i, p) << (((p - d.l4) & 1) ? 0 : 8);
  uint32_t c = fold16(s);
  if (d.udp && c == 0) c = 0xffff;  // RFC768 (udp.go:95-100)
  if (d.l4_zero) c = 0;
  if (d.corrupt == 2) c ^= 0x0100;
  put16(h + d.l4 + (d.udp ? 6 : 16), c);
}

// Emit the packet bytes in order: sink(p, byte).
template <class Sink>
GPK_HD void emit(const Desc& d, uint64_t i, Sink& sink) {
  uint32_t p = 0;
  for (; p < d.hlen; p++) sink(p, d.hdr[p]);
  for (; p < d.len && (p & 7); p++) sink(p, payload_byte(i, p));
  for (; p < d.len; p += 8) {
    uint64_t w = payload_group(i, p >> 3);
    for (uint32_t k = 0; k < 8 && p + k < d.len; k++) sink(p + k, (uint32_t)(w >> (8 * k)) & 0xff);
  }
}

}  // namespace gpk_synth

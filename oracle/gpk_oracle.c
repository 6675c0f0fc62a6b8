/*
 * gpk_oracle.c — CPU restatement of gopacket's DecodingLayerParser fast path.
 * TEST INFRASTRUCTURE ONLY (see gpk_oracle.h). Never linked into gopacket_amd.
 *
 * Every function names the reference lines it restates. Go slices are modelled
 * as (off, len) views into the packet with cap = caplen - off: every slice on
 * this path keeps its capacity to the end of the packet buffer (reslicing
 * data[:n] keeps cap), and the packet buffer handed to DecodeLayers is taken
 * to have cap == len (what pcapgo.Reader / NgReader return, read.go:122-137).
 */
#include "gpk_oracle.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../gopacket_amd/csrc/gpk_registry_gen.h"

/* ------------------------------------------------------------------------- */
/* checksum.go:35-58                                                          */
uint32_t oracle_compute_checksum(const uint8_t* data, uint32_t len, uint32_t csum) {
  /* checksum.go:40-49: 2 bytes per iteration, uint32 wrap-around, odd tail <<8 */
  int64_t length = (int64_t)len - 1;
  for (int64_t i = 0; i < length; i += 2) {
    csum += (uint32_t)data[i] << 8;
    csum += (uint32_t)data[i + 1];
  }
  if (len % 2 == 1) csum += (uint32_t)data[length] << 8;
  return csum;
}

uint16_t oracle_fold_checksum(uint32_t csum) {
  /* checksum.go:53-58 */
  while (csum > 0xffff) csum = (csum >> 16) + (csum & 0xffff);
  return (uint16_t)~csum;
}

/* flows.go:60-70, :69-70 constants */
#define FNV_BASIS 14695981039346656037ull
#define FNV_PRIME 1099511628211ull
uint64_t oracle_fnv_hash(const uint8_t* s, uint32_t len) {
  uint64_t h = FNV_BASIS;
  for (uint32_t i = 0; i < len; i++) {
    h ^= (uint64_t)s[i];
    h *= FNV_PRIME;
  }
  return h;
}

/* flows.go:167-174 (Flow.FastHash), NewFlow :214-224 */
uint64_t oracle_flow_fast_hash(int64_t typ, const uint8_t* src, uint32_t slen, const uint8_t* dst,
                               uint32_t dlen) {
  uint64_t h = oracle_fnv_hash(src, slen) + oracle_fnv_hash(dst, dlen);
  h ^= (uint64_t)typ;
  h *= FNV_PRIME;
  return h;
}

/* ------------------------------------------------------------------------- */
/* configuration: container (parser.go:74-169) + registry tables              */

static void put_type(oracle_config* c, int lt, int kind) {
  if (lt >= 0 && lt < GPK_MAX_LAYER_TYPE) c->dispatch[lt] = (uint8_t)kind;
}

void oracle_config_put(oracle_config* c, int kind) {
  /* DecodingLayerMap.Put (parser.go:150-158): every type of CanDecode(). */
  switch (kind) {
    case GPK_DEC_ETHERNET: put_type(c, GPK_LT_ETHERNET, kind); break;   /* ethernet.go:107-109 */
    case GPK_DEC_DOT1Q: put_type(c, GPK_LT_DOT1Q, kind); break;         /* dot1q.go:44-46 */
    case GPK_DEC_IPV4: put_type(c, GPK_LT_IPV4, kind); break;           /* ip4.go:273-275 */
    case GPK_DEC_IPV6: put_type(c, GPK_LT_IPV6, kind); break;           /* ip6.go:281-283 */
    case GPK_DEC_IPV6_EXT:                                              /* ip6.go:454-456, layertypes.go:200-206 */
      put_type(c, GPK_LT_IPV6_HOPBYHOP, kind);
      put_type(c, GPK_LT_IPV6_ROUTING, kind);
      put_type(c, GPK_LT_IPV6_FRAGMENT, kind);
      put_type(c, GPK_LT_IPV6_DESTINATION, kind);
      break;
    case GPK_DEC_TCP: put_type(c, GPK_LT_TCP, kind); break;             /* tcp.go:587-589 */
    case GPK_DEC_UDP: put_type(c, GPK_LT_UDP, kind); break;             /* udp.go:107-109 */
    case GPK_DEC_PAYLOAD: put_type(c, GPK_LT_PAYLOAD, kind); break;     /* base.go:61 */
    case GPK_DEC_FRAGMENT: put_type(c, GPK_LT_FRAGMENT, kind); break;   /* base.go:118 */
    default: break;
  }
}

void oracle_config_init(oracle_config* c, int64_t first) {
  memset(c, 0, sizeof(*c));
  c->first = first;
  c->outputs = GPK_OUT_ALL;
  /* enums_generated.go:76-86 / :146-156: unregistered values -> LayerType 0 */
  for (int i = 0; i < GPK_N_ETHERTYPE_ROWS; i++)
    c->ethertype[GPK_ETHERTYPE_ROWS[i].value] = GPK_ETHERTYPE_ROWS[i].layer_type;
  for (int i = 0; i < GPK_N_IPPROTOCOL_ROWS; i++)
    c->ipprotocol[GPK_IPPROTOCOL_ROWS[i].value] = GPK_IPPROTOCOL_ROWS[i].layer_type;
  /* ports.go:54-93 / :121-172: switch, default Payload; override bitfield
   * (:55-57, :122-124) set by init() in modbus.go:169-171, enip.go:137-140 */
  for (int p = 0; p < 65536; p++) c->tcp_port[p] = c->udp_port[p] = GPK_LT_PAYLOAD;
  for (int i = 0; i < GPK_N_TCP_PORT_SWITCH; i++)
    c->tcp_port[GPK_TCP_PORT_SWITCH[i].port] = GPK_TCP_PORT_SWITCH[i].layer_type;
  for (int i = 0; i < GPK_N_UDP_PORT_SWITCH; i++)
    c->udp_port[GPK_UDP_PORT_SWITCH[i].port] = GPK_UDP_PORT_SWITCH[i].layer_type;
  for (int i = 0; i < GPK_N_TCP_PORT_OVERRIDE; i++)
    c->tcp_port[GPK_TCP_PORT_OVERRIDE[i].port] = GPK_TCP_PORT_OVERRIDE[i].layer_type;
  for (int i = 0; i < GPK_N_UDP_PORT_OVERRIDE; i++)
    c->udp_port[GPK_UDP_PORT_OVERRIDE[i].port] = GPK_UDP_PORT_OVERRIDE[i].layer_type;
}

uint64_t oracle_sizeof_config(void) { return sizeof(oracle_config); }

void oracle_config_set(oracle_config* c, int ignore_unsupported, int ignore_panic, uint32_t outputs) {
  c->ignore_unsupported = ignore_unsupported;
  c->ignore_panic = ignore_panic;
  c->outputs = outputs;
}

int32_t* oracle_config_table(oracle_config* c, int which) {
  switch (which) {
    case 0: return c->ethertype;
    case 1: return c->ipprotocol;
    case 2: return c->tcp_port;
    default: return c->udp_port;
  }
}

/* ------------------------------------------------------------------------- */
/* per-packet decode state                                                    */

typedef struct {
  const uint8_t* b;    /* packet bytes */
  uint32_t caplen;
  int truncated;       /* DecodingLayerParser.Truncated (parser.go:192-209) */
  uint32_t err, a0, a1;
  /* per decoder instance: last successful DecodeFromBytes input range */
  uint32_t start[GPK_NUM_DEC], end[GPK_NUM_DEC];
  int dirty[GPK_NUM_DEC];
  int64_t list[64];
  uint32_t nlist;      /* may exceed 64; only the first 64 are stored */
  int last_net;        /* GPK_DEC_IPV4 / GPK_DEC_IPV6 of the last network layer decoded */
  int transport;       /* GPK_DEC_TCP / GPK_DEC_UDP if decoded */
  uint32_t udp_hlen;   /* bytes of UDP Contents+Payload (udp.go:41-51) */
} pkt_state;

typedef struct {  /* the decoder's LayerPayload() and NextLayerType() */
  uint32_t off, len;
  int64_t next;
} layer_out;

static inline uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }
static inline uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

static int fail(pkt_state* s, uint32_t code, uint32_t a0, uint32_t a1) {
  s->err = code;
  s->a0 = a0;
  s->a1 = a1;
  return 1;
}

static int64_t eth_lt(const oracle_config* c, uint32_t et) { return c->ethertype[et & 0xffff]; }
static int64_t ipp_lt(const oracle_config* c, uint32_t p) { return c->ipprotocol[p & 0xff]; }

/* layers/ethernet.go:42-63, NextLayerType :111-113 */
static int dec_ethernet(const oracle_config* c, pkt_state* s, uint32_t off, uint32_t len, layer_out* o) {
  const uint8_t* d = s->b + off;
  if (len < 14) return fail(s, GPK_ERR_ETH_TOO_SMALL, 0, 0);
  uint32_t et = be16(d + 12);
  o->off = off + 14;
  o->len = len - 14;
  if (et < 0x0600) {
    uint32_t length = et;
    et = 0; /* EthernetTypeLLC */
    int64_t cmp = (int64_t)o->len - (int64_t)length;
    if (cmp < 0) s->truncated = 1;
    else if (cmp > 0) o->len = length;
  }
  o->next = eth_lt(c, et);
  return 0;
}

/* layers/dot1q.go:30-41, :49-51 */
static int dec_dot1q(const oracle_config* c, pkt_state* s, uint32_t off, uint32_t len, layer_out* o) {
  const uint8_t* d = s->b + off;
  if (len < 4) {
    s->truncated = 1;
    return fail(s, GPK_ERR_DOT1Q_SHORT, len, 0);
  }
  o->off = off + 4;
  o->len = len - 4;
  o->next = eth_lt(c, be16(d + 2));
  return 0;
}

/* layers/ip4.go:178-271, NextLayerType :277-282 */
static int dec_ipv4(const oracle_config* c, pkt_state* s, uint32_t off, uint32_t len, layer_out* o) {
  const uint8_t* d = s->b + off;
  if (len < 20) {
    s->truncated = 1;
    return fail(s, GPK_ERR_IP4_HDR_SHORT, len, 0);
  }
  uint16_t length = be16(d + 2);
  uint8_t ihl = d[0] & 0x0f;
  if (length == 0) length = (uint16_t)len; /* ip4.go:189-193 (TSO), wraps */
  if (length < 20) return fail(s, GPK_ERR_IP4_LEN_SMALL, length, 0);
  if (ihl < 5) return fail(s, GPK_ERR_IP4_IHL_SMALL, ihl, 0);
  if ((uint32_t)ihl * 4 > length) return fail(s, GPK_ERR_IP4_IHL_GT_LEN, ihl, length);
  int64_t cmp = (int64_t)len - (int64_t)length;
  if (cmp > 0) {
    len = length;
  } else if (cmp < 0) {
    s->truncated = 1;
    if ((uint32_t)ihl * 4 > len) return fail(s, GPK_ERR_IP4_HDR_MISSING, 0, 0);
  }
  /* options loop ip4.go:217-256 over data[20:IHL*4] */
  uint32_t p = 20, rem = (uint32_t)ihl * 4 - 20;
  while (rem > 0) {
    uint8_t t = d[p];
    if (t == 0) break; /* EOL: Padding = rest (ip4.go:228-233) */
    if (t == 1) {
      p += 1;
      rem -= 1;
      continue;
    }
    if (rem < 2) {
      s->truncated = 1;
      return fail(s, GPK_ERR_IP4_OPT_SHORT, rem, 0);
    }
    uint8_t ol = d[p + 1];
    if (rem < ol) {
      s->truncated = 1;
      return fail(s, GPK_ERR_IP4_OPT_EXCEEDS, t, ol);
    }
    if (ol <= 2) return fail(s, GPK_ERR_IP4_OPT_BADLEN, t, ol);
    p += ol;
    rem -= ol;
  }
  uint16_t ff = be16(d + 6);
  uint8_t flags = (uint8_t)(ff >> 13);
  uint16_t frag = ff & 0x1fff;
  o->off = off + (uint32_t)ihl * 4;
  o->len = len - (uint32_t)ihl * 4;
  if ((flags & 1) || frag != 0) o->next = GPK_LT_FRAGMENT;
  else o->next = ipp_lt(c, d[9]);
  return 0;
}

/* decodeIPv6ExtensionBase, layers/ip6.go:418-432 */
static int ext_base(pkt_state* s, uint32_t off, uint32_t len, uint32_t* nh, uint32_t* actual) {
  const uint8_t* d = s->b + off;
  if (len < 2) {
    s->truncated = 1;
    return fail(s, GPK_ERR_IP6_EXT_SHORT, len, 0);
  }
  *nh = d[0];
  *actual = (uint32_t)d[1] * 8 + 8;
  if (len < *actual) return fail(s, GPK_ERR_IP6_EXT_LEN, len, *actual);
  return 0;
}

/* layers/ip6.go:221-278; HopByHop :509-526; TLV :327-346; jumbo :54-76;
 * NextLayerType :286-291 */
static int dec_ipv6(const oracle_config* c, pkt_state* s, uint32_t off, uint32_t len, layer_out* o) {
  const uint8_t* d = s->b + off;
  if (len < 40) {
    s->truncated = 1;
    return fail(s, GPK_ERR_IP6_HDR_SHORT, len, 0);
  }
  uint16_t length = be16(d + 4);
  uint32_t nh = d[6];
  uint32_t poff = off + 40, plen = len - 40;
  int hbh = 0;
  uint32_t hbh_nh = 0;
  if (nh == 0) { /* IPProtocolIPv6HopByHop */
    uint32_t actual;
    if (ext_base(s, poff, plen, &hbh_nh, &actual)) return 1;
    const uint8_t* h = s->b + poff;
    int have_jumbo_tlv = 0;
    uint32_t jumbo_off = 0, jumbo_len = 0;
    for (uint32_t o2 = 2; o2 < actual;) { /* ip6.go:516-524 over data = ipv6.Payload */
      uint32_t r = plen - o2;
      if (r < 2) {
        s->truncated = 1;
        return fail(s, GPK_ERR_IP6_TLV_SHORT, 0, 0);
      }
      uint32_t al;
      uint8_t otype = 0;
      if (h[o2] == 0) {
        al = 1;
      } else {
        otype = h[o2];
        al = (uint32_t)h[o2 + 1] + 2;
        if (r < al) {
          s->truncated = 1;
          return fail(s, GPK_ERR_IP6_TLV_TOO_SMALL, 0, 0);
        }
        if (otype == 0xC2 && !have_jumbo_tlv) {
          have_jumbo_tlv = 1;
          jumbo_off = o2 + 2;
          jumbo_len = al - 2;
        }
      }
      o2 += al;
    }
    hbh = 1;
    int jumbo = 0;
    uint32_t pend = 0;
    if (have_jumbo_tlv) { /* ip6.go:63-75 */
      if (jumbo_len != 4) return fail(s, GPK_ERR_IP6_JUMBO_TLV_LEN, 0, 0);
      uint32_t l = be32(h + jumbo_off);
      if (l <= 65535) return fail(s, GPK_ERR_IP6_JUMBO_SMALL, 0, 0);
      jumbo = 1;
      pend = l;
    }
    if (jumbo && length == 0) { /* ip6.go:249-256: payload NOT advanced past HBH */
      if (pend > plen) {
        s->truncated = 1;
        pend = plen;
      }
      o->off = poff;
      o->len = pend;
      o->next = ipp_lt(c, hbh_nh);
      return 0;
    } else if (jumbo && length != 0) {
      return fail(s, GPK_ERR_IP6_JUMBO_AND_LEN, 0, 0);
    } else if (!jumbo && length == 0) {
      return fail(s, GPK_ERR_IP6_LEN0_NO_JUMBO, 0, 0);
    } else {
      poff += actual; /* ip6.go:262 */
      plen -= actual;
    }
  }
  if (length == 0) return fail(s, GPK_ERR_IP6_LEN0, nh, 0);
  uint32_t pend = length;
  if (pend > plen) {
    s->truncated = 1;
    pend = plen;
  }
  o->off = poff;
  o->len = pend;
  o->next = ipp_lt(c, hbh ? hbh_nh : nh);
  return 0;
}

/* IPv6ExtensionSkipper, layers/ip6.go:443-461 */
static int dec_ipv6_ext(const oracle_config* c, pkt_state* s, uint32_t off, uint32_t len, layer_out* o) {
  uint32_t nh, actual;
  if (ext_base(s, off, len, &nh, &actual)) return 1;
  o->off = off + actual;
  o->len = len - actual;
  o->next = ipp_lt(c, nh);
  return 0;
}

/* MPTCP option body, layers/tcp.go:347-533 with Go bounds checks:
 * data[i] needs i < len; data[lo:hi] needs hi <= cap then lo <= hi;
 * data[lo:] needs lo <= len. */
typedef struct {
  uint32_t len, cap;
} goslice;
#define IDX(i)                                                        \
  do {                                                                \
    if ((uint32_t)(i) >= sl.len) return fail(s, GPK_ERR_PANIC_INDEX, (i), sl.len); \
  } while (0)
#define SL(lo, hi)                                                                       \
  do {                                                                                   \
    if ((uint32_t)(hi) > sl.cap) return fail(s, GPK_ERR_PANIC_SLICE_ACAP, (hi), sl.cap);  \
    if ((uint32_t)(lo) > (uint32_t)(hi)) return fail(s, GPK_ERR_PANIC_SLICE_B, (lo), (hi)); \
  } while (0)

static int mptcp_option(pkt_state* s, const uint8_t* d, goslice sl, uint8_t* out_len) {
  IDX(1);
  uint8_t ol = d[1];
  *out_len = ol;
  if (ol <= 0) return fail(s, GPK_ERR_MPTCP_LEN, ol, 0);
  IDX(2);
  uint8_t sub = d[2] >> 4;
  switch (sub) {
    case 0: /* MP_CAPABLE tcp.go:355-381 */
      if (ol != 4 && ol != 12 && ol != 20 && ol != 22 && ol != 24)
        return fail(s, GPK_ERR_MP_CAPABLE_LEN, ol, 0);
      IDX(3);
      if (ol >= 12) SL(4, 12);
      if (ol >= 20) SL(12, 20);
      if (ol >= 22) SL(20, 22);
      if (ol == 24) SL(22, 24);
      break;
    case 1: /* MP_JOIN tcp.go:382-405 */
      if (ol != 12 && ol != 16 && ol != 24) return fail(s, GPK_ERR_MP_JOIN_LEN, ol, 0);
      if (ol == 12) {
        IDX(3);
        SL(4, 8);
        SL(8, 12);
      } else if (ol == 16) {
        IDX(3);
        SL(4, 12);
        SL(12, 16);
      } else {
        SL(4, 24);
      }
      break;
    case 2: { /* DSS tcp.go:406-442, optionMptcpDsslen :553-571 */
      IDX(3);
      uint8_t f = d[3];
      int m = (f & 0x08) != 0, M = (f & 0x04) != 0, a = (f & 0x02) != 0, A = (f & 0x01) != 0;
      uint8_t l0 = 4, l1;
      if (A) {
        l0 += 4;
        if (a) l0 += 4;
      }
      if (M) {
        l0 += 10;
        if (m) l0 += 4;
      }
      l1 = l0;
      if (M) l1 += 2;
      if (ol != l0 && ol != l1) return fail(s, GPK_ERR_DSS_LEN, ol, 0);
      uint8_t lo = 4;
      if (A) {
        if (a) {
          SL(lo, lo + 8);
          lo += 8;
        } else {
          SL(lo, lo + 4);
          lo += 4;
        }
      }
      if (M) {
        if (m) {
          SL(lo, lo + 8);
          lo += 8;
        } else {
          SL(lo, lo + 4);
          lo += 4;
        }
        SL(lo, lo + 4);
        lo += 4;
        SL(lo, lo + 2);
        lo += 2;
        if ((uint8_t)(ol - lo) == 2) SL(lo, lo + 2);
      }
      break;
    }
    case 3: { /* ADD_ADDR tcp.go:443-484, isValidOptionMptcpAddAddrlen :573-585 */
      uint8_t b2 = d[2];
      int ver1, e = 0;
      if ((b2 & 0x0f) > 1) ver1 = 0;
      else {
        ver1 = 1;
        e = (b2 & 1) != 0;
      }
      uint8_t chk = ol;
      if (ver1 && !e) chk = (uint8_t)(chk - 8);
      if (!(chk == 8 || chk == 10 || chk == 20 || chk == 22)) return fail(s, GPK_ERR_ADD_ADDR_LEN, ol, 0);
      uint8_t lenopt = ol;
      IDX(3);
      if (ver1 && !e) {
        uint8_t lo = (uint8_t)(ol - 8);
        if (lo > sl.len) return fail(s, GPK_ERR_PANIC_SLICE_B, lo, sl.len);
        lenopt = (uint8_t)(lenopt - 8);
      }
      switch (lenopt) {
        case 8: SL(4, 8); break;
        case 10: SL(4, 8); SL(8, 10); break;
        case 20: SL(4, 20); break;
        case 22: SL(4, 20); SL(20, 22); break;
        default: break;
      }
      break;
    }
    case 4: /* REMOVE_ADDR tcp.go:485-496 */
      if (ol < 4) return fail(s, GPK_ERR_REM_ADDR_LEN, ol, 0);
      for (uint8_t n = 0; n < (uint8_t)(ol - 3); n++) IDX(3 + n);
      break;
    case 5: /* MP_PRIO tcp.go:497-506 */
      if (ol != 3 && ol != 4) return fail(s, GPK_ERR_MP_PRIO_LEN, ol, 0);
      if (ol == 4) IDX(3);
      break;
    case 6: /* MP_FAIL tcp.go:507-513 */
      if (ol != 12) return fail(s, GPK_ERR_MP_FAIL_LEN, ol, 0);
      SL(4, 12);
      break;
    case 7: /* MP_FASTCLOSE tcp.go:515-521 */
      if (ol != 12) return fail(s, GPK_ERR_MP_FASTCLOSE_LEN, ol, 0);
      SL(4, 12);
      break;
    case 8: /* MP_TCPRST tcp.go:522-532 */
      if (ol != 4) return fail(s, GPK_ERR_MP_TCPRST_LEN, ol, 0);
      IDX(3);
      break;
    default: break;
  }
  return 0;
}

/* layers/tcp.go:291-551, NextLayerType :591-597 */
static int dec_tcp(const oracle_config* c, pkt_state* s, uint32_t off, uint32_t len, layer_out* o) {
  const uint8_t* d = s->b + off;
  if (len < 20) {
    s->truncated = 1;
    return fail(s, GPK_ERR_TCP_HDR_SHORT, len, 0);
  }
  uint16_t sport = be16(d), dport = be16(d + 2);
  uint8_t doff = d[12] >> 4;
  if (doff < 5) return fail(s, GPK_ERR_TCP_DOFF_SMALL, doff, 0);
  uint32_t ds = (uint32_t)doff * 4;
  if (ds > len) {
    s->truncated = 1;
    return fail(s, GPK_ERR_TCP_DOFF_GT_LEN, 0, 0);
  }
  /* options loop tcp.go:335-549 over data = data[20:dataStart] */
  uint32_t p = off + 20;
  goslice sl = {ds - 20, s->caplen - (off + 20)};
  while (sl.len > 0) {
    const uint8_t* od = s->b + p;
    uint8_t t = od[0];
    uint8_t ol;
    if (t == 0) break; /* EndList: Padding = data[1:] */
    if (t == 1) {
      ol = 1;
    } else if (t == 30) {
      if (mptcp_option(s, od, sl, &ol)) return 1;
    } else {
      if (sl.len < 2) {
        s->truncated = 1;
        return fail(s, GPK_ERR_TCP_OPT_SHORT, sl.len, 0);
      }
      ol = od[1];
      if (ol < 2) return fail(s, GPK_ERR_TCP_OPT_LEN_SMALL, ol, 0);
      if ((uint32_t)ol > sl.len) {
        s->truncated = 1;
        return fail(s, GPK_ERR_TCP_OPT_EXCEEDS, ol, sl.len);
      }
    }
    /* data = data[opt.OptionLength:] (tcp.go:548) */
    if ((uint32_t)ol > sl.len) return fail(s, GPK_ERR_PANIC_SLICE_B, ol, sl.len);
    p += ol;
    sl.len -= ol;
    sl.cap -= ol;
  }
  o->off = off + ds;
  o->len = len - ds;
  int64_t lt = c->tcp_port[dport];
  if (lt == GPK_LT_PAYLOAD) lt = c->tcp_port[sport];
  o->next = lt;
  return 0;
}

/* layers/udp.go:30-56, NextLayerType :114-119 */
static int dec_udp(const oracle_config* c, pkt_state* s, uint32_t off, uint32_t len, layer_out* o) {
  const uint8_t* d = s->b + off;
  if (len < 8) {
    s->truncated = 1;
    return fail(s, GPK_ERR_UDP_HDR_SHORT, len, 0);
  }
  uint16_t sport = be16(d), dport = be16(d + 2), length = be16(d + 4);
  if (length >= 8) {
    uint32_t hlen = length;
    if (hlen > len) {
      s->truncated = 1;
      hlen = len;
    }
    o->off = off + 8;
    o->len = hlen - 8;
    s->udp_hlen = hlen;
  } else if (length == 0) {
    o->off = off + 8;
    o->len = len - 8;
    s->udp_hlen = len;
  } else {
    return fail(s, GPK_ERR_UDP_TOO_SMALL, length, 0);
  }
  int64_t lt = c->udp_port[dport];
  if (lt != GPK_LT_PAYLOAD) o->next = lt;
  else o->next = c->udp_port[sport];
  return 0;
}

/* gopacket.Payload / gopacket.Fragment: base.go:61-70, :115-124 */
static int dec_terminal(pkt_state* s, uint32_t off, uint32_t len, layer_out* o) {
  (void)s;
  o->off = off + len;
  o->len = 0; /* LayerPayload() == nil */
  o->next = GPK_LT_ZERO;
  return 0;
}

static int decode_one(const oracle_config* c, int kind, pkt_state* s, uint32_t off, uint32_t len,
                      layer_out* o) {
  switch (kind) {
    case GPK_DEC_ETHERNET: return dec_ethernet(c, s, off, len, o);
    case GPK_DEC_DOT1Q: return dec_dot1q(c, s, off, len, o);
    case GPK_DEC_IPV4: return dec_ipv4(c, s, off, len, o);
    case GPK_DEC_IPV6: return dec_ipv6(c, s, off, len, o);
    case GPK_DEC_IPV6_EXT: return dec_ipv6_ext(c, s, off, len, o);
    case GPK_DEC_TCP: return dec_tcp(c, s, off, len, o);
    case GPK_DEC_UDP: return dec_udp(c, s, off, len, o);
    default: return dec_terminal(s, off, len, o);
  }
}

static int kind_for(const oracle_config* c, int64_t typ) {
  /* DecodingLayerContainer.Decoder (parser.go:161-164) */
  if (typ < 0 || typ >= GPK_MAX_LAYER_TYPE) return GPK_DEC_NONE;
  return c->dispatch[typ];
}

/* DecodeLayers (parser.go:303-317) running LayersDecoder (layers_decoder.go:60-79).
 * Returns 1 if the first layer has no decoder (decoded left untouched, :12-16). */
static int run_parser(const oracle_config* c, pkt_state* s) {
  memset(s->start, 0xff, sizeof(s->start));
  memset(s->end, 0xff, sizeof(s->end));
  int kind = kind_for(c, c->first);
  if (kind == GPK_DEC_NONE) {
    if (!c->ignore_unsupported) fail(s, GPK_ERR_UNSUPPORTED, (uint32_t)c->first, 0);
    return 1;
  }
  int64_t typ = c->first;
  uint32_t off = 0, len = s->caplen;
  for (;;) {
    layer_out o;
    if (decode_one(c, kind, s, off, len, &o)) {
      s->dirty[kind] = 1;
      return 0; /* (LayerTypeZero, err) */
    }
    if (s->nlist < 64) s->list[s->nlist] = typ;
    s->nlist++;
    s->start[kind] = off;
    s->end[kind] = off + len;
    if (kind == GPK_DEC_IPV4 || kind == GPK_DEC_IPV6) s->last_net = kind;
    if (kind == GPK_DEC_TCP || kind == GPK_DEC_UDP) s->transport = kind;
    typ = o.next;
    off = o.off;
    len = o.len;
    if (len == 0) return 0; /* success */
    kind = kind_for(c, typ);
    if (kind == GPK_DEC_NONE) {
      if (typ != GPK_LT_ZERO && !c->ignore_unsupported)
        fail(s, GPK_ERR_UNSUPPORTED, (uint32_t)typ, 0);
      return 0;
    }
  }
}

static unsigned code_of(int64_t typ) {
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

static int clean(const pkt_state* s, int kind) { return s->start[kind] != 0xffffffffu && !s->dirty[kind]; }

/* tcpip.go:26-35 (IPv4) and :37-48 (IPv6) */
static uint32_t pseudo_sum(const pkt_state* s) {
  uint32_t csum = 0;
  const uint8_t* d = s->b + s->start[s->last_net];
  if (s->last_net == GPK_DEC_IPV4) {
    const uint8_t *src = d + 12, *dst = d + 16;
    csum += ((uint32_t)src[0] + src[2]) << 8;
    csum += (uint32_t)src[1] + src[3];
    csum += ((uint32_t)dst[0] + dst[2]) << 8;
    csum += (uint32_t)dst[1] + dst[3];
  } else {
    const uint8_t *src = d + 8, *dst = d + 24;
    for (int i = 0; i < 16; i += 2) {
      csum += (uint32_t)src[i] << 8;
      csum += src[i + 1];
      csum += (uint32_t)dst[i] << 8;
      csum += dst[i + 1];
    }
  }
  return csum;
}

static void decode_packet(const oracle_config* c, const uint8_t* pkt, uint32_t caplen, gpk_record* rec,
                          uint32_t* err_args, uint64_t* fl_link, uint64_t* fl_net, uint64_t* fl_tr,
                          gpk_layout* lay, uint16_t* actual) {
  pkt_state s;
  memset(&s, 0, sizeof(s));
  s.b = pkt;
  s.caplen = caplen;
  run_parser(c, &s);

  uint64_t layers = 0;
  for (uint32_t i = 0; i < s.nlist && i < GPK_MAX_INLINE_LAYERS; i++)
    layers |= (uint64_t)code_of(s.list[i]) << (4 * i);
  uint32_t st = s.err & GPK_ST_ERR_MASK;
  if (s.truncated) st |= GPK_ST_TRUNCATED;
  uint32_t nl = s.nlist > GPK_ST_NLAYERS_MASK ? GPK_ST_NLAYERS_MASK : s.nlist;
  st |= nl << GPK_ST_NLAYERS_SHIFT;
  uint16_t ip4c = 0, l4c = 0;

  /* IPv4.VerifyChecksum ip4.go:323-332 on the IPv4 struct (last writer) */
  if ((c->outputs & GPK_OUT_IP4_CSUM) && clean(&s, GPK_DEC_IPV4)) {
    const uint8_t* d = pkt + s.start[GPK_DEC_IPV4];
    uint32_t ihl = d[0] & 0x0f;
    uint16_t existing = be16(d + 10);
    uint32_t v = oracle_compute_checksum(d, ihl * 4, 0);
    ip4c = oracle_fold_checksum(v - (uint32_t)existing);
    if (actual) actual[0] = existing; /* IPv4.Checksum, ChecksumVerificationResult.Actual */
    st |= GPK_ST_IP4_CSUM;
    if (ip4c == existing) st |= GPK_ST_IP4_VALID;
  }
  /* TCP.VerifyChecksum tcp.go:626-640 / UDP.VerifyChecksum udp.go:144-158 with
   * SetNetworkLayerForChecksum(last network layer) (tcpip.go:75-85) */
  if ((c->outputs & GPK_OUT_L4_CSUM) && s.transport && clean(&s, s.transport) && s.last_net &&
      clean(&s, s.last_net)) {
    const uint8_t* d = pkt + s.start[s.transport];
    uint32_t blen = s.transport == GPK_DEC_TCP ? s.end[GPK_DEC_TCP] - s.start[GPK_DEC_TCP] : s.udp_hlen;
    uint16_t existing = be16(d + (s.transport == GPK_DEC_TCP ? 16 : 6));
    uint32_t proto = s.transport == GPK_DEC_TCP ? 6 : 17;
    uint32_t csum = pseudo_sum(&s); /* tcpip.go:54-69 */
    csum += proto;
    csum += blen & 0xffff;
    csum += blen >> 16;
    csum = oracle_compute_checksum(d, blen, csum);
    l4c = oracle_fold_checksum(csum - (uint32_t)existing);
    if (actual) actual[1] = existing; /* TCP/UDP.Checksum */
    st |= GPK_ST_L4_CSUM;
    if (s.transport == GPK_DEC_UDP) {
      st |= GPK_ST_L4_UDP;
      if (existing == 0 || l4c == existing) st |= GPK_ST_L4_VALID;
    } else if (l4c == existing) {
      st |= GPK_ST_L4_VALID;
    }
  }
  if (c->outputs & GPK_OUT_FLOWS) {
    uint64_t lf = 0, nf = 0, tf = 0;
    if (clean(&s, GPK_DEC_ETHERNET)) { /* ethernet.go:38-40, EndpointMAC = 3 */
      const uint8_t* d = pkt + s.start[GPK_DEC_ETHERNET];
      lf = oracle_flow_fast_hash(3, d + 6, 6, d, 6);
      st |= GPK_ST_LINK_FLOW;
    }
    if (s.last_net && clean(&s, s.last_net)) {
      const uint8_t* d = pkt + s.start[s.last_net];
      if (s.last_net == GPK_DEC_IPV4) nf = oracle_flow_fast_hash(1, d + 12, 4, d + 16, 4); /* ip4.go:63 */
      else {
        nf = oracle_flow_fast_hash(2, d + 8, 16, d + 24, 16); /* ip6.go:49 */
        st |= GPK_ST_NET_IPV6;
      }
      st |= GPK_ST_NET_FLOW;
    }
    if (s.transport && clean(&s, s.transport)) { /* tcp.go:614, udp.go:132 */
      const uint8_t* d = pkt + s.start[s.transport];
      tf = oracle_flow_fast_hash(s.transport == GPK_DEC_TCP ? 4 : 5, d, 2, d + 2, 2);
      st |= GPK_ST_TRANSPORT_FLOW;
    }
    if (fl_link) {
      *fl_link = lf;
      *fl_net = nf;
      *fl_tr = tf;
    }
  }
  rec->layers = layers;
  rec->status = st;
  rec->ip4_csum = ip4c;
  rec->l4_csum = l4c;
  if (err_args && s.err) {
    err_args[0] = s.a0;
    err_args[1] = s.a1;
  }
  if (lay) {
    static const int slot_kind[8] = {GPK_DEC_ETHERNET, GPK_DEC_DOT1Q, GPK_DEC_IPV4, GPK_DEC_IPV6,
                                     GPK_DEC_IPV6_EXT, GPK_DEC_TCP, GPK_DEC_UDP, GPK_DEC_PAYLOAD};
    for (int k = 0; k < 8; k++) {
      int kind = slot_kind[k];
      if (k == 7 && !clean(&s, GPK_DEC_PAYLOAD)) kind = GPK_DEC_FRAGMENT;
      if (clean(&s, kind)) {
        lay->start[k] = s.start[kind];
        lay->end[k] = s.end[kind];
      } else {
        lay->start[k] = lay->end[k] = GPK_LAYOUT_ABSENT;
      }
    }
  }
}

/* ---- layer fields (gpk_extract_fields) ------------------------------------ */
/* Option starts of a header whose DecodeFromBytes succeeded, as its option
 * loop walks them (ip4.go:219-256 pullOutOptions; tcp.go:336-549 OPTIONS):
 * kind 0 ends the list, kind 1 is one byte, every other kind advances by its
 * length byte (which that decode checked against the remaining header).
 * Bit k of the 40-bit map (byte k/8, bit k%8) = an option at header byte 20+k. */
static void option_map(const uint8_t* hdr, uint32_t hlen, uint8_t map[5]) {
  memset(map, 0, 5);
  const uint32_t n = hlen > 20 ? hlen - 20 : 0;
  const uint8_t* data = hdr + 20;
  for (uint32_t k = 0; k < n;) {
    map[k / 8] |= (uint8_t)(1u << (k % 8));
    if (data[k] == 0) break;                        /* End of options: Padding follows */
    const uint32_t len = data[k] == 1 ? 1u : data[k + 1]; /* No-op / OptionLength */
    if (len == 0) break;                            /* (never on a successful decode) */
    k += len;
  }
}

/* The field assignments of each DecodeFromBytes, applied to the slice the
 * layout records for the decoder (the slice of its last successful call). */
static void fields_of(const uint8_t* pkt, const gpk_layout* lay, gpk_fields* f) {
  memset(f, 0, sizeof(*f));
  f->ip4_start = f->tcp_start = 0xFF;
  for (int k = 0; k < 8; k++)
    if (lay->start[k] != GPK_LAYOUT_ABSENT) f->present |= 1u << k;
  if (lay->start[GPK_DEC_ETHERNET - 1] != GPK_LAYOUT_ABSENT) { /* ethernet.go:46-55 */
    const uint8_t* d = pkt + lay->start[GPK_DEC_ETHERNET - 1];
    memcpy(f->eth_dst, d, 6);
    memcpy(f->eth_src, d + 6, 6);
    f->eth_type = be16(d + 12);
    f->eth_length = 0;
    if (f->eth_type < 0x0600) {
      f->eth_length = f->eth_type;
      f->eth_type = 0; /* EthernetTypeLLC, enums.go:36 */
    }
  }
  if (lay->start[GPK_DEC_DOT1Q - 1] != GPK_LAYOUT_ABSENT) { /* dot1q.go:33-37 */
    const uint8_t* d = pkt + lay->start[GPK_DEC_DOT1Q - 1];
    const uint16_t priority = (d[0] & 0xE0) >> 5, de = (d[0] & 0x10) != 0, vid = be16(d) & 0x0FFF;
    f->d1q_tci = (uint16_t)(priority << 13 | de << 12 | vid);
    f->d1q_type = be16(d + 2);
  }
  if (lay->start[GPK_DEC_IPV4 - 1] != GPK_LAYOUT_ABSENT) { /* ip4.go:183-193, 257-267 */
    const uint32_t s = lay->start[GPK_DEC_IPV4 - 1];
    const uint8_t* d = pkt + s;
    f->ip4_length = be16(d + 2);
    f->ip4_ihl = d[0] & 0x0F;
    if (f->ip4_length == 0) f->ip4_length = (uint16_t)(lay->end[GPK_DEC_IPV4 - 1] - s); /* TSO: uint16(len(data)) */
    const uint16_t flagsfrags = be16(d + 6);
    f->ip4_version = d[0] >> 4;
    f->ip4_tos = d[1];
    f->ip4_id = be16(d + 4);
    f->ip4_flags_frag = (uint16_t)((flagsfrags >> 13) << 13 | (flagsfrags & 0x1FFF));
    f->ip4_ttl = d[8];
    f->ip4_protocol = d[9];
    f->ip4_checksum = be16(d + 10);
    memcpy(f->ip4_src, d + 12, 4);
    memcpy(f->ip4_dst, d + 16, 4);
    f->ip4_start = (uint8_t)(s < 0xFF ? s : 0xFF);
    option_map(d, (uint32_t)f->ip4_ihl * 4, f->ip4_opt_map);
  }
  if (lay->start[GPK_DEC_IPV6 - 1] != GPK_LAYOUT_ABSENT) { /* ip6.go:225-234 */
    const uint8_t* d = pkt + lay->start[GPK_DEC_IPV6 - 1];
    f->ip6_version = d[0] >> 4;
    f->ip6_traffic_class = (uint8_t)((be16(d) >> 4) & 0x00FF);
    f->ip6_flow_label = be32(d) & 0x000FFFFF;
    f->ip6_length = be16(d + 4);
    f->ip6_next_header = d[6];
    f->ip6_hop_limit = d[7];
    memcpy(f->ip6_src, d + 8, 16);
    memcpy(f->ip6_dst, d + 24, 16);
    /* ip6.go:244-246: NextHeader 0 is decoded inline as IPv6HopByHop from
     * data[40:]; its options (ip6.go:509-526 loop, TLVs :327-346), for
     * HeaderLength <= 2 (the map's 24 bits hold every start) */
    if (f->ip6_next_header == 0 && d[41] <= 2) {
      const uint32_t actual = (uint32_t)d[41] * 8 + 8;
      uint32_t map = 0;
      for (uint32_t off = 2; off < actual;) {
        map |= 1u << (off - 2);
        off += d[40 + off] == 0 ? 1u : (uint32_t)d[41 + off] + 2u; /* Pad1 | OptionLength + 2 */
      }
      f->hbh_opt_map[0] = (uint8_t)map;
      f->hbh_opt_map[1] = (uint8_t)(map >> 8);
      f->hbh_opt_map[2] = (uint8_t)(map >> 16);
    }
  }
  if (lay->start[GPK_DEC_TCP - 1] != GPK_LAYOUT_ABSENT) { /* tcp.go:296-313 */
    const uint8_t* d = pkt + lay->start[GPK_DEC_TCP - 1];
    f->tcp_src_port = be16(d);
    f->tcp_dst_port = be16(d + 2);
    f->tcp_seq = be32(d + 4);
    f->tcp_ack = be32(d + 8);
    f->tcp_data_offset = d[12] >> 4;
    f->tcp_flags = (uint16_t)((d[13] & 0x01 ? 1 : 0) | (d[13] & 0x02 ? 2 : 0) | (d[13] & 0x04 ? 4 : 0) |
                              (d[13] & 0x08 ? 8 : 0) | (d[13] & 0x10 ? 16 : 0) | (d[13] & 0x20 ? 32 : 0) |
                              (d[13] & 0x40 ? 64 : 0) | (d[13] & 0x80 ? 128 : 0) | (d[12] & 0x01 ? 256 : 0));
    f->tcp_window = be16(d + 14);
    f->tcp_checksum = be16(d + 16);
    f->tcp_urgent = be16(d + 18);
    const uint32_t s = lay->start[GPK_DEC_TCP - 1];
    f->tcp_start = (uint8_t)(s < 0xFF ? s : 0xFF);
    option_map(d, (uint32_t)f->tcp_data_offset * 4, f->tcp_opt_map);
  }
  if (lay->start[GPK_DEC_UDP - 1] != GPK_LAYOUT_ABSENT) { /* udp.go:34-41 */
    const uint8_t* d = pkt + lay->start[GPK_DEC_UDP - 1];
    f->udp_src_port = be16(d);
    f->udp_dst_port = be16(d + 2);
    f->udp_length = be16(d + 4);
    f->udp_checksum = be16(d + 6);
  }
}

void oracle_extract_fields(const uint8_t* data, const uint64_t* offsets, const gpk_layout* layouts, uint64_t n,
                           gpk_fields* out) {
  for (uint64_t i = 0; i < n; i++) fields_of(data + offsets[i], &layouts[i], &out[i]);
}

typedef struct {
  const oracle_config* c;
  const uint8_t* data;
  const uint64_t* offsets;
  const uint32_t* caplens;
  uint64_t n, lo, hi;
  gpk_record* records;
  uint32_t* err_args;
  uint64_t* flows;
  gpk_layout* layouts;
  gpk_record8* narrow; /* non-NULL: the narrow form (records then holds the side array) */
} work_t;

/* gpk_record8 of a decoded packet (include/gpk.h): the full record goes to the
 * side array only where Correct differs from the header's Checksum field
 * (Actual; checksum.go:9-21, udp.go:144-158) or the list has more than 8
 * entries. */
static void narrow_record(const gpk_record* r, const uint16_t actual[2], gpk_record8* r8, gpk_record* wide) {
  const uint32_t st = r->status, nl = (st >> GPK_ST_NLAYERS_SHIFT) & GPK_ST_NLAYERS_MASK;
  const int widen = nl > 8 || ((st & GPK_ST_IP4_CSUM) && r->ip4_csum != actual[0]) ||
                    ((st & GPK_ST_L4_CSUM) && r->l4_csum != actual[1]);
  r8->layers = (uint32_t)r->layers;
  r8->status = (st & ~(GPK_ST_NLAYERS_MASK << GPK_ST_NLAYERS_SHIFT)) |
               ((nl > 8 ? GPK_ST8_NLAYERS_MASK : nl) << GPK_ST_NLAYERS_SHIFT) | (widen ? GPK_ST8_WIDE : 0u);
  if (widen) *wide = *r;
}

static void* worker(void* arg) {
  work_t* w = (work_t*)arg;
  for (uint64_t i = w->lo; i < w->hi; i++) {
    uint64_t* fl = w->flows;
    gpk_record rec;
    uint16_t actual[2] = {0, 0};
    decode_packet(w->c, w->data + w->offsets[i], w->caplens[i], w->narrow ? &rec : &w->records[i],
                  w->err_args ? w->err_args + 2 * i : NULL, fl ? fl + i : NULL, fl ? fl + w->n + i : NULL,
                  fl ? fl + 2 * w->n + i : NULL, w->layouts ? w->layouts + i : NULL, actual);
    if (w->narrow) narrow_record(&rec, actual, &w->narrow[i], &w->records[i]);
  }
  return NULL;
}

void oracle_decode_batch(const oracle_config* c, const uint8_t* data, const uint64_t* offsets,
                         const uint32_t* caplens, uint64_t n, gpk_record* records, uint32_t* err_args,
                         uint64_t* flows, gpk_layout* layouts, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  work_t w[256];
  pthread_t th[256];
  for (int t = 0; t < nthreads; t++) {
    w[t] = (work_t){c, data, offsets, caplens, n, n * t / nthreads, n * (t + 1) / nthreads,
                    records, err_args, flows, layouts, NULL};
  }
  if (nthreads == 1) {
    worker(&w[0]);
    return;
  }
  for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, worker, &w[t]);
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

/* The same decode in the narrow form of gpk_decode_batch_narrow: records8[n],
 * and wide[i] written only for the packets whose record8 has GPK_ST8_WIDE. */
void oracle_decode_batch_narrow(const oracle_config* c, const uint8_t* data, const uint64_t* offsets,
                                const uint32_t* caplens, uint64_t n, gpk_record8* records8, gpk_record* wide,
                                uint32_t* err_args, uint64_t* flows, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  work_t w[256];
  pthread_t th[256];
  for (int t = 0; t < nthreads; t++) {
    w[t] = (work_t){c, data, offsets, caplens, n, n * t / nthreads, n * (t + 1) / nthreads,
                    wide, err_args, flows, NULL, records8};
  }
  if (nthreads == 1) {
    worker(&w[0]);
    return;
  }
  for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, worker, &w[t]);
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

uint32_t oracle_decoded_list(const oracle_config* c, const uint8_t* pkt, uint32_t caplen, int64_t* out,
                             uint32_t cap) {
  /* Full list, without the 64-entry bound of pkt_state: re-run the chain. */
  pkt_state s;
  memset(&s, 0, sizeof(s));
  s.b = pkt;
  s.caplen = caplen;
  memset(s.start, 0xff, sizeof(s.start));
  int kind = kind_for(c, c->first);
  if (kind == GPK_DEC_NONE) return 0;
  int64_t typ = c->first;
  uint32_t off = 0, len = caplen, n = 0;
  for (;;) {
    layer_out o;
    if (decode_one(c, kind, &s, off, len, &o)) return n;
    if (n < cap) out[n] = typ;
    n++;
    typ = o.next;
    off = o.off;
    len = o.len;
    if (len == 0) return n;
    kind = kind_for(c, typ);
    if (kind == GPK_DEC_NONE) return n;
  }
}

/* ------------------------------------------------------------------------- */
/* error text                                                                 */

static const char* lt_name(int64_t lt, char* tmp) {
  for (int i = 0; i < GPK_N_LAYER_TYPE_NAMES; i++)
    if (GPK_LAYER_TYPE_NAMES[i].id == lt) return GPK_LAYER_TYPE_NAMES[i].name;
  sprintf(tmp, "%lld", (long long)lt); /* layertype.go:107-109 strconv.Itoa */
  return tmp;
}

static const char* ipproto_name(uint32_t p) {
  /* IPProtocol.String(), enums_generated.go:131-140 */
  for (int i = 0; i < GPK_N_IPPROTOCOL_ROWS; i++)
    if ((uint32_t)GPK_IPPROTOCOL_ROWS[i].value == p) return GPK_IPPROTOCOL_ROWS[i].name;
  return "UnknownIPProtocol";
}

int oracle_error_string(const oracle_config* c, unsigned code, uint32_t a0, uint32_t a1, char* buf,
                        int cap) {
  (void)c;
  char tmp[32];
  switch (code) {
    case GPK_ERR_NONE: return snprintf(buf, cap, "%s", "");
    case GPK_ERR_UNSUPPORTED: return snprintf(buf, cap, "No decoder for layer type %s", lt_name((int32_t)a0, tmp));
    case GPK_ERR_PANIC_INDEX: return snprintf(buf, cap, "panic: runtime error: index out of range [%u] with length %u", a0, a1);
    case GPK_ERR_PANIC_SLICE_ACAP: return snprintf(buf, cap, "panic: runtime error: slice bounds out of range [:%u] with capacity %u", a0, a1);
    case GPK_ERR_PANIC_SLICE_B: return snprintf(buf, cap, "panic: runtime error: slice bounds out of range [%u:%u]", a0, a1);
    case GPK_ERR_ETH_TOO_SMALL: return snprintf(buf, cap, "Ethernet packet too small");
    case GPK_ERR_DOT1Q_SHORT: return snprintf(buf, cap, "802.1Q tag length %u too short", a0);
    case GPK_ERR_IP4_HDR_SHORT: return snprintf(buf, cap, "Invalid ip4 header. Length %u less than 20", a0);
    case GPK_ERR_IP4_LEN_SMALL: return snprintf(buf, cap, "Invalid (too small) IP length (%u < 20)", a0);
    case GPK_ERR_IP4_IHL_SMALL: return snprintf(buf, cap, "Invalid (too small) IP header length (%u < 5)", a0);
    case GPK_ERR_IP4_IHL_GT_LEN: return snprintf(buf, cap, "Invalid IP header length > IP length (%u > %u)", a0, a1);
    case GPK_ERR_IP4_HDR_MISSING: return snprintf(buf, cap, "Not all IP header bytes available");
    case GPK_ERR_IP4_OPT_SHORT: return snprintf(buf, cap, "Invalid ip4 option length. Length %u less than 2", a0);
    case GPK_ERR_IP4_OPT_EXCEEDS: return snprintf(buf, cap, "IP option length exceeds remaining IP header size, option type %u length %u", a0, a1);
    case GPK_ERR_IP4_OPT_BADLEN: return snprintf(buf, cap, "Invalid IP option type %u length %u. Must be greater than 2", a0, a1);
    case GPK_ERR_IP6_HDR_SHORT: return snprintf(buf, cap, "Invalid ip6 header. Length %u less than 40", a0);
    case GPK_ERR_IP6_JUMBO_AND_LEN: return snprintf(buf, cap, "IPv6 has jumbo length and IPv6 length is not 0");
    case GPK_ERR_IP6_LEN0_NO_JUMBO: return snprintf(buf, cap, "IPv6 length 0, but HopByHop header does not have jumbogram option");
    case GPK_ERR_IP6_LEN0: return snprintf(buf, cap, "IPv6 length 0, but next header is %s, not HopByHop", ipproto_name(a0));
    case GPK_ERR_IP6_TLV_SHORT: return snprintf(buf, cap, "IPv6 header option too small");
    case GPK_ERR_IP6_TLV_TOO_SMALL: return snprintf(buf, cap, "IPv6 header TLV option too small");
    case GPK_ERR_IP6_EXT_SHORT: return snprintf(buf, cap, "Invalid ip6-extension header. Length %u less than 2", a0);
    case GPK_ERR_IP6_EXT_LEN: return snprintf(buf, cap, "Invalid ip6-extension header. Length %u less than specified length %u", a0, a1);
    case GPK_ERR_IP6_JUMBO_TLV_LEN: return snprintf(buf, cap, "Jumbo length TLV data must have length 4");
    case GPK_ERR_IP6_JUMBO_SMALL: return snprintf(buf, cap, "Jumbo length cannot be less than 65536");
    case GPK_ERR_TCP_HDR_SHORT: return snprintf(buf, cap, "Invalid TCP header. Length %u less than 20", a0);
    case GPK_ERR_TCP_DOFF_SMALL: return snprintf(buf, cap, "Invalid TCP data offset %u < 5", a0);
    case GPK_ERR_TCP_DOFF_GT_LEN: return snprintf(buf, cap, "TCP data offset greater than packet length");
    case GPK_ERR_MPTCP_LEN: return snprintf(buf, cap, "MPTCP bad option length %u", a0);
    case GPK_ERR_MP_CAPABLE_LEN: return snprintf(buf, cap, "MP_CAPABLE bad option length %u", a0);
    case GPK_ERR_MP_JOIN_LEN: return snprintf(buf, cap, "MP_JOIN bad option length %u", a0);
    case GPK_ERR_DSS_LEN: return snprintf(buf, cap, "DSS bad option length %u", a0);
    case GPK_ERR_ADD_ADDR_LEN: return snprintf(buf, cap, "ADD_ADDR bad option length %u", a0);
    case GPK_ERR_REM_ADDR_LEN: return snprintf(buf, cap, "Rem_ADDR bad option length %u", a0);
    case GPK_ERR_MP_PRIO_LEN: return snprintf(buf, cap, "MP_PRIO bad option length %u", a0);
    case GPK_ERR_MP_FAIL_LEN: return snprintf(buf, cap, "MP_FAIL bad option length %u", a0);
    case GPK_ERR_MP_FASTCLOSE_LEN: return snprintf(buf, cap, "MP_FASTCLOSE bad option length %u", a0);
    case GPK_ERR_MP_TCPRST_LEN: return snprintf(buf, cap, "MP_TCPRST bad option length %u", a0);
    case GPK_ERR_TCP_OPT_SHORT: return snprintf(buf, cap, "Invalid TCP option length. Length %u less than 2", a0);
    case GPK_ERR_TCP_OPT_LEN_SMALL: return snprintf(buf, cap, "Invalid TCP option length %u < 2", a0);
    case GPK_ERR_TCP_OPT_EXCEEDS: return snprintf(buf, cap, "Invalid TCP option length %u exceeds remaining %u bytes", a0, a1);
    case GPK_ERR_UDP_HDR_SHORT: return snprintf(buf, cap, "Invalid UDP header. Length %u less than 8", a0);
    case GPK_ERR_UDP_TOO_SMALL: return snprintf(buf, cap, "UDP packet too small: %u bytes", a0);
    default: return snprintf(buf, cap, "unknown error code %u", code);
  }
}

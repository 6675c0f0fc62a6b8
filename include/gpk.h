/*
 * gpk.h — C ABI of the MI355X packet decode / checksum / flow-hash engine.
 *
 * This is the drop-in boundary for gopacket's DecodingLayerParser fast path.
 * A Go program binds it through cgo (stub in INTEGRATION.md); the Python and
 * C++ host mirrors in this repo bind it through ctypes / direct linking.
 * Plain C types only: pointers, sizes, fixed-width integers. No torch, no HIP
 * types leak through (streams are passed as void*).
 *
 * What each entry point replaces in the reference (gopacket, /root/reference):
 *   gpk_parser_create / gpk_parser_set_*   NewDecodingLayerParser(first, decoders...)
 *                                          parser.go:222-233, AddDecodingLayer :200,
 *                                          SetDecodingLayerContainer :238-241,
 *                                          DecodingLayerParserOptions :337-351
 *   gpk_parser_set_ethertype / _ipprotocol EthernetType/IPProtocol metadata tables
 *                                          layers/enums.go:294-353, enums_generated.go:76-156
 *   gpk_parser_set_tcp_port / _udp_port    RegisterTCPPortLayerType / RegisterUDPPortLayerType
 *                                          layers/ports.go:99-104,178-183 (defaults: the port
 *                                          switches :54-93,:121-172 + init overrides)
 *   gpk_ctx_create / gpk_ctx_destroy       one GPU (there is no reference counterpart: a
 *                                          DecodingLayerParser is per goroutine, doc.go:211-228)
 *   gpk_decode_batch                       DecodingLayerParser.DecodeLayers (parser.go:303-317)
 *                                          applied to every packet of a batch, plus, per packet,
 *                                          IPv4.VerifyChecksum (layers/ip4.go:323-332),
 *                                          TCP/UDP.VerifyChecksum (layers/tcp.go:626-640,
 *                                          layers/udp.go:144-158, layers/tcpip.go:54-69) and
 *                                          Flow.FastHash of LinkFlow/NetworkFlow/TransportFlow
 *                                          (flows.go:167-174, layers/ethernet.go:38,
 *                                          layers/ip4.go:63, layers/ip6.go:49, layers/tcp.go:614,
 *                                          layers/udp.go:132)
 *   gpk_decode_batch_host                  the same, starting and ending in host memory
 *                                          (pcap/afpacket sources hand over host buffers)
 *   gpk_decode_batch_narrow                gpk_decode_batch with an 8-byte record per packet (the
 *                                          full one only where it does not fit, gpk_record8)
 *   gpk_decode_batch_fields                gpk_decode_batch plus gpk_extract_fields in one launch
 *   gpk_extract_fields                     the scalar fields the six decoders' DecodeFromBytes set
 *                                          on their structs (layers/ethernet.go:42-55,
 *                                          dot1q.go:28-41, ip4.go:178-271, ip6.go:221-278,
 *                                          tcp.go:292-313, udp.go:30-43), from the layouts of a
 *                                          decode: the fields a consumer reads after DecodeLayers
 *   gpk_stop                               a break out of the ReadPacketData loop (ngread.go:629-632,
 *                                          afpacket.go:335-367) for the calls that push results
 *                                          through callbacks (gpk_replay_file, gpk_tpacket_pump)
 *   gpk_format_error                       the error values DecodeLayers returns
 *                                          (UnsupportedLayerType parser.go:321-327, panicToError
 *                                          :329-333, and every fmt.Errorf/errors.New site of
 *                                          layers/{ethernet,dot1q,ip4,ip6,tcp,udp}.go)
 *
 * Every function returns 0 on success or a negative GPK_E* status. No C++
 * exception crosses this boundary.
 */
#ifndef GPK_H
#define GPK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: gpk_fields bytes 1-3 carry the HopByHop option map (present is a u8);
 *    gpk_replay_stats gained alloc_wait_s; gpk_replay_opts and gpk_tp_pump_opts
 *    gained trailing fields and packets callbacks. A caller compiled against another
 *    version must not call in: check gpk_abi_version() == GPK_ABI_VERSION. */
#define GPK_ABI_VERSION 2

/* ---- status codes -------------------------------------------------------- */
#define GPK_OK 0
#define GPK_EINVAL (-1)     /* bad argument / batch description */
#define GPK_ENOMEM (-2)     /* device or host allocation failed */
#define GPK_EHIP (-3)       /* HIP runtime error (see gpk_last_hip_error) */
#define GPK_ENODEV (-4)     /* no gfx950 device / device ordinal out of range */
#define GPK_EUNSUPP (-5)    /* configuration the device path does not implement */
#define GPK_STOPPED 1       /* not an error: a replay or ring pump ended early at gpk_stop */

/* ---- LayerType ids (gopacket decode.go:106-117, layers/layertypes.go) ---- */
#define GPK_LT_ZERO 0
#define GPK_LT_PAYLOAD 2
#define GPK_LT_FRAGMENT 3
#define GPK_LT_DOT1Q 15
#define GPK_LT_ETHERNET 17
#define GPK_LT_IPV4 20
#define GPK_LT_IPV6 21
#define GPK_LT_TCP 44
#define GPK_LT_UDP 45
#define GPK_LT_IPV6_HOPBYHOP 46
#define GPK_LT_IPV6_ROUTING 47
#define GPK_LT_IPV6_FRAGMENT 48
#define GPK_LT_IPV6_DESTINATION 49
#define GPK_MAX_LAYER_TYPE 2000 /* layertype.go:41 maxLayerType */

/* ---- DecodingLayer implementations the device runs ----------------------- *
 * Each registers the LayerTypes of its CanDecode() class.                    */
#define GPK_DEC_NONE 0
#define GPK_DEC_ETHERNET 1      /* layers.Ethernet          {17}            */
#define GPK_DEC_DOT1Q 2         /* layers.Dot1Q             {15}            */
#define GPK_DEC_IPV4 3          /* layers.IPv4              {20}            */
#define GPK_DEC_IPV6 4          /* layers.IPv6              {21}            */
#define GPK_DEC_IPV6_EXT 5      /* layers.IPv6ExtensionSkipper {46,47,48,49} (ip6.go:437-461) */
#define GPK_DEC_TCP 6           /* layers.TCP               {44}            */
#define GPK_DEC_UDP 7           /* layers.UDP               {45}            */
#define GPK_DEC_PAYLOAD 8       /* gopacket.Payload         {2}  (base.go:40-70)   */
#define GPK_DEC_FRAGMENT 9      /* gopacket.Fragment        {3}  (base.go:97-124)  */
#define GPK_NUM_DEC 10

/* ---- compact codes of the decoded LayerType list --------------------------
 * gpk_record.layers holds decoded[i] as a 4-bit code in bits [4i, 4i+4).     */
#define GPK_CODE_NONE 0
#define GPK_CODE_ETHERNET 1
#define GPK_CODE_DOT1Q 2
#define GPK_CODE_IPV4 3
#define GPK_CODE_IPV6 4
#define GPK_CODE_IPV6_HOPBYHOP 5
#define GPK_CODE_IPV6_ROUTING 6
#define GPK_CODE_IPV6_FRAGMENT 7
#define GPK_CODE_IPV6_DESTINATION 8
#define GPK_CODE_TCP 9
#define GPK_CODE_UDP 10
#define GPK_CODE_PAYLOAD 11
#define GPK_CODE_FRAGMENT 12
#define GPK_MAX_INLINE_LAYERS 16

/* ---- error sites ----------------------------------------------------------
 * One code per error value DecodeLayers can return. Args are in
 * err_args[2*i], err_args[2*i+1]; gpk_format_error renders the exact Go text. */
enum gpk_err {
  GPK_ERR_NONE = 0,
  GPK_ERR_UNSUPPORTED = 1,        /* a0=LayerType      parser.go:326  */
  GPK_ERR_PANIC_INDEX = 2,        /* a0=index a1=len   runtime "index out of range [a0] with length a1" */
  GPK_ERR_PANIC_SLICE_ACAP = 3,   /* a0=high a1=cap    runtime "slice bounds out of range [:a0] with capacity a1" */
  GPK_ERR_PANIC_SLICE_B = 4,      /* a0=low a1=high    runtime "slice bounds out of range [a0:a1]" */
  GPK_ERR_ETH_TOO_SMALL = 10,     /* ethernet.go:44 */
  GPK_ERR_DOT1Q_SHORT = 11,       /* a0=len dot1q.go:33 */
  GPK_ERR_IP4_HDR_SHORT = 20,     /* a0=len ip4.go:181 */
  GPK_ERR_IP4_LEN_SMALL = 21,     /* a0=Length ip4.go:196 */
  GPK_ERR_IP4_IHL_SMALL = 22,     /* a0=IHL ip4.go:198 */
  GPK_ERR_IP4_IHL_GT_LEN = 23,    /* a0=IHL a1=Length ip4.go:200 */
  GPK_ERR_IP4_HDR_MISSING = 24,   /* ip4.go:208 */
  GPK_ERR_IP4_OPT_SHORT = 25,     /* a0=remaining ip4.go:241 */
  GPK_ERR_IP4_OPT_EXCEEDS = 26,   /* a0=type a1=length ip4.go:247 */
  GPK_ERR_IP4_OPT_BADLEN = 27,    /* a0=type a1=length ip4.go:250 */
  GPK_ERR_IP6_HDR_SHORT = 30,     /* a0=len ip6.go:224 */
  GPK_ERR_IP6_JUMBO_AND_LEN = 31, /* ip6.go:258 */
  GPK_ERR_IP6_LEN0_NO_JUMBO = 32, /* ip6.go:260 */
  GPK_ERR_IP6_LEN0 = 33,          /* a0=NextHeader ip6.go:267 */
  GPK_ERR_IP6_TLV_SHORT = 34,     /* ip6.go:330 */
  GPK_ERR_IP6_TLV_TOO_SMALL = 35, /* ip6.go:342 */
  GPK_ERR_IP6_EXT_SHORT = 36,     /* a0=len ip6.go:421 */
  GPK_ERR_IP6_EXT_LEN = 37,       /* a0=len a1=actual ip6.go:427 */
  GPK_ERR_IP6_JUMBO_TLV_LEN = 38, /* ip6.go:68 */
  GPK_ERR_IP6_JUMBO_SMALL = 39,   /* ip6.go:72 */
  GPK_ERR_TCP_HDR_SHORT = 40,     /* a0=len tcp.go:294 */
  GPK_ERR_TCP_DOFF_SMALL = 41,    /* a0=DataOffset tcp.go:323 */
  GPK_ERR_TCP_DOFF_GT_LEN = 42,   /* tcp.go:330 */
  GPK_ERR_MPTCP_LEN = 43,         /* a0=len tcp.go:351 */
  GPK_ERR_MP_CAPABLE_LEN = 44,    /* a0=len tcp.go:357 */
  GPK_ERR_MP_JOIN_LEN = 45,       /* a0=len tcp.go:384 */
  GPK_ERR_DSS_LEN = 46,           /* a0=len tcp.go:415 */
  GPK_ERR_ADD_ADDR_LEN = 47,      /* a0=len tcp.go:455 */
  GPK_ERR_REM_ADDR_LEN = 48,      /* a0=len tcp.go:487 */
  GPK_ERR_MP_PRIO_LEN = 49,       /* a0=len tcp.go:499 */
  GPK_ERR_MP_FAIL_LEN = 50,       /* a0=len tcp.go:509 */
  GPK_ERR_MP_FASTCLOSE_LEN = 51,  /* a0=len tcp.go:517 */
  GPK_ERR_MP_TCPRST_LEN = 52,     /* a0=len tcp.go:524 */
  GPK_ERR_TCP_OPT_SHORT = 53,     /* a0=remaining tcp.go:537 */
  GPK_ERR_TCP_OPT_LEN_SMALL = 54, /* a0=len tcp.go:541 */
  GPK_ERR_TCP_OPT_EXCEEDS = 55,   /* a0=len a1=remaining tcp.go:544 */
  GPK_ERR_UDP_HDR_SHORT = 60,     /* a0=len udp.go:33 */
  GPK_ERR_UDP_TOO_SMALL = 61      /* a0=Length udp.go:53 */
};

/* ---- per-packet result record (16 B, one dwordx4 store per packet) -------- */
typedef struct gpk_record {
  uint64_t layers;   /* decoded list, 4-bit GPK_CODE_* per entry (first 16) */
  uint32_t status;   /* GPK_ST_* bit fields below */
  uint16_t ip4_csum; /* IPv4 ChecksumVerificationResult.Correct */
  uint16_t l4_csum;  /* TCP/UDP ChecksumVerificationResult.Correct */
} gpk_record;

#define GPK_ST_ERR_MASK 0x7Fu          /* gpk_err code                         */
#define GPK_ST_TRUNCATED (1u << 7)      /* DecodingLayerParser.Truncated        */
#define GPK_ST_NLAYERS_SHIFT 8          /* len(decoded), saturating at 4095     */
#define GPK_ST_NLAYERS_MASK 0xFFFu
#define GPK_ST_IP4_CSUM (1u << 20)      /* IPv4 checksum computed               */
#define GPK_ST_IP4_VALID (1u << 21)     /* ... and Valid                        */
#define GPK_ST_L4_CSUM (1u << 22)       /* TCP or UDP checksum computed         */
#define GPK_ST_L4_VALID (1u << 23)      /* ... and Valid                        */
#define GPK_ST_L4_UDP (1u << 24)        /* the transport layer is UDP           */
#define GPK_ST_LINK_FLOW (1u << 25)     /* flows[0*n+i] holds LinkFlow().FastHash()      */
#define GPK_ST_NET_FLOW (1u << 26)      /* flows[1*n+i] holds NetworkFlow().FastHash()   */
#define GPK_ST_NET_IPV6 (1u << 27)      /* the network flow is IPv6                      */
#define GPK_ST_TRANSPORT_FLOW (1u << 28)/* flows[2*n+i] holds TransportFlow().FastHash() */

static inline unsigned gpk_record_err(const gpk_record* r) { return r->status & GPK_ST_ERR_MASK; }
static inline unsigned gpk_record_nlayers(const gpk_record* r) {
  return (r->status >> GPK_ST_NLAYERS_SHIFT) & GPK_ST_NLAYERS_MASK;
}

/* ---- narrow per-packet result record (8 B, gpk_decode_batch_narrow) --------
 * The same result in half the bytes, for the batches whose cost is the bytes a
 * decode writes (small packets: the 16-byte record is a fifth of C2's memory
 * traffic). ChecksumVerificationResult.Correct equals Actual whenever it is
 * Valid (checksum.go:9-21), except for a UDP checksum of 0, which is Valid
 * unchecked (udp.go:144-158); so the narrow record keeps the status bits and
 * the first 8 codes of the decoded list, and a packet whose record does not
 * fit (more than 8 layers, or an IPv4 / TCP / UDP Correct that differs from the
 * header's Checksum field) has GPK_ST8_WIDE set and its full gpk_record in
 * the side array wide[i], which is written for those packets only (as
 * err_args is written only on error). For a packet without GPK_ST8_WIDE the
 * gpk_record is {layers, status with nlayers, ip4_csum = the IPv4 Checksum
 * field when GPK_ST_IP4_CSUM (else 0), l4_csum = the TCP / UDP Checksum field
 * when GPK_ST_L4_CSUM (else 0)}: the fields of the layer structs DecodeLayers
 * filled (the last IPv4, the transport layer). */
typedef struct gpk_record8 {
  uint32_t layers;   /* decoded list, 4-bit GPK_CODE_* per entry (first 8)                    */
  uint32_t status;   /* the GPK_ST_* bits, with len(decoded) in 4 bits and GPK_ST8_WIDE below */
} gpk_record8;
#define GPK_ST8_NLAYERS_MASK 0xFu /* at GPK_ST_NLAYERS_SHIFT: len(decoded), 15 when more than 8 */
#define GPK_ST8_WIDE (1u << 12)   /* the packet's full gpk_record is in wide[i]                 */

typedef struct gpk_results8 {
  gpk_record8* records; /* [n]   required                                                 */
  gpk_record* wide;     /* [n]   required; written only where GPK_ST8_WIDE is set           */
  uint32_t* err_args;   /* [2n]  optional; written only for packets with err                */
  uint64_t* flows;      /* [3n]  as gpk_results.flows; required if GPK_OUT_FLOWS            */
} gpk_results8;

static inline unsigned gpk_record8_nlayers(const gpk_record8* r) {
  return (r->status >> GPK_ST_NLAYERS_SHIFT) & GPK_ST8_NLAYERS_MASK;
}

/* ---- optional per-packet layout (64 B): where each layer struct points ----
 * For every DecodingLayer implementation (slot = kind-1, Payload and Fragment
 * share slot 7) the byte range [start, end) — relative to the packet start —
 * of the data slice handed to the LAST successful DecodeFromBytes of that
 * instance (gopacket reuses one struct per type, parser.go:21-28, so the last
 * writer wins). 0xFFFFFFFF = the layer was not decoded. Every field value of
 * that struct is a pure function of the packet bytes in that range.          */
typedef struct gpk_layout {
  uint32_t start[8];
  uint32_t end[8];
} gpk_layout;
#define GPK_LAYOUT_ABSENT 0xFFFFFFFFu

/* ---- optional per-packet layer fields (128 B) -----------------------------
 * The scalar fields the decoders' DecodeFromBytes set on their structs, read
 * from the bytes of each decoder's last successful slice (the gpk_layout of a
 * gpk_decode_batch with layouts), so a consumer that reads layer fields after
 * DecodeLayers gets them from the device instead of decoding headers again.
 * present: bit k set = layout slot k holds a slice (k = GPK_DEC_* - 1; Payload
 * and Fragment share slot 7); every field of an absent layer is 0. Integers in
 * host byte order; MACs and addresses as their bytes. Variable-length parts
 * (Payload, option data) stay in the packet bytes; the IPv4, TCP and IPv6
 * HopByHop option lists are described by their option start maps.
 * Stacked layers (QinQ, IP in IP, 6in6): the fields are the LAST instance's,
 * as the reference's one struct per type holds them (parser.go:21-28, last
 * writer wins); ip4_start / tcp_start are 0xFF when that header starts at
 * packet byte 255 or later (the record has one byte each; Hydrate derives the
 * starts from the decoded list instead).                                     */
typedef struct gpk_fields {
  uint8_t present;           /*   0                                                       */
  uint8_t hbh_opt_map[3];    /*   1 IPv6.HopByHop.Options (the last IPv6's inline HopByHop,
                                    ip6.go:244-256, 509-526): bit k (byte k/8, bit k%8) set =
                                    an option starts at HopByHop byte 2 + k; covers headers of
                                    up to 24 bytes (HeaderLength <= 2), 0 for longer ones     */
  uint16_t eth_type;         /*   4 Ethernet.EthernetType (EthernetTypeLLC = 0 below 0x0600) */
  uint16_t eth_length;       /*   6 Ethernet.Length (802.3 frames, else 0)               */
  uint8_t eth_dst[6];        /*   8 Ethernet.DstMAC                                       */
  uint8_t eth_src[6];        /*  14 Ethernet.SrcMAC                                       */
  uint16_t d1q_tci;          /*  20 Dot1Q Priority << 13 | DropEligible << 12 | VLANIdentifier */
  uint16_t d1q_type;         /*  22 Dot1Q.Type                                            */
  uint8_t ip4_version;       /*  24 IPv4.Version                                          */
  uint8_t ip4_ihl;           /*  25 IPv4.IHL                                              */
  uint8_t ip4_tos;           /*  26 IPv4.TOS                                              */
  uint8_t ip4_ttl;           /*  27 IPv4.TTL                                              */
  uint16_t ip4_length;       /*  28 IPv4.Length (the slice's length when the field is 0: TSO) */
  uint16_t ip4_id;           /*  30 IPv4.Id                                               */
  uint16_t ip4_flags_frag;   /*  32 IPv4.Flags << 13 | IPv4.FragOffset                    */
  uint8_t ip4_protocol;      /*  34 IPv4.Protocol                                         */
  uint8_t ip6_version;       /*  35 IPv6.Version                                          */
  uint16_t ip4_checksum;     /*  36 IPv4.Checksum                                         */
  uint8_t ip6_traffic_class; /*  38 IPv6.TrafficClass                                     */
  uint8_t ip6_next_header;   /*  39 IPv6.NextHeader                                       */
  uint32_t ip6_flow_label;   /*  40 IPv6.FlowLabel                                        */
  uint16_t ip6_length;       /*  44 IPv6.Length (0 for a jumbogram)                       */
  uint8_t ip6_hop_limit;     /*  46 IPv6.HopLimit                                         */
  uint8_t tcp_data_offset;   /*  47 TCP.DataOffset                                        */
  uint8_t ip4_src[4];        /*  48 IPv4.SrcIP                                            */
  uint8_t ip4_dst[4];        /*  52 IPv4.DstIP                                            */
  uint8_t ip6_src[16];       /*  56 IPv6.SrcIP                                            */
  uint8_t ip6_dst[16];       /*  72 IPv6.DstIP                                            */
  uint16_t tcp_src_port;     /*  88 TCP.SrcPort                                           */
  uint16_t tcp_dst_port;     /*  90 TCP.DstPort                                           */
  uint32_t tcp_seq;          /*  92 TCP.Seq                                               */
  uint32_t tcp_ack;          /*  96 TCP.Ack                                               */
  uint16_t tcp_flags;        /* 100 FIN 1 SYN 2 RST 4 PSH 8 ACK 16 URG 32 ECE 64 CWR 128 NS 256 */
  uint16_t tcp_window;       /* 102 TCP.Window                                            */
  uint16_t tcp_checksum;     /* 104 TCP.Checksum                                          */
  uint16_t tcp_urgent;       /* 106 TCP.Urgent                                            */
  uint16_t udp_src_port;     /* 108 UDP.SrcPort                                           */
  uint16_t udp_dst_port;     /* 110 UDP.DstPort                                           */
  uint16_t udp_length;       /* 112 UDP.Length                                            */
  uint16_t udp_checksum;     /* 114 UDP.Checksum                                          */
  uint8_t ip4_start;         /* 116 packet offset of the IPv4 header (its layout start); 0xFF: absent or >= 255 */
  uint8_t tcp_start;         /* 117 packet offset of the TCP header; 0xFF: absent or >= 255   */
  uint8_t ip4_opt_map[5];    /* 118 IPv4.Options: bit k (byte k/8, bit k%8) set = an option starts at
                                    header byte 20 + k (ip4.go:219-256); see below              */
  uint8_t tcp_opt_map[5];    /* 123 TCP.Options: the same at TCP header byte 20 + k (tcp.go:336-549) */
} gpk_fields;
/* Option lists without decoding again: option j of the list is at the j-th set
 * bit k of the map, at packet byte b = <layer>_start + 20 + k; OptionType =
 * pkt[b]; OptionLength = 1 for kinds 0 (End of options) and 1 (No-op), else
 * pkt[b+1]; OptionData = pkt[b+2 : b+OptionLength] (IPv4 and TCP kinds other
 * than 0, 1 and 30). A list that ends with kind 0 has Padding = the header's
 * bytes after it (ip4.go:231, tcp.go:343). Every option lies inside the
 * header the layer decoded (the decode checked each length).
 * HopByHop (IPv6 NextHeader 0, header at the IPv6 start + 40): option j at the
 * j-th set bit k of hbh_opt_map, HopByHop byte b = 2 + k; OptionType = hbh[b];
 * type 0 (Pad1): ActualLength 1, no length or data; else OptionLength =
 * hbh[b+1], ActualLength = OptionLength + 2, OptionData = hbh[b+2 :
 * b+ActualLength] (ip6.go:327-346; the last option may extend past the
 * header's ActualLength, as the reference's loop allows). */

/* ---- outputs -------------------------------------------------------------- */
#define GPK_OUT_IP4_CSUM 0x1u  /* IPv4.VerifyChecksum for the last IPv4 in decoded        */
#define GPK_OUT_L4_CSUM 0x2u   /* TCP/UDP.VerifyChecksum, pseudo-header = last network layer */
#define GPK_OUT_FLOWS 0x4u     /* Link/Network/Transport Flow.FastHash                    */
#define GPK_OUT_ALL 0x7u

/* ---- parser configuration (opaque) ---------------------------------------- */
typedef struct gpk_parser gpk_parser;

/* NewDecodingLayerParser(first): an empty container, default options. */
int gpk_parser_create(gpk_parser** out, int64_t first_layer_type);
int gpk_parser_destroy(gpk_parser* p);
/* AddDecodingLayer(d) / DecodingLayerContainer.Put(d): registers every
 * LayerType of the decoder's CanDecode() class; a later Put overrides. */
int gpk_parser_add_decoder(gpk_parser* p, int decoder_kind);
/* DecodingLayerParserOptions. */
int gpk_parser_set_options(gpk_parser* p, int ignore_panic, int ignore_unsupported);
/* Which verification / hashing results to compute (GPK_OUT_*). */
int gpk_parser_set_outputs(gpk_parser* p, uint32_t outputs);
/* LayerType -> decoder kind currently registered (GPK_DEC_NONE if none). */
int gpk_parser_decoder_for(const gpk_parser* p, int64_t layer_type);

/* Next-layer tables: EthernetType[65536], IPProtocol[256], TCP port[65536],
 * UDP port[65536] -> LayerType. Defaults = the reference registry after init()
 * (including the Modbus/ENIP port overrides). Overrides made at run time by
 * RegisterTCPPortLayerType / RegisterUDPPortLayerType or by editing
 * EthernetTypeMetadata / IPProtocolMetadata are mirrored with these setters. */
int gpk_parser_set_ethertype(gpk_parser* p, uint32_t ethertype, int32_t layer_type);
int gpk_parser_set_ipprotocol(gpk_parser* p, uint32_t proto, int32_t layer_type);
int gpk_parser_set_tcp_port(gpk_parser* p, uint32_t port, int32_t layer_type);
int gpk_parser_set_udp_port(gpk_parser* p, uint32_t port, int32_t layer_type);

/* ---- device context ------------------------------------------------------- */
typedef struct gpk_ctx gpk_ctx;
int gpk_ctx_create(gpk_ctx** out, int device_ordinal);
int gpk_ctx_destroy(gpk_ctx* ctx);
/* Where the kernels read the parser's next-layer tables (EthernetType /
 * IPProtocol / TCPPort / UDPPort -> LayerType, layers/enums.go:294-353,
 * layers/ports.go:54-183). AUTO (default): a compact copy in LDS whenever the
 * tables fit (a few dozen non-default entries each, as the defaults are),
 * else the full tables in device memory. GLOBAL: always the full tables.
 * Results are identical; GLOBAL exists for testing and diagnosis. */
#define GPK_TABLES_AUTO 0
#define GPK_TABLES_GLOBAL 1
int gpk_ctx_set_table_mode(gpk_ctx* ctx, int mode);
/* Ends the gpk_replay_file, gpk_replay_file_range and gpk_tpacket_pump calls
 * running on ctx early: what a Go caller does by breaking out of its
 * ReadPacketData loop (ngread.go:629-632, afpacket.go:335-367), for the calls
 * that push results through callbacks. Callable from inside any of their
 * callbacks or from another thread, any number of times. Each such call checks
 * before every batch it delivers: from the first check after gpk_stop returned
 * it makes no further callback (a batch's packets, fields and results callbacks
 * are made for all of it or none of it), waits for its own reads, copies and
 * kernels, and returns GPK_STOPPED with stats.packets = the packets delivered;
 * a range replay is then not clean. A call that starts after gpk_stop returned
 * is not affected. */
int gpk_stop(gpk_ctx* ctx);

/* A packed, offset-indexed packet batch. Packet i is data[offsets[i] ..
 * offsets[i]+caplens[i]). In gpk_decode_batch every pointer is DEVICE memory;
 * data must be 16-byte aligned.
 * Reads: whole 16-byte-aligned chunks of data. Every chunk read lies between
 * the first and the last byte of the packets of one group of 64 consecutive
 * packets (a wave), so data must be one allocation covering all packets.
 * data_bytes: the size of data in bytes (gpk_decode_batch_host copies that
 * many); 0 = unknown. gpk_decode_batch uses it as a hint of the mean packet
 * size (data_bytes / n selects a kernel variant) and as the readable end of
 * data for the small-packet kernel, which loads header words at dword rather
 * than 16-byte alignment only below data + data_bytes rounded up to 16 (a
 * packet whose header window would reach past it, and every packet when
 * data_bytes is 0, uses 16-byte-aligned loads). Pass the packed buffer size
 * (or at least the summed capture lengths) for best results; never more than
 * the readable bytes of data. n: at most (2^31 - 1) * 256 packets per call
 * (one workgroup per 256 packets), else GPK_EINVAL. */
typedef struct gpk_batch {
  const uint8_t* data;
  const uint64_t* offsets;
  const uint32_t* caplens;
  uint64_t n;
  uint64_t data_bytes;
} gpk_batch;

typedef struct gpk_results {
  gpk_record* records;  /* [n]   required                                   */
  uint32_t* err_args;   /* [2n]  optional; written only for packets with err */
  uint64_t* flows;      /* [3n]  SoA link[n], net[n], transport[n]; required
                           if GPK_OUT_FLOWS (0 where the flow is absent)     */
  gpk_layout* layouts;  /* [n]   optional                                    */
} gpk_results;

/* Device-resident decode of every packet of the batch, enqueued on `stream`
 * (a hipStream_t, NULL = the null stream). Asynchronous: returns after the
 * launch. The parser configuration is uploaded once per (ctx, parser change). */
int gpk_decode_batch(gpk_ctx* ctx, const gpk_parser* p, const gpk_batch* batch,
                     const gpk_results* out, void* stream);

/* gpk_decode_batch with the narrow 8-byte record (gpk_record8 above) and its
 * side array of full records; device memory, same stream semantics. No
 * layouts. The results are exactly gpk_decode_batch's, in the narrow form. */
int gpk_decode_batch_narrow(gpk_ctx* ctx, const gpk_parser* p, const gpk_batch* batch,
                            const gpk_results8* out, void* stream);

/* Layer fields of every packet of a device batch from the layouts a
 * gpk_decode_batch with layouts wrote for it (device memory; fields[n] device
 * memory), enqueued on `stream`. Asynchronous. The batch is the one decoded. */
int gpk_extract_fields(const gpk_batch* batch, const gpk_layout* layouts, gpk_fields* fields, void* stream);

/* Device-resident decode of every packet plus the layer fields of each
 * (gpk_fields, as gpk_extract_fields writes them) in ONE launch: the decode
 * kernel reads the fields from the header bytes it parsed, so no layout
 * round trip through HBM. fields[n]: device memory. out->layouts NULL: the
 * fused launch; non-NULL: the decode with layouts, then gpk_extract_fields
 * (two launches, same results). Same stream semantics as gpk_decode_batch. */
int gpk_decode_batch_fields(gpk_ctx* ctx, const gpk_parser* p, const gpk_batch* batch,
                            const gpk_results* out, gpk_fields* fields, void* stream);

/* Diagnostic: the name of the kernel specialisation gpk_decode_batch launches
 * for this parser and batch (with_layouts 0 / 1), or gpk_decode_batch_fields
 * without layouts (with_layouts = GPK_NAME_FIELDS), e.g.
 * "gpk::decode_kernel<true,false,true,false,5,7,4>" — the name rocprofv3 lists.
 * Returns the name's length. */
#define GPK_NAME_FIELDS 2
int gpk_decode_kernel_name(gpk_ctx* ctx, const gpk_parser* p, const gpk_batch* batch, int with_layouts,
                           char* buf, size_t cap);

/* Diagnostic: how many 256-packet blocks of that specialisation are resident
 * per CU with this parser's LDS table blob (hipOccupancyMaxActiveBlocksPerMultiprocessor);
 * with_layouts as for gpk_decode_kernel_name. */
int gpk_decode_occupancy(gpk_ctx* ctx, const gpk_parser* p, const gpk_batch* batch, int with_layouts,
                         int* blocks_per_cu);

/* Diagnostic: device buffer (8 u64 per 64-packet wave, or NULL) that libraries
 * built with GPK_DIAG_TIMES fill with per-wave phase timestamps on every
 * decode launch (tools/wave_times.py). Ignored by the default build. */
int gpk_diag_set_buffer(void* buf);

/* Host-memory variant: batch and results live in host memory (ideally pinned
 * via gpk_host_alloc). Copies HtoD, decodes, copies DtoH; synchronous. */
int gpk_decode_batch_host(gpk_ctx* ctx, const gpk_parser* p, const gpk_batch* host_batch,
                          const gpk_results* host_out);
/* The same with the layer fields of every packet (gpk_fields, as
 * gpk_decode_batch_fields writes them) into host memory host_fields[n]: the
 * fused decode + fields launch, or with host_out->layouts the decode and then
 * gpk_extract_fields. For callers whose packets are in host memory (a cgo
 * caller without device buffers of its own). Synchronous. */
int gpk_decode_batch_host_fields(gpk_ctx* ctx, const gpk_parser* p, const gpk_batch* host_batch,
                                 const gpk_results* host_out, gpk_fields* host_fields);

/* Full decoded list of a packet whose list is longer than 16 entries
 * (gpk_record_nlayers > 16). Device batch, device result not needed; writes
 * up to `cap` LayerType values to host memory `out_types`, returns count. */
int gpk_decoded_list(gpk_ctx* ctx, const gpk_parser* p, const gpk_batch* batch,
                     uint64_t index, int64_t* out_types, uint32_t cap, uint32_t* out_n);

/* Same for one packet in host memory (the single-packet DecodeLayers path). */
int gpk_decoded_list_host(gpk_ctx* ctx, const gpk_parser* p, const uint8_t* pkt, uint32_t caplen,
                          int64_t* out_types, uint32_t cap, uint32_t* out_n);

/* Page-locked host memory for gpk_decode_batch_host and the replay paths:
 * below 4 MiB hipHostMalloc; from 4 MiB an anonymous 2 MiB-aligned mapping
 * (transparent huge pages) faulted in on up to 8 threads and registered with
 * hipHostRegister. Either way it is ordinary host memory for HIP copies, not a
 * device-mapped (zero-copy) pointer, and it must be released with
 * gpk_host_free (never hipHostFree / free). A request larger than the host's
 * MemAvailable fails with GPK_EHIP (hipErrorOutOfMemory) instead of faulting. */
int gpk_host_alloc(void** out, size_t bytes);
int gpk_host_free(void* p);

/* Exact Go error text of a record's error (no trailing NUL counted).
 * Returns the length written (truncated to cap-1 and NUL-terminated). */
int gpk_format_error(unsigned err_code, uint32_t a0, uint32_t a1, char* buf, size_t cap);
/* LayerType.String() (layertype.go:101-111). */
int gpk_layer_type_name(int64_t layer_type, char* buf, size_t cap);

/* Map a compact code to its LayerType id (GPK_CODE_* -> GPK_LT_*). */
int64_t gpk_code_layer_type(unsigned code);

const char* gpk_strerror(int status);
const char* gpk_last_hip_error(void);
int gpk_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* GPK_H */

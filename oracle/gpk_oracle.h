/*
 * gpk_oracle.h — CPU restatement of gopacket's DecodingLayerParser fast path.
 *
 * TEST INFRASTRUCTURE ONLY. This is the checker the HIP engine is compared
 * against: tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * load it; nothing in gopacket_amd/ links, loads or calls it.
 *
 * It is a line-by-line restatement of the reference Go code (cited per
 * function in gpk_oracle.c), written for obviousness, not speed: byte-serial
 * checksum (checksum.go:35-50), byte-serial FNV (flows.go:60-70), Go slice
 * semantics with explicit len/cap so that the reference's runtime panics
 * (MPTCP option parsing, tcp.go:347-548) are reproduced.
 *
 * Parity pinning: the oracle is checked against every known-answer vector the
 * reference's own tests hold for this path (tests/golden/, see
 * tests/test_oracle_golden.py). Flow.FastHash has no reference known-answer
 * test; it is pinned by the published FNV-1a-64 vectors and the symmetry
 * property documented at flows.go:159-166.
 *
 * Output format: exactly the gpk_record / err_args / flows / gpk_layout
 * arrays of include/gpk.h, so device and oracle results compare bytewise.
 */
#ifndef GPK_ORACLE_H
#define GPK_ORACLE_H

#include <stdint.h>
#include "../include/gpk.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_config {
  int64_t first;                 /* first LayerType                           */
  uint8_t dispatch[GPK_MAX_LAYER_TYPE]; /* LayerType -> GPK_DEC_* (container) */
  int ignore_unsupported;
  int ignore_panic;
  uint32_t outputs;              /* GPK_OUT_*                                 */
  int32_t ethertype[65536];
  int32_t ipprotocol[256];
  int32_t tcp_port[65536];
  int32_t udp_port[65536];
} oracle_config;

/* Empty container, first layer, registry defaults, all outputs. */
void oracle_config_init(oracle_config* c, int64_t first);
/* DecodingLayerContainer.Put for one of the GPK_DEC_* implementations. */
void oracle_config_put(oracle_config* c, int decoder_kind);

/* Decode packets [0, n). flows is SoA: link[n], net[n], transport[n]. Any
 * output pointer but records may be NULL. nthreads <= 1 runs serially. */
void oracle_decode_batch(const oracle_config* c, const uint8_t* data, const uint64_t* offsets,
                         const uint32_t* caplens, uint64_t n, gpk_record* records,
                         uint32_t* err_args, uint64_t* flows, gpk_layout* layouts, int nthreads);

/* The scalar layer fields (include/gpk.h gpk_fields) of packets [0, n) from
 * the layouts of a decode: each decoder's DecodeFromBytes field assignments
 * restated on its slice. */
void oracle_extract_fields(const uint8_t* data, const uint64_t* offsets, const gpk_layout* layouts, uint64_t n,
                           gpk_fields* out);

/* Full decoded LayerType list of one packet; returns its length (may exceed cap). */
uint32_t oracle_decoded_list(const oracle_config* c, const uint8_t* pkt, uint32_t caplen,
                             int64_t* out, uint32_t cap);

/* Go error text for (code, a0, a1), exactly as DecodeLayers' error prints. */
int oracle_error_string(const oracle_config* c, unsigned code, uint32_t a0, uint32_t a1,
                        char* buf, int cap);

/* Building blocks exposed for known-answer tests (checksum.go, flows.go). */
uint32_t oracle_compute_checksum(const uint8_t* data, uint32_t len, uint32_t csum);
uint16_t oracle_fold_checksum(uint32_t csum);
uint64_t oracle_fnv_hash(const uint8_t* s, uint32_t len);
uint64_t oracle_flow_fast_hash(int64_t typ, const uint8_t* src, uint32_t slen, const uint8_t* dst,
                               uint32_t dlen);

uint64_t oracle_sizeof_config(void);
void oracle_config_set(oracle_config* c, int ignore_unsupported, int ignore_panic, uint32_t outputs);
/* 0 = EthernetType[65536], 1 = IPProtocol[256], 2 = TCP port[65536], 3 = UDP port[65536] */
int32_t* oracle_config_table(oracle_config* c, int which);

#ifdef __cplusplus
}
#endif
#endif

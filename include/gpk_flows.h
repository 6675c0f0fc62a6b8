/*
 * gpk_flows.h — flow-keyed grouping of a decoded batch on the device
 * (SURVEY.md §8(f)3).
 *
 * The consumers of the decode path that key packets by flow do one map
 * lookup per packet on the CPU. This groups a whole batch by the same key in
 * HBM, so a consumer receives, per key, the packets it would have routed to
 * that key, in packet order:
 *
 *   GPK_GROUP_CONNECTION   tcpassembly: key{netFlow, tcp.TransportFlow()}
 *                          (tcpassembly/assembly.go:292, AssembleWithTimestamp
 *                          :525-545, StreamPool.getConnection :498-517), after its
 *                          "ignoring useless packet" filter (:527-532)
 *   GPK_GROUP_DEFRAG       ip4defrag: ipv4{ip.NetworkFlow(), ip.Id}
 *                          (ip4defrag/defrag.go:328-341), for the packets
 *                          DefragIPv4WithTimestamp looks up (:85-105: dontDefrag
 *                          :160-170, securityChecks :173-196)
 *   GPK_GROUP_NET_BUCKET   the sharding idiom of doc.go:219-225:
 *                          int(net.NetworkFlow().FastHash()) & (buckets-1)
 *
 * Harness rules (the reference leaves them to the caller; fixed here as the
 * L4 checksum's pseudo-header rule is):
 *   - netFlow for CONNECTION is the NetworkFlow() of the last network layer
 *     (IPv4 / IPv6) in `decoded` before TCP, holding the last-writer struct;
 *   - a packet is keyed when its layer was decoded (it is in `decoded`),
 *     whatever error a later layer returned; for DEFRAG the IPv4 struct must
 *     not have been left mid-decode by a failed IPv4 decode.
 *
 * Groups are numbered in order of first appearance (the order in which the
 * reference's map would have gained the key); inside a group packets are in
 * batch order. Keys are compared exactly (all Flow bytes), hashes only bucket.
 */
#ifndef GPK_FLOWS_H
#define GPK_FLOWS_H

#include <stddef.h>
#include <stdint.h>

#include "gpk.h"

#ifdef __cplusplus
extern "C" {
#endif

#define GPK_GROUP_CONNECTION 1
#define GPK_GROUP_DEFRAG 2
#define GPK_GROUP_NET_BUCKET 3

/* group_of[i] for a packet in no group */
#define GPK_GROUP_NONE (-1)           /* the key does not apply: no TCP / no network layer /
                                         not a fragment (dontDefrag)                      */
#define GPK_GROUP_USELESS (-2)        /* tcpassembly ignores it: no SYN/FIN/RST, no payload */
#define GPK_GROUP_FRAG_TOO_SMALL (-3) /* securityChecks: "fragment too small"  defrag.go:177 */
#define GPK_GROUP_FRAG_OFFSET (-4)    /* securityChecks: "fragment offset too big"     :183 */
#define GPK_GROUP_FRAG_OVERRUN (-5)   /* securityChecks: "fragment will overrun"       :190 */
#define GPK_GROUP_UNKNOWN (-6)        /* decoded list longer than 16 entries: the device does
                                         not see which network layer precedes TCP         */

typedef struct gpk_grouper gpk_grouper;

/* Workspace for batches of up to max_packets (< 2^28) on one device. A
 * grouper's workspace serves one call at a time: calls on one stream are
 * ordered; concurrent streams need one grouper each. */
int gpk_grouper_create(gpk_grouper** out, int device, uint64_t max_packets);
int gpk_grouper_destroy(gpk_grouper* g);

/* Device arrays, caller-allocated, n = batch size. */
typedef struct gpk_groups {
  int32_t* group_of; /* [n]   group id, or a GPK_GROUP_* code < 0                  */
  uint32_t* perm;    /* [n]   packets of group g: perm[start[g] .. start[g+1]),
                              ascending; keyed packets first                      */
  uint32_t* start;   /* [n+1]                                                      */
  uint32_t* first;   /* [n]   first packet of each group (its key's representative) */
  uint32_t* counts;  /* [2]   number of groups, number of keyed packets            */
} gpk_groups;

/* Group the packets of a decoded batch (device-resident, as for
 * gpk_decode_batch) by `kind`. res must hold records and layouts (CONNECTION,
 * DEFRAG; decoded with layouts) or records and flows (NET_BUCKET, decoded
 * with GPK_OUT_FLOWS); buckets is a power of two (NET_BUCKET only).
 * Asynchronous on `stream`. */
int gpk_group_batch(gpk_grouper* g, const gpk_batch* batch, const gpk_results* res, int kind, uint32_t buckets,
                    const gpk_groups* out, void* stream);

/* gpk_decode_batch and gpk_group_batch (CONNECTION or DEFRAG) in one: the
 * decode kernel derives each packet's key from the header bytes it already
 * holds in LDS, so the grouping reads no layouts and no header bytes again.
 * res as for gpk_decode_batch, without layouts (GPK_EINVAL otherwise); same
 * groups as gpk_decode_batch with layouts followed by gpk_group_batch. */
int gpk_decode_group_batch(gpk_ctx* ctx, const gpk_parser* p, const gpk_batch* batch, const gpk_results* res,
                           gpk_grouper* g, int kind, const gpk_groups* out, void* stream);

/* Pack packets order[0..m) of a batch into a dense batch, in that order:
 * out_data receives their bytes back to back (it must hold their total
 * length), out_offsets[j] / out_caplens[j] index packet order[j]. The send
 * side of a per-flow exchange between GPUs (gopacket_amd/shard.py
 * exchange_packets: the doc.go:219-225 sharding idiom across ranks), or a
 * filtered batch made dense. Device arrays; asynchronous on stream. */
int gpk_pack_batch(const gpk_batch* in, const uint32_t* order, uint64_t m, uint8_t* out_data, uint64_t* out_offsets,
                   uint32_t* out_caplens, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GPK_FLOWS_H */

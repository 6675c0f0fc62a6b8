/*
 * gpk_afpacket.h — AF_PACKET memory-mapped ring → packet batches
 * (SURVEY.md §8(f)2).
 *
 * A TPACKET_V3 ring hands user space whole blocks of packets; a retired
 * block is already a packed batch with per-frame offsets. This header
 * replaces, for a Go caller binding it through cgo:
 *
 *   gpk_tp_default_opts / gpk_tp_check_opts   afpacket parseOptions + options.check
 *                                             afpacket/options.go:160-211 (defaults :126-158)
 *   gpk_tpacket_new                           afpacket.NewTPacket  afpacket.go:261-294
 *                                             (bindToInterface :155-171, setRequestedTPacketVersion
 *                                             :182-194, setVNetHdrSize :197-202, setUpRing :205-240,
 *                                             InitSocketStats :378-399)
 *   gpk_tpacket_attach                        (no reference counterpart) the same reader over a ring
 *                                             the caller owns: tests, replays, the benchmark
 *   gpk_tpacket_index                         a loop of TPacket.ZeroCopyReadPacketData calls
 *                                             afpacket.go:335-367 (getTPacketHeader :462-486,
 *                                             pollForFirstPacket :488-516, releaseCurrentPacket
 *                                             :316-321) over the v1/v2/v3 headers of header.go
 *   gpk_tpacket_stats / _socket_stats         TPacket.Stats :370-375, SocketStats :402-431
 *   gpk_tpacket_set_bpf / _set_fanout         TPacket.SetBPF :297-309, SetFanout :542-548
 *   gpk_tpacket_set_ebpf / _set_promiscuous   TPacket.SetEBPF :312-314, SetPromiscuous :552-564
 *   gpk_tpacket_write                         TPacket.WritePacketData :567-570
 *   gpk_tpacket_init_socket_stats             TPacket.InitSocketStats :378-399
 *   gpk_tpacket_pump                          the capture loop: ZeroCopyReadPacketData +
 *                                             DecodingLayerParser.DecodeLayers per packet,
 *                                             pipelined through HBM
 *
 * Versions use the kernel's numbering, as OptTPacketVersion does:
 * TPACKET_V1 = 0, TPACKET_V2 = 1, TPACKET_V3 = 2, highest available = -1.
 */
#ifndef GPK_AFPACKET_H
#define GPK_AFPACKET_H

#include <stddef.h>
#include <stdint.h>

#include "gpk.h"

#ifdef __cplusplus
extern "C" {
#endif

#define GPK_TPACKET_V1 0
#define GPK_TPACKET_V2 1
#define GPK_TPACKET_V3 2
#define GPK_TPACKET_HIGHEST (-1)

/* afpacket options (options.go:84-99). Durations in nanoseconds. */
typedef struct gpk_tp_opts {
  int32_t version;          /* OptTPacketVersion                          */
  int32_t socktype;         /* OptSocketType: SOCK_RAW 3 / SOCK_DGRAM 2   */
  int32_t frame_size;       /* OptFrameSize   (DefaultFrameSize 4096)     */
  int32_t block_size;       /* OptBlockSize   (4096 * 128)                */
  int32_t num_blocks;       /* OptNumBlocks   (128)                       */
  int32_t frames_per_block; /* set by gpk_tp_check_opts: block/frame      */
  int32_t add_vlan_header;  /* OptAddVLANHeader                           */
  int32_t vnet_hdr_size;    /* OptVNetHdrSize                             */
  int64_t block_timeout_ns; /* OptBlockTimeout (64 ms)                    */
  int64_t poll_timeout_ns;  /* OptPollTimeout  (-1 ms: block forever)     */
  uint16_t protocol;        /* OptProtocol     (ETH_P_ALL)                */
  uint16_t _pad[3];
  char iface[64];           /* OptInterface ("" = every interface)        */
} gpk_tp_opts;

void gpk_tp_default_opts(gpk_tp_opts* o);
/* options.check(): 0, or GPK_EINVAL with Go's error text in err. On success
 * sets frames_per_block. */
int gpk_tp_check_opts(gpk_tp_opts* o, char* err, size_t cap);

typedef struct gpk_tpacket gpk_tpacket;

/* NewTPacket: AF_PACKET socket, ring, mmap (needs CAP_NET_RAW). On failure
 * returns GPK_EINVAL / GPK_EUNSUPP with the error text in err. */
int gpk_tpacket_new(gpk_tpacket** out, const gpk_tp_opts* o, char* err, size_t cap);
/* A reader over ring[0, bytes) laid out like the kernel's ring for `version`
 * (2 = TPACKET_V3 blocks, 0/1 = frames) with o's geometry. No socket: where
 * the reference would poll, gpk_tpacket_index returns GPK_TP_WAIT. */
int gpk_tpacket_attach(gpk_tpacket** out, void* ring, uint64_t bytes, int version, const gpk_tp_opts* o);
int gpk_tpacket_close(gpk_tpacket* t);
int gpk_tpacket_ring(const gpk_tpacket* t, void** ring, uint64_t* bytes, int* version, int* fd);

/* gopacket.CaptureInfo of one packet: Timestamp = time.Unix(ts_sec, ts_nsec),
 * CaptureLength = caplens[i], Length, InterfaceIndex, and AncillaryData =
 * [AncillaryVLAN{vlan}] when vlan >= 0 (header.go:224-230, v3 only). */
typedef struct gpk_tp_info {
  int64_t ts_sec;
  uint32_t ts_nsec;
  uint32_t length;
  int32_t iface;
  int32_t vlan;
} gpk_tp_info;

/* gpk_tpacket_index return values (>= 0) */
#define GPK_TP_WAIT 0  /* the next header is still the kernel's: where the reference polls.
                          Call again once it is handed over (or with wait=1 on a socket). */
#define GPK_TP_FULL 1  /* max packets written, or the side buffer is full             */
#define GPK_TP_ERROR 2 /* ZeroCopyReadPacketData returned an error: gpk_tpacket_error   */

/* Run ZeroCopyReadPacketData until max packets, a wait, or an error. Packet i
 * is ring[offsets[i], +caplens[i]) when offsets[i] < ring bytes, else
 * side[offsets[i] - ring bytes, ...): packets the reference copies to insert
 * an 802.1Q header (OptAddVLANHeader, header.go:147-155) are built in the
 * caller's side buffer. wait != 0 (socket readers): poll like
 * pollForFirstPacket, with the option's poll timeout.
 *
 * Release: the reference hands a header back to the kernel (status = 0) when
 * it moves to the next one. With deferred release on (gpk_tpacket_defer), a
 * finished header stays the user's until gpk_tpacket_release: the pump keeps
 * a block until its bytes are on the device. A deferred header the walk
 * comes round to again is treated as not yet handed over (GPK_TP_WAIT). */
int gpk_tpacket_index(gpk_tpacket* t, int wait, uint64_t* offsets, uint32_t* caplens, gpk_tp_info* ci, uint64_t max,
                      uint64_t* n, uint8_t* side, uint64_t side_cap, uint64_t* side_used);
int gpk_tpacket_defer(gpk_tpacket* t, int on);
/* Host threads for the parallel pre-walk of V3 blocks in large index calls
 * (default 16; 1 = the plain sequential walk). Results do not depend on it. */
int gpk_tpacket_set_threads(gpk_tpacket* t, int threads);
/* Header releases are numbered in walk order; *seq = the count so far. */
int gpk_tpacket_release_seq(const gpk_tpacket* t, uint64_t* seq);
/* Hand back every deferred header with release number < seq. */
int gpk_tpacket_release(gpk_tpacket* t, uint64_t seq);
/* The headers first read since the last call: ring positions [first, first+count)
 * (block or frame index, modulo the ring's header count). */
int gpk_tpacket_take_new_headers(gpk_tpacket* t, uint64_t* first, uint64_t* count);
/* Bytes per header (block size for V3, frame size for V1/V2) and header count. */
int gpk_tpacket_geometry(const gpk_tpacket* t, uint64_t* header_bytes, uint64_t* headers);

/* The error that ended the last GPK_TP_ERROR: Go text ("packet poll timeout
 * expired", "packet poll failed", an errno text, or a runtime panic with
 * *is_panic set); returns its length. */
int gpk_tpacket_error(const gpk_tpacket* t, char* buf, size_t cap, int* is_panic);

/* Stats(): packets returned, polls made. */
int gpk_tpacket_stats(const gpk_tpacket* t, int64_t* packets, int64_t* polls);
/* SocketStats(): accumulated PACKET_STATISTICS (v3 adds freeze_q_cnt). */
int gpk_tpacket_socket_stats(gpk_tpacket* t, uint32_t* packets, uint32_t* drops, uint32_t* freeze_q);
/* SetBPF with classic BPF instructions {code u16, jt u8, jf u8, k u32}; n = 0 detaches. */
int gpk_tpacket_set_bpf(gpk_tpacket* t, const void* insns, uint32_t n);
int gpk_tpacket_set_fanout(gpk_tpacket* t, int type, uint16_t id);
/* SetEBPF: attach the eBPF program prog_fd (SO_ATTACH_BPF). SetPromiscuous:
 * PACKET_MR_PROMISC membership on the bound interface (on != 0 adds, 0 drops).
 * WritePacketData: write the frame to the socket (transmit). InitSocketStats:
 * read and clear the kernel's counters and the accumulated ones. Socket
 * readers only (GPK_EINVAL on an attached ring or when the kernel refuses). */
int gpk_tpacket_set_ebpf(gpk_tpacket* t, int32_t prog_fd);
int gpk_tpacket_set_promiscuous(gpk_tpacket* t, int on);
int gpk_tpacket_write(gpk_tpacket* t, const void* pkt, uint64_t n);
int gpk_tpacket_init_socket_stats(gpk_tpacket* t);

/* ---- the capture loop through the GPU ------------------------------------ */
/* Per batch, before its gpk_tp_pump_cb: the layer fields of its n packets
 * (gpk_fields, include/gpk.h), valid during the call. */
typedef void (*gpk_tp_pump_fields_cb)(void* user, uint64_t first_packet, uint64_t n, const gpk_fields* fields);
/* Per batch, first of its callbacks: the batch's packets as
 * ZeroCopyReadPacketData returns their data, packet i = data[i][0, caplens[i])
 * (a frame in the ring, or the copy with the inserted VLAN header), valid
 * during the call. With it set, ring headers are handed back to the kernel
 * after their batch was delivered, not as soon as their bytes reached the
 * device. */
typedef void (*gpk_tp_pump_packets_cb)(void* user, uint64_t first_packet, uint64_t n, const uint8_t* const* data,
                                       const uint32_t* caplens);

typedef struct gpk_tp_pump_opts {
  uint64_t batch_pkts;  /* packets per device launch (default 1 Mi)              */
  uint64_t max_packets; /* stop after this many (0 = until the ring runs dry)     */
  int wait;             /* socket readers: poll when the ring is dry             */
  int inflight;         /* batches in flight (default 4)                          */
  gpk_tp_pump_fields_cb fields_cb; /* non-null: every launch is the fused decode +
                                      layer fields, delivered through it     */
  gpk_tp_pump_packets_cb packets_cb; /* non-null: the packets' bytes too        */
} gpk_tp_pump_opts;

typedef struct gpk_tp_pump_stats {
  uint64_t packets, packet_bytes, batches, ring_bytes_copied, waits;
  double wall_s;   /* first index .. last result delivered            */
  double index_s;  /* ring walk (gpk_tpacket_index)                   */
  double gpu_s;    /* HtoD + decode + DtoH, summed over batches        */
  double kernel_s; /* decode kernels alone                             */
  int status;      /* 0, or the GPK_TP_ERROR that ended the loop        */
  char error[160];
  char kernel[96]; /* the decode kernel specialisation of the last launch */
} gpk_tp_pump_stats;

typedef void (*gpk_tp_pump_cb)(void* user, uint64_t first_packet, uint64_t n, const gpk_record* records,
                               const uint32_t* err_args, const uint64_t* flows, const gpk_tp_info* ci,
                               const uint32_t* caplens);

/* Drain the ring through the decoder: the device keeps a mirror of the ring;
 * per batch, the headers first read in it are copied to their place in the
 * mirror straight from the ring (registered with HIP where it can be), the
 * side buffer follows, the decode kernel runs on the batch's index, results
 * come back in packet order through cb. Headers are deferred and released
 * once their HtoD has completed. gpk_stop(ctx) (gpk.h) ends the pump early:
 * no further callback, GPK_STOPPED, stats.packets = the packets delivered;
 * a pump waiting on a dry ring sees it once its wait ends (a frame, or the
 * socket's poll timeout). */
int gpk_tpacket_pump(gpk_ctx* ctx, const gpk_parser* p, gpk_tpacket* t, const gpk_tp_pump_opts* opts,
                     gpk_tp_pump_cb cb, void* user, gpk_tp_pump_stats* stats);

#ifdef __cplusplus
}
#endif
#endif /* GPK_AFPACKET_H */

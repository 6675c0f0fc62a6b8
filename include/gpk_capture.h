/*
 * gpk_capture.h — capture-file ingest for the batch decoder.
 *
 * The path of BASELINE config C5: a pcap / pcapng file is read into pinned
 * staging buffers, indexed IN PLACE (a packet's bytes stay where the file put
 * them: the staging buffer is the packed batch, offsets point into it), copied
 * to HBM and decoded. This header replaces, for a Go caller binding it through
 * cgo:
 *
 *   gpk_capreader_create(GPK_CAP_PCAPNG)  pcapgo.NewNgReader(r, NgReaderOptions)
 *                                         pcapgo/ngread.go:64-107; options :23-37
 *   gpk_capreader_create(GPK_CAP_PCAP)    pcapgo.NewReader(r)            pcapgo/read.go:65-119
 *   gpk_capreader_index                   a loop of ReadPacketData calls
 *                                         pcapgo/ngread.go:636-664 (ReadPacketDataWithOptions,
 *                                         reached through ReadPacketData :629-632 and the
 *                                         ZeroCopy variants :672-717), pcapgo/read.go:122-177
 *   gpk_capreader_packet_options          the NgPacketOptions ReadPacketDataWithOptions returns
 *                                         (readPacketOptions ngread.go:582-625)
 *   gpk_capreader_link_type               NgReader.LinkType() ngread.go:720 / Reader.LinkType() read.go:180
 *   gpk_capreader_section_* / _interface* NgReader.SectionInfo() :725, Interface(i) :730,
 *                                         NInterfaces() :738, SectionEndCallback (:32-34)
 *   gpk_capreader_nnames / _name          NgReader.NNames() :759 / Name(i) :751
 *   gpk_capreader_stat_event              NgReaderOptions.StatisticsCallback (:35-36)
 *   gpk_capreader_skip_section            NgReader.SkipSection() :330-335
 *   gpk_capreader_set_snaplen             Reader.SetSnaplen() read.go:216-218
 *   gpk_replay_file                       the C5 loop: NgReader/Reader + DecodingLayerParser
 *                                         over a whole file, pipelined through HBM
 *
 * Semantics are the reference's byte for byte, including its accounting
 * quirks: the indexer is a restatement of pcapgo's
 * bufio-stream reader, fed in chunks. Gzip-compressed files are inflated by
 * the file layer (gpk_replay_file) before indexing, as pcapgo does
 * transparently (read.go:80-86, ngread.go:75-91).
 */
#ifndef GPK_CAPTURE_H
#define GPK_CAPTURE_H

#include <stddef.h>
#include <stdint.h>

#include "gpk.h"

#ifdef __cplusplus
extern "C" {
#endif

#define GPK_CAP_PCAP 1
#define GPK_CAP_PCAPNG 2

/* NgReaderOptions (ngread.go:23-37) */
#define GPK_NG_WANT_MIXED_LINKTYPE 0x1u
#define GPK_NG_ERROR_ON_MISMATCHING_LINKTYPE 0x2u
#define GPK_NG_SKIP_UNKNOWN_VERSION 0x4u

/* gopacket.CaptureInfo (packet.go) of one packet. Timestamp = time.Unix(ts_sec,
 * ts_nsec).UTC(); the zero time.Time (simple packet blocks) is ts_sec =
 * -62135596800, ts_nsec = 0, which is what Time{}.Unix() returns. */
typedef struct gpk_capture_info {
  int64_t ts_sec;
  uint32_t ts_nsec;
  uint32_t length;    /* Length (original packet length)                      */
  int32_t iface;      /* InterfaceIndex                                       */
  int32_t link_type;  /* AncillaryData[0] with WantMixedLinkType, else -1     */
} gpk_capture_info;

typedef struct gpk_capreader gpk_capreader;

int gpk_capreader_create(gpk_capreader** out, int format, uint32_t ng_flags);
int gpk_capreader_destroy(gpk_capreader* r);

/* gpk_capreader_index return values (>= 0) */
#define GPK_CAP_MORE 0 /* every whole record of buf was read: feed buf[consumed..] + more bytes */
#define GPK_CAP_FULL 1 /* max_pkts packets written: call again with buf[consumed..]       */
#define GPK_CAP_END 2  /* ReadPacketData returned an error (io.EOF included): see
                          gpk_capreader_error. Calling again continues like another
                          ReadPacketData call after that error would.                 */

/* Index the packets of buf[0, len) — the capture stream from the reader's
 * current position on; eof != 0 when no byte follows buf[len-1]. Writes up to
 * max_pkts packets: data of packet i is buf[offsets[i], offsets[i]+caplens[i]),
 * its CaptureInfo is ci[i] (ci may be NULL). *consumed = the stream bytes the
 * reader is done with; every written packet lies in buf[0, *consumed). The
 * next call must pass the stream from buf + *consumed on. A record longer
 * than the bytes available returns GPK_CAP_MORE with *consumed possibly 0:
 * pass a longer buffer. Packets the reference returns together with an error
 * (a failed ReadPacketData) are not written. */
int gpk_capreader_index(gpk_capreader* r, const uint8_t* buf, uint64_t len, int eof, uint64_t* offsets,
                        uint32_t* caplens, gpk_capture_info* ci, uint64_t max_pkts, uint64_t* n_pkts,
                        uint64_t* consumed);

/* The same result as gpk_capreader_index called until it stops (unbounded
 * output), over buf[0, len), with the record walk split over `threads`
 * threads: segments after the first are walked speculatively from a plausible
 * chain of plain Enhanced Packet Blocks, and a segment's packets are kept
 * only where the exact walk lands on its start with unchanged reader state,
 * so the output is always the sequential one. Returns GPK_CAP_MORE or
 * GPK_CAP_END (never FULL); the arrays are malloc'd by the library (release
 * with gpk_capindex_free); offsets are relative to buf. */
typedef struct gpk_capindex {
  uint64_t n;
  uint64_t* offsets;
  uint32_t* caplens;
  gpk_capture_info* ci;
} gpk_capindex;
int gpk_capreader_index_all(gpk_capreader* r, const uint8_t* buf, uint64_t len, int eof, int threads,
                            gpk_capindex* out, uint64_t* consumed);
int gpk_capindex_free(gpk_capindex* x);

/* The error that ended the last GPK_CAP_END: the Go error text (io.EOF is
 * "EOF"); *is_eof = it is io.EOF; *is_panic = the reference panics there
 * (a runtime error its code does not recover). Returns the text length. */
int gpk_capreader_error(const gpk_capreader* r, char* buf, size_t cap, int* is_eof, int* is_panic);

/* Reader.LinkType() / NgReader.LinkType() (0 with WantMixedLinkType). */
int gpk_capreader_link_type(const gpk_capreader* r);
/* pcap header fields: snaplen, version, nanosecond resolution (read.go:94-117). */
int gpk_capreader_pcap_header(const gpk_capreader* r, uint32_t* snaplen, uint16_t* major, uint16_t* minor,
                              int* nanosecond);

/* pcapng sections: sections 0 .. nsections-1 ended (the SectionEndCallback
 * calls, ngread.go:239-245); section == nsections is the current one. */
int gpk_capreader_nsections(const gpk_capreader* r);
#define GPK_SECTION_COMMENT 0
#define GPK_SECTION_HARDWARE 1
#define GPK_SECTION_OS 2
#define GPK_SECTION_APPLICATION 3
/* NgSectionInfo string field; returns its length (bytes may include NUL). */
int gpk_capreader_section_info(const gpk_capreader* r, int section, int field, char* buf, size_t cap);
int gpk_capreader_ninterfaces(const gpk_capreader* r, int section);

/* NgInterface (pcapgo/pcapng.go) numeric fields and statistics. */
typedef struct gpk_ng_interface {
  uint16_t link_type;
  uint8_t ts_resolution;
  uint8_t has_statistics;
  uint32_t snap_length;
  uint64_t ts_offset;
  int64_t last_update_sec, start_time_sec, end_time_sec;
  uint32_t last_update_nsec, start_time_nsec, end_time_nsec, _pad;
  uint64_t packets_received, packets_dropped;
} gpk_ng_interface;
int gpk_capreader_interface(const gpk_capreader* r, int section, int index, gpk_ng_interface* out);
#define GPK_IFACE_NAME 0
#define GPK_IFACE_COMMENT 1
#define GPK_IFACE_DESCRIPTION 2
#define GPK_IFACE_FILTER 3
#define GPK_IFACE_OS 4
#define GPK_IFACE_STATS_COMMENT 5
int gpk_capreader_interface_str(const gpk_capreader* r, int section, int index, int field, char* buf, size_t cap);

/* The rest of NgReader's / Reader's interface. What the reader reports here
 * is the state after the packets it has returned through gpk_capreader_index
 * (and _index_all; a gpk_replay_file reader does not report it). */
/* SectionEndCallback's timing: section s (< nsections) ended during the call
 * that returned packet *at (or ended with an error there): *at = the packets
 * returned before it; *seq = its place among all SectionEndCallback and
 * StatisticsCallback calls (0, 1, ...). */
int gpk_capreader_section_end_at(const gpk_capreader* r, int section, uint64_t* at, uint64_t* seq);
/* StatisticsCallback(ifaceID, NgInterfaceStatistics) (ngread.go:35-36, made at
 * :485-487 after each interface statistics block): every call so far, in
 * order. Event k: *iface, the statistics in the statistics fields of *stats
 * (has_statistics 1, the rest 0), its comment into buf (returns the comment's
 * length), *at = the packets returned before it and *seq its place among all
 * callbacks (as in gpk_capreader_section_end_at). Any pointer may be NULL. */
int gpk_capreader_nstat_events(const gpk_capreader* r);
int gpk_capreader_stat_event(const gpk_capreader* r, int k, uint64_t* at, uint64_t* seq, int* iface,
                             gpk_ng_interface* stats, char* buf, size_t cap);
/* NgReader.NNames() / Name(i) (ngread.go:751-761): the name resolution records
 * of the current section (readNameResolutionBlock, ngread_nrb.go:64-130).
 * *kind = the record type: 1 IPv4 / 2 IPv6 (NgIPAddress: *addr_len 4 / 16),
 * 3 EUI-48 / 4 EUI-64 (NgEUIAddress: *addr_len 24, the reader's whole 24-byte
 * scratch buffer, which newHWAddress clones, ngread_nrb.go:56-61); addr has
 * room for 24 bytes. names: the record's Names, each followed by a NUL, as
 * far as cap holds whole names; returns the bytes all of them take. */
int gpk_capreader_nnames(const gpk_capreader* r);
int gpk_capreader_name(const gpk_capreader* r, int i, int* kind, uint8_t* addr, int* addr_len, int* nnames,
                       char* names, size_t cap);
/* NgReader.SkipSection (ngread.go:330-335): the next gpk_capreader_index call
 * first skips the rest of the current section and reads the next section
 * header; an error there ends that call with GPK_CAP_END and no packet (the
 * error SkipSection returns). */
int gpk_capreader_skip_section(gpk_capreader* r);
/* Reader.SetSnaplen (read.go:216-218), for the packets read from now on. */
int gpk_capreader_set_snaplen(gpk_capreader* r, uint32_t snaplen);
/* ReadPacketDataWithOptions's NgPacketOptions (ngread.go:636-664,
 * readPacketOptions :582-625). After gpk_capreader_keep_options(r, 1) each
 * gpk_capreader_index call keeps the options of the packets it returned:
 * for its packet i, *tlv = *bytes bytes of records {uint16_t code; uint16_t 0;
 * uint32_t len; len value bytes, zero-padded to a multiple of 4}, one per
 * option readPacketOptions read, in order, each with the value the reader
 * held for it (a zero-length option keeps the previous option's value,
 * ngread.go:214-232); none for simple and obsolete packet blocks. Valid until
 * the next index call (gpk_capreader_index_all's own calls included). */
int gpk_capreader_keep_options(gpk_capreader* r, int on);
int gpk_capreader_packet_options(const gpk_capreader* r, uint64_t i, const uint8_t** tlv, uint64_t* bytes);

/* ---- whole-file replay through the GPU (BASELINE config C5) -------------- */
/* The layer fields of one device launch's packets (gpk_replay_opts.fields_cb):
 * gpk_fields as gpk_decode_batch_fields writes them, in packet order, host
 * memory valid during the call only; called on the calling thread right
 * before gpk_replay_cb for the same packets. */
typedef void (*gpk_replay_fields_cb)(void* user, uint64_t first_packet, uint64_t n, const gpk_fields* fields);
/* The packets of one device launch, as ReadPacketData returned their data:
 * packet i is base[offsets[i], offsets[i] + caplens[i]), inside base[0, bytes),
 * in the pinned staging buffer the file was read into (no copy), valid during
 * the call only; called on the calling thread before the fields and results
 * callbacks for the same packets. */
typedef void (*gpk_replay_packets_cb)(void* user, uint64_t first_packet, uint64_t n, const uint8_t* base,
                                      uint64_t bytes, const uint64_t* offsets, const uint32_t* caplens);

typedef struct gpk_replay_opts {
  int format;            /* GPK_CAP_PCAP / GPK_CAP_PCAPNG, 0 = from the magic */
  uint32_t ng_flags;     /* GPK_NG_* */
  uint64_t slot_bytes;   /* file bytes per pinned staging slot (default 256 MiB); a record (pcap
                            record, pcapng block) may be as long as the slot's carry region:
                            slot_bytes up to 1 MiB, else max(1 MiB, slot_bytes / 16); a longer
                            one ends the call with GPK_EUNSUPP */
  int slots;             /* staging slots in flight (default 4)                 */
  uint64_t batch_pkts;   /* packets per device launch (default 1 Mi)            */
  int read_threads;      /* pread threads per slot (default 8)                  */
  gpk_replay_fields_cb fields_cb; /* non-NULL: each launch is the fused decode + layer fields
                            (gpk_decode_batch_fields) and the fields come back too, 128 B per
                            packet more DtoH; NULL: the decode alone */
  gpk_replay_packets_cb packets_cb; /* non-NULL: each launch's packet bytes too; a staging
                            slot is then refilled only after its packets were delivered */
} gpk_replay_opts;

typedef struct gpk_replay_stats {
  uint64_t packets, packet_bytes, file_bytes, stream_bytes, batches, slots;
  double wall_s;         /* open .. last result delivered                        */
  double read_s;         /* file -> pinned staging (read threads, busy time)     */
  double index_s;        /* record walk: device walk + host reader, and the waits for them */
  double gpu_s;          /* HtoD + decode + DtoH, summed over batches            */
  double kernel_s;       /* decode kernels alone                                 */
  double deliver_s;      /* result callback                                      */
  int reader_status;     /* the GPK_CAP_END error: 0 = io.EOF (clean end)        */
  char error[160];
  char kernel[96];       /* the decode kernel specialisation of the last launch */
  uint64_t device_walk_packets; /* packets the device record walk indexed (the rest: the host reader) */
  double alloc_wait_s;   /* first call with these sizes: time the reads and launches waited for their
                            staging buffers, which are allocated in the background (0 when kept) */
} gpk_replay_stats;

/* Results of one device launch, in packet order, delivered on the calling
 * thread: host arrays valid during the call only. */
typedef void (*gpk_replay_cb)(void* user, uint64_t first_packet, uint64_t n, const gpk_record* records,
                              const uint32_t* err_args, const uint64_t* flows, const gpk_capture_info* ci,
                              const uint32_t* caplens);

/* Replay a whole capture file through HBM. For pcapng the record walk runs
 * on the device once the section header and interfaces are read (plain
 * Enhanced Packet Blocks; the host reader takes every other block, same
 * results either way; GPK_REPLAY_HOST_WALK=1 in the environment keeps it on
 * the host). The pinned staging slots and device buffers stay with ctx for
 * the next call with the same sizes (gpk_ctx_destroy frees them).
 * The reader threads, and the calling thread for the duration of the call,
 * run on the CPUs of the current device's NUMA node that the caller may use
 * (its affinity is restored on return); environment GPK_REPLAY_NUMA=0 turns
 * this off, =1 pins the reader threads only.
 * gpk_stop(ctx) (gpk.h), from a callback or another thread, ends the call
 * early: no further callback, GPK_STOPPED, stats.packets = the packets
 * delivered. */
int gpk_replay_file(gpk_ctx* ctx, const gpk_parser* p, const char* path, const gpk_replay_opts* opts,
                    gpk_replay_cb cb, void* user, gpk_replay_stats* stats);

/* One caller's share of a pcapng file replayed by N callers (one per GPU, no
 * data exchange): the same loop as gpk_replay_file (pcapgo.NgReader +
 * DecodeLayers, ngread.go:494-718, parser.go:303-317) over the blocks that
 * START in [sync(begin), sync(end)). sync(X) is the first offset >= X, a
 * multiple of 4, where four plain Enhanced Packet Blocks chain inside the next
 * 4 MiB under the reader state after the file's leading non-packet blocks
 * (section header, interfaces), which every caller reads first: it depends on
 * X and the file only, so caller k's sync(end) is caller k+1's sync(begin).
 * begin 0: from the file's start; end 0: to its end. Callers number their
 * packets from 0. Cut the file at size*k/N.
 * The N results, concatenated in range order, are exactly gpk_replay_file's
 * when every caller but the last reports clean (its reader met io.EOF exactly
 * at sync_end, so sync_end is a real block boundary) and !state_changed (no
 * block inside its range changed reader state: a section header, an interface,
 * interface statistics, or an option value NgReader keeps for the next option,
 * as EPB options do). Otherwise let f be the
 * first caller that does not: its result and every later one's are replaced
 * by a replay of [f's sync_begin, end of file) (begin = sync_begin, end = 0),
 * which is exact. Uncompressed pcapng only (GPK_EUNSUPP otherwise). */
typedef struct gpk_replay_range {
  uint64_t begin, end;    /* in: this caller's cut of the file's bytes                       */
  uint64_t header_end;    /* out: the file's first packet block (the header every caller reads) */
  uint64_t sync_begin;    /* out: the first block this caller replayed (0: the file's start)  */
  uint64_t sync_end;      /* out: where its blocks had to end                                 */
  int clean;              /* out: the reader met io.EOF exactly at sync_end                   */
  int state_changed;      /* out: a block in the range changed reader state (see above)       */
} gpk_replay_range;
int gpk_replay_file_range(gpk_ctx* ctx, const gpk_parser* p, const char* path, gpk_replay_range* range,
                          const gpk_replay_opts* opts, gpk_replay_cb cb, void* user, gpk_replay_stats* stats);

#ifdef __cplusplus
}
#endif
#endif /* GPK_CAPTURE_H */

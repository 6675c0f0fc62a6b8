/*
 * gpk_bpf.h — classic BPF filters evaluated on the device over a packet batch
 * (SURVEY.md §8(f)4).
 *
 * Replaces, for a batch, what the reference does per packet:
 *   gpk_bpf_create    pcap.Handle.NewBPFInstructionFilter / bpfInstructionFilter
 *                     (pcap/pcap.go:506-517,565-576): the same two errors,
 *                     "bpfInstructions must not be empty" and "bpfInstructions
 *                     must not be larger than 4096" (MaxBpfInstructions, :36)
 *   gpk_bpf_run       BPF.Matches (pcap.go:599-601 -> pcap_unix.go:358-368
 *                     pcapOfflineFilter -> libpcap pcap_offline_filter /
 *                     bpf_filter over wirelen = ci.Length, buflen = len(data)):
 *                     the filter's return value per packet, Matches = != 0
 *   gpk_bpf_select    the batch a consumer behind the filter sees: the matching
 *                     packets' index entries, compacted in batch order
 * Compiling filter expressions (pcap_compile, NewBPF) needs libpcap, which is
 * absent: programs come as instructions (tcpdump -dd), as
 * NewBPFInstructionFilter takes them. Semantics: DESIGN.md §13.
 */
#ifndef GPK_BPF_H
#define GPK_BPF_H

#include <stddef.h>
#include <stdint.h>

#include "gpk.h"

#ifdef __cplusplus
extern "C" {
#endif

/* pcap.BPFInstruction / struct bpf_insn */
typedef struct gpk_bpf_insn {
  uint16_t code;
  uint8_t jt;
  uint8_t jf;
  uint32_t k;
} gpk_bpf_insn;

#define GPK_BPF_MAX_INSNS 4096 /* pcap.MaxBpfInstructions */

typedef struct gpk_bpf gpk_bpf;

/* Upload a program to the current device. GPK_EINVAL with the reference's
 * error text in err for an empty or oversized program. */
int gpk_bpf_create(gpk_bpf** out, const gpk_bpf_insn* insns, uint32_t n, char* err, size_t cap);
int gpk_bpf_destroy(gpk_bpf* f);

/* ret[i] = the filter's return value for packet i (device arrays; wirelens
 * NULL = each packet's caplen, i.e. ci.Length == CaptureLength). Async on stream. */
int gpk_bpf_run(gpk_bpf* f, const gpk_batch* batch, const uint32_t* wirelens, uint32_t* ret, void* stream);

/* The matching packets, in batch order: out_offsets/out_caplens/out_index
 * [n] (device), *out_count (device u32). Async on stream. The filter keeps
 * scratch for this call: use one filter from one stream at a time (one
 * filter per goroutine/thread, as a pcap handle is). */
int gpk_bpf_select(gpk_bpf* f, const gpk_batch* batch, const uint32_t* wirelens, uint64_t* out_offsets,
                   uint32_t* out_caplens, uint32_t* out_index, uint32_t* out_count, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GPK_BPF_H */

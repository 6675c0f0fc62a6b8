// gpk_walk.h — the pcapng record walk on the device (internal to libgpk:
// gpk_replay.cpp drives it, gpk_capture.cpp supplies the reader state,
// gpk_walk.hip runs it).
//
// A staging slot already sits in HBM before it is decoded, so its record
// walk runs there too: one thread per segment finds a plausible chain of
// plain Enhanced Packet Blocks (the same rule as the host's speculative walk,
// gpk_capture.cpp plain_epb / find_sync) and counts the chain's packets up to
// the segment's end; the host accepts segment k only when the chain of
// segments 0..k-1 lands exactly on its start, so the accepted packets are what
// NgReader.ReadPacketData returns (ngread.go:494-718: a plain EPB changes no
// reader state). A second pass writes each accepted packet's offset, caplen
// and CaptureInfo at its index. The host's exact reader takes over at the
// first block the chain does not cover.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gpk.h"
#include "../../include/gpk_capture.h"

namespace gpk {

constexpr int kWalkMaxIf = 32;

// One interface of the current section, as the walk needs it.
struct WalkIface {
  uint64_t second_mask, scale_up, scale_down, tsoff;  // convertTime (ngread.go:440-443)
  int32_t link_type;
  uint32_t plain;  // its EPBs may be plain: known link type rule (WantMixedLinkType or the reader's)
};

// The reader state a plain EPB depends on (constant over the blocks it walks).
struct WalkState {
  uint32_t be, mixed, nif, _pad;
  WalkIface ifc[kWalkMaxIf];
};

// Per-segment results of the first pass (device arrays of nseg entries).
struct WalkSegs {
  uint64_t* sync;   // first block of the segment's chain (~0: none found)
  uint64_t* end;    // where the chain stopped (>= the segment's end unless a block was not plain)
  uint32_t* count;  // packets of the chain
  uint64_t* base;   // second pass: index of the segment's first packet (~0: not accepted)
};

}  // namespace gpk

// gpk_capture.cpp: the reader's state for the device walk; false when the
// walk cannot run there (not pcapng, not opened yet, too many interfaces).
bool gpk_capreader_walk_state(const gpk_capreader* r, gpk::WalkState* out);
// gpk_capture.cpp: the first p in [from, to), p = 0 (mod 4), where four plain
// EPBs chain under the reader's state inside b[p, min(end, p + span)) (~0:
// none, or the reader is not an open pcapng reader); and the version of the
// state that rule depends on (sections ended, interfaces; 0 when not open),
// which changes when a block other than a packet changes it.
uint64_t gpk_capreader_sync(const gpk_capreader* r, const uint8_t* b, uint64_t from, uint64_t to, uint64_t end,
                            uint64_t span);
uint64_t gpk_capreader_state_version(const gpk_capreader* r);
// gpk_capture.cpp: how many changes of the reader's state (section, interfaces,
// the reused option buffer) the blocks read so far made; the same count after
// the same bytes however they were chunked.
uint64_t gpk_capreader_mutations(const gpk_capreader* r);

// gpk_walk.hip: pass 1 over buf[p0, len) (buf 16-byte aligned, the reader at
// p0, blocks at p0 + 4k) in segments of `seg` bytes from buf, pass 2 writing
// the accepted segments' packets (offsets relative to buf).
hipError_t gpk_walk_segments(const uint8_t* buf, uint64_t p0, uint64_t len, uint64_t seg, uint32_t nseg,
                             const gpk::WalkState& ws, const gpk::WalkSegs& out, hipStream_t stream);
hipError_t gpk_walk_emit(const uint8_t* buf, uint64_t len, uint32_t nseg, const gpk::WalkState& ws,
                         const gpk::WalkSegs& segs, uint64_t* offsets, uint32_t* caplens, gpk_capture_info* ci,
                         hipStream_t stream);

// gpk_host.cpp: the context's slot for gpk_replay_file's staging buffers,
// which a call takes over when their sizes match and leaves for the next call
// (gpk_ctx_destroy frees them). put() frees a buffer set already there.
void* gpk_ctx_replay_take(gpk_ctx* c);
void gpk_ctx_replay_put(gpk_ctx* c, void* p, void (*deleter)(void*));

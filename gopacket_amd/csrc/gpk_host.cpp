// gpk_host.cpp — C ABI (include/gpk.h) around the gfx950 decode kernels.
//
// Host-side pieces of the DecodingLayerParser surface:
//   * gpk_parser: the DecodingLayerContainer (parser.go:147-169, Map semantics:
//     later Put overrides) + DecodingLayerParserOptions (parser.go:337-351) +
//     the next-layer tables (layers/enums.go:294-353, layers/ports.go:54-183).
//   * gpk_ctx: one device, device copies of parser tables (one per parser
//     version in use, see TabSlot) and staging buffers.
//   * error text: the exact strings DecodeLayers returns (see gpk.h enum).
// There is no CPU decode path here: every packet is decoded by the device.
#include <hip/hip_runtime.h>

#include <sys/mman.h>

#include <cstdio>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <mutex>
#include <unordered_map>
#include <system_error>
#include <thread>
#include <vector>
#include <new>
#include <string>

#include "../../include/gpk.h"
#include "gpk_device.h"
#include "gpk_registry_gen.h"
#include "gpk_pinned.h"
#include "gpk_devguard.h"

extern "C" hipError_t gpk_launch_decode(const gpk::KParams* P, int with_l4, int with_layout, hipStream_t stream);
extern "C" int gpk_launch_describe(const gpk::KParams* P, int with_l4, int with_layout, char* buf, size_t cap);
extern "C" hipError_t gpk_launch_occupancy(const gpk::KParams* P, int with_l4, int with_layout, int* blocks);
extern "C" hipError_t gpk_launch_decode_fields(const gpk::KParams* P, hipStream_t stream, int* occ);
extern "C" void gpk_walk_preload(void);
extern "C" int gpk_launch_describe_fields(const gpk::KParams* P, char* buf, size_t cap);
extern "C" hipError_t gpk_launch_list(const gpk::KParams* P, uint64_t index, int64_t* out, uint32_t cap,
                                      uint32_t* out_n, hipStream_t stream);

namespace {

thread_local char g_hip_err[256] = "";

int hip_fail(hipError_t e, const char* what) {
  snprintf(g_hip_err, sizeof(g_hip_err), "%s: %s", what, hipGetErrorString(e));
  return GPK_EHIP;
}
#define HIPCHK(x)                                     \
  do {                                                \
    hipError_t _e = (x);                              \
    if (_e != hipSuccess) return hip_fail(_e, #x);    \
  } while (0)

}  // namespace

struct gpk_parser {
  int64_t first;
  int ignore_panic = 0;
  int ignore_unsupported = 0;
  uint32_t outputs = GPK_OUT_ALL;
  uint64_t version = 0;  // process-unique id of the current table contents (see bump())
  gpk::DevTables tab;
};

// Device copies of parser tables. A context keeps a few, keyed by the
// parser's table version, so parsers used alternately (on one stream or on
// several) each read their own copy: gopacket gives every parser its own
// state (doc.go:211-228), and a launch on one stream must never see a table
// rewritten for a launch on another. A copy is rewritten only for a new
// version, and everything is ordered on the device, never by blocking the
// host: the upload is enqueued on the launching stream behind a wait for
// every earlier launch that read the slot (done), from the slot's own pinned
// staging buffer (the parser may change as soon as the call returns), and a
// launch on another stream waits for the upload (ready).
struct TabSlot {
  gpk::DevTables* dtab = nullptr;
  uint32_t* dctab = nullptr;  // compact blob (gpk::kCtDwords), valid when compact
  bool compact = false;
  bool global_mode = false;   // built under GPK_TABLES_GLOBAL
  gpk::CompactGeom cg{};
  uint64_t version = 0;       // parser table version held, 0 = empty
  uint64_t last_use = 0;      // LRU tick
  uint8_t* staging = nullptr; // pinned: DevTables, then the compact blob; the last upload's source
  // Both events are recorded on an aggregation stream of the context (one per
  // caller stream, Agg), which waits for the caller's stream first, so they
  // never refer to a caller's stream that may be destroyed meanwhile.
  hipEvent_t ready = nullptr;  // the slot's last upload has landed
  hipEvent_t done = nullptr;   // every launch so far that read the slot has completed (cumulative:
                               // each record first waits for the previous one)
  bool uploaded = false, read = false;
  bool ready_seen = false;     // ready has been observed complete (no wait needed)
};
constexpr int kTabSlots = 8;

struct gpk_ctx {
  int device = 0;
  bool force_global = false;  // gpk_ctx_set_table_mode(GPK_TABLES_GLOBAL)
  TabSlot slots[kTabSlots];
  uint64_t tick = 0;
  // staging for gpk_decode_batch_host / gpk_decoded_list
  void* dbuf = nullptr;
  size_t dbuf_bytes = 0;
  hipStream_t stream = nullptr;
  // Aggregation streams, one per caller stream (the most recently used
  // kAggStreams callers): each carries only waits and event records, the
  // completion marks of launches and uploads on its caller's stream
  // (note_launch, upload), so a mark waits for its own caller's work only and
  // no event outlives the stream it was recorded on. ev: a reusable event
  // recorded on the caller's stream.
  struct Agg {
    hipStream_t agg = nullptr;
    hipEvent_t ev = nullptr;
    uint64_t last_use = 0;
  };
  std::unordered_map<hipStream_t, Agg> aggs;
  // retired aggregation streams whose marks may still be pending: destroyed
  // once their work has completed (agg_of polls them; never waits)
  std::vector<Agg> retired;
  std::mutex mu;
  // gpk_replay_file's staging buffers, kept for the next call (gpk_walk.h)
  void* replay_cache = nullptr;
  void (*replay_cache_free)(void*) = nullptr;
  std::atomic<uint64_t> stop_seq{0};  // gpk_stop calls so far
};

void* gpk_ctx_replay_take(gpk_ctx* c) {
  std::lock_guard<std::mutex> g(c->mu);
  void* p = c->replay_cache;
  c->replay_cache = nullptr;
  return p;
}

void gpk_ctx_replay_put(gpk_ctx* c, void* p, void (*deleter)(void*)) {
  void* old = nullptr;
  void (*old_free)(void*) = nullptr;
  {
    std::lock_guard<std::mutex> g(c->mu);
    old = c->replay_cache;
    old_free = c->replay_cache_free;
    c->replay_cache = p;
    c->replay_cache_free = deleter;
  }
  if (old && old_free) old_free(old);
}

// Every table change takes a new process-wide id, so a context never mistakes
// a new parser that reuses a freed parser's address for the one it uploaded.
static std::atomic<uint64_t> g_table_ids{1};
static void bump(gpk_parser* p) { p->version = g_table_ids.fetch_add(1); }

static void default_tables(gpk::DevTables& t) {
  memset(&t, 0, sizeof(t));
  for (int i = 0; i < GPK_N_ETHERTYPE_ROWS; i++) t.ethertype[GPK_ETHERTYPE_ROWS[i].value] = GPK_ETHERTYPE_ROWS[i].layer_type;
  for (int i = 0; i < GPK_N_IPPROTOCOL_ROWS; i++) t.ipprotocol[GPK_IPPROTOCOL_ROWS[i].value] = GPK_IPPROTOCOL_ROWS[i].layer_type;
  for (int p = 0; p < 65536; p++) t.tcp_port[p] = t.udp_port[p] = GPK_LT_PAYLOAD;
  for (int i = 0; i < GPK_N_TCP_PORT_SWITCH; i++) t.tcp_port[GPK_TCP_PORT_SWITCH[i].port] = GPK_TCP_PORT_SWITCH[i].layer_type;
  for (int i = 0; i < GPK_N_UDP_PORT_SWITCH; i++) t.udp_port[GPK_UDP_PORT_SWITCH[i].port] = GPK_UDP_PORT_SWITCH[i].layer_type;
  for (int i = 0; i < GPK_N_TCP_PORT_OVERRIDE; i++) t.tcp_port[GPK_TCP_PORT_OVERRIDE[i].port] = GPK_TCP_PORT_OVERRIDE[i].layer_type;
  for (int i = 0; i < GPK_N_UDP_PORT_OVERRIDE; i++) t.udp_port[GPK_UDP_PORT_OVERRIDE[i].port] = GPK_UDP_PORT_OVERRIDE[i].layer_type;
}

extern "C" {

int gpk_abi_version(void) { return GPK_ABI_VERSION; }

int gpk_ctx_device(const gpk_ctx* c) { return c ? c->device : -1; }

uint64_t gpk_ctx_stop_seq(const gpk_ctx* c) { return c ? c->stop_seq.load() : 0; }

int gpk_stop(gpk_ctx* c) {
  if (!c) return GPK_EINVAL;
  c->stop_seq.fetch_add(1);
  return GPK_OK;
}

const char* gpk_strerror(int status) {
  switch (status) {
    case GPK_OK: return "ok";
    case GPK_EINVAL: return "invalid argument";
    case GPK_ENOMEM: return "out of memory";
    case GPK_EHIP: return "HIP runtime error";
    case GPK_ENODEV: return "no such device";
    case GPK_EUNSUPP: return "unsupported configuration";
    case GPK_STOPPED: return "stopped";
    default: return "unknown status";
  }
}

const char* gpk_last_hip_error(void) { return g_hip_err; }

// ---- parser ------------------------------------------------------------------
int gpk_parser_create(gpk_parser** out, int64_t first) {
  if (!out) return GPK_EINVAL;
  gpk_parser* p = new (std::nothrow) gpk_parser;
  if (!p) return GPK_ENOMEM;
  p->first = first;
  default_tables(p->tab);
  bump(p);
  *out = p;
  return GPK_OK;
}

int gpk_parser_destroy(gpk_parser* p) {
  delete p;
  return GPK_OK;
}

static void put(gpk_parser* p, int lt, int kind) {
  if (lt >= 0 && lt < GPK_MAX_LAYER_TYPE) p->tab.dispatch[lt] = (uint8_t)kind;
}

int gpk_parser_add_decoder(gpk_parser* p, int kind) {
  if (!p) return GPK_EINVAL;
  switch (kind) {  // CanDecode() of each DecodingLayer
    case GPK_DEC_ETHERNET: put(p, GPK_LT_ETHERNET, kind); break;
    case GPK_DEC_DOT1Q: put(p, GPK_LT_DOT1Q, kind); break;
    case GPK_DEC_IPV4: put(p, GPK_LT_IPV4, kind); break;
    case GPK_DEC_IPV6: put(p, GPK_LT_IPV6, kind); break;
    case GPK_DEC_IPV6_EXT:  // LayerClassIPv6Extension, layertypes.go:200-206
      put(p, GPK_LT_IPV6_HOPBYHOP, kind);
      put(p, GPK_LT_IPV6_ROUTING, kind);
      put(p, GPK_LT_IPV6_FRAGMENT, kind);
      put(p, GPK_LT_IPV6_DESTINATION, kind);
      break;
    case GPK_DEC_TCP: put(p, GPK_LT_TCP, kind); break;
    case GPK_DEC_UDP: put(p, GPK_LT_UDP, kind); break;
    case GPK_DEC_PAYLOAD: put(p, GPK_LT_PAYLOAD, kind); break;
    case GPK_DEC_FRAGMENT: put(p, GPK_LT_FRAGMENT, kind); break;
    default: return GPK_EUNSUPP;
  }
  bump(p);
  return GPK_OK;
}

int gpk_parser_set_options(gpk_parser* p, int ignore_panic, int ignore_unsupported) {
  if (!p) return GPK_EINVAL;
  p->ignore_panic = ignore_panic != 0;
  p->ignore_unsupported = ignore_unsupported != 0;
  return GPK_OK;
}

int gpk_parser_set_outputs(gpk_parser* p, uint32_t outputs) {
  if (!p || (outputs & ~GPK_OUT_ALL)) return GPK_EINVAL;
  p->outputs = outputs;
  return GPK_OK;
}

int gpk_parser_decoder_for(const gpk_parser* p, int64_t lt) {
  if (!p || lt < 0 || lt >= GPK_MAX_LAYER_TYPE) return GPK_DEC_NONE;
  return p->tab.dispatch[lt];
}

int gpk_parser_set_ethertype(gpk_parser* p, uint32_t v, int32_t lt) {
  if (!p || v > 0xffff) return GPK_EINVAL;
  p->tab.ethertype[v] = lt;
  bump(p);
  return GPK_OK;
}
int gpk_parser_set_ipprotocol(gpk_parser* p, uint32_t v, int32_t lt) {
  if (!p || v > 0xff) return GPK_EINVAL;
  p->tab.ipprotocol[v] = lt;
  bump(p);
  return GPK_OK;
}
int gpk_parser_set_tcp_port(gpk_parser* p, uint32_t v, int32_t lt) {
  if (!p || v > 0xffff) return GPK_EINVAL;
  p->tab.tcp_port[v] = lt;
  bump(p);
  return GPK_OK;
}
int gpk_parser_set_udp_port(gpk_parser* p, uint32_t v, int32_t lt) {
  if (!p || v > 0xffff) return GPK_EINVAL;
  p->tab.udp_port[v] = lt;
  bump(p);
  return GPK_OK;
}

// ---- context -----------------------------------------------------------------
static void free_slots(gpk_ctx* c) {
  for (TabSlot& t : c->slots) {
    if (t.done) (void)hipEventDestroy(t.done);
    if (t.ready) (void)hipEventDestroy(t.ready);
    t.done = t.ready = nullptr;
    if (t.dtab) (void)hipFree(t.dtab);
    if (t.dctab) (void)hipFree(t.dctab);
    if (t.staging) (void)hipHostFree(t.staging);
    t.dtab = nullptr;
    t.dctab = nullptr;
    t.staging = nullptr;
  }
  for (auto& kv : c->aggs) c->retired.push_back(kv.second);
  c->aggs.clear();
  for (auto& a : c->retired) {  // context teardown: the one place that waits
    (void)hipStreamSynchronize(a.agg);
    (void)hipStreamDestroy(a.agg);
    (void)hipEventDestroy(a.ev);
  }
  c->retired.clear();
}

// The first C++ exception a process throws initialises the unwinder's
// frame tables for every loaded object: ~80 ms on the GPU box with PyTorch's
// libraries loaded (350 ms in this container), paid by whichever call throws
// first. The capture reader throws one at every chunk end (a record cut by
// the chunk: NeedMore, gpk_capture.cpp), so the first replay of a process
// paid it inside its wall time (GPK_REPLAY_TRACE=3: its first 64 KiB host
// walk took 83 ms, 0.06 ms afterwards). A context takes it at creation.
__attribute__((noinline)) static void warm_unwinder() {
  try {
    throw std::bad_alloc();
  } catch (const std::bad_alloc&) {
  }
}

int gpk_ctx_create(gpk_ctx** out, int device) {
  if (!out) return GPK_EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return GPK_ENODEV;
  gpk::DeviceScope dscope(device);  // the context's stream and buffers on its device; the caller's back after
  HIPCHK(dscope.err);
  gpk_walk_preload();  // the replay's record-walk module (gpk_walk.hip), loaded with the context
  warm_unwinder();
  gpk_ctx* c = new (std::nothrow) gpk_ctx;
  if (!c) return GPK_ENOMEM;
  c->device = device;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return GPK_EHIP;
  }
  // The first host<->device copies of a process pay a one-time setup inside
  // the HIP runtime (~80 ms before the first replay's first slot landed on the
  // box: tools/c5_cold.py with GPK_REPLAY_TRACE=2): paid here, with the
  // context, on a 4 MiB pinned buffer in both directions.
  {
    void* h = nullptr;
    void* d = nullptr;
    constexpr size_t kWarm = 4u << 20;
    if (gpk_pin_alloc(&h, kWarm) == hipSuccess && hipMalloc(&d, kWarm) == hipSuccess) {
      memset(h, 0, kWarm);
      if (hipMemcpyAsync(d, h, kWarm, hipMemcpyHostToDevice, c->stream) == hipSuccess &&
          hipMemcpyAsync(h, d, kWarm, hipMemcpyDeviceToHost, c->stream) == hipSuccess)
        (void)hipStreamSynchronize(c->stream);
    }
    if (d) (void)hipFree(d);
    if (h) (void)gpk_pin_free(h);
  }
  *out = c;
  return GPK_OK;
}

int gpk_ctx_destroy(gpk_ctx* c) {
  if (!c) return GPK_OK;
  gpk::DeviceScope dscope(c->device);
  (void)hipDeviceSynchronize();  // launches still reading the table copies
  if (c->stream) (void)hipStreamDestroy(c->stream);
  free_slots(c);
  if (c->dbuf) (void)hipFree(c->dbuf);
  if (c->replay_cache && c->replay_cache_free) c->replay_cache_free(c->replay_cache);
  delete c;
  return GPK_OK;
}

static uint32_t host_code_of(int64_t lt) {
  for (unsigned k = 1; k < 13; k++)
    if (gpk_code_layer_type(k) == lt) return k;
  return GPK_CODE_NONE;
}

// Compact LDS copy of the lookup tables (gpk_device.h LTab): a dictionary of
// the distinct LayerTypes the tables can produce (handles), the IP protocol
// table as handles, and for each 16-bit table its most common value plus an
// open-addressed hash of the keys that differ from it. Returns false when
// the tables do not fit (more than kCtMaxHandles distinct types or
// kCtMaxSlots slots): the kernels then read the global tables.
static bool build_compact(const gpk::DevTables& t, int64_t first, uint32_t* blob, gpk::CompactGeom& g) {
  using namespace gpk;
  std::vector<int32_t> vals;
  std::unordered_map<int32_t, uint32_t> idx;
  bool ok = true;
  auto handle = [&](int32_t lt) -> uint32_t {
    auto it = idx.find(lt);
    if (it != idx.end()) return it->second;
    if (vals.size() >= (size_t)kCtMaxHandles) {
      ok = false;
      return 0;
    }
    idx[lt] = (uint32_t)vals.size();
    vals.push_back(lt);
    return (uint32_t)vals.size() - 1;
  };
  memset(blob, 0, kCtDwords * 4);
  memset(&g, 0, sizeof(g));
  g.zero_h = handle(GPK_LT_ZERO);
  g.frag_h = handle(GPK_LT_FRAGMENT);
  g.payload_h = handle(GPK_LT_PAYLOAD);
  g.first_h = (first >= 0 && first < GPK_MAX_LAYER_TYPE) ? handle((int32_t)first) : 0;
  uint8_t* ipp = (uint8_t*)(blob + kCtIpp);
  for (int k = 0; k < 256; k++) ipp[k] = (uint8_t)handle(t.ipprotocol[k]);
  uint32_t next_slot = kCtSlots;
  auto hash_table = [&](const int32_t* tab, uint32_t& off, uint32_t& shift, uint32_t& mask, uint32_t& maxp,
                        uint32_t& def) {
    std::unordered_map<int32_t, uint32_t> count;
    for (int k = 0; k < 65536; k++) count[tab[k]]++;
    int32_t dv = tab[0];
    for (auto& kv : count)
      if (kv.second > count[dv]) dv = kv.first;
    def = handle(dv);
    uint32_t nex = 65536 - count[dv];
    uint32_t bits = 3;
    while ((1u << bits) < 2 * nex) bits++;
    const uint32_t size = 1u << bits;
    if (next_slot + size > (uint32_t)kCtDwords) {
      ok = false;
      return;
    }
    off = next_slot;
    shift = 32 - bits;
    mask = size - 1;
    maxp = 0;
    for (uint32_t i = 0; i < size; i++) blob[off + i] = 0xffffffffu;
    for (uint32_t k = 0; k < 65536; k++) {
      if (tab[k] == dv) continue;
      uint32_t h = (k * 0x9E3779B1u) >> shift, d = 0;
      while (blob[off + ((h + d) & mask)] != 0xffffffffu) d++;
      blob[off + ((h + d) & mask)] = k | (handle(tab[k]) << 16);
      if (d > maxp) maxp = d;
    }
    next_slot += size;
  };
  hash_table(t.ethertype, g.eth_off, g.eth_shift, g.eth_mask, g.eth_probe, g.eth_def);
  if (ok) hash_table(t.tcp_port, g.tcp_off, g.tcp_shift, g.tcp_mask, g.tcp_probe, g.tcp_def);
  if (ok) hash_table(t.udp_port, g.udp_off, g.udp_shift, g.udp_mask, g.udp_probe, g.udp_def);
  if (!ok) return false;
  uint8_t* kc = (uint8_t*)(blob + kCtKc);
  for (size_t h = 0; h < vals.size(); h++) {
    const int32_t lt = vals[h];
    const uint32_t kind = (lt >= 0 && lt < GPK_MAX_LAYER_TYPE) ? t.dispatch[lt] : GPK_DEC_NONE;
    kc[h] = (uint8_t)(kind | (host_code_of(lt) << 4));
    blob[kCtVal + h] = (uint32_t)lt;
  }
  g.words = next_slot;
  return true;
}

// Tables of parser p on the device (global copy always, compact copy when it
// fits), and the table fields of P.
int gpk_ctx_set_table_mode(gpk_ctx* c, int mode) {
  if (!c || (mode != GPK_TABLES_AUTO && mode != GPK_TABLES_GLOBAL)) return GPK_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  c->force_global = mode == GPK_TABLES_GLOBAL;  // copies are keyed by mode too
  return GPK_OK;
}

// Transitions the kernels' straight-line path may take for this parser
// (gpk_device.h fast_parser): each is allowed when the tables send it to the
// decoder the path hard-codes.
static uint32_t fast_flags(const gpk_parser* p) {
  auto kind = [&](int32_t lt) { return (lt >= 0 && lt < GPK_MAX_LAYER_TYPE) ? (int)p->tab.dispatch[lt] : GPK_DEC_NONE; };
  if (p->first != GPK_LT_ETHERNET || kind(GPK_LT_ETHERNET) != GPK_DEC_ETHERNET) return 0;
  uint32_t f = GPK_FAST_ON;
  if (kind(p->tab.ethertype[0x0800]) == GPK_DEC_IPV4) f |= GPK_FAST_IP4;
  if (kind(p->tab.ethertype[0x86dd]) == GPK_DEC_IPV6) f |= GPK_FAST_IP6;
  if (kind(p->tab.ethertype[0x8100]) == GPK_DEC_DOT1Q) f |= GPK_FAST_D1Q;
  if (kind(p->tab.ethertype[0x88a8]) == GPK_DEC_DOT1Q) f |= GPK_FAST_QINQ;
  if (kind(p->tab.ipprotocol[6]) == GPK_DEC_TCP) f |= GPK_FAST_TCP;
  if (kind(p->tab.ipprotocol[17]) == GPK_DEC_UDP) f |= GPK_FAST_UDP;
  return f;
}

// Caller streams with an aggregation stream of their own: enough for
// gpk_replay_file's one stream per staging slot plus the caller's (its slots
// option stays far below), so steady launches never create or retire one.
constexpr size_t kAggStreams = 32;

// The aggregation stream and reusable event of caller stream s (created on
// first use; beyond kAggStreams callers the least recently used one is
// retired WITHOUT waiting: it moves to c->retired, and is destroyed by a later
// call once hipStreamQuery reports its marks complete. Nothing here blocks
// while c->mu is held, so a caller stream that waits on host progress cannot
// deadlock another caller.
static int agg_of(gpk_ctx* c, hipStream_t s, gpk_ctx::Agg** out) {
  for (size_t k = 0; k < c->retired.size();) {
    const hipError_t q = hipStreamQuery(c->retired[k].agg);
    if (q == hipErrorNotReady) {
      k++;
      continue;
    }
    (void)hipStreamDestroy(c->retired[k].agg);
    (void)hipEventDestroy(c->retired[k].ev);
    c->retired[k] = c->retired.back();
    c->retired.pop_back();
  }
  auto it = c->aggs.find(s);
  if (it == c->aggs.end()) {
    if (c->aggs.size() >= kAggStreams) {
      auto lru = c->aggs.begin();
      for (auto j = c->aggs.begin(); j != c->aggs.end(); ++j)
        if (j->second.last_use < lru->second.last_use) lru = j;
      c->retired.push_back(lru->second);  // its marks may be pending: a completed event stays complete
      c->aggs.erase(lru);
    }
    gpk_ctx::Agg a;
    HIPCHK(hipStreamCreateWithFlags(&a.agg, hipStreamNonBlocking));
    if (hipEventCreateWithFlags(&a.ev, hipEventDisableTiming) != hipSuccess) {
      (void)hipStreamDestroy(a.agg);
      return hip_fail(hipErrorOutOfMemory, "hipEventCreateWithFlags");
    }
    it = c->aggs.emplace(s, a).first;
  }
  it->second.last_use = ++c->tick;
  *out = &it->second;
  return GPK_OK;
}

// Record, as mark, the point stream s has reached (on s's aggregation
// stream). cumulative: the mark also stays behind its own previous record
// (a slot's done covers every launch that read it, on any stream).
static int mark_after(gpk_ctx* c, hipStream_t s, hipEvent_t mark, bool cumulative) {
  gpk_ctx::Agg* a = nullptr;
  int rc = agg_of(c, s, &a);
  if (rc) return rc;
  HIPCHK(hipEventRecord(a->ev, s));
  HIPCHK(hipStreamWaitEvent(a->agg, a->ev, 0));
  if (cumulative) HIPCHK(hipStreamWaitEvent(a->agg, mark, 0));
  HIPCHK(hipEventRecord(mark, a->agg));
  return GPK_OK;
}

// The device copy of parser p's tables for a launch on stream s (found, or
// written into a free or the least recently used slot), and the table fields
// of P. Stream-ordered: returns without waiting for the device. Returns the
// slot index in *slot for note_launch.
static int upload(gpk_ctx* c, const gpk_parser* p, gpk::KParams& P, int* slot, hipStream_t s) {
  int k = -1;
  for (int i = 0; i < kTabSlots; i++)
    if (c->slots[i].version == p->version && c->slots[i].global_mode == c->force_global) k = i;
  if (k < 0) {
    for (int i = 0; i < kTabSlots; i++)
      if (k < 0 || c->slots[i].last_use < c->slots[k].last_use) k = i;  // empty slots have last_use 0
    TabSlot& t = c->slots[k];
    constexpr size_t kBlobOff = (sizeof(gpk::DevTables) + 255) & ~size_t(255);
    t.version = 0;
    if (!t.dtab && hipMalloc(&t.dtab, sizeof(gpk::DevTables)) != hipSuccess) return GPK_ENOMEM;
    if (!t.dctab && hipMalloc(&t.dctab, gpk::kCtDwords * 4) != hipSuccess) return GPK_ENOMEM;
    if (!t.staging && hipHostMalloc((void**)&t.staging, kBlobOff + gpk::kCtDwords * 4, hipHostMallocDefault) != hipSuccess)
      return GPK_ENOMEM;
    if (!t.ready) HIPCHK(hipEventCreateWithFlags(&t.ready, hipEventDisableTiming));
    if (!t.done) HIPCHK(hipEventCreateWithFlags(&t.done, hipEventDisableTiming));
    // the staging buffer is the source of the slot's previous upload: rewrite
    // it once that copy has landed (long ago unless slots are thrashing)
    if (t.uploaded && !t.ready_seen) HIPCHK(hipEventSynchronize(t.ready));
    // every launch that read the old contents completes before the new upload
    if (t.read) HIPCHK(hipStreamWaitEvent(s, t.done, 0));
    memcpy(t.staging, &p->tab, sizeof(gpk::DevTables));
    uint32_t* blob = reinterpret_cast<uint32_t*>(t.staging + kBlobOff);
    t.compact = !c->force_global && build_compact(p->tab, p->first, blob, t.cg);
    HIPCHK(hipMemcpyAsync(t.dtab, t.staging, sizeof(gpk::DevTables), hipMemcpyHostToDevice, s));
    if (t.compact) HIPCHK(hipMemcpyAsync(t.dctab, blob, gpk::kCtDwords * 4, hipMemcpyHostToDevice, s));
    int rc = mark_after(c, s, t.ready, false);
    if (rc) return rc;
    t.uploaded = true;
    t.ready_seen = false;
    t.version = p->version;
    t.global_mode = c->force_global;
  } else {
    // uploaded by a launch on some stream: this launch waits for the copy
    TabSlot& t = c->slots[k];
    if (!t.ready_seen) {
      const hipError_t q = hipEventQuery(t.ready);
      if (q == hipSuccess) {
        t.ready_seen = true;
      } else if (q == hipErrorNotReady) {
        HIPCHK(hipStreamWaitEvent(s, t.ready, 0));
      } else {
        return hip_fail(q, "hipEventQuery(ready)");
      }
    }
  }
  TabSlot& t = c->slots[k];
  t.last_use = ++c->tick;
  *slot = k;
  P.tab = t.dtab;
  P.ctab = t.compact ? t.dctab : nullptr;
  P.cg = t.cg;
  P.first_kind = (p->first >= 0 && p->first < GPK_MAX_LAYER_TYPE) ? p->tab.dispatch[p->first] : GPK_DEC_NONE;
  P.fast = fast_flags(p);
  // headers that fit the 4-chunk window: no decoder that adds tags, IPv6, extension headers or TCP options
  P.small_headers = 1;
  // headers that fit the 5-chunk dword-aligned window (>= 77 bytes): no IPv6 decoder (Ethernet + two tags +
  // IPv4 + TCP with timestamps is 74 bytes)
  P.mid_headers = 1;
  for (int t2 = 0; t2 < GPK_MAX_LAYER_TYPE; t2++) {
    const int kd = p->tab.dispatch[t2];
    if (kd == GPK_DEC_DOT1Q || kd == GPK_DEC_IPV6 || kd == GPK_DEC_IPV6_EXT || kd == GPK_DEC_TCP) P.small_headers = 0;
    if (kd == GPK_DEC_IPV6 || kd == GPK_DEC_IPV6_EXT) P.mid_headers = 0;
  }
  return GPK_OK;
}

// A launch on stream s reads slot k: the slot's done mark moves past it (on
// the aggregation stream, which waits for s there; one reusable event per
// caller stream), so the slot is rewritten only after it completes.
static int note_launch(gpk_ctx* c, int k, hipStream_t s) {
  TabSlot& t = c->slots[k];
  int rc = mark_after(c, s, t.done, t.read);
  if (rc) return rc;
  t.read = true;
  return GPK_OK;
}

// Diagnostic builds (GPK_DIAG_TIMES) write per-wave timestamps here.
static std::atomic<uint64_t*> g_diag{nullptr};

constexpr uint64_t kMaxBatchPackets = ((1ull << 31) - 1) * 256;  // include/gpk.h gpk_batch

static int make_params(gpk_ctx* c, const gpk_parser* p, const gpk_batch* b, const gpk_results* o,
                       gpk::KParams& P, uint64_t packet_bytes = 0) {
  if (!c || !p || !b) return GPK_EINVAL;
  if (b->n && (!b->data || !b->offsets || !b->caplens)) return GPK_EINVAL;
  // one 256-packet tile per workgroup: the grid's x dimension bounds a batch
  if (b->n > kMaxBatchPackets) return GPK_EINVAL;
  // 16-byte chunk reads never leave the 16-byte granule of a valid byte only
  // if the packet buffer itself is 16-byte aligned.
  if (((uintptr_t)b->data & 15) != 0) return GPK_EINVAL;
  if (o && b->n && !o->records) return GPK_EINVAL;
  if (o && (p->outputs & GPK_OUT_FLOWS) && b->n && !o->flows) return GPK_EINVAL;
  P.data = b->data;
  P.offsets = b->offsets;
  P.caplens = b->caplens;
  P.n = b->n;
  const uint64_t mean = b->n ? (packet_bytes ? packet_bytes : b->data_bytes) / b->n : 0;
  P.big_packets = mean >= 1024;
  P.mean_bytes = mean > 0xffffffffull ? 0xffffffffu : (uint32_t)mean;
  P.data_end = (b->data_bytes + 15) & ~15ull;
  P.records = o ? o->records : nullptr;
  P.err_args = o ? o->err_args : nullptr;
  P.flows = o && (p->outputs & GPK_OUT_FLOWS) ? o->flows : nullptr;
  P.layouts = o ? o->layouts : nullptr;
  P.tab = nullptr;  // upload()
  P.ctab = nullptr;
  P.first_kind = GPK_DEC_NONE;
  P.fast = 0;
  P.first = p->first;
  P.outputs = p->outputs;
  P.ignore_unsupported = p->ignore_unsupported;
  P.key_kind = 0;
  P.small_headers = 0;
  P.mid_headers = 0;
  P.keys = nullptr;
  P.khash = nullptr;
  P.kcode = nullptr;
  P.diag = g_diag.load();
  P.fields = nullptr;
  P.narrow = 0;
  P.wide = nullptr;
  return GPK_OK;
}

int gpk_diag_set_buffer(void* buf) {
  g_diag.store(static_cast<uint64_t*>(buf));
  return GPK_OK;
}

int gpk_decode_batch(gpk_ctx* c, const gpk_parser* p, const gpk_batch* b, const gpk_results* o, void* stream) {
  if (!o) return GPK_EINVAL;
  gpk::KParams P;
  int rc = make_params(c, p, b, o, P);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  std::lock_guard<std::mutex> g(c->mu);
  gpk::DeviceScope dscope(c->device);
  HIPCHK(dscope.err);
  int slot = 0;
  rc = upload(c, p, P, &slot, s);
  if (rc) return rc;
  HIPCHK(gpk_launch_decode(&P, (p->outputs & GPK_OUT_L4_CSUM) != 0, o->layouts != nullptr, s));
  return note_launch(c, slot, s);
}

int gpk_decode_batch_narrow(gpk_ctx* c, const gpk_parser* p, const gpk_batch* b, const gpk_results8* o8,
                            void* stream) {
  if (!o8 || (b && b->n && (!o8->records || !o8->wide))) return GPK_EINVAL;
  // the kernels take the narrow records through the record pointer
  const gpk_results o{reinterpret_cast<gpk_record*>(o8->records), o8->err_args, o8->flows, nullptr};
  gpk::KParams P;
  int rc = make_params(c, p, b, &o, P);
  if (rc) return rc;
  P.narrow = 1;
  P.wide = o8->wide;
  hipStream_t s = (hipStream_t)stream;
  std::lock_guard<std::mutex> g(c->mu);
  gpk::DeviceScope dscope(c->device);
  HIPCHK(dscope.err);
  int slot = 0;
  rc = upload(c, p, P, &slot, s);
  if (rc) return rc;
  HIPCHK(gpk_launch_decode(&P, (p->outputs & GPK_OUT_L4_CSUM) != 0, 0, s));
  return note_launch(c, slot, s);
}

int gpk_decode_batch_fields(gpk_ctx* c, const gpk_parser* p, const gpk_batch* b, const gpk_results* o,
                            gpk_fields* fields, void* stream) {
  if (!o || (b && b->n && !fields)) return GPK_EINVAL;
  if (o->layouts) {  // layouts too: the decode with layouts, then the extraction from them
    int rc = gpk_decode_batch(c, p, b, o, stream);
    return rc ? rc : gpk_extract_fields(b, o->layouts, fields, stream);
  }
  gpk::KParams P;
  int rc = make_params(c, p, b, o, P);
  if (rc) return rc;
  P.fields = fields;
  hipStream_t s = (hipStream_t)stream;
  std::lock_guard<std::mutex> g(c->mu);
  gpk::DeviceScope dscope(c->device);
  HIPCHK(dscope.err);
  int slot = 0;
  rc = upload(c, p, P, &slot, s);
  if (rc) return rc;
  HIPCHK(gpk_launch_decode_fields(&P, s, nullptr));
  return note_launch(c, slot, s);
}

// gpk_decode_batch for the library's own pipelines (gpk_replay_file,
// gpk_tpacket_pump), which know the batch's packet bytes apart from the
// readable end of data: data_bytes is the readable end only, packet_bytes the
// mean-size hint; the name of the kernel launched goes to kname when given.
// Library-internal, not part of the C ABI.
// fields: the fused decode + layer fields launch (gpk_decode_batch_fields,
// no layouts), else NULL.
extern "C" __attribute__((visibility("hidden"))) int gpk_decode_batch_ex(gpk_ctx* c, const gpk_parser* p,
                                                                         const gpk_batch* b, const gpk_results* o,
                                                                         void* stream, uint64_t packet_bytes,
                                                                         char* kname, size_t kcap, gpk_fields* fields) {
  if (!o || (fields && o->layouts)) return GPK_EINVAL;
  gpk::KParams P;
  int rc = make_params(c, p, b, o, P, packet_bytes);
  if (rc) return rc;
  P.fields = fields;
  hipStream_t s = (hipStream_t)stream;
  std::lock_guard<std::mutex> g(c->mu);
  gpk::DeviceScope dscope(c->device);
  HIPCHK(dscope.err);
  int slot = 0;
  rc = upload(c, p, P, &slot, s);
  if (rc) return rc;
  if (kname && kcap) {
    if (fields)
      gpk_launch_describe_fields(&P, kname, kcap);
    else
      gpk_launch_describe(&P, (p->outputs & GPK_OUT_L4_CSUM) != 0, o->layouts != nullptr, kname, kcap);
  }
  if (fields)
    HIPCHK(gpk_launch_decode_fields(&P, s, nullptr));
  else
    HIPCHK(gpk_launch_decode(&P, (p->outputs & GPK_OUT_L4_CSUM) != 0, o->layouts != nullptr, s));
  return note_launch(c, slot, s);
}

// gpk_decode_batch plus the fused grouping key per packet (gpk_flows.hip
// gpk_decode_group_batch): library-internal, not part of the C ABI.
extern "C" __attribute__((visibility("hidden"))) int gpk_decode_batch_keys(gpk_ctx* c, const gpk_parser* p, const gpk_batch* b,
                                                                const gpk_results* o, int key_kind, uint32_t* keys,
                                                                uint64_t* khash, int32_t* kcode, void* stream) {
  if (!o || o->layouts || (key_kind != 1 && key_kind != 2) || (b && b->n && (!keys || !khash || !kcode)))
    return GPK_EINVAL;
  gpk::KParams P;
  int rc = make_params(c, p, b, o, P);
  if (rc) return rc;
  P.key_kind = key_kind;
  P.keys = keys;
  P.khash = khash;
  P.kcode = kcode;
  hipStream_t s = (hipStream_t)stream;
  std::lock_guard<std::mutex> g(c->mu);
  gpk::DeviceScope dscope(c->device);
  HIPCHK(dscope.err);
  int slot = 0;
  rc = upload(c, p, P, &slot, s);
  if (rc) return rc;
  HIPCHK(gpk_launch_decode(&P, (p->outputs & GPK_OUT_L4_CSUM) != 0, o->layouts != nullptr, s));
  return note_launch(c, slot, s);
}

int gpk_decode_kernel_name(gpk_ctx* c, const gpk_parser* p, const gpk_batch* b, int with_layouts, char* buf,
                           size_t cap) {
  if (!buf || !cap) return GPK_EINVAL;
  gpk::KParams P;
  gpk_results o{nullptr, nullptr, nullptr, nullptr};
  int rc = make_params(c, p, b, nullptr, P);
  if (rc) return rc;
  (void)o;
  std::lock_guard<std::mutex> g(c->mu);
  gpk::DeviceScope dscope(c->device);
  HIPCHK(dscope.err);
  int slot = 0;
  rc = upload(c, p, P, &slot, c->stream);
  if (rc) return rc;
  if (with_layouts == GPK_NAME_FIELDS) return gpk_launch_describe_fields(&P, buf, cap);
  return gpk_launch_describe(&P, (p->outputs & GPK_OUT_L4_CSUM) != 0, with_layouts != 0, buf, cap);
}

int gpk_decode_occupancy(gpk_ctx* c, const gpk_parser* p, const gpk_batch* b, int with_layouts, int* blocks_per_cu) {
  if (!blocks_per_cu) return GPK_EINVAL;
  gpk::KParams P;
  int rc = make_params(c, p, b, nullptr, P);
  if (rc) return rc;
  std::lock_guard<std::mutex> g(c->mu);
  gpk::DeviceScope dscope(c->device);
  HIPCHK(dscope.err);
  int slot = 0;
  rc = upload(c, p, P, &slot, c->stream);
  if (rc) return rc;
  if (with_layouts == GPK_NAME_FIELDS) {
    P.fields = reinterpret_cast<gpk_fields*>(16);  // described, never written
    HIPCHK(gpk_launch_decode_fields(&P, nullptr, blocks_per_cu));
    return GPK_OK;
  }
  HIPCHK(gpk_launch_occupancy(&P, (p->outputs & GPK_OUT_L4_CSUM) != 0, with_layouts != 0, blocks_per_cu));
  return GPK_OK;
}

static int ensure_dbuf(gpk_ctx* c, size_t bytes) {
  if (c->dbuf_bytes >= bytes) return GPK_OK;
  if (c->dbuf) (void)hipFree(c->dbuf);
  c->dbuf = nullptr;
  c->dbuf_bytes = 0;
  if (hipMalloc(&c->dbuf, bytes) != hipSuccess) return GPK_ENOMEM;
  c->dbuf_bytes = bytes;
  return GPK_OK;
}

static size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

// The host-buffer decode, with the layer fields when hf is non-null (fused
// launch, or with layouts the decode then gpk_extract_fields, as
// gpk_decode_batch_fields does on the device).
static int decode_host(gpk_ctx* c, const gpk_parser* p, const gpk_batch* hb, const gpk_results* ho, gpk_fields* hf) {
  if (!c || !p || !hb || !ho) return GPK_EINVAL;
  if (hb->n && (!hb->data || !hb->offsets || !hb->caplens || !ho->records)) return GPK_EINVAL;
  const uint64_t n = hb->n;
  const bool flows = (p->outputs & GPK_OUT_FLOWS) && ho->flows;
  if ((p->outputs & GPK_OUT_FLOWS) && !ho->flows && n) return GPK_EINVAL;
  size_t o_data = 0, o_off = align_up(o_data + hb->data_bytes + 16), o_cap = align_up(o_off + n * 8),
         o_rec = align_up(o_cap + n * 4), o_err = align_up(o_rec + n * sizeof(gpk_record)),
         o_fl = align_up(o_err + (ho->err_args ? n * 8 : 0)), o_lay = align_up(o_fl + (flows ? n * 24 : 0)),
         o_fld = align_up(o_lay + (ho->layouts ? n * sizeof(gpk_layout) : 0)),
         total = align_up(o_fld + (hf ? n * sizeof(gpk_fields) : 0));
  std::lock_guard<std::mutex> g(c->mu);
  gpk::DeviceScope dscope(c->device);
  HIPCHK(dscope.err);
  int rc = ensure_dbuf(c, total);
  if (rc) return rc;
  char* d = (char*)c->dbuf;
  hipStream_t s = c->stream;
  HIPCHK(hipMemcpyAsync(d + o_data, hb->data, hb->data_bytes, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(d + o_off, hb->offsets, n * 8, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(d + o_cap, hb->caplens, n * 4, hipMemcpyHostToDevice, s));
  if (ho->err_args) HIPCHK(hipMemsetAsync(d + o_err, 0, n * 8, s));
  gpk_batch db{(const uint8_t*)(d + o_data), (const uint64_t*)(d + o_off), (const uint32_t*)(d + o_cap), n,
               hb->data_bytes};
  gpk_results dr{(gpk_record*)(d + o_rec), ho->err_args ? (uint32_t*)(d + o_err) : nullptr,
                 flows ? (uint64_t*)(d + o_fl) : nullptr, ho->layouts ? (gpk_layout*)(d + o_lay) : nullptr};
  gpk::KParams P;
  rc = make_params(c, p, &db, &dr, P);
  if (rc) return rc;
  int slot = 0;
  rc = upload(c, p, P, &slot, s);
  if (rc) return rc;
  gpk_fields* df = hf ? (gpk_fields*)(d + o_fld) : nullptr;
  if (df && !dr.layouts) {
    P.fields = df;
    HIPCHK(gpk_launch_decode_fields(&P, s, nullptr));
  } else {
    HIPCHK(gpk_launch_decode(&P, (p->outputs & GPK_OUT_L4_CSUM) != 0, dr.layouts != nullptr, s));
  }
  rc = note_launch(c, slot, s);
  if (rc) return rc;
  if (df && dr.layouts && n) {
    rc = gpk_extract_fields(&db, dr.layouts, df, s);
    if (rc) return rc;
  }
  HIPCHK(hipMemcpyAsync(ho->records, dr.records, n * sizeof(gpk_record), hipMemcpyDeviceToHost, s));
  if (ho->err_args) HIPCHK(hipMemcpyAsync(ho->err_args, dr.err_args, n * 8, hipMemcpyDeviceToHost, s));
  if (flows) HIPCHK(hipMemcpyAsync(ho->flows, dr.flows, n * 24, hipMemcpyDeviceToHost, s));
  if (ho->layouts) HIPCHK(hipMemcpyAsync(ho->layouts, dr.layouts, n * sizeof(gpk_layout), hipMemcpyDeviceToHost, s));
  if (df) HIPCHK(hipMemcpyAsync(hf, df, n * sizeof(gpk_fields), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return GPK_OK;
}

int gpk_decode_batch_host(gpk_ctx* c, const gpk_parser* p, const gpk_batch* hb, const gpk_results* ho) {
  return decode_host(c, p, hb, ho, nullptr);
}

int gpk_decode_batch_host_fields(gpk_ctx* c, const gpk_parser* p, const gpk_batch* hb, const gpk_results* ho,
                                 gpk_fields* host_fields) {
  if (hb && hb->n && !host_fields) return GPK_EINVAL;
  return decode_host(c, p, hb, ho, host_fields);
}

int gpk_decoded_list(gpk_ctx* c, const gpk_parser* p, const gpk_batch* b, uint64_t index, int64_t* out_types,
                     uint32_t cap, uint32_t* out_n) {
  if (!out_n || (cap && !out_types)) return GPK_EINVAL;
  gpk::KParams P;
  int rc = make_params(c, p, b, nullptr, P);
  if (rc) return rc;
  if (index >= b->n) return GPK_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  gpk::DeviceScope dscope(c->device);
  HIPCHK(dscope.err);
  rc = ensure_dbuf(c, align_up(8 * (size_t)cap) + 256);
  if (rc) return rc;
  int64_t* dl = (int64_t*)c->dbuf;
  uint32_t* dn = (uint32_t*)((char*)c->dbuf + align_up(8 * (size_t)cap));
  hipStream_t s = c->stream;
  int slot = 0;
  rc = upload(c, p, P, &slot, s);
  if (rc) return rc;
  HIPCHK(gpk_launch_list(&P, index, dl, cap, dn, s));
  rc = note_launch(c, slot, s);
  if (rc) return rc;
  uint32_t n = 0;
  HIPCHK(hipMemcpyAsync(&n, dn, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  uint32_t k = n < cap ? n : cap;
  if (k) HIPCHK(hipMemcpy(out_types, dl, 8 * (size_t)k, hipMemcpyDeviceToHost));
  *out_n = n;
  return GPK_OK;
}

int gpk_decoded_list_host(gpk_ctx* c, const gpk_parser* p, const uint8_t* pkt, uint32_t caplen, int64_t* out_types,
                          uint32_t cap, uint32_t* out_n) {
  if (!c || !p || !out_n || (caplen && !pkt) || (cap && !out_types)) return GPK_EINVAL;
  size_t o_off = align_up((size_t)caplen + 16), o_cap = o_off + 256, o_list = o_cap + 256,
         o_n = align_up(o_list + 8 * (size_t)cap), total = o_n + 256;
  std::lock_guard<std::mutex> g(c->mu);
  gpk::DeviceScope dscope(c->device);
  HIPCHK(dscope.err);
  int rc = ensure_dbuf(c, total);
  if (rc) return rc;
  char* d = (char*)c->dbuf;
  hipStream_t s = c->stream;
  uint64_t zero = 0;
  HIPCHK(hipMemcpyAsync(d, pkt, caplen, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(d + o_off, &zero, 8, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(d + o_cap, &caplen, 4, hipMemcpyHostToDevice, s));
  gpk_batch db{(const uint8_t*)d, (const uint64_t*)(d + o_off), (const uint32_t*)(d + o_cap), 1, caplen};
  gpk::KParams P;
  rc = make_params(c, p, &db, nullptr, P);
  if (rc) return rc;
  int slot = 0;
  rc = upload(c, p, P, &slot, s);
  if (rc) return rc;
  HIPCHK(gpk_launch_list(&P, 0, (int64_t*)(d + o_list), cap, (uint32_t*)(d + o_n), s));
  rc = note_launch(c, slot, s);
  if (rc) return rc;
  uint32_t n = 0;
  HIPCHK(hipMemcpyAsync(&n, d + o_n, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  uint32_t k = n < cap ? n : cap;
  if (k) HIPCHK(hipMemcpy(out_types, d + o_list, 8 * (size_t)k, hipMemcpyDeviceToHost));
  *out_n = n;
  return GPK_OK;
}

// ---- pinned host memory (gpk_pinned.h) --------------------------------------
namespace {
constexpr size_t kHuge = 2u << 20;
std::mutex g_pin_mu;
std::unordered_map<void*, size_t> g_pinned;  // mapped (huge-page) buffers -> their mapping length
}  // namespace

// Bytes the host can still back (MemAvailable of /proc/meminfo), or SIZE_MAX
// when unknown.
static size_t mem_available() {
  FILE* f = fopen("/proc/meminfo", "r");
  if (!f) return SIZE_MAX;
  char line[256];
  size_t kb = 0;
  bool found = false;
  while (fgets(line, sizeof line, f))
    if (sscanf(line, "MemAvailable: %zu kB", &kb) == 1) {
      found = true;
      break;
    }
  fclose(f);
  return found ? kb * 1024 : SIZE_MAX;
}

hipError_t gpk_pin_alloc(void** out, size_t bytes) {
  *out = nullptr;
  if (bytes >= 2 * kHuge) {
    const size_t len = (bytes + kHuge - 1) & ~(kHuge - 1);
    // Under the default overcommit policy an anonymous mapping the host cannot
    // back still succeeds, and touching it below would get the process
    // OOM-killed instead of returning an error: refuse a request larger than
    // what the host has available first.
    if (len > mem_available()) return hipErrorOutOfMemory;
    void* m = mmap(nullptr, len + kHuge, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (m != MAP_FAILED) {
      // 2 MiB-aligned, so transparent huge pages can back all of it
      const uintptr_t a = ((uintptr_t)m + kHuge - 1) & ~(uintptr_t)(kHuge - 1);
      if (a > (uintptr_t)m) munmap(m, a - (uintptr_t)m);
      const uintptr_t end = (uintptr_t)m + len + kHuge;
      if (end > a + len) munmap((void*)(a + len), end - (a + len));
      char* p = (char*)a;
      (void)madvise(p, len, MADV_HUGEPAGE);
      // fault it in (one fault per huge page; the kernel zeroes each): a
      // buffer of 64 MiB or more on up to 8 threads (pin_probe: 4 x 512 MiB
      // in 18 ms touched 4 ways each)
      const size_t nt = len >= (64u << 20) ? std::min<size_t>(8, len / (32u << 20)) : 1;
      const size_t per = ((len / nt) + kHuge - 1) & ~(kHuge - 1);
      auto touch = [p, len, per](size_t t) {
        const size_t a = t * per, b = std::min(len, a + per);
        for (size_t o = a; o < b; o += 4096) p[o] = 0;
      };
      std::vector<std::thread> th;
      size_t t = 1;
      try {
        for (; t < nt; t++) th.emplace_back(touch, t);
      } catch (const std::system_error&) {  // no thread to spare: the rest on this one
        for (size_t u = t; u < nt; u++) touch(u);
      }
      touch(0);
      for (auto& x : th) x.join();
      if (hipHostRegister(p, len, hipHostRegisterDefault) == hipSuccess) {
        std::lock_guard<std::mutex> g(g_pin_mu);
        g_pinned[p] = len;
        *out = p;
        return hipSuccess;
      }
      munmap(p, len);
    }
  }
  return hipHostMalloc(out, bytes, hipHostMallocDefault);
}

hipError_t gpk_pin_free(void* p) {
  if (!p) return hipSuccess;
  size_t len = 0;
  {
    std::lock_guard<std::mutex> g(g_pin_mu);
    auto it = g_pinned.find(p);
    if (it != g_pinned.end()) {
      len = it->second;
      g_pinned.erase(it);
    }
  }
  if (!len) return hipHostFree(p);
  const hipError_t e = hipHostUnregister(p);
  munmap(p, len);
  return e;
}

int gpk_host_alloc(void** out, size_t bytes) {
  if (!out) return GPK_EINVAL;
  HIPCHK(gpk_pin_alloc(out, bytes));
  return GPK_OK;
}

int gpk_host_free(void* p) {
  if (p) HIPCHK(gpk_pin_free(p));
  return GPK_OK;
}

// ---- error values ------------------------------------------------------------
int gpk_layer_type_name(int64_t lt, char* buf, size_t cap) {
  // LayerType.String(), layertype.go:101-111
  for (int i = 0; i < GPK_N_LAYER_TYPE_NAMES; i++)
    if (GPK_LAYER_TYPE_NAMES[i].id == lt) return snprintf(buf, cap, "%s", GPK_LAYER_TYPE_NAMES[i].name);
  return snprintf(buf, cap, "%lld", (long long)lt);
}

static const char* ip_protocol_name(uint32_t v) {
  // IPProtocol.String(), enums_generated.go:131-140
  for (int i = 0; i < GPK_N_IPPROTOCOL_ROWS; i++)
    if ((uint32_t)GPK_IPPROTOCOL_ROWS[i].value == v) return GPK_IPPROTOCOL_ROWS[i].name;
  return "UnknownIPProtocol";
}

int gpk_format_error(unsigned code, uint32_t a0, uint32_t a1, char* buf, size_t cap) {
  char lt[64];
  switch (code) {
    case GPK_ERR_NONE: return snprintf(buf, cap, "%s", "");
    case GPK_ERR_UNSUPPORTED:  // parser.go:325-327
      gpk_layer_type_name((int32_t)a0, lt, sizeof(lt));
      return snprintf(buf, cap, "No decoder for layer type %s", lt);
    // panicToError parser.go:329-333 wrapping Go runtime bounds errors
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
    case GPK_ERR_IP4_OPT_EXCEEDS:
      return snprintf(buf, cap, "IP option length exceeds remaining IP header size, option type %u length %u", a0, a1);
    case GPK_ERR_IP4_OPT_BADLEN: return snprintf(buf, cap, "Invalid IP option type %u length %u. Must be greater than 2", a0, a1);
    case GPK_ERR_IP6_HDR_SHORT: return snprintf(buf, cap, "Invalid ip6 header. Length %u less than 40", a0);
    case GPK_ERR_IP6_JUMBO_AND_LEN: return snprintf(buf, cap, "IPv6 has jumbo length and IPv6 length is not 0");
    case GPK_ERR_IP6_LEN0_NO_JUMBO: return snprintf(buf, cap, "IPv6 length 0, but HopByHop header does not have jumbogram option");
    case GPK_ERR_IP6_LEN0: return snprintf(buf, cap, "IPv6 length 0, but next header is %s, not HopByHop", ip_protocol_name(a0));
    case GPK_ERR_IP6_TLV_SHORT: return snprintf(buf, cap, "IPv6 header option too small");
    case GPK_ERR_IP6_TLV_TOO_SMALL: return snprintf(buf, cap, "IPv6 header TLV option too small");
    case GPK_ERR_IP6_EXT_SHORT: return snprintf(buf, cap, "Invalid ip6-extension header. Length %u less than 2", a0);
    case GPK_ERR_IP6_EXT_LEN: return snprintf(buf, cap, "Invalid ip6-extension header. Length %u less than specified length %u", a0, a1);
    case GPK_ERR_IP6_JUMBO_TLV_LEN: return snprintf(buf, cap, "Jumbo length TLV data must have length 4");
    case GPK_ERR_IP6_JUMBO_SMALL: return snprintf(buf, cap, "Jumbo length cannot be less than %d", 65535 + 1);
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
    default: return snprintf(buf, cap, "unknown gpk error %u", code);
  }
}

int64_t gpk_code_layer_type(unsigned code) {
  static const int64_t map[13] = {GPK_LT_ZERO,          GPK_LT_ETHERNET,       GPK_LT_DOT1Q,
                                  GPK_LT_IPV4,          GPK_LT_IPV6,           GPK_LT_IPV6_HOPBYHOP,
                                  GPK_LT_IPV6_ROUTING,  GPK_LT_IPV6_FRAGMENT,  GPK_LT_IPV6_DESTINATION,
                                  GPK_LT_TCP,           GPK_LT_UDP,            GPK_LT_PAYLOAD,
                                  GPK_LT_FRAGMENT};
  return code < 13 ? map[code] : -1;
}

}  // extern "C"

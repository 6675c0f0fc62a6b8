// gpk_replay.cpp — whole-capture replay through HBM (gpk_replay_file,
// include/gpk_capture.h): BASELINE config C5, the path that starts and ends in
// host memory.
//
// The reference loop this replaces (examples/pcapdump, gopacket_benchmark):
//   r, _ := pcapgo.NewNgReader(f, opts)            pcapgo/ngread.go:64-107
//   for { data, ci, err := r.ReadPacketData()      ngread.go:629-632
//         parser.DecodeLayers(data, &decoded)      parser.go:303-317
//         ... VerifyChecksum / Flow.FastHash }
//
// MI355X-first shape of it:
//   * the file is read straight into pinned staging slots (several pread
//     threads per slot, or zlib for gzip files); the capture bytes are never
//     repacked: the slot IS the packet batch, indexed in place by the record
//     walker (gpk_capture.cpp);
//   * per slot, one HtoD of the whole slot, then per batch of packets one
//     HtoD of its index (12 B/packet), the decode kernel, one DtoH of the
//     records/flows; every slot has its own HIP stream, so the copy engines
//     and the CUs work on different slots at once;
//   * the next slot is read while the current one is walked and the previous
//     ones are on the device; the unfinished record at a slot's end is
//     carried into the head of the next slot (a reserved carry region);
//   * the record walk itself runs on the device once the reader has read the
//     section header and interfaces (gpk_walk.h): the slot goes to HBM first,
//     a segmented walk indexes its plain Enhanced Packet Blocks in place, and
//     the host's exact reader takes over only where a block is not plain, so
//     the host CPUs are left to the file reads.
// Results are delivered in packet order through the callback.
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <pthread.h>
#include <sched.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <cstdlib>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <deque>
#include <future>
#include <string>
#include <thread>
#include <vector>

#include "../../include/gpk_capture.h"
#include "gpk_pinned.h"
#include "gpk_devguard.h"
#include "gpk_walk.h"

extern "C" int gpk_decode_batch_ex(gpk_ctx* c, const gpk_parser* p, const gpk_batch* b, const gpk_results* o,
                                   void* stream, uint64_t packet_bytes, char* kname, size_t kcap,
                                   gpk_fields* fields);

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// The CPUs of the device's NUMA node (sysfs local_cpulist of its PCI
// function) that this thread may run on; false when unknown or empty. The
// reader threads copy the file into pinned staging memory that the device's
// DMA then reads, and the calling thread walks and launches: on the device's
// node (profiles/r14_c5_numa.txt). GPK_REPLAY_NUMA: 0 leaves every thread
// where it is, 1 pins the reader threads, 2 (default) also the calling thread
// for the duration of the call.
int numa_level() {
  const char* env = getenv("GPK_REPLAY_NUMA");
  return env && env[0] >= '0' && env[0] <= '2' ? env[0] - '0' : 2;
}
bool device_local_cpus(int dev, cpu_set_t& out) {
  if (numa_level() == 0) return false;
  char bdf[64] = {0};
  if (hipDeviceGetPCIBusId(bdf, (int)sizeof(bdf) - 1, dev) != hipSuccess) return false;
  for (char* p = bdf; *p; p++) *p = (char)tolower((unsigned char)*p);
  char path[160];
  snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/local_cpulist", bdf);
  FILE* f = fopen(path, "r");
  if (!f) return false;
  char buf[4096] = {0};
  const size_t k = fread(buf, 1, sizeof(buf) - 1, f);
  fclose(f);
  buf[k] = 0;
  cpu_set_t allowed;
  CPU_ZERO(&allowed);
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return false;
  CPU_ZERO(&out);
  for (char* p = buf; *p;) {  // "a-b,c,d-e\n"
    char* e = nullptr;
    const long lo = strtol(p, &e, 10);
    if (e == p) break;
    long hi = lo;
    p = e;
    if (*p == '-') {
      hi = strtol(p + 1, &e, 10);
      p = e;
    }
    for (long c = lo; c <= hi && c < CPU_SETSIZE; c++)
      if (c >= 0 && CPU_ISSET(c, &allowed)) CPU_SET(c, &out);
    while (*p == ',' || *p == '\n' || *p == ' ') p++;
  }
  return CPU_COUNT(&out) > 0;
}

struct Src {  // the capture byte stream: plain file (parallel pread) or gzip (zlib)
  int fd = -1;
  gzFile gz = nullptr;
  uint64_t size = 0, pos = 0;  // size: of the stream (the file, or the parts' sum)
  bool at_end = false;
  int threads = 8;
  bool pin = false;  // run the reader threads on `cpus` (the device's NUMA node)
  cpu_set_t cpus;
  // A byte-range replay reads a stream made of file parts (the section header
  // and interfaces, then the range's blocks): (file offset, length) in order.
  // Empty: the whole file.
  std::vector<std::pair<uint64_t, uint64_t>> parts;

  // stream bytes [at, at + n) into dst (across parts); returns the count read
  uint64_t pread_at(uint8_t* dst, uint64_t at, uint64_t n) const {
    uint64_t done = 0, vbase = 0;
    for (size_t k = 0; k < (parts.empty() ? 1 : parts.size()) && done < n; k++) {
      const uint64_t foff = parts.empty() ? 0 : parts[k].first, plen = parts.empty() ? size : parts[k].second;
      const uint64_t v = at + done;
      if (v >= vbase + plen) {
        vbase += plen;
        continue;
      }
      uint64_t rel = v - vbase;
      const uint64_t want = std::min<uint64_t>(n - done, plen - rel);
      uint64_t got = 0;
      while (got < want) {
        const ssize_t r = pread(fd, dst + done + got, want - got, (off_t)(foff + rel + got));
        if (r <= 0) return done + got;
        got += (uint64_t)r;
      }
      done += got;
      vbase += plen;
    }
    return done;
  }

  // Fill dst with up to cap bytes of the stream; returns the count.
  uint64_t read(uint8_t* dst, uint64_t cap) {
    if (at_end) return 0;
    if (gz) {
      uint64_t got = 0;
      while (got < cap) {
        unsigned ask = (unsigned)std::min<uint64_t>(cap - got, 1u << 30);
        int k = gzread(gz, dst + got, ask);
        if (k <= 0) {  // end, or a truncated / corrupt body: the stream ends here
          at_end = true;
          break;
        }
        got += (uint64_t)k;
      }
      return got;
    }
    uint64_t want = std::min<uint64_t>(cap, size - pos);
    const uint64_t base = pos;
    const int T = want >= (8u << 20) ? threads : 1;
    std::vector<std::thread> th;
    std::vector<uint64_t> got(T, 0);
    const uint64_t per = (want + T - 1) / T;
    for (int t = 0; t < T; t++) {
      th.emplace_back([&, t] {
        if (pin) (void)pthread_setaffinity_np(pthread_self(), sizeof(cpus), &cpus);
        uint64_t a = (uint64_t)t * per, e = std::min<uint64_t>(want, a + per);
        if (a < e) got[t] = pread_at(dst + a, base + a, e - a);
      });
    }
    for (auto& x : th) x.join();
    uint64_t total = 0;
    for (int t = 0; t < T; t++) total += got[t];
    pos += total;
    if (pos >= size || total < want) at_end = true;
    return total;
  }
};

struct Fill {      // one read of a slot's fresh bytes
  uint64_t bytes;  // read
  bool end;        // the stream ended with this read
  double t0, t1;   // read start / end (GPK_REPLAY_TRACE=2)
  hipEvent_t sent; // recorded after the read's HtoD (device walk), or null
  std::string err; // the slot's allocation failed (the read did not run)
};

struct Slot {
  uint8_t* host = nullptr;  // [carry region | fresh bytes | 16 B slack], pinned
  uint8_t* dev = nullptr;
  // device record walk (gpk_walk.h): per-segment results, and the slot's
  // packet index on the device (offsets relative to dev)
  gpk::WalkSegs d_seg{}, h_seg{};
  uint64_t* d_off = nullptr;
  uint32_t* d_cap = nullptr;
  gpk_capture_info* d_ci = nullptr;
  uint64_t idx_cap = 0;  // entries of d_off / d_cap / d_ci
  hipStream_t stream = nullptr;
  hipEvent_t h2d = nullptr;  // the slot's HtoD finished: host buffer reusable
  hipEvent_t sent = nullptr; // the read thread's HtoD of the fresh bytes finished (orders the next one)
  hipError_t h2d_err = hipSuccess;  // the read thread's HtoD of the fresh bytes (device walk)
  bool h2d_pending = false;
  std::shared_future<struct Fill> fill;  // async read of the fresh bytes
  bool fill_pending = false;
};

struct Bat {
  uint64_t* h_off = nullptr;
  uint32_t* h_cap = nullptr;
  gpk_capture_info* h_ci = nullptr;
  gpk_record* h_rec = nullptr;
  uint32_t* h_err = nullptr;
  uint64_t* h_flow = nullptr;
  uint64_t* d_off = nullptr;
  uint32_t* d_cap = nullptr;
  gpk_record* d_rec = nullptr;
  uint32_t* d_err = nullptr;
  uint64_t* d_flow = nullptr;
  gpk_fields* h_fields = nullptr;  // opts.fields_cb: the layer fields (allocated on the first call that asks)
  gpk_fields* d_fields = nullptr;
  hipEvent_t e0 = nullptr, k0 = nullptr, k1 = nullptr, done = nullptr;
  uint64_t first = 0, n = 0, flows_n = 0;
  bool with_fields = false;  // this launch wrote fields
  const uint8_t* base = nullptr;  // opts.packets_cb: the staging bytes h_off is relative to
  uint64_t base_bytes = 0;        // ... how many of them hold the slot's records
  int slot = -1;                  // ... and their slot, held until this batch is delivered
};

struct Pipeline {
  std::vector<Slot> slots;
  std::vector<Bat> bats;
  std::deque<int> free_bats, inflight;
  uint64_t P = 0;
  gpk_replay_cb cb = nullptr;
  gpk_replay_fields_cb fields_cb = nullptr;
  gpk_replay_packets_cb packets_cb = nullptr;
  std::vector<int> slot_batches;  // undelivered batches per staging slot (packets_cb)
  void* user = nullptr;
  gpk_replay_stats* st = nullptr;
  std::string herr;
  // gpk_stop: the context and its stop count when the call started; once it
  // has changed no callback is made and the rest only drains
  const gpk_ctx* ctx = nullptr;
  uint64_t stop0 = 0;
  bool stopped = false;
  uint64_t delivered = 0;  // packets whose callbacks were made
  bool stop_seen() {
    if (!stopped && gpk_ctx_stop_seq(ctx) != stop0) stopped = true;
    return stopped;
  }
  // first call: the slots' and batches' buffers are allocated in the
  // background (slot 0 and the first two batches first, the rest behind
  // them while slot 0 is read); the read of a slot and the first use of a
  // batch wait for their own allocation (empty string = done)
  std::vector<std::shared_future<std::string>> slot_ready, bat_ready;
  std::atomic<uint64_t> alloc_wait_ns{0};  // time the pipeline waited for them

  bool ok(hipError_t e, const char* what) {
    if (e != hipSuccess && herr.empty()) herr = std::string(what) + ": " + hipGetErrorString(e);
    return e == hipSuccess;
  }

  // wait for the oldest in-flight batch and hand its results to the caller
  bool deliver_oldest() {
    int b = inflight.front();
    inflight.pop_front();
    Bat& B = bats[b];
    if (!ok(hipEventSynchronize(B.done), "hipEventSynchronize")) return false;
    float ms = 0, kms = 0;
    if (hipEventElapsedTime(&ms, B.e0, B.done) == hipSuccess) st->gpu_s += ms * 1e-3;
    if (hipEventElapsedTime(&kms, B.k0, B.k1) == hipSuccess) st->kernel_s += kms * 1e-3;
    double t = now_s();
    const bool deliver = !stop_seen();  // a batch is delivered whole or not at all
    if (deliver) {
      for (uint64_t i = 0; i < B.n; i++) st->packet_bytes += B.h_cap[i];
      delivered += B.n;
    }
    if (deliver && packets_cb && B.base) packets_cb(user, B.first, B.n, B.base, B.base_bytes, B.h_off, B.h_cap);
    if (B.slot >= 0 && (size_t)B.slot < slot_batches.size()) slot_batches[B.slot]--;
    B.slot = -1;
    B.base = nullptr;
    if (deliver && fields_cb && B.with_fields) fields_cb(user, B.first, B.n, B.h_fields);  // before the batch's results
    if (deliver && cb) cb(user, B.first, B.n, B.h_rec, B.h_err, B.h_flow, B.h_ci, B.h_cap);
    st->deliver_s += now_s() - t;
    free_bats.push_back(b);
    return true;
  }

  int acquire() {
    while (free_bats.empty())
      if (!deliver_oldest()) return -1;
    int b = free_bats.front();
    free_bats.pop_front();
    if ((size_t)b < bat_ready.size() && bat_ready[b].valid()) {
      const double t = now_s();
      const std::string e = bat_ready[b].get();
      alloc_wait_ns += (uint64_t)((now_s() - t) * 1e9);
      bat_ready[b] = std::shared_future<std::string>();
      if (!e.empty()) {
        if (herr.empty()) herr = e;
        return -1;
      }
    }
    return b;
  }

  // every background allocation has finished (their buffers can be freed or kept)
  std::string settle() {
    std::string first;
    for (auto* v : {&slot_ready, &bat_ready})
      for (auto& f : *v)
        if (f.valid()) {
          const std::string e = f.get();
          if (first.empty()) first = e;
          f = std::shared_future<std::string>();
        }
    return first;
  }

  ~Pipeline() {
    (void)settle();
    for (auto& s : slots) {
      if (s.fill_pending) s.fill.wait();
      if (s.stream) (void)hipStreamSynchronize(s.stream);
      if (s.host) (void)gpk_pin_free(s.host);
      if (s.dev) (void)hipFree(s.dev);
      for (void* p : {(void*)s.d_seg.sync, (void*)s.d_seg.end, (void*)s.d_seg.count, (void*)s.d_seg.base,
                      (void*)s.d_off, (void*)s.d_cap, (void*)s.d_ci})
        if (p) (void)hipFree(p);
      for (void* p : {(void*)s.h_seg.sync, (void*)s.h_seg.end, (void*)s.h_seg.count, (void*)s.h_seg.base})
        if (p) (void)hipHostFree(p);
      if (s.h2d) (void)hipEventDestroy(s.h2d);
      if (s.sent) (void)hipEventDestroy(s.sent);
      if (s.stream) (void)hipStreamDestroy(s.stream);
    }
    for (auto& B : bats) {
      for (void* p : {(void*)B.h_off, (void*)B.h_cap, (void*)B.h_ci, (void*)B.h_rec, (void*)B.h_err,
                      (void*)B.h_flow, (void*)B.h_fields})
        if (p) (void)gpk_pin_free(p);
      for (void* p : {(void*)B.d_off, (void*)B.d_cap, (void*)B.d_rec, (void*)B.d_err, (void*)B.d_flow,
                      (void*)B.d_fields})
        if (p) (void)hipFree(p);
      for (hipEvent_t e : {B.e0, B.k0, B.k1, B.done})
        if (e) (void)hipEventDestroy(e);
    }
  }
};

constexpr uint32_t kMaxSeg = 65536;  // device-walk segments per slot (>= 4 KiB each)
constexpr uint64_t kOpenPrefix = 64 << 10;  // host-read bytes before the device walk when the reader is not open

#define ALLOC_OK(call, what) \
  do {                       \
    if ((call) != hipSuccess) return std::string(what) + ": " + hipGetErrorString(hipGetLastError()); \
  } while (0)

std::string alloc_slot(Slot& s, uint64_t C, uint64_t R, bool dev_walk, uint64_t max_pk) {
  ALLOC_OK(gpk_pin_alloc((void**)&s.host, C + R + 16), "pinned slot");
  memset(s.host + C + R, 0, 16);
  ALLOC_OK(hipMalloc((void**)&s.dev, C + R + 16), "hipMalloc slot");
  ALLOC_OK(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking), "hipStreamCreate");
  ALLOC_OK(hipEventCreateWithFlags(&s.h2d, hipEventDisableTiming), "hipEventCreate");
  ALLOC_OK(hipEventCreateWithFlags(&s.sent, hipEventDisableTiming), "hipEventCreate");
  if (!dev_walk) return "";
  ALLOC_OK(hipMalloc((void**)&s.d_seg.sync, kMaxSeg * 8), "hipMalloc walk");
  ALLOC_OK(hipMalloc((void**)&s.d_seg.end, kMaxSeg * 8), "hipMalloc walk");
  ALLOC_OK(hipMalloc((void**)&s.d_seg.count, kMaxSeg * 4), "hipMalloc walk");
  ALLOC_OK(hipMalloc((void**)&s.d_seg.base, kMaxSeg * 8), "hipMalloc walk");
  ALLOC_OK(hipHostMalloc((void**)&s.h_seg.sync, kMaxSeg * 8, 0), "hipHostMalloc walk");
  ALLOC_OK(hipHostMalloc((void**)&s.h_seg.end, kMaxSeg * 8, 0), "hipHostMalloc walk");
  ALLOC_OK(hipHostMalloc((void**)&s.h_seg.count, kMaxSeg * 4, 0), "hipHostMalloc walk");
  ALLOC_OK(hipHostMalloc((void**)&s.h_seg.base, kMaxSeg * 8, 0), "hipHostMalloc walk");
  ALLOC_OK(hipMalloc((void**)&s.d_off, max_pk * 8), "hipMalloc index");
  ALLOC_OK(hipMalloc((void**)&s.d_cap, max_pk * 4), "hipMalloc index");
  ALLOC_OK(hipMalloc((void**)&s.d_ci, max_pk * sizeof(gpk_capture_info)), "hipMalloc index");
  s.idx_cap = max_pk;
  return "";
}

// The slot's device index must hold `need` entries, of which the first `keep`
// (the device walk's packets, written on the slot's stream) are kept. The
// first size assumes the device walk's blocks (plain EPBs, >= 32 bytes); the
// host reader's packets that follow can be smaller records (Simple Packet
// Blocks of 16 bytes, ngread.go:515-530), so a slot full of them grows it.
std::string grow_index(Slot& s, uint64_t keep, uint64_t need) {
  if (need <= s.idx_cap) return "";
  const uint64_t cap = std::max<uint64_t>(need, 2 * s.idx_cap);
  uint64_t* o = nullptr;
  uint32_t* c = nullptr;
  gpk_capture_info* ci = nullptr;
  ALLOC_OK(hipMalloc((void**)&o, cap * 8), "hipMalloc index");
  ALLOC_OK(hipMalloc((void**)&c, cap * 4), "hipMalloc index");
  ALLOC_OK(hipMalloc((void**)&ci, cap * sizeof(gpk_capture_info)), "hipMalloc index");
  if (keep) {
    ALLOC_OK(hipMemcpyAsync(o, s.d_off, keep * 8, hipMemcpyDeviceToDevice, s.stream), "DtoD index");
    ALLOC_OK(hipMemcpyAsync(c, s.d_cap, keep * 4, hipMemcpyDeviceToDevice, s.stream), "DtoD index");
    ALLOC_OK(hipMemcpyAsync(ci, s.d_ci, keep * sizeof(gpk_capture_info), hipMemcpyDeviceToDevice, s.stream),
             "DtoD index");
  }
  ALLOC_OK(hipStreamSynchronize(s.stream), "hipStreamSynchronize");
  (void)hipFree(s.d_off);
  (void)hipFree(s.d_cap);
  (void)hipFree(s.d_ci);
  s.d_off = o;
  s.d_cap = c;
  s.d_ci = ci;
  s.idx_cap = cap;
  return "";
}

std::string alloc_bat(Bat& B, uint64_t P) {
  ALLOC_OK(gpk_pin_alloc((void**)&B.h_off, P * 8), "pinned batch");
  ALLOC_OK(gpk_pin_alloc((void**)&B.h_cap, P * 4), "pinned batch");
  ALLOC_OK(gpk_pin_alloc((void**)&B.h_ci, P * sizeof(gpk_capture_info)), "pinned batch");
  ALLOC_OK(gpk_pin_alloc((void**)&B.h_rec, P * sizeof(gpk_record)), "pinned batch");
  ALLOC_OK(gpk_pin_alloc((void**)&B.h_err, P * 8), "pinned batch");
  ALLOC_OK(gpk_pin_alloc((void**)&B.h_flow, P * 24), "pinned batch");
  ALLOC_OK(hipMalloc((void**)&B.d_off, P * 8), "hipMalloc");
  ALLOC_OK(hipMalloc((void**)&B.d_cap, P * 4), "hipMalloc");
  ALLOC_OK(hipMalloc((void**)&B.d_rec, P * sizeof(gpk_record)), "hipMalloc");
  ALLOC_OK(hipMalloc((void**)&B.d_err, P * 8), "hipMalloc");
  ALLOC_OK(hipMalloc((void**)&B.d_flow, P * 24), "hipMalloc");
  ALLOC_OK(hipEventCreate(&B.e0), "hipEventCreate");
  ALLOC_OK(hipEventCreate(&B.k0), "hipEventCreate");
  ALLOC_OK(hipEventCreate(&B.k1), "hipEventCreate");
  ALLOC_OK(hipEventCreate(&B.done), "hipEventCreate");
  return "";
}

// The buffers of a finished call, left in the context for the next one.
struct Cached {
  uint64_t C, R, P;
  bool dev_walk;
  std::vector<Slot> slots;
  std::vector<Bat> bats;
};
void free_cached(void* p) {
  Cached* c = (Cached*)p;
  Pipeline pl;  // its destructor frees what it holds
  pl.slots = std::move(c->slots);
  pl.bats = std::move(c->bats);
  delete c;
}

}  // namespace

// ---- byte-range replay (gpk_replay_file_range) --------------------------------
// N callers (one per GPU) replay one pcapng file by byte ranges with no data
// exchange. The range [begin, end) of a caller becomes the blocks that START
// in [sync(begin), sync(end)), where sync(X) is the first offset >= X (a
// multiple of 4) at which four plain EPBs chain inside the next 4 MiB under
// the reader state after the file's leading non-packet blocks (the section
// header and interfaces, read once by every caller): a property of the offset
// alone, so a caller's end and the next caller's begin are the same offset.
// The caller's reader sees the stream [0, H) ++ [sync(begin), sync(end)),
// H = the first packet block, and does exactly what NgReader.ReadPacketData
// does over it (ngread.go:494-718). The split is exact when, for every caller
// but the last, its reader met a clean io.EOF at sync(end) (so sync(end) was a
// real block boundary: a chain from a real boundary lands on real boundaries
// only) and no block in its range changed the reader state (a new section or
// interface): gpk_replay_range.clean / state_changed. Otherwise the caller
// that first fails must replay from its sync_begin to the end of the file
// (end = 0) and the later callers' results are dropped.
namespace {

uint32_t rd32(const uint8_t* p, bool be) {
  return be ? (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]
            : (uint32_t)p[3] << 24 | (uint32_t)p[2] << 16 | (uint32_t)p[1] << 8 | p[0];
}

// The first packet block (EPB 6, SPB 3, obsolete PB 2) of the file, walking
// block headers from the section header on; where the walk cannot go on (a
// malformed length, or 64 MiB of leading blocks), the offset it stopped at.
uint64_t ng_header_end(int fd, uint64_t size) {
  uint64_t p = 0;
  bool be = false;
  uint8_t h[12];
  while (p + 12 <= size && p < (64ull << 20)) {
    if (pread(fd, h, 12, (off_t)p) != 12) break;
    if (rd32(h, false) == 0x0A0D0D0Au) {  // section header (a palindrome): its byte-order magic
      if (rd32(h + 8, false) == 0x1A2B3C4Du) be = false;
      else if (rd32(h + 8, true) == 0x1A2B3C4Du) be = true;
      else break;
    }
    const uint32_t typ = rd32(h, be), len = rd32(h + 4, be);
    if (typ == 2 || typ == 3 || typ == 6) return p;
    if (len < 12 || (len & 3) || len > size - p) break;
    p += len;
  }
  return p;
}

}  // namespace

static int plan_range(Src& src, uint32_t ng_flags, gpk_replay_range* rg, uint64_t* hdr_version,
                      uint64_t* hdr_mutations) {
  const uint64_t size = src.size;
  const uint64_t H = ng_header_end(src.fd, size);
  gpk_capreader* hr = nullptr;
  if (gpk_capreader_create(&hr, GPK_CAP_PCAPNG, ng_flags)) return GPK_ENOMEM;
  struct Free {
    gpk_capreader* r;
    ~Free() { gpk_capreader_destroy(r); }
  } free_hr{hr};
  std::vector<uint8_t> buf(H + 16, 0);
  if (H && (uint64_t)pread(src.fd, buf.data(), H, 0) != H) return GPK_EINVAL;
  // the leading blocks as a stream that ends at H: the reader applies every one
  // of them and meets io.EOF at H (with more bytes to come it would roll the
  // blocks it read while looking for the first packet back)
  gpk_capindex x{};
  uint64_t used = 0;
  const int st = gpk_capreader_index_all(hr, buf.data(), H, 1, 1, &x, &used);
  const bool none = x.n == 0;
  gpk_capindex_free(&x);
  int at_eof = 0;
  gpk_capreader_error(hr, nullptr, 0, &at_eof, nullptr);
  const bool ok = st == GPK_CAP_END && at_eof && none && used == H;
  *hdr_version = ok ? gpk_capreader_state_version(hr) : 0;
  *hdr_mutations = gpk_capreader_mutations(hr);
  constexpr uint64_t kSpan = 4ull << 20, kWin = 4ull << 20;
  auto sync_at = [&](uint64_t X) -> uint64_t {
    if (X <= H) return H;
    if (X >= size || !*hdr_version) return size;  // no header state to sync under: the first caller takes all
    for (uint64_t a = X & ~3ull, from = X - a; a < size; a += kWin, from = 0) {
      const uint64_t w = std::min<uint64_t>(kWin + kSpan, size - a), to = std::min<uint64_t>(kWin, w);
      buf.assign(w, 0);
      const uint64_t got = (uint64_t)std::max<ssize_t>(0, pread(src.fd, buf.data(), w, (off_t)a));
      const uint64_t p = gpk_capreader_sync(hr, buf.data(), from, to, got, kSpan);
      if (p != ~0ull) return a + p;
    }
    return size;
  };
  const uint64_t b = rg->begin == 0 ? 0 : sync_at(rg->begin);
  const uint64_t e = rg->end == 0 || rg->end >= size ? size : std::max<uint64_t>(b, sync_at(rg->end));
  rg->header_end = H;
  rg->sync_begin = b;
  rg->sync_end = e;
  src.parts.clear();
  if (b == 0) {
    src.parts.push_back({0, e});
  } else {
    src.parts.push_back({0, H});
    if (e > b) src.parts.push_back({b, e - b});
  }
  src.size = 0;
  for (auto& p : src.parts) src.size += p.second;
  return GPK_OK;
}

static int replay_file(gpk_ctx* ctx, const gpk_parser* parser, const char* path, const gpk_replay_opts* o,
                       gpk_replay_cb cb, void* user, gpk_replay_stats* stats, gpk_replay_range* rg) {
  const double t_start = now_s();
  const uint64_t stop0 = gpk_ctx_stop_seq(ctx);  // gpk_stop calls from here on end this call
  gpk_replay_opts opt{0, 0, 256ull << 20, 4, 1ull << 20, 8, nullptr, nullptr};
  if (o) {
    opt.fields_cb = o->fields_cb;
    opt.packets_cb = o->packets_cb;
    opt.format = o->format;
    opt.ng_flags = o->ng_flags;
    if (o->slot_bytes) opt.slot_bytes = o->slot_bytes;
    if (o->slots > 0) opt.slots = o->slots;
    if (o->batch_pkts) opt.batch_pkts = o->batch_pkts;
    if (o->read_threads > 0) opt.read_threads = o->read_threads;
  }
  if (opt.slots < 2 || opt.slot_bytes < 4096 || opt.batch_pkts < 1) return GPK_EINVAL;

  // ---- the stream ------------------------------------------------------------
  Src src;
  src.threads = opt.read_threads;
  cpu_set_t caller_cpus;  // restored on every return (the calling thread pinned at level 2)
  bool caller_pinned = false;
  {
    int d = 0;
    (void)hipGetDevice(&d);
    src.pin = device_local_cpus(d, src.cpus);
    if (src.pin && numa_level() == 2 && pthread_getaffinity_np(pthread_self(), sizeof(caller_cpus), &caller_cpus) == 0)
      caller_pinned = pthread_setaffinity_np(pthread_self(), sizeof(src.cpus), &src.cpus) == 0;
  }
  struct Restore {
    bool on;
    cpu_set_t* set;
    ~Restore() {
      if (on) (void)pthread_setaffinity_np(pthread_self(), sizeof(*set), set);
    }
  } restore{caller_pinned, &caller_cpus};
  // the file, its gzip stream and the record reader are released on every
  // return, an exception's included (declared before the pipeline, whose
  // destructor waits for the read threads that use them)
  gpk_capreader* rd = nullptr;
  struct Release {
    Src* src;
    gpk_capreader** rd;
    ~Release() {
      if (*rd) gpk_capreader_destroy(*rd);
      if (src->gz) gzclose(src->gz);
      if (src->fd >= 0) close(src->fd);
    }
  } release{&src, &rd};
  src.fd = open(path, O_RDONLY);
  if (src.fd < 0) {
    snprintf(stats->error, sizeof(stats->error), "open %s failed", path);
    return GPK_EINVAL;
  }
  struct stat sb;
  fstat(src.fd, &sb);
  src.size = (uint64_t)sb.st_size;
  stats->file_bytes = src.size;
  uint8_t magic[4] = {0, 0, 0, 0};
  ssize_t mk = pread(src.fd, magic, 4, 0);
  if (mk >= 2 && magic[0] == 0x1f && magic[1] == 0x8b) {  // read.go:80-86, ngread.go:75-91
    if (src.size < 10) {  // gzip.NewReader: the header read hits EOF
      snprintf(stats->error, sizeof(stats->error), "unexpected EOF");
      stats->reader_status = 1;
      return GPK_OK;
    }
    src.gz = gzdopen(dup(src.fd), "rb");
    if (!src.gz) return GPK_ENOMEM;
    gzbuffer(src.gz, 1u << 20);
    if (gzread(src.gz, magic, 4) < 4) memset(magic, 0, 4);
    gzrewind(src.gz);
  }
  int format = opt.format;
  if (!format) {
    const uint32_t m = (uint32_t)magic[0] | (uint32_t)magic[1] << 8 | (uint32_t)magic[2] << 16 | (uint32_t)magic[3] << 24;
    format = m == 0x0A0D0D0Au ? GPK_CAP_PCAPNG : GPK_CAP_PCAP;
  }
  // ---- a byte range of the file (gpk_replay_file_range) ---------------------
  uint64_t hdr_version = 0, hdr_mutations = 0;
  if (rg) {
    if (src.gz || format != GPK_CAP_PCAPNG) {
      snprintf(stats->error, sizeof(stats->error), "byte-range replay needs an uncompressed pcapng file");
      return GPK_EUNSUPP;
    }
    const int rrc = plan_range(src, opt.ng_flags, rg, &hdr_version, &hdr_mutations);
    if (rrc) {
      snprintf(stats->error, sizeof(stats->error), "byte-range replay: reading the file failed");
      return rrc;
    }
    stats->file_bytes = src.size;
  }
  int rc = gpk_capreader_create(&rd, format, opt.ng_flags);
  if (rc) return rc;

  // ---- buffers ---------------------------------------------------------------
  // (kept in the context between calls: the pinned staging slots are ~GBs and
  // allocating them costs as much as replaying a 10 GB file)
  // fresh bytes per slot, and the carry region before them (the record cut by
  // the previous slot's end is moved there, so a record may be as long as
  // it): the whole slot up to 1 MiB, else a sixteenth of it and at least 1 MiB
  // (16 MiB of 256 MiB: 64 times the largest snap length pcap writers use; a
  // longer pcapng block exists only in theory, and the region is pinned memory
  // every slot holds: C5's first call allocated 3.4 GB of pinned staging with
  // 256 MiB carry regions and 8 batches of 2 Mi packets, 1.6 GB now)
  const uint64_t R = opt.slot_bytes, C = R <= (1ull << 20) ? R : std::max<uint64_t>(1ull << 20, R / 16);
  Pipeline pl;
  pl.cb = cb;
  pl.fields_cb = opt.fields_cb;
  pl.packets_cb = opt.packets_cb;
  pl.user = user;
  pl.st = stats;
  pl.ctx = ctx;
  pl.stop0 = stop0;
  pl.P = opt.batch_pkts;
  const uint64_t P = pl.P;
  // device record walk buffers (pcapng only; GPK_REPLAY_HOST_WALK=1 keeps the walk on the host)
  const char* hw = getenv("GPK_REPLAY_HOST_WALK");
  const bool dev_walk = format == GPK_CAP_PCAPNG && !(hw && hw[0] == '1');
  const uint64_t max_pk = (C + R) / 32 + 1;  // a block is at least 32 bytes
  bool good = true;
  Cached* cached = (Cached*)gpk_ctx_replay_take(ctx);
  if (cached && cached->C == C && cached->R == R && cached->P == P && cached->dev_walk == dev_walk &&
      cached->slots.size() == (size_t)opt.slots) {
    pl.slots = std::move(cached->slots);
    pl.bats = std::move(cached->bats);
    delete cached;
    for (auto& s : pl.slots) s.fill_pending = s.h2d_pending = false;
  } else {
    if (cached) free_cached(cached);
    pl.slots.resize(opt.slots);
    pl.bats.resize(opt.slots + 2);  // batches in flight: about one per slot (a slot of the C4 mix holds ~0.7 Mi packets)
    // Every slot and batch is allocated on its own thread, in the background:
    // slot 0 and the first two batches first, the rest once slot 0 is done,
    // while it is being read; the read of a slot and the first use of a batch
    // wait for their own allocation. With 1.6 GB of pinned staging from
    // huge-page memory (gpk_pinned.h) a cold call took 0.215 s this way against
    // 0.223 s allocating everything first and 0.20 s with the buffers kept
    // (tools/c5_cold.py, profiles/r15_c5_cold.txt); with 3.4 GB from
    // hipHostMalloc (0.38 s to pin) it was 0.45 s. GPK_REPLAY_EAGER_ALLOC=1
    // allocates everything before the first read.
    int dev = 0;
    (void)hipGetDevice(&dev);
    const bool lazy = !(getenv("GPK_REPLAY_EAGER_ALLOC") && getenv("GPK_REPLAY_EAGER_ALLOC")[0] == '1');
    auto slot_job = [&pl, C, R, dev_walk, max_pk, dev](size_t k, std::shared_future<std::string> after) {
      return std::async(std::launch::async, [&pl, C, R, dev_walk, max_pk, dev, k, after] {
               if (after.valid()) after.wait();
               (void)hipSetDevice(dev);
               return alloc_slot(pl.slots[k], C, R, dev_walk, max_pk);
             }).share();
    };
    auto bat_job = [&pl, P, dev](size_t b, std::shared_future<std::string> after) {
      return std::async(std::launch::async, [&pl, P, dev, b, after] {
               if (after.valid()) after.wait();
               (void)hipSetDevice(dev);
               return alloc_bat(pl.bats[b], P);
             }).share();
    };
    pl.slot_ready.resize(pl.slots.size());
    pl.bat_ready.resize(pl.bats.size());
    pl.slot_ready[0] = slot_job(0, {});
    const std::shared_future<std::string> gate = lazy ? pl.slot_ready[0] : std::shared_future<std::string>();
    for (size_t b = 0; b < pl.bats.size(); b++) pl.bat_ready[b] = bat_job(b, b < 2 ? std::shared_future<std::string>() : gate);
    for (size_t k = 1; k < pl.slots.size(); k++) pl.slot_ready[k] = slot_job(k, gate);
    if (!lazy) {
      const std::string e = pl.settle();
      if (!e.empty()) {
        good = false;
        pl.herr = e;
      }
    }
  }
  for (size_t i = 0; i < pl.bats.size(); i++) pl.free_bats.push_back((int)i);
  if (!good) {
    snprintf(stats->error, sizeof(stats->error), "%s", pl.herr.c_str());
    return GPK_ENOMEM;
  }

  // With the device walk the device copy of a slot mirrors its host layout
  // ([carry region | fresh bytes]), so the fresh bytes go to HBM from the
  // read thread as soon as they are read (on the slot's stream, after
  // everything earlier that reads the slot), overlapping the previous slot's
  // walk and decode; only the short carry is copied later.
  int dev = 0;
  (void)hipGetDevice(&dev);
  // Reads run ahead of the walk by up to slots-1 slots (a slot is refilled
  // once its carry has moved on and its last HtoD has landed); they are
  // chained, so the stream is still read strictly in order, one read at a
  // time, and each read's HtoD is issued as soon as it has finished.
  std::shared_future<Fill> last_fill;
  auto start_fill = [&](Slot& s) {
    s.h2d_err = hipSuccess;
    std::shared_future<Fill> prev = last_fill;
    // (mutable: the previous fill's future is dropped as soon as it has been
    // read, so the async states do not chain every fill of the call together)
    std::shared_future<std::string> ready;  // the slot's allocation (first call)
    const size_t si = (size_t)(&s - pl.slots.data());
    if (si < pl.slot_ready.size()) {
      ready = pl.slot_ready[si];
      pl.slot_ready[si] = std::shared_future<std::string>();
    }
    s.fill = std::async(std::launch::async, [&src, &s, &pl, C, R, stats, dev, dev_walk, prev, ready]() mutable {
      if (src.pin) (void)pthread_setaffinity_np(pthread_self(), sizeof(src.cpus), &src.cpus);
      if (ready.valid()) {
        const double ta = now_s();
        std::string e = ready.get();
        pl.alloc_wait_ns += (uint64_t)((now_s() - ta) * 1e9);
        if (!e.empty()) {
          if (prev.valid()) (void)prev.get();  // keep the chain's order
          return Fill{0, true, ta, ta, nullptr, e};
        }
      }
      hipEvent_t before = nullptr;
      if (prev.valid()) before = prev.get().sent;
      prev = std::shared_future<Fill>();
      double t = now_s();
      const uint64_t k = src.read(s.host + C, R);
      const bool end = src.at_end;
      const double t1 = now_s();
      stats->read_s += t1 - t;
      hipEvent_t sent = nullptr;
      if (dev_walk && k) {
        // the slots' copies go over the link one after another, in stream
        // order: several in flight at once share the link, and the slot the
        // walk needs next would land last (A/B r12: 49-52 GB/s against 45-47
        // with the copies overlapping)
        (void)hipSetDevice(dev);
        s.h2d_err = before ? hipStreamWaitEvent(s.stream, before, 0) : hipSuccess;
        if (s.h2d_err == hipSuccess) s.h2d_err = hipMemcpyAsync(s.dev + C, s.host + C, k, hipMemcpyHostToDevice, s.stream);
        if (s.h2d_err == hipSuccess) s.h2d_err = hipEventRecord(s.sent, s.stream);
        if (s.h2d_err == hipSuccess) sent = s.sent;
      }
      return Fill{k, end, t, t1, sent, std::string()};
    }).share();
    s.fill_pending = true;
    last_fill = s.fill;
  };
  uint64_t next_fill = 0;  // sequence number of the next slot to fill
  auto fill_ahead = [&](uint64_t upto) {  // issue the fills of slots [next_fill, upto)
    while (good && next_fill < upto) {
      Slot& N = pl.slots[next_fill % pl.slots.size()];
      // packets_cb: the slot's bytes are the packets its batches hand out
      while (good && pl.packets_cb && pl.slot_batches[next_fill % pl.slots.size()] > 0 && !pl.inflight.empty())
        good = pl.deliver_oldest();
      if (N.h2d_pending) {  // the slot's last HtoD read the host bytes about to be overwritten
        good = pl.ok(hipEventSynchronize(N.h2d), "hipEventSynchronize");
        N.h2d_pending = false;
      }
      if (good) start_fill(N);
      next_fill++;
    }
  };

  const double t_loop = now_s();
  const char* trace = getenv("GPK_REPLAY_TRACE");
  // ---- the loop --------------------------------------------------------------
  const uint8_t* carry = nullptr;
  uint64_t carry_len = 0, packet_index = 0;
  bool finished = false, clean_eof = false;
  rc = GPK_OK;
  pl.slot_batches.assign(pl.slots.size(), 0);
  fill_ahead(1);
  for (uint64_t si = 0; !finished && good && !pl.stop_seen(); si++) {
    Slot& S = pl.slots[si % pl.slots.size()];
    const double t_get = now_s();
    const Fill fl = S.fill.get();
    const double t_got = now_s();
    S.fill_pending = false;
    if (!fl.err.empty()) {
      good = false;
      if (pl.herr.empty()) pl.herr = fl.err;
      rc = GPK_ENOMEM;
      break;
    }
    const uint64_t fresh = fl.bytes;
    const bool eof = fl.end;
    if (carry_len > C) {  // a record longer than the carry region: not supported
      snprintf(stats->error, sizeof(stats->error), "capture record larger than the %llu-byte staging carry region",
               (unsigned long long)C);
      rc = GPK_EUNSUPP;
      break;
    }
    const uint64_t start = C - carry_len, len = carry_len + fresh;
    if (carry_len) memmove(S.host + start, carry, carry_len);
    stats->stream_bytes += fresh;
    // read ahead into every slot whose carry has moved on (the one just
    // taken from slot si - 1 included)
    // (with packets_cb the slot refilled next is the previous one, whose packets
    // are handed out with its batches' results: refilled after this slot's
    // batches are launched, so waiting for that delivery overlaps them)
    if (!eof && !pl.packets_cb) fill_ahead(si + pl.slots.size());
    // walk the records of [start, start+len): on the device once the reader
    // is open (gpk_walk.h), the rest (and everything before) on the host
    // (parallel, gpk_capreader_index_all)
    gpk_capindex xi{};
    uint64_t used = 0, G = 0;  // G: packets indexed on the device (the slot's first G)
    double t_ix = now_s();
    // the walk is a dependent load per record: more chains than cores hide DRAM latency
    const int walk_threads = std::min(64, 4 * opt.read_threads);
    gpk::WalkState ws;
    const bool dwalk = dev_walk;  // device index (S.d_*), slot layout mirrored on the device
    bool on_dev = dev_walk && gpk_capreader_walk_state(rd, &ws);  // ... and the walk runs there
    // positions relative to the 16-byte-aligned base the kernels get
    const uint64_t base_off = start & ~15ull, p0 = start & 15, L = p0 + len;
    int st = GPK_CAP_MORE;
    if (dwalk) {
      // the carry next to the fresh bytes the read thread has sent
      good = pl.ok(S.h2d_err, "HtoD slot");
      if (good && carry_len)
        good = pl.ok(hipMemcpyAsync(S.dev + start, S.host + start, carry_len, hipMemcpyHostToDevice, S.stream),
                     "HtoD carry");
      good = good && pl.ok(hipEventRecord(S.h2d, S.stream), "hipEventRecord");
      S.h2d_pending = true;
      uint64_t pos = p0, dev_pk = 0, g_emit = 0;  // g_emit: index entries sized for the emit kernel
      bool ended = false;  // a host stretch met the reader's end (GPK_CAP_END or an error): no further call
      std::vector<std::pair<uint64_t, gpk_capindex>> chunks;  // host stretches: (first index, packets)
      if (good && dev_walk && !on_dev && L - pos > kOpenPrefix) {
        // the reader is not open yet (the file's first slot): the host reads
        // the section header and interfaces, then the device walks the rest
        gpk_capindex hx{};
        uint64_t hu = 0;
        st = gpk_capreader_index_all(rd, S.host + base_off + pos, kOpenPrefix, 0, walk_threads, &hx, &hu);
        for (uint64_t i = 0; i < hx.n; i++) hx.offsets[i] += pos;
        if (hx.n) chunks.push_back({G, hx});
        else gpk_capindex_free(&hx);
        G += hx.n;
        pos += hu;
        ended = st != GPK_CAP_MORE;
        on_dev = !ended && gpk_capreader_walk_state(rd, &ws);
        if (trace && trace[0] == '3') fprintf(stderr, "  slot %llu host prefix %.2f ms\n", (unsigned long long)si, (now_s() - t_ix) * 1e3);
      }
      if (good && on_dev) {
        const uint64_t seg = std::max<uint64_t>(4096, ((L + kMaxSeg - 1) / kMaxSeg + 3) & ~3ull);
        const uint32_t nseg = (uint32_t)((L + seg - 1) / seg);
        good = pl.ok(gpk_walk_segments(S.dev + base_off, pos, L, seg, nseg, ws, S.d_seg, S.stream), "walk kernel") &&
               pl.ok(hipMemcpyAsync(S.h_seg.sync, S.d_seg.sync, nseg * 8ull, hipMemcpyDeviceToHost, S.stream),
                     "DtoH walk") &&
               pl.ok(hipMemcpyAsync(S.h_seg.end, S.d_seg.end, nseg * 8ull, hipMemcpyDeviceToHost, S.stream), "DtoH walk") &&
               pl.ok(hipMemcpyAsync(S.h_seg.count, S.d_seg.count, nseg * 4ull, hipMemcpyDeviceToHost, S.stream),
                     "DtoH walk") &&
               pl.ok(hipStreamSynchronize(S.stream), "hipStreamSynchronize");
        if (trace && trace[0] == '3') fprintf(stderr, "  slot %llu device walk %.2f ms\n", (unsigned long long)si, (now_s() - t_ix) * 1e3);
        // Accept segments while each starts where the previous one's chain
        // ended (segment 0 starts where the reader stands) and covers its
        // segment. Where one does not, the exact reader walks on the host from
        // there up to a later segment's chain start; if it lands on it exactly
        // with its walk state unchanged (a real block boundary, read the way the
        // device chain assumed), the device segments resume there. A fake
        // chain inside a payload, or one block longer than a segment, costs a
        // host walk of that stretch, not of the rest of the slot.
        for (uint32_t q = 0; q < nseg; q++) S.h_seg.base[q] = ~0ull;
        uint32_t k = (uint32_t)(pos / seg);  // the segment the reader stands in
        while (good && k < nseg) {
          while (k < nseg && S.h_seg.sync[k] == pos) {
            const uint64_t s1 = std::min<uint64_t>(L, (uint64_t)(k + 1) * seg);
            S.h_seg.base[k] = G;
            G += S.h_seg.count[k];
            dev_pk += S.h_seg.count[k];
            pos = S.h_seg.end[k];
            k++;
            if (pos < s1) break;  // a block that is not plain ended the chain
          }
          uint32_t j = k;  // the next chain start past pos
          while (j < nseg && (S.h_seg.sync[j] == ~0ull || S.h_seg.sync[j] <= pos)) j++;
          if (j >= nseg) break;
          gpk_capindex hx{};
          uint64_t hu = 0;
          st = gpk_capreader_index_all(rd, S.host + base_off + pos, S.h_seg.sync[j] - pos, 0, walk_threads, &hx, &hu);
          if (st < 0) {
            gpk_capindex_free(&hx);
            ended = true;
            break;
          }
          for (uint64_t i = 0; i < hx.n; i++) hx.offsets[i] += pos;
          if (hx.n) chunks.push_back({G, hx});
          else gpk_capindex_free(&hx);
          G += hx.n;
          pos += hu;
          if (st != GPK_CAP_MORE) {
            ended = true;
            break;
          }
          gpk::WalkState w2;
          if (!gpk_capreader_walk_state(rd, &w2) || memcmp(&w2, &ws, sizeof(ws)) != 0) break;  // the host takes the rest
          k = pos == S.h_seg.sync[j] ? j : j + 1;  // landed: resume there; else sync[j] was inside a record
        }
        if (trace && trace[0] == '3') fprintf(stderr, "  slot %llu accepted %.2f ms\n", (unsigned long long)si, (now_s() - t_ix) * 1e3);
        if (good && dev_pk) {
          g_emit = G;
          const std::string ge = grow_index(S, 0, G);
          if (!ge.empty()) {
            good = false;
            if (pl.herr.empty()) pl.herr = ge;
          }
          good = good &&
                 pl.ok(hipMemcpyAsync(S.d_seg.base, S.h_seg.base, nseg * 8ull, hipMemcpyHostToDevice, S.stream),
                       "HtoD walk") &&
                 pl.ok(gpk_walk_emit(S.dev + base_off, L, nseg, ws, S.d_seg, S.d_off, S.d_cap, S.d_ci, S.stream),
                       "emit kernel");
        }
      }
      if (good && !ended) {
        // the exact reader from the last block the device walk did not take
        st = gpk_capreader_index_all(rd, S.host + base_off + pos, L - pos, eof ? 1 : 0, walk_threads, &xi, &used);
        if (st >= 0) {
          for (uint64_t i = 0; i < xi.n; i++) xi.offsets[i] += pos;
          const uint64_t first = G;
          G += xi.n;
          if (xi.n) chunks.push_back({first, xi});
          else gpk_capindex_free(&xi);  // an empty index still holds its arrays (~1.8 MB leaked per slot before)
          xi = gpk_capindex{};
        }
      } else {
        used = 0;
      }
      used += pos - p0;
      if (good && st >= 0 && !chunks.empty()) {
        const std::string ge = grow_index(S, g_emit, G);  // (keeps what the emit kernel wrote)
        if (!ge.empty()) {
          good = false;
          if (pl.herr.empty()) pl.herr = ge;
        }
        for (const auto& ch : chunks) {
          const gpk_capindex& h = ch.second;
          good = good &&
                 pl.ok(hipMemcpyAsync(S.d_off + ch.first, h.offsets, h.n * 8, hipMemcpyHostToDevice, S.stream),
                       "HtoD index") &&
                 pl.ok(hipMemcpyAsync(S.d_cap + ch.first, h.caplens, h.n * 4, hipMemcpyHostToDevice, S.stream),
                       "HtoD index") &&
                 pl.ok(hipMemcpyAsync(S.d_ci + ch.first, h.ci, h.n * sizeof(gpk_capture_info), hipMemcpyHostToDevice,
                                      S.stream),
                       "HtoD index");
        }
        good = pl.ok(hipStreamSynchronize(S.stream), "hipStreamSynchronize") && good;  // the chunks are freed below
        if (trace && trace[0] == '3') fprintf(stderr, "  slot %llu host chunks copied %.2f ms\n", (unsigned long long)si, (now_s() - t_ix) * 1e3);
      }
      for (auto& ch : chunks) gpk_capindex_free(&ch.second);
      stats->device_walk_packets += dev_pk;
    } else {
      st = gpk_capreader_index_all(rd, S.host + start, len, eof ? 1 : 0, walk_threads, &xi, &used);
    }
    stats->index_s += now_s() - t_ix;
    const double t_walked = now_s();
    if (st < 0) {
      gpk_capindex_free(&xi);
      rc = st;
      finished = true;
      break;
    }
    if (!good) {
      gpk_capindex_free(&xi);
      break;
    }
    const uint64_t pos = start + used, total = G + xi.n;
    bool copied = dwalk;
    for (uint64_t first = 0; first < total && good && !pl.stop_seen();) {  // batches of up to P packets
      const uint64_t n = std::min<uint64_t>(P, total - first);
      const int b = pl.acquire();
      if (b < 0) {
        good = false;
        break;
      }
      Bat& B = pl.bats[b];
      B.with_fields = opt.fields_cb != nullptr;
      if (B.with_fields && !B.d_fields) {  // first call that asks for fields: this batch's buffers
        if ((!B.h_fields && gpk_pin_alloc((void**)&B.h_fields, P * sizeof(gpk_fields)) != hipSuccess) ||
            hipMalloc((void**)&B.d_fields, P * sizeof(gpk_fields)) != hipSuccess) {
          B.d_fields = nullptr;  // h_fields, when it was allocated, is kept for the next call
          (void)pl.ok(hipErrorOutOfMemory, "fields buffers");
          rc = GPK_ENOMEM;
          pl.free_bats.push_back(b);
          good = false;
          break;
        }
      }
      if (!dwalk) {
        memcpy(B.h_off, xi.offsets + first, n * 8);  // relative to the slot's device copy (start)
        memcpy(B.h_cap, xi.caplens + first, n * 4);
        memcpy(B.h_ci, xi.ci + first, n * sizeof(gpk_capture_info));
      }
      if (!copied) {  // the whole slot, once, before its first kernel
        good = pl.ok(hipMemcpyAsync(S.dev, S.host + start, len + 16, hipMemcpyHostToDevice, S.stream), "HtoD slot") &&
               pl.ok(hipEventRecord(S.h2d, S.stream), "hipEventRecord");
        S.h2d_pending = true;
        copied = true;
      }
      B.first = packet_index;
      B.n = n;
      if (pl.packets_cb) {  // the packets stay in this slot's staging bytes until delivered
        B.slot = (int)(si % pl.slots.size());
        B.base = dwalk ? S.host + base_off : S.host + start;
        B.base_bytes = dwalk ? start + len - base_off : len;  // the slot's bytes from base on
        pl.slot_batches[B.slot]++;
      }
      good = good && pl.ok(hipEventRecord(B.e0, S.stream), "hipEventRecord");
      if (!dwalk)
        good = good &&
               pl.ok(hipMemcpyAsync(B.d_off, B.h_off, n * 8, hipMemcpyHostToDevice, S.stream), "HtoD offsets") &&
               pl.ok(hipMemcpyAsync(B.d_cap, B.h_cap, n * 4, hipMemcpyHostToDevice, S.stream), "HtoD caplens");
      good = good && pl.ok(hipMemsetAsync(B.d_err, 0, n * 8, S.stream), "hipMemsetAsync") &&
             pl.ok(hipEventRecord(B.k0, S.stream), "hipEventRecord");
      if (!good) {
        pl.free_bats.push_back(b);
        break;
      }
      // data_bytes: the readable end of data (the device slot and its 16-byte
      // slack, measured from the base the kernels get); the mean-size hint
      // apart: the batch's capture lengths (host index), or its share of the
      // slot's bytes (device index: the capture lengths stay on the device)
      uint64_t pk_bytes = 0;
      if (dwalk) {
        pk_bytes = total ? (uint64_t)((double)L * (double)n / (double)total) : 0;
      } else {
        for (uint64_t i = 0; i < n; i++) pk_bytes += B.h_cap[i];
      }
      gpk_batch db{dwalk ? S.dev + base_off : S.dev, dwalk ? S.d_off + first : B.d_off,
                   dwalk ? S.d_cap + first : B.d_cap, n, dwalk ? C + R + 16 - base_off : len + 16};
      gpk_results dr{B.d_rec, B.d_err, B.d_flow, nullptr};
      int drc = gpk_decode_batch_ex(ctx, parser, &db, &dr, S.stream, pk_bytes ? pk_bytes : 1, stats->kernel,
                                    sizeof(stats->kernel), B.with_fields ? B.d_fields : nullptr);
      if (drc) {
        rc = drc;
        finished = true;
        good = false;
        pl.free_bats.push_back(b);
        break;
      }
      good = pl.ok(hipEventRecord(B.k1, S.stream), "hipEventRecord") &&
             pl.ok(hipMemcpyAsync(B.h_rec, B.d_rec, n * sizeof(gpk_record), hipMemcpyDeviceToHost, S.stream), "DtoH") &&
             pl.ok(hipMemcpyAsync(B.h_err, B.d_err, n * 8, hipMemcpyDeviceToHost, S.stream), "DtoH") &&
             pl.ok(hipMemcpyAsync(B.h_flow, B.d_flow, n * 24, hipMemcpyDeviceToHost, S.stream), "DtoH");
      if (B.with_fields)
        good = good && pl.ok(hipMemcpyAsync(B.h_fields, B.d_fields, n * sizeof(gpk_fields), hipMemcpyDeviceToHost,
                                            S.stream), "DtoH fields");
      if (dwalk && pl.packets_cb)  // the device walk's offsets, for the packets' bytes on the host
        good = good && pl.ok(hipMemcpyAsync(B.h_off, S.d_off + first, n * 8, hipMemcpyDeviceToHost, S.stream),
                             "DtoH offsets");
      if (dwalk)
        good = good &&
               pl.ok(hipMemcpyAsync(B.h_cap, S.d_cap + first, n * 4, hipMemcpyDeviceToHost, S.stream), "DtoH caplens") &&
               pl.ok(hipMemcpyAsync(B.h_ci, S.d_ci + first, n * sizeof(gpk_capture_info), hipMemcpyDeviceToHost,
                                    S.stream), "DtoH capture info");
      good = good && pl.ok(hipEventRecord(B.done, S.stream), "hipEventRecord");
      pl.inflight.push_back(b);
      packet_index += n;
      stats->batches++;
      first += n;
    }
    gpk_capindex_free(&xi);
    if (!eof && pl.packets_cb && good) fill_ahead(si + pl.slots.size());
    if (st == GPK_CAP_END) {
      int is_eof = 0, is_panic = 0;
      gpk_capreader_error(rd, stats->error, sizeof(stats->error), &is_eof, &is_panic);
      stats->reader_status = is_eof ? 0 : (is_panic ? 2 : 1);
      clean_eof = is_eof != 0;
      finished = true;
    }
    stats->slots++;
    if (trace && trace[0] == '2')
      fprintf(stderr, "gpk_replay slot %llu: read %.2f-%.2f ms, got %.2f (waited %.2f), walked %.2f, launched %.2f\n",
              (unsigned long long)si, (fl.t0 - t_loop) * 1e3, (fl.t1 - t_loop) * 1e3, (t_got - t_loop) * 1e3,
              (t_got - t_get) * 1e3, (t_walked - t_loop) * 1e3, (now_s() - t_loop) * 1e3);
    carry = S.host + pos;
    carry_len = start + len - pos;
    if (eof && !finished) {  // cannot happen: at the end of the stream the walker ends with an error
      snprintf(stats->error, sizeof(stats->error), "internal: record walk did not end at end of stream");
      rc = GPK_EINVAL;
      finished = true;
    }
  }
  const double t_tail = now_s();
  while (good && !pl.inflight.empty()) good = pl.deliver_oldest();
  const double t_delivered = now_s();
  for (auto& s : pl.slots)
    if (s.fill_pending) {
      s.fill.wait();
      s.fill_pending = false;
    }
  const double t_fills = now_s();
  stats->packets = pl.stopped ? pl.delivered : packet_index;
  if (pl.stopped && rc == GPK_OK) rc = GPK_STOPPED;
  // allocations the call did not reach: one that failed has cost the call
  // nothing (every packet was delivered), so the call succeeds and only the
  // buffers are not kept for the next one
  const bool keep = pl.settle().empty();
  if (trace && trace[0] == '2')
    fprintf(stderr, "gpk_replay tail: delivered %.2f ms, fills %.2f, settled %.2f (from the last launch)\n",
            (t_delivered - t_tail) * 1e3, (t_fills - t_tail) * 1e3, (now_s() - t_tail) * 1e3);
  stats->alloc_wait_s = pl.alloc_wait_ns.load() * 1e-9;
  stats->wall_s = now_s() - t_start;
  if (rg) {
    rg->clean = good && rc == GPK_OK && clean_eof && stats->stream_bytes == src.size ? 1 : 0;  // (not when stopped)
    // any change of the reader's state past the leading blocks (a section, an
    // interface, statistics, an option value the next block could reuse)
    rg->state_changed = gpk_capreader_mutations(rd) != hdr_mutations ? 1 : 0;
  }
  if (trace && trace[0] == '1')
    fprintf(stderr, "gpk_replay: setup %.4f s, loop %.4f s, %llu slots\n", t_loop - t_start, now_s() - t_loop,
            (unsigned long long)stats->slots);
  if (!good) {
    snprintf(stats->error, sizeof(stats->error), "%s", pl.herr.c_str());
    return rc ? rc : GPK_EHIP;
  }
  for (auto& s : pl.slots)
    if (s.stream) good = good && pl.ok(hipStreamSynchronize(s.stream), "hipStreamSynchronize");
  if (good && keep)  // idle buffers for the next call
    gpk_ctx_replay_put(ctx, new Cached{C, R, P, dev_walk, std::move(pl.slots), std::move(pl.bats)}, free_cached);
  return rc;
}

// The C entry points: no C++ exception crosses them (a thread or an allocation
// the host cannot provide ends the call with an error; the pipeline's
// destructors have waited for its streams and threads by then).
static int replay_entry(gpk_ctx* ctx, const gpk_parser* parser, const char* path, const gpk_replay_opts* o,
                        gpk_replay_cb cb, void* user, gpk_replay_stats* stats, gpk_replay_range* rg) {
  if (!ctx || !parser || !path || !stats) return GPK_EINVAL;
  memset(stats, 0, sizeof(*stats));
  try {
    // the context's device for the pipeline's buffers, streams and launches
    // (callbacks included); the caller's device is back on return
    gpk::DeviceScope dscope(gpk_ctx_device(ctx));
    if (dscope.err != hipSuccess) {
      snprintf(stats->error, sizeof(stats->error), "hipSetDevice: %s", hipGetErrorString(dscope.err));
      return GPK_EHIP;
    }
    return replay_file(ctx, parser, path, o, cb, user, stats, rg);
  } catch (const std::bad_alloc&) {
    snprintf(stats->error, sizeof(stats->error), "out of host memory");
    return GPK_ENOMEM;
  } catch (const std::exception& e) {
    snprintf(stats->error, sizeof(stats->error), "%s", e.what());
    return GPK_EHIP;
  }
}

extern "C" int gpk_replay_file(gpk_ctx* ctx, const gpk_parser* parser, const char* path, const gpk_replay_opts* o,
                               gpk_replay_cb cb, void* user, gpk_replay_stats* stats) {
  return replay_entry(ctx, parser, path, o, cb, user, stats, nullptr);
}

extern "C" int gpk_replay_file_range(gpk_ctx* ctx, const gpk_parser* parser, const char* path,
                                     gpk_replay_range* range, const gpk_replay_opts* o, gpk_replay_cb cb, void* user,
                                     gpk_replay_stats* stats) {
  if (!range) return GPK_EINVAL;
  range->header_end = range->sync_begin = range->sync_end = 0;
  range->clean = range->state_changed = 0;
  if (range->end && range->end < range->begin) return GPK_EINVAL;
  return replay_entry(ctx, parser, path, o, cb, user, stats, range);
}

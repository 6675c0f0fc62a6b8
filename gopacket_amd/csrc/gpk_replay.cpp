// gpk_replay.cpp — whole-capture replay through HBM (gpk_replay_file,
// include/gpk_capture.h): BASELINE config C5, the path that starts and ends in
// host memory.
//
// The reference loop this replaces (examples/pcapdump, gopacket_benchmark):
//   r, _ := pcapgo.NewNgReader(f, opts)            pcapgo/ngread.go:64-106
//   for { data, ci, err := r.ReadPacketData()      ngread.go:636-640
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
//     carried into the head of the next slot (a reserved carry region).
// Results are delivered in packet order through the callback.
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <deque>
#include <future>
#include <string>
#include <thread>
#include <vector>

#include "../../include/gpk_capture.h"

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Src {  // the capture byte stream: plain file (parallel pread) or gzip (zlib)
  int fd = -1;
  gzFile gz = nullptr;
  uint64_t size = 0, pos = 0;
  bool at_end = false;
  int threads = 8;

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
        uint64_t a = (uint64_t)t * per, e = std::min<uint64_t>(want, a + per);
        while (a < e) {
          ssize_t k = pread(fd, dst + a, e - a, (off_t)(base + a));
          if (k <= 0) break;
          a += (uint64_t)k;
          got[t] += (uint64_t)k;
        }
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

struct Slot {
  uint8_t* host = nullptr;  // [carry region | fresh bytes | 16 B slack], pinned
  uint8_t* dev = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t h2d = nullptr;  // the slot's HtoD finished: host buffer reusable
  bool h2d_pending = false;
  std::future<uint64_t> fill;  // async read of the fresh bytes
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
  hipEvent_t e0 = nullptr, k0 = nullptr, k1 = nullptr, done = nullptr;
  uint64_t first = 0, n = 0, flows_n = 0;
};

struct Pipeline {
  std::vector<Slot> slots;
  std::vector<Bat> bats;
  std::deque<int> free_bats, inflight;
  uint64_t P = 0;
  gpk_replay_cb cb = nullptr;
  void* user = nullptr;
  gpk_replay_stats* st = nullptr;
  std::string herr;

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
    if (cb) cb(user, B.first, B.n, B.h_rec, B.h_err, B.h_flow, B.h_ci, B.h_cap);
    st->deliver_s += now_s() - t;
    free_bats.push_back(b);
    return true;
  }

  int acquire() {
    while (free_bats.empty())
      if (!deliver_oldest()) return -1;
    int b = free_bats.front();
    free_bats.pop_front();
    return b;
  }

  ~Pipeline() {
    for (auto& s : slots) {
      if (s.fill_pending) s.fill.wait();
      if (s.stream) (void)hipStreamSynchronize(s.stream);
      if (s.host) (void)hipHostFree(s.host);
      if (s.dev) (void)hipFree(s.dev);
      if (s.h2d) (void)hipEventDestroy(s.h2d);
      if (s.stream) (void)hipStreamDestroy(s.stream);
    }
    for (auto& B : bats) {
      for (void* p : {(void*)B.h_off, (void*)B.h_cap, (void*)B.h_ci, (void*)B.h_rec, (void*)B.h_err,
                      (void*)B.h_flow})
        if (p) (void)hipHostFree(p);
      for (void* p : {(void*)B.d_off, (void*)B.d_cap, (void*)B.d_rec, (void*)B.d_err, (void*)B.d_flow})
        if (p) (void)hipFree(p);
      for (hipEvent_t e : {B.e0, B.k0, B.k1, B.done})
        if (e) (void)hipEventDestroy(e);
    }
  }
};

}  // namespace

extern "C" int gpk_replay_file(gpk_ctx* ctx, const gpk_parser* parser, const char* path, const gpk_replay_opts* o,
                               gpk_replay_cb cb, void* user, gpk_replay_stats* stats) {
  if (!ctx || !parser || !path || !stats) return GPK_EINVAL;
  memset(stats, 0, sizeof(*stats));
  const double t_start = now_s();
  gpk_replay_opts opt{0, 0, 256ull << 20, 4, 2ull << 20, 8};
  if (o) {
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
  if (mk >= 2 && magic[0] == 0x1f && magic[1] == 0x8b) {  // read.go:74-84, ngread.go:80-95
    if (src.size < 10) {  // gzip.NewReader: the header read hits EOF
      close(src.fd);
      snprintf(stats->error, sizeof(stats->error), "unexpected EOF");
      stats->reader_status = 1;
      return GPK_OK;
    }
    src.gz = gzdopen(dup(src.fd), "rb");
    if (!src.gz) {
      close(src.fd);
      return GPK_ENOMEM;
    }
    gzbuffer(src.gz, 1u << 20);
    if (gzread(src.gz, magic, 4) < 4) memset(magic, 0, 4);
    gzrewind(src.gz);
  }
  int format = opt.format;
  if (!format) {
    const uint32_t m = (uint32_t)magic[0] | (uint32_t)magic[1] << 8 | (uint32_t)magic[2] << 16 | (uint32_t)magic[3] << 24;
    format = m == 0x0A0D0D0Au ? GPK_CAP_PCAPNG : GPK_CAP_PCAP;
  }
  gpk_capreader* rd = nullptr;
  int rc = gpk_capreader_create(&rd, format, opt.ng_flags);
  if (rc) {
    if (src.gz) gzclose(src.gz);
    close(src.fd);
    return rc;
  }

  // ---- buffers ---------------------------------------------------------------
  const uint64_t R = opt.slot_bytes, C = opt.slot_bytes;  // fresh bytes, carry region
  Pipeline pl;
  pl.cb = cb;
  pl.user = user;
  pl.st = stats;
  pl.P = opt.batch_pkts;
  pl.slots.resize(opt.slots);
  pl.bats.resize(2 * opt.slots);
  bool good = true;
  for (auto& s : pl.slots) {
    good = good && pl.ok(hipHostMalloc((void**)&s.host, C + R + 16, hipHostMallocDefault), "hipHostMalloc slot") &&
           pl.ok(hipMalloc((void**)&s.dev, C + R + 16), "hipMalloc slot") &&
           pl.ok(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking), "hipStreamCreate") &&
           pl.ok(hipEventCreateWithFlags(&s.h2d, hipEventDisableTiming), "hipEventCreate");
    if (good) memset(s.host + C + R, 0, 16);
  }
  const uint64_t P = pl.P;
  for (size_t i = 0; good && i < pl.bats.size(); i++) {
    Bat& B = pl.bats[i];
    good = pl.ok(hipHostMalloc((void**)&B.h_off, P * 8, 0), "hipHostMalloc") &&
           pl.ok(hipHostMalloc((void**)&B.h_cap, P * 4, 0), "hipHostMalloc") &&
           pl.ok(hipHostMalloc((void**)&B.h_ci, P * sizeof(gpk_capture_info), 0), "hipHostMalloc") &&
           pl.ok(hipHostMalloc((void**)&B.h_rec, P * sizeof(gpk_record), 0), "hipHostMalloc") &&
           pl.ok(hipHostMalloc((void**)&B.h_err, P * 8, 0), "hipHostMalloc") &&
           pl.ok(hipHostMalloc((void**)&B.h_flow, P * 24, 0), "hipHostMalloc") &&
           pl.ok(hipMalloc((void**)&B.d_off, P * 8), "hipMalloc") && pl.ok(hipMalloc((void**)&B.d_cap, P * 4), "hipMalloc") &&
           pl.ok(hipMalloc((void**)&B.d_rec, P * sizeof(gpk_record)), "hipMalloc") &&
           pl.ok(hipMalloc((void**)&B.d_err, P * 8), "hipMalloc") && pl.ok(hipMalloc((void**)&B.d_flow, P * 24), "hipMalloc") &&
           pl.ok(hipEventCreate(&B.e0), "hipEventCreate") && pl.ok(hipEventCreate(&B.k0), "hipEventCreate") &&
           pl.ok(hipEventCreate(&B.k1), "hipEventCreate") && pl.ok(hipEventCreate(&B.done), "hipEventCreate");
    pl.free_bats.push_back((int)i);
  }
  if (!good) {
    gpk_capreader_destroy(rd);
    if (src.gz) gzclose(src.gz);
    close(src.fd);
    snprintf(stats->error, sizeof(stats->error), "%s", pl.herr.c_str());
    return GPK_ENOMEM;
  }

  auto start_fill = [&](Slot& s) {
    s.fill = std::async(std::launch::async, [&src, &s, C, R, stats] {
      double t = now_s();
      uint64_t k = src.read(s.host + C, R);
      stats->read_s += now_s() - t;
      return k;
    });
    s.fill_pending = true;
  };

  // ---- the loop --------------------------------------------------------------
  const uint8_t* carry = nullptr;
  uint64_t carry_len = 0, packet_index = 0;
  bool finished = false;
  rc = GPK_OK;
  start_fill(pl.slots[0]);
  for (uint64_t si = 0; !finished && good; si++) {
    Slot& S = pl.slots[si % pl.slots.size()];
    const uint64_t fresh = S.fill.get();  // reads are strictly sequential: one fill at a time
    S.fill_pending = false;
    const bool eof = src.at_end;
    if (carry_len > C) {  // a record longer than the carry region: not supported
      snprintf(stats->error, sizeof(stats->error), "capture record larger than the %llu-byte staging slot",
               (unsigned long long)C);
      rc = GPK_EUNSUPP;
      break;
    }
    const uint64_t start = C - carry_len, len = carry_len + fresh;
    if (carry_len) memmove(S.host + start, carry, carry_len);
    stats->stream_bytes += fresh;
    // prefetch the next slot once its previous HtoD is done
    Slot& N = pl.slots[(si + 1) % pl.slots.size()];
    if (!eof) {
      if (N.h2d_pending) {
        good = pl.ok(hipEventSynchronize(N.h2d), "hipEventSynchronize");
        N.h2d_pending = false;
      }
      if (good) start_fill(N);
    }
    // walk the records of [start, start+len) (parallel, gpk_capreader_index_all)
    gpk_capindex xi;
    uint64_t used = 0;
    double t_ix = now_s();
    // the walk is a dependent load per record: more chains than cores hide DRAM latency
    const int walk_threads = std::min(64, 4 * opt.read_threads);
    int st = gpk_capreader_index_all(rd, S.host + start, len, eof ? 1 : 0, walk_threads, &xi, &used);
    stats->index_s += now_s() - t_ix;
    if (st < 0) {
      rc = st;
      finished = true;
      break;
    }
    const uint64_t pos = start + used;
    bool copied = false;
    for (uint64_t first = 0; first < xi.n && good;) {  // batches of up to P packets
      const uint64_t n = std::min<uint64_t>(P, xi.n - first);
      const int b = pl.acquire();
      if (b < 0) {
        good = false;
        break;
      }
      Bat& B = pl.bats[b];
      memcpy(B.h_off, xi.offsets + first, n * 8);  // relative to the slot's device copy (start)
      memcpy(B.h_cap, xi.caplens + first, n * 4);
      memcpy(B.h_ci, xi.ci + first, n * sizeof(gpk_capture_info));
      if (!copied) {  // the whole slot, once, before its first kernel
        good = pl.ok(hipMemcpyAsync(S.dev, S.host + start, len + 16, hipMemcpyHostToDevice, S.stream), "HtoD slot") &&
               pl.ok(hipEventRecord(S.h2d, S.stream), "hipEventRecord");
        S.h2d_pending = true;
        copied = true;
      }
      B.first = packet_index;
      B.n = n;
      good = good && pl.ok(hipEventRecord(B.e0, S.stream), "hipEventRecord") &&
             pl.ok(hipMemcpyAsync(B.d_off, B.h_off, n * 8, hipMemcpyHostToDevice, S.stream), "HtoD offsets") &&
             pl.ok(hipMemcpyAsync(B.d_cap, B.h_cap, n * 4, hipMemcpyHostToDevice, S.stream), "HtoD caplens") &&
             pl.ok(hipMemsetAsync(B.d_err, 0, n * 8, S.stream), "hipMemsetAsync") &&
             pl.ok(hipEventRecord(B.k0, S.stream), "hipEventRecord");
      if (!good) {
        pl.free_bats.push_back(b);
        break;
      }
      // data_bytes: the batch's span in the slot as the mean-packet-size hint (gpk.h)
      gpk_batch db{S.dev, B.d_off, B.d_cap, n, n ? B.h_off[n - 1] + B.h_cap[n - 1] - B.h_off[0] : 0};
      gpk_results dr{B.d_rec, B.d_err, B.d_flow, nullptr};
      int drc = gpk_decode_batch(ctx, parser, &db, &dr, S.stream);
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
             pl.ok(hipMemcpyAsync(B.h_flow, B.d_flow, n * 24, hipMemcpyDeviceToHost, S.stream), "DtoH") &&
             pl.ok(hipEventRecord(B.done, S.stream), "hipEventRecord");
      pl.inflight.push_back(b);
      packet_index += n;
      stats->batches++;
      for (uint64_t i = 0; i < n; i++) stats->packet_bytes += B.h_cap[i];
      first += n;
    }
    gpk_capindex_free(&xi);
    if (st == GPK_CAP_END) {
      int is_eof = 0, is_panic = 0;
      gpk_capreader_error(rd, stats->error, sizeof(stats->error), &is_eof, &is_panic);
      stats->reader_status = is_eof ? 0 : (is_panic ? 2 : 1);
      finished = true;
    }
    stats->slots++;
    carry = S.host + pos;
    carry_len = start + len - pos;
    if (eof && !finished) {  // cannot happen: at the end of the stream the walker ends with an error
      snprintf(stats->error, sizeof(stats->error), "internal: record walk did not end at end of stream");
      rc = GPK_EINVAL;
      finished = true;
    }
  }
  while (good && !pl.inflight.empty()) good = pl.deliver_oldest();
  for (auto& s : pl.slots)
    if (s.fill_pending) {
      s.fill.wait();
      s.fill_pending = false;
    }
  stats->packets = packet_index;
  stats->wall_s = now_s() - t_start;
  gpk_capreader_destroy(rd);
  if (src.gz) gzclose(src.gz);
  close(src.fd);
  if (!good) {
    snprintf(stats->error, sizeof(stats->error), "%s", pl.herr.c_str());
    return rc ? rc : GPK_EHIP;
  }
  return rc;
}

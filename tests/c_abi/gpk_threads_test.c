/* The Go-shaped multi-GPU caller: one process, several OS threads, one
 * gpk_ctx + parser per thread (a DecodingLayerParser per goroutine,
 * doc.go:211-228; cgo runs goroutines on arbitrary OS threads), each thread
 * decoding its byte-balanced slice of one batch concurrently with the others.
 *
 *   gpk_threads_test <golden dir> <threads> <copies> <reps>
 *   gpk_threads_test replay <pcapng> <threads>
 *   (the replay mode also ends replays early with gpk_stop, from a callback and
 *   from another thread: a Go caller's break out of its ReadPacketData loop)
 *
 * The batch is <copies> shuffled copies of the golden packets of
 * tests/golden/c_abi (reference vectors, the reference's capture files,
 * fuzzed packets), packed back to back in pinned host memory. Thread t owns a
 * context on device t % ndev and runs, <reps> times and interleaved:
 *   - gpk_decode_batch_host over its slice (host buffers);
 *   - gpk_decode_batch over a device copy of its slice, on a stream of its own;
 *   - gpk_decode_batch_host over its slice through ONE context shared by all
 *     threads (the context lock serialises them).
 * Before its calls each thread makes device (t + 1) % ndev current, as a
 * caller that uses HIP itself would, and after every gpk_* call checks that
 * hipGetDevice still returns it (the library restores the caller's device).
 * At the end the slices' records, error arguments and flow hashes, put back
 * together in packet order, must equal one context's decode of the whole
 * batch bit for bit, and that decode must equal the committed oracle
 * expectations for every packet. Exit status 0 = every check passed. */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <hip/hip_runtime_api.h>

#include "gpk.h"
#include "gpk_capture.h"

static int failures = 0;
static pthread_mutex_t fail_mu = PTHREAD_MUTEX_INITIALIZER;
#define CHECK(c, ...)                                        \
  do {                                                       \
    if (!(c)) {                                              \
      pthread_mutex_lock(&fail_mu);                          \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);   \
      fprintf(stderr, __VA_ARGS__);                          \
      fprintf(stderr, "\n");                                 \
      failures++;                                            \
      pthread_mutex_unlock(&fail_mu);                        \
    }                                                        \
  } while (0)

static void* slurp(const char* dir, const char* name, size_t* len) {
  char path[4096];
  snprintf(path, sizeof(path), "%s/%s", dir, name);
  FILE* f = fopen(path, "rb");
  if (!f) {
    fprintf(stderr, "cannot open %s\n", path);
    exit(2);
  }
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  void* p = malloc((size_t)n + 1);
  if (fread(p, 1, (size_t)n, f) != (size_t)n) exit(2);
  fclose(f);
  *len = (size_t)n;
  return p;
}

static gpk_parser* make_parser(void) { /* the statsassembly decoders, every output */
  static const int dec[] = {GPK_DEC_ETHERNET, GPK_DEC_DOT1Q, GPK_DEC_IPV4, GPK_DEC_IPV6,
                            GPK_DEC_IPV6_EXT, GPK_DEC_TCP,   GPK_DEC_UDP,  GPK_DEC_PAYLOAD};
  gpk_parser* p = NULL;
  if (gpk_parser_create(&p, GPK_LT_ETHERNET) != GPK_OK) return NULL;
  for (int k = 0; k < 8; k++) gpk_parser_add_decoder(p, dec[k]);
  gpk_parser_set_outputs(p, GPK_OUT_ALL);
  return p;
}

/* One batch and its results (flows SoA: link[n], net[n], transport[n]). */
struct out {
  gpk_record* rec;
  uint32_t* err;
  uint64_t* fl;
};

static struct {
  const uint8_t* data;
  const uint64_t* off;
  const uint32_t* cap;
  uint64_t n;
  uint64_t* bounds; /* threads + 1 packet indices */
  int ndev, reps;
  gpk_ctx* shared;
  struct out host, dev, sh; /* each thread writes its slice's part */
} G;

/* shard.byte_balanced_bounds: cut k at the first packet whose preceding bytes
 * reach total*k/world, so every thread reads about the same number of bytes */
static void byte_balanced_bounds(const uint32_t* cap, uint64_t n, int world, uint64_t* bounds) {
  uint64_t total = 0;
  for (uint64_t i = 0; i < n; i++) total += cap[i];
  bounds[0] = 0;
  uint64_t i = 0, csum = 0;
  for (int k = 1; k < world; k++) {
    const uint64_t want = total * (uint64_t)k / (uint64_t)world;
    while (i < n && csum < want) csum += cap[i++];
    bounds[k] = i;
  }
  bounds[world] = n;
}

static void scatter(const struct out* dst, uint64_t n, uint64_t lo, uint64_t k, const gpk_record* rec,
                    const uint32_t* err, const uint64_t* fl) {
  memcpy(dst->rec + lo, rec, k * sizeof(gpk_record));
  memcpy(dst->err + 2 * lo, err, k * 8);
  for (int j = 0; j < 3; j++) memcpy(dst->fl + (size_t)j * n + lo, fl + (size_t)j * k, k * 8);
}

struct worker {
  int t;
  pthread_t th;
};

#define DEVCHK(own, what)                                                                        \
  do {                                                                                           \
    int d_ = -1;                                                                                 \
    CHECK(hipGetDevice(&d_) == hipSuccess && d_ == (own), "thread %d: current device %d after %s, " \
          "the caller had %d", t, d_, what, own);                                                \
  } while (0)

static void* run(void* arg) {
  const int t = ((struct worker*)arg)->t;
  const int dev = t % G.ndev, own = (t + 1) % G.ndev;
  const uint64_t lo = G.bounds[t], hi = G.bounds[t + 1], k = hi - lo;
  CHECK(hipSetDevice(own) == hipSuccess, "thread %d: hipSetDevice(%d)", t, own);
  gpk_ctx* ctx = NULL;
  int rc = gpk_ctx_create(&ctx, dev);
  CHECK(rc == GPK_OK, "thread %d: gpk_ctx_create(%d): %s %s", t, dev, gpk_strerror(rc), gpk_last_hip_error());
  DEVCHK(own, "gpk_ctx_create");
  gpk_parser* p = make_parser();
  if (!ctx || !p || !k) return NULL;
  /* the slice as a batch of its own: 16-byte-aligned base, offsets rebased */
  const uint64_t base = G.off[lo] & ~15ull, end = G.off[hi - 1] + G.cap[hi - 1], bytes = end - base;
  uint64_t* off = (uint64_t*)malloc(k * 8);
  for (uint64_t i = 0; i < k; i++) off[i] = G.off[lo + i] - base;
  gpk_record* rec = (gpk_record*)malloc(k * sizeof(gpk_record));
  uint32_t* err = (uint32_t*)malloc(k * 8);
  uint64_t* fl = (uint64_t*)malloc(k * 24);
  /* device copies on the context's device, and a stream of the thread's own */
  void *d_data = NULL, *d_off = NULL, *d_cap = NULL, *d_rec = NULL, *d_err = NULL, *d_fl = NULL;
  hipStream_t s = NULL;
  int ok = hipSetDevice(dev) == hipSuccess && hipMalloc(&d_data, bytes + 16) == hipSuccess &&
           hipMalloc(&d_off, k * 8) == hipSuccess && hipMalloc(&d_cap, k * 4) == hipSuccess &&
           hipMalloc(&d_rec, k * sizeof(gpk_record)) == hipSuccess && hipMalloc(&d_err, k * 8) == hipSuccess &&
           hipMalloc(&d_fl, k * 24) == hipSuccess && hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess &&
           hipMemset(d_data, 0, bytes + 16) == hipSuccess &&
           hipMemcpy(d_data, G.data + base, bytes, hipMemcpyHostToDevice) == hipSuccess &&
           hipMemcpy(d_off, off, k * 8, hipMemcpyHostToDevice) == hipSuccess &&
           hipMemcpy(d_cap, G.cap + lo, k * 4, hipMemcpyHostToDevice) == hipSuccess &&
           hipSetDevice(own) == hipSuccess;
  CHECK(ok, "thread %d: device buffers", t);
  const gpk_batch hb = {G.data + base, off, G.cap + lo, k, bytes};
  const gpk_batch db = {(const uint8_t*)d_data, (const uint64_t*)d_off, (const uint32_t*)d_cap, k, bytes};
  for (int r = 0; ok && r < G.reps; r++) {
    /* host buffers, own context */
    memset(err, 0, k * 8);
    gpk_results ho = {rec, err, fl, NULL};
    rc = gpk_decode_batch_host(ctx, p, &hb, &ho);
    CHECK(rc == GPK_OK, "thread %d: gpk_decode_batch_host: %s %s", t, gpk_strerror(rc), gpk_last_hip_error());
    DEVCHK(own, "gpk_decode_batch_host");
    if (r == G.reps - 1) scatter(&G.host, G.n, lo, k, rec, err, fl);
    /* device buffers, own context, own stream */
    CHECK(hipMemsetAsync(d_err, 0, k * 8, s) == hipSuccess, "memset");
    gpk_results dr = {(gpk_record*)d_rec, (uint32_t*)d_err, (uint64_t*)d_fl, NULL};
    rc = gpk_decode_batch(ctx, p, &db, &dr, s);
    CHECK(rc == GPK_OK, "thread %d: gpk_decode_batch: %s %s", t, gpk_strerror(rc), gpk_last_hip_error());
    DEVCHK(own, "gpk_decode_batch");
    ok = hipStreamSynchronize(s) == hipSuccess &&
         hipMemcpy(rec, d_rec, k * sizeof(gpk_record), hipMemcpyDeviceToHost) == hipSuccess &&
         hipMemcpy(err, d_err, k * 8, hipMemcpyDeviceToHost) == hipSuccess &&
         hipMemcpy(fl, d_fl, k * 24, hipMemcpyDeviceToHost) == hipSuccess;
    CHECK(ok, "thread %d: device results", t);
    if (r == G.reps - 1) scatter(&G.dev, G.n, lo, k, rec, err, fl);
    /* host buffers, the context every thread shares */
    memset(err, 0, k * 8);
    rc = gpk_decode_batch_host(G.shared, p, &hb, &ho);
    CHECK(rc == GPK_OK, "thread %d: shared gpk_decode_batch_host: %s %s", t, gpk_strerror(rc), gpk_last_hip_error());
    DEVCHK(own, "gpk_decode_batch_host (shared context)");
    if (r == G.reps - 1) scatter(&G.sh, G.n, lo, k, rec, err, fl);
  }
  if (s) (void)hipStreamDestroy(s);
  void* bufs[] = {d_data, d_off, d_cap, d_rec, d_err, d_fl};
  for (int j = 0; j < 6; j++)
    if (bufs[j]) (void)hipFree(bufs[j]);
  (void)hipSetDevice(own);
  gpk_parser_destroy(p);
  rc = gpk_ctx_destroy(ctx);
  DEVCHK(own, "gpk_ctx_destroy");
  free(off);
  free(rec);
  free(err);
  free(fl);
  return NULL;
}

static int alloc_out(struct out* o, uint64_t n) {
  o->rec = (gpk_record*)calloc(n, sizeof(gpk_record));
  o->err = (uint32_t*)calloc(n, 8);
  o->fl = (uint64_t*)calloc(n, 24);
  return o->rec && o->err && o->fl;
}

static int same(const struct out* a, const struct out* b, uint64_t n, const char* what) {
  int good = memcmp(a->rec, b->rec, n * sizeof(gpk_record)) == 0 && memcmp(a->err, b->err, n * 8) == 0 &&
             memcmp(a->fl, b->fl, n * 24) == 0;
  CHECK(good, "%s: results differ from one context's decode of the whole batch", what);
  return good;
}

/* ---- replay: one pcapng file, a thread (and context) per byte range -------- *
 * The Go shape of C5 on N GPUs in one process: goroutines each replaying their
 * range of one file (gpk_replay_file_range) on their own context at the same
 * time. The ranges' results, concatenated, must equal one context's
 * gpk_replay_file of the whole file: records, error arguments, flow hashes,
 * capture info, capture lengths; every range clean and unchanged (a synthetic
 * capture has no interface blocks past its header); the threads' devices kept. */
struct collected {
  gpk_record* rec;
  uint32_t* err;
  uint64_t* fl; /* per packet: link, network, transport */
  gpk_capture_info* ci;
  uint32_t* cap;
  uint64_t n, room;
};

static void grow(struct collected* c, uint64_t need) {
  if (need <= c->room) return;
  uint64_t r = c->room ? c->room : 4096;
  while (r < need) r *= 2;
  c->rec = (gpk_record*)realloc(c->rec, r * sizeof(gpk_record));
  c->err = (uint32_t*)realloc(c->err, r * 8);
  c->fl = (uint64_t*)realloc(c->fl, r * 24);
  c->ci = (gpk_capture_info*)realloc(c->ci, r * sizeof(gpk_capture_info));
  c->cap = (uint32_t*)realloc(c->cap, r * 4);
  c->room = r;
}

static void on_results(void* user, uint64_t first, uint64_t n, const gpk_record* rec, const uint32_t* err,
                       const uint64_t* flows, const gpk_capture_info* ci, const uint32_t* caplens) {
  struct collected* c = (struct collected*)user;
  CHECK(first == c->n, "results for packet %llu, expected %llu", (unsigned long long)first, (unsigned long long)c->n);
  grow(c, c->n + n);
  memcpy(c->rec + c->n, rec, n * sizeof(gpk_record));
  memcpy(c->err + 2 * c->n, err, n * 8);
  for (uint64_t i = 0; i < n; i++)
    for (int j = 0; j < 3; j++) c->fl[3 * (c->n + i) + j] = flows[(uint64_t)j * n + i];
  memcpy(c->ci + c->n, ci, n * sizeof(gpk_capture_info));
  memcpy(c->cap + c->n, caplens, n * 4);
  c->n += n;
}

static struct {
  const char* path;
  uint64_t size;
  int threads, ndev;
  struct collected* parts;
  gpk_replay_range* ranges;
  gpk_replay_stats* stats;
} R;

static void* replay_run(void* arg) {
  const int t = ((struct worker*)arg)->t;
  const int dev = t % R.ndev, own = (t + 1) % R.ndev;
  CHECK(hipSetDevice(own) == hipSuccess, "thread %d: hipSetDevice(%d)", t, own);
  gpk_ctx* ctx = NULL;
  int rc = gpk_ctx_create(&ctx, dev);
  CHECK(rc == GPK_OK, "thread %d: gpk_ctx_create: %s", t, gpk_strerror(rc));
  DEVCHK(own, "gpk_ctx_create");
  gpk_parser* p = make_parser();
  if (!ctx || !p) return NULL;
  gpk_replay_range* rg = &R.ranges[t];
  rg->begin = R.size * (uint64_t)t / (uint64_t)R.threads;
  rg->end = t == R.threads - 1 ? 0 : R.size * (uint64_t)(t + 1) / (uint64_t)R.threads;
  gpk_replay_opts o;
  memset(&o, 0, sizeof(o));
  o.slot_bytes = 8u << 20; /* small slots: several per range */
  o.slots = 3;
  o.batch_pkts = 50000;
  rc = gpk_replay_file_range(ctx, p, R.path, rg, &o, on_results, &R.parts[t], &R.stats[t]);
  CHECK(rc == GPK_OK, "thread %d: gpk_replay_file_range: %s %s", t, gpk_strerror(rc), R.stats[t].error);
  DEVCHK(own, "gpk_replay_file_range");
  gpk_parser_destroy(p);
  gpk_ctx_destroy(ctx);
  DEVCHK(own, "gpk_ctx_destroy");
  return NULL;
}

/* ---- gpk_stop: a replay ended early ---------------------------------------- */
struct stopper {
  gpk_ctx* ctx;
  struct collected got;
  int batches, stop_after, sleep_us;
  volatile int started;
};

static void on_results_stop(void* user, uint64_t first, uint64_t n, const gpk_record* rec, const uint32_t* err,
                            const uint64_t* flows, const gpk_capture_info* ci, const uint32_t* caplens) {
  struct stopper* s = (struct stopper*)user;
  on_results(&s->got, first, n, rec, err, flows, ci, caplens);
  s->batches++;
  __atomic_store_n(&s->started, 1, __ATOMIC_SEQ_CST);
  if (s->batches == s->stop_after) CHECK(gpk_stop(s->ctx) == GPK_OK, "gpk_stop");
  if (s->sleep_us) {
    struct timespec ts = {0, (long)s->sleep_us * 1000};
    nanosleep(&ts, NULL);
  }
}

static struct {
  struct stopper* s;
  gpk_parser* p;
  const char* path;
  int rc;
  gpk_replay_stats st;
} SR;

static void* stop_run(void* arg) {
  (void)arg;
  gpk_replay_opts o;
  memset(&o, 0, sizeof(o));
  o.slot_bytes = 4u << 20;
  o.slots = 3;
  o.batch_pkts = 2000;
  SR.rc = gpk_replay_file(SR.s->ctx, SR.p, SR.path, &o, on_results_stop, SR.s, &SR.st);
  return NULL;
}

static int prefix_equal(const struct collected* a, const struct collected* whole) {
  for (uint64_t i = 0; i < a->n; i++)
    if (i >= whole->n || memcmp(&a->rec[i], &whole->rec[i], sizeof(gpk_record)) != 0 ||
        memcmp(&a->fl[3 * i], &whole->fl[3 * i], 24) != 0 || memcmp(&a->ci[i], &whole->ci[i], sizeof(gpk_capture_info)) != 0)
      return 0;
  return 1;
}

static void stop_checks(gpk_ctx* ctx, gpk_parser* p, const char* path, const struct collected* whole) {
  /* from inside the second batch's callback */
  struct stopper a;
  memset(&a, 0, sizeof(a));
  a.ctx = ctx;
  a.stop_after = 2;
  gpk_replay_opts o;
  memset(&o, 0, sizeof(o));
  o.slot_bytes = 4u << 20;
  o.slots = 3;
  o.batch_pkts = 1000;
  gpk_replay_stats st;
  int rc = gpk_replay_file(ctx, p, path, &o, on_results_stop, &a, &st);
  CHECK(rc == GPK_STOPPED && a.batches == 2 && a.got.n == 2000 && st.packets == 2000,
        "stop in a callback: %s, %d batches, %llu packets delivered, stats %llu", gpk_strerror(rc), a.batches,
        (unsigned long long)a.got.n, (unsigned long long)st.packets);
  CHECK(prefix_equal(&a.got, whole), "stop in a callback: results differ from the whole replay's");
  /* from another thread, while the replay runs */
  struct stopper b;
  memset(&b, 0, sizeof(b));
  b.ctx = ctx;
  b.sleep_us = 20000;
  SR.s = &b;
  SR.p = p;
  SR.path = path;
  pthread_t th;
  if (pthread_create(&th, NULL, stop_run, NULL)) {
    CHECK(0, "pthread_create");
    return;
  }
  while (!__atomic_load_n(&b.started, __ATOMIC_SEQ_CST)) {
    struct timespec ts = {0, 100000};
    nanosleep(&ts, NULL);
  }
  CHECK(gpk_stop(ctx) == GPK_OK, "gpk_stop from another thread");
  pthread_join(th, NULL);
  CHECK(SR.rc == GPK_STOPPED && b.got.n == SR.st.packets && b.got.n < whole->n,
        "stop from another thread: %s, %llu delivered, stats %llu, whole %llu", gpk_strerror(SR.rc),
        (unsigned long long)b.got.n, (unsigned long long)SR.st.packets, (unsigned long long)whole->n);
  CHECK(prefix_equal(&b.got, whole), "stop from another thread: results differ from the whole replay's");
  /* the next call runs to the end */
  struct collected c;
  memset(&c, 0, sizeof(c));
  rc = gpk_replay_file(ctx, p, path, &o, on_results, &c, &st);
  CHECK(rc == GPK_OK && c.n == whole->n && prefix_equal(&c, whole), "replay after a stop: %s, %llu of %llu",
        gpk_strerror(rc), (unsigned long long)c.n, (unsigned long long)whole->n);
  printf("stop: in a callback after 2 of %llu batches, from another thread after %llu packets, then whole again\n",
         (unsigned long long)((whole->n + 999) / 1000), (unsigned long long)b.got.n);
}

static int replay_main(const char* path, int T) {
  if (hipGetDeviceCount(&R.ndev) != hipSuccess || R.ndev < 1) return 2;
  FILE* f = fopen(path, "rb");
  if (!f) return 2;
  fseek(f, 0, SEEK_END);
  R.size = (uint64_t)ftell(f);
  fclose(f);
  R.path = path;
  R.threads = T;
  R.parts = (struct collected*)calloc(T, sizeof(struct collected));
  R.ranges = (gpk_replay_range*)calloc(T, sizeof(gpk_replay_range));
  R.stats = (gpk_replay_stats*)calloc(T, sizeof(gpk_replay_stats));
  /* one context, the whole file */
  struct collected whole;
  memset(&whole, 0, sizeof(whole));
  gpk_ctx* ctx = NULL;
  if (gpk_ctx_create(&ctx, 0) != GPK_OK) return 2;
  gpk_parser* p = make_parser();
  gpk_replay_opts o;
  memset(&o, 0, sizeof(o));
  gpk_replay_stats st;
  int rc = gpk_replay_file(ctx, p, path, &o, on_results, &whole, &st);
  CHECK(rc == GPK_OK && strcmp(st.error, "EOF") == 0, "whole replay: %s %s", gpk_strerror(rc), st.error);
  stop_checks(ctx, p, path, &whole);
  /* the ranges, a thread and context each, at once */
  struct worker* w = (struct worker*)calloc(T, sizeof(*w));
  for (int t = 0; t < T; t++) {
    w[t].t = t;
    if (pthread_create(&w[t].th, NULL, replay_run, &w[t])) return 2;
  }
  for (int t = 0; t < T; t++) pthread_join(w[t].th, NULL);
  uint64_t total = 0, bad = 0;
  for (int t = 0; t < T; t++) {
    const gpk_replay_range* g = &R.ranges[t];
    CHECK(g->clean && !g->state_changed, "range %d not exact: clean %d state_changed %d", t, g->clean,
          g->state_changed);
    CHECK(t == 0 || g->sync_begin == R.ranges[t - 1].sync_end, "range %d does not start where %d ended", t, t - 1);
    const struct collected* c = &R.parts[t];
    for (uint64_t i = 0; i < c->n && total + i < whole.n; i++) {
      const uint64_t k = total + i;
      int good = memcmp(&c->rec[i], &whole.rec[k], sizeof(gpk_record)) == 0 &&
                 memcmp(&c->fl[3 * i], &whole.fl[3 * k], 24) == 0 &&
                 memcmp(&c->ci[i], &whole.ci[k], sizeof(gpk_capture_info)) == 0 && c->cap[i] == whole.cap[k];
      if (good && gpk_record_err(&c->rec[i])) good = memcmp(&c->err[2 * i], &whole.err[2 * k], 8) == 0;
      if (!good && bad++ < 5) CHECK(0, "range %d packet %llu differs from the whole replay", t, (unsigned long long)i);
    }
    total += c->n;
  }
  CHECK(total == whole.n, "%llu packets across ranges, %llu in the whole replay", (unsigned long long)total,
        (unsigned long long)whole.n);
  printf("replay: %d ranges on %d device(s) at once, packets", T, R.ndev);
  for (int t = 0; t < T; t++) printf(" %llu", (unsigned long long)R.parts[t].n);
  printf(" = %llu of %llu, %s\n", (unsigned long long)total, (unsigned long long)whole.n,
         bad || total != whole.n ? "DIFFER" : "bit-exact");
  gpk_parser_destroy(p);
  gpk_ctx_destroy(ctx);
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("gpk C ABI: all checks passed (threads replay)\n");
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 4 && strcmp(argv[1], "replay") == 0) return replay_main(argv[2], atoi(argv[3]));
  if (argc < 5) {
    fprintf(stderr, "usage: %s <golden dir> <threads> <copies> <reps>\n", argv[0]);
    return 2;
  }
  const char* dir = argv[1];
  const int T = atoi(argv[2]), copies = atoi(argv[3]);
  G.reps = atoi(argv[4]);
  if (T < 1 || T > 64 || copies < 1 || G.reps < 1) return 2;
  if (hipGetDeviceCount(&G.ndev) != hipSuccess || G.ndev < 1) {
    fprintf(stderr, "no device\n");
    return 2;
  }
  size_t plen, elen;
  uint8_t* pk = (uint8_t*)slurp(dir, "packets.bin", &plen);
  uint8_t* ex = (uint8_t*)slurp(dir, "expect.bin", &elen);
  uint32_t m;
  memcpy(&m, pk, 4);
  CHECK(elen == 2 * (size_t)m * 48, "expect.bin size %zu", elen);
  /* the golden packets' positions in packets.bin */
  size_t* at = (size_t*)malloc(m * sizeof(size_t));
  uint32_t* len = (uint32_t*)malloc(m * 4);
  size_t pos = 4, gbytes = 0;
  for (uint32_t i = 0; i < m; i++) {
    memcpy(&len[i], pk + pos, 4);
    at[i] = pos + 4;
    pos += 4 + len[i];
    gbytes += len[i];
  }
  /* copies x the golden packets, each copy in its own (LCG) shuffled order */
  const uint64_t n = (uint64_t)m * (uint64_t)copies, total = (uint64_t)gbytes * (uint64_t)copies;
  uint8_t* data;
  uint64_t* off;
  uint32_t* cap;
  uint32_t* src = (uint32_t*)malloc(n * 4);
  if (gpk_host_alloc((void**)&data, total + 64) || gpk_host_alloc((void**)&off, n * 8) ||
      gpk_host_alloc((void**)&cap, n * 4)) {
    fprintf(stderr, "gpk_host_alloc: %s\n", gpk_last_hip_error());
    return 2;
  }
  memset(data + total, 0, 64);
  uint32_t* perm = (uint32_t*)malloc(m * 4);
  uint64_t lcg = 0x9E3779B97F4A7C15ull, o = 0, i = 0;
  for (int c = 0; c < copies; c++) {
    for (uint32_t j = 0; j < m; j++) perm[j] = j;
    for (uint32_t j = m - 1; j > 0; j--) {
      lcg = lcg * 6364136223846793005ull + 1442695040888963407ull;
      const uint32_t r = (uint32_t)((lcg >> 33) % (j + 1)), x = perm[j];
      perm[j] = perm[r];
      perm[r] = x;
    }
    for (uint32_t j = 0; j < m; j++, i++) {
      src[i] = perm[j];
      cap[i] = len[perm[j]];
      off[i] = o;
      memcpy(data + o, pk + at[perm[j]], cap[i]);
      o += cap[i];
    }
  }
  G.data = data;
  G.off = off;
  G.cap = cap;
  G.n = n;
  /* one context, the whole batch */
  struct out ref;
  if (!alloc_out(&ref, n) || !alloc_out(&G.host, n) || !alloc_out(&G.dev, n) || !alloc_out(&G.sh, n)) return 2;
  gpk_ctx* ctx = NULL;
  int rc = gpk_ctx_create(&ctx, 0);
  if (rc) {
    fprintf(stderr, "gpk_ctx_create: %s %s\n", gpk_strerror(rc), gpk_last_hip_error());
    return 2;
  }
  gpk_parser* p = make_parser();
  const gpk_batch b = {data, off, cap, n, total};
  gpk_results r = {ref.rec, ref.err, ref.fl, NULL};
  rc = gpk_decode_batch_host(ctx, p, &b, &r);
  CHECK(rc == GPK_OK, "whole-batch decode: %s %s", gpk_strerror(rc), gpk_last_hip_error());
  /* ... equals the oracle's expectations (cfg 0 of expect.bin) for every packet */
  const gpk_record* erec = (const gpk_record*)ex;
  const uint32_t* eerr = (const uint32_t*)(ex + 16 * (size_t)m);
  const uint64_t* efl = (const uint64_t*)(ex + 24 * (size_t)m);
  uint64_t bad = 0;
  for (i = 0; i < n; i++) {
    const uint32_t s = src[i];
    int good = memcmp(&ref.rec[i], &erec[s], 16) == 0;
    if (good && gpk_record_err(&ref.rec[i]))
      good = ref.err[2 * i] == eerr[2 * s] && ref.err[2 * i + 1] == eerr[2 * s + 1];
    for (int j = 0; j < 3 && good; j++) good = ref.fl[(size_t)j * n + i] == efl[(size_t)j * m + s];
    if (!good && bad++ < 5) CHECK(0, "packet %llu (golden %u) differs from the oracle", (unsigned long long)i, s);
  }
  printf("whole batch: %llu packets (%d x %u golden), %llu differ from the oracle\n", (unsigned long long)n, copies,
         m, (unsigned long long)bad);
  /* the threads */
  rc = gpk_ctx_create(&G.shared, 0);
  CHECK(rc == GPK_OK, "shared context");
  G.bounds = (uint64_t*)malloc((T + 1) * 8);
  byte_balanced_bounds(cap, n, T, G.bounds);
  struct worker* w = (struct worker*)calloc(T, sizeof(*w));
  for (int t = 0; t < T; t++) {
    w[t].t = t;
    if (pthread_create(&w[t].th, NULL, run, &w[t])) {
      fprintf(stderr, "pthread_create\n");
      return 2;
    }
  }
  for (int t = 0; t < T; t++) pthread_join(w[t].th, NULL);
  const int h = same(&G.host, &ref, n, "host buffers, a context per thread");
  const int d = same(&G.dev, &ref, n, "device buffers, a context and stream per thread");
  const int s = same(&G.sh, &ref, n, "host buffers, one context shared by the threads");
  printf("threads: %d contexts on %d device(s), %d reps, slices", T, G.ndev, G.reps);
  for (int t = 0; t < T; t++) printf(" %llu", (unsigned long long)(G.bounds[t + 1] - G.bounds[t]));
  printf("; per-thread host %s, device %s, shared %s\n", h ? "bit-exact" : "DIFFER", d ? "bit-exact" : "DIFFER",
         s ? "bit-exact" : "DIFFER");
  gpk_ctx_destroy(G.shared);
  gpk_parser_destroy(p);
  gpk_ctx_destroy(ctx);
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("gpk C ABI: all checks passed (threads)\n");
  return 0;
}

/* A C-language caller of the drop-in boundary, the way the cgo package in
 * INTEGRATION.md uses it: only include/gpk.h, linked with -lgpk.
 *
 *   gpk_abi_test host <golden dir>     no GPU: struct layouts, error texts,
 *                                      LayerType names, code mapping
 *   gpk_abi_test decode <golden dir>   decodes the golden packets with
 *                                      gpk_decode_batch_host under two parser
 *                                      configurations and compares records,
 *                                      error arguments, flow hashes and the
 *                                      Go error text with the committed
 *                                      expectations (tools/make_c_abi_golden.py)
 * Exit status 0 = every check passed. */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gpk.h"
#include "gpk_capture.h"

/* the layouts cgo sees (INTEGRATION.md's Go structs mirror these offsets) */
_Static_assert(sizeof(gpk_record) == 16, "gpk_record is 16 bytes");
_Static_assert(offsetof(gpk_record, status) == 8, "status at 8");
_Static_assert(offsetof(gpk_record, ip4_csum) == 12, "ip4_csum at 12");
_Static_assert(offsetof(gpk_record, l4_csum) == 14, "l4_csum at 14");
_Static_assert(sizeof(gpk_layout) == 64, "gpk_layout is 64 bytes");
_Static_assert(sizeof(gpk_record8) == 8 && offsetof(gpk_record8, status) == 4, "gpk_record8 is 8 bytes");
_Static_assert(sizeof(gpk_results8) == 32 && offsetof(gpk_results8, wide) == 8, "gpk_results8 is 4 pointers");
_Static_assert(sizeof(gpk_replay_range) == 48 && offsetof(gpk_replay_range, clean) == 40,
               "gpk_replay_range: 5 words, then clean and state_changed");
_Static_assert(sizeof(gpk_batch) == 40, "gpk_batch is 5 words");
_Static_assert(sizeof(gpk_results) == 32, "gpk_results is 4 pointers");
_Static_assert(sizeof(gpk_fields) == 128, "gpk_fields is 128 bytes");
_Static_assert(offsetof(gpk_fields, present) == 0 && sizeof(((gpk_fields*)0)->present) == 1 &&
                   offsetof(gpk_fields, hbh_opt_map) == 1,
               "gpk_fields presence byte and HopByHop option map (ABI 2)");
_Static_assert(offsetof(gpk_fields, eth_dst) == 8 && offsetof(gpk_fields, d1q_tci) == 20, "gpk_fields link part");
_Static_assert(offsetof(gpk_fields, ip4_length) == 28 && offsetof(gpk_fields, ip6_flow_label) == 40 &&
                   offsetof(gpk_fields, ip4_src) == 48 && offsetof(gpk_fields, ip6_dst) == 72,
               "gpk_fields network part");
_Static_assert(offsetof(gpk_fields, tcp_seq) == 92 && offsetof(gpk_fields, tcp_flags) == 100 &&
                   offsetof(gpk_fields, udp_checksum) == 114,
               "gpk_fields transport part");

static int failures = 0;
#define CHECK(c, ...)                            \
  do {                                           \
    if (!(c)) {                                  \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);              \
      fprintf(stderr, "\n");                     \
      failures++;                                \
    }                                            \
  } while (0)

static int code_slot(unsigned code);

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
  ((char*)p)[n] = 0;
  *len = (size_t)n;
  return p;
}

static void host_checks(void) {
  char buf[256];
  CHECK(gpk_abi_version() == GPK_ABI_VERSION, "abi version %d", gpk_abi_version());
  /* parser.go:325-327 and layer names (layertype.go:101-111) */
  gpk_format_error(GPK_ERR_UNSUPPORTED, GPK_LT_PAYLOAD, 0, buf, sizeof(buf));
  CHECK(strcmp(buf, "No decoder for layer type Payload") == 0, "[%s]", buf);
  gpk_format_error(GPK_ERR_UNSUPPORTED, 107, 0, buf, sizeof(buf));
  CHECK(strcmp(buf, "No decoder for layer type DNS") == 0, "[%s]", buf);
  /* tcp_test.go:173-188: "MPTCP bad option length 0" */
  gpk_format_error(GPK_ERR_MPTCP_LEN, 0, 0, buf, sizeof(buf));
  CHECK(strcmp(buf, "MPTCP bad option length 0") == 0, "[%s]", buf);
  /* ip4_test.go:102-113 */
  gpk_format_error(GPK_ERR_IP4_OPT_BADLEN, 131, 2, buf, sizeof(buf));
  CHECK(strcmp(buf, "Invalid IP option type 131 length 2. Must be greater than 2") == 0, "[%s]", buf);
  /* panicToError parser.go:329-333 */
  gpk_format_error(GPK_ERR_PANIC_INDEX, 3, 3, buf, sizeof(buf));
  CHECK(strcmp(buf, "panic: runtime error: index out of range [3] with length 3") == 0, "[%s]", buf);
  /* truncation to cap: NUL-terminated, full length returned */
  char small[8];
  int n = gpk_format_error(GPK_ERR_ETH_TOO_SMALL, 0, 0, small, sizeof(small));
  CHECK(n == (int)strlen("Ethernet packet too small") && strlen(small) == 7, "truncation n=%d [%s]", n, small);
  gpk_layer_type_name(GPK_LT_ETHERNET, buf, sizeof(buf));
  CHECK(strcmp(buf, "Ethernet") == 0, "[%s]", buf);
  gpk_layer_type_name(12345, buf, sizeof(buf));
  CHECK(strcmp(buf, "12345") == 0, "[%s]", buf);
  CHECK(gpk_code_layer_type(GPK_CODE_TCP) == GPK_LT_TCP, "code map");
  CHECK(gpk_code_layer_type(GPK_CODE_FRAGMENT) == GPK_LT_FRAGMENT, "code map");
  CHECK(gpk_code_layer_type(13) == -1, "code map bound");
  CHECK(strcmp(gpk_strerror(GPK_EINVAL), "invalid argument") == 0, "strerror");
  /* parser configuration needs no device */
  gpk_parser* p = NULL;
  CHECK(gpk_parser_create(&p, GPK_LT_ETHERNET) == GPK_OK && p, "parser_create");
  CHECK(gpk_parser_add_decoder(p, GPK_DEC_TCP) == GPK_OK, "add TCP");
  CHECK(gpk_parser_decoder_for(p, GPK_LT_TCP) == GPK_DEC_TCP, "decoder_for");
  CHECK(gpk_parser_add_decoder(p, 99) == GPK_EUNSUPP, "unknown decoder kind");
  CHECK(gpk_parser_set_outputs(p, 0x8) == GPK_EINVAL, "bad outputs");
  CHECK(gpk_parser_set_tcp_port(p, 70000, 2) == GPK_EINVAL, "port range");
  gpk_parser_destroy(p);
}

static gpk_parser* make_parser(int cfg) {
  static const int stats[] = {GPK_DEC_ETHERNET, GPK_DEC_DOT1Q, GPK_DEC_IPV4, GPK_DEC_IPV6,
                              GPK_DEC_IPV6_EXT, GPK_DEC_TCP,   GPK_DEC_UDP,  GPK_DEC_PAYLOAD};
  static const int simple[] = {GPK_DEC_ETHERNET, GPK_DEC_IPV4, GPK_DEC_TCP, GPK_DEC_PAYLOAD};
  gpk_parser* p = NULL;
  if (gpk_parser_create(&p, GPK_LT_ETHERNET) != GPK_OK) return NULL;
  const int* d = cfg == 0 ? stats : simple;
  int nd = cfg == 0 ? 8 : 4;
  for (int k = 0; k < nd; k++) gpk_parser_add_decoder(p, d[k]);
  gpk_parser_set_outputs(p, GPK_OUT_ALL);
  return p;
}

static int decode_checks(const char* dir) {
  size_t plen, elen, tlen;
  uint8_t* pk = (uint8_t*)slurp(dir, "packets.bin", &plen);
  uint8_t* ex = (uint8_t*)slurp(dir, "expect.bin", &elen);
  char* txt = (char*)slurp(dir, "errors.txt", &tlen);
  uint32_t n;
  memcpy(&n, pk, 4);
  /* pack contiguously into pinned memory, as a capture source would */
  size_t pos = 4, total = 0;
  for (uint32_t i = 0; i < n; i++) {
    uint32_t c;
    memcpy(&c, pk + pos, 4);
    pos += 4 + c;
    total += c;
  }
  uint8_t* data;
  uint64_t* off;
  uint32_t* cap;
  gpk_record* rec;
  uint32_t* err;
  uint64_t* fl;
  if (gpk_host_alloc((void**)&data, total + 64) || gpk_host_alloc((void**)&off, 8 * (size_t)n) ||
      gpk_host_alloc((void**)&cap, 4 * (size_t)n) || gpk_host_alloc((void**)&rec, 16 * (size_t)n) ||
      gpk_host_alloc((void**)&err, 8 * (size_t)n) || gpk_host_alloc((void**)&fl, 24 * (size_t)n)) {
    fprintf(stderr, "gpk_host_alloc: %s\n", gpk_last_hip_error());
    return 2;
  }
  memset(data, 0, total + 64);
  pos = 4;
  size_t o = 0;
  for (uint32_t i = 0; i < n; i++) {
    memcpy(&cap[i], pk + pos, 4);
    memcpy(data + o, pk + pos + 4, cap[i]);
    off[i] = o;
    o += cap[i];
    pos += 4 + cap[i];
  }
  gpk_ctx* ctx = NULL;
  int rc = gpk_ctx_create(&ctx, 0);
  if (rc) {
    fprintf(stderr, "gpk_ctx_create: %s %s\n", gpk_strerror(rc), gpk_last_hip_error());
    return 2;
  }
  const char* names[2] = {"statsassembly", "eth_ip4_tcp_payload"};
  const size_t per = (size_t)n * (16 + 8 + 24);
  CHECK(elen == 2 * per, "expect.bin size %zu", elen);
  for (int cfg = 0; cfg < 2; cfg++) {
    gpk_parser* p = make_parser(cfg);
    gpk_batch b = {data, off, cap, n, total};
    memset(err, 0, 8 * (size_t)n);
    gpk_results r = {rec, err, fl, NULL};
    rc = gpk_decode_batch_host(ctx, p, &b, &r);
    CHECK(rc == GPK_OK, "decode %s: %s %s", names[cfg], gpk_strerror(rc), gpk_last_hip_error());
    const uint8_t* e = ex + cfg * per;
    int bad = 0;
    for (uint32_t i = 0; i < n && bad < 5; i++) {
      if (memcmp(&rec[i], e + 16 * (size_t)i, 16) != 0) {
        CHECK(0, "%s packet %u: record differs", names[cfg], i);
        bad++;
        continue;
      }
      const uint32_t* ea = (const uint32_t*)(e + 16 * (size_t)n) + 2 * (size_t)i;
      if (gpk_record_err(&rec[i]) && (err[2 * i] != ea[0] || err[2 * i + 1] != ea[1])) {
        CHECK(0, "%s packet %u: err_args differ", names[cfg], i);
        bad++;
      }
    }
    CHECK(memcmp(fl, e + 24 * (size_t)n, 24 * (size_t)n) == 0, "%s: flow hashes differ", names[cfg]);
    /* the Go error text of every packet that failed */
    char want_prefix[64];
    snprintf(want_prefix, sizeof(want_prefix), "%s ", names[cfg]);
    int texts = 0;
    for (char* line = txt; line && *line;) {
      char* nl = strchr(line, '\n');
      if (nl) *nl = 0;
      if (strncmp(line, want_prefix, strlen(want_prefix)) == 0) {
        char* q = line + strlen(want_prefix);
        uint32_t i = (uint32_t)strtoul(q, &q, 10);
        q++;
        char got[512];
        CHECK(i < n, "index");
        gpk_format_error(gpk_record_err(&rec[i]), err[2 * i], err[2 * i + 1], got, sizeof(got));
        CHECK(strcmp(got, q) == 0, "%s packet %u: [%s] vs [%s]", names[cfg], i, got, q);
        texts++;
      }
      if (nl) *nl = '\n';
      line = nl ? nl + 1 : NULL;
    }
    /* the same batch with the layer fields (host buffers): the same records, and
       for every packet without error the decoders the fields mark present are
       the ones its decoded list names */
    gpk_fields* hf = (gpk_fields*)malloc(sizeof(gpk_fields) * (size_t)n);
    gpk_record* rec2 = (gpk_record*)malloc(16 * (size_t)n);
    uint64_t* fl2 = (uint64_t*)malloc(24 * (size_t)n);
    gpk_results r2 = {rec2, NULL, fl2, NULL};
    rc = gpk_decode_batch_host_fields(ctx, p, &b, &r2, hf);
    CHECK(rc == GPK_OK, "decode with fields %s: %s", names[cfg], gpk_strerror(rc));
    CHECK(memcmp(rec2, rec, 16 * (size_t)n) == 0, "%s: records differ with fields", names[cfg]);
    int present_checked = 0;
    for (uint32_t i = 0; i < n && rc == GPK_OK; i++) {
      const unsigned nl = gpk_record_nlayers(&rec[i]);
      if (gpk_record_err(&rec[i]) || nl > 16) continue;
      unsigned want = 0;
      for (unsigned k = 0; k < nl; k++) {
        const int sl = code_slot((unsigned)(rec[i].layers >> (4 * k)) & 0xF);
        if (sl >= 0) want |= 1u << sl;
      }
      CHECK(hf[i].present == want, "%s packet %u: present %#x, decoded %#x", names[cfg], i, hf[i].present, want);
      present_checked++;
    }
    free(hf);
    free(rec2);
    free(fl2);
    printf("%s: %u packets, %d error texts checked, %d fields records checked\n", names[cfg], n, texts,
           present_checked);
    gpk_parser_destroy(p);
  }
  gpk_ctx_destroy(ctx);
  gpk_host_free(data);
  gpk_host_free(off);
  gpk_host_free(cap);
  gpk_host_free(rec);
  gpk_host_free(err);
  gpk_host_free(fl);
  free(pk);
  free(ex);
  free(txt);
  return 0;
}

/* ---- replay: gpk_replay_file with the fields callback, from C ----------------
 * What a cgo caller of the C5 loop sees: results in packet order, each batch's
 * gpk_fields delivered right before its records for the same packets, and for
 * every packet decoded without error a record whose decoded list names exactly
 * the decoders the fields record marks present (gpk.h gpk_fields.present). */
struct replay_state {
  uint64_t next_first, fields_first, fields_n, packets, checked, bytes_checked;
  int have_fields;
  const uint8_t* raw;      /* the capture file and the reader's index of it, to */
  const gpk_capindex* x;   /* check the packets the replay hands out            */
  uint8_t* present; /* this batch's present bytes (fields valid during the callback only) */
  uint64_t cap;
};

static void on_fields(void* user, uint64_t first, uint64_t n, const gpk_fields* f) {
  struct replay_state* st = (struct replay_state*)user;
  if (n > st->cap) {
    free(st->present);
    st->present = (uint8_t*)malloc(n);
    st->cap = n;
  }
  for (uint64_t i = 0; i < n; i++) st->present[i] = f[i].present;
  st->fields_first = first;
  st->fields_n = n;
  st->have_fields = 1;
}

static void on_packets(void* user, uint64_t first, uint64_t n, const uint8_t* base, uint64_t bytes,
                       const uint64_t* offsets, const uint32_t* caplens) {
  struct replay_state* st = (struct replay_state*)user;
  for (uint64_t i = 0; i < n; i++) {
    const uint64_t k = first + i;
    CHECK(offsets[i] + caplens[i] <= bytes, "packet %llu outside the batch's bytes", (unsigned long long)k);
    if (k >= st->x->n) {
      CHECK(0, "packet %llu past the reader's %llu", (unsigned long long)k, (unsigned long long)st->x->n);
      return;
    }
    if (caplens[i] != st->x->caplens[k] || memcmp(base + offsets[i], st->raw + st->x->offsets[k], caplens[i]) != 0) {
      CHECK(0, "packet %llu: bytes differ from the reader's", (unsigned long long)k);
      return;
    }
    st->bytes_checked++;
  }
}

static int code_slot(unsigned code) { /* decoded-list code -> gpk_fields.present bit */
  switch (code) {
    case GPK_CODE_ETHERNET: return 0;
    case GPK_CODE_DOT1Q: return 1;
    case GPK_CODE_IPV4: return 2;
    case GPK_CODE_IPV6: return 3;
    case GPK_CODE_IPV6_HOPBYHOP:
    case GPK_CODE_IPV6_ROUTING:
    case GPK_CODE_IPV6_FRAGMENT:
    case GPK_CODE_IPV6_DESTINATION: return 4;
    case GPK_CODE_TCP: return 5;
    case GPK_CODE_UDP: return 6;
    case GPK_CODE_PAYLOAD:
    case GPK_CODE_FRAGMENT: return 7;
    default: return -1;
  }
}

static void on_results(void* user, uint64_t first, uint64_t n, const gpk_record* rec, const uint32_t* err,
                       const uint64_t* flows, const gpk_capture_info* ci, const uint32_t* caplens) {
  struct replay_state* st = (struct replay_state*)user;
  (void)err;
  (void)flows;
  (void)ci;
  (void)caplens;
  CHECK(first == st->next_first, "results for packet %llu, expected %llu", (unsigned long long)first,
        (unsigned long long)st->next_first);
  CHECK(st->have_fields && st->fields_first == first && st->fields_n == n, "fields not delivered before results");
  for (uint64_t i = 0; i < n && st->have_fields; i++) {
    const unsigned nl = gpk_record_nlayers(&rec[i]);
    if (gpk_record_err(&rec[i]) || nl > 16) continue;
    unsigned want = 0;
    for (unsigned k = 0; k < nl; k++) {
      const int sl = code_slot((unsigned)(rec[i].layers >> (4 * k)) & 0xF);
      if (sl >= 0) want |= 1u << sl;
    }
    CHECK(st->present[i] == want, "packet %llu: present %#x, decoded list %#x", (unsigned long long)(first + i),
          st->present[i], want);
    st->checked++;
  }
  st->have_fields = 0;
  st->next_first = first + n;
  st->packets += n;
}

static int replay_checks(int nfiles, char** files) {
  gpk_ctx* ctx = NULL;
  int rc = gpk_ctx_create(&ctx, 0);
  if (rc) {
    fprintf(stderr, "gpk_ctx_create: %s %s\n", gpk_strerror(rc), gpk_last_hip_error());
    return 2;
  }
  gpk_parser* p = make_parser(0);
  for (int f = 0; f < nfiles; f++) {
    /* the packets the capture holds, by the reader alone */
    size_t len = 0;
    uint8_t* raw = (uint8_t*)slurp(files[f][0] == '/' ? "" : ".", files[f], &len);
    const int fmt = len >= 4 && raw[0] == 0x0A && raw[1] == 0x0D && raw[2] == 0x0D && raw[3] == 0x0A ? GPK_CAP_PCAPNG
                                                                                                   : GPK_CAP_PCAP;
    gpk_capreader* r = NULL;
    gpk_capindex x = {0, NULL, NULL, NULL};
    uint64_t used = 0;
    CHECK(gpk_capreader_create(&r, fmt, 0) == GPK_OK, "capreader_create");
    CHECK(gpk_capreader_index_all(r, raw, len, 1, 4, &x, &used) >= 0, "index_all");
    gpk_capreader_destroy(r);
    /* the same file through the GPU, small slots and batches: many launches */
    struct replay_state st;
    memset(&st, 0, sizeof(st));
    gpk_replay_opts o;
    memset(&o, 0, sizeof(o));
    o.format = fmt;
    o.slot_bytes = 1 << 20;
    o.slots = 3;
    o.batch_pkts = 777;
    o.fields_cb = on_fields;
    o.packets_cb = on_packets;
    st.raw = raw;
    st.x = &x;
    gpk_replay_stats s;
    rc = gpk_replay_file(ctx, p, files[f], &o, on_results, &st, &s);
    CHECK(rc == GPK_OK, "replay %s: %s %s", files[f], gpk_strerror(rc), s.error);
    CHECK(st.packets == s.packets && s.packets == x.n, "%s: %llu delivered, stats %llu, reader %llu", files[f],
          (unsigned long long)st.packets, (unsigned long long)s.packets, (unsigned long long)x.n);
    CHECK(st.bytes_checked == x.n, "%s: %llu packets' bytes checked of %llu", files[f],
          (unsigned long long)st.bytes_checked, (unsigned long long)x.n);
    const char* base = strrchr(files[f], '/') ? strrchr(files[f], '/') + 1 : files[f];
    printf("replay %s: %llu packets, %llu checked against their fields\n", base,
           (unsigned long long)st.packets, (unsigned long long)st.checked);
    gpk_capindex_free(&x);
    free(st.present);
    free(raw);
  }
  gpk_parser_destroy(p);
  gpk_ctx_destroy(ctx);
  return 0;
}

/* ---- the capture reader's interface beyond ReadPacketData, from C ---------- *
 * What a cgo binding of pcapgo.NgReader does: index a file in one call, then
 * read the options of its packets (ReadPacketDataWithOptions), the name
 * records (Name / NNames) and the statistics callbacks. Pinned by the
 * reference's tests: ngread_test.go:2028-2100 (tests/epb.pcapng's options) and
 * ngread_nrb_test.go:50-79 (tests/le/test016.pcapng's name records). */
static unsigned char* slurp_file(const char* dir, const char* name, size_t* len) {
  char path[1024];
  snprintf(path, sizeof(path), "%s/%s", dir, name);
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  unsigned char* b = (unsigned char*)malloc((size_t)n + 1);
  if (fread(b, 1, (size_t)n, f) != (size_t)n) n = 0;
  fclose(f);
  *len = (size_t)n;
  return b;
}

static int capture_checks(const char* dir) {
  size_t len = 0;
  unsigned char* raw = slurp_file(dir, "epb.pcapng", &len);
  CHECK(raw && len > 0, "epb.pcapng");
  if (!raw) return 1;
  gpk_capreader* r = NULL;
  CHECK(gpk_capreader_create(&r, GPK_CAP_PCAPNG, 0) == GPK_OK, "create");
  CHECK(gpk_capreader_keep_options(r, 1) == GPK_OK, "keep_options");
  uint64_t off[8], n = 0, used = 0;
  uint32_t cap[8];
  int rc = gpk_capreader_index(r, raw, len, 1, off, cap, NULL, 8, &n, &used);
  CHECK(rc == GPK_CAP_END && n >= 1, "index epb.pcapng: %d, %llu packets", rc, (unsigned long long)n);
  const uint8_t* tlv = NULL;
  uint64_t nb = 0;
  CHECK(gpk_capreader_packet_options(r, 0, &tlv, &nb) == GPK_OK, "packet_options");
  /* the option codes in order: 2 comments, flags, 2 hashes, drop count, packet id, queue, 2 verdicts */
  const uint16_t want[] = {1, 1, 2, 3, 3, 4, 5, 6, 7, 7};
  int k = 0, good = 1;
  uint64_t packet_id = 0;
  for (uint64_t q = 0; q + 8 <= nb; k++) {
    uint16_t code;
    uint32_t olen;
    memcpy(&code, tlv + q, 2);
    memcpy(&olen, tlv + q + 4, 4);
    if (k >= 10 || code != want[k]) good = 0;
    if (code == 5 && olen >= 8) memcpy(&packet_id, tlv + q + 8, 8); /* little-endian, as the reference reads it */
    if (k == 0 && (olen != 17 || memcmp(tlv + q + 8, "this is a comment", 17) != 0)) good = 0;
    q += 8 + ((olen + 3u) & ~3u);
  }
  CHECK(good && k == 10, "epb.pcapng options: %d records", k);
  CHECK(packet_id == 0x1234567890abcdefull, "PacketID %llx", (unsigned long long)packet_id);
  gpk_capreader_destroy(r);
  free(raw);

  raw = slurp_file(dir, "le/test016.pcapng", &len);
  CHECK(raw && len > 0, "le/test016.pcapng");
  if (!raw) return 1;
  CHECK(gpk_capreader_create(&r, GPK_CAP_PCAPNG, GPK_NG_SKIP_UNKNOWN_VERSION) == GPK_OK, "create");
  /* read to io.EOF, past other errors (readNgNRB, ngread_nrb_test.go:11-47) */
  uint64_t pos = 0;
  for (int calls = 0; calls < 100; calls++) {
    rc = gpk_capreader_index(r, raw + pos, len - pos, 1, off, cap, NULL, 8, &n, &used);
    pos += used;
    int is_eof = 0;
    if (rc == GPK_CAP_END) {
      gpk_capreader_error(r, NULL, 0, &is_eof, NULL);
      if (is_eof) break;
    }
  }
  CHECK(gpk_capreader_nnames(r) == 10, "test016: %d name records", gpk_capreader_nnames(r));
  int kind = 0, alen = 0, nn = 0;
  uint8_t addr[24];
  char names[256];
  gpk_capreader_name(r, 2, &kind, addr, &alen, &nn, names, sizeof(names));
  CHECK(kind == 1 && alen == 4 && addr[0] == 10 && addr[1] == 1 && addr[2] == 2 && addr[3] == 3,
        "test016 record 2: kind %d, %d address bytes", kind, alen);
  gpk_capreader_name(r, 6, &kind, addr, &alen, &nn, names, sizeof(names));
  CHECK(nn >= 1 && strcmp(names, "qux.example.com") == 0, "test016 record 6: %s", names);
  gpk_capreader_destroy(r);
  free(raw);
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s host|decode <golden dir> | capture <pcapgo golden dir> | replay <capture>...\n", argv[0]);
    return 2;
  }
  host_checks();
  if (strcmp(argv[1], "decode") == 0) {
    int rc = decode_checks(argv[2]);
    if (rc) return rc;
  } else if (strcmp(argv[1], "replay") == 0) {
    int rc = replay_checks(argc - 2, argv + 2);
    if (rc) return rc;
  } else if (strcmp(argv[1], "capture") == 0) {
    int rc = capture_checks(argv[2]);
    if (rc) return rc;
  }
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("gpk C ABI: all checks passed (%s)\n", argv[1]);
  return 0;
}

// Host-side fuzz driver under AddressSanitizer + UBSan (test infrastructure).
//
// The two host parsers of untrusted input in libgpk — the pcap/pcapng capture
// reader (gpk_capture.cpp: gpk_capreader_index / _index_all and the metadata
// getters) and the AF_PACKET ring walk (gpk_afpacket.cpp: gpk_tpacket_index,
// deferred release, VLAN copies into the side buffer) — compiled from the
// product sources with -fsanitize=address,undefined and driven over mutated
// capture files and randomly corrupted V1/V2/V3 rings. Every buffer handed to
// the library is an exact-size heap allocation, so a read one byte past what
// the caller passed is reported. The checks here are memory safety and the
// API's own contracts (packets inside the bytes consumed, counts within max,
// packets inside the ring or the side buffer); parity with the reference is
// the oracle tests' job (tests/test_capture_cpu.py, tests/test_afpacket_cpu.py).
//
//   fuzz_host SEED ITERS FILE...   (FILE: seed captures; *.pcap read as pcap)
#include <linux/if_packet.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/gpk_afpacket.h"
#include "../../include/gpk_capture.h"
#include "../../gopacket_amd/csrc/gpk_pinned.h"
#include "../../gopacket_amd/csrc/gpk_walk.h"

// The pump and the replay are not driven here (they need a device); the
// symbols they reference from other translation units abort if reached.
extern "C" int gpk_decode_batch_ex(gpk_ctx*, const gpk_parser*, const gpk_batch*, const gpk_results*, void*, uint64_t,
                                   char*, size_t, gpk_fields*) {
  abort();
}
hipError_t gpk_pin_alloc(void**, size_t) { abort(); }
extern "C" int gpk_ctx_device(const gpk_ctx*) { abort(); }
extern "C" uint64_t gpk_ctx_stop_seq(const gpk_ctx*) { abort(); }
hipError_t gpk_pin_free(void*) { abort(); }

namespace {

struct Rng {
  uint64_t s;
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  uint64_t below(uint64_t n) { return n ? next() % n : 0; }
  bool chance(double p) { return (next() >> 11) * (1.0 / 9007199254740992.0) < p; }
};

#define CHECK(c)                                                               \
  do {                                                                         \
    if (!(c)) {                                                                \
      fprintf(stderr, "fuzz_host: contract broken at %s:%d: %s\n", __FILE__, __LINE__, #c); \
      abort();                                                                 \
    }                                                                          \
  } while (0)

// An exact-size copy: ASan's redzone starts right after the last byte.
struct Exact {
  std::unique_ptr<uint8_t[]> p;
  uint64_t n = 0;
  Exact(const uint8_t* src, uint64_t len) : p(new uint8_t[len ? len : 1]), n(len) {
    if (len) memcpy(p.get(), src, len);
  }
  uint8_t* data() { return n ? p.get() : nullptr; }
};

volatile uint64_t g_sink;

uint64_t touch(const uint8_t* b, uint64_t n) {
  uint64_t s = 0;
  for (uint64_t i = 0; i < n; i++) s += b[i];
  return s;
}

std::vector<uint8_t> read_file(const char* path) {
  std::vector<uint8_t> out;
  FILE* f = fopen(path, "rb");
  if (!f) return out;
  uint8_t buf[65536];
  size_t k;
  while ((k = fread(buf, 1, sizeof(buf), f)) > 0) out.insert(out.end(), buf, buf + k);
  fclose(f);
  return out;
}

// ---- capture files -----------------------------------------------------------

void put32(std::vector<uint8_t>& b, size_t at, uint32_t v) {
  if (at + 4 <= b.size()) memcpy(&b[at], &v, 4);
}

void mutate(std::vector<uint8_t>& b, Rng& r) {
  const int k = 1 + (int)r.below(5);
  for (int j = 0; j < k && !b.empty(); j++) {
    const size_t n = b.size();
    switch (r.below(7)) {
      case 0:
        b[r.below(n)] ^= (uint8_t)(1u << r.below(8));
        break;
      case 1: {  // a length-like word at a 4-byte boundary
        static const uint32_t edge[] = {0,          1,          4,          8,          12,         16,
                                        20,         28,         32,         0x7FFFFFFF, 0x80000000, 0xFFFFFFFF,
                                        0xFFFFFFFC, 0x0A0D0D0A, 0x1A2B3C4D, 0x4D3C2B1A, 0x00000006, 0x00000003};
        uint32_t v = r.chance(0.7) ? edge[r.below(sizeof(edge) / 4)] : (uint32_t)r.next();
        if (r.chance(0.2)) v = (uint32_t)(n - r.below(64));
        if (r.chance(0.3)) v = __builtin_bswap32(v);
        put32(b, r.below(n) & ~(size_t)3, v);
        break;
      }
      case 2:
        b.resize(r.below(n + 1));
        break;
      case 3: {  // duplicate a range (a block spliced in again)
        size_t a = r.below(n), len = std::min<size_t>(n - a, 1 + r.below(256));
        std::vector<uint8_t> seg(b.begin() + a, b.begin() + a + len);
        size_t at = r.below(b.size() + 1);
        b.insert(b.begin() + at, seg.begin(), seg.end());
        break;
      }
      case 4: {
        size_t a = r.below(n), len = std::min<size_t>(n - a, 1 + r.below(64));
        b.erase(b.begin() + a, b.begin() + a + len);
        break;
      }
      case 5: {
        size_t a = r.below(n), len = std::min<size_t>(n - a, 1 + r.below(32));
        for (size_t i = 0; i < len; i++) b[a + i] = (uint8_t)r.next();
        break;
      }
      default:  // an option code / length pair (pcapng options are 2+2 bytes)
        if (n >= 4) {
          size_t at = r.below(n - 3) & ~(size_t)1;
          uint16_t c = (uint16_t)r.below(12), l = (uint16_t)(r.chance(0.5) ? r.below(40) : r.next());
          memcpy(&b[at], &c, 2);
          memcpy(&b[at + 2], &l, 2);
        }
    }
  }
}

void metadata(gpk_capreader* rd) {
  char s[256];
  int e = 0, p = 0;
  gpk_capreader_error(rd, s, sizeof(s), &e, &p);
  gpk_capreader_error(rd, s, 1, &e, &p);  // a one-byte buffer still NUL-terminates
  g_sink += gpk_capreader_link_type(rd);
  uint32_t snap = 0;
  uint16_t ma = 0, mi = 0;
  int ns = 0;
  gpk_capreader_pcap_header(rd, &snap, &ma, &mi, &ns);
  const int nsec = gpk_capreader_nsections(rd);
  for (int sec = -1; sec <= nsec + 1; sec++) {
    for (int f = -1; f <= 4; f++) g_sink += gpk_capreader_section_info(rd, sec, f, s, sizeof(s));
    const int ni = gpk_capreader_ninterfaces(rd, sec);
    for (int i = -1; i <= ni; i++) {
      gpk_ng_interface itf;
      g_sink += gpk_capreader_interface(rd, sec, i, &itf);
      for (int f = -1; f <= 6; f++) g_sink += gpk_capreader_interface_str(rd, sec, i, f, s, sizeof(s));
    }
    uint64_t at = 0, seq = 0;
    g_sink += gpk_capreader_section_end_at(rd, sec, &at, &seq) + at + seq;
  }
  // name records, statistics callbacks (every index, a few out of range)
  const int nn = gpk_capreader_nnames(rd);
  for (int i = -1; i <= nn; i++) {
    int kind = 0, alen = 0, nnames = 0;
    uint8_t addr[24];
    const int need = gpk_capreader_name(rd, i, &kind, addr, &alen, &nnames, nullptr, 0);
    if (need >= 0) {
      CHECK(alen == 4 || alen == 16 || alen == 24);
      std::vector<char> names((size_t)need + 1);
      CHECK(gpk_capreader_name(rd, i, nullptr, nullptr, nullptr, nullptr, names.data(), (size_t)need) == need);
      CHECK(gpk_capreader_name(rd, i, nullptr, nullptr, nullptr, nullptr, names.data(), (size_t)need / 2) == need);
      g_sink += touch(addr, (uint64_t)alen) + (uint64_t)nnames;
    }
  }
  const int ne = gpk_capreader_nstat_events(rd);
  for (int k = -1; k <= ne; k++) {
    uint64_t at = 0, seq = 0;
    int iface = 0;
    gpk_ng_interface st;
    g_sink += gpk_capreader_stat_event(rd, k, &at, &seq, &iface, &st, s, sizeof(s)) + at + seq;
    g_sink += gpk_capreader_stat_event(rd, k, nullptr, nullptr, nullptr, nullptr, s, 1);
  }
}

void run_capture(const std::vector<uint8_t>& file, int fmt, Rng& r) {
  const uint32_t flags = (uint32_t)r.below(8);
  gpk_capreader* rd = nullptr;
  CHECK(gpk_capreader_create(&rd, fmt, flags) == GPK_OK);
  const bool opts = r.chance(0.7);  // ReadPacketDataWithOptions: the options kept per packet
  CHECK(gpk_capreader_keep_options(rd, opts ? 1 : 0) == GPK_OK);
  if (fmt == GPK_CAP_PCAP && r.chance(0.3)) CHECK(gpk_capreader_set_snaplen(rd, (uint32_t)r.next()) == GPK_OK);
  uint64_t pos = 0, chunk = 1 + r.below(std::max<uint64_t>(1, file.size())), calls = 0, ends = 0;
  while (calls++ < 4096) {
    if (fmt == GPK_CAP_PCAPNG && r.chance(0.02)) g_sink += (uint64_t)gpk_capreader_skip_section(rd);
    const uint64_t avail = std::min<uint64_t>(file.size() - pos, chunk);
    const int eof = pos + avail == file.size();
    Exact in(file.data() + pos, avail);
    const uint64_t max = 1 + r.below(64);
    std::unique_ptr<uint64_t[]> off(new uint64_t[max]);
    std::unique_ptr<uint32_t[]> cap(new uint32_t[max]);
    std::unique_ptr<gpk_capture_info[]> ci(new gpk_capture_info[max]);
    uint64_t n = 0, used = 0;
    const int rc = gpk_capreader_index(rd, in.data(), avail, eof, off.get(), cap.get(), r.chance(0.8) ? ci.get() : nullptr,
                                       max, &n, &used);
    CHECK(rc >= 0);
    CHECK(n <= max && used <= avail);
    for (uint64_t i = 0; i < n; i++) {
      CHECK(off[i] + cap[i] <= used);
      g_sink += touch(in.data() + off[i], cap[i]);
      const uint8_t* tlv = nullptr;
      uint64_t nb = 0;
      if (opts) {
        CHECK(gpk_capreader_packet_options(rd, i, &tlv, &nb) == GPK_OK);
        for (uint64_t q = 0; q < nb;) {  // well-formed records, inside the bytes given
          uint32_t len = 0;
          CHECK(q + 8 <= nb);
          memcpy(&len, tlv + q + 4, 4);
          q += 8 + ((len + 3ull) & ~3ull);
          CHECK(q <= nb);
        }
        g_sink += touch(tlv, nb);
      }
    }
    if (opts) CHECK(gpk_capreader_packet_options(rd, n, nullptr, nullptr) == GPK_EINVAL);
    pos += used;
    if (rc == GPK_CAP_END) {
      metadata(rd);
      if (++ends > 2 || eof) break;  // calling again continues like another ReadPacketData
    } else if (rc == GPK_CAP_MORE) {
      if (eof) break;
      if (used == 0) chunk = chunk * 2 + 1;  // a record longer than the bytes given
    }
  }
  metadata(rd);
  gpk_capreader_destroy(rd);

  // the whole buffer at once, the walk split over threads
  CHECK(gpk_capreader_create(&rd, fmt, flags) == GPK_OK);
  Exact all(file.data(), file.size());
  gpk_capindex x{};
  uint64_t used = 0;
  const int rc = gpk_capreader_index_all(rd, all.data(), all.n, 1, 1 + (int)r.below(4), &x, &used);
  CHECK(rc >= 0 && used <= all.n);
  for (uint64_t i = 0; i < x.n; i++) {
    CHECK(x.offsets[i] + x.caplens[i] <= used);
    g_sink += touch(all.data() + x.offsets[i], x.caplens[i]) + (uint64_t)x.ci[i].ts_sec;
  }
  gpk_capindex_free(&x);
  // the byte-range replay's block sync (gpk_replay_file_range) over random windows of the
  // bytes: inside [from, to), 4-aligned, reading nothing past end
  for (int k = 0; k < 8 && all.n; k++) {
    const uint64_t from = r.below(all.n), to = from + r.below(all.n - from + 1), span = 32 + r.below(1u << 16);
    const uint64_t p = gpk_capreader_sync(rd, all.data(), from, to, all.n, span);
    CHECK(p == ~0ull || (p >= from && p < to && p % 4 == 0));
  }
  g_sink += gpk_capreader_state_version(rd);
  metadata(rd);
  gpk_capreader_destroy(rd);
}

// ---- AF_PACKET rings ---------------------------------------------------------

uint32_t wild(Rng& r, uint32_t good, uint32_t span) {  // usually `good`, sometimes anything
  if (!r.chance(0.06)) return good;
  switch (r.below(4)) {
    case 0: return 0;
    case 1: return 0xFFFFFFFFu - (uint32_t)r.below(64);
    case 2: return good + (uint32_t)r.below(span + 1);
    default: return (uint32_t)r.next();
  }
}

void fill_v3(uint8_t* ring, uint64_t bs, uint64_t nb, Rng& r) {
  for (uint64_t b = 0; b < nb; b++) {
    uint8_t* blk = ring + b * bs;
    auto* bd = reinterpret_cast<tpacket_block_desc*>(blk);
    const uint32_t first = 48;
    uint32_t pos = first, npk = 0;
    uint32_t prev_next_at = 0;
    const uint32_t want = (uint32_t)r.below(14);
    for (uint32_t k = 0; k < want; k++) {
      const uint32_t dlen = (uint32_t)r.below(300);
      const uint32_t mac = r.chance(0.9) ? 82 : (uint32_t)(r.below(2) ? 98 : r.below(0x10000));
      const uint32_t step = (uint32_t)((std::min<uint64_t>(mac, 200) + dlen + 15) & ~15u);
      if ((uint64_t)pos + sizeof(tpacket3_hdr) + 64 + step > bs) break;
      auto* h = reinterpret_cast<tpacket3_hdr*>(blk + pos);
      h->tp_next_offset = 0;
      h->tp_sec = (uint32_t)r.next();
      h->tp_nsec = (uint32_t)r.next();
      h->tp_snaplen = wild(r, dlen, (uint32_t)bs);
      h->tp_len = r.chance(0.1) ? 0 : wild(r, dlen, 1 << 16);
      h->tp_status = (uint32_t)(r.below(2) ? TP_STATUS_USER : TP_STATUS_USER | TP_STATUS_VLAN_VALID) |
                     (r.chance(0.3) ? TP_STATUS_VLAN_TPID_VALID : 0);
      h->tp_mac = (uint16_t)mac;
      h->tp_net = (uint16_t)(mac + 14);
      h->hv1.tp_rxhash = (uint32_t)r.next();
      h->hv1.tp_vlan_tci = (uint32_t)r.below(0x20000);
      h->hv1.tp_vlan_tpid = (uint16_t)(r.below(2) ? 0x8100 : r.next());
      if (k) reinterpret_cast<tpacket3_hdr*>(blk + prev_next_at)->tp_next_offset =
                 wild(r, pos - prev_next_at, (uint32_t)bs);
      prev_next_at = pos;
      pos += std::max<uint32_t>(step, 64);
      npk++;
    }
    bd->version = TPACKET_V3;
    bd->offset_to_priv = 48;
    bd->hdr.bh1.block_status = r.chance(0.8) ? TP_STATUS_USER : (r.below(2) ? 0 : (uint32_t)r.next());
    bd->hdr.bh1.num_pkts = r.chance(0.05) ? (uint32_t)(npk + 1 + r.below(r.below(2) ? 4 : 1u << 20)) : npk;
    bd->hdr.bh1.offset_to_first_pkt = wild(r, first, (uint32_t)bs);
    bd->hdr.bh1.blk_len = pos;
    bd->hdr.bh1.seq_num = b + 1;
  }
}

void fill_frames(uint8_t* ring, int version, uint64_t fz, uint64_t nf, Rng& r) {
  for (uint64_t f = 0; f < nf; f++) {
    uint8_t* p = ring + f * fz;
    const uint32_t mac = r.chance(0.9) ? 66 : (uint32_t)r.below(0x10000);
    const uint32_t room = fz > 66 ? (uint32_t)(fz - 66) : 0;
    const uint32_t dlen = (uint32_t)r.below(room + 1);
    const uint32_t status = r.chance(0.8) ? TP_STATUS_USER : (r.below(2) ? 0 : (uint32_t)r.next());
    if (version == GPK_TPACKET_V1) {
      auto* h = reinterpret_cast<tpacket_hdr*>(p);
      h->tp_status = status;
      h->tp_len = r.chance(0.1) ? 0 : wild(r, dlen, 1 << 16);
      h->tp_snaplen = wild(r, dlen, (uint32_t)fz * 4);
      h->tp_mac = (uint16_t)mac;
      h->tp_net = (uint16_t)(mac + 14);
      h->tp_sec = (uint32_t)r.next();
      h->tp_usec = (uint32_t)r.next();
    } else {
      auto* h = reinterpret_cast<tpacket2_hdr*>(p);
      h->tp_status = status | (r.chance(0.3) ? TP_STATUS_VLAN_VALID : 0);
      h->tp_len = r.chance(0.1) ? 0 : wild(r, dlen, 1 << 16);
      h->tp_snaplen = wild(r, dlen, (uint32_t)fz * 4);
      h->tp_mac = (uint16_t)mac;
      h->tp_net = (uint16_t)(mac + 14);
      h->tp_sec = (uint32_t)r.next();
      h->tp_nsec = (uint32_t)r.next();
      h->tp_vlan_tci = (uint16_t)r.next();
      h->tp_vlan_tpid = (uint16_t)r.next();
    }
  }
}

void rearm(uint8_t* ring, int version, uint64_t hb, uint64_t nh, Rng& r) {  // an emulated kernel
  for (uint64_t h = 0; h < nh; h++) {
    if (!r.chance(0.3)) continue;
    uint8_t* p = ring + h * hb;
    if (version == GPK_TPACKET_V3) {
      auto* bd = reinterpret_cast<tpacket_block_desc*>(p);
      if (bd->hdr.bh1.block_status == 0) bd->hdr.bh1.block_status = TP_STATUS_USER;
    } else if (version == GPK_TPACKET_V1) {
      auto* f = reinterpret_cast<tpacket_hdr*>(p);
      if (f->tp_status == 0) f->tp_status = TP_STATUS_USER;
    } else {
      auto* f = reinterpret_cast<tpacket2_hdr*>(p);
      if (f->tp_status == 0) f->tp_status = TP_STATUS_USER;
    }
  }
}

void run_ring(Rng& r) {
  const int version = (int)r.below(3);
  gpk_tp_opts o;
  gpk_tp_default_opts(&o);
  o.version = version;
  if (version == GPK_TPACKET_V3) {
    o.frame_size = 4096;
    o.block_size = 4096 * (int)(1 + r.below(4));
    o.num_blocks = 1 + (int)r.below(6);
  } else {
    static const int fz[] = {128, 256, 512, 1024, 2048, 4096};
    o.frame_size = fz[r.below(6)];
    o.block_size = 4096;
    o.num_blocks = 1 + (int)r.below(3);
  }
  o.add_vlan_header = (int)r.below(2);
  CHECK(gpk_tp_check_opts(&o, nullptr, 0) == GPK_OK);
  const uint64_t bytes = (uint64_t)o.block_size * o.num_blocks;
  std::unique_ptr<uint8_t[]> ring(new uint8_t[bytes]);
  for (uint64_t i = 0; i < bytes; i++) ring[i] = (uint8_t)r.next();
  uint64_t hb, nh;
  if (version == GPK_TPACKET_V3) {
    hb = (uint64_t)o.block_size;
    nh = (uint64_t)o.num_blocks;
    fill_v3(ring.get(), hb, nh, r);
  } else {
    hb = (uint64_t)o.frame_size;
    nh = bytes / hb;
    fill_frames(ring.get(), version, hb, nh, r);
  }
  gpk_tpacket* t = nullptr;
  CHECK(gpk_tpacket_attach(&t, ring.get(), bytes, version, &o) == GPK_OK);
  uint64_t g_hb = 0, g_nh = 0;
  gpk_tpacket_geometry(t, &g_hb, &g_nh);
  CHECK(g_hb == hb && g_nh == nh);
  gpk_tpacket_set_threads(t, 1 + (int)r.below(4));
  const bool defer = r.chance(0.4);
  gpk_tpacket_defer(t, defer ? 1 : 0);
  int waits = 0;
  for (int call = 0; call < 64; call++) {
    // now and then a call large enough for the parallel pre-walk of V3 blocks
    const uint64_t max = r.chance(0.2) ? 4096 + r.below(4096) : 1 + r.below(40);
    const uint64_t side_cap = r.chance(0.2) ? r.below(64) : 1 + r.below(8192);
    std::unique_ptr<uint8_t[]> side(new uint8_t[side_cap ? side_cap : 1]);
    std::unique_ptr<uint64_t[]> off(new uint64_t[max]);
    std::unique_ptr<uint32_t[]> cap(new uint32_t[max]);
    std::unique_ptr<gpk_tp_info[]> ci(new gpk_tp_info[max]);
    uint64_t n = 0, used = 0;
    const int rc = gpk_tpacket_index(t, 0, off.get(), cap.get(), ci.get(), max, &n, side.get(), side_cap, &used);
    CHECK(rc >= 0 && n <= max && used <= side_cap);
    for (uint64_t i = 0; i < n; i++) {
      if (off[i] < bytes) {
        CHECK(off[i] + cap[i] <= bytes);
        g_sink += touch(ring.get() + off[i], cap[i]);
      } else {
        CHECK(off[i] - bytes + cap[i] <= used);
        g_sink += touch(side.get() + (off[i] - bytes), cap[i]);
      }
    }
    uint64_t nf = 0, nc = 0, seq = 0;
    gpk_tpacket_take_new_headers(t, &nf, &nc);
    gpk_tpacket_release_seq(t, &seq);
    if (defer && r.chance(0.7)) gpk_tpacket_release(t, r.chance(0.5) ? seq : seq / 2);
    if (rc == GPK_TP_ERROR) {
      char e[200];
      int pan = 0;
      g_sink += gpk_tpacket_error(t, e, sizeof(e), &pan);
      break;
    }
    if (rc == GPK_TP_WAIT) {
      if (++waits > 4) break;
      rearm(ring.get(), version, hb, nh, r);
    }
  }
  int64_t pk = 0, polls = 0;
  gpk_tpacket_stats(t, &pk, &polls);
  if (defer) gpk_tpacket_release(t, UINT64_MAX);
  gpk_tpacket_close(t);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: fuzz_host SEED ITERS [FILE...]\n");
    return 2;
  }
  Rng r{strtoull(argv[1], nullptr, 0)};
  const long iters = strtol(argv[2], nullptr, 0);
  std::vector<std::pair<std::vector<uint8_t>, int>> seeds;
  for (int i = 3; i < argc; i++) {
    std::string p = argv[i];
    auto d = read_file(argv[i]);
    if (d.empty()) continue;
    const bool pcap = p.size() > 5 && p.compare(p.size() - 5, 5, ".pcap") == 0;
    seeds.push_back({std::move(d), pcap ? GPK_CAP_PCAP : GPK_CAP_PCAPNG});
  }
  long caps = 0, rings = 0;
  const bool verbose = getenv("FUZZ_VERBOSE") != nullptr;
  for (long it = 0; it < iters; it++) {
    if (verbose) fprintf(stderr, "iter %ld\n", it);
    if (!seeds.empty() && r.chance(0.5)) {
      auto& s = seeds[r.below(seeds.size())];
      std::vector<uint8_t> b = s.first;
      if (r.chance(0.9)) mutate(b, r);
      // the wrong format now and then: a pcapng through the pcap reader and back
      const int fmt = r.chance(0.05) ? (GPK_CAP_PCAP + GPK_CAP_PCAPNG - s.second) : s.second;
      if (verbose) fprintf(stderr, "  capture: %zu bytes, format %d\n", b.size(), fmt);
      run_capture(b, fmt, r);
      caps++;
    } else {
      if (verbose) fprintf(stderr, "  ring\n");
      run_ring(r);
      rings++;
    }
  }
  printf("fuzz_host ok: %ld capture runs, %ld ring runs\n", caps, rings);
  return 0;
}

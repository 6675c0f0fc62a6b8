// gpk_capture.cpp — pcap / pcapng batch indexer (include/gpk_capture.h).
//
// A restatement of pcapgo's readers as a resumable byte-stream machine: the
// capture arrives in chunks (pinned staging slots), the machine walks the
// records in place and emits (offset, caplen, CaptureInfo) per packet, so the
// staging buffer itself is the packed batch the device decodes — no copy of
// packet bytes on the host.
//
// Each "call" below is one ReadPacketData of the reference. The reader's
// position and state advance exactly as Go's bufio-backed reader does,
// including its accounting quirks (block length tracked as uint32 and allowed
// to wrap, the reused option value buffer, the 24-byte EUI address length in
// name records), so a malformed capture desynchronises the same way. When a
// call needs bytes beyond the chunk (and the chunk is not the end of the
// stream) the call is undone — position back to its start, state restored
// from a snapshot taken lazily at the first mutation — and indexing stops
// there: the caller re-presents the rest with more bytes appended.
//
// Reference functions (pcapgo/): NewNgReader ngread.go:64-107, readBytes
// :113-126, discard :128-137, readBlock :165-193, readOption :196-234,
// readSectionHeader :238-312, skipSection :315-327, firstInterface :338-373,
// readInterfaceDescriptor :376-437, convertTime :440-443,
// readInterfaceStatistics :446-489, readPacketHeader :494-580,
// readPacketOptions :582-625, ReadPacketDataWithOptions :636-664,
// readNameResolutionBlock ngread_nrb.go:64-130, readDecryptionSecretsBlock
// ngread_dsb.go:18-39; NewReader/readHeader read.go:65-119, ReadPacketData
// :122-137, readPacketHeader :169-177.
#include <algorithm>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <functional>
#include <mutex>
#include <cstring>
#include <cstdlib>
#include <new>
#include <string>
#include <thread>
#include <sched.h>
#include <vector>

#include "../../include/gpk_capture.h"
#include "gpk_walk.h"

namespace {

constexpr int64_t kZeroTimeSec = -62135596800LL;  // time.Time{}.Unix()
constexpr uint64_t kNoValue64 = ~0ull;             // NgNoValue64
constexpr uint32_t kSHB = 0x0A0D0D0A, kIDB = 1, kPB = 2, kSPB = 3, kNRB = 4, kISB = 5, kEPB = 6, kDSB = 0xA;
constexpr uint32_t kByteOrderMagic = 0x1A2B3C4D;

const char* const kEOF = "EOF";
const char* const kUnexpectedEOF = "unexpected EOF";

struct NeedMore {};
struct GoErr {
  std::string text;
  bool panic;
};
[[noreturn]] void fail(const std::string& s, bool panic = false) { throw GoErr{s, panic}; }

std::string fmt(const char* f, ...) __attribute__((format(printf, 1, 2)));
std::string fmt(const char* f, ...) {
  char b[256];
  va_list ap;
  va_start(ap, f);
  vsnprintf(b, sizeof(b), f, ap);
  va_end(ap);
  return b;
}

inline uint16_t ld16(const uint8_t* p, bool be) {
  return be ? (uint16_t)(p[0] << 8 | p[1]) : (uint16_t)(p[1] << 8 | p[0]);
}
inline uint32_t ld32(const uint8_t* p, bool be) {
  return be ? ((uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3])
            : ((uint32_t)p[3] << 24 | (uint32_t)p[2] << 16 | (uint32_t)p[1] << 8 | p[0]);
}
inline uint64_t ld64(const uint8_t* p, bool be) {
  return be ? ((uint64_t)ld32(p, true) << 32 | ld32(p + 4, true)) : ((uint64_t)ld32(p + 4, false) << 32 | ld32(p, false));
}

// time.Unix(sec, nsec).UTC() normalisation
void unix_norm(int64_t sec, int64_t nsec, int64_t* os, uint32_t* ons) {
  if (nsec < 0 || nsec >= 1000000000LL) {
    int64_t n = nsec / 1000000000LL;  // truncates toward zero, like Go
    sec = (int64_t)((uint64_t)sec + (uint64_t)n);
    nsec -= n * 1000000000LL;
    if (nsec < 0) {
      nsec += 1000000000LL;
      sec = (int64_t)((uint64_t)sec - 1);
    }
  }
  *os = sec;
  *ons = (uint32_t)nsec;
}

struct Stats {
  int64_t lu_s = kZeroTimeSec, st_s = kZeroTimeSec, et_s = kZeroTimeSec;
  uint32_t lu_ns = 0, st_ns = 0, et_ns = 0;
  std::string comment;
  uint64_t received = 0, dropped = 0;
};

struct Iface {
  std::string name, comment, description, filter, os;
  uint16_t link_type = 0;
  uint8_t tsres = 0;
  uint64_t tsoff = 0;
  uint32_t snap = 0;
  uint64_t second_mask = 0, scale_up = 0, scale_down = 0;
  bool has_stats = false;
  Stats stats;
};

struct Section {
  std::string comment, hardware, os, application;
};

struct NgState {  // what a rollback restores
  bool be = false;
  std::vector<Iface> ifaces;
  Section section;
  uint16_t link_type = 0;
  bool first_section_found = false, active_section = false;
  std::vector<std::pair<Section, std::vector<Iface>>> ended;
  std::vector<uint64_t> ended_at;   // packets returned before each SectionEndCallback call
  std::vector<uint64_t> ended_seq;  // ... and its place among all the reader's callbacks
  uint64_t ncb = 0;                 // SectionEndCallback + StatisticsCallback calls so far
};

// One NgNameRecord (pcapng.go NgNameRecord; readNameResolutionBlock,
// ngread_nrb.go:64-130): IPv4 / IPv6 addresses as their 4 / 16 bytes, EUI
// addresses as the 24 bytes newHWAddress clones (the reader's whole scratch
// buffer, ngread_nrb.go:56-61), and the names with their NULs trimmed.
struct NameRec {
  uint16_t rtype = 0;
  uint8_t addr[24] = {0};
  uint32_t alen = 0;
  std::vector<std::string> names;
};

// One StatisticsCallback call (ngread.go:485-487): the interface id and the
// statistics as the block left them, after `at` packets were returned.
struct StatEvent {
  uint64_t at = 0, seq = 0;
  uint32_t iface = 0;
  Stats stats;
};

struct OptBuf {  // NgReader.currentOption.value: backing array + length
  std::vector<uint8_t> back = std::vector<uint8_t>(1024, 0);
  uint32_t len = 1024;
};

}  // namespace

struct gpk_capreader {
  int format = 0;
  uint32_t flags = 0;
  // stream cursor over the current chunk
  const uint8_t* b = nullptr;
  uint64_t n = 0, pos = 0;
  bool eof = false;
  // life cycle
  bool opened = false, open_failed = false;
  std::string err_text;
  bool err_eof = false, err_panic = false;
  // pcap
  bool pbe = false;
  uint32_t factor = 1, snaplen = 0;
  uint16_t major = 0, minor = 0;
  uint32_t plink = 0;
  // pcapng
  NgState st, st_snap;
  bool st_saved = false;
  OptBuf opt, opt_snap;
  bool opt_saved = false;
  // every change of st or opt counts one (touch / touch_opt), undone with the
  // change on a rollback: equal counts after the same bytes whatever the
  // chunking, so a byte-range replay can tell whether its range changed any
  // reader state (gpk_replay_file_range)
  uint64_t mutations = 0;
  // NgReader.buf, the 24-byte scratch buffer block and option headers are read
  // into (EUI name records clone all of it); undone with a rolled-back call
  uint8_t gobuf[24] = {0};
  uint64_t npk = 0;  // packets returned so far (by gpk_capreader_index / _index_all)
  // name records of the current section (NgReader.nameRecords), snapshot like opt
  std::vector<NameRec> names, names_snap;
  bool names_saved = false;
  std::vector<StatEvent> stat_events;  // every StatisticsCallback call so far
  // gpk_capreader_keep_options: the options of the packets of the last index
  // call, as records {u16 code, u16 0, u32 len, value padded to 4}
  bool keep_opts = false;
  std::vector<uint8_t> opt_arena;
  std::vector<uint64_t> opt_at;  // packet k's records: opt_arena[opt_at[k], opt_at[k+1])
  bool pending_skip = false;     // gpk_capreader_skip_section: SkipSection first
  uint32_t typ = 0, blen = 0;  // currentBlock
  uint16_t opt_code = 0;
  // ci of the current call
  uint32_t ci_iface = 0, ci_caplen = 0, ci_len = 0;
  int64_t ci_s = 0;
  uint32_t ci_ns = 0;

  // ---- primitives (bufio.Reader over the chunk) ----------------------------
  uint64_t avail() const { return n - pos; }
  // NgReader.readBytes: reads k <= m bytes; short only at end of stream
  uint64_t read_into(uint8_t* dst, uint64_t m) {
    if (m > avail()) {
      if (!eof) throw NeedMore{};
      uint64_t k = avail();
      if (dst && k) memcpy(dst, b + pos, k);
      pos = n;
      return k;
    }
    if (dst && m) memcpy(dst, b + pos, m);
    pos += m;
    return m;
  }
  const uint8_t* read_view(uint64_t m) {  // readBytes into a scratch buffer, error on short read
    if (m > avail()) {
      if (!eof) throw NeedMore{};
      pos = n;
      fail(kUnexpectedEOF);
    }
    const uint8_t* p = b + pos;
    pos += m;
    return p;
  }
  // readBytes(r.buf[:m]) (ngread.go:113-126): the bytes land in NgReader.buf
  // (partly when the stream ends first, with the error)
  const uint8_t* read_gobuf(uint64_t m) {
    if (m > avail() && eof) to_gobuf(0, b + pos, avail());
    const uint8_t* p = read_view(m);
    to_gobuf(0, p, m);
    return p;
  }
  void discard(uint64_t m) {  // NgReader.discard
    if (m > avail()) {
      if (!eof) throw NeedMore{};
      pos = n;
      fail(kUnexpectedEOF);
    }
    pos += m;
    blen -= (uint32_t)m;
  }
  bool be() const { return st.be; }
  void touch() {
    mutations++;
    if (!st_saved) {
      st_snap = st;
      st_saved = true;
    }
  }
  void touch_opt() {
    mutations++;
    if (!opt_saved) {
      opt_snap = opt;
      opt_saved = true;
    }
  }
  // name records are no state a later packet depends on (no mutation counted:
  // a byte-range replay may split across them)
  void touch_names() {
    if (!names_saved) {
      names_snap = names;
      names_saved = true;
    }
  }
  // bytes readBytes put into NgReader.buf[at, at + m)
  void to_gobuf(uint32_t at, const uint8_t* p, uint64_t m) {
    if (m) memcpy(gobuf + at, p, m);
  }

  // ---- pcapng --------------------------------------------------------------
  void read_block() {
    if (avail() < 8) {
      if (!eof) throw NeedMore{};
      uint64_t k = avail();
      to_gobuf(0, b + pos, k);
      pos = n;
      fail(k == 0 ? kEOF : kUnexpectedEOF);
    }
    const uint8_t* h = b + pos;
    pos += 8;
    to_gobuf(0, h, 8);
    typ = ld32(h, be());
    if (typ == kSHB) {
      if (avail() < 4 && eof) to_gobuf(8, b + pos, avail());
      const uint8_t* m = read_view(4);
      to_gobuf(8, m, 4);
      bool nbe;
      if (ld32(m, true) == kByteOrderMagic)
        nbe = true;
      else if (ld32(m, false) == kByteOrderMagic)
        nbe = false;
      else
        fail("Wrong byte order value in Section Header");
      if (nbe != st.be) {
        touch();
        st.be = nbe;
      }
      blen = ld32(h + 4, be()) - 8 - 4;
      return;
    }
    blen = ld32(h + 4, be()) - 8;
  }

  void read_option() {
    if (blen == 4) {
      opt_code = 0;
      return;
    }
    const uint8_t* h = read_gobuf(4);
    blen -= 4;
    opt_code = ld16(h, be());
    uint16_t olen = ld16(h + 2, be());
    if (opt_code == 0) {
      if (olen != 0) fail("End of Options must be zero length");
      return;
    }
    if (olen != 0) {
      touch_opt();
      if (olen < opt.back.size()) {
        opt.len = olen;
      } else {
        opt.back.assign(olen, 0);
        opt.len = olen;
      }
      uint64_t k = read_into(opt.back.data(), olen);
      if (k < olen) fail(kUnexpectedEOF);
      uint16_t pad = olen % 4;
      if (pad > 0) discard(4 - pad);
      blen -= olen;
    }
  }
  std::string opt_str(uint32_t skip = 0) const {
    return skip >= opt.len ? std::string() : std::string((const char*)opt.back.data() + skip, opt.len - skip);
  }
  uint64_t opt_u64() const { return ld64(opt.back.data(), be()); }  // value[:8] (cap >= 1024)
  uint32_t opt_u32(uint32_t o) const { return ld32(opt.back.data() + o, be()); }

  void read_section_header() {
    touch();
    if (st.active_section) {
      st.ended.emplace_back(st.section, st.ifaces);
      st.ended_at.push_back(npk);
      st.ended_seq.push_back(st.ncb++);
    }
    st.ifaces.clear();
    touch_names();
    names.clear();
    st.active_section = false;
    for (;;) {  // RESTART
      const uint8_t* h = read_gobuf(12);
      blen -= 12;
      uint16_t vmaj = ld16(h, be()), vmin = ld16(h + 2, be());
      if (vmaj != 1 || vmin != 0) {
        if (!(flags & GPK_NG_SKIP_UNKNOWN_VERSION)) fail("Unknown pcapng Version in Section Header");
        discard(blen);
        skip_section();
        continue;
      }
      break;
    }
    Section sec;
    for (;;) {
      read_option();
      if (opt_code == 0) break;
      switch (opt_code) {
        case 1: sec.comment = opt_str(); break;
        case 2: sec.hardware = opt_str(); break;
        case 3: sec.os = opt_str(); break;
        case 4: sec.application = opt_str(); break;
      }
    }
    discard(blen);
    st.active_section = true;
    st.section = sec;
    if (!(flags & GPK_NG_WANT_MIXED_LINKTYPE)) first_interface();
  }

  void skip_section() {
    for (;;) {
      read_block();
      if (typ == kSHB) return;
      discard(blen);
    }
  }

  void first_interface() {
    for (;;) {
      read_block();
      switch (typ) {
        case kIDB:
          read_interface_descriptor();
          if (!st.first_section_found) {
            st.link_type = st.ifaces[0].link_type;
            st.first_section_found = true;
          } else if (st.link_type != st.ifaces[0].link_type) {
            if (flags & GPK_NG_ERROR_ON_MISMATCHING_LINKTYPE)
              fail("Link type of current interface is different from first one");
            continue;
          }
          return;
        case kPB:
        case kEPB:
        case kSPB:
        case kISB:
          fail("A section must have an interface before a packet block");
        case kDSB:
          read_decryption_secrets();
          break;
        case kNRB:
          read_name_resolution();
          break;
      }
      discard(blen);
    }
  }

  void read_interface_descriptor() {
    const uint8_t* h = read_gobuf(8);
    blen -= 8;
    Iface it;
    it.link_type = ld16(h, be());
    it.snap = ld32(h + 4, be());
    for (;;) {
      read_option();
      if (opt_code == 0) break;
      switch (opt_code) {
        case 2: it.name = opt_str(); break;
        case 1: it.comment = opt_str(); break;
        case 3: it.description = opt_str(); break;
        case 11: it.filter = opt_str(1); break;
        case 12: it.os = opt_str(); break;
        case 14: it.tsoff = opt_u64(); break;
        case 9: it.tsres = opt.back[0]; break;
      }
    }
    discard(blen);
    if (it.tsres == 0) it.tsres = 6;
    const uint32_t e = it.tsres & 0x7f;
    if (it.tsres & 0x80) {
      it.second_mask = e < 64 ? (1ull << e) : 0;  // Go: shifts >= 64 give 0
    } else {
      it.second_mask = 1;
      for (uint32_t j = 0; j < e; j++) it.second_mask *= 10;
    }
    it.scale_down = 1;
    it.scale_up = 1;
    if (it.second_mask < 1000000000ull) {
      if (it.second_mask == 0) fail("runtime error: integer divide by zero", true);
      it.scale_up = 1000000000ull / it.second_mask;
    } else {
      it.scale_down = it.second_mask / 1000000000ull;
    }
    touch();
    st.ifaces.push_back(std::move(it));
  }

  // convertTime (ngread.go:440-443) in uint64 arithmetic. The common
  // resolutions divide by constants (multiply-shift) or shift: a 64-bit
  // hardware divide per packet would dominate the record walk.
  void convert_time(uint32_t idx, uint64_t ts, int64_t* s, uint32_t* ns) const { iface_time(st.ifaces[idx], ts, s, ns); }
  static void iface_time(const Iface& it, uint64_t ts, int64_t* s, uint32_t* ns) {
    const uint64_t m = it.second_mask;
    uint64_t q, r;
    if (m == 1000000ull) {
      q = ts / 1000000ull;
      r = ts - q * 1000000ull;
    } else if (m == 1000000000ull) {
      q = ts / 1000000000ull;
      r = ts - q * 1000000000ull;
    } else if (m == 1000ull) {
      q = ts / 1000ull;
      r = ts - q * 1000ull;
    } else if ((m & (m - 1)) == 0) {
      q = ts >> __builtin_ctzll(m);
      r = ts & (m - 1);
    } else {
      q = ts / m;
      r = ts % m;
    }
    uint64_t nsec = r * it.scale_up;
    if (it.scale_down != 1) nsec /= it.scale_down;
    unix_norm((int64_t)(q + it.tsoff), (int64_t)nsec, s, ns);
  }

  void read_interface_statistics() {
    const uint8_t* h = read_gobuf(12);
    blen -= 12;
    uint32_t idx = ld32(h, be());
    uint64_t ts = (uint64_t)ld32(h + 4, be()) << 32 | ld32(h + 8, be());
    if (idx >= st.ifaces.size())
      fail(fmt("Interface id %u not present in section (have only %zu interfaces)", idx, st.ifaces.size()));
    touch();
    Iface& it = st.ifaces[idx];
    it.has_stats = true;
    it.stats = Stats();
    it.stats.received = it.stats.dropped = kNoValue64;
    convert_time(idx, ts, &it.stats.lu_s, &it.stats.lu_ns);
    for (;;) {
      read_option();
      if (opt_code == 0) break;
      Stats& S = st.ifaces[idx].stats;
      switch (opt_code) {
        case 1: S.comment = opt_str(); break;
        case 2: convert_time(idx, (uint64_t)opt_u32(0) << 32 | opt_u32(4), &S.st_s, &S.st_ns); break;
        case 3: convert_time(idx, (uint64_t)opt_u32(0) << 32 | opt_u32(4), &S.et_s, &S.et_ns); break;
        case 4: S.received = opt_u64(); break;
        case 5: S.dropped = opt_u64(); break;
      }
    }
    discard(blen);
    StatEvent ev;  // StatisticsCallback(ifaceID, *stats)
    ev.at = npk;
    ev.seq = st.ncb++;  // (st was saved by touch() above)
    ev.iface = idx;
    ev.stats = st.ifaces[idx].stats;
    stat_events.push_back(std::move(ev));
  }

  void read_decryption_secrets() {
    if (read_into(gobuf, 8) < 8) fail(fmt("could not read DecryptionSecret Header block length: %s", kUnexpectedEOF));
    blen -= 8;
    uint32_t slen = ld32(gobuf + 4, be());
    if (read_into(nullptr, slen) < slen)
      fail(fmt("could not read %u bytes from DecryptionSecret payload: %s", slen, kUnexpectedEOF));
    blen -= slen;
  }

  void read_name_resolution() {
    while (blen > 0) {
      if (read_into(gobuf, 4) < 4) fail(fmt("could not read NameRecord Header block length: %s", kUnexpectedEOF));
      blen -= 4;
      uint16_t rtype = ld16(gobuf, be()), rlen = ld16(gobuf + 2, be());
      int64_t length = rlen < (int64_t)blen ? (int64_t)rlen : (int64_t)blen;
      int64_t padding = length % 4 ? 4 - length % 4 : 0;
      int64_t alen;
      NameRec rec;
      rec.rtype = rtype;
      if (rtype == 1 || rtype == 2) {
        uint64_t m = rtype == 1 ? 4 : 16;
        if (read_into(gobuf, m) < m)
          fail(fmt("could not read %s address: could not read IP address: %s", rtype == 1 ? "IPv4" : "IPv6",
                   kUnexpectedEOF));
        alen = (int64_t)m;  // netip.AddrFromSlice(r.buf[:m])
        memcpy(rec.addr, gobuf, m);
        rec.alen = (uint32_t)m;
      } else if (rtype == 3 || rtype == 4) {
        uint64_t m = rtype == 3 ? 6 : 8;
        if (read_into(gobuf, m) < m)
          fail(fmt("could not read %s address: could not read EUI address: %s", rtype == 3 ? "EUI-48" : "EUI-64",
                   kUnexpectedEOF));
        alen = 24;  // newHWAddress(r.buf[:]) clones the whole 24-byte buffer
        memcpy(rec.addr, gobuf, 24);
        rec.alen = 24;
      } else if (rtype == 0) {
        break;
      } else {
        uint64_t m = (uint64_t)(length + padding);
        if (m > avail()) {
          if (!eof) throw NeedMore{};
          pos = n;
          fail(fmt("could not discard unknown name record: %s", kUnexpectedEOF));
        }
        pos += m;
        blen -= (uint32_t)m;
        continue;
      }
      blen -= (uint32_t)length;
      length -= alen;
      while (length > 0) {  // bufio.Reader.ReadBytes(0)
        const void* z = memchr(b + pos, 0, avail());
        if (!z) {
          if (!eof) throw NeedMore{};
          pos = n;
          fail(fmt("could not read name: %s", kEOF));
        }
        uint64_t k = (const uint8_t*)z - (b + pos) + 1;
        // string(bytes.Trim(bstr, "\x00")): the NUL is last, and NULs can only lead when the name is empty
        rec.names.emplace_back((const char*)b + pos, k - 1);
        pos += k;
        length -= (int64_t)k;
      }
      touch_names();
      names.push_back(std::move(rec));
      discard((uint64_t)padding);
    }
    discard(blen);
  }

  void read_packet_header() {
    for (;;) {  // RESTART
      for (;;) {  // FIND_PACKET
        read_block();
        if (typ == kEPB) {
          const uint8_t* h = read_gobuf(20);
          blen -= 20;
          uint32_t idx = ld32(h, be());
          if (idx >= st.ifaces.size())
            fail(fmt("Interface id %u not present in section (have only %zu interfaces)", idx, st.ifaces.size()));
          ci_iface = idx;
          convert_time(idx, (uint64_t)ld32(h + 4, be()) << 32 | ld32(h + 8, be()), &ci_s, &ci_ns);
          ci_caplen = ld32(h + 12, be());
          ci_len = ld32(h + 16, be());
          break;
        } else if (typ == kSPB) {
          const uint8_t* h = read_gobuf(4);
          blen -= 4;
          ci_s = kZeroTimeSec;
          ci_ns = 0;
          ci_iface = 0;
          ci_len = ld32(h, be());
          ci_caplen = ci_len;
          if (st.ifaces.empty()) fail("At least one Interface is needed for a packet");
          if (st.ifaces[0].snap != 0 && ci_caplen > st.ifaces[0].snap) ci_caplen = st.ifaces[0].snap;
          break;
        } else if (typ == kIDB) {
          read_interface_descriptor();
        } else if (typ == kISB) {
          read_interface_statistics();
        } else if (typ == kSHB) {
          read_section_header();
        } else if (typ == kPB) {
          const uint8_t* h = read_gobuf(20);
          blen -= 20;
          uint32_t idx = ld16(h, be());
          if (idx >= st.ifaces.size())
            fail(fmt("Interface id %u not present in section (have only %zu interfaces)", idx, st.ifaces.size()));
          ci_iface = idx;
          convert_time(idx, (uint64_t)ld32(h + 4, be()) << 32 | ld32(h + 8, be()), &ci_s, &ci_ns);
          ci_caplen = ld32(h + 12, be());
          ci_len = ld32(h + 16, be());
          break;
        } else if (typ == kNRB) {
          read_name_resolution();
        } else {
          discard(blen);
        }
      }
      if (!(flags & GPK_NG_WANT_MIXED_LINKTYPE)) {
        if (st.ifaces[ci_iface].link_type != st.link_type) {
          discard(blen);
          if (flags & GPK_NG_ERROR_ON_MISMATCHING_LINKTYPE)
            fail("Link type of current interface is different from first one");
          continue;
        }
      }
      return;
    }
  }

  void read_packet_options() {
    for (;;) {
      read_option();
      if (opt_code == 0) return;
      if ((opt_code == 2 || opt_code == 6) && opt.len < 4)  // binary.LittleEndian.Uint32: _ = b[3]
        fail(fmt("runtime error: index out of range [3] with length %u", opt.len), true);
      if ((opt_code == 4 || opt_code == 5) && opt.len < 8)  // binary.LittleEndian.Uint64: _ = b[7]
        fail(fmt("runtime error: index out of range [7] with length %u", opt.len), true);
      if (keep_opts) {  // the option as readPacketOptions saw it (its value: the reused buffer's)
        const size_t at = opt_arena.size(), padded = (opt.len + 3u) & ~3u;
        opt_arena.resize(at + 8 + padded, 0);
        uint8_t* q = opt_arena.data() + at;
        memcpy(q, &opt_code, 2);
        memcpy(q + 4, &opt.len, 4);
        memcpy(q + 8, opt.back.data(), opt.len);
      }
    }
  }

  // One ReadPacketDataWithOptions; returns the data offset in the chunk.
  uint64_t ng_read_packet() {
    read_packet_header();
    const uint64_t off = pos;
    if (ci_caplen > avail()) {
      if (!eof) throw NeedMore{};
      pos = n;
      fail(kUnexpectedEOF);
    }
    pos += ci_caplen;
    blen -= ci_caplen;
    uint32_t pad = (4 - (ci_caplen & 3)) & 3;
    if (pad > 0) discard(pad);
    if (typ == kEPB) read_packet_options();
    discard(blen);
    return off;
  }

  void ng_open() {
    if (avail() < 2) {  // reader.r.Peek(2)
      if (!eof) throw NeedMore{};
      fail(avail() > 0 ? kUnexpectedEOF : kEOF);
    }
    read_block();
    if (typ != kSHB) fail(fmt("Unknown magic %x", typ));
    read_section_header();
  }

  // ---- pcap ------------------------------------------------------------------
  void pcap_open() {
    if (avail() < 2) {  // br.Peek(2)
      if (!eof) throw NeedMore{};
      fail(kEOF);
    }
    if (avail() < 24) {  // io.ReadFull(r.r, buf[24])
      if (!eof) throw NeedMore{};
      pos = n;
      fail(kUnexpectedEOF);
    }
    const uint8_t* h = b + pos;
    pos += 24;
    uint32_t magic = ld32(h, false);
    if (magic == 0xA1B23C4D) {
      pbe = false, factor = 1;
    } else if (magic == 0x4D3CB2A1) {
      pbe = true, factor = 1;
    } else if (magic == 0xA1B2C3D4) {
      pbe = false, factor = 1000;
    } else if (magic == 0xD4C3B2A1) {
      pbe = true, factor = 1000;
    } else {
      fail(fmt("Unknown magic %x", magic));
    }
    major = ld16(h + 4, pbe);
    if (major != 2) fail(fmt("Unknown major version %u", major));
    minor = ld16(h + 6, pbe);
    if (minor != 4) fail(fmt("Unknown minor version %u", minor));
    snaplen = ld32(h + 16, pbe);
    plink = ld32(h + 20, pbe) & 0xFFFF;  // layers.LinkType is uint16
  }

  uint64_t pcap_read_packet() {
    if (avail() < 16) {  // io.ReadFull(r.r, r.buf[:16])
      if (!eof) throw NeedMore{};
      uint64_t k = avail();
      pos = n;
      fail(k == 0 ? kEOF : kUnexpectedEOF);
    }
    const uint8_t* h = b + pos;
    pos += 16;
    uint32_t sec = ld32(h, pbe), usec = ld32(h + 4, pbe);
    unix_norm((int64_t)sec, (int64_t)(uint32_t)(usec * factor), &ci_s, &ci_ns);  // uint32 product wraps
    ci_caplen = ld32(h + 8, pbe);
    ci_len = ld32(h + 12, pbe);
    ci_iface = 0;
    if (ci_caplen > snaplen) fail(fmt("capture length exceeds snap length: %u > %u", ci_caplen, snaplen));
    if (ci_caplen > ci_len) fail(fmt("capture length exceeds original packet length: %u > %u", ci_caplen, ci_len));
    const uint64_t off = pos;
    if (ci_caplen > avail()) {  // io.ReadFull(r.r, data)
      if (!eof) throw NeedMore{};
      uint64_t k = avail();
      pos = n;
      fail(k == 0 ? kEOF : kUnexpectedEOF);
    }
    pos += ci_caplen;
    return off;
  }
};

extern "C" {

int gpk_capreader_create(gpk_capreader** out, int format, uint32_t flags) {
  if (!out || (format != GPK_CAP_PCAP && format != GPK_CAP_PCAPNG)) return GPK_EINVAL;
  if (flags & ~7u) return GPK_EINVAL;
  gpk_capreader* r = new (std::nothrow) gpk_capreader();
  if (!r) return GPK_ENOMEM;
  r->format = format;
  r->flags = format == GPK_CAP_PCAPNG ? flags : 0;
  *out = r;
  return GPK_OK;
}

int gpk_capreader_destroy(gpk_capreader* r) {
  delete r;
  return GPK_OK;
}

int gpk_capreader_index(gpk_capreader* r, const uint8_t* buf, uint64_t len, int eof, uint64_t* offsets,
                        uint32_t* caplens, gpk_capture_info* ci, uint64_t max_pkts, uint64_t* n_pkts,
                        uint64_t* consumed) {
  if (!r || (!buf && len) || !offsets || !caplens || !n_pkts || !consumed) return GPK_EINVAL;
  *n_pkts = 0;
  *consumed = 0;
  if (r->keep_opts) {  // the options of this call's packets only
    r->opt_arena.clear();
    r->opt_at.assign(1, 0);
  }
  if (r->open_failed) return GPK_CAP_END;  // NewReader/NewNgReader failed: no reader
  r->b = buf;
  r->n = len;
  r->pos = 0;
  r->eof = eof != 0;
  const bool ng = r->format == GPK_CAP_PCAPNG;
  const bool mixed = (r->flags & GPK_NG_WANT_MIXED_LINKTYPE) != 0;
  uint64_t k = 0;
  int status = GPK_CAP_MORE;
  // One reference call (NewNgReader, SkipSection or ReadPacketData) at a time:
  // run() undoes everything a call changed when it needs bytes beyond buf.
  struct Undo {
    uint64_t start, m0;
    size_t ev0, oa0;
    uint8_t gb0[24];
  };
  auto begin = [r](Undo& u) {
    u.start = r->pos;
    u.m0 = r->mutations;
    u.ev0 = r->stat_events.size();
    u.oa0 = r->opt_arena.size();
    memcpy(u.gb0, r->gobuf, 24);
    r->st_saved = r->opt_saved = r->names_saved = false;
  };
  auto undo = [r](const Undo& u) {
    if (r->st_saved) r->st = std::move(r->st_snap);
    if (r->opt_saved) r->opt = std::move(r->opt_snap);
    if (r->names_saved) r->names = std::move(r->names_snap);
    r->stat_events.resize(u.ev0);
    r->opt_arena.resize(u.oa0);
    memcpy(r->gobuf, u.gb0, 24);
    r->mutations = u.m0;
    r->pos = u.start;
  };
  auto end_with = [r](const GoErr& e) {
    r->err_text = e.text;
    r->err_eof = e.text == kEOF;
    r->err_panic = e.panic;
  };
  try {
    Undo u;
    if (!r->opened) {
      begin(u);
      try {
        if (ng)
          r->ng_open();
        else
          r->pcap_open();
      } catch (NeedMore&) {
        undo(u);
        throw;
      } catch (GoErr& e) {
        r->open_failed = true;
        end_with(e);
        *consumed = r->pos;
        return GPK_CAP_END;
      }
      r->opened = true;
    }
    if (r->pending_skip) {  // NgReader.SkipSection (ngread.go:330-335)
      begin(u);
      try {
        r->skip_section();
        r->read_section_header();
        r->pending_skip = false;
      } catch (NeedMore&) {
        undo(u);
        throw;
      } catch (GoErr& e) {
        r->pending_skip = false;
        end_with(e);
        *consumed = r->pos;
        return GPK_CAP_END;
      }
    }
    for (;;) {
      if (k == max_pkts) {
        status = GPK_CAP_FULL;
        break;
      }
      begin(u);
      try {
        const uint64_t off = ng ? r->ng_read_packet() : r->pcap_read_packet();
        offsets[k] = off;
        caplens[k] = r->ci_caplen;
        if (ci) {
          ci[k].ts_sec = r->ci_s;
          ci[k].ts_nsec = r->ci_ns;
          ci[k].length = r->ci_len;
          ci[k].iface = (int32_t)r->ci_iface;
          ci[k].link_type = (ng && mixed) ? (int32_t)r->st.ifaces[r->ci_iface].link_type : -1;
        }
        k++;
        r->npk++;
        if (r->keep_opts) r->opt_at.push_back(r->opt_arena.size());
      } catch (NeedMore&) {
        undo(u);
        status = GPK_CAP_MORE;
        break;
      } catch (GoErr& e) {
        end_with(e);
        status = GPK_CAP_END;
        break;
      }
    }
  } catch (NeedMore&) {
    status = GPK_CAP_MORE;
  } catch (...) {
    return GPK_ENOMEM;
  }
  *n_pkts = k;
  *consumed = r->pos;
  return status;
}

int gpk_capreader_error(const gpk_capreader* r, char* buf, size_t cap, int* is_eof, int* is_panic) {
  if (!r) return GPK_EINVAL;
  if (is_eof) *is_eof = r->err_eof;
  if (is_panic) *is_panic = r->err_panic;
  if (buf && cap) snprintf(buf, cap, "%s", r->err_text.c_str());
  return (int)r->err_text.size();
}

int gpk_capreader_link_type(const gpk_capreader* r) {
  if (!r) return GPK_EINVAL;
  return r->format == GPK_CAP_PCAP ? (int)r->plink : (int)r->st.link_type;
}

int gpk_capreader_pcap_header(const gpk_capreader* r, uint32_t* snaplen, uint16_t* major, uint16_t* minor,
                              int* nanosecond) {
  if (!r || r->format != GPK_CAP_PCAP) return GPK_EINVAL;
  if (snaplen) *snaplen = r->snaplen;
  if (major) *major = r->major;
  if (minor) *minor = r->minor;
  if (nanosecond) *nanosecond = r->factor == 1;
  return GPK_OK;
}

int gpk_capreader_nsections(const gpk_capreader* r) {
  if (!r) return GPK_EINVAL;
  return (int)r->st.ended.size();
}

static const Section* section_at(const gpk_capreader* r, int s, const std::vector<Iface>** ifaces) {
  if (!r || r->format != GPK_CAP_PCAPNG || s < 0 || s > (int)r->st.ended.size()) return nullptr;
  if (s == (int)r->st.ended.size()) {
    *ifaces = &r->st.ifaces;
    return &r->st.section;
  }
  *ifaces = &r->st.ended[s].second;
  return &r->st.ended[s].first;
}

static int put_str(const std::string& s, char* buf, size_t cap) {
  if (buf && cap) {
    size_t m = s.size() < cap - 1 ? s.size() : cap - 1;
    memcpy(buf, s.data(), m);
    buf[m] = 0;
  }
  return (int)s.size();
}

int gpk_capreader_section_info(const gpk_capreader* r, int s, int field, char* buf, size_t cap) {
  const std::vector<Iface>* ifs;
  const Section* sec = section_at(r, s, &ifs);
  if (!sec) return GPK_EINVAL;
  switch (field) {
    case GPK_SECTION_COMMENT: return put_str(sec->comment, buf, cap);
    case GPK_SECTION_HARDWARE: return put_str(sec->hardware, buf, cap);
    case GPK_SECTION_OS: return put_str(sec->os, buf, cap);
    case GPK_SECTION_APPLICATION: return put_str(sec->application, buf, cap);
  }
  return GPK_EINVAL;
}

int gpk_capreader_ninterfaces(const gpk_capreader* r, int s) {
  const std::vector<Iface>* ifs;
  if (!section_at(r, s, &ifs)) return GPK_EINVAL;
  return (int)ifs->size();
}

int gpk_capreader_interface(const gpk_capreader* r, int s, int i, gpk_ng_interface* out) {
  const std::vector<Iface>* ifs;
  if (!section_at(r, s, &ifs) || i < 0 || i >= (int)ifs->size() || !out) return GPK_EINVAL;
  const Iface& it = (*ifs)[i];
  memset(out, 0, sizeof(*out));
  out->link_type = it.link_type;
  out->ts_resolution = it.tsres;
  out->has_statistics = it.has_stats;
  out->snap_length = it.snap;
  out->ts_offset = it.tsoff;
  out->last_update_sec = it.stats.lu_s;
  out->last_update_nsec = it.stats.lu_ns;
  out->start_time_sec = it.stats.st_s;
  out->start_time_nsec = it.stats.st_ns;
  out->end_time_sec = it.stats.et_s;
  out->end_time_nsec = it.stats.et_ns;
  out->packets_received = it.stats.received;
  out->packets_dropped = it.stats.dropped;
  return GPK_OK;
}

int gpk_capreader_interface_str(const gpk_capreader* r, int s, int i, int field, char* buf, size_t cap) {
  const std::vector<Iface>* ifs;
  if (!section_at(r, s, &ifs) || i < 0 || i >= (int)ifs->size()) return GPK_EINVAL;
  const Iface& it = (*ifs)[i];
  switch (field) {
    case GPK_IFACE_NAME: return put_str(it.name, buf, cap);
    case GPK_IFACE_COMMENT: return put_str(it.comment, buf, cap);
    case GPK_IFACE_DESCRIPTION: return put_str(it.description, buf, cap);
    case GPK_IFACE_FILTER: return put_str(it.filter, buf, cap);
    case GPK_IFACE_OS: return put_str(it.os, buf, cap);
    case GPK_IFACE_STATS_COMMENT: return put_str(it.stats.comment, buf, cap);
  }
  return GPK_EINVAL;
}

int gpk_capreader_nnames(const gpk_capreader* r) {
  if (!r || r->format != GPK_CAP_PCAPNG) return GPK_EINVAL;
  return (int)r->names.size();
}

int gpk_capreader_name(const gpk_capreader* r, int i, int* kind, uint8_t* addr, int* addr_len, int* nnames,
                       char* names, size_t cap) {
  if (!r || r->format != GPK_CAP_PCAPNG || i < 0 || i >= (int)r->names.size()) return GPK_EINVAL;
  const NameRec& x = r->names[(size_t)i];
  if (kind) *kind = x.rtype;
  if (addr) memcpy(addr, x.addr, x.alen);
  if (addr_len) *addr_len = (int)x.alen;
  if (nnames) *nnames = (int)x.names.size();
  size_t need = 0;
  for (const auto& nm : x.names) {
    if (names && need + nm.size() + 1 <= cap) {
      memcpy(names + need, nm.data(), nm.size());
      names[need + nm.size()] = 0;
    }
    need += nm.size() + 1;
  }
  return (int)need;
}

int gpk_capreader_nstat_events(const gpk_capreader* r) {
  if (!r || r->format != GPK_CAP_PCAPNG) return GPK_EINVAL;
  return (int)r->stat_events.size();
}

int gpk_capreader_stat_event(const gpk_capreader* r, int k, uint64_t* at, uint64_t* seq, int* iface,
                             gpk_ng_interface* stats, char* comment, size_t cap) {
  if (!r || r->format != GPK_CAP_PCAPNG || k < 0 || k >= (int)r->stat_events.size()) return GPK_EINVAL;
  const StatEvent& e = r->stat_events[(size_t)k];
  if (at) *at = e.at;
  if (seq) *seq = e.seq;
  if (iface) *iface = (int)e.iface;
  if (stats) {
    memset(stats, 0, sizeof(*stats));
    stats->has_statistics = 1;
    stats->last_update_sec = e.stats.lu_s;
    stats->last_update_nsec = e.stats.lu_ns;
    stats->start_time_sec = e.stats.st_s;
    stats->start_time_nsec = e.stats.st_ns;
    stats->end_time_sec = e.stats.et_s;
    stats->end_time_nsec = e.stats.et_ns;
    stats->packets_received = e.stats.received;
    stats->packets_dropped = e.stats.dropped;
  }
  return put_str(e.stats.comment, comment, cap);
}

int gpk_capreader_section_end_at(const gpk_capreader* r, int s, uint64_t* at, uint64_t* seq) {
  if (!r || r->format != GPK_CAP_PCAPNG || s < 0 || s >= (int)r->st.ended_at.size()) return GPK_EINVAL;
  if (at) *at = r->st.ended_at[(size_t)s];
  if (seq) *seq = r->st.ended_seq[(size_t)s];
  return GPK_OK;
}

int gpk_capreader_skip_section(gpk_capreader* r) {
  if (!r || r->format != GPK_CAP_PCAPNG || r->open_failed) return GPK_EINVAL;
  r->pending_skip = true;
  return GPK_OK;
}

int gpk_capreader_set_snaplen(gpk_capreader* r, uint32_t snaplen) {
  if (!r || r->format != GPK_CAP_PCAP) return GPK_EINVAL;
  r->snaplen = snaplen;
  return GPK_OK;
}

int gpk_capreader_keep_options(gpk_capreader* r, int on) {
  if (!r) return GPK_EINVAL;
  r->keep_opts = on != 0;
  r->opt_arena.clear();
  r->opt_at.assign(1, 0);
  return GPK_OK;
}

int gpk_capreader_packet_options(const gpk_capreader* r, uint64_t i, const uint8_t** tlv, uint64_t* bytes) {
  if (!r || !r->keep_opts || !tlv || !bytes || i + 1 >= r->opt_at.size()) return GPK_EINVAL;
  *tlv = r->opt_arena.data() + r->opt_at[i];
  *bytes = r->opt_at[i + 1] - r->opt_at[i];
  return GPK_OK;
}

}  // extern "C"

// ---- parallel record walk (gpk_capreader_index_all) -------------------------
// The record walk is a pointer chase through the capture: one DRAM stream per
// thread, ~4-5 GB/s. To walk a large staging slot with T threads, segments
// 1..T-1 are walked speculatively: each worker finds a plausible chain of
// plain Enhanced Packet Blocks after its segment's start and walks it. The
// exact walk (the restated reader) then runs up to each worker's start; where
// it lands exactly there with the reader state unchanged since the workers'
// snapshot, the worker's packets are what ReadPacketData would return (a plain
// EPB changes no reader state, see plain_epb) and the exact walk resumes after
// them. Anywhere else the exact walk simply continues: the result is always
// the sequential one.
namespace {

struct PktVec {  // growable, uninitialised arrays (malloc: gpk_capindex_free)
  uint64_t* off = nullptr;
  uint32_t* cap = nullptr;
  gpk_capture_info* ci = nullptr;
  uint64_t n = 0, room = 0;
  bool reserve(uint64_t m) {
    if (m <= room) return true;
    uint64_t r = room ? room : 4096;
    while (r < m) r *= 2;
    void* a = realloc(off, r * 8);
    if (!a) return false;
    off = (uint64_t*)a;
    void* c = realloc(cap, r * 4);
    if (!c) return false;
    cap = (uint32_t*)c;
    void* d = realloc(ci, r * sizeof(gpk_capture_info));
    if (!d) return false;
    ci = (gpk_capture_info*)d;
    room = r;
    return true;
  }
  void release() {
    free(off);
    free(cap);
    free(ci);
    off = nullptr;
    cap = nullptr;
    ci = nullptr;
    n = room = 0;
  }
};

// CPUs this process may actually run on at once: the affinity mask, a cgroup
// CPU quota (v2 cpu.max, v1 cfs_quota_us / cfs_period_us) and OMP_NUM_THREADS
// when set. A GPU box gives a process a quota of a few cores of a large
// machine whose every CPU is in its mask: threads beyond the quota exhaust it
// and are then all throttled until the next scheduler period.
unsigned usable_cpus() {
  unsigned n = std::thread::hardware_concurrency();
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) {
    const int c = CPU_COUNT(&set);
    if (c > 0 && (unsigned)c < n) n = (unsigned)c;
  }
  auto quota = [](const char* qf, const char* pf) -> long {  // ceil(quota / period), 0 = none
    long q = 0, p = 0;
    if (FILE* f = fopen(qf, "r")) {
      char buf[64] = {0};
      if (fgets(buf, sizeof(buf), f)) {
        if (!pf) {  // v2: "quota period" or "max period"
          if (sscanf(buf, "%ld %ld", &q, &p) != 2) q = 0;
        } else {
          q = strtol(buf, nullptr, 10);
        }
      }
      fclose(f);
    }
    if (pf) {
      if (FILE* f = fopen(pf, "r")) {
        if (fscanf(f, "%ld", &p) != 1) p = 0;
        fclose(f);
      }
    }
    return q > 0 && p > 0 ? (q + p - 1) / p : 0;
  };
  long c = quota("/sys/fs/cgroup/cpu.max", nullptr);
  if (!c) c = quota("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "/sys/fs/cgroup/cpu/cpu.cfs_period_us");
  if (c > 0 && (unsigned long)c < n) n = (unsigned)c;
  if (const char* e = getenv("OMP_NUM_THREADS")) {
    const long o = strtol(e, nullptr, 10);
    if (o > 0 && (unsigned long)o < n) n = (unsigned)o;
  }
  return n ? n : 1;
}

// Persistent worker threads for the walk (one set per process, created on
// first use, one per usable CPU): a staging slot is walked every few
// milliseconds, and spawning dozens of threads per slot cost about as much as
// the walk itself.
class Pool {
 public:
  static Pool& get() {
    static Pool p;
    return p;
  }
  // f(0) .. f(n-1) on the pool's threads and the caller's; returns when all are done.
  // The pool is process-wide and holds one job at a time: callers on other
  // threads (two replays, two readers, ctypes calls that release the GIL)
  // queue here until the running job has finished; f must not call run().
  void run(int n, const std::function<void(int)>& f) {
    if (n <= 0) return;
    std::lock_guard<std::mutex> one_job(run_mu_);
    std::unique_lock<std::mutex> lk(mu_);
    job_ = &f;
    next_ = 0;
    total_ = n;
    left_ = n;
    gen_++;
    cv_.notify_all();
    lk.unlock();
    work();
    lk.lock();
    done_.wait(lk, [&] { return left_ == 0; });
    job_ = nullptr;
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }

 private:
  Pool() {
    unsigned n = usable_cpus();
    n = n < 2 ? 2 : (n > 64 ? 64 : n);
    for (unsigned k = 0; k + 1 < n; k++) th_.emplace_back([this] { loop(); });
  }
  void work() {  // take tasks of the current job until none is left
    for (;;) {
      std::unique_lock<std::mutex> lk(mu_);
      if (!job_ || next_ >= total_) return;
      const int k = next_++;
      const std::function<void(int)>* f = job_;
      lk.unlock();
      (*f)(k);
      lk.lock();
      if (--left_ == 0) done_.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      work();
    }
  }
  std::vector<std::thread> th_;
  std::mutex run_mu_;  // held for a whole job
  std::mutex mu_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* job_ = nullptr;
  int next_ = 0, total_ = 0, left_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// What ReadPacketData does on a plain EPB at b[p] (ngread.go:494-514, 642-675):
// block header; 20-byte EPB header; interface known (else an error) and, without
// WantMixedLinkType, of the first interface's link type (else the block is
// skipped); data + padding; the 4 bytes left make readOption return end of
// options at once (ngread.go:197-201); discard(4). No state changes. "Plain":
// total length == 32 + caplen + padding (no options) and the block inside
// b[p, end). Returns the block length, 0 for anything else.
uint32_t plain_epb(const NgState& st, uint32_t flags, const uint8_t* b, uint64_t p, uint64_t end, uint64_t* off,
                   uint32_t* cap, gpk_capture_info* ci) {
  if (end - p < 32) return 0;
  const bool be = st.be;
  const uint8_t* h = b + p;
  if (ld32(h, be) != kEPB) return 0;
  const uint32_t L = ld32(h + 4, be), idx = ld32(h + 8, be), cl = ld32(h + 20, be);
  if (idx >= st.ifaces.size()) return 0;
  if ((uint64_t)L != 32ull + cl + ((4u - (cl & 3u)) & 3u) || L > end - p) return 0;
  const Iface& it = st.ifaces[idx];
  const bool mixed = (flags & GPK_NG_WANT_MIXED_LINKTYPE) != 0;
  if (!mixed && it.link_type != st.link_type) return 0;
  if (ci) {
    gpk_capreader::iface_time(it, (uint64_t)ld32(h + 12, be) << 32 | ld32(h + 16, be), &ci->ts_sec, &ci->ts_nsec);
    ci->length = ld32(h + 24, be);
    ci->iface = (int32_t)idx;
    ci->link_type = mixed ? (int32_t)it.link_type : -1;
  }
  *off = p + 28;
  *cap = cl;
  return L;
}

// First p in [from, to), p = ref (mod 4) (blocks are 4-byte multiples), where
// four plain EPBs with matching trailers follow each other.
uint64_t find_sync(const NgState& st, uint32_t flags, const uint8_t* b, uint64_t from, uint64_t to, uint64_t end,
                   uint64_t ref) {
  for (uint64_t p = from + ((ref - from) & 3); p < to; p += 4) {
    uint64_t q = p, o;
    uint32_t c;
    int k = 0;
    for (; k < 4; k++) {
      const uint32_t L = plain_epb(st, flags, b, q, end, &o, &c, nullptr);
      if (!L || ld32(b + q + L - 4, st.be) != L) break;
      q += L;
    }
    if (k == 4) return p;
  }
  return ~0ull;
}

struct Seg {
  uint64_t sync = ~0ull, end = 0;
  PktVec v;
};

void walk_seg(const NgState& st, uint32_t flags, const uint8_t* b, uint64_t p, uint64_t seg_end, uint64_t end,
              Seg& s) {
  s.sync = p;
  while (p < seg_end && s.v.reserve(s.v.n + 1)) {
    const uint32_t L = plain_epb(st, flags, b, p, end, &s.v.off[s.v.n], &s.v.cap[s.v.n], &s.v.ci[s.v.n]);
    if (!L) break;
    s.v.n++;
    p += L;
  }
  s.end = p;
}

// Exact walk: ReadPacketData calls over b[from, to); *stop = where the next
// call starts. Returns GPK_CAP_MORE / GPK_CAP_END or a negative status.
int seq_walk(gpk_capreader* r, const uint8_t* b, uint64_t from, uint64_t to, int eof, PktVec& v, uint64_t* stop) {
  uint64_t pos = from;
  for (;;) {
    const uint64_t room = 1u << 16;
    if (!v.reserve(v.n + room)) return GPK_ENOMEM;
    uint64_t k = 0, used = 0;
    const int st = gpk_capreader_index(r, b + pos, to - pos, eof, v.off + v.n, v.cap + v.n, v.ci + v.n, room, &k, &used);
    if (st < 0) return st;
    for (uint64_t i = 0; i < k; i++) v.off[v.n + i] += pos;
    v.n += k;
    pos += used;
    if (st != GPK_CAP_FULL) {
      *stop = pos;
      return st;
    }
  }
}

uint64_t state_version(const gpk_capreader* r) {  // anything plain_epb depends on changes one of these
  return (uint64_t)r->st.ended.size() << 32 | r->st.ifaces.size();
}

}  // namespace

// The reader state the device walk needs (gpk_walk.h): the same inputs as
// plain_epb, taken where the host walk would take its workers' snapshot.
bool gpk_capreader_walk_state(const gpk_capreader* r, gpk::WalkState* out) {
  if (!r || !out || r->format != GPK_CAP_PCAPNG || !r->opened || r->open_failed) return false;
  const NgState& st = r->st;
  if (st.ifaces.size() > (size_t)gpk::kWalkMaxIf) return false;
  memset(out, 0, sizeof(*out));
  out->be = st.be;
  out->mixed = (r->flags & GPK_NG_WANT_MIXED_LINKTYPE) != 0;
  out->nif = (uint32_t)st.ifaces.size();
  for (size_t i = 0; i < st.ifaces.size(); i++) {
    const Iface& it = st.ifaces[i];
    gpk::WalkIface& w = out->ifc[i];
    w.second_mask = it.second_mask;
    w.scale_up = it.scale_up;
    w.scale_down = it.scale_down;
    w.tsoff = it.tsoff;
    w.link_type = it.link_type;
    w.plain = it.second_mask != 0 && (out->mixed || it.link_type == st.link_type);
  }
  return true;
}

// The byte-range replay (gpk_replay_file_range): where a range's first block
// lies, by the same rule as the speculative walk (four chained plain EPBs
// under the reader's current state), and the reader-state version that tells
// whether a range changed what the next one assumed.
uint64_t gpk_capreader_sync(const gpk_capreader* r, const uint8_t* b, uint64_t from, uint64_t to, uint64_t end,
                            uint64_t span) {
  if (!r || r->format != GPK_CAP_PCAPNG || !r->opened || r->open_failed) return ~0ull;
  for (uint64_t p = (from + 3) & ~3ull; p < to; p += 4) {  // the chain inside [p, p + span): a property of p alone
    const uint64_t e = std::min<uint64_t>(end, p + span);
    if (find_sync(r->st, r->flags, b, p, p + 1, e, p) == p) return p;
  }
  return ~0ull;
}

uint64_t gpk_capreader_mutations(const gpk_capreader* r) { return r ? r->mutations : 0; }

uint64_t gpk_capreader_state_version(const gpk_capreader* r) {
  if (!r || r->format != GPK_CAP_PCAPNG || !r->opened || r->open_failed) return 0;
  return state_version(r) | 1ull << 63;  // nonzero once open
}

extern "C" int gpk_capreader_index_all(gpk_capreader* r, const uint8_t* buf, uint64_t len, int eof, int threads,
                                       gpk_capindex* out, uint64_t* consumed) {
  if (!r || (!buf && len) || !out || !consumed) return GPK_EINVAL;
  memset(out, 0, sizeof(*out));
  *consumed = 0;
  PktVec v;
  uint64_t pos = 0, stop = 0;
  int st = GPK_CAP_MORE;
  bool done = false;
  try {
    if (r->format == GPK_CAP_PCAPNG && threads > 1 && len >= (1u << 20) && !r->open_failed) {
      if (!r->opened) {  // NewNgReader (section header, first interface) first
        const uint64_t pre = len < (1u << 16) ? len : (1u << 16);
        st = seq_walk(r, buf, 0, pre, pre == len ? eof : 0, v, &stop);
        pos = stop;
        done = st != GPK_CAP_MORE || pre == len;
      }
      if (!done && r->opened) {
        const NgState snap = r->st;
        const uint64_t ver = state_version(r), span = len - pos, base = pos;
        const int T = threads > 64 ? 64 : threads;
        std::vector<Seg> seg(T);
        PktVec tail;  // exact-walk packets between and after the segments
        auto fail_all = [&](int code) {
          for (auto& sg : seg) sg.v.release();
          tail.release();
          v.release();
          return code;
        };
        // task 0: the exact walk of the first segment (it alone mutates the
        // reader; the workers use the snapshot); tasks 1..T-1: speculative
        int st0 = GPK_CAP_MORE;
        uint64_t stop0 = pos;
        Pool::get().run(T, [&](int k) {
          if (k == 0) {
            st0 = seq_walk(r, buf, pos, base + span / T, 0, v, &stop0);
            return;
          }
          const uint64_t s0 = base + span * k / T, s1 = k + 1 < T ? base + span * (k + 1) / T : len;
          const uint64_t to = s1 < s0 + (1u << 20) ? s1 : s0 + (1u << 20);
          const uint64_t p = find_sync(snap, r->flags, buf, s0, to, len, base);
          if (p != ~0ull) walk_seg(snap, r->flags, buf, p, s1, len, seg[k]);
        });
        st = st0;
        pos = stop0;
        if (st < 0) return fail_all(st);
        if (st != GPK_CAP_MORE) done = true;
        // Stitch in order: the exact walk runs up to each accepted segment's
        // start (normally nothing is left to walk), the segment's packets
        // follow. Pieces are copied into the result in parallel afterwards.
        struct Piece {
          const PktVec* src;  // nullptr: v itself
          uint64_t from, n, at;
        };
        std::vector<Piece> pieces;
        uint64_t total = v.n;
        pieces.push_back({nullptr, 0, v.n, 0});
        for (int k = 1; k < T && !done; k++) {
          Seg& s = seg[k];
          if (s.sync == ~0ull || s.sync < pos) continue;
          const uint64_t t0 = tail.n;
          st = seq_walk(r, buf, pos, s.sync, 0, tail, &stop);
          if (st < 0) return fail_all(st);
          pos = stop;
          if (tail.n > t0) {
            pieces.push_back({&tail, t0, tail.n - t0, total});
            total += tail.n - t0;
          }
          if (st != GPK_CAP_MORE) {
            done = true;
          } else if (pos == s.sync && state_version(r) == ver) {
            pieces.push_back({&s.v, 0, s.v.n, total});
            total += s.v.n;
            pos = s.end;
            // what the exact reader would have left: the packets counted, and
            // NgReader.buf holding the last block's 20-byte EPB header
            r->npk += s.v.n;
            if (s.v.n) r->to_gobuf(0, buf + s.v.off[s.v.n - 1] - 20, 20);
          }
        }
        if (!done) {  // the rest of the slot, exactly
          const uint64_t t0 = tail.n;
          st = seq_walk(r, buf, pos, len, eof, tail, &stop);
          if (st < 0) return fail_all(st);
          pos = stop;
          if (tail.n > t0) {
            pieces.push_back({&tail, t0, tail.n - t0, total});
            total += tail.n - t0;
          }
          done = true;
        }
        PktVec out_v;
        if (!out_v.reserve(total ? total : 1)) return fail_all(GPK_ENOMEM);
        Pool::get().run((int)pieces.size(), [&](int k) {
          const Piece& pc = pieces[k];
          const PktVec& src = pc.src ? *pc.src : v;
          memcpy(out_v.off + pc.at, src.off + pc.from, pc.n * 8);
          memcpy(out_v.cap + pc.at, src.cap + pc.from, pc.n * 4);
          memcpy(out_v.ci + pc.at, src.ci + pc.from, pc.n * sizeof(gpk_capture_info));
        });
        out_v.n = total;
        for (auto& sg : seg) sg.v.release();
        tail.release();
        v.release();
        v = out_v;
      }
    }
    if (!done) {
      st = seq_walk(r, buf, pos, len, eof, v, &stop);
      pos = stop;
    }
  } catch (...) {
    v.release();
    return GPK_ENOMEM;
  }
  if (st < 0) {
    v.release();
    return st;
  }
  out->n = v.n;
  out->offsets = v.off;
  out->caplens = v.cap;
  out->ci = v.ci;
  *consumed = pos;
  return st;
}

extern "C" int gpk_capindex_free(gpk_capindex* x) {
  if (!x) return GPK_EINVAL;
  free(x->offsets);
  free(x->caplens);
  free(x->ci);
  memset(x, 0, sizeof(*x));
  return GPK_OK;
}

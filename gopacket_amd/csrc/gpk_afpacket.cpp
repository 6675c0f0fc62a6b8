// gpk_afpacket.cpp — AF_PACKET ring reader and the ring → HBM capture loop
// (include/gpk_afpacket.h).
//
// The reader restates afpacket.TPacket.ZeroCopyReadPacketData
// (afpacket/afpacket.go:335-367) over the three header layouts of
// afpacket/header.go: the same ring position arithmetic (getTPacketHeader
// :469-492), the same release-when-moving-on rule (releaseCurrentPacket
// :316-321), the same "empty block" retry, the same v3 next-packet step
// (header.go:254-268) and the same VLAN-header insertion (:147-155).
// Differences are confined to what a batch interface must change:
//   * where the reference blocks in poll(2), the walk stops (GPK_TP_WAIT) and
//     resumes exactly there on the next call;
//   * with deferred release, a finished header is handed back only once the
//     pump's copy of it has reached HBM;
//   * accesses the reference would make outside the ring (a corrupt chain)
//     are reported as an error instead of faulting.
//
// The capture loop (gpk_tpacket_pump) keeps a device mirror of the ring:
// a header's bytes go to the same offset in HBM, so the packet offsets the
// walk produces index the mirror directly and a V3 block is copied once, as
// one contiguous DMA, no matter how many packets it holds.
#include <hip/hip_runtime.h>
#include <errno.h>
#include <net/if.h>
#include <poll.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <unistd.h>
#include <linux/if_packet.h>
#include <linux/filter.h>
#include <arpa/inet.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <cstdio>
#include <cstring>
#include <deque>
#include <string>
#include <thread>
#include <vector>

#include "gpk_pinned.h"
#include "gpk_devguard.h"
#include "../../include/gpk_afpacket.h"

extern "C" int gpk_decode_batch_ex(gpk_ctx* c, const gpk_parser* p, const gpk_batch* b, const gpk_results* o,
                                   void* stream, uint64_t packet_bytes, char* kname, size_t kcap,
                                   gpk_fields* fields);

namespace {

constexpr uint32_t kStatusUser = 1;        // TP_STATUS_USER
constexpr uint32_t kStatusVlanValid = 0x10; // TP_STATUS_VLAN_VALID
constexpr uint64_t kAlign = 16;            // TPACKET_ALIGNMENT
constexpr int64_t kPageSize = 4096;

inline uint64_t tp_align(uint64_t x) { return (x + kAlign - 1) & ~(kAlign - 1); }
template <class T>
inline T ld(const uint8_t* p) {
  T v;
  memcpy(&v, p, sizeof(T));
  return v;
}
inline uint32_t ld_status_acquire(const uint8_t* p) {
  return __atomic_load_n(reinterpret_cast<const uint32_t*>(p), __ATOMIC_ACQUIRE);
}

// time.Unix(sec, nsec) normalisation (Go time.go)
inline void go_unix(int64_t sec, int64_t nsec, int64_t* os, uint32_t* ons) {
  if (nsec < 0 || nsec >= 1000000000) {
    int64_t n = nsec / 1000000000;
    sec += n;
    nsec -= n * 1000000000;
    if (nsec < 0) {
      nsec += 1000000000;
      sec--;
    }
  }
  *os = sec;
  *ons = (uint32_t)nsec;
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Header sizes (header.go:135-137) and the sockaddr_ll that follows each.
constexpr uint64_t kV1Hdr = 0x20, kV2Hdr = 0x20, kV3Hdr = 0x30;

// A fixed set of worker threads that run one function per call: the
// pre-walk runs on every large index call, so spawning threads there would
// cost as much as the walk of a few blocks.
class Pool {
 public:
  ~Pool() {
    {
      std::lock_guard<std::mutex> l(m_);
      stop_ = true;
      gen_++;
    }
    cv_.notify_all();
    for (auto& x : th_) x.join();
  }
  // fn(w, T) on workers w = 0..T-1; returns when all are done
  void run(int T, const std::function<void(int, int)>& fn) {
    while ((int)th_.size() < T) {
      const int w = (int)th_.size();
      th_.emplace_back([this, w] { loop(w); });
    }
    std::unique_lock<std::mutex> l(m_);
    fn_ = &fn;
    T_ = T;
    left_ = T;
    gen_++;
    cv_.notify_all();
    done_.wait(l, [this] { return left_ == 0; });
    fn_ = nullptr;
  }

 private:
  void loop(int w) {
    uint64_t seen = 0;
    for (;;) {
      std::unique_lock<std::mutex> l(m_);
      cv_.wait(l, [&] { return gen_ != seen; });
      seen = gen_;
      if (stop_) return;
      if (w >= T_) continue;
      const std::function<void(int, int)>* f = fn_;
      const int T = T_;
      l.unlock();
      (*f)(w, T);
      l.lock();
      if (--left_ == 0) done_.notify_one();
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void(int, int)>* fn_ = nullptr;
  int T_ = 0, left_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// Go-side reader state that one ZeroCopyReadPacketData call mutates.
struct GoState {
  int64_t offset = 0;             // TPacket.offset
  bool have_current = false;      // TPacket.current != nil
  uint64_t cur_hdr = 0;           // header index of current
  uint64_t pkt = 0;               // ring position of the current packet header (v3 w.packet; v1/v2 = header)
  uint32_t used = 0;              // v3wrapper.used
  bool header_next_needed = false;
  bool should_release = false;
  bool polling = false;           // stopped inside pollForFirstPacket (batch form only)
  int64_t packets = 0, polls = 0; // Stats
};

}  // namespace

struct gpk_tpacket {
  uint8_t* ring = nullptr;
  uint64_t bytes = 0;
  int version = GPK_TPACKET_V3;
  gpk_tp_opts o{};
  int fd = -1;
  int ifindex = 0;  // the interface bound to (0: every interface), for SetPromiscuous
  bool mapped = false;
  uint64_t hdr_bytes = 0, nhdr = 0;
  GoState s;
  // deferred release
  bool defer = false;
  std::vector<uint8_t> pending;  // header is finished but not handed back yet
  std::deque<std::pair<uint64_t, uint64_t>> pq;  // (release seq, header)
  uint64_t rel_seq = 0;
  // headers first read since gpk_tpacket_take_new_headers
  std::vector<uint8_t> fresh;  // header must be counted as new when next read
  uint64_t new_first = 0, new_count = 0;
  // last error
  std::string err;
  bool panic = false, dead = false;
  // SocketStats accumulators
  uint32_t ss_packets = 0, ss_drops = 0, ss_freeze = 0;
  // V3 blocks walked ahead in parallel (prewalk), valid for one index call
  struct Pre {
    uint64_t epoch = 0;
    bool direct = false;  // written to the caller's arrays at pred
    uint64_t pred = 0;
    uint32_t n = 0;
    uint64_t first_off = 0, first_pos = 0, last_pos = 0;
    std::vector<uint64_t> off, pos;
    std::vector<uint32_t> cap;
    std::vector<gpk_tp_info> ci;
  };
  std::vector<Pre> pre;
  uint64_t epoch = 0;
  int threads = 16;
  Pool pool;
};

namespace {

uint64_t header_pos(const gpk_tpacket* t, uint64_t h) { return h * t->hdr_bytes; }

uint32_t header_status(const gpk_tpacket* t, uint64_t h) {
  const uint8_t* p = t->ring + header_pos(t, h);
  // v1 tp_status is an unsigned long; only its low word carries TP_STATUS_USER
  // on little-endian, and getStatus() returns int(tp_status)
  return t->version == GPK_TPACKET_V3 ? ld_status_acquire(p + 8) : ld_status_acquire(p);
}

void clear_status(gpk_tpacket* t, uint64_t h) {  // clearStatus (header.go:163-165,189-191,235-237)
  uint8_t* p = t->ring + header_pos(t, h);
  if (t->version == GPK_TPACKET_V3) {
    __atomic_store_n(reinterpret_cast<uint32_t*>(p + 8), 0u, __ATOMIC_RELEASE);
  } else if (t->version == GPK_TPACKET_V2) {
    __atomic_store_n(reinterpret_cast<uint32_t*>(p), 0u, __ATOMIC_RELEASE);
  } else {
    __atomic_store_n(reinterpret_cast<uint64_t*>(p), (uint64_t)0, __ATOMIC_RELEASE);
  }
}

// One ZeroCopyReadPacketData call. Returns 1 = a packet, 0 = wait, -1 = error,
// -2 = no room in the side buffer (state untouched by the caller's snapshot).
struct Call {
  gpk_tpacket* t;
  std::vector<uint64_t>* releases;  // headers released by this call, in order
  std::vector<uint64_t>* fresh_hdrs;
  bool wait;
  uint8_t* side;
  uint64_t side_cap, side_used;
  // outputs
  uint64_t off = 0;
  uint32_t caplen = 0;
  gpk_tp_info ci{};

  bool in_ring(uint64_t pos, uint64_t len) const { return pos <= t->bytes && len <= t->bytes - pos; }
  int fault(uint64_t pos) {
    char b[96];
    snprintf(b, sizeof(b), "unexpected fault address (ring offset %llu)", (unsigned long long)pos);
    t->err = b;
    t->panic = true;
    t->dead = true;
    return -1;
  }

  // getTPacketHeader (afpacket.go:462-486)
  int get_header() {
    GoState& s = t->s;
    if (t->version == GPK_TPACKET_V3) {
      if (s.offset >= t->o.num_blocks) s.offset = 0;
    } else if (s.offset >= (int64_t)t->o.frames_per_block * t->o.num_blocks) {
      s.offset = 0;
    }
    s.cur_hdr = (uint64_t)s.offset;
    s.have_current = true;
    const uint64_t pos = header_pos(t, s.cur_hdr);
    if (t->version == GPK_TPACKET_V3) {  // initV3Wrapper (header.go:217-222)
      if (!in_ring(pos, 48)) return fault(pos);
      s.pkt = pos + ld<uint32_t>(t->ring + pos + 16);  // offset_to_first_pkt
      s.used = 0;
    } else {
      s.pkt = pos;
    }
    return 0;
  }

  // the v3 next() step (header.go:254-268); v1/v2 next() is always false
  bool next() {
    GoState& s = t->s;
    if (t->version != GPK_TPACKET_V3) return false;
    s.used++;
    const uint32_t num_pkts = ld<uint32_t>(t->ring + header_pos(t, s.cur_hdr) + 12);
    if (s.used >= num_pkts) return false;
    const uint8_t* p = t->ring + s.pkt;
    const uint32_t next_off = ld<uint32_t>(p);
    if (next_off != 0) {
      s.pkt += next_off;
    } else {
      const uint32_t snap = ld<uint32_t>(p + 12);
      const uint16_t mac = ld<uint16_t>(p + 24);
      s.pkt += tp_align((uint64_t)snap + mac);
    }
    return true;
  }

  void release_current() {  // releaseCurrentPacket (afpacket.go:316-321)
    releases->push_back(t->s.cur_hdr);
    t->s.offset++;
    t->s.should_release = false;
  }

  // pollForFirstPacket (afpacket.go:488-516): 1 = ready, 0 = wait, -1 = error
  int poll_first() {
    GoState& s = t->s;
    const uint64_t h = s.cur_hdr;
    for (;;) {
      const bool deferred = t->defer && t->pending[h];
      // released earlier in this same step (the walk went round the ring over
      // empty headers): the reference's release has already handed it to the
      // kernel, so it is not the user's; the release is committed when this
      // step returns, and the next call polls it
      const bool released_now = std::find(releases->begin(), releases->end(), h) != releases->end();
      if (!deferred && !released_now && (header_status(t, h) & kStatusUser)) break;
      if (!wait || released_now) {
        s.polling = true;
        return 0;
      }
      const int tm = (int)(t->o.poll_timeout_ns / 1000000);
      if (t->fd < 0) {  // an attached ring: spin for the producer, bounded by the poll timeout
        const double t0 = now_s();
        bool ready = false;
        while (!ready) {
          ready = !(t->defer && t->pending[h]) && (header_status(t, h) & kStatusUser);
          if (ready) break;
          if (t->defer && t->pending[h]) {  // only gpk_tpacket_release can hand it back
            s.polling = true;
            return 0;
          }
          if (tm >= 0 && (now_s() - t0) * 1e3 >= tm) break;
          sched_yield();
        }
        if (!ready) {
          t->err = "packet poll timeout expired";
          return -1;
        }
        s.polls++;
        continue;
      }
      struct pollfd pfd{t->fd, POLLIN, 0};
      int n = ::poll(&pfd, 1, tm);
      int e = n < 0 ? errno : 0;
      if (n == 0) {
        t->err = "packet poll timeout expired";  // ErrTimeout
        return -1;
      }
      s.polls++;
      if (pfd.revents & POLLERR) {
        t->err = "packet poll failed";  // ErrPoll
        return -1;
      }
      if (e == EINTR) continue;
      if (n < 0) {
        t->err = strerror(e);
        return -1;
      }
    }
    s.polling = false;
    s.should_release = true;
    if (t->fresh[h]) {
      t->fresh[h] = 0;
      fresh_hdrs->push_back(h);
    }
    return 1;
  }

  uint64_t hdr_size() const { return t->version == GPK_TPACKET_V3 ? kV3Hdr : (t->version == GPK_TPACKET_V2 ? kV2Hdr : kV1Hdr); }

  uint32_t get_length() const {
    const uint8_t* p = t->ring + t->s.pkt;
    return t->version == GPK_TPACKET_V3 ? ld<uint32_t>(p + 16) : (t->version == GPK_TPACKET_V2 ? ld<uint32_t>(p + 4)
                                                                                               : ld<uint32_t>(p + 8));
  }

  int run() {
    GoState& s = t->s;
    if (s.polling) goto poll;  // resume inside pollForFirstPacket
  retry:
    if (!s.have_current || !s.header_next_needed || !next()) {
      if (s.should_release) release_current();
      if (get_header() < 0) return -1;
    poll:
      int r = poll_first();
      if (r <= 0) {
        if (r < 0) {
          s.header_next_needed = false;
          s.polling = false;
        }
        return r;
      }
      if (!in_ring(s.pkt, hdr_size())) return fault(s.pkt);
      if (get_length() == 0) goto retry;  // "We received an empty block"
    }
    if (!in_ring(s.pkt, hdr_size())) return fault(s.pkt);
    // getData / getTime / getLength / getIfaceIndex / getVLAN
    const uint8_t* p = t->ring + s.pkt;
    uint32_t snap, tci = 0;
    uint16_t mac;
    int64_t sec, nsec;
    int32_t vlan = -1;
    uint64_t ll;
    if (t->version == GPK_TPACKET_V3) {
      snap = ld<uint32_t>(p + 12);
      mac = ld<uint16_t>(p + 24);
      sec = ld<uint32_t>(p + 4);
      nsec = ld<uint32_t>(p + 8);
      tci = ld<uint32_t>(p + 32);  // tpacketHdrVarient1.vlanTCI
      if (ld<uint32_t>(p + 20) & kStatusVlanValid) vlan = (int32_t)(tci & 0xfff);
      ll = s.pkt + tp_align(kV3Hdr);
    } else if (t->version == GPK_TPACKET_V2) {
      snap = ld<uint32_t>(p + 8);
      mac = ld<uint16_t>(p + 12);
      sec = ld<uint32_t>(p + 16);
      nsec = ld<uint32_t>(p + 20);
      tci = ld<uint16_t>(p + 24);
      ll = s.pkt + tp_align(kV2Hdr);
    } else {
      snap = ld<uint32_t>(p + 12);
      mac = ld<uint16_t>(p + 16);
      sec = ld<uint32_t>(p + 20);
      nsec = (int64_t)ld<uint32_t>(p + 24) * 1000;
      ll = s.pkt + tp_align(kV1Hdr);
    }
    const uint64_t dpos = s.pkt + mac;
    if (!in_ring(dpos, snap)) return fault(dpos);
    if (!in_ring(ll, 8)) return fault(ll);
    if (t->version != GPK_TPACKET_V1 && tci != 0 && t->o.add_vlan_header) {  // insertVlanHeader
      if (snap < 12) {
        char b[96];
        snprintf(b, sizeof(b), "runtime error: slice bounds out of range [:12] with capacity %u", snap);
        t->err = b;
        t->panic = true;
        t->dead = true;
        return -1;
      }
      const uint64_t need = (uint64_t)snap + 4;
      if (!side || side_cap - side_used < need) return -2;
      uint8_t* d = side + side_used;
      memcpy(d, t->ring + dpos, 12);
      d[12] = 0x81;
      d[13] = 0;
      d[14] = (uint8_t)((tci >> 8) & 0xff);
      d[15] = (uint8_t)(tci & 0xff);
      memcpy(d + 16, t->ring + dpos + 12, snap - 12);
      off = t->bytes + side_used;
      caplen = (uint32_t)need;
      side_used += need;
    } else {
      off = dpos;
      caplen = snap;
    }
    go_unix(sec, nsec, &ci.ts_sec, &ci.ts_nsec);
    ci.length = get_length();
    ci.iface = ld<int32_t>(t->ring + ll + 4);  // sockaddr_ll.sll_ifindex
    ci.vlan = vlan;
    s.packets++;
    s.header_next_needed = true;
    return 1;
  }
};

void commit_releases(gpk_tpacket* t, const std::vector<uint64_t>& rel) {
  for (uint64_t h : rel) {
    t->fresh[h] = 1;
    if (t->defer) {
      t->pending[h] = 1;
      t->pq.emplace_back(t->rel_seq, h);
    } else {
      clear_status(t, h);
    }
    t->rel_seq++;
  }
}

void commit_fresh(gpk_tpacket* t, const std::vector<uint64_t>& fr) {
  for (uint64_t h : fr) {
    if (t->new_count == 0) t->new_first = h;
    t->new_count++;
  }
}

int init_geometry(gpk_tpacket* t) {
  const gpk_tp_opts& o = t->o;
  if (t->version == GPK_TPACKET_V3) {
    t->hdr_bytes = (uint64_t)o.frame_size * o.frames_per_block;
    t->nhdr = (uint64_t)o.num_blocks;
  } else {
    t->hdr_bytes = (uint64_t)o.frame_size;
    t->nhdr = (uint64_t)o.frames_per_block * o.num_blocks;
  }
  if (t->hdr_bytes * t->nhdr > t->bytes) return GPK_EINVAL;
  t->pending.assign(t->nhdr, 0);
  t->fresh.assign(t->nhdr, 1);
  if (t->version == GPK_TPACKET_V3) t->pre.resize(t->nhdr);
  return GPK_OK;
}

// Walk V3 blocks the way consecutive ZeroCopyReadPacketData calls would,
// from each one's first packet to its last, without touching the reader's
// state. A walk is valid only for a block the reference would read packet by
// packet with no special case (handed over, not deferred, a non-empty first
// packet, every header and byte inside the ring, no VLAN header to insert).
// The chain inside a block is a dependent load per packet; G blocks are
// walked in lockstep so that G loads are in flight at once.
struct Chain {
  gpk_tpacket::Pre* P;
  uint64_t pos;
  uint32_t k, n;
  bool live;
  uint64_t* off;  // where the block's packets go: the caller's arrays at the
  uint32_t* cap;  // predicted position (direct), or the block's own arrays
  gpk_tp_info* ci;
  uint64_t* posv;  // header positions (own arrays only)
};

bool chain_start(gpk_tpacket* t, uint64_t h, Chain& c) {
  c.live = false;
  if (t->pending[h] || !(header_status(t, h) & kStatusUser)) return false;
  const uint64_t base = header_pos(t, h);
  c.n = ld<uint32_t>(t->ring + base + 12);
  if (c.n == 0) return false;
  gpk_tpacket::Pre& P = *c.P;
  if (!P.direct) {
    P.off.resize(c.n);
    P.pos.resize(c.n);
    P.cap.resize(c.n);
    P.ci.resize(c.n);
    c.off = P.off.data();
    c.cap = P.cap.data();
    c.ci = P.ci.data();
    c.posv = P.pos.data();
  }
  c.pos = base + ld<uint32_t>(t->ring + base + 16);
  c.k = 0;
  c.live = true;
  return true;
}

// one packet of a chain: false when the chain ended (done or refused)
inline bool chain_step(const gpk_tpacket* t, Chain& c, bool& ok) {
  const uint64_t pos = c.pos;
  if (pos > t->bytes || t->bytes - pos < kV3Hdr + 8 + 4) return ok = false;  // header + sockaddr_ll ifindex
  const uint8_t* p = t->ring + pos;
  const uint32_t snap = ld<uint32_t>(p + 12), len = ld<uint32_t>(p + 16), st = ld<uint32_t>(p + 20);
  const uint16_t mac = ld<uint16_t>(p + 24);
  const uint32_t tci = ld<uint32_t>(p + 32);
  if ((c.k == 0 && len == 0) || (tci != 0 && t->o.add_vlan_header)) return ok = false;
  const uint64_t d = pos + mac;
  if (d > t->bytes || t->bytes - d < snap) return ok = false;
  c.off[c.k] = d;
  c.cap[c.k] = snap;
  if (c.ci) {
    gpk_tp_info& ci = c.ci[c.k];
    go_unix(ld<uint32_t>(p + 4), ld<uint32_t>(p + 8), &ci.ts_sec, &ci.ts_nsec);
    ci.length = len;
    ci.iface = ld<int32_t>(p + tp_align(kV3Hdr) + 4);
    ci.vlan = (st & kStatusVlanValid) ? (int32_t)(tci & 0xfff) : -1;
  }
  if (c.posv) c.posv[c.k] = pos;
  if (c.k == 0) {
    c.P->first_off = d;
    c.P->first_pos = pos;
  }
  c.P->last_pos = pos;
  const uint32_t nx = ld<uint32_t>(p);
  c.pos = pos + (nx ? nx : tp_align((uint64_t)snap + mac));
  ok = true;
  return ++c.k < c.n;
}

void prewalk_group(gpk_tpacket* t, Chain* c, int G, uint64_t epoch) {
  int live = 0;
  for (int g = 0; g < G; g++) {
    c[g].P->epoch = 0;
    if (chain_start(t, c[g].P - t->pre.data(), c[g])) live++;
  }
  while (live) {
    for (int g = 0; g < G; g++) {
      if (!c[g].live) continue;
      bool ok = true;
      if (!chain_step(t, c[g], ok)) {
        c[g].live = false;
        live--;
        if (ok) {
          c[g].P->epoch = epoch;
          c[g].P->n = c[g].n;
        }
      }
    }
  }
}

// Pre-walk, on up to t->threads threads, the handed-over blocks the walk will
// reach next, until they hold `max` packets. A block is written straight to
// the caller's arrays at the position it will have if every block before it
// contributes all of its packets (the exact walk checks that); the block that
// crosses `max` goes to its own arrays, to be taken in part.
void prewalk(gpk_tpacket* t, uint64_t max, uint64_t* offsets, uint32_t* caplens, gpk_tp_info* ci) {
  t->epoch++;  // every earlier pre-walk is stale from here on
  const GoState& s = t->s;
  uint64_t pos = 0;  // the current block's remaining packets come first
  if (s.have_current && !s.polling && s.header_next_needed) {
    const uint32_t n = ld<uint32_t>(t->ring + header_pos(t, s.cur_hdr) + 12);
    pos = n > s.used + 1 ? n - s.used - 1 : 0;
  }
  uint64_t h = (s.have_current && !s.polling) ? (s.cur_hdr + 1) % t->nhdr
                                               : (uint64_t)(s.offset >= (int64_t)t->nhdr ? 0 : s.offset);
  std::vector<Chain> list;
  for (uint64_t i = 0; i + 1 < t->nhdr && pos < max; i++, h = (h + 1) % t->nhdr) {
    if (t->pending[h] || !(header_status(t, h) & kStatusUser)) break;
    const uint32_t n = ld<uint32_t>(t->ring + header_pos(t, h) + 12);
    gpk_tpacket::Pre& P = t->pre[h];
    Chain c{};
    c.P = &P;
    P.direct = pos + n <= max;
    P.pred = pos;
    if (P.direct) {
      c.off = offsets + pos;
      c.cap = caplens + pos;
      c.ci = ci ? ci + pos : nullptr;
      c.posv = nullptr;
    }
    list.push_back(c);
    pos += n;
  }
  if (list.size() < 2) return;
  // chains in flight per thread: up to 4, fewer when there are few blocks per thread
  const int G = (int)std::max<size_t>(1, std::min<size_t>(4, list.size() / std::max(1, t->threads)));
  const size_t groups = (list.size() + G - 1) / G;
  const int T = (int)std::min<size_t>(std::max(1, t->threads), groups);
  const uint64_t epoch = t->epoch;
  t->pool.run(T, [t, G, groups, epoch, &list](int w, int T) {
    for (size_t j = (size_t)w; j < groups; j += (size_t)T)
      prewalk_group(t, list.data() + j * G, (int)std::min<size_t>(G, list.size() - j * G), epoch);
  });
}

void set_err(char* err, size_t cap, const std::string& s) {
  if (err && cap) snprintf(err, cap, "%s", s.c_str());
}

}  // namespace

extern "C" {

void gpk_tp_default_opts(gpk_tp_opts* o) {  // defaultOpts (options.go:149-158)
  memset(o, 0, sizeof(*o));
  o->frame_size = 4096;
  o->block_size = 4096 * 128;
  o->num_blocks = 128;
  o->block_timeout_ns = 64ll * 1000000;
  o->poll_timeout_ns = -1ll * 1000000;
  o->version = GPK_TPACKET_HIGHEST;
  o->socktype = SOCK_RAW;
  o->protocol = 0x0003;  // ETH_P_ALL
}

int gpk_tp_check_opts(gpk_tp_opts* o, char* err, size_t cap) {  // options.check (options.go:197-211)
  if (!o) return GPK_EINVAL;
  char b[160];
  auto dur = [](int64_t ns, char* out, size_t n) {  // time.Duration.String for the values check() prints
    if (ns == 0) {
      snprintf(out, n, "0s");
    } else if (ns % 1000000 == 0 && ns / 1000000 < 1000 && ns / 1000000 > -1000) {
      snprintf(out, n, "%lldms", (long long)(ns / 1000000));
    } else if (ns > -1000 && ns < 1000) {
      snprintf(out, n, "%lldns", (long long)ns);
    } else if (ns > -1000000 && ns < 1000000) {
      snprintf(out, n, "%gµs", ns / 1e3);
    } else if (ns > -1000000000 && ns < 1000000000) {
      snprintf(out, n, "%gms", ns / 1e6);
    } else {
      snprintf(out, n, "%gs", ns / 1e9);
    }
  };
  if (o->block_size % kPageSize != 0) {
    snprintf(b, sizeof(b), "block size %d must be divisible by page size %lld", o->block_size, (long long)kPageSize);
  } else if (o->frame_size == 0 || o->block_size % o->frame_size != 0) {
    if (o->frame_size == 0) {
      snprintf(b, sizeof(b), "runtime error: integer divide by zero");
    } else {
      snprintf(b, sizeof(b), "block size %d must be divisible by frame size %d", o->block_size, o->frame_size);
    }
  } else if (o->num_blocks < 1) {
    snprintf(b, sizeof(b), "num blocks %d must be >= 1", o->num_blocks);
  } else if (o->block_timeout_ns < 1000000) {
    char d[48];
    dur(o->block_timeout_ns, d, sizeof(d));
    snprintf(b, sizeof(b), "block timeout %s must be > 1ms", d);
  } else if (o->version < -1 || o->version > GPK_TPACKET_V3) {
    const char* name = "InvalidVersion";
    snprintf(b, sizeof(b), "tpacket version %s is invalid", name);
  } else {
    o->frames_per_block = o->block_size / o->frame_size;
    return GPK_OK;
  }
  set_err(err, cap, b);
  return GPK_EINVAL;
}

int gpk_tpacket_attach(gpk_tpacket** out, void* ring, uint64_t bytes, int version, const gpk_tp_opts* o) {
  if (!out || !ring || !o || version < GPK_TPACKET_V1 || version > GPK_TPACKET_V3) return GPK_EINVAL;
  gpk_tp_opts oc = *o;
  if (gpk_tp_check_opts(&oc, nullptr, 0) != GPK_OK) return GPK_EINVAL;
  gpk_tpacket* t = new (std::nothrow) gpk_tpacket();
  if (!t) return GPK_ENOMEM;
  t->ring = static_cast<uint8_t*>(ring);
  t->bytes = bytes;
  t->version = version;
  t->o = oc;
  if (init_geometry(t) != GPK_OK) {
    delete t;
    return GPK_EINVAL;
  }
  *out = t;
  return GPK_OK;
}

int gpk_tpacket_new(gpk_tpacket** out, const gpk_tp_opts* o, char* err, size_t cap) {
  if (!out || !o) return GPK_EINVAL;
  gpk_tp_opts oc = *o;
  if (gpk_tp_check_opts(&oc, err, cap) != GPK_OK) return GPK_EINVAL;
  int fd = socket(AF_PACKET, oc.socktype, htons(oc.protocol));
  if (fd < 0) {
    set_err(err, cap, strerror(errno));
    return GPK_EUNSUPP;
  }
  auto fail = [&](const std::string& m) {
    set_err(err, cap, m);
    close(fd);
    return GPK_EUNSUPP;
  };
  // bindToInterface (afpacket.go:155-171)
  int ifindex = 0;
  if (oc.iface[0]) {
    ifindex = (int)if_nametoindex(oc.iface);
    if (!ifindex) return fail("InterfaceByName: route ip+net: no such network interface");
  }
  struct sockaddr_ll sll;
  memset(&sll, 0, sizeof(sll));
  sll.sll_family = AF_PACKET;
  sll.sll_protocol = htons(oc.protocol);
  sll.sll_ifindex = ifindex;
  if (bind(fd, (struct sockaddr*)&sll, sizeof(sll)) < 0) return fail(strerror(errno));
  // setRequestedTPacketVersion (:182-194)
  int version = -1;
  for (int v = GPK_TPACKET_V3; v >= GPK_TPACKET_V1; v--) {
    if (oc.version != GPK_TPACKET_HIGHEST && oc.version != v) continue;
    int val = v;
    if (setsockopt(fd, SOL_PACKET, PACKET_VERSION, &val, sizeof(val)) == 0) {
      version = v;
      break;
    }
  }
  if (version < 0) return fail("no known tpacket versions work on this machine");
  if (oc.vnet_hdr_size > 0) {
    int val = oc.vnet_hdr_size;
    if (setsockopt(fd, SOL_PACKET, PACKET_VNET_HDR, &val, sizeof(val)) < 0)
      return fail(std::string("setsockopt packet_vnet_hdr_sz: ") + strerror(errno));
  }
  // setUpRing (:205-240)
  const uint64_t total = (uint64_t)oc.frames_per_block * oc.num_blocks * oc.frame_size;
  if (version == GPK_TPACKET_V3) {
    struct tpacket_req3 req;
    memset(&req, 0, sizeof(req));
    req.tp_block_size = (unsigned)oc.block_size;
    req.tp_block_nr = (unsigned)oc.num_blocks;
    req.tp_frame_size = (unsigned)oc.frame_size;
    req.tp_frame_nr = (unsigned)(oc.frames_per_block * oc.num_blocks);
    req.tp_retire_blk_tov = (unsigned)(oc.block_timeout_ns / 1000000);
    if (setsockopt(fd, SOL_PACKET, PACKET_RX_RING, &req, sizeof(req)) < 0)
      return fail(std::string("setsockopt packet_rx_ring v3: ") + strerror(errno));
  } else {
    struct tpacket_req req;
    req.tp_block_size = (unsigned)oc.block_size;
    req.tp_block_nr = (unsigned)oc.num_blocks;
    req.tp_frame_size = (unsigned)oc.frame_size;
    req.tp_frame_nr = (unsigned)(oc.frames_per_block * oc.num_blocks);
    if (setsockopt(fd, SOL_PACKET, PACKET_RX_RING, &req, sizeof(req)) < 0)
      return fail(std::string("setsockopt packet_rx_ring: ") + strerror(errno));
  }
  void* ring = mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (ring == MAP_FAILED) return fail(strerror(errno));
  // InitSocketStats (:370-391): reading the counters clears them
  struct tpacket_stats_v3 st3;
  socklen_t sl = version == GPK_TPACKET_V3 ? sizeof(struct tpacket_stats_v3) : sizeof(struct tpacket_stats);
  if (getsockopt(fd, SOL_PACKET, PACKET_STATISTICS, &st3, &sl) < 0) {
    munmap(ring, total);
    return fail(strerror(errno));
  }
  gpk_tpacket* t = new (std::nothrow) gpk_tpacket();
  if (!t) {
    munmap(ring, total);
    close(fd);
    return GPK_ENOMEM;
  }
  t->ring = static_cast<uint8_t*>(ring);
  t->bytes = total;
  t->version = version;
  t->o = oc;
  t->fd = fd;
  t->ifindex = ifindex;
  t->mapped = true;
  init_geometry(t);
  *out = t;
  return GPK_OK;
}

int gpk_tpacket_close(gpk_tpacket* t) {
  if (!t) return GPK_EINVAL;
  if (t->mapped) munmap(t->ring, t->bytes);
  if (t->fd >= 0) close(t->fd);
  delete t;
  return GPK_OK;
}

int gpk_tpacket_ring(const gpk_tpacket* t, void** ring, uint64_t* bytes, int* version, int* fd) {
  if (!t) return GPK_EINVAL;
  if (ring) *ring = t->ring;
  if (bytes) *bytes = t->bytes;
  if (version) *version = t->version;
  if (fd) *fd = t->fd;
  return GPK_OK;
}

int gpk_tpacket_index(gpk_tpacket* t, int wait, uint64_t* offsets, uint32_t* caplens, gpk_tp_info* ci, uint64_t max,
                      uint64_t* n, uint8_t* side, uint64_t side_cap, uint64_t* side_used) {
  if (!t || !n || (max && (!offsets || !caplens))) return GPK_EINVAL;
  *n = 0;
  if (t->dead) return GPK_TP_ERROR;
  std::vector<uint64_t> rel, fr;
  Call c{t, &rel, &fr, wait != 0, side, side ? side_cap : 0, 0};
  uint64_t k = 0;
  int ret = GPK_TP_FULL;
  // large calls over V3 blocks: the blocks ahead are walked in parallel, and
  // the exact walk below takes a block's packets from there after reading its
  // first packet itself (a DRAM-latency-bound pointer chase per packet otherwise)
  const bool bulk = t->version == GPK_TPACKET_V3 && max >= 4096 && t->threads > 1;
  // the block the last call stopped in, if that call pre-walked it: its
  // remaining packets come from there too
  const GoState& s0 = t->s;
  gpk_tpacket::Pre* carry = nullptr;
  if (bulk && s0.have_current && !s0.polling && s0.header_next_needed) {
    gpk_tpacket::Pre& P = t->pre[s0.cur_hdr];
    if (P.epoch == t->epoch && !P.direct && s0.used < P.pos.size() && P.pos[s0.used] == s0.pkt) carry = &P;
  }
  if (bulk) prewalk(t, max, offsets, caplens, ci);
  if (carry) {
    const uint64_t m = std::min<uint64_t>(carry->n - 1 - t->s.used, max);
    memcpy(offsets, carry->off.data() + t->s.used + 1, m * 8);
    memcpy(caplens, carry->cap.data() + t->s.used + 1, m * 4);
    if (ci) memcpy(ci, carry->ci.data() + t->s.used + 1, m * sizeof(gpk_tp_info));
    t->s.used += (uint32_t)m;
    t->s.pkt = carry->pos[t->s.used];
    t->s.packets += (int64_t)m;
    k = m;
  }
  std::vector<uint8_t> visited;  // a block's pre-walk serves its first visit only
  if (bulk) visited.assign(t->nhdr, 0);
  while (k < max) {
    const GoState snap = t->s;
    rel.clear();
    fr.clear();
    const int r = c.run();
    if (r == -2) {  // no room for a VLAN-tagged copy: undo this call
      t->s = snap;
      for (uint64_t h : fr) t->fresh[h] = 1;
      if (k == 0) {
        t->err = "side buffer too small for one packet";
        ret = GPK_TP_ERROR;  // not a reference error: the caller's buffer is too small
      }
      break;
    }
    commit_releases(t, rel);
    commit_fresh(t, fr);
    if (r == 0) {
      ret = GPK_TP_WAIT;
      break;
    }
    if (r < 0) {
      ret = GPK_TP_ERROR;
      break;
    }
    offsets[k] = c.off;
    caplens[k] = c.caplen;
    if (ci) ci[k] = c.ci;
    k++;
    if (bulk && t->s.used == 0 && !visited[t->s.cur_hdr]) {
      const uint64_t h = t->s.cur_hdr;
      visited[h] = 1;
      gpk_tpacket::Pre& P = t->pre[h];
      if (P.epoch == t->epoch && P.first_off == c.off && P.first_pos == t->s.pkt) {
        // packets 1.. of the block: what the next() calls would return
        uint64_t m = 0;
        if (P.direct) {
          if (P.pred == k - 1) {  // already in place
            m = P.n - 1;
            t->s.pkt = P.last_pos;
          }
        } else {
          m = std::min<uint64_t>(P.n - 1, max - k);
          memcpy(offsets + k, P.off.data() + 1, m * 8);
          memcpy(caplens + k, P.cap.data() + 1, m * 4);
          if (ci) memcpy(ci + k, P.ci.data() + 1, m * sizeof(gpk_tp_info));
          t->s.pkt = P.pos[m];
        }
        k += m;
        t->s.used = (uint32_t)m;
        t->s.packets += (int64_t)m;
      }
    }
  }
  *n = k;
  if (side_used) *side_used = c.side_used;
  return ret;
}

int gpk_tpacket_set_threads(gpk_tpacket* t, int threads) {
  if (!t || threads < 1 || threads > 256) return GPK_EINVAL;
  t->threads = threads;
  return GPK_OK;
}

int gpk_tpacket_defer(gpk_tpacket* t, int on) {
  if (!t) return GPK_EINVAL;
  if (!on && t->defer) gpk_tpacket_release(t, UINT64_MAX);
  t->defer = on != 0;
  return GPK_OK;
}

int gpk_tpacket_release_seq(const gpk_tpacket* t, uint64_t* seq) {
  if (!t || !seq) return GPK_EINVAL;
  *seq = t->rel_seq;
  return GPK_OK;
}

int gpk_tpacket_release(gpk_tpacket* t, uint64_t seq) {
  if (!t) return GPK_EINVAL;
  while (!t->pq.empty() && t->pq.front().first < seq) {
    const uint64_t h = t->pq.front().second;
    t->pq.pop_front();
    t->pending[h] = 0;
    clear_status(t, h);
  }
  return GPK_OK;
}

int gpk_tpacket_take_new_headers(gpk_tpacket* t, uint64_t* first, uint64_t* count) {
  if (!t || !first || !count) return GPK_EINVAL;
  *first = t->new_first;
  *count = t->new_count;
  t->new_count = 0;
  return GPK_OK;
}

int gpk_tpacket_geometry(const gpk_tpacket* t, uint64_t* header_bytes, uint64_t* headers) {
  if (!t) return GPK_EINVAL;
  if (header_bytes) *header_bytes = t->hdr_bytes;
  if (headers) *headers = t->nhdr;
  return GPK_OK;
}

int gpk_tpacket_error(const gpk_tpacket* t, char* buf, size_t cap, int* is_panic) {
  if (!t) return GPK_EINVAL;
  if (is_panic) *is_panic = t->panic ? 1 : 0;
  if (buf && cap) snprintf(buf, cap, "%s", t->err.c_str());
  return (int)t->err.size();
}

int gpk_tpacket_stats(const gpk_tpacket* t, int64_t* packets, int64_t* polls) {
  if (!t) return GPK_EINVAL;
  if (packets) *packets = t->s.packets;
  if (polls) *polls = t->s.polls;
  return GPK_OK;
}

int gpk_tpacket_socket_stats(gpk_tpacket* t, uint32_t* packets, uint32_t* drops, uint32_t* freeze_q) {
  if (!t) return GPK_EINVAL;
  if (t->fd >= 0) {  // the kernel clears its counters on every read: accumulate (afpacket.go:378-431)
    struct tpacket_stats_v3 st{};
    socklen_t sl = t->version == GPK_TPACKET_V3 ? sizeof(struct tpacket_stats_v3) : sizeof(struct tpacket_stats);
    if (getsockopt(t->fd, SOL_PACKET, PACKET_STATISTICS, &st, &sl) < 0) return GPK_EINVAL;
    t->ss_packets += st.tp_packets;
    t->ss_drops += st.tp_drops;
    if (t->version == GPK_TPACKET_V3) t->ss_freeze += st.tp_freeze_q_cnt;
  }
  if (packets) *packets = t->ss_packets;
  if (drops) *drops = t->ss_drops;
  if (freeze_q) *freeze_q = t->ss_freeze;
  return GPK_OK;
}

int gpk_tpacket_set_bpf(gpk_tpacket* t, const void* insns, uint32_t n) {
  if (!t || t->fd < 0) return GPK_EINVAL;
  if (n == 0) {
    int z = 0;
    return setsockopt(t->fd, SOL_SOCKET, SO_DETACH_FILTER, &z, sizeof(z)) == 0 ? GPK_OK : GPK_EINVAL;
  }
  if (n > 0xFFFF || !insns) return GPK_EINVAL;  // "filter too large"
  struct sock_fprog p;
  p.len = (unsigned short)n;
  p.filter = (struct sock_filter*)const_cast<void*>(insns);
  return setsockopt(t->fd, SOL_SOCKET, SO_ATTACH_FILTER, &p, sizeof(p)) == 0 ? GPK_OK : GPK_EINVAL;
}

int gpk_tpacket_set_fanout(gpk_tpacket* t, int type, uint16_t id) {
  if (!t || t->fd < 0) return GPK_EINVAL;
  int arg = (type << 16) | id;
  return setsockopt(t->fd, SOL_PACKET, PACKET_FANOUT, &arg, sizeof(arg)) == 0 ? GPK_OK : GPK_EINVAL;
}

int gpk_tpacket_set_ebpf(gpk_tpacket* t, int32_t prog_fd) {  // SetEBPF (afpacket.go:312-314)
  if (!t || t->fd < 0) return GPK_EINVAL;
  return setsockopt(t->fd, SOL_SOCKET, SO_ATTACH_BPF, &prog_fd, sizeof(prog_fd)) == 0 ? GPK_OK : GPK_EINVAL;
}

int gpk_tpacket_set_promiscuous(gpk_tpacket* t, int on) {  // SetPromiscuous (afpacket.go:552-564)
  if (!t || t->fd < 0) return GPK_EINVAL;
  struct packet_mreq mr;
  memset(&mr, 0, sizeof(mr));
  mr.mr_ifindex = t->ifindex;
  mr.mr_type = PACKET_MR_PROMISC;
  return setsockopt(t->fd, SOL_PACKET, on ? PACKET_ADD_MEMBERSHIP : PACKET_DROP_MEMBERSHIP, &mr, sizeof(mr)) == 0
             ? GPK_OK
             : GPK_EINVAL;
}

int gpk_tpacket_write(gpk_tpacket* t, const void* pkt, uint64_t n) {  // WritePacketData (afpacket.go:567-570)
  if (!t || t->fd < 0 || (!pkt && n)) return GPK_EINVAL;
  return write(t->fd, pkt, (size_t)n) >= 0 ? GPK_OK : GPK_EINVAL;
}

int gpk_tpacket_init_socket_stats(gpk_tpacket* t) {  // InitSocketStats (afpacket.go:378-399)
  if (!t || t->fd < 0) return GPK_EINVAL;
  struct tpacket_stats_v3 st{};
  socklen_t sl = t->version == GPK_TPACKET_V3 ? sizeof(struct tpacket_stats_v3) : sizeof(struct tpacket_stats);
  if (getsockopt(t->fd, SOL_PACKET, PACKET_STATISTICS, &st, &sl) < 0) return GPK_EINVAL;
  t->ss_packets = t->ss_drops = t->ss_freeze = 0;
  return GPK_OK;
}

}  // extern "C"

// ---- the capture loop through HBM ------------------------------------------

namespace {

struct PBat {
  uint64_t *h_off = nullptr, *d_off = nullptr;
  uint32_t *h_cap = nullptr, *d_cap = nullptr;
  gpk_tp_info* h_ci = nullptr;
  gpk_record *h_rec = nullptr, *d_rec = nullptr;
  uint32_t *h_err = nullptr, *d_err = nullptr;
  uint64_t *h_flow = nullptr, *d_flow = nullptr;
  gpk_fields *h_fields = nullptr, *d_fields = nullptr;
  uint8_t* h_side = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t e0 = nullptr, h2d = nullptr, k0 = nullptr, k1 = nullptr, done = nullptr;
  uint64_t first = 0, n = 0, rel_seq = 0, gen = 0;
  bool inflight = false, h2d_pending = false;
};

}  // namespace

static int tpacket_pump(gpk_ctx* ctx, const gpk_parser* parser, gpk_tpacket* t, const gpk_tp_pump_opts* o,
                        gpk_tp_pump_cb cb, void* user, gpk_tp_pump_stats* st) {
  gpk_tp_pump_opts opt{1ull << 20, 0, 0, 4, nullptr, nullptr};
  if (o) {
    if (o->batch_pkts) opt.batch_pkts = o->batch_pkts;
    opt.max_packets = o->max_packets;
    opt.wait = o->wait;
    if (o->inflight > 0) opt.inflight = o->inflight;
    opt.fields_cb = o->fields_cb;
    opt.packets_cb = o->packets_cb;
  }
  const bool with_fields = opt.fields_cb != nullptr;
  // packets_cb: ring headers stay the user's until their batch was delivered
  const bool hold = opt.packets_cb != nullptr;
  std::vector<const uint8_t*> ptrs(hold ? opt.batch_pkts : 0);
  const uint64_t P = opt.batch_pkts;
  const int NB = std::max(2, opt.inflight);
  const uint64_t side_cap = std::min<uint64_t>(64ull << 20, std::max<uint64_t>(1ull << 20, P * 256));
  std::string herr;
  auto ok = [&](hipError_t e, const char* what) {
    if (e != hipSuccess && herr.empty()) herr = std::string(what) + ": " + hipGetErrorString(e);
    return e == hipSuccess;
  };
  std::vector<PBat> B(NB);
  uint8_t* dev = nullptr;  // ring mirror + NB side regions
  const uint64_t ring_bytes = t->bytes;
  bool good = ok(hipMalloc((void**)&dev, ring_bytes + NB * side_cap + 64), "hipMalloc ring mirror");
  for (auto& b : B) {
    good = good && ok(gpk_pin_alloc((void**)&b.h_off, P * 8), "pinned batch") &&
           ok(gpk_pin_alloc((void**)&b.h_cap, P * 4), "pinned batch") &&
           ok(gpk_pin_alloc((void**)&b.h_ci, P * sizeof(gpk_tp_info)), "pinned batch") &&
           ok(gpk_pin_alloc((void**)&b.h_rec, P * sizeof(gpk_record)), "pinned batch") &&
           ok(gpk_pin_alloc((void**)&b.h_err, P * 8), "pinned batch") &&
           ok(gpk_pin_alloc((void**)&b.h_flow, P * 24), "pinned batch") &&
           ok(gpk_pin_alloc((void**)&b.h_side, side_cap), "pinned batch") &&
           ok(hipMalloc((void**)&b.d_off, P * 8), "hipMalloc") && ok(hipMalloc((void**)&b.d_cap, P * 4), "hipMalloc") &&
           ok(hipMalloc((void**)&b.d_rec, P * sizeof(gpk_record)), "hipMalloc") &&
           ok(hipMalloc((void**)&b.d_err, P * 8), "hipMalloc") && ok(hipMalloc((void**)&b.d_flow, P * 24), "hipMalloc") &&
           ok(hipStreamCreateWithFlags(&b.stream, hipStreamNonBlocking), "hipStreamCreate") &&
           ok(hipEventCreate(&b.e0), "hipEventCreate") &&
           ok(hipEventCreateWithFlags(&b.h2d, hipEventDisableTiming), "hipEventCreate") &&
           ok(hipEventCreate(&b.k0), "hipEventCreate") && ok(hipEventCreate(&b.k1), "hipEventCreate") &&
           ok(hipEventCreate(&b.done), "hipEventCreate");
    if (with_fields)
      good = good && ok(gpk_pin_alloc((void**)&b.h_fields, P * sizeof(gpk_fields)), "pinned batch") &&
             ok(hipMalloc((void**)&b.d_fields, P * sizeof(gpk_fields)), "hipMalloc");
  }
  // the ring itself is DMA'd from: pin it where the memory allows (an AF_PACKET
  // mapping may refuse; then the copies go through the runtime's staging)
  const bool registered = good && hipHostRegister(t->ring, ring_bytes, hipHostRegisterDefault) == hipSuccess;
  if (!registered) (void)hipGetLastError();
  const bool was_deferred = t->defer;
  t->defer = true;
  uint64_t hb = 0, nh = 0;
  gpk_tpacket_geometry(t, &hb, &nh);
  // last batch (slot, generation) that read each header: its kernel must finish
  // before the header's bytes in the mirror are overwritten
  std::vector<int> hdr_slot(nh, -1);
  std::vector<uint64_t> hdr_gen(nh, 0);
  std::deque<int> order;  // in-flight slots, oldest first
  int prev_slot = -1;
  uint64_t packet_index = 0;
  const double t0 = now_s();
  int rc = GPK_OK;
  // gpk_stop: from its first check after a stop no callback is made
  const uint64_t stop0 = gpk_ctx_stop_seq(ctx);
  bool stopped = false;
  uint64_t delivered = 0;
  auto stop_seen = [&]() {
    if (!stopped && gpk_ctx_stop_seq(ctx) != stop0) stopped = true;
    return stopped;
  };

  auto release_done = [&](bool block) {  // hand back headers whose HtoD has completed
    if (hold) return true;  // ... only once delivered (deliver_oldest)
    for (int s : order) {
      PBat& b = B[s];
      if (!b.h2d_pending) continue;
      hipError_t q = block ? hipEventSynchronize(b.h2d) : hipEventQuery(b.h2d);
      if (q == hipErrorNotReady) break;
      if (!ok(q, "h2d event")) return false;
      b.h2d_pending = false;
      gpk_tpacket_release(t, b.rel_seq);
      if (block) return true;  // one at a time when blocking
    }
    return true;
  };
  auto deliver_oldest = [&]() {
    const int s = order.front();
    order.pop_front();
    PBat& b = B[s];
    if (!ok(hipEventSynchronize(b.done), "hipEventSynchronize")) return false;
    if (b.h2d_pending && !hold) {
      b.h2d_pending = false;
      gpk_tpacket_release(t, b.rel_seq);
    }
    float ms = 0, kms = 0;
    if (hipEventElapsedTime(&ms, b.e0, b.done) == hipSuccess) st->gpu_s += ms * 1e-3;
    if (hipEventElapsedTime(&kms, b.k0, b.k1) == hipSuccess) st->kernel_s += kms * 1e-3;
    const bool deliver = !stop_seen();  // a batch is delivered whole or not at all
    if (deliver) delivered += b.n;
    if (deliver && hold) {  // the packets: ring frames, or this slot's VLAN copies (h_off moved for the device mirror)
      for (uint64_t i = 0; i < b.n; i++)
        ptrs[i] = b.h_off[i] < ring_bytes ? t->ring + b.h_off[i] : b.h_side + (b.h_off[i] - ring_bytes - s * side_cap);
      opt.packets_cb(user, b.first, b.n, ptrs.data(), b.h_cap);
    }
    if (deliver && with_fields) opt.fields_cb(user, b.first, b.n, b.h_fields);
    if (deliver && cb) cb(user, b.first, b.n, b.h_rec, b.h_err, b.h_flow, b.h_ci, b.h_cap);
    if (hold && b.h2d_pending) {  // delivered: the headers go back to the kernel
      b.h2d_pending = false;
      gpk_tpacket_release(t, b.rel_seq);
    }
    b.inflight = false;
    return true;
  };

  int slot = 0;
  while (good && !stop_seen()) {
    if (opt.max_packets && packet_index >= opt.max_packets) break;
    // a free slot
    while (B[slot].inflight && good) good = deliver_oldest();
    if (!good) break;
    PBat& b = B[slot];
    if (!release_done(false)) {
      good = false;
      break;
    }
    const uint64_t want = opt.max_packets ? std::min<uint64_t>(P, opt.max_packets - packet_index) : P;
    const bool had_current = t->s.have_current && t->s.should_release;
    const uint64_t cur0 = t->s.cur_hdr;
    uint64_t n = 0, side_used = 0;
    double ti = now_s();
    int r = gpk_tpacket_index(t, 0, b.h_off, b.h_cap, b.h_ci, want, &n, b.h_side, side_cap, &side_used);
    st->index_s += now_s() - ti;
    if (r == GPK_TP_ERROR) {
      char e[160];
      int pan = 0;
      gpk_tpacket_error(t, e, sizeof(e), &pan);
      snprintf(st->error, sizeof(st->error), "%s", e);
      st->status = GPK_TP_ERROR;
    }
    uint64_t nf = 0, nc = 0;
    gpk_tpacket_take_new_headers(t, &nf, &nc);
    if (n == 0 && nc == 0) {
      if (r == GPK_TP_ERROR) break;
      // dry: release what has reached the device (with packets_cb: what was
      // delivered), then wait or stop
      if (!order.empty()) {
        bool any = false;
        for (int s : order) any = any || B[s].h2d_pending;
        if (any) {
          if (!(hold ? deliver_oldest() : release_done(true))) good = false;
          continue;
        }
      }
      if (!opt.wait) break;
      st->waits++;
      // block inside the walk (poll / spin) for one packet, then take the rest
      // of the batch without blocking
      uint64_t n2 = 0, su2 = 0;
      double tw = now_s();
      int r2;
      r2 = gpk_tpacket_index(t, 1, b.h_off, b.h_cap, b.h_ci, 1, &n2, b.h_side, side_cap, &su2);
      st->index_s += now_s() - tw;
      if (r2 == GPK_TP_ERROR) {
        char e[160];
        int pan = 0;
        gpk_tpacket_error(t, e, sizeof(e), &pan);
        snprintf(st->error, sizeof(st->error), "%s", e);
        st->status = GPK_TP_ERROR;
        break;
      }
      if (n2 == 0) continue;
      // the packet read while waiting starts this batch
      uint64_t n3 = 0, su3 = 0;
      r = gpk_tpacket_index(t, 0, b.h_off + 1, b.h_cap + 1, b.h_ci + 1, want > 1 ? want - 1 : 0, &n3,
                            b.h_side + su2, side_cap - su2, &su3);
      for (uint64_t i = 1; i <= n3; i++)
        if (b.h_off[i] >= ring_bytes) b.h_off[i] += su2;
      n = 1 + n3;
      side_used = su2 + su3;
      gpk_tpacket_take_new_headers(t, &nf, &nc);
    }
    // ---- enqueue the batch on its slot's stream -------------------------------
    b.gen++;
    b.first = packet_index;
    b.n = n;
    good = ok(hipEventRecord(b.e0, b.stream), "hipEventRecord");
    // order after the previous batch's copies (it may have copied the header
    // this batch continues in)
    if (good && prev_slot >= 0 && B[prev_slot].inflight)
      good = ok(hipStreamWaitEvent(b.stream, B[prev_slot].h2d, 0), "hipStreamWaitEvent");
    // overwrite a header's mirror bytes only after the last kernel reading them
    for (uint64_t j = 0; good && j < nc; j++) {
      const uint64_t h = (nf + j) % nh;
      const int s = hdr_slot[h];
      if (s >= 0 && s != slot && B[s].inflight && B[s].gen == hdr_gen[h])
        good = ok(hipStreamWaitEvent(b.stream, B[s].done, 0), "hipStreamWaitEvent");
    }
    for (uint64_t j = 0; good && j < nc;) {  // contiguous runs of new headers
      const uint64_t h = (nf + j) % nh;
      const uint64_t run = std::min<uint64_t>(nc - j, nh - h);
      good = ok(hipMemcpyAsync(dev + h * hb, t->ring + h * hb, run * hb, hipMemcpyHostToDevice, b.stream), "HtoD ring");
      st->ring_bytes_copied += run * hb;
      j += run;
    }
    if (good && side_used) {
      good = ok(hipMemcpyAsync(dev + ring_bytes + slot * side_cap, b.h_side, side_used, hipMemcpyHostToDevice, b.stream),
                "HtoD side");
      for (uint64_t i = 0; i < n; i++)
        if (b.h_off[i] >= ring_bytes) b.h_off[i] += slot * side_cap;
    }
    good = good && ok(hipMemcpyAsync(b.d_off, b.h_off, n * 8, hipMemcpyHostToDevice, b.stream), "HtoD offsets") &&
           ok(hipMemcpyAsync(b.d_cap, b.h_cap, n * 4, hipMemcpyHostToDevice, b.stream), "HtoD caplens") &&
           ok(hipEventRecord(b.h2d, b.stream), "hipEventRecord") &&
           ok(hipMemsetAsync(b.d_err, 0, n * 8, b.stream), "hipMemsetAsync") &&
           ok(hipEventRecord(b.k0, b.stream), "hipEventRecord");
    if (!good) break;
    gpk_tpacket_release_seq(t, &b.rel_seq);
    b.h2d_pending = true;
    // data_bytes: the readable end of the mirror (ring, side regions, slack);
    // the mean-size hint apart: the batch's capture lengths
    uint64_t pk_bytes = 0;
    for (uint64_t i = 0; i < n; i++) pk_bytes += b.h_cap[i];
    gpk_batch db{dev, b.d_off, b.d_cap, n, ring_bytes + NB * side_cap + 64};
    gpk_results dr{b.d_rec, b.d_err, b.d_flow, nullptr};
    int drc = gpk_decode_batch_ex(ctx, parser, &db, &dr, b.stream, pk_bytes ? pk_bytes : 1, st->kernel,
                                  sizeof(st->kernel), with_fields ? b.d_fields : nullptr);
    if (drc) {
      rc = drc;
      good = false;
      break;
    }
    good = ok(hipEventRecord(b.k1, b.stream), "hipEventRecord") &&
           ok(hipMemcpyAsync(b.h_rec, b.d_rec, n * sizeof(gpk_record), hipMemcpyDeviceToHost, b.stream), "DtoH") &&
           ok(hipMemcpyAsync(b.h_err, b.d_err, n * 8, hipMemcpyDeviceToHost, b.stream), "DtoH") &&
           ok(hipMemcpyAsync(b.h_flow, b.d_flow, n * 24, hipMemcpyDeviceToHost, b.stream), "DtoH") &&
           (!with_fields ||
            ok(hipMemcpyAsync(b.h_fields, b.d_fields, n * sizeof(gpk_fields), hipMemcpyDeviceToHost, b.stream), "DtoH")) &&
           ok(hipEventRecord(b.done, b.stream), "hipEventRecord");
    b.inflight = true;
    order.push_back(slot);
    // headers this batch reads: the one it continued in, and the new ones
    if (had_current && cur0 < nh) {
      hdr_slot[cur0] = slot;
      hdr_gen[cur0] = b.gen;
    }
    for (uint64_t j = 0; j < nc; j++) {
      const uint64_t h = (nf + j) % nh;
      hdr_slot[h] = slot;
      hdr_gen[h] = b.gen;
    }
    for (uint64_t i = 0; i < n; i++) st->packet_bytes += b.h_cap[i];
    packet_index += n;
    st->batches++;
    prev_slot = slot;
    slot = (slot + 1) % NB;
    if (r == GPK_TP_ERROR) break;
  }
  while (good && !order.empty()) good = deliver_oldest();
  for (auto& b : B)  // this pump's copies out of the ring have finished (other streams' work is not waited for)
    if (b.stream) (void)hipStreamSynchronize(b.stream);
  gpk_tpacket_release(t, UINT64_MAX);
  t->defer = was_deferred;
  st->packets = stopped ? delivered : packet_index;
  st->wall_s = now_s() - t0;
  if (registered) (void)hipHostUnregister(t->ring);
  for (auto& b : B) {
    if (b.stream) (void)hipStreamSynchronize(b.stream);
    for (void* p : {(void*)b.h_off, (void*)b.h_cap, (void*)b.h_ci, (void*)b.h_rec, (void*)b.h_err, (void*)b.h_flow,
                    (void*)b.h_side, (void*)b.h_fields})
      if (p) (void)gpk_pin_free(p);
    for (void* p : {(void*)b.d_off, (void*)b.d_cap, (void*)b.d_rec, (void*)b.d_err, (void*)b.d_flow, (void*)b.d_fields})
      if (p) (void)hipFree(p);
    for (hipEvent_t e : {b.e0, b.h2d, b.k0, b.k1, b.done})
      if (e) (void)hipEventDestroy(e);
    if (b.stream) (void)hipStreamDestroy(b.stream);
  }
  if (dev) (void)hipFree(dev);
  if (!good && rc == GPK_OK) {
    snprintf(st->error, sizeof(st->error), "%s", herr.c_str());
    return GPK_EHIP;
  }
  return stopped && rc == GPK_OK ? GPK_STOPPED : rc;
}

// The C entry point: no C++ exception crosses it (a thread or an allocation
// the host cannot provide ends the call with an error).
extern "C" int gpk_tpacket_pump(gpk_ctx* ctx, const gpk_parser* parser, gpk_tpacket* t, const gpk_tp_pump_opts* o,
                                gpk_tp_pump_cb cb, void* user, gpk_tp_pump_stats* st) {
  if (!ctx || !parser || !t || !st) return GPK_EINVAL;
  memset(st, 0, sizeof(*st));
  try {
    // the context's device for the pipeline's buffers, streams and launches
    // (callbacks included); the caller's device is back on return
    gpk::DeviceScope dscope(gpk_ctx_device(ctx));
    if (dscope.err != hipSuccess) {
      snprintf(st->error, sizeof(st->error), "hipSetDevice: %s", hipGetErrorString(dscope.err));
      return GPK_EHIP;
    }
    return tpacket_pump(ctx, parser, t, o, cb, user, st);
  } catch (const std::bad_alloc&) {
    snprintf(st->error, sizeof(st->error), "out of host memory");
    return GPK_ENOMEM;
  } catch (const std::exception& e) {
    snprintf(st->error, sizeof(st->error), "%s", e.what());
    return GPK_EHIP;
  }
}

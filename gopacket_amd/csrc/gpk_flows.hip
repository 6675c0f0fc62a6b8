// gpk_flows.hip — flow-keyed grouping of a decoded batch (include/gpk_flows.h,
// SURVEY.md §8(f)3).
//
// What the reference does per packet with a Go map, done for a batch in HBM:
//   1. key_kernel     one lane per packet: derive the consumer's key from the
//                     decode results (records, layouts) and the packet bytes,
//                     exactly as the consumer would build it (a [2]Flow, an
//                     ipv4{Flow, Id}, or a FastHash bucket), or the reason the
//                     packet has no key; store the key words and a 64-bit hash
//   2. insert_kernel  open-addressing table in HBM: the hash picks the slot,
//                     the full key words decide equality (a hash collision
//                     probes on), a 64-bit atomicMin of the slot word keeps
//                     each key's first packet in its index field
//   3. first_kernel   every keyed packet gets its key's first packet index
//   4. radix sort     (first index, packet index) pairs, stable, on the bits
//                     the batch size needs: groups in order of first
//                     appearance, packets in batch order inside a group
//   5. heads + scan   group boundaries, group ids, counts
// The table never stores a key twice: keys are compared word for word, so
// the grouping is exact whatever the hash does.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>
#include <new>

#include "../../include/gpk_flows.h"
#include "gpk_devguard.h"

// gpk_host.cpp: gpk_decode_batch with the fused key derivation (library-internal)
extern "C" int gpk_decode_batch_keys(gpk_ctx* c, const gpk_parser* p, const gpk_batch* b, const gpk_results* o, int key_kind,
                          uint32_t* keys, uint64_t* khash, int32_t* kcode, void* stream);

namespace {

constexpr int kKeyWords = 10;
constexpr uint64_t kEmpty = ~0ull;
constexpr int kIdxBits = 28;  // packet index bits in a table word
constexpr uint32_t kIdxMask = (1u << kIdxBits) - 1;
constexpr int kSlotTcp = 5, kSlotIp4 = 2, kSlotIp6 = 3;  // gpk_layout slots (decoder kind - 1)
constexpr uint32_t kCodeIp4 = 3, kCodeIp6 = 4, kCodeTcp = 9;  // GPK_CODE_*

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint32_t ld4(const uint8_t* p) {  // raw bytes, any alignment
  return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

struct KeyArgs {
  const uint8_t* data;
  const uint64_t* offsets;
  const uint32_t* caplens;
  const gpk_record* records;
  const gpk_layout* layouts;
  const uint64_t* flows;
  uint64_t n;
  int kind;
  uint32_t buckets;
  uint32_t* keys;    // [n * kKeyWords]
  uint64_t* hash;    // [n]
  int32_t* code;     // [n] 0 = keyed, else GPK_GROUP_*
  uint32_t* bucket_min;  // [buckets] (NET_BUCKET)
};

// The consumer's key of packet i. Returns 0 (keyed, w[] and the hash set) or a
// GPK_GROUP_* code.
__device__ int packet_key(const KeyArgs& a, uint64_t i, uint32_t* w) {
  const gpk_record rec = a.records[i];
  for (int k = 0; k < kKeyWords; k++) w[k] = 0;
  if (a.kind == GPK_GROUP_NET_BUCKET) {
    if (!(rec.status & GPK_ST_NET_FLOW)) return GPK_GROUP_NONE;  // packet.NetworkLayer() == nil
    const uint64_t h = a.flows[a.n + i];                        // NetworkFlow().FastHash()
    w[0] = (uint32_t)(h & (uint64_t)(a.buckets - 1));            // int(h) & (buckets-1)
    return 0;
  }
  const gpk_layout& L = a.layouts[i];
  const uint8_t* p = a.data + a.offsets[i];
  const uint32_t nl = (rec.status >> GPK_ST_NLAYERS_SHIFT) & GPK_ST_NLAYERS_MASK;
  if (a.kind == GPK_GROUP_CONNECTION) {
    const uint32_t t0 = L.start[kSlotTcp];
    if (t0 == GPK_LAYOUT_ABSENT) return GPK_GROUP_NONE;  // no TCP layer in decoded
    // the last network layer before TCP in decoded (assembly.go:534 takes the caller's netFlow)
    uint32_t net = 0;
    bool seen_tcp = false;
    const uint32_t m = nl < GPK_MAX_INLINE_LAYERS ? nl : GPK_MAX_INLINE_LAYERS;
    for (uint32_t k = 0; k < m && !seen_tcp; k++) {
      const uint32_t c = (uint32_t)(rec.layers >> (4 * k)) & 15u;
      if (c == kCodeIp4 || c == kCodeIp6) net = c;
      seen_tcp = c == kCodeTcp;
    }
    if (!seen_tcp) return GPK_GROUP_UNKNOWN;
    if (!net) return GPK_GROUP_NONE;
    // "ignoring useless packet" (assembly.go:527-532): no SYN/FIN/RST and an empty payload
    const uint32_t flags = p[t0 + 13], doff = p[t0 + 12] >> 4;
    const uint32_t plen = (L.end[kSlotTcp] - t0) - doff * 4;
    if (!(flags & 0x07u) && plen == 0) return GPK_GROUP_USELESS;
    // key{netFlow, TransportFlow()}: Flow{EndpointIPv4|IPv6, src, dst}, Flow{EndpointTCPPort, sport, dport}
    if (net == kCodeIp4) {
      const uint8_t* ip = p + L.start[kSlotIp4];
      w[0] = 1u | 1u << 8 | 4u << 16;
      w[1] = ld4(ip + 12);
      w[5] = ld4(ip + 16);
    } else {
      const uint8_t* ip = p + L.start[kSlotIp6];
      w[0] = 1u | 2u << 8 | 4u << 16;
      for (int k = 0; k < 4; k++) {
        w[1 + k] = ld4(ip + 8 + 4 * k);
        w[5 + k] = ld4(ip + 24 + 4 * k);
      }
    }
    w[9] = ld4(p + t0);  // source and destination port bytes
    return 0;
  }
  // GPK_GROUP_DEFRAG
  const uint32_t s = L.start[kSlotIp4];
  if (s == GPK_LAYOUT_ABSENT) return GPK_GROUP_NONE;
  const uint32_t err = rec.status & GPK_ST_ERR_MASK;
  if (err >= GPK_ERR_IP4_HDR_SHORT && err <= GPK_ERR_IP4_OPT_BADLEN) return GPK_GROUP_NONE;  // struct left mid-decode
  const uint8_t* ip = p + s;
  const uint32_t ff = (uint32_t)ip[6] << 8 | ip[7];
  const uint32_t flags = ff >> 13, fo = ff & 0x1FFF;  // ip4.go:214-215
  if (flags & 2u) return GPK_GROUP_NONE;              // dontDefrag: DF (defrag.go:162)
  if (!(flags & 1u) && fo == 0) return GPK_GROUP_NONE;  // not fragmented (:166)
  uint32_t len = (uint32_t)ip[2] << 8 | ip[3];
  if (len == 0) len = (L.end[kSlotIp4] - s) & 0xFFFF;  // ip4.go:189-193 (TSO): uint16(len(data))
  const uint32_t ihl = ip[0] & 15u;
  const uint32_t frag_size = (len - ihl * 4) & 0xFFFF;  // uint16 arithmetic (defrag.go:174)
  if ((flags & 1u) && frag_size < 8) return GPK_GROUP_FRAG_TOO_SMALL;
  if (fo > 8183) return GPK_GROUP_FRAG_OFFSET;
  if (((fo * 8 + len) & 0xFFFF) > 65535u) return GPK_GROUP_FRAG_OVERRUN;  // uint16: never true, as in Go
  w[0] = 2u | 1u << 8;
  w[1] = ld4(ip + 12);
  w[5] = ld4(ip + 16);
  w[9] = (uint32_t)ip[4] << 8 | ip[5];  // Id
  return 0;
}

__global__ void __launch_bounds__(256) key_kernel(KeyArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  uint32_t w[kKeyWords];
  const int c = packet_key(a, i, w);
  a.code[i] = c;
  if (c) return;
  if (a.kind == GPK_GROUP_NET_BUCKET) {
    // a few buckets shared by every packet: the lowest lane of the wave per
    // bucket, and only while the bucket's minimum can still drop
    const uint32_t b = w[0];
    uint64_t todo = __ballot(1);
    while (todo) {
      const uint32_t lead = (uint32_t)__builtin_ctzll(todo);
      const uint32_t lb = (uint32_t)__shfl((int)b, (int)lead);
      const uint64_t same = __ballot(b == lb);
      todo &= ~same;
      if (b == lb && (uint32_t)__lane_id() == lead &&
          __hip_atomic_load(&a.bucket_min[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > (uint32_t)i)
        atomicMin(&a.bucket_min[b], (uint32_t)i);
    }
    a.hash[i] = b;
    return;
  }
  uint64_t h = 0x9E3779B97F4A7C15ull;
  for (int k = 0; k < kKeyWords; k++) {
    a.keys[i * kKeyWords + k] = w[k];
    h = (h ^ w[k]) * 0xBF58476D1CE4E5B9ull;
    h ^= h >> 29;
  }
  a.hash[i] = mix64(h);
}

__device__ __forceinline__ bool same_key(const uint32_t* keys, uint64_t a, uint64_t b) {
  const uint32_t* x = keys + a * kKeyWords;
  const uint32_t* y = keys + b * kKeyWords;
  bool eq = true;
  for (int k = 0; k < kKeyWords; k++) eq &= x[k] == y[k];
  return eq;
}

__global__ void __launch_bounds__(256) insert_kernel(const uint32_t* keys, const uint64_t* hash, const int32_t* code,
                                                     uint64_t n, unsigned long long* table, uint64_t tmask,
                                                     uint32_t* slot_of) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || code[i]) return;
  const uint64_t h = hash[i];
  const unsigned long long tag = h >> kIdxBits;
  const unsigned long long word = tag << kIdxBits | i;
  uint64_t pos = h & tmask;
  // a table of 2x the batch never fills, so every probe sequence ends
  for (;;) {
    unsigned long long cur = __hip_atomic_load(&table[pos], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == kEmpty) {
      cur = atomicCAS(&table[pos], kEmpty, word);
      if (cur == kEmpty) break;  // this packet's key is new here
    }
    if ((cur >> kIdxBits) == tag && same_key(keys, i, cur & kIdxMask)) break;
    pos = (pos + 1) & tmask;
  }
  // The slot word's index field becomes the key's first packet: the tag is the
  // same for every packet of the key, so a 64-bit atomicMin of the word lowers
  // only the index. Elephant flows hit one slot many times: skip the atomic
  // once it cannot lower it.
  if ((__hip_atomic_load(&table[pos], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & kIdxMask) > i)
    atomicMin(&table[pos], word);
  slot_of[i] = (uint32_t)pos;
}

// FastHash buckets: each occupied bucket's rank by first appearance, so the
// sort key needs log2(buckets) bits instead of log2(batch) (one radix pass)
__global__ void __launch_bounds__(1024) bucket_rank_kernel(const uint32_t* bucket_min, uint32_t B, uint32_t* rank) {
  for (uint32_t b = threadIdx.x; b < B; b += blockDim.x) {
    const uint32_t m = bucket_min[b];
    uint32_t r = 0;
    for (uint32_t c = 0; c < B; c++) r += bucket_min[c] < m;  // distinct minima: no ties
    rank[b] = r;
  }
}

__global__ void __launch_bounds__(256) first_kernel(const int32_t* code, const uint32_t* slot_of,
                                                    const unsigned long long* table, const uint64_t* hash,
                                                    const uint32_t* bucket_key, int kind, uint64_t n, uint32_t sentinel,
                                                    uint32_t* f, uint32_t* iota) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t v = sentinel;  // not keyed: sorts after every group
  if (!code[i]) v = kind == GPK_GROUP_NET_BUCKET ? bucket_key[hash[i]] : (uint32_t)(table[slot_of[i]] & kIdxMask);
  f[i] = v;
  iota[i] = (uint32_t)i;
}

__global__ void __launch_bounds__(256) heads_kernel(const uint32_t* fs, uint64_t n, uint32_t sentinel,
                                                    uint32_t* heads) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t v = fs[j];
  heads[j] = v < sentinel && (j == 0 || fs[j - 1] != v) ? 1u : 0u;
}

__global__ void __launch_bounds__(256) finish_kernel(const uint32_t* fs, const uint32_t* perm, const uint32_t* gid,
                                                     const int32_t* code, uint64_t n, uint32_t sentinel,
                                                     int32_t* group_of, uint32_t* start, uint32_t* first,
                                                     uint32_t* counts) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t v = fs[j], pkt = perm[j];
  if (v >= sentinel) {
    group_of[pkt] = code[pkt];
    return;
  }
  const uint32_t g = gid[j] - 1;
  group_of[pkt] = (int32_t)g;
  if (j == 0 || fs[j - 1] != v) {
    start[g] = (uint32_t)j;
    first[g] = pkt;
  }
  if (j + 1 == n || fs[j + 1] >= sentinel) {  // the last keyed packet
    counts[0] = g + 1;
    counts[1] = (uint32_t)(j + 1);
    start[g + 1] = (uint32_t)(j + 1);
  }
}

// pack: caplens of the packets in `order`, then one wave per packet copying
// its bytes (64 consecutive bytes per wave instruction on both sides)
__global__ void __launch_bounds__(256) pack_caplens_kernel(const uint32_t* caplens, const uint32_t* order, uint64_t m,
                                                           uint32_t* out_caplens) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < m) out_caplens[j] = caplens[order[j]];
}

__global__ void __launch_bounds__(256) pack_bytes_kernel(const uint8_t* data, const uint64_t* offsets,
                                                         const uint32_t* order, const uint32_t* out_caplens,
                                                         const uint64_t* out_offsets, uint64_t m, uint8_t* out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / 64);
  for (uint64_t j = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); j < m; j += waves) {
    const uint8_t* src = data + offsets[order[j]];
    uint8_t* dst = out + out_offsets[j];
    const uint32_t n = out_caplens[j];
    for (uint32_t b = lane; b < n; b += 64) dst[b] = src[b];
  }
}

struct Widen64 {
  __host__ __device__ uint64_t operator()(uint32_t v) const { return v; }
};

}  // namespace

extern "C" int gpk_pack_batch(const gpk_batch* in, const uint32_t* order, uint64_t m, uint8_t* out_data,
                              uint64_t* out_offsets, uint32_t* out_caplens, void* stream) {
  if (!in || (m && (!order || !out_data || !out_offsets || !out_caplens || !in->data || !in->offsets ||
                    !in->caplens)))
    return GPK_EINVAL;
  if (m == 0) return GPK_OK;
  if (m >= (1ull << 31)) return GPK_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const dim3 blk(256), grd((unsigned)((m + 255) / 256));
  hipLaunchKernelGGL(pack_caplens_kernel, grd, blk, 0, s, in->caplens, order, m, out_caplens);
  hipcub::TransformInputIterator<uint64_t, Widen64, const uint32_t*> it(out_caplens, Widen64());
  size_t tb = 0;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, tb, it, out_offsets, (int)m, s) != hipSuccess) return GPK_EHIP;
  void* tmp = nullptr;
  if (hipMallocAsync(&tmp, tb, s) != hipSuccess) return GPK_ENOMEM;
  const bool ok = hipcub::DeviceScan::ExclusiveSum(tmp, tb, it, out_offsets, (int)m, s) == hipSuccess;
  (void)hipFreeAsync(tmp, s);
  if (!ok) return GPK_EHIP;
  const uint64_t want = (m + 3) / 4;  // 4 waves per block, one packet per wave per pass
  const unsigned blocks = (unsigned)(want < 65536 ? want : 65536);
  hipLaunchKernelGGL(pack_bytes_kernel, dim3(blocks), blk, 0, s, in->data, in->offsets, order, out_caplens,
                     out_offsets, m, out_data);
  return hipGetLastError() == hipSuccess ? GPK_OK : GPK_EHIP;
}

struct gpk_grouper {
  int device = 0;
  uint64_t cap = 0, tsize = 0;
  uint32_t* keys = nullptr;
  uint64_t* hash = nullptr;
  int32_t* code = nullptr;
  uint32_t* slot_of = nullptr;
  unsigned long long* table = nullptr;
  uint32_t* bucket_min = nullptr;
  uint32_t* brank = nullptr;
  uint32_t buckets = 0;
  uint32_t* f = nullptr;
  uint32_t* fs = nullptr;
  uint32_t* iota = nullptr;
  uint32_t* heads = nullptr;
  uint32_t* gid = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
};

namespace {

int end_bit(uint64_t n) {  // bits to hold 0..n
  int b = 1;
  while (b < 32 && (1ull << b) <= n) b++;
  return b;
}

void free_all(gpk_grouper* g) {
  for (void* p : {(void*)g->keys, (void*)g->hash, (void*)g->code, (void*)g->slot_of, (void*)g->table,
                  (void*)g->bucket_min, (void*)g->brank, (void*)g->f, (void*)g->fs, (void*)g->iota,
                  (void*)g->heads, (void*)g->gid, g->tmp})
    if (p) (void)hipFree(p);
}

}  // namespace

static int group_rest(gpk_grouper* g, uint64_t n, int kind, const gpk_groups& o, hipStream_t s);

extern "C" int gpk_grouper_create(gpk_grouper** out, int device, uint64_t max_packets) {
  if (!out || max_packets == 0 || max_packets >= (1ull << kIdxBits)) return GPK_EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return GPK_ENODEV;
  gpk::DeviceScope dscope(device);  // the caller's device is restored on return
  if (dscope.err != hipSuccess) return GPK_EHIP;
  gpk_grouper* g = new (std::nothrow) gpk_grouper();
  if (!g) return GPK_ENOMEM;
  g->device = device;
  g->cap = max_packets;
  g->tsize = 1;
  while (g->tsize < 2 * max_packets) g->tsize <<= 1;
  const uint64_t n = max_packets;
  size_t sort_bytes = 0, scan_bytes = 0;
  bool ok = hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                               (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, 32) == hipSuccess &&
            hipcub::DeviceScan::InclusiveSum(nullptr, scan_bytes, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n) ==
                hipSuccess;
  g->tmp_bytes = std::max(sort_bytes, scan_bytes);
  ok = ok && hipMalloc((void**)&g->keys, n * kKeyWords * 4) == hipSuccess &&
       hipMalloc((void**)&g->hash, n * 8) == hipSuccess && hipMalloc((void**)&g->code, n * 4) == hipSuccess &&
       hipMalloc((void**)&g->slot_of, n * 4) == hipSuccess &&
       hipMalloc((void**)&g->table, g->tsize * 8) == hipSuccess &&
       hipMalloc((void**)&g->bucket_min, (1u << 16) * 4) == hipSuccess &&
       hipMalloc((void**)&g->brank, (1u << 16) * 4) == hipSuccess &&
       hipMalloc((void**)&g->f, n * 4) == hipSuccess && hipMalloc((void**)&g->fs, n * 4) == hipSuccess &&
       hipMalloc((void**)&g->iota, n * 4) == hipSuccess && hipMalloc((void**)&g->heads, n * 4) == hipSuccess &&
       hipMalloc((void**)&g->gid, n * 4) == hipSuccess && hipMalloc(&g->tmp, g->tmp_bytes) == hipSuccess;
  if (!ok) {
    free_all(g);
    delete g;
    return GPK_ENOMEM;
  }
  *out = g;
  return GPK_OK;
}

extern "C" int gpk_grouper_destroy(gpk_grouper* g) {
  if (!g) return GPK_EINVAL;
  gpk::DeviceScope dscope(g->device);
  (void)hipDeviceSynchronize();
  free_all(g);
  delete g;
  return GPK_OK;
}

extern "C" int gpk_group_batch(gpk_grouper* g, const gpk_batch* b, const gpk_results* r, int kind, uint32_t buckets,
                               const gpk_groups* o, void* stream) {
  if (!g || !b || !r || !o || !r->records || !o->group_of || !o->perm || !o->start || !o->first || !o->counts)
    return GPK_EINVAL;
  if (kind != GPK_GROUP_CONNECTION && kind != GPK_GROUP_DEFRAG && kind != GPK_GROUP_NET_BUCKET) return GPK_EINVAL;
  if (kind == GPK_GROUP_NET_BUCKET && (!r->flows || buckets == 0 || buckets > (1u << 16) || (buckets & (buckets - 1))))
    return GPK_EINVAL;
  if (kind != GPK_GROUP_NET_BUCKET && (!r->layouts || !b->data || !b->offsets)) return GPK_EINVAL;
  const uint64_t n = b->n;
  if (n > g->cap) return GPK_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  gpk::DeviceScope dscope(g->device);
  if (dscope.err != hipSuccess) return GPK_EHIP;
  if (hipMemsetAsync(o->counts, 0, 8, s) != hipSuccess || hipMemsetAsync(o->start, 0, 4, s) != hipSuccess)
    return GPK_EHIP;
  if (n == 0) return GPK_OK;
  const dim3 blk(256), grd((unsigned)((n + 255) / 256));
  if (kind == GPK_GROUP_NET_BUCKET) {
    if (hipMemsetAsync(g->bucket_min, 0xFF, (size_t)buckets * 4, s) != hipSuccess) return GPK_EHIP;
  } else if (hipMemsetAsync(g->table, 0xFF, g->tsize * 8, s) != hipSuccess) {
    return GPK_EHIP;
  }
  KeyArgs a{b->data, b->offsets, b->caplens, r->records, r->layouts, r->flows, n, kind, buckets,
            g->keys, g->hash, g->code, g->bucket_min};
  hipLaunchKernelGGL(key_kernel, grd, blk, 0, s, a);
  g->buckets = buckets;
  return group_rest(g, n, kind, *o, s);
}

extern "C" int gpk_decode_group_batch(gpk_ctx* ctx, const gpk_parser* p, const gpk_batch* b, const gpk_results* r,
                                      gpk_grouper* g, int kind, const gpk_groups* o, void* stream) {
  if (!ctx || !p || !b || !r || !g || !o || !o->group_of || !o->perm || !o->start || !o->first || !o->counts)
    return GPK_EINVAL;
  if (kind != GPK_GROUP_CONNECTION && kind != GPK_GROUP_DEFRAG) return GPK_EINVAL;
  const uint64_t n = b->n;
  if (n > g->cap) return GPK_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  int rc = gpk_decode_batch_keys(ctx, p, b, r, kind, g->keys, g->hash, g->code, stream);
  if (rc) return rc;
  gpk::DeviceScope dscope(g->device);
  if (dscope.err != hipSuccess) return GPK_EHIP;
  if (hipMemsetAsync(o->counts, 0, 8, s) != hipSuccess || hipMemsetAsync(o->start, 0, 4, s) != hipSuccess)
    return GPK_EHIP;
  if (n == 0) return GPK_OK;
  if (hipMemsetAsync(g->table, 0xFF, g->tsize * 8, s) != hipSuccess) return GPK_EHIP;
  return group_rest(g, n, kind, *o, s);
}

static int group_rest(gpk_grouper* g, uint64_t n, int kind, const gpk_groups& o, hipStream_t s) {
  const dim3 blk(256), grd((unsigned)((n + 255) / 256));
  if (kind != GPK_GROUP_NET_BUCKET)
    hipLaunchKernelGGL(insert_kernel, grd, blk, 0, s, g->keys, g->hash, g->code, n, g->table, g->tsize - 1,
                       g->slot_of);
  // sort key: the key's first packet index (sentinel n), or for buckets the
  // bucket's first-appearance rank (sentinel = buckets: a few bits)
  uint32_t sentinel = (uint32_t)n;
  const uint32_t* bkey = g->bucket_min;
  if (kind == GPK_GROUP_NET_BUCKET && g->buckets <= 4096) {
    hipLaunchKernelGGL(bucket_rank_kernel, dim3(1), dim3(1024), 0, s, g->bucket_min, g->buckets, g->brank);
    sentinel = g->buckets;
    bkey = g->brank;
  }
  hipLaunchKernelGGL(first_kernel, grd, blk, 0, s, g->code, g->slot_of, g->table, g->hash, bkey, kind, n, sentinel,
                     g->f, g->iota);
  size_t tb = g->tmp_bytes;
  if (hipcub::DeviceRadixSort::SortPairs(g->tmp, tb, g->f, g->fs, g->iota, o.perm, (int)n, 0, end_bit(sentinel), s) !=
      hipSuccess)
    return GPK_EHIP;
  hipLaunchKernelGGL(heads_kernel, grd, blk, 0, s, g->fs, n, sentinel, g->heads);
  tb = g->tmp_bytes;
  if (hipcub::DeviceScan::InclusiveSum(g->tmp, tb, g->heads, g->gid, (int)n, s) != hipSuccess) return GPK_EHIP;
  hipLaunchKernelGGL(finish_kernel, grd, blk, 0, s, g->fs, o.perm, g->gid, g->code, n, sentinel, o.group_of, o.start,
                     o.first, o.counts);
  return hipGetLastError() == hipSuccess ? GPK_OK : GPK_EHIP;
}

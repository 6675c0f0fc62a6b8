/*
 * flows_oracle.c — C restatement of the flow consumers' keying
 * (oracle/flows_oracle.py) with a hash map, for the CPU
 * baseline of the grouping bench (the Go reference keys each packet with one
 * map lookup: tcpassembly/assembly.go:498-545, ip4defrag/defrag.go:85-105).
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/ (checked against the Python
 * oracle) and bench.py's CPU baseline; nothing in gopacket_amd/ calls it.
 * Same keys, same harness rules, same codes as the Python restatement.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/gpk.h"

#define KW 10

static uint32_t ld4(const uint8_t* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }

/* 0 = keyed (w set), else a GPK_GROUP_* code (include/gpk_flows.h) */
static int key_of(int kind, const uint8_t* p, const gpk_record* rec, const gpk_layout* L, uint64_t net_hash,
                  uint32_t buckets, uint32_t* w) {
  memset(w, 0, KW * 4);
  const uint32_t st = rec->status, nl = (st >> 8) & 0xFFF;
  if (kind == 3) {
    if (!(st & GPK_ST_NET_FLOW)) return -1;
    w[0] = (uint32_t)(net_hash & (uint64_t)(buckets - 1));
    return 0;
  }
  if (kind == 1) {
    const uint32_t t0 = L->start[5];
    if (t0 == GPK_LAYOUT_ABSENT) return -1;
    uint32_t net = 0, seen = 0, m = nl < 16 ? nl : 16;
    for (uint32_t k = 0; k < m && !seen; k++) {
      uint32_t c = (uint32_t)(rec->layers >> (4 * k)) & 15;
      if (c == 3 || c == 4) net = c;
      seen = c == 9;
    }
    if (!seen) return -6;
    if (!net) return -1;
    const uint32_t flags = p[t0 + 13], doff = p[t0 + 12] >> 4;
    if (!(flags & 7) && (L->end[5] - t0) - doff * 4 == 0) return -2;
    if (net == 3) {
      const uint8_t* ip = p + L->start[2];
      w[0] = 1 | 1 << 8 | 4 << 16;
      w[1] = ld4(ip + 12);
      w[5] = ld4(ip + 16);
    } else {
      const uint8_t* ip = p + L->start[3];
      w[0] = 1 | 2 << 8 | 4 << 16;
      for (int k = 0; k < 4; k++) {
        w[1 + k] = ld4(ip + 8 + 4 * k);
        w[5 + k] = ld4(ip + 24 + 4 * k);
      }
    }
    w[9] = ld4(p + t0);
    return 0;
  }
  const uint32_t s = L->start[2];
  const uint32_t err = st & 0x7F;
  if (s == GPK_LAYOUT_ABSENT || (err >= 20 && err <= 27)) return -1;
  const uint8_t* ip = p + s;
  const uint32_t ff = (uint32_t)ip[6] << 8 | ip[7], flags = ff >> 13, fo = ff & 0x1FFF;
  if (flags & 2) return -1;
  if (!(flags & 1) && fo == 0) return -1;
  uint32_t len = (uint32_t)ip[2] << 8 | ip[3];
  if (len == 0) len = (L->end[2] - s) & 0xFFFF;
  if ((flags & 1) && ((len - (ip[0] & 15) * 4) & 0xFFFF) < 8) return -3;
  if (fo > 8183) return -4;
  if (((fo * 8 + len) & 0xFFFF) > 65535) return -5;
  w[0] = 2 | 1 << 8;
  w[1] = ld4(ip + 12);
  w[5] = ld4(ip + 16);
  w[9] = (uint32_t)ip[4] << 8 | ip[5];
  return 0;
}

/* group_of[i] = group id (first-appearance order) or a code < 0; returns the
 * number of groups, or -1 when out of memory. */
int64_t oracle_group_batch(int kind, const uint8_t* data, const uint64_t* offsets, const gpk_record* records,
                           const gpk_layout* layouts, const uint64_t* flows, uint64_t n, uint32_t buckets,
                           int32_t* group_of) {
  uint64_t cap = 16;
  while (cap < 2 * n + 2) cap <<= 1;
  uint32_t* keys = (uint32_t*)malloc(cap * KW * 4);
  int64_t* gid = (int64_t*)malloc(cap * 8);
  if (!keys || !gid) {
    free(keys);
    free(gid);
    return -1;
  }
  for (uint64_t k = 0; k < cap; k++) gid[k] = -1;
  int64_t groups = 0;
  uint32_t w[KW];
  for (uint64_t i = 0; i < n; i++) {
    const int c = key_of(kind, data + offsets[i], &records[i], layouts ? &layouts[i] : NULL,
                         flows ? flows[n + i] : 0, buckets, w);
    if (c) {
      group_of[i] = c;
      continue;
    }
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (int k = 0; k < KW; k++) {
      h = (h ^ w[k]) * 0xBF58476D1CE4E5B9ull;
      h ^= h >> 29;
    }
    uint64_t pos = h & (cap - 1);
    for (;;) {  /* the map lookup of the reference, one per packet */
      if (gid[pos] < 0) {
        memcpy(keys + pos * KW, w, KW * 4);
        gid[pos] = groups++;
        break;
      }
      if (!memcmp(keys + pos * KW, w, KW * 4)) break;
      pos = (pos + 1) & (cap - 1);
    }
    group_of[i] = (int32_t)gid[pos];
  }
  free(keys);
  free(gid);
  return groups;
}

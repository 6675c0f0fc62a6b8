// gpk_kernels.hip — batched DecodingLayerParser + Internet checksum + Flow
// hash for gfx950 (MI355X). Hand-written HIP; no MFMA (byte parse and integer
// reduction, HBM-bandwidth bound).
//
// One workgroup = 256 packets = 4 waves. Per packet the bytes are read once:
//
//  Phase A (lane per packet): the packet's first 128 B (16-byte aligned
//    chunks) are loaded with global_load_dwordx4 into the lane's LDS slot;
//    the lane runs DecodeLayers (gpk_device.h) out of LDS, computes the IPv4
//    header checksum (ip4.go:323-332), the three Flow.FastHash values
//    (flows.go:167-174) and, when the whole TCP/UDP segment sits inside the
//    window, the L4 checksum (tcpip.go:54-69) too.
//  Phase B (wave-cooperative): TCP/UDP segments that extend past the window
//    are summed by the whole wave. The wave's segments are cut into 16-byte
//    chunks laid end to end (exclusive scan of chunk counts); lane l takes
//    chunk t+l, so consecutive lanes load consecutive 16-byte chunks of the
//    same packet (coalesced dwordx4). Partial sums are combined with a
//    segmented scan keyed by packet and added into a per-packet LDS
//    accumulator. RFC1071 sums are position independent except for byte
//    parity, and ComputeChecksum wraps mod 2^32 (checksum.go:40-49), so
//    summing mod 2^32 in any order is bit-exact.
#include <hip/hip_runtime.h>

#include "gpk_device.h"

namespace gpk {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Streaming 16-byte load (read-once packet bytes: non-temporal).
__device__ __forceinline__ uint4 ld16(const uint8_t* p) {
  u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(x.x, x.y, x.z, x.w);
}

// Sum of big-endian 16-bit words over LDS bytes [q, q+n) (ComputeChecksum
// with csum = 0; an odd tail byte counts <<8). n <= window size.
__device__ __forceinline__ uint32_t sum_words_lds(uint32_t q, uint32_t n) {
  uint32_t e = q + n;
  uint32_t E = 0, O = 0;
  for (uint32_t a = q & ~3u; a < e; a += 4) {
    uint32_t w = gpk_smem[a >> 2];
    uint32_t lo = q > a ? q - a : 0u;
    uint32_t hi = e - a < 4u ? e - a : 4u;
    w &= (0xffffffffu >> (8 * (4 - hi))) & (0xffffffffu << (8 * lo));
    E += w & 0x00ff00ffu;
    O += (w >> 8) & 0x00ff00ffu;
  }
  E = (E & 0xffff) + (E >> 16);
  O = (O & 0xffff) + (O >> 16);
  return (q & 1) ? (O << 8) + E : (E << 8) + O;
}

// Same over packet positions [p, p+n), from LDS when inside the window.
__device__ __forceinline__ uint32_t sum_words(const Rd& r, uint32_t p, uint32_t n) {
  if (p + n <= r.win) return sum_words_lds(r.lb + p, n);
  uint32_t s = 0;
  for (uint32_t k = 0; k + 1 < n; k += 2) s += rd16(r, p + k);
  if (n & 1) s += rd8(r, p + n - 1) << 8;
  return s;
}

// 16 bytes of a 16-aligned chunk at absolute address A, restricted to
// [s, e), each byte weighted <<8 when (pos - s) is even.
__device__ __forceinline__ uint32_t chunk_sum(uint4 v, uint64_t A, uint64_t s, uint64_t e) {
  uint32_t lo = s > A ? (uint32_t)(s - A) : 0u;          // 0..15
  uint32_t hi = e < A + 16 ? (uint32_t)(e - A) : 16u;    // 1..16
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t E = 0, O = 0;
#pragma unroll
  for (int d = 0; d < 4; d++) {
    int l = (int)lo - 4 * d, h = (int)hi - 4 * d;
    l = l < 0 ? 0 : (l > 4 ? 4 : l);
    h = h < 0 ? 0 : (h > 4 ? 4 : h);
    uint32_t m = h > l ? ((0xffffffffu >> (8 * (4 - (h - l)))) << (8 * l)) : 0u;
    uint32_t x = w[d] & m;
    E += x & 0x00ff00ffu;
    O += (x >> 8) & 0x00ff00ffu;
  }
  E = (E & 0xffff) + (E >> 16);
  O = (O & 0xffff) + (O >> 16);
  return (s & 1) ? (O << 8) + E : (E << 8) + O;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, uint32_t lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t o = __shfl_up(v, d, 64);
    if (lane >= (uint32_t)d) v += o;
  }
  return v;
}

template <bool kL4, bool kLayout>
__global__ __launch_bounds__(kBlock) void decode_kernel(KParams P) {
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63;
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + tid;
  const bool active = i < P.n;

  uint64_t off = 0;
  uint32_t cl = 0;
  if (active) {
    off = P.offsets[i];
    cl = P.caplens[i];
  }
  // ---- header window -> LDS slot (coalesced 16-byte chunk loads) ----------
  const uint32_t m = (uint32_t)(off & 15);
  const uint32_t slot_dw = tid * kSlotDw;
  uint32_t win = kWinChunks * 16 - m;
  if (cl < win) win = cl;
  const uint32_t nchunk = active ? (m + win + 15) >> 4 : 0;
  {
    const uint8_t* src = P.data + (off - m);
    uint4 v[kWinChunks];
#pragma unroll
    for (int k = 0; k < kWinChunks; k++)
      if ((uint32_t)k < nchunk) v[k] = ld16(src + 16 * k);
#pragma unroll
    for (int k = 0; k < kWinChunks; k++)
      if ((uint32_t)k < nchunk) {
        gpk_smem[slot_dw + 4 * k + 0] = v[k].x;
        gpk_smem[slot_dw + 4 * k + 1] = v[k].y;
        gpk_smem[slot_dw + 4 * k + 2] = v[k].z;
        gpk_smem[slot_dw + 4 * k + 3] = v[k].w;
      }
  }
  Rd r{P.data + off, slot_dw * 4 + m, win};

  // ---- Phase A: DecodeLayers ------------------------------------------------
  Parse q;
  q.init();
  Outcome s{0, 0, 0, 0};
  if (active) s = run_parser<false>(P, r, cl, q);

  uint32_t st = (s.err & GPK_ST_ERR_MASK) | (s.trunc ? GPK_ST_TRUNCATED : 0u) |
                ((q.nlayers > GPK_ST_NLAYERS_MASK ? GPK_ST_NLAYERS_MASK : q.nlayers) << GPK_ST_NLAYERS_SHIFT);
  uint32_t ip4c = 0, l4c = 0;
  uint64_t lflow = 0, nflow = 0, tflow = 0;

  // Job for the L4 checksum: bytes [jstart, jstart+jlen) of data.
  uint64_t jstart = 0;
  uint32_t jlen = 0, jinit = 0, jexist = 0;
  bool jdone = true;

  if (active) {
    if ((P.outputs & GPK_OUT_IP4_CSUM) && clean(q, GPK_DEC_IPV4)) {  // ip4.go:323-332
      uint32_t s4 = q.start(GPK_DEC_IPV4);
      uint32_t hl = (rd8(r, s4) & 15) * 4;
      uint32_t existing = rd16(r, s4 + 10);
      ip4c = fold(sum_words(r, s4, hl) - existing);
      st |= GPK_ST_IP4_CSUM | (ip4c == existing ? GPK_ST_IP4_VALID : 0u);
    }
    const uint32_t tk = q.transport, nk = q.last_net;
    if ((P.outputs & GPK_OUT_L4_CSUM) && tk && clean(q, tk) && nk && clean(q, nk)) {
      // tcp.go:626-640 / udp.go:144-158 via tcpip.go:54-69
      uint32_t t0 = q.start(tk);
      uint32_t blen = tk == GPK_DEC_TCP ? q.end(tk) - t0 : q.udp_hlen;
      uint32_t ns = q.start(nk);
      uint32_t init = nk == GPK_DEC_IPV4 ? sum_words(r, ns + 12, 8) : sum_words(r, ns + 8, 32);
      init += (tk == GPK_DEC_TCP ? 6u : 17u) + (blen & 0xffff) + (blen >> 16);
      jexist = rd16(r, t0 + (tk == GPK_DEC_TCP ? 16 : 6));
      st |= GPK_ST_L4_CSUM | (tk == GPK_DEC_UDP ? GPK_ST_L4_UDP : 0u);
      if (t0 + blen <= r.win) {
        uint32_t c = init + sum_words_lds(r.lb + t0, blen);
        l4c = fold(c - jexist);
      } else {
        jdone = false;
        jstart = off + t0;
        jlen = blen;
        jinit = init;
      }
    }
    if (P.outputs & GPK_OUT_FLOWS) {
      if (clean(q, GPK_DEC_ETHERNET)) {  // ethernet.go:38-40 (EndpointMAC = 3)
        uint32_t e0 = q.start(GPK_DEC_ETHERNET);
        lflow = flow_hash(fnv_range(r, e0 + 6, 6), fnv_range(r, e0, 6), 3);
        st |= GPK_ST_LINK_FLOW;
      }
      if (nk && clean(q, nk)) {
        uint32_t ns = q.start(nk);
        if (nk == GPK_DEC_IPV4) {  // ip4.go:63-65 (EndpointIPv4 = 1)
          nflow = flow_hash(fnv_range(r, ns + 12, 4), fnv_range(r, ns + 16, 4), 1);
        } else {  // ip6.go:49-51 (EndpointIPv6 = 2)
          nflow = flow_hash(fnv_range(r, ns + 8, 16), fnv_range(r, ns + 24, 16), 2);
          st |= GPK_ST_NET_IPV6;
        }
        st |= GPK_ST_NET_FLOW;
      }
      if (tk && clean(q, tk)) {  // tcp.go:614-616 (4), udp.go:132-134 (5)
        uint32_t t0 = q.start(tk);
        tflow = flow_hash(fnv_range(r, t0, 2), fnv_range(r, t0 + 2, 2), tk == GPK_DEC_TCP ? 4 : 5);
        st |= GPK_ST_TRANSPORT_FLOW;
      }
    }
  }

  // ---- Phase B: wave-cooperative L4 checksum of segments past the window ---
  if (kL4) {
    // Per-wave scratch overlays this wave's LDS slots (no longer read).
    uint32_t* W = gpk_smem + (tid & ~63u) * kSlotDw;
    uint64_t* Jst = reinterpret_cast<uint64_t*>(W);  // [64] (slot base is 8-aligned: 64*33*4 per wave)
    uint64_t* Jen = Jst + 64;                           // [64]
    uint32_t* Base = W + 256;                           // [65]
    uint32_t* Acc = W + 256 + 72;                       // [64]
    uint32_t nch = 0;
    if (!jdone) nch = (uint32_t)(((jstart + jlen + 15) >> 4) - (jstart >> 4));
    uint32_t incl = wave_incl_scan(nch, lane);
    uint32_t total = __shfl(incl, 63, 64);
    if (total) {
      __builtin_amdgcn_wave_barrier();
      Jst[lane] = jstart;
      Jen[lane] = jstart + jlen;
      Base[lane] = incl - nch;
      if (lane == 63) Base[64] = total;
      Acc[lane] = 0;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      constexpr int U = 4;
      for (uint32_t t = 0; t < total; t += 64 * U) {
        uint4 v[U];
        uint32_t key[U];
        uint64_t A[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
          uint32_t c = t + u * 64 + lane;
          key[u] = 64;
          if (c < total) {
            uint32_t j = 0;
#pragma unroll
            for (uint32_t stp = 32; stp; stp >>= 1)
              if (Base[j + stp] <= c) j += stp;
            key[u] = j;
            A[u] = ((Jst[j] >> 4) + (c - Base[j])) << 4;
            v[u] = ld16(P.data + A[u]);
          }
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
          uint32_t j = key[u];
          uint32_t val = j < 64 ? chunk_sum(v[u], A[u], Jst[j], Jen[j]) : 0u;
          // segmented inclusive scan keyed by packet (keys are non-decreasing)
#pragma unroll
          for (int d = 1; d < 64; d <<= 1) {
            uint32_t vo = __shfl_up(val, d, 64);
            uint32_t ko = __shfl_up(j, d, 64);
            if (lane >= (uint32_t)d && ko == j) val += vo;
          }
          uint32_t kn = __shfl_down(j, 1, 64);
          bool last = (lane == 63) || kn != j;
          if (last && j < 64) Acc[j] += val;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
      }
      if (!jdone) {
        uint32_t c = jinit + Acc[lane];
        l4c = fold(c - jexist);
      }
    }
  }
  if (active && (st & GPK_ST_L4_CSUM)) {
    bool udp = (st & GPK_ST_L4_UDP) != 0;
    if (l4c == jexist || (udp && jexist == 0)) st |= GPK_ST_L4_VALID;
  }

  // ---- outputs ---------------------------------------------------------------
  if (active) {
    uint4 rec = make_uint4((uint32_t)q.layers, (uint32_t)(q.layers >> 32), st, ip4c | (l4c << 16));
    reinterpret_cast<uint4*>(P.records)[i] = rec;
    if (P.flows) {
      P.flows[i] = lflow;
      P.flows[P.n + i] = nflow;
      P.flows[2 * P.n + i] = tflow;
    }
    if (s.err && P.err_args) {
      P.err_args[2 * i] = s.a0;
      P.err_args[2 * i + 1] = s.a1;
    }
    if (kLayout) {
      const int slot_kind[8] = {GPK_DEC_ETHERNET, GPK_DEC_DOT1Q, GPK_DEC_IPV4, GPK_DEC_IPV6,
                                       GPK_DEC_IPV6_EXT, GPK_DEC_TCP,  GPK_DEC_UDP,  GPK_DEC_PAYLOAD};
      uint32_t so[8], eo[8];
#pragma unroll
      for (int k = 0; k < 8; k++) {
        int kd = slot_kind[k];
        if (k == 7 && !clean(q, GPK_DEC_PAYLOAD)) kd = GPK_DEC_FRAGMENT;
        bool c = clean(q, kd);
        so[k] = c ? q.start(kd) : GPK_LAYOUT_ABSENT;
        eo[k] = c ? q.end(kd) : GPK_LAYOUT_ABSENT;
      }
      uint4* L = reinterpret_cast<uint4*>(P.layouts + i);
      L[0] = make_uint4(so[0], so[1], so[2], so[3]);
      L[1] = make_uint4(so[4], so[5], so[6], so[7]);
      L[2] = make_uint4(eo[0], eo[1], eo[2], eo[3]);
      L[3] = make_uint4(eo[4], eo[5], eo[6], eo[7]);
    }
  }
}

// Full decoded list of one packet (lists longer than the 16 inline codes).
__global__ void list_kernel(KParams P, uint64_t index, int64_t* out, uint32_t cap, uint32_t* out_n) {
  if (threadIdx.x != 0) return;
  uint64_t off = P.offsets[index];
  uint32_t cl = P.caplens[index];
  Rd r{P.data + off, 0, 0};  // no LDS window: every byte from global memory
  Parse q;
  run_parser<true>(P, r, cl, q, out, cap);
  *out_n = q.nlayers;
}

}  // namespace gpk

extern "C" hipError_t gpk_launch_decode(const gpk::KParams* P, int with_l4, int with_layout, hipStream_t stream) {
  using namespace gpk;
  if (P->n == 0) return hipSuccess;
  dim3 grid((unsigned)((P->n + kBlock - 1) / kBlock));
  dim3 block(kBlock);
  if (with_l4 && with_layout)
    hipLaunchKernelGGL((decode_kernel<true, true>), grid, block, kLdsBytes, stream, *P);
  else if (with_l4)
    hipLaunchKernelGGL((decode_kernel<true, false>), grid, block, kLdsBytes, stream, *P);
  else if (with_layout)
    hipLaunchKernelGGL((decode_kernel<false, true>), grid, block, kLdsBytes, stream, *P);
  else
    hipLaunchKernelGGL((decode_kernel<false, false>), grid, block, kLdsBytes, stream, *P);
  return hipGetLastError();
}

extern "C" hipError_t gpk_launch_list(const gpk::KParams* P, uint64_t index, int64_t* out, uint32_t cap,
                                      uint32_t* out_n, hipStream_t stream) {
  hipLaunchKernelGGL(gpk::list_kernel, dim3(1), dim3(64), 0, stream, *P, index, out, cap, out_n);
  return hipGetLastError();
}

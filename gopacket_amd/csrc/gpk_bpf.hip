// gpk_bpf.hip — classic BPF over a packet batch on gfx950 (include/gpk_bpf.h,
// SURVEY.md §8(f)4).
//
// One lane per packet, one program for the wave. Every lane keeps its own
// program counter; the wave executes, at each step, the instruction at the
// smallest program counter among its live lanes (a wave minimum), fetched
// once with scalar loads, and only the lanes standing there execute it. BPF
// programs from tcpdump/pcap_compile jump forward only, so the lanes of a
// wave walk the program together and each instruction is issued at most once
// per wave with a wave-uniform opcode (no divergent switch); the rare backward
// JA (ip6 protochain) just lowers the minimum again. Scratch memory M[16] is
// per lane in LDS. Packet loads are byte loads from the packet in HBM, bounds
// checked against the caplen as libpcap's bpf_filter does.
//
// Semantics: libpcap 1.10 bpf_filter (restated in oracle/bpf_oracle.c, which
// also lists what is undefined there and what this does instead).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdio>
#include <cstring>
#include <new>

#include "../../include/gpk_bpf.h"

extern "C" __device__ uint32_t __ockl_wfred_min_u32(uint32_t);

namespace {

constexpr uint32_t kMaxSteps = 1u << 20;  // a program that never returns: no match
constexpr int kBlock = 256;

__device__ __forceinline__ uint32_t be32(const uint8_t* p) {
  return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}
__device__ __forceinline__ uint32_t be16(const uint8_t* p) { return (uint32_t)p[0] << 8 | p[1]; }

__global__ void __launch_bounds__(kBlock) bpf_kernel(const gpk_bpf_insn* __restrict__ prog, uint32_t len,
                                                     const uint8_t* __restrict__ data,
                                                     const uint64_t* __restrict__ offsets,
                                                     const uint32_t* __restrict__ caplens,
                                                     const uint32_t* __restrict__ wirelens, uint64_t n,
                                                     uint32_t* __restrict__ ret, uint8_t* __restrict__ flags) {
  __shared__ uint32_t M[16 * kBlock];
  const uint32_t t = threadIdx.x;
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + t;
  bool live = i < n;
  const uint8_t* p = data;
  uint32_t buflen = 0, wirelen = 0;
  if (live) {
    p = data + offsets[i];
    buflen = caplens[i];
    wirelen = wirelens ? wirelens[i] : buflen;
  }
#pragma unroll
  for (int k = 0; k < 16; k++) M[k * kBlock + t] = 0;
  uint32_t A = 0, X = 0, r = 0, lpc = 0, steps = 0;
  for (;;) {
    if (live && (lpc >= len || steps == kMaxSteps)) {  // ran past the end / never returns
      r = 0;
      live = false;
    }
    const uint32_t pc = __builtin_amdgcn_readfirstlane(__ockl_wfred_min_u32(live ? lpc : 0xFFFFFFFFu));
    if (pc == 0xFFFFFFFFu) break;  // every lane has returned
    const gpk_bpf_insn ins = prog[pc];  // wave-uniform: scalar loads
    const uint32_t code = __builtin_amdgcn_readfirstlane(ins.code);
    const uint32_t K = __builtin_amdgcn_readfirstlane(ins.k);
    const uint32_t jt = __builtin_amdgcn_readfirstlane(ins.jt), jf = __builtin_amdgcn_readfirstlane(ins.jf);
    if (live && lpc == pc) {
      steps++;
      bool done = false, ok = true;
      uint32_t k;
      switch (code) {
        case 0x06: r = K; done = true; break;  // RET K
        case 0x16: r = A; done = true; break;  // RET A
        case 0x20:                            // LD W ABS
          ok = !(K > buflen || 4 > buflen - K);
          if (ok) A = be32(p + K);
          break;
        case 0x28:  // LD H ABS
          ok = !(K > buflen || 2 > buflen - K);
          if (ok) A = be16(p + K);
          break;
        case 0x30:  // LD B ABS
          ok = K < buflen;
          if (ok) A = p[K];
          break;
        case 0x80: A = wirelen; break;  // LD W LEN
        case 0x81: X = wirelen; break;  // LDX W LEN
        case 0x40:                      // LD W IND
          k = X + K;
          ok = !(K > buflen || X > buflen - K || 4 > buflen - k);
          if (ok) A = be32(p + k);
          break;
        case 0x48:  // LD H IND
          k = X + K;
          ok = !(X > buflen || K > buflen - X || 2 > buflen - k);
          if (ok) A = be16(p + k);
          break;
        case 0x50:  // LD B IND
          k = X + K;
          ok = !(K >= buflen || X >= buflen - K);
          if (ok) A = p[k];
          break;
        case 0xb1:  // LDX MSH B
          ok = K < buflen;
          if (ok) X = (uint32_t)(p[K] & 0xf) << 2;
          break;
        case 0x00: A = K; break;  // LD IMM
        case 0x01: X = K; break;  // LDX IMM
        case 0x60: ok = K < 16; if (ok) A = M[K * kBlock + t]; break;  // LD MEM
        case 0x61: ok = K < 16; if (ok) X = M[K * kBlock + t]; break;  // LDX MEM
        case 0x02: ok = K < 16; if (ok) M[K * kBlock + t] = A; break;  // ST
        case 0x03: ok = K < 16; if (ok) M[K * kBlock + t] = X; break;  // STX
        case 0x05: lpc += K; break;                                    // JA (sign-extended k)
        case 0x25: lpc += (A > K) ? jt : jf; break;                    // JGT K
        case 0x35: lpc += (A >= K) ? jt : jf; break;                   // JGE K
        case 0x15: lpc += (A == K) ? jt : jf; break;                   // JEQ K
        case 0x45: lpc += (A & K) ? jt : jf; break;                    // JSET K
        case 0x2d: lpc += (A > X) ? jt : jf; break;                    // JGT X
        case 0x3d: lpc += (A >= X) ? jt : jf; break;                   // JGE X
        case 0x1d: lpc += (A == X) ? jt : jf; break;                   // JEQ X
        case 0x4d: lpc += (A & X) ? jt : jf; break;                    // JSET X
        case 0x0c: A += X; break;
        case 0x1c: A -= X; break;
        case 0x2c: A *= X; break;
        case 0x3c: ok = X != 0; if (ok) A /= X; break;
        case 0x9c: ok = X != 0; if (ok) A %= X; break;
        case 0x5c: A &= X; break;
        case 0x4c: A |= X; break;
        case 0xac: A ^= X; break;
        case 0x6c: A = X < 32 ? A << X : 0u; break;
        case 0x7c: A = X < 32 ? A >> X : 0u; break;
        case 0x04: A += K; break;
        case 0x14: A -= K; break;
        case 0x24: A *= K; break;
        case 0x34: ok = K != 0; if (ok) A /= K; break;
        case 0x94: ok = K != 0; if (ok) A %= K; break;
        case 0x54: A &= K; break;
        case 0x44: A |= K; break;
        case 0xa4: A ^= K; break;
        case 0x64: A <<= (K & 31); break;
        case 0x74: A >>= (K & 31); break;
        case 0x84: A = 0u - A; break;  // NEG
        case 0x07: X = A; break;       // TAX
        case 0x87: A = X; break;       // TXA
        default: ok = false; break;    // libpcap aborts
      }
      if (!ok) {
        r = 0;
        done = true;
      }
      if (done) {
        live = false;
      } else {
        lpc++;
      }
    }
  }
  if (i < n) {
    ret[i] = r;
    if (flags) flags[i] = r != 0;
  }
}

__global__ void gather_kernel(const uint32_t* __restrict__ idx, const uint32_t* __restrict__ count,
                              const uint64_t* __restrict__ offsets, const uint32_t* __restrict__ caplens,
                              uint64_t* __restrict__ out_off, uint32_t* __restrict__ out_cap, uint64_t n) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n || j >= *count) return;
  const uint32_t k = idx[j];
  out_off[j] = offsets[k];
  out_cap[j] = caplens[k];
}

}  // namespace

struct gpk_bpf {
  gpk_bpf_insn* prog = nullptr;
  uint32_t len = 0;
  uint32_t* ret = nullptr;  // select scratch
  uint8_t* flags = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  uint64_t cap = 0;
};

extern "C" int gpk_bpf_create(gpk_bpf** out, const gpk_bpf_insn* insns, uint32_t n, char* err, size_t cap) {
  if (!out) return GPK_EINVAL;
  if (n < 1 || !insns) {  // bpfInstructionFilter (pcap.go:506-517)
    if (err && cap) snprintf(err, cap, "bpfInstructions must not be empty");
    return GPK_EINVAL;
  }
  if (n > GPK_BPF_MAX_INSNS) {
    if (err && cap) snprintf(err, cap, "bpfInstructions must not be larger than %d", GPK_BPF_MAX_INSNS);
    return GPK_EINVAL;
  }
  gpk_bpf* f = new (std::nothrow) gpk_bpf();
  if (!f) return GPK_ENOMEM;
  if (hipMalloc((void**)&f->prog, n * sizeof(gpk_bpf_insn)) != hipSuccess ||
      hipMemcpy(f->prog, insns, n * sizeof(gpk_bpf_insn), hipMemcpyHostToDevice) != hipSuccess) {
    if (f->prog) (void)hipFree(f->prog);
    delete f;
    if (err && cap) snprintf(err, cap, "device allocation failed");
    return GPK_EHIP;
  }
  f->len = n;
  *out = f;
  return GPK_OK;
}

extern "C" int gpk_bpf_destroy(gpk_bpf* f) {
  if (!f) return GPK_EINVAL;
  (void)hipDeviceSynchronize();
  for (void* p : {(void*)f->prog, (void*)f->ret, (void*)f->flags, f->tmp})
    if (p) (void)hipFree(p);
  delete f;
  return GPK_OK;
}

extern "C" int gpk_bpf_run(gpk_bpf* f, const gpk_batch* b, const uint32_t* wirelens, uint32_t* ret, void* stream) {
  if (!f || !b || !ret || (b->n && (!b->data || !b->offsets || !b->caplens))) return GPK_EINVAL;
  if (!b->n) return GPK_OK;
  const uint64_t blocks = (b->n + kBlock - 1) / kBlock;
  if (blocks > 0x7fffffffull) return GPK_EINVAL;  // the grid's x dimension
  hipLaunchKernelGGL(bpf_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, (hipStream_t)stream, f->prog, f->len,
                     b->data, b->offsets, b->caplens, wirelens, b->n, ret, (uint8_t*)nullptr);
  return hipGetLastError() == hipSuccess ? GPK_OK : GPK_EHIP;
}

extern "C" int gpk_bpf_select(gpk_bpf* f, const gpk_batch* b, const uint32_t* wirelens, uint64_t* out_offsets,
                              uint32_t* out_caplens, uint32_t* out_index, uint32_t* out_count, void* stream) {
  if (!f || !b || !out_offsets || !out_caplens || !out_index || !out_count) return GPK_EINVAL;
  if (b->n >= (1ull << 31)) return GPK_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (!b->n) return hipMemsetAsync(out_count, 0, 4, s) == hipSuccess ? GPK_OK : GPK_EHIP;
  if (b->n > f->cap) {  // scratch for this batch size
    for (void* p : {(void*)f->ret, (void*)f->flags, f->tmp})
      if (p) (void)hipFree(p);
    f->ret = nullptr;
    f->flags = nullptr;
    f->tmp = nullptr;
    size_t tb = 0;
    hipcub::CountingInputIterator<uint32_t> it(0);
    if (hipcub::DeviceSelect::Flagged(nullptr, tb, it, (uint8_t*)nullptr, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                      (int)b->n) != hipSuccess ||
        hipMalloc((void**)&f->ret, b->n * 4) != hipSuccess || hipMalloc((void**)&f->flags, b->n) != hipSuccess ||
        hipMalloc(&f->tmp, tb) != hipSuccess) {
      f->cap = 0;
      return GPK_ENOMEM;
    }
    f->tmp_bytes = tb;
    f->cap = b->n;
  }
  const uint64_t blocks = (b->n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(bpf_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, s, f->prog, f->len, b->data, b->offsets,
                     b->caplens, wirelens, b->n, f->ret, f->flags);
  size_t tb = f->tmp_bytes;
  hipcub::CountingInputIterator<uint32_t> it(0);
  if (hipcub::DeviceSelect::Flagged(f->tmp, tb, it, f->flags, out_index, out_count, (int)b->n, s) != hipSuccess)
    return GPK_EHIP;
  hipLaunchKernelGGL(gather_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, s, out_index, out_count, b->offsets,
                     b->caplens, out_offsets, out_caplens, b->n);
  return hipGetLastError() == hipSuccess ? GPK_OK : GPK_EHIP;
}

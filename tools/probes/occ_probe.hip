// Occupancy probe: how many 256-thread workgroups of a given dynamic LDS size
// are resident on one CU at once, and how long a CU's freed slot stays empty
// before the next workgroup starts there (dispatch gap). Every wave records its
// entry and exit time (s_memrealtime, 100 MHz) and HW_ID / XCC_ID, holds its
// slot for `hold_us`, and exits; the host sweeps the per-CU timelines.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/probes/bin/occ_probe tools/probes/occ_probe.hip
//   tools/probes/bin/occ_probe [hold_us] [lds_bytes ...]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

extern __shared__ uint32_t occ_smem[];

__global__ __launch_bounds__(256) void occ_kernel(uint64_t* rec, uint32_t hold_ticks, uint32_t slow_mult) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  // slow_mult > 1: blocks on XCD 0 hold their slots that many times longer (does a
  // full XCD hold back the dispatch of the other XCDs' blocks?)
  if (slow_mult > 1 && (__builtin_amdgcn_s_getreg((31 << 11) | 20) & 0xf) == 0) hold_ticks *= slow_mult;
  // touch the LDS so the allocation is real work, not just a reservation
  occ_smem[threadIdx.x] = threadIdx.x;
  uint64_t t = t0;
  while (t - t0 < hold_ticks) {  // every wave reaches the bound: the clock only moves forward
    __builtin_amdgcn_s_sleep(8);
    t = __builtin_amdgcn_s_memrealtime();
  }
  const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
  const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
  if ((threadIdx.x & 63) == 0) {
    const uint64_t w = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
    rec[3 * w + 0] = t0;
    rec[3 * w + 1] = __builtin_amdgcn_s_memrealtime() + occ_smem[(threadIdx.x + 1) & 255] * 0;
    rec[3 * w + 2] = (uint64_t)hw | (uint64_t)xcc << 32;
  }
}

int main(int argc, char** argv) {
  const double hold_us = argc > 1 ? atof(argv[1]) : 20.0;
  const char* sm = getenv("OCC_SLOW_XCD0");
  const uint32_t slow_mult = sm ? (uint32_t)atoi(sm) : 1u;
  std::vector<int> sizes;
  for (int k = 2; k < argc; k++) sizes.push_back(atoi(argv[k]));
  if (sizes.empty()) sizes = {16384, 20480, 22528, 24576, 25600, 26112, 26624, 27136, 27648, 28672, 32768};
  int dev = 0, ncu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  CK(hipFuncSetAttribute((const void*)occ_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  const int grid = ncu * 8 * 6;  // up to 8 per CU, six rounds
  uint64_t* rec;
  CK(hipMalloc(&rec, (size_t)grid * 4 * 3 * 8));
  std::vector<uint64_t> h((size_t)grid * 4 * 3);
  printf("{\"hold_us\": %.1f, \"cus\": %d, \"runs\": [\n", hold_us, ncu);
  for (size_t si = 0; si < sizes.size(); si++) {
    const int lds = sizes[si];
    int api = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&api, occ_kernel, 256, lds));
    for (int rep = 0; rep < 2; rep++) {  // first launch warms up; the second is recorded
      CK(hipMemset(rec, 0, (size_t)grid * 4 * 3 * 8));
      hipLaunchKernelGGL(occ_kernel, dim3(grid), dim3(256), lds, 0, rec, (uint32_t)(hold_us * 100.0), slow_mult);
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
    }
    CK(hipMemcpy(h.data(), rec, h.size() * 8, hipMemcpyDeviceToHost));
    // per CU: events (+1 at a block's first wave start, -1 at its last wave end)
    struct Blk { uint64_t s = ~0ull, e = 0; uint64_t cu = 0; };
    std::vector<Blk> blks(grid);
    uint64_t tmin = ~0ull, tmax = 0;
    for (int b = 0; b < grid; b++) {
      for (int w = 0; w < 4; w++) {
        const uint64_t* r = &h[3 * ((size_t)b * 4 + w)];
        blks[b].s = std::min(blks[b].s, r[0]);
        blks[b].e = std::max(blks[b].e, r[1]);
        const uint64_t hw = r[2] & 0xffffffffull, xcc = (r[2] >> 32) & 0xf;
        const uint64_t cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
        blks[b].cu = ((xcc * 8 + se) * 2 + sh) * 16 + cu;
      }
      tmin = std::min(tmin, blks[b].s);
      tmax = std::max(tmax, blks[b].e);
    }
    std::map<uint64_t, std::vector<std::pair<uint64_t, int>>> ev;
    for (auto& b : blks) {
      ev[b.cu].push_back({b.s, +1});
      ev[b.cu].push_back({b.e, -1});
    }
    int maxc_min = 1 << 30, maxc_max = 0;
    double gap_sum = 0;
    long gap_n = 0;
    std::map<int, int> hist;  // per-CU maximum -> CUs
    for (auto& kv : ev) {
      auto& v = kv.second;
      std::sort(v.begin(), v.end(), [](auto& a, auto& b) { return a.first != b.first ? a.first < b.first : a.second < b.second; });
      int c = 0, mx = 0;
      for (auto& x : v) {
        c += x.second;
        mx = std::max(mx, c);
      }
      hist[mx]++;
      maxc_min = std::min(maxc_min, mx);
      maxc_max = std::max(maxc_max, mx);
      // dispatch gap: for each block end, the next block start on this CU after it
      std::vector<uint64_t> st, en;
      for (auto& x : v) (x.second > 0 ? st : en).push_back(x.first);
      for (uint64_t e : en) {
        auto it = std::lower_bound(st.begin(), st.end(), e);
        if (it != st.end() && *it - e < 100000) {
          gap_sum += (double)(*it - e);
          gap_n++;
        }
      }
    }
    // mean resident blocks per CU over the middle 80 % of the span, per XCD
    double xres[8] = {0};
    int xcus[8] = {0};
    const uint64_t lo = tmin + (tmax - tmin) / 10, hi = tmax - (tmax - tmin) / 10;
    for (auto& kv : ev) {
      const int x = (int)(kv.first / 256) & 7;
      xcus[x]++;
      for (auto& b : blks)
        if (b.cu == kv.first) {
          const uint64_t s0 = std::max(b.s, lo), e0 = std::min(b.e, hi);
          if (e0 > s0) xres[x] += (double)(e0 - s0) / (double)(hi - lo);
        }
    }
    printf("  {\"xcd_mean_resident\": [");
    for (int x = 0; x < 8; x++) printf("%s%.2f", x ? ", " : "", xcus[x] ? xres[x] / xcus[x] : 0.0);
    printf("],\n");
    printf("   \"lds\": %d, \"api_blocks_per_cu\": %d, \"cus_seen\": %zu, \"max_resident_min\": %d, \"max_resident_max\": %d, "
           "\"hist\": {",
           lds, api, ev.size(), maxc_min, maxc_max);
    bool first = true;
    for (auto& kv : hist) {
      printf("%s\"%d\": %d", first ? "" : ", ", kv.first, kv.second);
      first = false;
    }
    printf("}, \"span_us\": %.1f, \"ideal_span_us\": %.1f, \"dispatch_gap_us\": %.3f}%s\n", (tmax - tmin) / 100.0,
           hold_us * ((grid + (double)ncu * api - 1) / ((double)ncu * api)), gap_n ? gap_sum / gap_n / 100.0 : -1.0,
           si + 1 < sizes.size() ? "," : "");
    fflush(stdout);
  }
  printf("]}\n");
  CK(hipFree(rec));
  return 0;
}

// Probe: how fast can the replay's pinned staging memory be obtained, and do
// the ways differ in HtoD rate? For K buffers of S MiB, each way allocates
// them (all K in parallel threads), then copies every buffer to the device.
//   pin_probe [K] [S_MiB] [touch_threads]
//   a: hipHostMalloc
//   b: mmap anonymous, touched by T threads, hipHostRegister
//   c: the same with madvise(MADV_HUGEPAGE) before the touch
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static void touch(char* p, size_t len, int threads) {
  std::vector<std::thread> th;
  const size_t per = (len / threads + 4095) & ~(size_t)4095;
  for (int t = 0; t < threads; t++)
    th.emplace_back([=] {
      const size_t a = (size_t)t * per, b = a + per < len ? a + per : len;
      for (size_t o = a; o < b; o += 4096) p[o] = 0;
    });
  for (auto& x : th) x.join();
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 4;
  const size_t S = (size_t)(argc > 2 ? atol(argv[2]) : 512) << 20;
  const int T = argc > 3 ? atoi(argv[3]) : 4;
  void* d = nullptr;
  if (hipMalloc(&d, S) != hipSuccess) return 3;
  hipStream_t st;
  (void)hipStreamCreate(&st);
  for (int way = 0; way < 3; way++) {
    std::vector<char*> bufs(K, nullptr);
    const double t0 = now();
    std::vector<std::thread> th;
    for (int k = 0; k < K; k++)
      th.emplace_back([&, k] {
        (void)hipSetDevice(0);
        if (way == 0) {
          if (hipHostMalloc((void**)&bufs[k], S, hipHostMallocDefault) != hipSuccess) bufs[k] = nullptr;
          return;
        }
        void* p = mmap(nullptr, S, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p == MAP_FAILED) return;
        if (way == 2) (void)madvise(p, S, MADV_HUGEPAGE);
        touch((char*)p, S, T);
        if (hipHostRegister(p, S, hipHostRegisterDefault) != hipSuccess) {
          munmap(p, S);
          return;
        }
        bufs[k] = (char*)p;
      });
    for (auto& x : th) x.join();
    const double t1 = now();
    int ok = 0;
    for (char* b : bufs) ok += b != nullptr;
    double best = 1e9;
    for (int r = 0; r < 3; r++)
      for (char* b : bufs) {
        if (!b) continue;
        const double a = now();
        (void)hipMemcpyAsync(d, b, S, hipMemcpyHostToDevice, st);
        (void)hipStreamSynchronize(st);
        const double e = now() - a;
        if (e < best) best = e;
      }
    const double t2 = now();
    for (char* b : bufs) {
      if (!b) continue;
      if (way == 0) (void)hipHostFree(b);
      else {
        (void)hipHostUnregister(b);
        munmap(b, S);
      }
    }
    const double t3 = now();
    printf("way %c: %d x %zu MiB: allocate %.4f s (%.1f GB/s), best HtoD %.1f GB/s, free %.4f s\n", "abc"[way], ok,
           S >> 20, t1 - t0, (double)S * ok / (t1 - t0) / 1e9, (double)S / best / 1e9, t3 - t2);
    fflush(stdout);
  }
  return 0;
}

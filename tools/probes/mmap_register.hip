// Probe: can a read-only mmap of a (page-cached) capture file be registered
// with hipHostRegister and copied to the device without a host-side copy?
//   mmap_register FILE [MiB]
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const int fd = open(argv[1], O_RDONLY);
  if (fd < 0) { perror("open"); return 2; }
  struct stat sb;
  fstat(fd, &sb);
  size_t len = (size_t)sb.st_size;
  if (argc > 2) { size_t m = (size_t)atol(argv[2]) << 20; if (m < len) len = m; }
  len &= ~(size_t)4095;
  void* p = mmap(nullptr, len, PROT_READ, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) { perror("mmap"); return 2; }
  const size_t chunk = 256u << 20;
  void* d = nullptr;
  if (hipMalloc(&d, chunk) != hipSuccess) return 3;
  std::vector<unsigned char> back(4096);
  double treg = 0, tcp = 0, tun = 0;
  int bad = 0;
  for (size_t off = 0; off + chunk <= len; off += chunk) {
    char* q = (char*)p + off;
    double t0 = now();
    hipError_t e = hipHostRegister(q, chunk, hipHostRegisterReadOnly);
    if (e != hipSuccess) e = hipHostRegister(q, chunk, hipHostRegisterDefault);
    double t1 = now();
    if (e != hipSuccess) { printf("hipHostRegister failed at %zu: %s\n", off, hipGetErrorString(e)); return 4; }
    e = hipMemcpy(d, q, chunk, hipMemcpyHostToDevice);
    double t2 = now();
    if (e != hipSuccess) { printf("hipMemcpy failed: %s\n", hipGetErrorString(e)); return 5; }
    (void)hipMemcpy(back.data(), (char*)d + chunk - 4096, 4096, hipMemcpyDeviceToHost);
    if (memcmp(back.data(), q + chunk - 4096, 4096)) bad++;
    (void)hipHostUnregister(q);
    double t3 = now();
    treg += t1 - t0; tcp += t2 - t1; tun += t3 - t2;
  }
  const double gb = (double)(len / chunk * chunk) / 1e9;
  printf("%.2f GB: register %.3f s, HtoD %.3f s (%.1f GB/s), unregister %.3f s, mismatches %d\n", gb, treg, tcp, gb / tcp, tun, bad);
  return bad ? 6 : 0;
}

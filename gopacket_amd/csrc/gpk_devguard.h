// gpk_devguard.h — the caller's current HIP device, handed back on every
// return (library-internal).
//
// Every entry point that works on a context's (or a grouper's) device makes it
// current for the duration of the call and restores the caller's device on
// every return path, early errors included. A cgo caller runs goroutines on
// arbitrary OS threads and may multiplex contexts of several devices on one of
// them, or use HIP itself: after any gpk_* call its thread's device is the one
// it had before. The reference path has no such side effect either:
// DecodeLayers mutates only its own parser (parser.go:303-317).
#ifndef GPK_DEVGUARD_H
#define GPK_DEVGUARD_H

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gpk {

struct DeviceScope {
  int prev = -1;          // the caller's device (-1: unknown, never restored)
  bool switched = false;  // this scope changed it
  hipError_t err = hipSuccess;
  explicit DeviceScope(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) {
      err = hipSetDevice(dev);
      switched = err == hipSuccess;
    }
  }
  ~DeviceScope() {
    if (switched && prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceScope(const DeviceScope&) = delete;
  DeviceScope& operator=(const DeviceScope&) = delete;
};

}  // namespace gpk

// The device of a context (gpk_host.cpp), for the library's own pipelines.
struct gpk_ctx;
extern "C" __attribute__((visibility("hidden"))) int gpk_ctx_device(const gpk_ctx* c);
// How many times gpk_stop was called on the context: a replay or pump takes it
// when it starts and ends early once it has changed.
extern "C" __attribute__((visibility("hidden"))) uint64_t gpk_ctx_stop_seq(const gpk_ctx* c);

#endif  // GPK_DEVGUARD_H

// gpk_pinned.h — pinned host memory for the staging buffers (library-internal).
//
// hipHostMalloc hands out pinned pages at ~5 GB/s on the GPU box (the
// kernel faults, zeroes and locks 4 KiB pages one by one): the replay's first
// call spent 0.38 s obtaining its 2 GiB of staging slots. Anonymous memory
// aligned to 2 MiB with madvise(MADV_HUGEPAGE), touched once and then
// registered with hipHostRegister, comes at ~120-140 GB/s and copies to the
// device at the same rate (tools/probes/pin_probe.hip, profiles/r15_pin_probe.txt:
// 57.6 GB/s HtoD either way). Small buffers, and any failure of that path, use
// hipHostMalloc.
#ifndef GPK_PINNED_H
#define GPK_PINNED_H

#include <hip/hip_runtime.h>

#include <cstddef>

extern "C" {
__attribute__((visibility("hidden"))) hipError_t gpk_pin_alloc(void** out, size_t bytes);
__attribute__((visibility("hidden"))) hipError_t gpk_pin_free(void* p);
}

#endif  // GPK_PINNED_H

#!/usr/bin/env python3
"""Do host->device and device->host copies overlap on this box? Pinned
buffers, 256 MiB copies: HtoD alone, DtoH alone, and both at once on two
streams (and both directions on one stream), GB/s per direction."""
import time

import torch


def main(mib=256, reps=8):
    n = mib << 20
    h_in = torch.empty(n * 2, dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty(n * 2, dtype=torch.uint8, pin_memory=True)
    d_in = torch.empty(n * 2, dtype=torch.uint8, device="cuda")
    d_out = torch.empty(n * 2, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def run(h2d, d2h, same=False):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(reps):
            o = (k & 1) * n
            if h2d:
                with torch.cuda.stream(s1):
                    d_in[o:o + n].copy_(h_in[o:o + n], non_blocking=True)
            if d2h:
                with torch.cuda.stream(s1 if same else s2):
                    h_out[o:o + n].copy_(d_out[o:o + n], non_blocking=True)
        torch.cuda.synchronize()
        return n * reps / (time.perf_counter() - t0) / 1e9

    run(True, True)
    for name, a, b, same in (("HtoD alone", True, False, False), ("DtoH alone", False, True, False),
                             ("both, two streams", True, True, False), ("both, one stream", True, True, True)):
        print("%-20s %6.1f GB/s per direction" % (name, run(a, b, same)), flush=True)
    # the device->host direction as kernel stores into pinned memory instead of a copy
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from gopacket_amd import _lib
    S = _lib.synth_lib()

    def run_w(h2d, blocks):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(reps):
            o = (k & 1) * n
            if h2d:
                with torch.cuda.stream(s1):
                    d_in[o:o + n].copy_(h_in[o:o + n], non_blocking=True)
            assert S.gpk_probe_hostwrite(h_out.data_ptr() + o, n, blocks, s2.cuda_stream) == 0
        torch.cuda.synchronize()
        return n * reps / (time.perf_counter() - t0) / 1e9

    for blocks in (64, 256, 1024):
        run_w(False, blocks)
        print("kernel stores to host, %4d blocks: alone %6.1f GB/s, with HtoD copies %6.1f GB/s per direction"
              % (blocks, run_w(False, blocks), run_w(True, blocks)), flush=True)


def ring_memory(mib=256):
    """HtoD rate from host memory of the kinds the pump copies from: a pinned
    allocation, and ordinary (numpy) memory registered with hipHostRegister as
    the pump registers a ring, in 4 MiB (a V3 block) and 64 MiB copies."""
    import ctypes
    import os
    import sys
    import numpy as np
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from gopacket_amd import _lib
    S = _lib.synth_lib()
    n = mib << 20
    pinned = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    plain = np.ones(n, np.uint8)
    for chunk in (4 << 20, 64 << 20):
        for streams in (1, 4):
            a = S.gpk_probe_h2d_rate(ctypes.c_void_p(pinned.data_ptr()), n, chunk, streams, 4, 0)
            b = S.gpk_probe_h2d_rate(ctypes.c_void_p(plain.ctypes.data), n, chunk, streams, 4, 1)
            print("HtoD %3d MiB copies on %d stream(s): pinned %5.1f GB/s, registered numpy memory %5.1f GB/s"
                  % (chunk >> 20, streams, a, b), flush=True)


if __name__ == "__main__":
    import sys as _sys
    if len(_sys.argv) > 1 and _sys.argv[1] == "ring":
        ring_memory()
        raise SystemExit(0)
    main()

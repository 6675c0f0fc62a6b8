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


if __name__ == "__main__":
    main()

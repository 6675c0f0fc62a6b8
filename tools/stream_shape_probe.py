#!/usr/bin/env python3
"""Does the shape of the decode's stream make its rate depend on where its
batch lies in HBM? (the C3 spread between boxes and
allocations.) Over several allocations of a C3-sized buffer (each placed
behind a spacer of a different size, so its physical pages differ), time:
  read   gpk_probe_read: one grid-wide sweep (the streaming probe)
  wave   gpk_probe_reread mode 0: each wave streams its own 64 x 1500 B region
         in 1 KiB passes, 8 in flight (the decode kernel's phase-B shape)
  block  gpk_probe_reread mode 4: the same bytes, the block's 4 waves streaming
         its 256-packet region together in 4 KiB passes
Interleaved rounds, HIP events, medians; one JSON line per allocation.

    python tools/stream_shape_probe.py [--gib 96] [--allocs 3]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=96.0)
    ap.add_argument("--allocs", type=int, default=3)
    ap.add_argument("--spacer-gib", type=float, default=7.0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--pkt", type=int, default=1500)
    ap.add_argument("--occ", default="", help="blocks per CU to sweep for the wave shape, e.g. 8,6,4,3,2 (one allocation)")
    a = ap.parse_args()
    import torch
    from gopacket_amd import _lib
    S = _lib.synth_lib()
    stream = torch.cuda.current_stream()
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    nbytes = int(a.gib * 2**30) & ~4095
    used = nbytes // (256 * a.pkt) * (256 * a.pkt)
    if a.occ:
        buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        buf[::4096] = 1
        for bpc in [int(x) for x in a.occ.split(",")]:
            lds = (160 * 1024) // bpc // 512 * 512 - 512 if bpc > 1 else 96 * 1024
            t = []
            for rnd in range(a.rounds + 1):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(a.steps):
                    assert S.gpk_probe_reread_lds(buf.data_ptr(), used, a.pkt, 0, lds, sink.data_ptr(),
                                                  stream.cuda_stream) == 0
                e1.record(stream)
                torch.cuda.synchronize()
                if rnd:
                    t.append(e0.elapsed_time(e1) / a.steps)
            ms = float(np.median(t))
            print(json.dumps({"blocks_per_cu": bpc, "lds": lds, "wave_ms": round(ms, 4),
                              "wave_GBps": round(used / (ms * 1e-3) / 1e9, 1)}), flush=True)
        return
    for k in range(a.allocs):
        spacer = torch.empty(max(1, int(k * a.spacer_gib * 2**30)), dtype=torch.uint8, device="cuda")
        buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        buf[::4096] = 1  # touch every page once (content does not matter for timing)

        def run(which):
            if which == "read":
                assert S.gpk_probe_read(buf.data_ptr(), used, sink.data_ptr(), 256 * 8, stream.cuda_stream) == 0
            else:
                m = 0 if which == "wave" else 4
                assert S.gpk_probe_reread(buf.data_ptr(), used, a.pkt, m, sink.data_ptr(), stream.cuda_stream) == 0

        times = {w: [] for w in ("read", "wave", "block")}
        for rnd in range(a.rounds + 1):
            for w in times:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(a.steps):
                    run(w)
                e1.record(stream)
                torch.cuda.synchronize()
                if rnd:
                    times[w].append(e0.elapsed_time(e1) / a.steps)
        row = {"alloc": k, "addr": hex(buf.data_ptr()), "bytes": used}
        for w, t in times.items():
            ms = float(np.median(t))
            row[w + "_ms"] = round(ms, 4)
            row[w + "_GBps"] = round(used / (ms * 1e-3) / 1e9, 1)
        print(json.dumps(row), flush=True)
        del buf, spacer
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

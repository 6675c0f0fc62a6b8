#!/usr/bin/env python3
"""Does the placement of the decode's OUTPUT buffers explain the per-allocation
spread of C3? One batch allocation, several sets of output buffers (records,
error arguments, flows; torch allocations made one after another, plus one
hipDeviceMallocContiguous set), the decode timed with each in interleaved
rounds; also the memory skeleton with each set's record buffer as its write
target."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(sets=4, rounds=3, steps=5):
    import torch
    import bench
    from gopacket_amd import _lib, engine, synth
    from alloc_probe import Raw
    S = _lib.synth_lib()
    ctx = engine.Context(0)
    stream = torch.cuda.current_stream()
    cfg = bench.CONFIGS["c3"]
    n = 64 * 2**20
    parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in cfg["decoders"]], outputs=cfg["outputs"])
    d, o, c = synth.device_batch(3, 0, n, stream=stream)
    outs = []
    for k in range(sets):
        outs.append(("torch%d" % k, torch.empty(n * 16, dtype=torch.uint8, device="cuda"),
                     torch.zeros(2 * n, dtype=torch.int32, device="cuda"),
                     torch.empty(3 * n, dtype=torch.int64, device="cuda")))
    zero = torch.zeros(8 * n, dtype=torch.uint8, device="cuda")
    ce = Raw(S, 8 * n, 4, 4)
    assert S.gpk_probe_d2d(ce.data_ptr(), zero.data_ptr(), 8 * n) == 0
    outs.append(("contig", Raw(S, 16 * n, 4), ce, Raw(S, 24 * n, 4, 8)))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = {x[0]: [] for x in outs}
    for rnd in range(rounds + 1):
        for name, rec, err, fl in outs:
            e0.record(stream)
            for _ in range(steps):
                ctx.decode_device(parser, d, o, c, rec, err, fl, stream=stream)
            e1.record(stream)
            torch.cuda.synchronize()
            if rnd:
                times[name].append(e0.elapsed_time(e1) / steps)
    for name, rec, err, fl in outs:
        print("outputs %-7s at %#x: decode median %.3f ms" % (name, rec.data_ptr(), float(np.median(times[name]))),
              flush=True)


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    main()

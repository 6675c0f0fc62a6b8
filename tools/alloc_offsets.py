#!/usr/bin/env python3
"""C3 with one batch allocation and one output arena: the records, error
arguments and flows placed at shifting offsets inside the arena (0, 1, 2, 4,
8, 16, 32, 64, 128 MiB), decode timed per offset in interleaved rounds. A
periodic or offset-dependent time points at the physical relation between
the stream being read and the outputs being written back."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(rounds=3, steps=5):
    import torch
    import bench
    from gopacket_amd import engine, synth
    ctx = engine.Context(0)
    stream = torch.cuda.current_stream()
    cfg = bench.CONFIGS["c3"]
    n = 64 * 2**20
    parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in cfg["decoders"]], outputs=cfg["outputs"])
    d, o, c = synth.device_batch(3, 0, n, stream=stream)
    MiB = 1 << 20
    offs = [0, 1, 2, 4, 8, 16, 32, 64, 128]
    slack = max(offs) * MiB
    rec_a = torch.empty(16 * n + slack, dtype=torch.uint8, device="cuda")
    err_a = torch.zeros(8 * n + slack, dtype=torch.uint8, device="cuda")
    fl_a = torch.empty(24 * n + slack, dtype=torch.uint8, device="cuda")
    sets = []
    for k in offs:
        b = k * MiB
        sets.append((k, rec_a[b:b + 16 * n], err_a[b:b + 8 * n].view(torch.int32), fl_a[b:b + 24 * n].view(torch.int64)))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = {k: [] for k in offs}
    for rnd in range(rounds + 1):
        for k, rec, err, fl in sets:
            e0.record(stream)
            for _ in range(steps):
                ctx.decode_device(parser, d, o, c, rec, err, fl, stream=stream)
            e1.record(stream)
            torch.cuda.synchronize()
            if rnd:
                times[k].append(e0.elapsed_time(e1) / steps)
    print("data at %#x, outputs arena at %#x: " % (d.data_ptr(), rec_a.data_ptr()) +
          "  ".join("+%dMiB %.3f" % (k, float(np.median(times[k]))) for k in offs), flush=True)


if __name__ == "__main__":
    main()

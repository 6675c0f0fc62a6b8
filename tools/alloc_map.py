#!/usr/bin/env python3
"""Where is a slow C3 allocation slow? One 96 GiB batch allocation (torch),
the decode timed over the whole batch, then the streaming-read probe
(gpk_probe_read) timed over each 1 GiB chunk of it and over the whole buffer:
a uniformly slower allocation points at the address translation of the whole
range, a few slow chunks at the physical memory behind them."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import bench
    from gopacket_amd import _lib, engine, synth
    S = _lib.synth_lib()
    ctx = engine.Context(0)
    stream = torch.cuda.current_stream()
    cfg = bench.CONFIGS["c3"]
    n = 64 * 2**20
    parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in cfg["decoders"]], outputs=cfg["outputs"])
    d, o, c = synth.device_batch(3, 0, n, stream=stream)
    rec = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    err = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
    fl = torch.empty(3 * n, dtype=torch.int64, device="cuda")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(fn, reps):
        fn()
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    dec = timed(lambda: ctx.decode_device(parser, d, o, c, rec, err, fl, stream=stream), 5)
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    total = d.numel() - 256
    whole = timed(lambda: S.gpk_probe_read(d.data_ptr(), total, sink.data_ptr(), 2048, stream.cuda_stream), 5)
    G = 1 << 30
    rates = []
    for k in range(total // G):
        p = d.data_ptr() + k * G
        ms = timed(lambda: S.gpk_probe_read(p, G, sink.data_ptr(), 2048, stream.cuda_stream), 5)
        rates.append(G / (ms * 1e-3) / 1e9)
    r = np.array(rates)
    print("allocation at %#x: decode %.3f ms (%.1f%% of 8 TB/s); probe over the whole %.0f GiB %.0f GB/s; "
          "per 1 GiB chunk: min %.0f  p10 %.0f  median %.0f  p90 %.0f  max %.0f GB/s" % (
              d.data_ptr(), dec, (total + 12 * n) / (dec * 1e-3) / 8e12 * 100, total / G,
              total / (whole * 1e-3) / 1e9, r.min(), np.percentile(r, 10), np.median(r), np.percentile(r, 90),
              r.max()), flush=True)
    print("chunk GB/s:", " ".join("%.0f" % x for x in r), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Is a slow C3 allocation slow for one stride only? One 96 GiB allocation
(torch), C3 generated into it and decoded, then the decode's stream shape
without its work (gpk_probe_reread mode 0: each wave streams its own 64 x P
byte region in 1 KiB passes) at several region strides P over the same bytes.
Run in several fresh processes to catch both the fast and the slow mode."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
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
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(fn, reps=5):
        fn()
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    total = d.numel() - 256
    out = ["decode %.3f ms" % timed(lambda: ctx.decode_device(parser, d, o, c, rec, err, fl, stream=stream))]
    for P in (1500, 1499, 1504, 1472, 1536, 1024, 4096):
        used = total // (256 * P) * (256 * P)
        ms = timed(lambda: S.gpk_probe_reread(d.data_ptr(), used, P, 0, sink.data_ptr(), stream.cuda_stream))
        out.append("P=%d %.0f GB/s" % (P, used / (ms * 1e-3) / 1e9))
    print("  ".join(out), flush=True)


if __name__ == "__main__":
    main()

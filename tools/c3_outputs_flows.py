#!/usr/bin/env python3
"""Is C3's output-side slow mode the flows? One C3 batch allocation, SETS
output sets (records, error arguments, flows; torch allocations one after
another), in interleaved rounds: the decode with every output (C3's parser),
and the same decode without the flow hashes (records only) into the same
record buffers. If the slow sets are slow only with the flows, the three flow
sub-arrays (written in lockstep n*8 bytes apart) are where it is."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(sets=8, rounds=3, steps=5):
    import torch
    import bench
    from gopacket_amd import engine, synth
    ctx = engine.Context(0)
    stream = torch.cuda.current_stream()
    cfg = bench.CONFIGS["c3"]
    n = 64 * 2**20
    kinds = [engine.DECODER_KINDS[d] for d in cfg["decoders"]]
    full = engine.ParserConfig(17, kinds, outputs=cfg["outputs"])
    noflows = engine.ParserConfig(17, kinds, outputs=cfg["outputs"] & ~4)
    d, o, c = synth.device_batch(3, 0, n, stream=stream)
    outs = [(torch.empty(n * 16, dtype=torch.uint8, device="cuda"), torch.zeros(2 * n, dtype=torch.int32, device="cuda"),
             torch.empty(3 * n, dtype=torch.int64, device="cuda")) for _ in range(sets)]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t = {(k, v): [] for k in range(sets) for v in ("full", "noflows")}
    for rnd in range(rounds + 1):
        for k, (rec, err, fl) in enumerate(outs):
            for v, p, f in (("full", full, fl), ("noflows", noflows, None)):
                e0.record(stream)
                for _ in range(steps):
                    ctx.decode_device(p, d, o, c, rec, err, f, stream=stream)
                e1.record(stream)
                torch.cuda.synchronize()
                if rnd:
                    t[(k, v)].append(e0.elapsed_time(e1) / steps)
        print("round %d done" % rnd, flush=True)
    for k, (rec, err, fl) in enumerate(outs):
        print("set %d rec %#x fl %#x: full %.3f ms  noflows %.3f ms" % (
            k, rec.data_ptr(), fl.data_ptr(), float(np.median(t[(k, "full")])), float(np.median(t[(k, "noflows")]))),
            flush=True)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))

#!/usr/bin/env python3
"""Upper bound of a narrower per-packet record before
building it: on the C2 and C4 batches in HBM, the decode next to its memory
skeleton (gpk_probe_skeleton_idx: index, header windows, the wave's stream,
the per-packet writes; none of the work) with the writes the decode makes now
(C2: the 16-byte record; C4: the record and three flow hashes, 40 B) and with
the 8-byte narrow record in their place (8 / 32 B). Interleaved rounds, HIP
events, medians. One JSON line.

    python tools/narrow_probe.py [--packets 67108864]
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
    ap.add_argument("--packets", type=int, default=64 * 2**20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--configs", default="c2,c4")
    a = ap.parse_args()
    import torch
    import bench
    from gopacket_amd import _lib, engine, synth
    S = _lib.synth_lib()
    stream = torch.cuda.current_stream()
    ctx = engine.Context()
    out = {}
    for name in a.configs.split(","):
        cfg = bench.CONFIGS[name]
        n = a.packets
        data, off, cap = synth.device_batch(cfg["synth"], 0, n, stream=stream)
        parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in cfg["decoders"]], outputs=cfg["outputs"])
        rec = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
        err = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
        fl = torch.empty(3 * n, dtype=torch.int64, device="cuda") if cfg["outputs"] & 4 else None
        wide, streamed = bench.skeleton_shape(cfg)
        narrow = wide - 8
        wbuf = torch.empty(wide * n, dtype=torch.uint8, device="cuda")
        sink = torch.zeros(1, dtype=torch.int32, device="cuda")

        def skel(wb):
            return lambda: S.gpk_probe_skeleton_idx(data.data_ptr(), off.data_ptr(), cap.data_ptr(), n,
                                                    wbuf.data_ptr(), wbuf.numel(), wb,
                                                    2 | (0 if streamed else 64), sink.data_ptr(), stream.cuda_stream)

        runs = {"decode": lambda: ctx.decode_device(parser, data, off, cap, rec, err, fl, stream=stream),
                "skeleton_w%d" % wide: skel(wide), "skeleton_w%d" % narrow: skel(narrow),
                "skeleton_w0": skel(0)}
        times = {k: [] for k in runs}
        for _ in range(a.rounds):
            for k, f in runs.items():
                f()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(a.steps):
                    assert f() in (0, None)
                e1.record(stream)
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1) / a.steps)
        med = {k: round(float(np.median(v)), 4) for k, v in times.items()}
        med["narrow_over_wide_skeleton"] = round(med["skeleton_w%d" % narrow] / med["skeleton_w%d" % wide], 4)
        out[name] = med
        del data, off, cap, rec, err, fl, wbuf
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()

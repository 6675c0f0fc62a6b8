#!/usr/bin/env python3
"""C3's decode against its memory skeleton: on the C3 batch
itself (64 M x 1500 B in HBM), gpk_probe_skeleton makes the decode kernel's
memory accesses per wave without its work, adding them one at a time:
  stream            each wave streams its 64 packets (1 KiB passes, 8 in flight)
  +windows          first each lane's 6-chunk header window into LDS (temporal)
  +index            before that the lane's index entry, the windows waiting for it
  +writes           after the stream the record and three flow hashes (40 B/packet,
                    non-temporal); the same with the default store policy, and
                    with the block's waves storing together after a barrier
  stream+writes     the stream and the writes alone
and times the decode (gpk_decode_batch, C3's parser and outputs) beside them,
interleaved rounds, HIP events, medians. One JSON line.

    python tools/skeleton_probe.py [--packets 67108864]
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
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    import torch
    import bench
    from gopacket_amd import _lib, engine, synth
    S = _lib.synth_lib()
    stream = torch.cuda.current_stream()
    n = a.packets
    cfg = bench.CONFIGS["c3"]
    data, off, cap = synth.device_batch(cfg["synth"], 0, n, stream=stream)
    pkt = 1500
    assert int(cap.min().item()) == pkt and int(cap.max().item()) == pkt
    nbytes = n * pkt
    idx = torch.empty(3 * n, dtype=torch.int32, device="cuda")
    idx[:2 * n] = off.view(torch.int32)
    idx[2 * n:] = cap.view(torch.int32)
    wbuf = torch.empty(40 * n, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    ctx = engine.Context()
    parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in cfg["decoders"]], outputs=cfg["outputs"])
    rec = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    err = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
    fl = torch.empty(3 * n, dtype=torch.int64, device="cuda")

    def skeleton(flags):
        return lambda: S.gpk_probe_skeleton(data.data_ptr(), nbytes, pkt, idx.data_ptr(), wbuf.data_ptr(), flags,
                                            sink.data_ptr(), stream.cuda_stream)

    def decode():
        ctx.decode_device(parser, data, off, cap, rec, err, fl, stream=stream)
        return 0

    runs = {"stream": skeleton(0), "+windows": skeleton(2), "+index": skeleton(3), "+writes": skeleton(7),
            "+writes temporal": skeleton(15), "+writes per block": skeleton(23), "stream+writes": skeleton(4),
            "decode": decode}
    times = {k: [] for k in runs}
    for rnd in range(a.rounds + 1):
        for k, f in runs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.steps):
                assert f() == 0
            e1.record(stream)
            torch.cuda.synchronize()
            if rnd:
                times[k].append(e0.elapsed_time(e1) / a.steps)
    algo = nbytes + 12 * n
    row = {"packets": n, "algorithmic_bytes": algo}
    for k, t in times.items():
        ms = float(np.median(t))
        row[k + "_ms"] = round(ms, 4)
        row[k + "_GBps"] = round(algo / (ms * 1e-3) / 1e9, 1)
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()

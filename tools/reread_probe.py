#!/usr/bin/env python3
"""Does a header-window line that phase B reads again cost DRAM bandwidth?
 gpk_probe_reread over a buffer far
larger than the 256 MiB Infinity Cache, with C3's geometry (64 packets of
1500 B per wave) and C4's mean (362 B):
  mode 0  the regions streamed once
  mode 1  each packet's 6-chunk header window first (temporal), then the stream
  mode 2  the header windows alone
Each mode is timed in interleaved rounds (HIP events, median). The bytes mode 1
reads twice are the window lines: if their second fetch went to DRAM, mode 1
would take mode 0 x (1 + re-fetched share); if it is served on chip, mode 1
takes about mode 0. PMC passes of the same command (tools/reread_pmc.sh) give
FETCH_SIZE and the L2->fabric read requests per mode.

    python tools/reread_probe.py [--gib 32] [--json out.json]
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
    ap.add_argument("--gib", type=float, default=32.0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--pkts", default="1500,362")
    ap.add_argument("--modes", default="0,1,2,3")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    import torch
    from gopacket_amd import _lib
    S = _lib.synth_lib()
    nbytes = int(a.gib * 2**30) & ~4095
    buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    buf.random_(0, 256)
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()
    out = {}
    for pkt in [int(x) for x in a.pkts.split(",")]:
        modes = [int(m) for m in a.modes.split(",")]
        times = {m: [] for m in modes}
        for rnd in range(a.rounds + 1):
            for m in modes:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(a.steps):
                    assert S.gpk_probe_reread(buf.data_ptr(), nbytes, pkt, m, sink.data_ptr(), stream.cuda_stream) == 0
                e1.record(stream)
                torch.cuda.synchronize()
                if rnd:
                    times[m].append(e0.elapsed_time(e1) / a.steps)
        region = 64 * pkt
        used = nbytes // region * region
        # distinct 128-B lines of the header windows (6 chunks from the 16-B-aligned packet start)
        starts = (np.arange(64, dtype=np.int64) * pkt) & ~15
        lines = len(set(int(x) for s0 in starts for x in range(s0 // 128, (s0 + 95) // 128 + 1)))
        win_share = lines * 128 / region
        row = {"pkt": pkt, "bytes": used, "window_line_share": round(win_share, 4)}
        for m in modes:
            t = float(np.median(times[m]))
            row["mode%d_ms" % m] = round(t, 4)
            row["mode%d_GBps" % m] = round(used / (t * 1e-3) / 1e9, 1)
        if 0 in modes and 1 in modes:
            row["mode1_over_mode0"] = round(row["mode1_ms"] / row["mode0_ms"], 4)
            row["if_dram_mode1_over_mode0"] = round(1 + win_share, 4)
        print(json.dumps(row), flush=True)
        out[str(pkt)] = row
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

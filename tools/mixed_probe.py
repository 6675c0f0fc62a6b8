#!/usr/bin/env python3
"""Achievable HBM rate for a decode's read + write mix ("what
bounds"): gpk_probe_mixed streams a config's packet buffer (non-temporal
16-byte loads, as gpk_probe_read) while other blocks of the same launch store
as many bytes as the decode writes per packet (records 16 B, flows 24 B,
fields 128 B). The best split of blocks between the two sides over a small
sweep is the box's ceiling for that mix; compare the decode's bytes moved
(PMC fetch + write, profiles/hbm_traffic.json) over its kernel time with it.

    python tools/mixed_probe.py [--configs c1,c2,c4,c4f,c3] [--steps 10]

Prints one JSON line per config.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# bytes a decode writes per packet for each config (records 16, flows 24 with
# the hash output, fields 128 for the fused launch)
WRITES = {"c1": 16, "c2": 16, "c3": 40, "c4": 40, "c4f": 168}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c1,c2,c4,c4f,c3")
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    import torch
    import bench
    from gopacket_amd import _lib, synth
    S = _lib.synth_lib()
    stream = torch.cuda.current_stream()
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    blocks = 256 * 8
    for name in a.configs.split(","):
        cfg = bench.CONFIGS[name.rstrip("f")]
        n = cfg.get("packets", 64 * 2**20)
        if "pcap" in cfg:
            data, off, cap = bench.pcap_tiled(cfg["pcap"], n)
        else:
            data, off, cap = synth.device_batch(cfg["synth"], 0, n, stream=stream)
        rbytes = int(cap.sum(dtype=torch.int64).item()) & ~15
        wbytes = (WRITES[name] * n) & ~15
        wbuf = torch.empty(wbytes, dtype=torch.uint8, device="cuda")

        def timed(writers):
            def go():
                if writers == 0:
                    assert S.gpk_probe_read(data.data_ptr(), rbytes, sink.data_ptr(), blocks, stream.cuda_stream) == 0
                else:
                    assert S.gpk_probe_mixed(data.data_ptr(), rbytes, wbuf.data_ptr(), wbytes, blocks, writers,
                                             sink.data_ptr(), stream.cuda_stream) == 0
            go()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.steps):
                go()
            e1.record(stream)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / a.steps

        read_ms = timed(0)
        prop = max(1, round(blocks * wbytes / (rbytes + wbytes)))
        sweep = {}
        for w in sorted({max(1, prop // 2), prop, prop * 3 // 2, prop * 2, prop * 3}):
            if w < blocks:
                sweep[w] = timed(w)
        best_w = min(sweep, key=sweep.get)
        ms = sweep[best_w]
        print(json.dumps({
            "config": name, "packets": n, "read_bytes": rbytes, "written_bytes": wbytes,
            "read_only_ms": round(read_ms, 4), "read_only_GBps": round(rbytes / read_ms / 1e6, 1),
            "mixed_ms": round(ms, 4), "mixed_GBps": round((rbytes + wbytes) / ms / 1e6, 1),
            "writer_blocks": best_w, "sweep_ms": {str(k): round(v, 4) for k, v in sweep.items()},
        }), flush=True)
        del data, off, cap, wbuf
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Rate of gpk_extract_fields (layer fields from a decode's layouts) on a
full-size synthetic batch in HBM: the decode with layouts, then the field
extraction, each timed with HIP events on the launch stream.

    python tools/fields_rate.py [--configs c4,c3] [--packets N] [--steps 5]

Bytes per packet counted for the field kernel: its 64-byte layout, the 8-byte
offset and the 128-byte record it writes (the header bytes it reads were
just read by the decode and are reported apart, not counted).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c4,c3")
    ap.add_argument("--packets", type=int, default=64 * 2**20)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    import torch
    import bench
    from gopacket_amd import engine, synth
    ctx = engine.Context(0)
    stream = torch.cuda.current_stream()
    out = {}
    for name in a.configs.split(","):
        cfg = bench.CONFIGS[name]
        n = a.packets
        data, off, cap = synth.device_batch(cfg["synth"], 0, n, stream=stream)
        parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in cfg["decoders"]], outputs=cfg["outputs"])
        rec = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
        err = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
        fl = torch.empty(3 * n, dtype=torch.int64, device="cuda")
        lay = torch.empty(n * 64, dtype=torch.uint8, device="cuda")
        fields = torch.empty(n * 128, dtype=torch.uint8, device="cuda")
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        dec_ms, fld_ms = [], []
        for k in range(a.steps + 2):
            ev[0].record(stream)
            ctx.decode_device(parser, data, off, cap, rec, err, fl, lay, stream=stream)
            ev[1].record(stream)
            ctx.extract_fields(data, off, cap, lay, fields, stream=stream)
            ev[2].record(stream)
            torch.cuda.synchronize()
            if k >= 2:
                dec_ms.append(ev[0].elapsed_time(ev[1]))
                fld_ms.append(ev[1].elapsed_time(ev[2]))
        f = sorted(fld_ms)[len(fld_ms) // 2]
        d = sorted(dec_ms)[len(dec_ms) // 2]
        moved = n * (64 + 8 + 128)
        out[name] = dict(packets=n, decode_with_layouts_ms=round(d, 4), extract_fields_ms=round(f, 4),
                         fields_Mpkts_s=round(n / f / 1e3, 1), fields_GBps_layout_index_record=round(moved / f / 1e6, 1),
                         kernel=ctx.kernel_name(parser, data, off, cap, layouts=True))
        print(json.dumps({name: out[name]}), flush=True)
        del data, off, cap, rec, err, fl, lay, fields
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Each config's decode against its memory skeleton: on the
config's own batch in HBM, gpk_probe_skeleton_idx makes the decode's memory
accesses without its work. Per wave of 64 packets it reads the index entries
and the header windows (6 chunks at each packet), streams the wave's extent
(1 KiB passes, 8 in flight; not for configs without an L4 checksum, whose
decode reads the windows only), and writes the bytes the decode writes per
packet (16: record; 40: + flows; 168: + layer fields). The decode runs beside
it in interleaved rounds (HIP events, medians); decode / skeleton = how much of
its own memory pattern's rate the decode reaches. One JSON line per config.

    python tools/skeleton_all.py [--configs c3,c4,c4f,c2,c1]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# bytes written per packet, and whether the decode streams the packet bytes
SHAPE = {"c1": (16, True), "c2": (16, False), "c3": (40, True), "c4": (40, True), "c4f": (168, True)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3,c4,c4f,c2,c1")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--no-write", action="store_true", help="also time the skeleton without its writes")
    ap.add_argument("--write-forms", action="store_true",
                    help="also time the skeleton with default-policy stores, and with block-synchronous stores")
    a = ap.parse_args()
    import torch
    import bench
    from gopacket_amd import _lib, engine, synth
    S = _lib.synth_lib()
    stream = torch.cuda.current_stream()
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    ctx = engine.Context()
    for name in a.configs.split(","):
        fields = name.endswith("f")
        cfg = bench.CONFIGS[name.rstrip("f")]
        n = cfg.get("packets", 64 * 2**20)
        if "pcap" in cfg:
            data, off, cap = bench.pcap_tiled(cfg["pcap"], n)
        else:
            data, off, cap = synth.device_batch(cfg["synth"], 0, n, stream=stream)
        wbytes, streamed = SHAPE[name]
        wbuf = torch.empty(wbytes * n, dtype=torch.uint8, device="cuda")
        parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in cfg["decoders"]], outputs=cfg["outputs"])
        rec = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
        err = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
        fl = torch.empty(3 * n, dtype=torch.int64, device="cuda")
        fld = torch.empty(n * 128 if fields else 16, dtype=torch.uint8, device="cuda")
        flags = 2 | (0 if streamed else 64)

        def skeleton():
            assert S.gpk_probe_skeleton_idx(data.data_ptr(), off.data_ptr(), cap.data_ptr(), n, wbuf.data_ptr(),
                                            wbuf.numel(), wbytes, flags, sink.data_ptr(), stream.cuda_stream) == 0

        def decode():
            if fields:
                ctx.decode_device_fields(parser, data, off, cap, rec, err, fl, fld, stream=stream)
            else:
                ctx.decode_device(parser, data, off, cap, rec, err, fl, stream=stream)

        def skeleton_nowrite():
            assert S.gpk_probe_skeleton_idx(data.data_ptr(), off.data_ptr(), cap.data_ptr(), n, wbuf.data_ptr(),
                                            wbuf.numel(), 0, flags, sink.data_ptr(), stream.cuda_stream) == 0

        def skeleton_flags(extra):
            def go():
                rc = S.gpk_probe_skeleton_idx(data.data_ptr(), off.data_ptr(), cap.data_ptr(), n, wbuf.data_ptr(),
                                              wbuf.numel(), wbytes, flags | extra, sink.data_ptr(), stream.cuda_stream)
                assert rc == 0, "skeleton form %d rejected for %d-byte outputs" % (extra, wbytes)
            return go

        runs = {"skeleton": skeleton, "decode": decode}
        if a.no_write:
            runs["skeleton_no_writes"] = skeleton_nowrite
        if a.write_forms:
            runs["skeleton_temporal_writes"] = skeleton_flags(8)
            runs["skeleton_block_writes"] = skeleton_flags(16)
            runs["skeleton_writes_first"] = skeleton_flags(32)
            runs["skeleton_writes_ring"] = skeleton_flags(128)
            runs["skeleton_writes_ring_temporal"] = skeleton_flags(128 | 8)
            runs["skeleton_writes_l2ring_temporal"] = skeleton_flags(1024 | 8)
            runs["skeleton_writes_l2ring"] = skeleton_flags(1024)
            runs["skeleton_writes_by_wave0"] = skeleton_flags(256)
            if wbytes == 40:  # record + flows interleaved, one 2560-byte run per wave; and the records alone
                runs["skeleton_writes_interleaved"] = skeleton_flags(512)
                runs["skeleton_records_only"] = lambda: S.gpk_probe_skeleton_idx(
                    data.data_ptr(), off.data_ptr(), cap.data_ptr(), n, wbuf.data_ptr(), wbuf.numel(), 16, flags,
                    sink.data_ptr(), stream.cuda_stream)
            if streamed:  # a fifth wave per block that only stores (the others only read)
                runs["skeleton_storer_wave"] = lambda: S.gpk_probe_skeleton_storer(
                    data.data_ptr(), off.data_ptr(), cap.data_ptr(), n, wbuf.data_ptr(), wbuf.numel(), wbytes,
                    sink.data_ptr(), stream.cuda_stream)
        times = {k: [] for k in runs}
        for rnd in range(a.rounds + 1):
            for k, f in runs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(a.steps):
                    f()
                e1.record(stream)
                torch.cuda.synchronize()
                if rnd:
                    times[k].append(e0.elapsed_time(e1) / a.steps)
        algo = int(cap.sum(dtype=torch.int64).item()) + 12 * n
        sk, de = float(np.median(times["skeleton"])), float(np.median(times["decode"]))
        print(json.dumps({"config": name, "packets": n, "written_bytes_per_packet": wbytes, "streamed": streamed,
                          "skeleton_ms": round(sk, 4), "decode_ms": round(de, 4),
                          "decode_algorithmic_GBps": round(algo / (de * 1e-3) / 1e9, 1),
                          "decode_over_skeleton_rate": round(sk / de, 4),
                          **{k + "_ms": round(float(np.median(v)), 4) for k, v in times.items()
                             if k not in ("skeleton", "decode")}}), flush=True)
        del data, off, cap, wbuf, rec, err, fl, fld
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

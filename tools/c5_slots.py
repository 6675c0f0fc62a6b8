#!/usr/bin/env python3
"""Per-slot timeline of a C5 replay (GPK_REPLAY_TRACE=2 in the library prints
one line per staging slot to stderr: read start/end, when the main loop got
the slot, when its walk finished, when its launches were issued).

    GPK_REPLAY_TRACE=2 python tools/c5_slots.py [--gib 10] [--read-threads 16] [--slots 4]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=10.0)
    ap.add_argument("--read-threads", type=int, default=16)
    ap.add_argument("--slots", type=int, default=4)
    ap.add_argument("--slot-mib", type=int, default=256)
    a = ap.parse_args()
    import torch  # noqa: F401
    from gopacket_amd import _lib, engine
    import bench
    S = _lib.synth_lib()
    cfg = bench.CONFIGS["c4"]
    parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in cfg["decoders"]], outputs=cfg["outputs"])
    per = S.gpk_synth_bytes(4, 0, 1 << 20) / (1 << 20) + 33.5
    n = int(a.gib * 2**30 / per)
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "gpk_c5s_%d.pcapng" % os.getpid())
    S.gpk_synth_write_pcapng(path.encode(), 4, 0, n, 16)
    ctx = engine.Context(0)
    try:
        for r in range(2):
            print("== call %d" % r, file=sys.stderr, flush=True)
            t0 = time.perf_counter()
            _, st = ctx.replay_file(parser, path, collect=False, on_batch=lambda *x: None, read_threads=a.read_threads,
                                    slots=a.slots, slot_bytes=a.slot_mib << 20)
            w = time.perf_counter() - t0
            print("call %d: %.4f s, %.2f GB/s, read %.3f index %.3f gpu %.3f" % (
                r, st["wall_s"], st["file_bytes"] / st["wall_s"] / 1e9, st["read_s"], st["index_s"], st["gpu_s"]),
                file=sys.stderr, flush=True)
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()

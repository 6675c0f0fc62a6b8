#!/usr/bin/env python3
"""C5 cold call: gpk_replay_file on a fresh context (staging buffers not yet
allocated) against the same call with the context's kept buffers, and the
background allocation behind the first read (default) against allocating
everything before it (GPK_REPLAY_EAGER_ALLOC=1), alternating, in one
process.

    python tools/c5_cold.py [--gib 10] [--rounds 3]

Each cold call uses a new gpk_ctx (so nothing is kept); the process's first
call also pays the first use of the HIP modules, so it is reported apart.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=10.0)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--no-fsync", action="store_true", help="replay while the file's writeback may still run")
    a = ap.parse_args()
    import torch  # noqa: F401
    import bench
    from gopacket_amd import _lib, engine
    S = _lib.synth_lib()
    cfg = bench.CONFIGS["c4"]
    per = S.gpk_synth_bytes(4, 0, 1 << 20) / (1 << 20) + 32 + 1.5
    n = int(a.gib * 2**30 / per)
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "gpk_c5cold_%d.pcapng" % os.getpid())
    size = S.gpk_synth_write_pcapng(path.encode(), 4, 0, n, 16)
    if not a.no_fsync:  # writeback done before the first call (as bench.py's C5)
        fd = os.open(path, os.O_RDONLY)
        os.fsync(fd)
        os.close(fd)
    out = dict(file_bytes=size, packets=n, runs=[])

    def call(ctx, label):
        parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in cfg["decoders"]], outputs=cfg["outputs"])
        t = time.perf_counter()
        _, st = ctx.replay_file(parser, path, collect=False, read_threads=8)
        w = time.perf_counter() - t
        r = dict(label=label, wall_s=round(st["wall_s"], 4), py_wall_s=round(w, 4),
                 GBps=round(st["file_bytes"] / st["wall_s"] / 1e9, 2), alloc_wait_s=round(st["alloc_wait_s"], 4),
                 packets=st["packets"], error=st["error"])
        out["runs"].append(r)
        print(json.dumps(r), flush=True)

    try:
        first = engine.Context(0)
        call(first, "process first call (the context loaded the walk module)")
        call(first, "warm (kept buffers)")
        for k in range(a.rounds):
            for eager in (False, True):
                if eager:
                    os.environ["GPK_REPLAY_EAGER_ALLOC"] = "1"
                else:
                    os.environ.pop("GPK_REPLAY_EAGER_ALLOC", None)
                ctx = engine.Context(0)
                call(ctx, "cold eager" if eager else "cold background allocation (default)")
                call(ctx, "warm")
                del ctx
        os.environ.pop("GPK_REPLAY_EAGER_ALLOC", None)
    finally:
        os.unlink(path)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

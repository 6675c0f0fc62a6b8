#!/usr/bin/env python3
"""Where does host memory grow over replays with many small batches? One C4
pcapng, small staging (8 MiB slots, 16 Ki-packet batches: ~125 batches per
call), REPS calls per phase: (a) Context.replay_file (numpy views per batch),
with tracemalloc's top growth sites; (b) gpk_replay_file through ctypes with
a no-op callback (no Python objects per batch); (c) as (b) with
GPK_REPLAY_HOST_WALK=1 semantics left to the env of the run. SLOT_MIB and
BATCH set the staging shape; ONLY_RAW=1 runs (b) alone."""
import ctypes
import gc
import os
import sys
import tracemalloc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from soak import rss_mib  # noqa: E402


def main(reps=int(os.environ.get("REPS", "60"))):
    import bench
    from gopacket_amd import _lib, engine
    cfg = bench.CONFIGS["c4"]
    parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in cfg["decoders"]], outputs=cfg["outputs"])
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "gpk_rrss_%d.pcapng" % os.getpid())
    n = 2_000_000
    assert _lib.synth_lib().gpk_synth_write_pcapng(path.encode(), 4, 0, n, 16) > 0
    ctx = engine.Context(0)
    shape = dict(slot_bytes=int(os.environ.get("SLOT_MIB", "8")) << 20, slots=3,
                 batch_pkts=int(os.environ.get("BATCH", str(1 << 14))))
    L = _lib.lib()
    calls = [0]

    def noop(*a):
        calls[0] += 1

    c_cb = _lib.REPLAY_CB(noop)

    def raw():
        o = _lib.ReplayOpts(0, 0, shape["slot_bytes"], shape["slots"], shape["batch_pkts"], int(os.environ.get("RT", "0")), _lib.REPLAY_FIELDS_CB(),
                            _lib.REPLAY_PACKETS_CB())
        st = _lib.ReplayStats()
        _lib.check(L.gpk_replay_file(ctx.h, parser.h, path.encode(), ctypes.byref(o), c_cb, None, ctypes.byref(st)))
        assert st.packets == n

    try:
        for _ in range(5):
            ctx.replay_file(parser, path, collect=False, on_batch=lambda *a: None, **shape)
            raw()
        gc.collect()
        if os.environ.get("ONLY_RAW") == "1":
            class MallInfo2(ctypes.Structure):
                _fields_ = [(f, ctypes.c_size_t) for f in ("arena", "ordblks", "smblks", "hblks", "hblkhd", "usmblks",
                                                            "fsmblks", "uordblks", "fordblks", "keepcost")]
            libc = ctypes.CDLL("libc.so.6")
            libc.mallinfo2.restype = MallInfo2
            m0 = libc.mallinfo2()
            r0, calls[0] = rss_mib(), 0
            for _ in range(reps):
                raw()
            gc.collect()
            m1 = libc.mallinfo2()
            print("malloc (main arena) in use %+.1f MiB, mmapped blocks %+.1f MiB (%+d)" % (
                (m1.uordblks - m0.uordblks) / 2**20, (m1.hblkhd - m0.hblkhd) / 2**20, m1.hblks - m0.hblks), flush=True)
            print("%s: %d calls, %d batches: rss %+.1f MiB, %.2f KB per call, %.2f KB per batch" % (
                shape, reps, calls[0], rss_mib() - r0, (rss_mib() - r0) * 1024 / reps,
                (rss_mib() - r0) * 1024 / max(calls[0], 1)), flush=True)
            return
        tracemalloc.start(8)
        s0, r0 = tracemalloc.take_snapshot(), rss_mib()
        for _ in range(reps):
            ctx.replay_file(parser, path, collect=False, on_batch=lambda *a: None, **shape)
        gc.collect()
        s1, r1 = tracemalloc.take_snapshot(), rss_mib()
        tracemalloc.stop()
        print("(a) replay_file x%d: rss %+.1f MiB; tracemalloc top growth:" % (reps, r1 - r0), flush=True)
        for st in s1.compare_to(s0, "lineno")[:6]:
            print("    ", st, flush=True)
        gc.collect()
        r0, calls[0] = rss_mib(), 0
        for _ in range(reps):
            raw()
        gc.collect()
        print("(b) raw gpk_replay_file x%d, no-op callback (%d batches): rss %+.1f MiB" % (
            reps, calls[0], rss_mib() - r0), flush=True)
        r0 = rss_mib()
        for _ in range(reps):
            raw()
        gc.collect()
        print("(b') again: rss %+.1f MiB" % (rss_mib() - r0), flush=True)
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()

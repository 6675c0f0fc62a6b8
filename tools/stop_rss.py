#!/usr/bin/env python3
"""Host RSS across many replays of one C4 pcapng on one context, four phases
of REPS calls each: a fixed staging shape run to the end; the same shape
stopped (gpk_stop) in its third batch; the staging shape changed every call
(three shapes in turn) run to the end; changed every call and stopped.
Growth in one phase and not in the others points at what holds memory."""
import gc
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from soak import rss_mib  # noqa: E402


def main(reps=int(os.environ.get("REPS", "100"))):
    import bench
    from gopacket_amd import _lib, engine
    cfg = bench.CONFIGS["c4"]
    parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in cfg["decoders"]], outputs=cfg["outputs"])
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "gpk_stoprss_%d.pcapng" % os.getpid())
    n = 2_000_000
    assert _lib.synth_lib().gpk_synth_write_pcapng(path.encode(), 4, 0, n, 16) > 0
    ctx = engine.Context(0)
    shapes = [dict(slot_bytes=8 << 20, slots=3, batch_pkts=1 << 14), dict(slot_bytes=32 << 20, slots=2, batch_pkts=1 << 16),
              dict(slot_bytes=64 << 20, slots=4, batch_pkts=1 << 18)]

    def call(shape, stop):
        seen = [0]

        def cb(*a):
            seen[0] += 1
            if stop and seen[0] == 3:
                ctx.stop()

        _, st = ctx.replay_file(parser, path, collect=False, on_batch=cb, **shape)
        assert st["stopped"] == stop, st
        assert stop or st["packets"] == n

    try:
        for _ in range(5):
            call(shapes[0], False)
        for phase, (churn, stop) in enumerate([(False, False), (False, True), (True, False), (True, True)]):
            gc.collect()
            r0 = rss_mib()
            for k in range(reps):
                call(shapes[k % 3] if churn else shapes[0], stop)
            gc.collect()
            print("phase %d (%s shape, %s): rss %.1f -> %.1f MiB (%+.1f)" % (
                phase, "changing" if churn else "fixed", "stopped in batch 3" if stop else "to the end", r0, rss_mib(),
                rss_mib() - r0), flush=True)
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()

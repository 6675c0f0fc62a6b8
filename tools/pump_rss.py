#!/usr/bin/env python3
"""Heap in use (glibc mallinfo2) and RSS over many AF_PACKET ring pumps on one
context: an emulated TPACKET_V3 ring re-armed before each pump, small
batches (many per pump), with and without fields and packets, as
tools/replay_rss.py does for the replay."""
import ctypes
import gc
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from soak import rss_mib  # noqa: E402


class MallInfo2(ctypes.Structure):
    _fields_ = [(f, ctypes.c_size_t) for f in ("arena", "ordblks", "smblks", "hblks", "hblkhd", "usmblks", "fsmblks",
                                                "uordblks", "fordblks", "keepcost")]


def main(reps=int(os.environ.get("REPS", "200"))):
    import bench
    from gopacket_amd import _lib, afpacket, engine
    libc = ctypes.CDLL("libc.so.6")
    libc.mallinfo2.restype = MallInfo2
    cfg = bench.CONFIGS["c4"]
    parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in cfg["decoders"]], outputs=cfg["outputs"])
    ctx = engine.Context(0)
    bs, nb = 1 << 20, 16
    ring = np.zeros(bs * nb, np.uint8)
    _lib.synth_lib().gpk_synth_tpacket_v3(ring.ctypes.data, bs, nb, 4, 0, 2, 0, None)

    def pump(k):
        ring[8::bs] = 1
        tp = afpacket.AttachRing(ring, afpacket.TPacketVersion3, afpacket.OptFrameSize(4096),
                                 afpacket.OptBlockSize(bs), afpacket.OptNumBlocks(nb))
        _, st = tp.Pump(ctx, parser, batch_pkts=1000 + 37 * (k % 7), collect=False, on_batch=lambda *a: None,
                        fields=bool(k & 1), packets=bool(k & 2))
        tp.Close()
        return st["packets"]

    for k in range(10):
        pump(k)
    gc.collect()
    m0, r0 = libc.mallinfo2(), rss_mib()
    total = sum(pump(k) for k in range(reps))
    gc.collect()
    m1 = libc.mallinfo2()
    print("%d pumps, %d packets: heap in use %+.1f MiB, RSS %+.1f MiB" % (
        reps, total, (m1.uordblks - m0.uordblks) / 2**20, rss_mib() - r0), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Host RSS over many plain replays of one small file (does it level off?)."""
import ctypes
import gc
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from soak import rss_mib  # noqa: E402


def main(reps=int(os.environ.get("SOAK_REPS", "200")), walk=os.environ.get("GPK_REPLAY_HOST_WALK", "0")):
    import bench
    from gopacket_amd import _lib, engine
    S = _lib.synth_lib()
    cfg = bench.CONFIGS["c4"]
    parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in cfg["decoders"]], outputs=cfg["outputs"])
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "gpk_soakl_%d.pcapng" % os.getpid())
    n = 2_000_000
    assert S.gpk_synth_write_pcapng(path.encode(), 4, 0, n, 16) > 0
    ctx = engine.Context(0)
    cb = _lib.REPLAY_CB(lambda *a: None)
    import numpy as np

    def views(user, first, k, base, nbytes, off, cap):  # the packets' offsets and lengths as numpy views
        o_ = np.ctypeslib.as_array(ctypes.cast(off, ctypes.POINTER(ctypes.c_uint64)), (k,))
        c_ = np.ctypeslib.as_array(ctypes.cast(cap, ctypes.POINTER(ctypes.c_uint32)), (k,))
        int((o_ + c_.astype(np.uint64)).max())

    import time

    def views_only(user, first, k, base, nbytes, off, cap):  # the views alone, no arithmetic
        np.ctypeslib.as_array(ctypes.cast(off, ctypes.POINTER(ctypes.c_uint64)), (k,))
        np.ctypeslib.as_array(ctypes.cast(cap, ctypes.POINTER(ctypes.c_uint32)), (k,))

    def frombuf(user, first, k, base, nbytes, off, cap):  # views through from_address + frombuffer
        o_ = np.frombuffer((ctypes.c_uint8 * (8 * k)).from_address(off), np.uint64)
        c_ = np.frombuffer((ctypes.c_uint8 * (4 * k)).from_address(cap), np.uint32)
        int((o_ + c_.astype(np.uint64)).max())

    def read_only(user, first, k, base, nbytes, off, cap):  # read the pinned offsets, no temporaries
        int(np.ctypeslib.as_array(ctypes.cast(off, ctypes.POINTER(ctypes.c_uint64)), (k,)).max())

    def temps_only(user, first, k, base, nbytes, off, cap):  # temporaries of the same size, no pinned reads
        int((np.zeros(k, np.uint64) + np.ones(k, np.uint32).astype(np.uint64)).max())

    def sleeper(user, first, k, base, nbytes, off, cap):  # a slow consumer that touches nothing
        time.sleep(0.005)

    mode = os.environ.get("SOAK_PACKETS", "0")
    pcb = _lib.REPLAY_PACKETS_CB({"1": views, "sleep": sleeper, "vo": views_only, "fb": frombuf, "ro": read_only,
                                    "to": temps_only}[mode]) if mode != "0" else _lib.REPLAY_PACKETS_CB()
    slow_cb = os.environ.get("SOAK_SLOW_CB") == "1"
    if slow_cb:  # the results callback slow instead, no packets callback
        cb = _lib.REPLAY_CB(lambda *a: time.sleep(0.005))
    o = _lib.ReplayOpts(0, 0, 0, 0, 0, 0, _lib.REPLAY_FIELDS_CB(), pcb)
    try:
        line = []
        for k in range(reps + 1):
            st = _lib.ReplayStats()
            assert _lib.lib().gpk_replay_file(ctx.h, parser.h, path.encode(), ctypes.byref(o), cb, None,
                                              ctypes.byref(st)) == 0
            if k % 50 == 0:
                gc.collect()
                line.append("%d:%.0f" % (k, rss_mib()))
        print("host walk %s, packets %s, slow cb %s, rss MiB by replay: %s" % (
            walk, mode, slow_cb, " ".join(line)), flush=True)
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Host RSS of the context's launch marks (gpk_host.cpp mark_after) in
isolation: per iteration, record an event on stream s, make the aggregation
stream wait for it, and record a mark on the aggregation stream; 'cumulative'
also makes the aggregation stream wait for the mark's own previous record
first (the table slot's done mark). Does a mark re-recorded behind itself
keep every earlier record alive?"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from soak import rss_mib  # noqa: E402


def main(n=int(os.environ.get("ITERS", "50000"))):
    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipSetDevice(0) == 0

    def mk_stream():
        s = ctypes.c_void_p()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0
        return s

    def mk_event():
        e = ctypes.c_void_p()
        assert hip.hipEventCreateWithFlags(ctypes.byref(e), 2) == 0
        return e

    s, agg, ev, mark = mk_stream(), mk_stream(), mk_event(), mk_event()
    for variant in ("plain", "cumulative", "plain", "cumulative", "cumulative+sync"):
        r0 = rss_mib()
        for i in range(n):
            hip.hipEventRecord(ev, s)
            hip.hipStreamWaitEvent(agg, ev, 0)
            if variant.startswith("cumulative"):
                hip.hipStreamWaitEvent(agg, mark, 0)
            hip.hipEventRecord(mark, agg)
            if variant.endswith("sync") and i % 1000 == 999:
                hip.hipStreamSynchronize(agg)
        hip.hipDeviceSynchronize()
        print("%d iterations %-16s rss %+.1f MiB" % (n, variant, rss_mib() - r0), flush=True)
    # the replay's slot pattern: three streams in turn, each copy waiting for the previous slot's
    # "sent" event on another stream, then recording its own; the consumer synchronizes each slot
    ss = [mk_stream() for _ in range(3)]
    es = [mk_event() for _ in range(3)]
    dbuf, hbuf = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(dbuf), ctypes.c_size_t(1 << 20)) == 0
    assert hip.hipHostMalloc(ctypes.byref(hbuf), ctypes.c_size_t(1 << 20), 0) == 0
    for variant in ("copy-chain", "copy-chain", "copy-nowait"):
        r0 = rss_mib()
        m = n // 5
        for i in range(m):
            k = i % 3
            if variant == "copy-chain":
                hip.hipStreamWaitEvent(ss[k], es[(k + 2) % 3], 0)
            hip.hipMemcpyAsync(dbuf, hbuf, ctypes.c_size_t(1 << 16), 1, ss[k])
            hip.hipEventRecord(es[k], ss[k])
            hip.hipStreamSynchronize(ss[(k + 2) % 3])
        hip.hipDeviceSynchronize()
        print("%d iterations %-16s rss %+.1f MiB (%.2f KB per iteration)" % (
            m, variant, rss_mib() - r0, (rss_mib() - r0) * 1024 / m), flush=True)


if __name__ == "__main__":
    main()

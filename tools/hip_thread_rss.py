#!/usr/bin/env python3
"""Host RSS over short-lived threads: N threads that only start and exit,
then N threads that each make HIP calls (hipSetDevice, hipStreamQuery on the
null stream) and exit, then N that each do what a replay fill thread does
(wait on an event, copy, record, on one stream). Does the HIP runtime keep per-thread state after a
thread that called it has ended?"""
import ctypes
import sys
import threading

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
from soak import rss_mib  # noqa: E402


def main(n=2000):
    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipSetDevice(0) == 0 and hip.hipDeviceSynchronize() == 0

    def run(f):
        for _ in range(n // 100):
            ts = [threading.Thread(target=f) for _ in range(100)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()

    def hip_calls():
        hip.hipSetDevice(0)
        hip.hipStreamQuery(None)

    stream, ev = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(stream), 1) == 0
    assert hip.hipEventCreateWithFlags(ctypes.byref(ev), 2) == 0
    dbuf, hbuf = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(dbuf), ctypes.c_size_t(1 << 16)) == 0
    assert hip.hipHostMalloc(ctypes.byref(hbuf), ctypes.c_size_t(1 << 16), 0) == 0

    def async_calls():  # what a replay fill thread does: wait, copy, record on the slot's stream
        hip.hipSetDevice(0)
        hip.hipStreamWaitEvent(stream, ev, 0)
        hip.hipMemcpyAsync(dbuf, hbuf, ctypes.c_size_t(1 << 16), 1, stream)
        hip.hipEventRecord(ev, stream)
        hip.hipStreamSynchronize(stream)

    for name, f in (("empty", lambda: None), ("hip", hip_calls), ("empty", lambda: None), ("hip", hip_calls),
                    ("async-copy", async_calls), ("async-copy", async_calls), ("async-copy", async_calls)):
        r0 = rss_mib()
        run(f)
        print("%d %s threads: rss %+.1f MiB" % (n, name, rss_mib() - r0), flush=True)


if __name__ == "__main__":
    main()

"""pcapng record walk speed on this host: gpk_capreader_index_all over a
256 MiB in-memory slot of C4-mix EPBs, by thread count, repeated calls."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
from gopacket_amd import _lib  # noqa: E402

S = _lib.synth_lib()
L = _lib.lib()
path = "/tmp/cap_walk_%d.pcapng" % os.getpid()
size = S.gpk_synth_write_pcapng(path.encode(), 4, 0, 700000, 16)
buf = np.fromfile(path, np.uint8)
os.unlink(path)
print("file", size, "bytes")
for T in (1, 4, 8, 16, 32):
    ts = []
    for rep in range(4):
        r = ctypes.c_void_p()
        _lib.check(L.gpk_capreader_create(ctypes.byref(r), _lib.CAP_PCAPNG, 0))
        xi = _lib.CapIndex()
        used = ctypes.c_uint64()
        t = time.perf_counter()
        st = L.gpk_capreader_index_all(r, buf.ctypes.data, len(buf), 1, T, ctypes.byref(xi), ctypes.byref(used))
        ts.append(time.perf_counter() - t)
        n = xi.n
        L.gpk_capindex_free(ctypes.byref(xi))
        L.gpk_capreader_destroy(r)
    print("T=%2d  %d pkts  best %.2f ms (%.1f ns/pkt), first %.2f ms" % (T, n, min(ts) * 1e3, min(ts) / n * 1e9,
                                                                      ts[0] * 1e3), flush=True)

"""Ring walk speed on this host: index calls over a 256 MiB V3 ring, by thread count."""
import sys, os, time, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
from gopacket_amd import _lib, afpacket
S = _lib.synth_lib(); L = _lib.lib()
bs, nb = 4 << 20, 64
ring = np.zeros(bs * nb, np.uint8)
n = S.gpk_synth_tpacket_v3(ring.ctypes.data, bs, nb, 4, 0, 2, 0, None)
for T in (1, 2, 4, 8, 16, 32):
    for m in (1 << 18, 1 << 20):
        ring[8::bs] = 1
        tp = afpacket.AttachRing(ring, 2, afpacket.OptFrameSize(4096), afpacket.OptBlockSize(bs), afpacket.OptNumBlocks(nb))
        L.gpk_tpacket_set_threads(tp.h, T)
        off = np.zeros(m, np.uint64); cap = np.zeros(m, np.uint32); ci = np.zeros(m, _lib.TPINFO_DTYPE)
        k = ctypes.c_uint64(); u = ctypes.c_uint64(); tot = 0
        t = time.perf_counter()
        while True:
            st = L.gpk_tpacket_index(tp.h, 0, off.ctypes.data, cap.ctypes.data, ci.ctypes.data, m, ctypes.byref(k), None, 0, ctypes.byref(u))
            tot += k.value
            if st != 1: break
        dt = time.perf_counter() - t
        print("T=%2d m=%7d  %d pkts  %.2f ns/pkt  %.1f Mpkts/s" % (T, m, tot, dt / tot * 1e9, tot / dt / 1e6), flush=True)
        tp.Close()

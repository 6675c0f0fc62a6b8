#!/usr/bin/env python3
"""A config's memory skeleton (gpk_probe_skeleton_idx) in one write form,
launched a few times, for rocprofv3 --pmc passes ("What the
writes cost"): forms 'writes' (the decode's non-temporal stores), 'nowrite',
'l2ring' (outputs at i mod 2^14, temporal: they stay in each XCD's L2) and
'ring' (i mod 2^20, temporal: 40 MiB, they leave L2 and stay in the Infinity
Cache).

    rocprofv3 --pmc TCC_EA0_WRREQ ... -- python3 tools/skeleton_pmc.py --config c4 --form writes
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FORMS = {"writes": (None, 0), "nowrite": (0, 0), "l2ring": (None, 1024 | 8), "ring": (None, 128 | 8)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--form", default="writes", choices=sorted(FORMS))
    ap.add_argument("--launches", type=int, default=4)
    a = ap.parse_args()
    import torch
    import bench
    from gopacket_amd import _lib, synth
    S = _lib.synth_lib()
    cfg = bench.CONFIGS[a.config]
    n = 64 * 2**20
    stream = torch.cuda.current_stream()
    data, off, cap = synth.device_batch(cfg["synth"], 0, n, stream=stream)
    w, streamed = bench.skeleton_shape(cfg)
    wbytes, extra = FORMS[a.form]
    wbytes = w if wbytes is None else wbytes
    wbuf = torch.empty(max(w, 16) * n, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    flags = 2 | (0 if streamed else 64) | extra
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for k in range(a.launches + 1):
        if k == 1:
            e0.record(stream)
        assert S.gpk_probe_skeleton_idx(data.data_ptr(), off.data_ptr(), cap.data_ptr(), n, wbuf.data_ptr(),
                                        wbuf.numel(), wbytes, flags, sink.data_ptr(), stream.cuda_stream) == 0
    e1.record(stream)
    torch.cuda.synchronize()
    print("%s %s: %.4f ms per launch" % (a.config, a.form, e0.elapsed_time(e1) / a.launches))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""In-process A/B of kernel variants: every variant library is loaded into one
process (ctypes, RTLD_LOCAL: each keeps its own gpk_* symbols and HIP
module), the synthetic batch is generated once, and the variants are timed
in interleaved rounds so clocks and thermals affect them alike.

    python tools/ab_inproc.py --configs c3,c2,c4 --rounds 5 --steps 5 base w6 w7 ...

"base" = gopacket_amd/libgpk.so, NAME = gopacket_amd/build/libgpk_NAME.so;
NAME@global runs that library with gpk_ctx_set_table_mode(GPK_TABLES_GLOBAL);
NAME@narrow runs gpk_decode_batch_narrow (the 8-byte record and its side array)
instead of gpk_decode_batch, and --check compares it with a 16-byte variant by
the gpk_record8 rules (include/gpk.h).
--fields times gpk_decode_batch_fields (the fused decode + layer fields launch)
instead of gpk_decode_batch. --check compares every variant's records, error
arguments and flows (and fields) with the first variant's, bit for bit.
Prints, per config and variant, the median and min kernel ms over rounds.
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def load(name):
    import torch  # noqa: F401  (one HIP runtime: torch's)
    path = os.path.join(ROOT, "gopacket_amd", "libgpk.so" if name == "base" else "build/libgpk_%s.so" % name)
    L = ctypes.CDLL(path)
    vp = ctypes.c_void_p
    L.gpk_ctx_create.argtypes = [ctypes.POINTER(vp), ctypes.c_int]
    L.gpk_parser_create.argtypes = [ctypes.POINTER(vp), ctypes.c_int64]
    L.gpk_parser_add_decoder.argtypes = [vp, ctypes.c_int]
    L.gpk_parser_set_outputs.argtypes = [vp, ctypes.c_uint32]
    L.gpk_decode_batch.argtypes = [vp, vp, vp, vp, vp]
    if hasattr(L, "gpk_decode_batch_fields"):
        L.gpk_decode_batch_fields.argtypes = [vp, vp, vp, vp, vp, vp]
    if hasattr(L, "gpk_decode_batch_narrow"):
        L.gpk_decode_batch_narrow.argtypes = [vp, vp, vp, vp, vp]
    return L


def narrow_matches(rec16, rec8, wide, n):
    """gpk_record8 rules: a widened packet's side record is the 16-byte record;
    every other packet's layers and status bits (nlayers in 4 bits) are."""
    import numpy as np
    from gopacket_amd import _lib
    r = rec16.cpu().numpy().view(_lib.RECORD_DTYPE)
    r8 = rec8.cpu().numpy().view(_lib.RECORD8_DTYPE)
    w8 = wide.cpu().numpy().view(_lib.RECORD_DTYPE)
    w = (r8["status"] & _lib.ST8_WIDE) != 0
    nl = (r["status"] >> 8) & 0xFFF
    keep = ~np.uint32(0xFFF << 8)
    return bool(np.array_equal(w8[w], r[w]) and np.array_equal(r8["layers"][~w].astype(np.uint64), r["layers"][~w])
                and np.array_equal(r8["status"][~w] & keep, r["status"][~w] & keep)
                and np.array_equal((r8["status"] >> 8) & 0xF, np.where(nl > 8, 15, nl).astype(np.uint32)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3,c2,c4")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--packets", type=int, default=64 * 2**20)
    ap.add_argument("--fields", action="store_true")
    ap.add_argument("--check", action="store_true")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from gopacket_amd import _lib, engine, synth
    libs = {v: load(v.split("@")[0]) for v in a.variants}
    narrow = {v: v.endswith("@narrow") for v in a.variants}
    stream = torch.cuda.current_stream()
    for name in a.configs.split(","):
        cfg = bench.CONFIGS[name]
        n = cfg.get("packets", a.packets)
        if "pcap" in cfg:
            data, off, cap = bench.pcap_tiled(cfg["pcap"], n)
        else:
            data, off, cap = synth.device_batch(cfg["synth"], 0, n, stream=stream)
        rec = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
        err = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
        fl = torch.empty(3 * n, dtype=torch.int64, device="cuda")
        algo = int(cap.sum(dtype=torch.int64).item()) + 12 * n
        fields = torch.empty(n * 128 if a.fields else 16, dtype=torch.uint8, device="cuda")
        b = _lib.Batch(data.data_ptr(), off.data_ptr(), cap.data_ptr(), n, data.numel())
        r = _lib.Results(rec.data_ptr(), err.data_ptr(), fl.data_ptr(), None)
        rec8 = torch.empty(n * 8 if any(narrow.values()) else 8, dtype=torch.uint8, device="cuda")
        wide = torch.zeros(n * 16 if any(narrow.values()) else 16, dtype=torch.uint8, device="cuda")
        r8 = _lib.Results8(rec8.data_ptr(), wide.data_ptr(), err.data_ptr(), fl.data_ptr())

        def run(v, L, ctx, p):
            if narrow[v]:
                return L.gpk_decode_batch_narrow(ctx, p, ctypes.byref(b), ctypes.byref(r8),
                                                 ctypes.c_void_p(stream.cuda_stream))
            if a.fields:
                return L.gpk_decode_batch_fields(ctx, p, ctypes.byref(b), ctypes.byref(r),
                                                 ctypes.c_void_p(fields.data_ptr()), ctypes.c_void_p(stream.cuda_stream))
            return L.gpk_decode_batch(ctx, p, ctypes.byref(b), ctypes.byref(r), ctypes.c_void_p(stream.cuda_stream))
        handles = {}
        for v, L in libs.items():
            ctx, p = ctypes.c_void_p(), ctypes.c_void_p()
            assert L.gpk_ctx_create(ctypes.byref(ctx), 0) == 0
            if v.endswith("@global"):
                assert L.gpk_ctx_set_table_mode(ctx, 1) == 0
            assert L.gpk_parser_create(ctypes.byref(p), 17) == 0
            for d in cfg["decoders"]:
                assert L.gpk_parser_add_decoder(p, engine.DECODER_KINDS[d]) == 0
            assert L.gpk_parser_set_outputs(p, cfg["outputs"]) == 0
            handles[v] = (ctx, p)
        occ = {}
        for v, L in libs.items():
            try:
                f = L.gpk_decode_occupancy
            except AttributeError:  # a library from before the diagnostic
                occ[v] = "?"
                continue
            o = ctypes.c_int()
            f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
            occ[v] = o.value if f(handles[v][0], handles[v][1], ctypes.byref(b), _lib.NAME_FIELDS if a.fields else 0,
                                  ctypes.byref(o)) == 0 else "?"
        times = {v: [] for v in libs}
        for rnd in range(a.rounds + 1):
            for v, L in libs.items():
                ctx, p = handles[v]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(a.steps):
                    assert run(v, L, ctx, p) == 0
                e1.record(stream)
                torch.cuda.synchronize()
                if rnd:  # round 0 warms every variant up
                    times[v].append(e0.elapsed_time(e1) / a.steps)
        for v in libs:
            t = np.array(times[v])
            print("%-4s %-10s median %8.3f ms  min %8.3f ms  %7.1f GB/s (%.1f%% of 8 TB/s)  blocks/CU %s" % (
                name, v, np.median(t), t.min(), algo / (np.median(t) * 1e-3) / 1e9,
                algo / (np.median(t) * 1e-3) / 8e12 * 100, occ[v]), flush=True)
        if a.check:
            ref = None
            for v, L in libs.items():
                ctx, p = handles[v]
                rec.fill_(0xA5)
                err.fill_(-1)
                fl.fill_(-1)
                fields.fill_(0x5A)
                wide.zero_()
                assert run(v, L, ctx, p) == 0
                torch.cuda.synchronize()
                out = [x.clone() for x in (rec, err, fl, fields)]
                if narrow[v]:  # the 16-byte records this narrow result stands for, where it can say them
                    out[0] = (rec8.clone(), wide.clone())
                if ref is None:
                    ref = out
                    continue
                if narrow[v]:
                    same = all(torch.equal(x, y) for x, y in zip(ref[1:3], out[1:3])) and \
                        narrow_matches(ref[0], *out[0], n)
                else:
                    same = all(torch.equal(x, y) for x, y in zip(ref, out))
                print("%-4s %-10s outputs %s the first variant's" % (name, v, "equal" if same else "DIFFER from"), flush=True)
            del ref, out
        del data, off, cap, rec, err, fl, fields, rec8, wide
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Where a decode wave's time goes: per-wave phase timestamps from a library
built with GPK_DIAG_TIMES (make -C gopacket_amd/csrc variant V=diag
VDEFS=-DGPK_DIAG_TIMES=1), one launch per config after warmup.

Per wave the kernel records (s_memrealtime, 100 MHz, one clock for the chip):
  t0 entry, t1 index landed, t2 header windows + table blob in LDS (after the
  block barrier), t3 DecodeLayers + IPv4 checksum + flows done, t4 phase B
  (segment sums) done, t5 record stored; HW_ID | XCC_ID << 32; phase-B region
  bytes | job lanes << 32.

Prints the mean phase durations, the kernel span, the mean number of resident
waves per SIMD (sum of wave lifetimes / (SIMDs x span)), per-phase
concurrency, and the gap between a wave slot's consecutive waves (dispatch +
the block's LDS held until its last wave ends).

    python tools/wave_times.py --lib diag --configs c4,c3,c2,c1
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def analyse(name, d, n_waves, out):
    t = d[:, :6].astype(np.int64)
    ok = (t[:, 0] > 0) & (t[:, 5] >= t[:, 0])
    t = t[ok]
    hw = d[ok, 6]
    pb = d[ok, 7]
    us = 0.01  # 10 ns ticks -> us
    span = (t[:, 5].max() - t[:, 0].min()) * us
    life = (t[:, 5] - t[:, 0]) * us
    ph = np.diff(t, axis=1) * us  # idx, win, parse, phaseB, tail
    hwid = (hw & 0xffffffff).astype(np.int64)
    xcc = (hw >> 32).astype(np.int64) & 0xf
    simd = (hwid >> 4) & 3
    cu = (hwid >> 8) & 15
    sh = (hwid >> 12) & 1
    se = (hwid >> 13) & 7
    wslot = hwid & 15
    key_simd = (((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
    nsimd = len(np.unique(key_simd))
    res = life.sum() / (nsimd * span)
    lines = []
    lines.append("%s: %d waves recorded (of %d), %d SIMDs, %d CUs, kernel span %.1f us" % (
        name, len(t), n_waves, nsimd, len(np.unique(key_simd // 4)), span))
    lines.append("  wave lifetime mean %.2f us (p10 %.2f, p50 %.2f, p90 %.2f)" % (
        life.mean(), *np.percentile(life, [10, 50, 90])))
    names = ("index", "window+blob+barrier", "parse+ip4+flows", "phase B", "tail")
    for k, nm in enumerate(names):
        lines.append("  %-22s mean %7.3f us  p50 %7.3f  p90 %7.3f  share %5.1f %%   concurrency %.2f waves/SIMD" % (
            nm, ph[:, k].mean(), np.percentile(ph[:, k], 50), np.percentile(ph[:, k], 90),
            100 * ph[:, k].sum() / life.sum(), ph[:, k].sum() / (nsimd * span)))
    lines.append("  resident waves per SIMD (mean over the span): %.2f" % res)
    lines.append("  resident waves per SIMD by XCD: %s" % " ".join(
        "%.2f" % (life[xcc == x].sum() / (max(1, len(np.unique(key_simd[xcc == x]))) * span)) for x in range(8)))
    # steady state: the middle 80 % of the span
    t0, t1 = t[:, 0].min() + 0.1 * (span / us), t[:, 0].min() + 0.9 * (span / us)
    ov = np.clip(np.minimum(t[:, 5], t1) - np.maximum(t[:, 0], t0), 0, None) * us
    lines.append("  resident waves per SIMD (middle 80 %% of the span): %.2f" % (ov.sum() / (nsimd * 0.8 * span)))
    # gaps between consecutive waves of one hardware wave slot
    key_slot = key_simd * 16 + wslot
    o = np.lexsort((t[:, 0], key_slot))
    ks, s0, s5 = key_slot[o], t[o, 0], t[o, 5]
    same = ks[1:] == ks[:-1]
    gap = (s0[1:] - s5[:-1])[same] * us
    lines.append("  wave-slot gap (next wave start - previous end): mean %.2f us, p50 %.2f, p90 %.2f, <0: %d" % (
        gap.mean(), np.percentile(gap, 50), np.percentile(gap, 90), int((gap < 0).sum())))
    # block skew: waves of one block end at different times; the block's LDS is freed at the last
    nb = len(d) // 4
    blk = d[: nb * 4, :6].astype(np.int64).reshape(nb, 4, 6)
    good = (blk[:, :, 0] > 0).all(axis=1)
    blk = blk[good]
    bend = blk[:, :, 5].max(axis=1)
    idle = ((bend[:, None] - blk[:, :, 5]) * us).mean()
    lines.append("  block skew: a wave ends %.2f us before its block's last wave (LDS held meanwhile)" % idle)
    # blocks resident per CU: a block holds its CU from its first wave's entry to its last wave's exit
    hwb = d[: nb * 4, 6].reshape(nb, 4)[good][:, 0]
    hwid_b = (hwb & 0xffffffff).astype(np.int64)
    cu_b = ((((hwb >> 32).astype(np.int64) & 0xf) * 8 + ((hwid_b >> 13) & 7)) * 2 + ((hwid_b >> 12) & 1)) * 16 + ((hwid_b >> 8) & 15)
    bstart = blk[:, :, 0].min(axis=1)
    ev_t = np.concatenate([bstart, bend])
    ev_d = np.concatenate([np.ones(len(bstart), np.int64), -np.ones(len(bend), np.int64)])
    ev_c = np.concatenate([cu_b, cu_b])
    o = np.lexsort((ev_d, ev_t, ev_c))
    ev_t, ev_d, ev_c = ev_t[o], ev_d[o], ev_c[o]
    conc = np.zeros(len(ev_t), np.int64)
    for c in np.unique(ev_c):
        m = ev_c == c
        conc[m] = np.cumsum(ev_d[m])
    maxc = np.array([conc[ev_c == c].max() for c in np.unique(ev_c)])
    # time-weighted share of the middle 80 % of the span at k resident blocks (all CUs)
    lo, hi = t[:, 0].min() + 0.1 * (span / us), t[:, 0].min() + 0.9 * (span / us)
    share = {}
    for c in np.unique(ev_c):
        m = ev_c == c
        tt, cc = ev_t[m], conc[m]
        dur = np.clip(np.minimum(np.append(tt[1:], tt[-1]), hi) - np.maximum(tt, lo), 0, None)
        for k in np.unique(cc):
            share[int(k)] = share.get(int(k), 0) + int(dur[cc == k].sum())
    tot = sum(share.values()) or 1
    lines.append("  blocks resident per CU: max over the span p10 %d p50 %d max %d; time share (middle 80 %%): %s" % (
        np.percentile(maxc, 10), np.percentile(maxc, 50), maxc.max(),
        " ".join("%d:%.1f%%" % (k, 100.0 * v / tot) for k, v in sorted(share.items()))))
    # persistent kernels: tile t runs on wave t mod S (S = resident waves); the first S tiles
    # should all start at the launch, a late one means its wave found no free slot
    S = 24 * 256
    if len(t) > 2 * S:
        f0 = (t[:S, 0] - t[:, 0].min()) * us
        lines.append("  start of tiles [0, %d): p50 %.2f us, p90 %.2f, p99 %.2f, max %.2f; after 1 %% of the span: %d" % (
            S, *np.percentile(f0, [50, 90, 99]), f0.max(), int((f0 > 0.01 * span).sum())))
        e = (t[:, 5] - t[:, 0].min()) * us
        lines.append("  last tile end per wave slot: p10 %.1f us, p50 %.1f, min %.1f (span %.1f)" % (
            *np.percentile([e[k::S].max() for k in range(0, S, 7)], [10, 50]), min(e[k::S].max() for k in range(0, S, 7)), span))
    lines.append("  phase-B region bytes per wave mean %.0f, job lanes mean %.1f" % (
        (pb & 0xffffffff).astype(np.float64).mean(), (pb >> 32).astype(np.float64).mean()))
    for ln in lines:
        print(ln, flush=True)
    out[name] = dict(span_us=span, life_us=float(life.mean()), resident=float(res),
                     phases_us={nm: float(ph[:, k].mean()) for k, nm in enumerate(names)},
                     gap_us=float(gap.mean()), block_skew_us=float(idle))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="diag")
    ap.add_argument("--configs", default="c4")
    ap.add_argument("--packets", type=int, default=64 * 2**20)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    import torch
    import bench
    from ab_inproc import load
    from gopacket_amd import _lib, engine, synth
    L = load(a.lib)
    L.gpk_diag_set_buffer.argtypes = [ctypes.c_void_p]
    stream = torch.cuda.current_stream()
    out = {}
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
        b = _lib.Batch(data.data_ptr(), off.data_ptr(), cap.data_ptr(), n, data.numel())
        r = _lib.Results(rec.data_ptr(), err.data_ptr(), fl.data_ptr(), None)
        ctx, p = ctypes.c_void_p(), ctypes.c_void_p()
        assert L.gpk_ctx_create(ctypes.byref(ctx), 0) == 0
        assert L.gpk_parser_create(ctypes.byref(p), 17) == 0
        for dn in cfg["decoders"]:
            assert L.gpk_parser_add_decoder(p, engine.DECODER_KINDS[dn]) == 0
        assert L.gpk_parser_set_outputs(p, cfg["outputs"]) == 0
        waves = (n + 63) // 64
        diag = torch.zeros(waves * 8, dtype=torch.int64, device="cuda")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for k in range(12):
            if k == 11:
                assert L.gpk_diag_set_buffer(ctypes.c_void_p(diag.data_ptr())) == 0
                e0.record(stream)
            assert L.gpk_decode_batch(ctx, p, ctypes.byref(b), ctypes.byref(r), ctypes.c_void_p(stream.cuda_stream)) == 0
        e1.record(stream)
        torch.cuda.synchronize()
        assert L.gpk_diag_set_buffer(None) == 0
        print("%s: launch %.3f ms (HIP events)" % (name, e0.elapsed_time(e1)), flush=True)
        d = diag.view(waves, 8).cpu().numpy().view(np.uint64)
        analyse(name, d, waves, out)
        L.gpk_ctx_destroy(ctx)
        del data, off, cap, rec, err, fl, diag
        torch.cuda.empty_cache()
    if a.json:
        import json
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Soak: the library's long-lived paths run many times in one process, with
host RSS and free device memory checked for growth. 30 replays of a ~2 GiB
C4 pcapng (cycling plain / fields / packets / fields+packets, contexts kept
and re-created), 2000 decode launches over 8 caller streams, 20 contexts
created and destroyed, 30 AF_PACKET pumps over a lapping ring; round 6: 10
byte-range splits of the same file (2-4 ranges each, every range clean and the
packets summing to the file's) and 2000 narrow-record launches; gpk_stop at
random points of replays, byte ranges and pumps (stop_soak: every call
returns, and what was delivered equals an unstopped run's first packets)."""
import gc
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rss_mib():
    for line in open("/proc/self/status"):
        if line.startswith("VmRSS:"):
            return int(line.split()[1]) / 1024
    return -1


def stop_soak(ctx, parser, path, size, n):
    """gpk_stop at random points: SOAK_STOPS replays (whole file or one byte
    range, with and without fields/packets) ended from inside a random batch's
    callback or from a timer thread. Every call must return (no hang), every
    delivered batch must follow the last one (firsts are the running sum), and
    its records and flows must equal the same packets of an unstopped replay;
    the next call on the context runs to the end."""
    import threading
    from gopacket_amd import shard
    rng = np.random.default_rng(int(os.environ.get("SOAK_SEED", "6")))
    full, st = ctx.replay_file(parser, path)
    assert st["packets"] == n
    rec_all, fl_all = full["records"], full["flows"].reshape(3, -1)
    halves = [shard.file_range(size, r, 2) for r in range(2)]
    first_of = {0: 0}  # the first packet of each half (a range's `first` counts from 0), from unstopped replays
    for r, rg in enumerate(halves):
        _, st = ctx.replay_file(parser, path, byte_range=rg, collect=False, on_batch=lambda *a: None)
        assert st["range"]["clean"], st
        first_of[r + 1] = first_of[r] + st["packets"]
    assert first_of[2] == n, first_of
    stops = int(os.environ.get("SOAK_STOPS", "24"))
    counts = {"callback": 0, "thread": 0, "ran to the end": 0}
    for k in range(stops):
        fields, packets = bool(k & 1), bool(k & 2)
        half = int(rng.integers(-1, 2))  # -1: the whole file
        base = first_of[half] if half >= 0 else 0
        at = int(rng.integers(1, 100))
        by_thread = k % 3 == 2
        small = dict(slot_bytes=int(rng.choice([8, 32, 64])) << 20, slots=int(rng.integers(2, 5)),
                     batch_pkts=int(rng.choice([1 << 14, 1 << 16, 1 << 18])))
        seen = []

        def on_batch(first, m, rec, err, fl, ci, cap, *rest):
            g = base + first
            assert not seen or first == seen[-1][0] + seen[-1][1], (first, seen[-1])
            assert np.array_equal(rec, rec_all[g:g + m]), ("records", k, first)
            assert np.array_equal(fl.reshape(3, -1), fl_all[:, g:g + m]), ("flows", k, first)
            seen.append((first, m))
            if not by_thread and len(seen) == at:
                ctx.stop()

        timer = threading.Timer(float(rng.uniform(0.0, 0.25)), ctx.stop) if by_thread else None
        t0 = time.time()
        if timer:
            timer.start()
        _, st = ctx.replay_file(parser, path, byte_range=halves[half] if half >= 0 else None, collect=False,
                                on_batch=on_batch, fields=fields, packets=packets, **small)
        if timer:
            timer.join()
        delivered = sum(m for _, m in seen)
        assert st["packets"] == delivered and (not seen or seen[0][0] == 0), (k, st["packets"], delivered)
        want = first_of[half + 1] - first_of[half] if half >= 0 else n
        if st["stopped"]:
            assert delivered <= want and (by_thread or len(seen) == at), (k, delivered, want, len(seen))
            counts["thread" if by_thread else "callback"] += 1
        else:  # the timer fired after the last batch, or the range had fewer batches than `at`
            assert delivered == want, (k, delivered, want)
            counts["ran to the end"] += 1
        print("  stop %2d: %s, %s, slots %d x %d MiB, batch %d%s%s: %d batches, %d packets%s, %.2f s" % (
            k, "half %d" % half if half >= 0 else "whole file", "thread" if by_thread else "at batch %d" % at,
            small["slots"], small["slot_bytes"] >> 20, small["batch_pkts"],
            ", fields" if fields else "", ", packets" if packets else "", len(seen), delivered,
            " (stopped)" if st["stopped"] else "", time.time() - t0), flush=True)
    _, st = ctx.replay_file(parser, path, collect=False, on_batch=lambda *a: None)
    assert st["packets"] == n and not st["stopped"]
    print("stop soak: %s; the next whole replay delivered all %d packets" % (counts, n), flush=True)


def main():
    import torch
    import bench
    from gopacket_amd import _lib, afpacket, engine, synth
    S = _lib.synth_lib()
    cfg = bench.CONFIGS["c4"]
    kinds = [engine.DECODER_KINDS[d] for d in cfg["decoders"]]
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "gpk_soak_%d.pcapng" % os.getpid())
    n = 5_000_000
    assert S.gpk_synth_write_pcapng(path.encode(), 4, 0, n, 16) > 0
    t0 = time.time()
    marks = []

    def mark(what):
        gc.collect()
        torch.cuda.synchronize()
        free, total = torch.cuda.mem_get_info()
        marks.append((what, rss_mib(), free / 2**20))
        print("%-34s rss %8.1f MiB  device free %10.1f MiB  %5.1f s" % (what, marks[-1][1], marks[-1][2],
                                                                          time.time() - t0), flush=True)

    try:
        ctx = engine.Context(0)
        parser = engine.ParserConfig(17, kinds, outputs=cfg["outputs"])
        mark("start")
        reps = int(os.environ.get("SOAK_REPLAYS", "30"))
        for k in range(reps):
            if k % 10 == 9 and os.environ.get("SOAK_RECREATE", "1") == "1":  # a fresh context now and then
                del ctx
                gc.collect()
                ctx = engine.Context(0)
            fields, packets = bool(k & 1), bool(k & 2)
            cnt = [0]

            def on_batch(first, m, *v):
                cnt[0] += m

            _, st = ctx.replay_file(parser, path, collect=False, on_batch=on_batch, fields=fields, packets=packets)
            assert st["packets"] == n == cnt[0] and st["error"] == "EOF", st
            if k == 0 or k % 10 == 9:
                mark("replay %d" % k)
        from gopacket_amd import shard
        size = os.path.getsize(path)
        for k in range(int(os.environ.get("SOAK_SPLITS", "10"))):  # byte-range replays (gpk_replay_file_range)
            world, got = 2 + k % 3, 0
            for r in range(world):
                cnt = [0]

                def on_batch(first, m, *v):
                    cnt[0] += m

                _, st = ctx.replay_file(parser, path, byte_range=shard.file_range(size, r, world), collect=False,
                                        on_batch=on_batch)
                assert st["range"]["clean"] and not st["range"]["state_changed"] and st["packets"] == cnt[0], st
                got += cnt[0]
            assert got == n, (k, got, n)
        mark("10 byte-range splits")
        stop_soak(ctx, parser, path, size, n)
        mark("stops at random points")
        d, o, c = synth.device_batch(4, 0, 1 << 16)
        streams = [torch.cuda.Stream() for _ in range(8)]
        outs = [(torch.empty(16 << 16, dtype=torch.uint8, device="cuda"), torch.zeros(2 << 16, dtype=torch.int32,
                 device="cuda"), torch.empty(3 << 16, dtype=torch.int64, device="cuda")) for _ in streams]
        for k in range(2000):
            s = streams[k % 8]
            rec, err, fl = outs[k % 8]
            ctx.decode_device(parser, d, o, c, rec, err, fl, stream=s)
        mark("2000 launches on 8 streams")
        r8 = [(torch.empty(8 << 16, dtype=torch.uint8, device="cuda"), torch.zeros(16 << 16, dtype=torch.uint8,
               device="cuda")) for _ in streams]
        for k in range(2000):
            rec, err, fl = outs[k % 8]
            ctx.decode_device_narrow(parser, d, o, c, r8[k % 8][0], r8[k % 8][1], err, fl, stream=streams[k % 8])
        mark("2000 narrow launches on 8 streams")
        for k in range(20):
            x = engine.Context(0)
            p = engine.ParserConfig(17, kinds, outputs=cfg["outputs"])
            x.decode_device(p, d, o, c, *outs[0])
            torch.cuda.synchronize()
            del x, p
        mark("20 contexts")
        bs, nb = 1 << 20, 16
        ring = np.zeros(bs * nb, np.uint8)
        S.gpk_synth_tpacket_v3(ring.ctypes.data, bs, nb, 4, 0, 2, 0, None)
        for k in range(30):
            ring[8::bs] = 1
            tp = afpacket.AttachRing(ring, afpacket.TPacketVersion3, afpacket.OptFrameSize(4096),
                                     afpacket.OptBlockSize(bs), afpacket.OptNumBlocks(nb))
            _, st = tp.Pump(ctx, parser, batch_pkts=1 << 14, collect=False, on_batch=lambda *a: None,
                            fields=bool(k & 1), packets=bool(k & 2))
            tp.Close()
            assert st["packets"] > 0
        mark("30 pumps")
        ring[8::bs] = 1
        tp = afpacket.AttachRing(ring, afpacket.TPacketVersion3, afpacket.OptFrameSize(4096),
                                 afpacket.OptBlockSize(bs), afpacket.OptNumBlocks(nb))
        whole, st = tp.Pump(ctx, parser, batch_pkts=1 << 12)
        tp.Close()
        total, rng = st["packets"], np.random.default_rng(7)
        for k in range(int(os.environ.get("SOAK_PUMP_STOPS", "12"))):  # gpk_stop inside a random batch's callback
            ring[8::bs] = 1
            tp = afpacket.AttachRing(ring, afpacket.TPacketVersion3, afpacket.OptFrameSize(4096),
                                     afpacket.OptBlockSize(bs), afpacket.OptNumBlocks(nb))
            at, seen = int(rng.integers(1, 12)), []

            def on_pump(first, m, rec, *rest):
                assert (first == seen[-1][0] + seen[-1][1]) if seen else first == 0, (first, seen)
                assert np.array_equal(rec, whole["records"][first:first + m]), ("pump records", k, first)
                seen.append((first, m))
                if len(seen) == at:
                    ctx.stop()

            _, st = tp.Pump(ctx, parser, batch_pkts=int(rng.choice([1 << 10, 1 << 12])), inflight=int(rng.integers(1, 4)),
                            collect=False, on_batch=on_pump, fields=bool(k & 1), packets=bool(k & 2))
            tp.Close()
            delivered = sum(m for _, m in seen)
            assert st["packets"] == delivered, (k, st, delivered)
            if len(seen) == at:  # stopped (or the ring held exactly `at` batches)
                assert st["stopped"] or delivered == total, (k, st, delivered, total)
            else:
                assert not st["stopped"] and delivered == total, (k, st, delivered, total)
        print("pump stops: %d pumps stopped at a random batch, delivered prefixes equal an unstopped pump's"
              % int(os.environ.get("SOAK_PUMP_STOPS", "12")), flush=True)
        mark("pump stops")
        rss0, free0 = marks[1][1], marks[1][2]
        print("soak done: rss %+.1f MiB, device free %+.1f MiB since the first replay" % (
            marks[-1][1] - rss0, marks[-1][2] - free0), flush=True)
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()

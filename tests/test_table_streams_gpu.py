"""Two parsers with different next-layer tables used alternately on two HIP
streams with no synchronisation between calls: each launch must see its own
parser's tables (gopacket gives every parser its own state, doc.go:211-228;
port overrides as RegisterTCPPortLayerType / RegisterUDPPortLayerType make
them, ports.go:99-104). Checked bit for bit against the oracle."""
import numpy as np
import pytest

import pktutil
from configs import CONFIGS, device_parser, oracle_parser

pytestmark = pytest.mark.gpu


def test_alternating_parsers_on_two_streams(gpu_ctx):
    import torch
    from gopacket_amd import _lib
    g = pktutil.golden()
    base = [bytes.fromhex(v["hex"]) for k, v in sorted(g.items()) if "hex" in v]
    base += pktutil.read_pcap(pktutil.GOLDEN + "/test_ethernet.pcap")[1]
    base += pktutil.read_pcap(pktutil.GOLDEN + "/test_dns.pcap")[1]
    base += pktutil.fuzz_packets(77, 4000)
    reps = (8 << 20) // len(base) + 1
    n1 = len(base)
    data1, off1, cap1 = pktutil.pack(base)
    # the batch: the unique set tiled `reps` times (oracle decodes the unique set once)
    span = int(off1[-1]) + int(cap1[-1])
    n = n1 * reps
    data = np.zeros(span * reps + 64, np.uint8)
    for r in range(reps):
        data[r * span:(r + 1) * span] = data1[:span]
    off = (np.tile(off1.astype(np.uint64), reps) + np.repeat(np.arange(reps, dtype=np.uint64) * span, n1))
    cap = np.tile(cap1, reps)
    names = ("overrides", "eth_ip4_udp_payload")
    refs = {k: oracle_parser(CONFIGS[k]).decode(data1, off1, cap1, nthreads=8) for k in names}
    assert not np.array_equal(refs[names[0]]["records"], refs[names[1]]["records"])
    parsers = {k: device_parser(CONFIGS[k]) for k in names}
    d = torch.from_numpy(data).cuda()
    o = torch.from_numpy(off.astype(np.int64)).cuda()
    c = torch.from_numpy(cap.astype(np.int32)).cuda()
    streams = {k: torch.cuda.Stream() for k in names}
    outs = []
    torch.cuda.synchronize()
    for it in range(3):
        for k in names:
            with torch.cuda.stream(streams[k]):  # the zero fill is ordered before the launch on its stream
                rec = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
                err = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
                fl = torch.empty(3 * n, dtype=torch.int64, device="cuda")
                gpu_ctx.decode_device(parsers[k], d, o, c, rec, err, fl, stream=streams[k])
            outs.append((k, rec, err, fl))
    torch.cuda.synchronize()
    for k, rec, err, fl in outs:
        ref = refs[k]
        got = rec.cpu().numpy().view(_lib.RECORD_DTYPE)
        assert np.array_equal(got, np.tile(ref["records"], reps)), k
        rf = ref["flows"].reshape(3, n1)
        assert np.array_equal(fl.cpu().numpy().view(np.uint64).reshape(3, n), np.tile(rf, (1, reps))), k
        e = (got["status"] & 0x7F) != 0
        assert np.array_equal(err.cpu().numpy().view(np.uint32).reshape(n, 2)[e],
                              np.tile(ref["err_args"].reshape(n1, 2), (reps, 1))[e]), k


def test_slot_eviction_across_three_streams(gpu_ctx):
    """More parsers than the context keeps table copies (10 > kTabSlots = 8,
    gpk_host.cpp), each with its own port / EtherType overrides, cycled over
    three HIP streams on 8 M-packet batches with no synchronisation between
    the calls: every launch takes a least-recently-used slot whose previous
    readers may still be running on another stream. The rewrite is ordered on
    the device, and each launch must match its own
    parser's oracle bit for bit (ports.go:99-104, doc.go:211-228)."""
    import torch
    from gopacket_amd import _lib
    g = pktutil.golden()
    base = [bytes.fromhex(v["hex"]) for k, v in sorted(g.items()) if "hex" in v]
    base += pktutil.read_pcap(pktutil.GOLDEN + "/test_ethernet.pcap")[1]
    base += pktutil.read_pcap(pktutil.GOLDEN + "/test_dns.pcap")[1]
    base += pktutil.fuzz_packets(91, 3000)
    reps = (8 << 20) // len(base) + 1
    n1 = len(base)
    data1, off1, cap1 = pktutil.pack(base)
    span = int(off1[-1]) + int(cap1[-1])
    n = n1 * reps
    data = np.zeros(span * reps + 64, np.uint8)
    for r in range(reps):
        data[r * span:(r + 1) * span] = data1[:span]
    off = (np.tile(off1.astype(np.uint64), reps) + np.repeat(np.arange(reps, dtype=np.uint64) * span, n1))
    cap = np.tile(cap1, reps)
    cfgs = []
    for i in range(10):
        cfgs.append(dict(first=17, decoders=["ETHERNET", "DOT1Q", "IPV4", "IPV6", "TCP", "UDP", "PAYLOAD"],
                         ethertype={0x88b5 + i: 20}, tcp_port={80: 1200 + i, 1024 + 7 * i: 2},
                         udp_port={53: 2 if i % 2 else 1300 + i, 5353: 1400 + i},
                         ipprotocol={(200 + i) & 255: 44}))
    refs = [oracle_parser(cf).decode(data1, off1, cap1, nthreads=8) for cf in cfgs]
    for i in range(1, 10):
        assert not np.array_equal(refs[0]["err_args"], refs[i]["err_args"]), i
    parsers = [device_parser(cf) for cf in cfgs]
    d = torch.from_numpy(data).cuda()
    o = torch.from_numpy(off.astype(np.int64)).cuda()
    c = torch.from_numpy(cap.astype(np.int32)).cuda()
    streams = [torch.cuda.Stream() for _ in range(3)]
    outs = []
    torch.cuda.synchronize()
    k = 0
    for it in range(2):
        for i in range(10):
            st = streams[k % 3]
            k += 1
            with torch.cuda.stream(st):  # the zero fill is ordered before the launch on its stream
                rec = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
                err = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
                fl = torch.empty(3 * n, dtype=torch.int64, device="cuda")
                gpu_ctx.decode_device(parsers[i], d, o, c, rec, err, fl, stream=st)
            outs.append((i, rec, err, fl))
    torch.cuda.synchronize()
    for i, rec, err, fl in outs:
        ref = refs[i]
        got = rec.cpu().numpy().view(_lib.RECORD_DTYPE)
        assert np.array_equal(got, np.tile(ref["records"], reps)), i
        rf = ref["flows"].reshape(3, n1)
        assert np.array_equal(fl.cpu().numpy().view(np.uint64).reshape(3, n), np.tile(rf, (1, reps))), i
        e = (got["status"] & 0x7F) != 0
        assert np.array_equal(err.cpu().numpy().view(np.uint32).reshape(n, 2)[e],
                              np.tile(ref["err_args"].reshape(n1, 2), (reps, 1))[e]), i


def test_many_caller_streams_one_context(gpu_ctx):
    """More caller streams than the context keeps aggregation streams for
    (40 > kAggStreams = 32, gpk_host.cpp agg_of), three parsers cycled over
    them with no synchronisation, the first stream held behind ~1 s of device
    work: retiring its aggregation stream must not wait for that work (ADVICE
    r04: it held the context lock while it waited), so the 80 launches are
    enqueued in a fraction of the hold; every launch matches its parser's
    oracle."""
    import time
    import torch
    from gopacket_amd import _lib
    base = pktutil.fuzz_packets(93, 3000) + pktutil.read_pcap(pktutil.GOLDEN + "/test_ethernet.pcap")[1]
    data, off, cap = pktutil.pack(base)
    n = len(base)
    names = ("overrides", "eth_ip4_udp_payload", "statsassembly")
    refs = {k: oracle_parser(CONFIGS[k]).decode(data, off, cap, nthreads=8) for k in names}
    parsers = {k: device_parser(CONFIGS[k]) for k in names}
    d = torch.from_numpy(data).cuda()
    o = torch.from_numpy(off.astype(np.int64)).cuda()
    c = torch.from_numpy(cap.astype(np.int32)).cuda()
    streams = [torch.cuda.Stream() for _ in range(40)]
    # calibrate the spin kernel, then hold stream 0 for ~1 s
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(10_000_000)
    e1.record()
    torch.cuda.synchronize()
    cycles = int(10_000_000 * 1000.0 / max(e0.elapsed_time(e1), 1e-3))
    h0, h1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    h0.record(streams[0])
    with torch.cuda.stream(streams[0]):
        torch.cuda._sleep(cycles)
    h1.record(streams[0])
    outs = []
    t0 = time.perf_counter()
    for rnd in range(2):
        for j, st in enumerate(streams):
            k = names[(j + rnd) % 3]
            with torch.cuda.stream(st):
                rec = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
                err = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
                fl = torch.empty(3 * n, dtype=torch.int64, device="cuda")
                gpu_ctx.decode_device(parsers[k], d, o, c, rec, err, fl, stream=st)
            outs.append((k, rec, err, fl))
    enqueue_ms = (time.perf_counter() - t0) * 1e3
    torch.cuda.synchronize()
    hold_ms = h0.elapsed_time(h1)
    assert hold_ms > 300 and enqueue_ms < hold_ms / 2, (enqueue_ms, hold_ms)
    for k, rec, err, fl in outs:
        ref = refs[k]
        assert np.array_equal(rec.cpu().numpy().view(_lib.RECORD_DTYPE), ref["records"]), k
        assert np.array_equal(fl.cpu().numpy().view(np.uint64), ref["flows"]), k

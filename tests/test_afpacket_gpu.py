"""gpk_tpacket_pump (AF_PACKET ring -> HBM mirror -> decode -> results)
against the oracles: the afpacket ring-walk oracle for the packet stream and
CaptureInfo, the decode oracle for every result. Small batches and few
in-flight slots force blocks to be continued across batches, mirror regions
to be reused and deferred headers to be released mid-run.
"""
import numpy as np
import pytest

import pktutil
import ringgen
from configs import CONFIGS, assert_same, device_parser, oracle_parser
from gopacket_amd import _lib, afpacket, synth
from oracle import afpacket_oracle as AO

pytestmark = pytest.mark.gpu


def expect(ring, version, opts):
    orc = AO.TPacketOracle(bytearray(ring), version, dict(opts))
    out, kind, err = orc.read_until_stop()
    return [orc.data(e[0], e[1]) for e in out], out


def check(gpu_ctx, tp, pk, exp, cfg="statsassembly", **kw):
    got, st = tp.Pump(gpu_ctx, device_parser(CONFIGS[cfg]), **kw)
    assert st["packets"] == len(pk), st
    data, off, cap = pktutil.pack(pk)
    ref = oracle_parser(CONFIGS[cfg]).decode(data, off, cap, nthreads=8, layouts=False)
    assert_same(got, ref, "pump")
    assert np.array_equal(got["caplens"], cap)
    ci = got["ci"]
    assert [(int(a), int(b), int(c), int(d), int(e)) for a, b, c, d, e in
            zip(ci["ts_sec"], ci["ts_nsec"], ci["length"], ci["iface"], ci["vlan"])] == \
        [(e[2], e[3], e[4], e[5], e[6]) for e in exp]
    return st


@pytest.mark.parametrize("vlan", [False, True])
@pytest.mark.parametrize("batch,inflight", [(97, 2), (1000, 3), (1 << 20, 4)])
def test_pump_synth_v3_ring(gpu_ctx, vlan, batch, inflight):
    S = _lib.synth_lib()
    bs, nb = 65536, 16
    ring = np.zeros(bs * nb, np.uint8)
    n = S.gpk_synth_tpacket_v3(ring.ctypes.data, bs, nb, synth.C4_IMIX, 1234, 7, 3, None)
    opts = dict(frame_size=4096, block_size=bs, num_blocks=nb, add_vlan_header=vlan)
    pk, exp = expect(ring.tobytes(), AO.V3, opts)
    assert len(pk) == n
    args = [afpacket.OptFrameSize(4096), afpacket.OptBlockSize(bs), afpacket.OptNumBlocks(nb)]
    if vlan:
        args.append(afpacket.OptAddVLANHeader(True))
    tp = afpacket.AttachRing(ring, afpacket.TPacketVersion3, *args)
    st = check(gpu_ctx, tp, pk, exp, batch_pkts=batch, inflight=inflight)
    assert st["ring_bytes_copied"] == bs * nb
    # every block handed back to the kernel at the end
    assert all(int(ring[b * bs + 8]) == 0 for b in range(nb))
    tp.Close()


def test_pump_laps_the_ring_with_a_producer(gpu_ctx):
    """An emulated kernel re-arms each released block: the pump goes round the
    ring several times; packet k is ring packet k mod n."""
    S = _lib.synth_lib()
    bs, nb = 65536, 8
    ring = np.zeros(bs * nb, np.uint8)
    n = int(S.gpk_synth_tpacket_v3(ring.ctypes.data, bs, nb, synth.C3_TCP1500, 0, 7, 0, None))
    opts = dict(frame_size=4096, block_size=bs, num_blocks=nb)
    pk, exp = expect(ring.tobytes(), AO.V3, opts)
    tp = afpacket.AttachRing(ring, afpacket.TPacketVersion3, afpacket.OptFrameSize(4096), afpacket.OptBlockSize(bs),
                             afpacket.OptNumBlocks(nb), afpacket.OptPollTimeout(5_000_000_000))
    prod = S.gpk_synth_tp_producer_start(ring.ctypes.data, bs, nb)
    try:
        laps = 5
        st = check(gpu_ctx, tp, pk * laps, exp * laps, cfg="eth_ip4_tcp_payload", batch_pkts=50, inflight=3,
                   max_packets=n * laps, wait=True)
    finally:
        rearmed = S.gpk_synth_tp_producer_stop(prod)
    assert rearmed >= nb * (laps - 1)
    assert st["ring_bytes_copied"] >= bs * nb * laps
    tp.Close()


@pytest.mark.parametrize("version", [AO.V1, AO.V2])
def test_pump_frame_rings(gpu_ctx, version):
    fz = pktutil.fuzz_packets(21 + version, 64)
    # well-formed C4 packets and fuzzed ones; frame 50 not handed over (the walk stops there)
    pkts = [synth.packet(synth.C4_IMIX, i * 7) if i % 3 else fz[i] for i in range(64)]
    frames = [dict(status=0 if i == 50 else 1, data=p[:1900], tci=(i * 11) & 0xFFF if i % 4 == 0 else 0)
              for i, p in enumerate(pkts)]
    ring = ringgen.frame_ring(version, frames, 2048, 64)
    opts = dict(frame_size=2048, block_size=8192, num_blocks=16, add_vlan_header=True)
    pk, exp = expect(ring, version, opts)
    assert len(pk) == 50
    tp = afpacket.AttachRing(np.frombuffer(ring, np.uint8).copy(), version, afpacket.OptFrameSize(2048),
                             afpacket.OptBlockSize(8192), afpacket.OptNumBlocks(16), afpacket.OptAddVLANHeader(True))
    check(gpu_ctx, tp, pk, exp, batch_pkts=7, inflight=2)
    tp.Close()


def test_pump_stops_at_a_corrupt_chain_and_at_max_packets(gpu_ctx):
    """A block whose chain leaves the ring ends the walk with the fault error
    after the packets before it were delivered; max_packets stops early."""
    import struct
    pk = [synth.packet(synth.C4_IMIX, i) for i in range(30)]
    blocks = [dict(status=1, pkts=[dict(data=p) for p in pk[:10]]),
              dict(status=1, pkts=[dict(data=p) for p in pk[10:20]]),
              dict(status=1, pkts=[dict(data=pk[20], next=1 << 24), dict(data=pk[21])])]
    ring = np.frombuffer(ringgen.v3_ring(blocks, 8192, 4), np.uint8).copy()
    opts = dict(frame_size=4096, block_size=8192, num_blocks=4)
    exp_pk, exp = expect(ring.tobytes(), AO.V3, opts)
    assert len(exp_pk) == 21  # 10 + 10 + the first packet of block 2, then the fault
    tp = afpacket.AttachRing(ring, afpacket.TPacketVersion3, afpacket.OptFrameSize(4096),
                             afpacket.OptBlockSize(8192), afpacket.OptNumBlocks(4))
    got, st = tp.Pump(gpu_ctx, device_parser(CONFIGS["statsassembly"]), batch_pkts=8, inflight=2)
    assert st["packets"] == 21 and st["status"] == _lib.TP_ERROR and "unexpected fault address" in st["error"]
    data, off, cap = pktutil.pack(exp_pk)
    ref = oracle_parser(CONFIGS["statsassembly"]).decode(data, off, cap, layouts=False)
    assert_same(got, ref, "pump before fault")
    tp.Close()
    ring2 = np.frombuffer(ringgen.v3_ring(blocks[:2], 8192, 4), np.uint8).copy()
    tp = afpacket.AttachRing(ring2, afpacket.TPacketVersion3, afpacket.OptFrameSize(4096),
                             afpacket.OptBlockSize(8192), afpacket.OptNumBlocks(4))
    got, st = tp.Pump(gpu_ctx, device_parser(CONFIGS["statsassembly"]), batch_pkts=4, max_packets=13)
    assert st["packets"] == 13 and np.array_equal(got["caplens"], [len(p) for p in pk[:13]])
    # block 0 was finished and handed back; block 1 is still current, so still the reader's
    assert struct.unpack_from("<I", ring2, 8)[0] == 0
    tp.Close()


@pytest.mark.parametrize("vlan,batch", [(False, 1000), (True, 97)])
def test_pump_fields(gpu_ctx, vlan, batch):
    """fields=True: the fused decode + layer fields per batch (the packets with
    an inserted VLAN tag decoded from the side regions); the gpk_fields records
    equal the oracle's extraction over its layouts, and the results are
    unchanged."""
    from oracle import oracle as O
    S = _lib.synth_lib()
    bs, nb = 65536, 16
    ring = np.zeros(bs * nb, np.uint8)
    S.gpk_synth_tpacket_v3(ring.ctypes.data, bs, nb, synth.C4_IMIX, 99, 7, 3, None)
    opts = dict(frame_size=4096, block_size=bs, num_blocks=nb, add_vlan_header=vlan)
    pk, exp = expect(ring.tobytes(), AO.V3, opts)
    args = [afpacket.OptFrameSize(4096), afpacket.OptBlockSize(bs), afpacket.OptNumBlocks(nb)]
    if vlan:
        args.append(afpacket.OptAddVLANHeader(True))
    tp = afpacket.AttachRing(ring, afpacket.TPacketVersion3, *args)
    seen = []
    got, st = tp.Pump(gpu_ctx, device_parser(CONFIGS["statsassembly"]), batch_pkts=batch, inflight=3, fields=True,
                      on_batch=lambda first, n, *v: seen.append((first, n, len(v[-1]))))
    tp.Close()
    assert st["packets"] == len(pk) and all(n == k for _, n, k in seen)
    data, off, cap = pktutil.pack(pk)
    ref = oracle_parser(CONFIGS["statsassembly"]).decode(data, off, cap, nthreads=8, layouts=True)
    assert_same(got, ref, "pump+fields")
    assert np.array_equal(got["fields"].view(np.uint8).reshape(-1, 128), O.extract_fields(data, off, ref["layouts"]))


def test_pump_callback_exception_reaches_the_caller(gpu_ctx):
    """An exception raised in on_batch is raised by Pump once the call returns."""
    S = _lib.synth_lib()
    bs, nb = 65536, 4
    ring = np.zeros(bs * nb, np.uint8)
    S.gpk_synth_tpacket_v3(ring.ctypes.data, bs, nb, synth.C4_IMIX, 3, 7, 0, None)
    tp = afpacket.AttachRing(ring, afpacket.TPacketVersion3, afpacket.OptFrameSize(4096), afpacket.OptBlockSize(bs),
                             afpacket.OptNumBlocks(nb))

    def boom(first, n, *views):
        raise KeyError("consumer")

    calls = []

    def boom_counted(first, n, *views):
        calls.append(first)
        boom(first, n, *views)

    with pytest.raises(KeyError):
        tp.Pump(gpu_ctx, device_parser(CONFIGS["statsassembly"]), batch_pkts=100, collect=False, on_batch=boom_counted)
    assert calls == [0]  # the exception ended the pump (gpk_stop): no further callback
    tp.Close()


def test_pump_stop_from_a_callback(gpu_ctx):
    """ctx.stop() inside the third batch's callback ends the pump: no further
    callback, stats["stopped"], and the delivered packets are the oracle's
    first ones."""
    S = _lib.synth_lib()
    bs, nb = 1 << 20, 4
    ring = np.zeros(bs * nb, np.uint8)
    S.gpk_synth_tpacket_v3(ring.ctypes.data, bs, nb, synth.C4_IMIX, 11, 7, 0, None)
    opts = dict(frame_size=4096, block_size=bs, num_blocks=nb)
    pk, exp = expect(ring.tobytes(), AO.V3, opts)
    tp = afpacket.AttachRing(ring, afpacket.TPacketVersion3, afpacket.OptFrameSize(4096), afpacket.OptBlockSize(bs),
                             afpacket.OptNumBlocks(nb))
    seen = []

    def stop_at_third(first, n, *views):
        seen.append((first, n))
        if len(seen) == 3:
            gpu_ctx.stop()

    got, st = tp.Pump(gpu_ctx, device_parser(CONFIGS["statsassembly"]), batch_pkts=50, inflight=3,
                      on_batch=stop_at_third)
    k = sum(n for _, n in seen)
    assert st["stopped"] and len(seen) == 3 and st["packets"] == k < len(pk)
    assert [f for f, _ in seen] == [0, seen[0][1], seen[0][1] + seen[1][1]]
    data, off, cap = pktutil.pack(pk[:k])
    ref = oracle_parser(CONFIGS["statsassembly"]).decode(data, off, cap, nthreads=8, layouts=False)
    assert_same(got, ref, "pump stopped")
    tp.Close()


@pytest.mark.parametrize("vlan", [False, True])
def test_pump_packets(gpu_ctx, vlan):
    """packets=True: each batch's packets as ZeroCopyReadPacketData returns
    them (ring frames, or the copies with the inserted VLAN header), equal to
    the ring oracle's; the ring laps with an emulated kernel re-arming blocks
    only after their batch was delivered."""
    import ctypes
    S = _lib.synth_lib()
    bs, nb = 65536, 8
    ring = np.zeros(bs * nb, np.uint8)
    n = int(S.gpk_synth_tpacket_v3(ring.ctypes.data, bs, nb, synth.C4_IMIX, 17, 7, 3, None))
    opts = dict(frame_size=4096, block_size=bs, num_blocks=nb, add_vlan_header=vlan)
    pk, exp = expect(ring.tobytes(), AO.V3, opts)
    args = [afpacket.OptFrameSize(4096), afpacket.OptBlockSize(bs), afpacket.OptNumBlocks(nb),
            afpacket.OptPollTimeout(5_000_000_000)]
    if vlan:
        args.append(afpacket.OptAddVLANHeader(True))
    tp = afpacket.AttachRing(ring, afpacket.TPacketVersion3, *args)
    prod = S.gpk_synth_tp_producer_start(ring.ctypes.data, bs, nb)
    got = []
    try:
        laps = 3

        def on_batch(first, k, rec, err, fl, ci, cap, packets):
            ptrs, caps = packets
            assert np.array_equal(caps, cap)
            got.extend(ctypes.string_at(int(p), int(c)) for p, c in zip(ptrs, caps))

        _, st = tp.Pump(gpu_ctx, device_parser(CONFIGS["statsassembly"]), batch_pkts=97, inflight=3,
                        max_packets=n * laps, wait=True, collect=False, on_batch=on_batch, packets=True)
    finally:
        S.gpk_synth_tp_producer_stop(prod)
    tp.Close()
    assert st["packets"] == n * laps and got == pk * laps

"""gpk_replay_file (BASELINE config C5: capture file -> pinned staging -> HBM ->
decode -> results) against the oracles: the pcapgo reader oracle for the
packet stream and CaptureInfo, the decode oracle for every result. Small
staging slots and batches force records across slot boundaries and many
launches per slot.
"""
import gzip
import os

import numpy as np
import pytest

import pcapgen
from configs import CONFIGS, assert_same, device_parser, oracle_parser
from oracle import pcapgo_oracle as PO

pytestmark = pytest.mark.gpu


def packets_and_expect(raw, fmt="ng", **kw):
    res = PO.read_all(raw, kind=fmt, **kw)  # the oracle inflates gzip input itself
    s = res["stream"]
    pk = [bytes(s[p.offset:p.offset + p.caplen]) for p in res["packets"]]
    return res, pk


def check(gpu_ctx, path, raw, cfg_name="statsassembly", fmt="ng", **opts):
    res, pk = packets_and_expect(raw, fmt)
    got, st = gpu_ctx.replay_file(device_parser(CONFIGS[cfg_name]), path, **opts)
    assert st["packets"] == len(pk)
    assert st["error"] == res["err"]
    import pktutil
    data, off, cap = pktutil.pack(pk)
    ref = oracle_parser(CONFIGS[cfg_name]).decode(data, off, cap, nthreads=8, layouts=False)
    assert_same(got, ref, "replay")
    assert np.array_equal(got["caplens"], cap)
    ci = got["ci"]
    assert [(int(a), int(b), int(c), int(d)) for a, b, c, d in zip(ci["ts_sec"], ci["ts_nsec"], ci["length"], ci["iface"])] \
        == [(p.ts_sec, p.ts_nsec, p.length, p.iface) for p in res["packets"]]
    return st


@pytest.fixture(scope="module")
def capture(tmp_path_factory):
    from gopacket_amd import _lib
    d = tmp_path_factory.mktemp("cap")
    path = str(d / "imix.pcapng")
    size = _lib.synth_lib().gpk_synth_write_pcapng(path.encode(), 4, 777, 30000, 4)
    assert size > 0
    return path, open(path, "rb").read()


@pytest.mark.parametrize("slot_bytes,slots,batch", [(4096, 2, 7), (65536, 3, 1000), (1 << 20, 4, 1 << 16), (0, 0, 0)])
def test_replay_imix(gpu_ctx, capture, slot_bytes, slots, batch):
    path, raw = capture
    st = check(gpu_ctx, path, raw, slot_bytes=slot_bytes, slots=slots, batch_pkts=batch)
    assert st["reader_status"] == 0 and st["file_bytes"] == len(raw)


def test_replay_gzip_and_pcap(gpu_ctx, tmp_path, capture):
    _, raw = capture
    gz = gzip.compress(raw[:3_000_000], compresslevel=1)
    p = tmp_path / "imix.pcapng.gz"
    p.write_bytes(gz)
    st = check(gpu_ctx, str(p), gz, slot_bytes=1 << 16, slots=3, batch_pkts=999)
    assert st["error"] == "unexpected EOF"  # the 3 MB cut ends inside a record
    from gopacket_amd import synth
    pk = [synth.packet(4, i) for i in range(5000)]
    pc = pcapgen.pcap_file(pk)
    q = tmp_path / "imix.pcap"
    q.write_bytes(pc)
    check(gpu_ctx, str(q), pc, fmt="pcap", slot_bytes=8192, slots=2, batch_pkts=300)


def test_replay_mixed_blocks(gpu_ctx, tmp_path):
    """SPB/PB/EPB, statistics, name records, a second section in the other byte order."""
    import pktutil
    g = pktutil.golden()
    pk = [bytes.fromhex(v["hex"]) for k, v in sorted(g.items()) if "hex" in v][:40]
    raw = pcapgen.shb() + pcapgen.idb(1, 0) + b"".join(pcapgen.epb(p, ts=i) for i, p in enumerate(pk[:10]))
    raw += pcapgen.nrb([(1, b"\x0a\x00\x00\x01x\x00")]) + b"".join(pcapgen.spb(p) for p in pk[10:20])
    raw += pcapgen.isb(0, 5) + pcapgen.shb(">") + pcapgen.idb(1, 0, ">") + b"".join(
        pcapgen.pb(p, bo=">") for p in pk[20:])
    path = tmp_path / "mixed.pcapng"
    path.write_bytes(raw)
    st = check(gpu_ctx, str(path), raw, slot_bytes=4096, slots=2, batch_pkts=3)
    assert st["error"] == "EOF"


def walk_capture(bo="<"):
    """Plain EPBs over three interfaces with different timestamp resolutions
    (if_tsresol 6, 9 and 2^-10), payloads that hold fake EPB chains at 4-byte
    aligned positions, and a few blocks the device walk must leave to the host
    (an EPB with options, a name record, an interface statistics block)."""
    import struct
    rng = np.random.default_rng(5)
    fake = b"".join(pcapgen.epb(bytes(rng.integers(0, 256, 40, dtype=np.uint8)), bo=bo) for _ in range(5))
    raw = pcapgen.shb(bo) + pcapgen.idb(1, 0, bo) + pcapgen.idb(1, 0, bo, pcapgen.opt(9, b"\x09", bo) + pcapgen.end_opt(bo)) \
        + pcapgen.idb(1, 0, bo, pcapgen.opt(9, b"\x8a", bo) + pcapgen.end_opt(bo))
    from gopacket_amd import synth
    blocks = []
    for i in range(12000):
        p = synth.packet(4, i)
        if i % 97 == 5:
            p = p[:14] + fake + p[14:]  # a plausible block chain inside the packet bytes
        ts = int(rng.integers(0, 1 << 62))
        if i == 4000:
            blocks.append(pcapgen.epb(p, iface=i % 3, ts=ts, bo=bo, options=pcapgen.opt(1, b"note", bo) + pcapgen.end_opt(bo)))
        elif i == 7000:
            blocks.append(pcapgen.nrb([(1, b"\x0a\x00\x00\x01x\x00")], bo=bo))
        elif i == 9000:
            blocks.append(pcapgen.isb(1, ts, bo=bo))
        else:
            blocks.append(pcapgen.epb(p, iface=i % 3, ts=ts, length=len(p) + (i % 5), bo=bo))
    return raw + b"".join(blocks)


@pytest.mark.parametrize("bo", ["<", ">"])
def test_replay_device_walk(gpu_ctx, tmp_path, bo):
    """The device record walk (gpk_walk.hip) against the reader oracle, and the
    same file with the walk kept on the host (GPK_REPLAY_HOST_WALK=1)."""
    raw = walk_capture(bo)
    path = tmp_path / "walk.pcapng"
    path.write_bytes(raw)
    for slot in (1 << 16, 1 << 20):
        st = check(gpu_ctx, str(path), raw, slot_bytes=slot, slots=3, batch_pkts=5000)
        assert st["error"] == "EOF"
        # the host walks only the stretches the device chains did not cover (a
        # fake chain, a block that is not plain, a record across the slot
        # boundary) and hands back to the device walk after each
        assert st["device_walk_packets"] >= 0.9 * st["packets"], (slot, st["device_walk_packets"], st["packets"])
    os.environ["GPK_REPLAY_HOST_WALK"] = "1"
    try:
        check(gpu_ctx, str(path), raw, slot_bytes=1 << 16, slots=3, batch_pkts=5000)
    finally:
        del os.environ["GPK_REPLAY_HOST_WALK"]


def block_starts(raw, bo="<"):
    """Offsets of the pcapng blocks of an intact file (type, total length)."""
    import struct
    out, p = [], 0
    while p + 8 <= len(raw):
        L = struct.unpack_from(bo + "I", raw, p + 4)[0]
        out.append((p, L))
        p += L
    return out


@pytest.mark.parametrize("seed", range(12))
def test_replay_device_walk_corrupt(gpu_ctx, tmp_path, seed):
    """Byte flips in the blocks of a file the device walks: block type, the low
    byte of a block length, interface id, capture length, original length,
    trailer, packet bytes. The device walk must stop at every block that is not
    a plain EPB and leave it to the host reader, which desynchronises or fails
    exactly as Go's reader does (ngread.go:494-580); packets, capture info and
    the reader's error then match the reader oracle. One record longer than
    the staging carry region ends the call with GPK_EUNSUPP by design: the
    flips keep block lengths small, but Go reads options past a short block
    (ngread.go:196-234), so a shrunk capture length can make the following
    megabytes one record's options. Small slots may refuse such a file; the
    default slots must match the oracle."""
    from gopacket_amd import _lib
    bo = ">" if seed >= 8 else "<"  # seeds 8-11: a big-endian section
    raw = bytearray(walk_capture(bo))
    blocks = block_starts(bytes(raw), bo)[4:]  # after the section header and the three interfaces
    rng = np.random.default_rng(1000 + seed)
    for _ in range(int(rng.integers(1, 5))):
        p, L = blocks[int(rng.integers(0, len(blocks)))]
        field = int(rng.integers(0, 7))
        lo = 0 if bo == "<" else 3  # the low byte of a 32-bit field
        pos = [p + lo, p + 4 + lo, p + 8 + lo, p + 20 + lo, p + 24 + lo, p + L - 4 + lo,
               p + 28 + int(rng.integers(0, max(1, L - 32)))][field]
        raw[pos] ^= int(rng.integers(1, 256)) if field != 1 else int(rng.integers(1, 256)) & 0xFC | 4
    path = tmp_path / "corrupt.pcapng"
    path.write_bytes(bytes(raw))
    for slot in (1 << 16, 1 << 20, 0):
        try:
            st = check(gpu_ctx, str(path), bytes(raw), slot_bytes=slot, slots=3 if slot else 0,
                       batch_pkts=5000 if slot else 0)
        except _lib.GpkError as e:
            assert slot and "carry region" in str(e), (slot, str(e))
            continue
        assert st["packets"] > 0


@pytest.mark.parametrize("seed", range(8))
def test_replay_pcap_corrupt(gpu_ctx, tmp_path, seed):
    """Classic pcap with byte flips in record headers (timestamps, capture
    length, original length), both byte orders, micro- and nanosecond files:
    Reader.ReadPacketData's checks (read.go:122-177: capture length over the
    snap length or over the original length) end the stream where Go's do,
    and every packet before matches the reader and decode oracles."""
    import struct
    from gopacket_amd import synth
    pk = [synth.packet(4, i) for i in range(6000)]
    bo = ">" if seed % 2 else "<"
    raw = bytearray(pcapgen.pcap_file(pk, bo=bo, nano=seed % 4 >= 2, snaplen=2000))
    starts, p = [], 24
    while p + 16 <= len(raw):
        starts.append(p)
        p += 16 + struct.unpack_from(bo + "I", raw, p + 8)[0]
    rng = np.random.default_rng(2000 + seed)
    for _ in range(int(rng.integers(1, 4))):
        p = starts[int(rng.integers(0, len(starts)))]
        raw[p + 4 * int(rng.integers(0, 4)) + (0 if bo == "<" else 3)] ^= int(rng.integers(1, 256))
    path = tmp_path / "corrupt.pcap"
    path.write_bytes(bytes(raw))
    for slot, slots, batch in ((8192, 2, 300), (0, 0, 0)):
        check(gpu_ctx, str(path), bytes(raw), fmt="pcap", slot_bytes=slot, slots=slots, batch_pkts=batch)


def test_replay_small_records_grow_device_index(gpu_ctx, tmp_path):
    """Simple Packet Blocks of 16 bytes (zero-length packets, ngread.go:515-530)
    are walked by the host reader and appended to the slot's device index,
    which was sized for the device walk's >= 32-byte blocks: a slot full of
    them must grow the index, both after device-walked EPBs (the
    walked entries are kept) and on their own."""
    from gopacket_amd import synth
    raw = pcapgen.shb() + pcapgen.idb(1, 0)
    for r in range(4):
        raw += b"".join(pcapgen.epb(synth.packet(4, 100 * r + i)[:60], ts=i) for i in range(40))
        raw += b"".join(pcapgen.spb(b"") for _ in range(1500))
        raw += b"".join(pcapgen.spb(synth.packet(4, i)[:20]) for i in range(300))
    path = tmp_path / "spb.pcapng"
    path.write_bytes(raw)
    for slot in (4096, 1 << 14):
        st = check(gpu_ctx, str(path), raw, slot_bytes=slot, slots=2, batch_pkts=777)
        assert st["error"] == "EOF"


def test_replay_kernel_choice(gpu_ctx, tmp_path):
    """The readable end a replay batch passes is measured from the base the
    kernels get (the batch span understated it and the
    dword-aligned small-packet window was never used): with the C1 parser
    (no IPv6 decoder) and small packets the launch is the AL = 4 kernel, on
    the device walk and on the host walk; packets still match the oracle."""
    from gopacket_amd import synth
    pk = [synth.packet(2, i) for i in range(20000)]
    raw = pcapgen.ng_file(pk)
    path = tmp_path / "small.pcapng"
    path.write_bytes(raw)
    for host_walk in (False, True):
        if host_walk:
            os.environ["GPK_REPLAY_HOST_WALK"] = "1"
        try:
            st = check(gpu_ctx, str(path), raw, cfg_name="eth_ip4_tcp_payload", slot_bytes=1 << 20, slots=2, batch_pkts=4096)
        finally:
            os.environ.pop("GPK_REPLAY_HOST_WALK", None)
        assert st["kernel"].endswith(",5,7,4>"), (host_walk, st["kernel"])


def test_replay_device_walk_resumes(gpu_ctx, tmp_path):
    """Blocks longer than a walk segment (16-64 KiB packets), blocks the device
    walk leaves to the host (an EPB with options, a name record) and a new
    interface mid-slot (the reader's walk state changes: the host takes the
    rest of that slot, the next slot walks with the new interface table): the
    device walk resumes after each host stretch where the reader's state
    allows, and every packet matches the reader and decode oracles."""
    from gopacket_amd import synth
    rng = np.random.default_rng(11)
    raw = pcapgen.shb() + pcapgen.idb(1, 0)
    n_big = 0
    for i in range(30000):
        p = synth.packet(4, i)
        if i % 2500 == 17:
            p = p + bytes(rng.integers(0, 256, int(rng.integers(16, 64)) << 10, dtype=np.uint8))
            n_big += 1
        if i == 12345:
            raw += pcapgen.epb(p, ts=i, options=pcapgen.opt(1, b"note") + pcapgen.end_opt())
        elif i == 20000:
            raw += pcapgen.nrb([(1, b"\x0a\x00\x00\x01x\x00")])
        elif i == 25000:
            raw += pcapgen.idb(1, 0)
        else:
            raw += pcapgen.epb(p, iface=1 if i > 25000 and i % 2 else 0, ts=i)
    path = tmp_path / "resume.pcapng"
    path.write_bytes(raw)
    st = check(gpu_ctx, str(path), raw, slot_bytes=1 << 20, slots=3, batch_pkts=4096)
    assert st["error"] == "EOF"
    assert n_big >= 10
    assert st["device_walk_packets"] >= 0.9 * st["packets"], (st["device_walk_packets"], st["packets"])


@pytest.mark.parametrize("cfg_name,slot_bytes,slots,batch", [("statsassembly", 65536, 3, 1000),
                                                             ("statsassembly", 0, 0, 0), ("fragment_no_payload", 1 << 20, 2, 4097)])
def test_replay_fields(gpu_ctx, capture, cfg_name, slot_bytes, slots, batch):
    """fields=True: every launch is the fused decode + layer fields; the
    gpk_fields records reach the host through fields_cb (called before the
    batch's results callback) and equal the oracle's field extraction over the
    oracle's layouts, packet for packet; the decode results are unchanged."""
    from oracle import oracle as O
    import pktutil
    path, raw = capture
    res, pk = packets_and_expect(raw)
    seen = []

    def on_batch(first, n, rec, err, fl, ci, cap, fields):
        assert len(fields) == n
        seen.append((first, n))

    got, st = gpu_ctx.replay_file(device_parser(CONFIGS[cfg_name]), path, slot_bytes=slot_bytes, slots=slots,
                                  batch_pkts=batch, fields=True, on_batch=on_batch)
    assert st["packets"] == len(pk) and st["error"] == res["err"]
    assert sum(n for _, n in seen) == len(pk)
    assert [f for f, _ in seen] == sorted(f for f, _ in seen)
    data, off, cap = pktutil.pack(pk)
    ref = oracle_parser(CONFIGS[cfg_name]).decode(data, off, cap, nthreads=8, layouts=True)
    assert_same(got, ref, "replay+fields")
    want = O.extract_fields(data, off, ref["layouts"])
    assert np.array_equal(got["fields"].view(np.uint8).reshape(-1, 128), want)


def test_replay_callback_exception_reaches_the_caller(gpu_ctx, capture):
    """An exception raised in on_batch (inside the ctypes callback) is raised
    by replay_file once the call returns, and the context stays usable."""
    path, raw = capture

    def boom(first, n, *views):
        raise ValueError("consumer failed at packet %d" % first)

    calls = []

    def boom_counted(first, n, *views):
        calls.append(first)
        boom(first, n, *views)

    with pytest.raises(ValueError, match="consumer failed at packet 0"):
        gpu_ctx.replay_file(device_parser(CONFIGS["statsassembly"]), path, collect=False, on_batch=boom_counted,
                            slot_bytes=1 << 20, slots=2, batch_pkts=5000)
    assert calls == [0]  # the exception ended the call (gpk_stop): no further callback
    check(gpu_ctx, path, raw, slot_bytes=1 << 20, slots=2, batch_pkts=5000)


@pytest.mark.parametrize("packets", [False, True])
def test_replay_stop_from_a_callback(gpu_ctx, capture, packets):
    """ctx.stop() (gpk_stop) inside the second batch's callback: a Go caller's
    break out of its ReadPacketData loop. No further callback, GPK_STOPPED
    (stats["stopped"]), stats["packets"] = the packets delivered, and those
    results are the whole-file replay's first packets; the next call on the
    context runs to the end."""
    path, raw = capture
    res, pk = packets_and_expect(raw)
    firsts = []

    def stop_at_second(first, n, rec, err, fl, ci, cap, *rest):
        firsts.append((first, n))
        if len(firsts) == 2:
            gpu_ctx.stop()

    got, st = gpu_ctx.replay_file(device_parser(CONFIGS["statsassembly"]), path, collect=not packets,
                                  on_batch=stop_at_second, packets=packets, slot_bytes=1 << 18, slots=3,
                                  batch_pkts=700)
    k = sum(n for _, n in firsts)  # (a launch holds at most 700 packets, fewer at a staging slot's end)
    assert st["stopped"] and len(firsts) == 2 and firsts[1][0] == firsts[0][1] and st["packets"] == k
    full, st2 = gpu_ctx.replay_file(device_parser(CONFIGS["statsassembly"]), path, slot_bytes=1 << 18, slots=3,
                                    batch_pkts=700)
    assert not st2["stopped"] and st2["packets"] == len(pk)
    if not packets:
        for key in ("records", "ci", "caplens"):
            assert np.array_equal(got[key], full[key][:k]), key
        assert np.array_equal(got["err_args"], full["err_args"][:2 * k])
        assert np.array_equal(got["flows"].reshape(3, -1), full["flows"].reshape(3, -1)[:, :k])


def test_replay_stop_from_another_thread(gpu_ctx, capture):
    """gpk_stop from a thread other than the replay's: the replay ends early
    with every delivered batch whole."""
    import threading
    import time
    path, raw = capture
    started, seen = threading.Event(), []

    def slow(first, n, *views):
        seen.append((first, n))
        started.set()
        time.sleep(0.02)

    out = {}
    t = threading.Thread(target=lambda: out.update(r=gpu_ctx.replay_file(
        device_parser(CONFIGS["statsassembly"]), path, collect=False, on_batch=slow, slot_bytes=1 << 18, slots=3,
        batch_pkts=300)))
    t.start()
    assert started.wait(60)
    gpu_ctx.stop()
    t.join(120)
    assert not t.is_alive()
    _, st = out["r"]
    total = len(packets_and_expect(raw)[1])
    assert st["stopped"] and st["packets"] == sum(n for _, n in seen) < total
    assert [f for f, _ in seen] == list(np.cumsum([0] + [n for _, n in seen])[:-1])


def test_replay_packets_and_hydrate(gpu_ctx, capture):
    """packets=True: every launch's packet bytes as views of the staging
    buffers (gpk_replay_opts.packets_cb), delivered with the fields and the
    results; small slots force the slots to be refilled, which must wait for
    their packets to be handed out. Every packet's bytes equal the reader
    oracle's, and layer structs hydrated from the fields record over those
    bytes equal a host-side decode's of the same packets."""
    import hydrate_cases as H
    from gopacket_amd import gopacket as G
    path, raw = capture
    res, pk = packets_and_expect(raw)
    seen = []
    pf, pr = H.parser(), H.parser()
    pf._ctx = pr._ctx = gpu_ctx

    def on_batch(first, n, rec, err, fl, ci, cap, fields, packets):
        data, off, caps = packets
        assert np.array_equal(caps, cap)
        for i in range(n):
            assert bytes(data[off[i]:off[i] + caps[i]]) == pk[first + i], first + i
        k = min(n, 300)
        rb = G.BatchResult(pf, G.PacketBatch(data, off, caps),
                           dict(records=rec.copy(), err_args=err.copy(), flows=fl.copy(), layouts=None))
        rb.fields = fields.copy()
        ra = pr.DecodeBatch(G.PacketBatch.from_packets(pk[first:first + k]), layouts=True)
        H.compare(ra, rb, pr, pf, range(k))
        seen.append(n)

    _, st = gpu_ctx.replay_file(device_parser(CONFIGS["statsassembly"]), path, slot_bytes=1 << 20, slots=2,
                                batch_pkts=4000, collect=False, on_batch=on_batch, fields=True, packets=True)
    assert st["packets"] == len(pk) == sum(seen)
    with pytest.raises(ValueError):
        gpu_ctx.replay_file(device_parser(CONFIGS["statsassembly"]), path, packets=True)


def test_replay_device_walk_holds_no_heap(gpu_ctx, tmp_path):
    """Every staging slot's tail goes through the host reader after the device
    walk; its index, empty or not, is freed (an empty one leaked ~1.8 MB per
    slot before round 6's fix). 12 replays of ~50 slots each must leave glibc's
    heap in use where it was (mallinfo2), within a few MB."""
    import ctypes
    from gopacket_amd import _lib

    class MallInfo2(ctypes.Structure):
        _fields_ = [(f, ctypes.c_size_t) for f in ("arena", "ordblks", "smblks", "hblks", "hblkhd", "usmblks",
                                                    "fsmblks", "uordblks", "fordblks", "keepcost")]

    libc = ctypes.CDLL("libc.so.6")
    if not hasattr(libc, "mallinfo2"):
        pytest.skip("glibc without mallinfo2")
    libc.mallinfo2.restype = MallInfo2
    path = str(tmp_path / "c4.pcapng")
    n = 500_000
    assert _lib.synth_lib().gpk_synth_write_pcapng(path.encode(), 4, 0, n, 8) > 0
    parser = device_parser(CONFIGS["statsassembly"])
    shape = dict(slot_bytes=4 << 20, slots=3, batch_pkts=1 << 16)

    def run():
        _, st = gpu_ctx.replay_file(parser, path, collect=False, on_batch=lambda *a: None, **shape)
        assert st["packets"] == n and st["error"] == "EOF" and st["device_walk_packets"] > 0, st
        return st["slots"]

    run()
    h0 = libc.mallinfo2().uordblks
    slots = sum(run() for _ in range(12))
    grown = (libc.mallinfo2().uordblks - h0) / 2**20
    assert slots >= 400 and grown < 16, (slots, grown)

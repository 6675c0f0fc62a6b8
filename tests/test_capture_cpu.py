"""Native capture indexer (libgpk gpk_capreader_*, host code, no GPU) against the
pcapgo oracle (oracle/pcapgo_oracle.py, pinned by tests/test_pcapgo_oracle.py).

Bit-exact on every packet (stream offset, caplen, CaptureInfo), the error
that ends the stream (Go text and panic flag) and the section/interface
metadata; fed whole and in chunks of many sizes (the resumable walk must not
depend on where a chunk ends); on the reference's fixtures, on generated
edge-case captures and on mutated (fuzzed) captures.
"""
import ctypes
import gzip
import os
import random
import struct

import numpy as np
import pytest

import pcapgen
from gopacket_amd import _lib, pcapgo
from oracle import pcapgo_oracle as PO

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "pcapgo")
FILES = sorted([os.path.join(be, f) for be in ("le", "be") for f in os.listdir(os.path.join(GOLD, be))]) + ["epb.pcapng"]
FLAG_SETS = [0, 1, 2, 4, 6, 7]


def tlv_options(tlv):
    """gpk_capreader_packet_options records -> [(code, value)]."""
    out, p = [], 0
    while p < len(tlv):
        code, n = struct.unpack_from("<H2xI", tlv, p)
        out.append((code, bytes(tlv[p + 8:p + 8 + n])))
        p += 8 + ((n + 3) & ~3)
    return out


def native_events(stream, fmt, flags, chunk=None, max_pkts=1 << 30, errors=1, max_events=100000):
    """Drive gpk_capreader_index like a ReadPacketDataWithOptions loop; returns events:
    ("pkt", abs_offset, caplen, ts_sec, ts_nsec, length, iface, ancil, options) or ("err", text, panic)."""
    L = _lib.lib()
    h = ctypes.c_void_p()
    _lib.check(L.gpk_capreader_create(ctypes.byref(h), fmt, flags))
    _lib.check(L.gpk_capreader_keep_options(h, 1))
    ev = []
    base, have = 0, (len(stream) if chunk is None else min(len(stream), chunk))
    nerr = 0
    try:
        while len(ev) < max_events:
            buf = np.frombuffer(stream[base:have], np.uint8) if have > base else np.zeros(1, np.uint8)
            m = max(1, min(max_pkts, 4096))
            off = np.empty(m, np.uint64)
            cap = np.empty(m, np.uint32)
            ci = np.empty(m, _lib.CAPINFO_DTYPE)
            n, used = ctypes.c_uint64(), ctypes.c_uint64()
            eof = have >= len(stream)
            rc = L.gpk_capreader_index(h, buf.ctypes.data, have - base, int(eof), off.ctypes.data, cap.ctypes.data,
                                       ci.ctypes.data, m, ctypes.byref(n), ctypes.byref(used))
            assert rc >= 0, rc
            for i in range(n.value):
                r = ci[i]
                assert int(off[i]) + int(cap[i]) <= used.value
                tlv, nb = ctypes.c_void_p(), ctypes.c_uint64()
                _lib.check(L.gpk_capreader_packet_options(h, i, ctypes.byref(tlv), ctypes.byref(nb)))
                ev.append(("pkt", base + int(off[i]), int(cap[i]), int(r["ts_sec"]), int(r["ts_nsec"]),
                           int(r["length"]), int(r["iface"]), None if int(r["link_type"]) < 0 else int(r["link_type"]),
                           tlv_options(ctypes.string_at(tlv, nb.value) if nb.value else b"")))
            base += used.value
            if rc == _lib.CAP_END:
                b = ctypes.create_string_buffer(512)
                e, p = ctypes.c_int(), ctypes.c_int()
                k = L.gpk_capreader_error(h, b, 512, ctypes.byref(e), ctypes.byref(p))
                ev.append(("err", b.raw[:k].decode("latin-1"), bool(p.value)))
                nerr += 1
                if bool(e.value) or nerr >= errors:
                    break
            elif rc == _lib.CAP_MORE:
                assert not eof
                have = len(stream) if chunk is None else min(len(stream), have + chunk)
        meta = native_meta(L, h, fmt)
    finally:
        L.gpk_capreader_destroy(h)
    return ev, meta


def native_meta(L, h, fmt):
    if fmt != _lib.CAP_PCAPNG:
        return None

    def s(fn, *a):
        n = fn(h, *a, None, 0)
        if n < 0:
            return None
        b = ctypes.create_string_buffer(n + 1)
        fn(h, *a, b, n + 1)
        return b.raw[:n]

    out = []
    for sec in range(L.gpk_capreader_nsections(h) + 1):
        info = dict(comment=s(L.gpk_capreader_section_info, sec, 0), hardware=s(L.gpk_capreader_section_info, sec, 1),
                    os=s(L.gpk_capreader_section_info, sec, 2), application=s(L.gpk_capreader_section_info, sec, 3))
        ifs = []
        for i in range(L.gpk_capreader_ninterfaces(h, sec)):
            x = _lib.NgInterface()
            assert L.gpk_capreader_interface(h, sec, i, ctypes.byref(x)) == 0
            f = L.gpk_capreader_interface_str
            ifs.append(dict(name=s(f, sec, i, 0), comment=s(f, sec, i, 1), description=s(f, sec, i, 2),
                            filter=s(f, sec, i, 3), os=s(f, sec, i, 4), link_type=x.link_type,
                            ts_resolution=x.ts_resolution, ts_offset=x.ts_offset, snap_length=x.snap_length,
                            stats=dict(last_update=(x.last_update_sec, x.last_update_nsec),
                                       start_time=(x.start_time_sec, x.start_time_nsec),
                                       end_time=(x.end_time_sec, x.end_time_nsec), comment=s(f, sec, i, 5),
                                       received=x.packets_received, dropped=x.packets_dropped)))
        out.append((info, ifs))
    return dict(sections=out, **native_reader_state(L, h))


def native_reader_state(L, h):
    """Name records, StatisticsCallback and SectionEndCallback calls."""
    names = []
    for i in range(L.gpk_capreader_nnames(h)):
        kind, alen, nn = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        addr = (ctypes.c_uint8 * 24)()
        need = L.gpk_capreader_name(h, i, ctypes.byref(kind), addr, ctypes.byref(alen), ctypes.byref(nn), None, 0)
        b = ctypes.create_string_buffer(max(need, 1))
        assert L.gpk_capreader_name(h, i, None, None, None, None, b, need) == need
        names.append((kind.value, bytes(addr)[:alen.value], b.raw[:need].split(b"\x00")[:nn.value]))
    stats = []
    for k in range(L.gpk_capreader_nstat_events(h)):
        at, seq, iface, x = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int(), _lib.NgInterface()
        n = L.gpk_capreader_stat_event(h, k, ctypes.byref(at), ctypes.byref(seq), ctypes.byref(iface), ctypes.byref(x),
                                       None, 0)
        b = ctypes.create_string_buffer(n + 1)
        L.gpk_capreader_stat_event(h, k, None, None, None, None, b, n + 1)
        stats.append((at.value, seq.value, iface.value,
                      dict(last_update=(x.last_update_sec, x.last_update_nsec),
                           start_time=(x.start_time_sec, x.start_time_nsec), end_time=(x.end_time_sec, x.end_time_nsec),
                           comment=b.raw[:n], received=x.packets_received, dropped=x.packets_dropped)))
    ends = []
    for sec in range(L.gpk_capreader_nsections(h)):
        at, seq = ctypes.c_uint64(), ctypes.c_uint64()
        _lib.check(L.gpk_capreader_section_end_at(h, sec, ctypes.byref(at), ctypes.byref(seq)))
        ends.append((at.value, seq.value))
    return dict(names=names, stat_events=stats, section_ends=ends)


def oracle_events(stream, fmt, flags, errors=1, max_events=100000):
    kw = dict(want_mixed=bool(flags & 1), error_on_mismatch=bool(flags & 2), skip_unknown_version=bool(flags & 4))
    try:
        r = PO.NgReader(stream, **kw) if fmt == _lib.CAP_PCAPNG else PO.Reader(stream)
    except PO.GoError as e:
        return [("err", e.text, e.panic)], "open"
    ev = []
    nerr = 0
    while len(ev) < max_events:
        try:
            p = r.read_packet()
            ev.append(("pkt",) + p.key() + (list(p.opts),))
        except PO.GoError as e:
            ev.append(("err", e.text, e.panic))
            nerr += 1
            if e.text == "EOF" or nerr >= errors:
                break
    meta = None
    if fmt == _lib.CAP_PCAPNG:
        meta = oracle_meta(r)
    return ev, meta


def oracle_meta(r):
    return dict(sections=list(r.ended_sections) + [r.section_state()], **oracle_reader_state(r))


def oracle_reader_state(r):
    return dict(names=[(t, a, list(n)) for t, a, n in r.names], stat_events=list(r.stat_events),
                section_ends=list(r.ended_at))


def compare(stream, fmt, flags, chunk=None, errors=1):
    want, wmeta = oracle_events(stream, fmt, flags, errors=errors)
    if wmeta == "open":  # NewReader failed: there is no reader to call again
        errors = 1
    got, gmeta = native_events(stream, fmt, flags, chunk=chunk, errors=errors)
    assert got == want
    if wmeta != "open" and fmt == _lib.CAP_PCAPNG:
        assert gmeta == wmeta
    return want


@pytest.mark.parametrize("f", FILES)
@pytest.mark.parametrize("flags", FLAG_SETS)
def test_fixtures_match_oracle(f, flags):
    data = open(os.path.join(GOLD, f), "rb").read()
    ev = compare(data, _lib.CAP_PCAPNG, flags)
    assert ev[-1][0] == "err"
    for chunk in (1, 13, 64, 333, 4096):
        if len(data) // chunk > 3000:
            continue
        compare(data, _lib.CAP_PCAPNG, flags, chunk=chunk)


def test_errors_can_be_read_past():
    """After an error, the next ReadPacketData continues from where Go's reader stands."""
    for f in ("le/test006.pcapng", "be/test006.pcapng", "le/test901.pcapng"):
        data = open(os.path.join(GOLD, f), "rb").read()
        for flags in (2, 0):
            compare(data, _lib.CAP_PCAPNG, flags, errors=5)


def edge_captures():
    bo_cases = []
    for bo in ("<", ">"):
        shb = pcapgen.shb(bo, options=pcapgen.opt(1, b"c", bo) + pcapgen.opt(2, b"hw", bo) + pcapgen.end_opt(bo))
        idb = pcapgen.idb(1, 0, bo, options=pcapgen.opt(2, b"eth0", bo) + pcapgen.opt(9, b"\x89", bo) +
                          pcapgen.opt(14, (5).to_bytes(8, "big" if bo == ">" else "little"), bo) + pcapgen.end_opt(bo))
        pk = [bytes(range(i % 256)) * 3 for i in range(20)]
        bo_cases += [
            shb + idb + b"".join(pcapgen.epb(p, ts=i * 7777777, bo=bo) for i, p in enumerate(pk)),
            shb + idb + b"".join(pcapgen.spb(p, bo=bo) for p in pk),
            shb + idb + b"".join(pcapgen.pb(p, ts=i, bo=bo) for i, p in enumerate(pk)),
            # name resolution + decryption secrets + statistics between packets
            shb + pcapgen.nrb([(1, b"\x0a\x00\x00\x01host\x00"), (3, b"\x01\x02\x03\x04\x05\x06mac\x00"),
                               (9, b"xyz")], bo) + pcapgen.dsb(0x544c534b, b"secret", bo) + idb +
            pcapgen.epb(pk[5], bo=bo) + pcapgen.isb(0, 99, bo, options=pcapgen.opt(4, (3).to_bytes(8, "little"), bo) +
                                                  pcapgen.end_opt(bo)) + pcapgen.epb(pk[6], bo=bo),
            # EPB options, including ones the reference panics on
            shb + idb + pcapgen.epb(pk[7], bo=bo, options=pcapgen.opt(2, b"\x01\x00\x00\x00", bo) + pcapgen.end_opt(bo)),
            shb + idb + pcapgen.epb(pk[7], bo=bo, options=pcapgen.opt(2, b"\x01", bo) + pcapgen.end_opt(bo)),
            shb + idb + pcapgen.epb(pk[7], bo=bo, options=pcapgen.opt(4, b"\x01\x02", bo) + pcapgen.end_opt(bo)),
            # second section with another byte order, an unknown block, a bad interface id
            shb + idb + pcapgen.epb(pk[3], bo=bo) + pcapgen.shb(">" if bo == "<" else "<") +
            pcapgen.idb(0, 0, ">" if bo == "<" else "<") + pcapgen.block(0x777, b"abcd", bo) +
            pcapgen.epb(pk[4], bo=">" if bo == "<" else "<"),
            shb + idb + pcapgen.epb(pk[3], iface=3, bo=bo),
            # resolution exponent 64: the reference panics (divide by zero)
            shb + pcapgen.idb(1, 0, bo, options=pcapgen.opt(9, b"\x40", bo) + pcapgen.end_opt(bo)),
            shb + pcapgen.idb(1, 0, bo, options=pcapgen.opt(9, b"\x86", bo) + pcapgen.end_opt(bo)) +
            pcapgen.epb(pk[9], ts=(1 << 40) + 12345, bo=bo),
            # zero-length options keep the previous option value
            shb + pcapgen.idb(1, 0, bo, options=pcapgen.opt(2, b"name", bo) + pcapgen.opt(1, b"", bo) +
                              pcapgen.end_opt(bo)) + pcapgen.epb(pk[2], bo=bo),
            # packet blocks before any interface, version mismatch
            shb + pcapgen.epb(pk[2], bo=bo),
            pcapgen.shb(bo, major=2) + idb + pcapgen.epb(pk[2], bo=bo) + shb + idb + pcapgen.epb(pk[3], bo=bo),
        ]
    return bo_cases


@pytest.mark.parametrize("k", range(len(edge_captures())))
def test_edge_captures(k):
    data = edge_captures()[k]
    for flags in FLAG_SETS:
        compare(data, _lib.CAP_PCAPNG, flags)
        compare(data, _lib.CAP_PCAPNG, flags, chunk=17)
        compare(data, _lib.CAP_PCAPNG, flags, errors=4)


def mutate(rng, data):
    d = bytearray(data)
    kind = rng.randrange(4)
    if kind == 0:  # flip bytes
        for _ in range(rng.randrange(1, 4)):
            i = rng.randrange(len(d))
            d[i] = rng.randrange(256)
    elif kind == 1:  # truncate
        d = d[:rng.randrange(len(d) + 1)]
    elif kind == 2:  # small length-field perturbation
        i = rng.randrange(0, max(1, len(d) - 4)) & ~3
        d[i] = (d[i] + rng.choice((1, 3, 4, 252, 255))) & 0xFF
    else:  # splice a random slice elsewhere
        a = rng.randrange(len(d))
        b = min(len(d), a + rng.randrange(1, 64))
        j = rng.randrange(len(d))
        d = d[:j] + d[a:b] + d[j:]
    return bytes(d)


def test_fuzz_pcapng_matches_oracle():
    rng = random.Random(1234)
    seeds = [open(os.path.join(GOLD, f), "rb").read() for f in FILES if os.path.getsize(os.path.join(GOLD, f)) < 3000]
    seeds += [e for e in edge_captures()]
    for it in range(1500):
        data = mutate(rng, rng.choice(seeds))
        flags = rng.choice(FLAG_SETS)
        compare(data, _lib.CAP_PCAPNG, flags, errors=3)
        if it % 10 == 0:
            compare(data, _lib.CAP_PCAPNG, flags, chunk=rng.randrange(1, 200), errors=3)


def pcap_cases():
    pk = [bytes([i]) * (i * 5 % 97) for i in range(30)]
    out = []
    for bo in ("<", ">"):
        for nano in (False, True):
            out.append(pcapgen.pcap_file(pk, bo=bo, nano=nano))
        out.append(pcapgen.pcap_file(pk, bo=bo, snaplen=50))  # "capture length exceeds snap length"
    return out


def test_pcap_matches_oracle():
    rng = random.Random(99)
    cases = pcap_cases()
    for c in cases:
        for chunk in (None, 1, 7, 100):
            compare(c, _lib.CAP_PCAP, 0, chunk=chunk, errors=6)
    for _ in range(800):
        data = mutate(rng, rng.choice(cases))
        compare(data, _lib.CAP_PCAP, 0, errors=4)
    # usec * 1000 wraps in uint32 (read.go:173): usec = 4294968 -> 4294968000 mod 2^32
    hdr = pcapgen.pcap_file([])
    rec = (5).to_bytes(4, "little") + (4294968).to_bytes(4, "little") + (2).to_bytes(4, "little") * 2 + b"ab"
    ev = compare(hdr + rec, _lib.CAP_PCAP, 0)
    assert ev[0][3:5] == (5, (4294968000 - (1 << 32)))


def test_python_mirror_reads_like_pcapgo():
    """gopacket_amd.pcapgo on the harvested test table (the same checks as ngRunFileReadTest)."""
    import json
    exp = json.load(open(os.path.join(GOLD, "expect.json")))
    from test_pcapgo_oracle import b, want_iface
    for t in exp["tests"]:
        for be in ("le", "be"):
            raw = open(os.path.join(GOLD, be, b(t["testName"]).decode() + ".pcapng"), "rb").read()
            opts = pcapgo.NgReaderOptions(t["wantMixedLinkType"], t["errorOnMismatchingLinkType"],
                                          t["skipUnknownVersion"])
            r = pcapgo.NewNgReader(raw, opts)
            assert r.LinkType() == (0 if t["wantMixedLinkType"] else t["linkType"])
            for p in t["packets"]:
                if "err" in p:
                    with pytest.raises(pcapgo.PcapgoError) as e:
                        r.ReadPacketData()
                    assert e.value.text == p["err"]["err"]
                    break
                data, ci = r.ReadPacketData()
                assert data == b(p["data"])
                w = p["ci"]
                assert ci.Timestamp == tuple(w["Timestamp"]["time"])
                assert (ci.CaptureLength, ci.Length, ci.InterfaceIndex) == (w["CaptureLength"], w["Length"],
                                                                           w.get("InterfaceIndex", 0))
                assert ci.AncillaryData == (w.get("AncillaryData") or [])
            else:
                with pytest.raises(EOFError):
                    r.ReadPacketData()
                secs = r.SectionEnds() + [(r.SectionInfo(), [r.Interface(i) for i in range(r.NInterfaces())])]
                assert len(secs) == len(t["sections"])
                for (info, ifs), w in zip(secs, t["sections"]):
                    wi = w["sectionInfo"]
                    assert info.Comment == b(wi.get("Comment", {"str": ""}))
                    assert info.Hardware == b(wi.get("Hardware", {"str": ""}))
                    assert [i.Name for i in ifs] == [want_iface(x)["name"] for x in w.get("ifaces", [])]
                    assert [i.Statistics.PacketsDropped for i in ifs] == \
                        [want_iface(x)["stats"]["dropped"] for x in w.get("ifaces", [])]


def test_python_mirror_gzip_and_batches():
    raw = pcapgen.ng_file([bytes([i & 0xFF]) * (60 + i) for i in range(1000)])
    for src in (raw, gzip.compress(raw)):
        r = pcapgo.NewNgReader(src)
        total = 0
        while True:
            try:
                bt = r.ReadBatch(300)
            except EOFError:
                break
            for i in range(len(bt)):
                o, c = int(bt.offsets[i]), int(bt.caplens[i])
                assert bytes(bt.data[o:o + c]) == bytes([(total + i) & 0xFF]) * (60 + total + i)
            total += len(bt)
        assert total == 1000
    with pytest.raises(pcapgo.PcapgoError) as e:
        pcapgo.NewNgReader(b"\x1f\x8b\x08")
    assert e.value.text == "unexpected EOF"
    with pytest.raises(EOFError):
        pcapgo.NewNgReader(b"")


def index_all_events(stream, flags, threads, chunk=None, state=False):
    """gpk_capreader_index_all over the stream (whole or in chunks), as events
    (state=True: and the reader's name records and callback calls after it)."""
    L = _lib.lib()
    h = ctypes.c_void_p()
    _lib.check(L.gpk_capreader_create(ctypes.byref(h), _lib.CAP_PCAPNG, flags))
    ev = []
    base, have = 0, (len(stream) if chunk is None else min(len(stream), chunk))
    try:
        while True:
            buf = np.frombuffer(stream[base:have], np.uint8) if have > base else np.zeros(1, np.uint8)
            eof = have >= len(stream)
            out, used = _lib.CapIndex(), ctypes.c_uint64()
            rc = L.gpk_capreader_index_all(h, buf.ctypes.data, have - base, int(eof), threads, ctypes.byref(out),
                                           ctypes.byref(used))
            assert rc in (_lib.CAP_MORE, _lib.CAP_END), rc
            n = out.n
            if n:
                off = np.ctypeslib.as_array(ctypes.cast(out.offsets, ctypes.POINTER(ctypes.c_uint64)), (n,))
                cap = np.ctypeslib.as_array(ctypes.cast(out.caplens, ctypes.POINTER(ctypes.c_uint32)), (n,))
                ci = np.ctypeslib.as_array(ctypes.cast(out.ci, ctypes.POINTER(ctypes.c_uint8)), (n * 24,)).view(
                    _lib.CAPINFO_DTYPE)
                for i in range(n):
                    r = ci[i]
                    ev.append(("pkt", base + int(off[i]), int(cap[i]), int(r["ts_sec"]), int(r["ts_nsec"]),
                               int(r["length"]), int(r["iface"]),
                               None if int(r["link_type"]) < 0 else int(r["link_type"])))
            L.gpk_capindex_free(ctypes.byref(out))
            base += used.value
            if rc == _lib.CAP_END:
                b = ctypes.create_string_buffer(512)
                e, p = ctypes.c_int(), ctypes.c_int()
                k = L.gpk_capreader_error(h, b, 512, ctypes.byref(e), ctypes.byref(p))
                ev.append(("err", b.raw[:k].decode("latin-1"), bool(p.value)))
                break
            assert not eof
            have = len(stream) if chunk is None else min(len(stream), have + chunk)
        st = native_reader_state(L, h)
    finally:
        L.gpk_capreader_destroy(h)
    return (ev, st) if state else ev


def big_capture(n=60000, seed=3):
    from gopacket_amd import synth
    rng = random.Random(seed)
    pk = [synth.packet(4, i) for i in range(n)]
    blocks = [pcapgen.epb(p, ts=i * 1000) for i, p in enumerate(pk)]
    return pcapgen.shb() + pcapgen.idb(1, 0) + pcapgen.idb(1, 0), blocks, rng


def test_parallel_walk_equals_sequential():
    head, blocks, rng = big_capture()
    variants = {"plain": blocks}
    # state changes, non-plain blocks and a fake block chain inside packet data
    v = list(blocks)
    v.insert(20000, pcapgen.idb(0, 0))  # a Null-link interface: later packets on it are skipped
    v[25000] = pcapgen.epb(bytes(100), iface=2)
    v.insert(30000, pcapgen.epb(bytes(70), options=pcapgen.opt(1, b"comment") + pcapgen.end_opt()))
    v.insert(35000, pcapgen.spb(bytes(90)))
    v.insert(41000, pcapgen.shb(">") + pcapgen.idb(1, 0, ">"))
    v[41001:] = [pcapgen.epb(pcapgen_payload(b), bo=">") for b in v[41001:]]
    fake = b"".join(pcapgen.epb(bytes([7]) * 40, ts=5) for _ in range(6))
    v.insert(15000, pcapgen.epb(bytes(3) + fake + bytes(5)))
    variants["mixed"] = v
    # name records after long plain runs (EUI records clone the reader's scratch
    # buffer: the last block header the speculative walk skipped over) and
    # statistics blocks (StatisticsCallback's packet count after those runs)
    w = list(blocks)
    for at in (9000, 33000, 52000):
        w.insert(at, pcapgen.nrb([(1, b"\x0a\x00\x00\x01" + b"v4\x00"), (2, bytes(range(16)) + b"v6\x00x\x00")]))
        w.insert(at + 1, pcapgen.isb(1, at, options=pcapgen.opt(4, struct.pack("<Q", at)) + pcapgen.end_opt()))
    # an EUI record desynchronises the rest of the stream as in Go: the last block
    w.append(pcapgen.nrb([(1, b"\x0a\x00\x00\x02" + b"w\x00"), (3, bytes(range(6)) + b"eui48\x00")]))
    variants["names"] = w
    for name, bl in variants.items():
        data = head + b"".join(bl)
        for flags in (0, 1, 2):
            want, meta = native_events(data, _lib.CAP_PCAPNG, flags, errors=1, max_events=10 ** 7)
            want = [e[:8] if e[0] == "pkt" else e for e in want]  # (index_all keeps no options)
            wstate = {k: meta[k] for k in ("names", "stat_events", "section_ends")}
            for threads in (1, 3, 8):
                assert index_all_events(data, flags, threads, state=True) == (want, wstate), (name, flags, threads)
            assert index_all_events(data, flags, 8, chunk=(5 << 20) + 13, state=True) == (want, wstate), (name, flags)
        if name == "names":
            # an EUI record clones the reader's whole scratch buffer: its first 6 bytes,
            # the NRB block length's high half, then the ts-low / caplen / length words
            # the last EPB header before the block left there (a plain run the
            # speculative walk took); the reference's 24-byte address length then
            # desynchronises the rest of the block, as in Go (ngread_nrb.go:56-61,108)
            nm = wstate["names"]
            assert nm[:2] == [(1, b"\x0a\x00\x00\x01", [b"v4"]), (2, bytes(range(16)), [b"v6", b"x"])]
            assert len(nm) == 8 and nm[6] == (1, b"\x0a\x00\x00\x02", [b"w"]) and nm[7][0] == 3
            prev = blocks[-1]
            assert nm[7][1][:6] == bytes(range(6)) and nm[7][1][8:20] == prev[16:28] and nm[7][1][20:] == bytes(4)
            assert [e[0] for e in wstate["stat_events"]] == [9000, 33000 - 2, 52000 - 4]  # packets before each


def pcapgen_payload(block):
    """The packet bytes of a little-endian plain EPB built by pcapgen.epb."""
    cl = int.from_bytes(block[20:24], "little")
    return block[28:28 + cl]


@pytest.mark.timeout(300)
def test_parallel_walk_concurrent_callers():
    """The walk's worker pool is process-wide: two readers indexing at once on
    two threads (ctypes releases the GIL) must each get their own sequential
    result (the pool held one job and a second caller overwrote it)."""
    import threading
    head, blocks, _ = big_capture(n=40000, seed=5)
    a = head + b"".join(blocks)
    b = head + b"".join(blocks[::-1][:30000])
    want = {k: index_all_events(d, 0, 8) for k, d in (("a", a), ("b", b))}
    got, errs = {}, []

    def go(k, d):
        try:
            for r in range(4):
                got[(k, r)] = index_all_events(d, 0, 8)
        except Exception as e:  # surfaced below
            errs.append(e)

    th = [threading.Thread(target=go, args=(k, d)) for k, d in (("a", a), ("b", b))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for (k, r), ev in got.items():
        assert ev == want[k], (k, r)

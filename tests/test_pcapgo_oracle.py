"""Pin the pcapgo reader oracle (oracle/pcapgo_oracle.py) to the reference's own tests.

Every expectation comes from tests/golden/pcapgo/expect.json, harvested from
pcapgo/ngread_test.go and pcapgo/read_test.go by tools/harvest_pcapgo.py, and
is checked the way the reference's harness checks it (ngRunFileReadTest,
ngread_test.go:58-198).
"""
import gzip
import json
import os

import pytest

import pcapgen
from oracle import pcapgo_oracle as PO

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "pcapgo")
EXPECT = json.load(open(os.path.join(GOLD, "expect.json")))


def b(v):
    if isinstance(v, dict):
        return bytes.fromhex(v["hex"]) if "hex" in v else v["str"].encode("latin-1")
    return v


def name(t):
    return b(t["testName"]).decode() + (b(t["testType"]).decode() if t["testType"] else "")


CASES = [(t, be) for t in EXPECT["tests"] for be in ("le", "be")]


def want_iface(w):
    res = w.get("TimestampResolution", 0) or 6  # "fix non-zero defaults" (ngread_test.go:92-95)
    st = w.get("Statistics", {})
    z = [-62135596800, 0]
    return dict(name=b(w.get("Name", {"str": ""})), comment=b(w.get("Comment", {"str": ""})),
                description=b(w.get("Description", {"str": ""})), filter=b(w.get("Filter", {"str": ""})),
                os=b(w.get("OS", {"str": ""})), link_type=w.get("LinkType", 0), ts_resolution=res,
                ts_offset=w.get("TimestampOffset", 0), snap_length=w.get("SnapLength", 0),
                stats=dict(last_update=tuple(st.get("LastUpdate", {"time": z})["time"]),
                           start_time=tuple(st.get("StartTime", {"time": z})["time"]),
                           end_time=tuple(st.get("EndTime", {"time": z})["time"]),
                           comment=b(st.get("Comment", {"str": ""})),
                           received=st.get("PacketsReceived", 0), dropped=st.get("PacketsDropped", 0)))


def check_section(got, want):
    info, ifaces = got
    wi = want["sectionInfo"]
    assert info == dict(comment=b(wi.get("Comment", {"str": ""})), hardware=b(wi.get("Hardware", {"str": ""})),
                        os=b(wi.get("OS", {"str": ""})), application=b(wi.get("Application", {"str": ""})))
    assert len(ifaces) == len(want.get("ifaces", []))
    for g, w in zip(ifaces, want.get("ifaces", [])):
        assert g == want_iface(w)


@pytest.mark.parametrize("t,be", CASES, ids=["%s-%s" % (name(t), be) for t, be in CASES])
def test_ng_file_read(t, be):
    """ngRunFileReadTest (ngread_test.go:58-198) on the oracle."""
    data = open(os.path.join(GOLD, be, b(t["testName"]).decode() + ".pcapng"), "rb").read()
    r = PO.NgReader(data, want_mixed=t["wantMixedLinkType"], error_on_mismatch=t["errorOnMismatchingLinkType"],
                    skip_unknown_version=t["skipUnknownVersion"])
    assert r.link_type == (0 if t["wantMixedLinkType"] else t["linkType"])
    for p in t["packets"]:
        if "err" in p:
            with pytest.raises(PO.GoError) as e:
                r.read_packet()
            assert e.value.text == p["err"]["err"]
            if p["err"]["err"] != PO.ERR_NG_VERSION:
                check_section(r.section_state(), t["sections"][len(r.ended_sections)])
            return
        pk = r.read_packet()
        assert r.s.d[pk.offset:pk.offset + pk.caplen] == b(p["data"])
        ci = p["ci"]
        assert (pk.ts_sec, pk.ts_nsec) == tuple(ci["Timestamp"]["time"])
        assert (pk.caplen, pk.length, pk.iface) == (ci["CaptureLength"], ci["Length"], ci.get("InterfaceIndex", 0))
        want_anc = ci.get("AncillaryData")
        assert pk.ancil == (want_anc[0] if want_anc else None)
    with pytest.raises(PO.GoError) as e:
        r.read_packet()
    assert e.value.text == "EOF"
    secs = r.ended_sections + [r.section_state()]
    assert len(secs) == len(t["sections"])
    for g, w in zip(secs, t["sections"]):
        check_section(g, w)


def pv(name):
    return bytes.fromhex(EXPECT["pcap_vectors"][name])


def test_pcap_reader_vectors():
    """read_test.go:15-255."""
    PO.Reader(pv("TestCreatePcapReader"))
    PO.Reader(pv("TestCreatePcapReaderBigEndian"))
    with pytest.raises(PO.GoError):
        PO.Reader(pv("TestCreatePcapReaderFail"))
    with pytest.raises(PO.GoError):
        PO.Reader(pv("TestTruncatedGzipPacket"))
    for vec, nsec in (("TestPacket", 1000), ("TestPacketNano", 1), ("TestGzipPacket", 1000)):
        r = PO.Reader(pv(vec))
        p = r.read_packet()
        # time.Date(2014, 9, 18, 12, 13, 14, nsec, time.UTC)
        assert (p.ts_sec, p.ts_nsec) == (1411042394, nsec)
        assert (p.caplen, p.length) == (4, 8)
        assert r.s.d[p.offset:p.offset + 4] == bytes([1, 2, 3, 4])
    r = PO.Reader(pv("TestPacketBufferReuse"))
    assert [r.s.d[p.offset:p.offset + 4] for p in (r.read_packet(), r.read_packet())] == [bytes([1, 2, 3, 4])] * 2
    r = PO.Reader(pv("TestPacketZeroCopy"))
    assert [r.s.d[p.offset:p.offset + 4] for p in (r.read_packet(), r.read_packet())] == [bytes([1, 2, 3, 4]),
                                                                                          bytes([5, 6, 7, 8])]


def test_ng_gzip_and_truncation():
    """ngread_test.go:1845-1971."""
    v = bytes.fromhex(EXPECT["ng_vectors"]["TestNgFileReadGzipPacket"])
    r = PO.NgReader(v)
    p = r.read_packet()
    assert (p.ts_sec, p.ts_nsec, p.caplen, p.length) == (1411042394, 1000, 4, 8)
    assert r.s.d[p.offset:p.offset + 4] == bytes([1, 2, 3, 4])
    for data, err in ((b"", "EOF"), (b"\x1f", "unexpected EOF"), (b"\x1f\x8b\x08", "unexpected EOF")):
        with pytest.raises(PO.GoError) as e:
            PO.NgReader(data)
        assert e.value.text == err
    one = pcapgen.ng_file([b"\x01\x02"])  # the NgWriter one-packet capture of getBasicOnePacketPcap
    r = PO.NgReader(one[:-1])  # TestTruncatedDiscard
    with pytest.raises(PO.GoError) as e:
        r.read_packet()
    assert e.value.text == "unexpected EOF"
    with pytest.raises(PO.GoError) as e:  # TestTruncatedBlockHeader
        PO.NgReader(one[:4])
    assert e.value.text == "unexpected EOF"
    # the same capture gzip-compressed reads identically
    r = PO.NgReader(gzip.compress(one))
    assert r.s.d[r.read_packet().offset:][:2] == b"\x01\x02"


def test_ng_benchmark_stream():
    """setupNgReadBenchmark (ngread_test.go:1985-2026): big-endian SHB + IDB, then EPBs."""
    hdr = bytes.fromhex(EXPECT["ng_vectors"]["setupNgReadBenchmark.header"])
    e1 = pcapgen.epb(bytes(range(1, 17)), bo=">")
    e2 = pcapgen.epb(bytes(range(8, 0, -1)), bo=">")
    res = PO.read_all(hdr + (e1 + e2) * 50)
    assert res["err"] == "EOF" and len(res["packets"]) == 100
    assert [p.caplen for p in res["packets"][:4]] == [16, 8, 16, 8]


def test_epb_options_file():
    """ngread_test.go:2028-2105: the EPB-with-options capture reads without error."""
    data = open(os.path.join(GOLD, "epb.pcapng"), "rb").read()
    r = PO.NgReader(data)
    r.read_packet()

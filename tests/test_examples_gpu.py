"""examples/statsassembly.py (the reference's examples/statsassembly loop over a
capture file, decode on the GPU) against the oracles: the capture reader
oracle's packets, decoded by the decode oracle with the example's parser
(Ethernet, Dot1Q, IPv4, IPv6, IPv6ExtensionSkipper, TCP, Payload:
main.go:134-142), keyed by the grouping oracle's tcpassembly key. The
example's streams must be the oracle's keys of the packets DecodeLayers
returned no error for, in the same order, with the same packets, payload
bytes and SYN / FIN-RST flags; --device-groups checks gpk_group_batch against
the loop on every batch."""
import importlib.util
import os

import numpy as np
import pytest

from configs import oracle_parser
from oracle import flows_oracle as FO
from oracle import pcapgo_oracle as PO

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PARSER = dict(first=17, decoders=["ETHERNET", "DOT1Q", "IPV4", "IPV6", "IPV6_EXT", "TCP", "PAYLOAD"])


def example():
    spec = importlib.util.spec_from_file_location("statsassembly", os.path.join(ROOT, "examples", "statsassembly.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def expected(path):
    raw = open(path, "rb").read()
    r = PO.read_all(raw, kind="ng" if raw[:4] == b"\x0a\x0d\x0d\x0a" else "pcap")
    s = r["stream"]
    pk = [bytes(s[p.offset:p.offset + p.caplen]) for p in r["packets"]]
    cap = np.array([len(p) for p in pk], np.uint32)
    off = np.zeros(len(pk), np.uint64)
    off[1:] = np.cumsum(cap[:-1], dtype=np.uint64)
    ref = oracle_parser(PARSER).decode(np.frombuffer(b"".join(pk) + bytes(16), np.uint8), off, cap, layouts=True)
    streams = {}
    for i, p in enumerate(pk):
        rec, lay = ref["records"][i], ref["layouts"][i]
        if int(rec["status"]) & 0x7F:  # DecodeLayers returned an error: the loop skips the packet
            continue
        key = FO.packet_key(FO.CONNECTION, p, rec, lay, 0, 8)
        if not isinstance(key, tuple):
            continue
        t0, t1 = int(lay["start"][5]), int(lay["end"][5])  # the TCP layer's bytes
        flags, doff = p[t0 + 13], p[t0 + 12] >> 4
        s = streams.setdefault(key, [0, 0, False, False])
        s[0] += 1
        s[1] += (t1 - t0) - 4 * doff
        s[2] |= bool(flags & 2)
        s[3] |= bool(flags & 5)
    return list(streams.values()), len(pk)


@pytest.mark.parametrize("src", ["c6_pcapng", "test_ethernet_pcap"])
def test_statsassembly_example(gpu_ctx, tmp_path, src):
    from gopacket_amd import _lib
    if src == "c6_pcapng":
        path = str(tmp_path / "c6.pcapng")
        assert _lib.synth_lib().gpk_synth_write_pcapng(path.encode(), 6, 0, 40000, 4) > 0
    else:
        path = os.path.join(ROOT, "tests", "golden", "test_ethernet.pcap")
    want, n = expected(path)
    logs = []
    streams, read, _ = example().run(path, batch=7000, device_groups=True, log=logs.append)
    assert read == n
    got = [[s.packets, s.bytes, s.sawStart, s.sawEnd] for s in streams]
    assert got == want, (len(got), len(want))
    assert len(want) > (100 if src == "c6_pcapng" else 0)
    assert sum(line.startswith("new stream ") for line in logs) == len(want)
    assert logs[-1].startswith("processed ")

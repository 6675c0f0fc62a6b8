"""gpk_decode_batch_narrow (the 8-byte gpk_record8 and its side array of full
records, include/gpk.h) against the oracle's narrow form
(oracle_decode_batch_narrow, which derives it from the same decode and the
header Checksum fields it read) bit for bit: records8, the whole side array
(zero where no record was widened), error arguments and flow hashes; and
against the device's own 16-byte decode of the same batch: every widened
packet's side record is that decode's record, every other packet's layers and
status bits are. Cases: the golden packets and 40 000 fuzzed packets under
every test parser at two alignments, the C2/C3/C4 synthetic mixes, lists longer
than 8 and 16 entries, UDP zero checksums, invalid IPv4 / TCP / UDP checksums,
an empty batch."""
import struct
import zlib

import numpy as np
import pytest

import pktutil
from configs import CONFIGS, device_parser, oracle_parser
from test_gpu_parity import golden_packets

pytestmark = pytest.mark.gpu


def narrow_device(ctx, cfg, data, off, cap):
    import torch
    n = len(off)
    d = torch.from_numpy(np.ascontiguousarray(data)).cuda()
    o = torch.from_numpy(np.ascontiguousarray(off).view(np.int64)).cuda()
    c = torch.from_numpy(np.ascontiguousarray(cap).view(np.int32)).cuda()
    rec8 = torch.full((max(n, 1) * 8,), 0xAB, dtype=torch.uint8, device="cuda")
    wide = torch.zeros(max(n, 1) * 16, dtype=torch.uint8, device="cuda")
    err = torch.zeros(max(2 * n, 1), dtype=torch.int32, device="cuda")
    fl = torch.zeros(max(3 * n, 1), dtype=torch.int64, device="cuda")
    ctx.decode_device_narrow(device_parser(cfg), d, o, c, rec8, wide, err, fl)
    torch.cuda.synchronize()
    from gopacket_amd import _lib
    return dict(records8=rec8.cpu().numpy()[:8 * n].view(_lib.RECORD8_DTYPE),
                wide=wide.cpu().numpy()[:16 * n].view(_lib.RECORD_DTYPE),
                err_args=err.cpu().numpy()[:2 * n].view(np.uint32), flows=fl.cpu().numpy()[:3 * n].view(np.uint64))


def check_narrow(ctx, cfg, data, off, cap, what):
    got = narrow_device(ctx, cfg, data, off, cap)
    ref = oracle_parser(cfg).decode_narrow(data, off, cap, nthreads=8)
    n = len(off)
    for k in ("records8", "wide", "err_args", "flows"):
        a, b = got[k], ref[k]
        if k == "records8":
            bad = np.nonzero((a["layers"] != b["layers"]) | (a["status"] != b["status"]))[0]
        elif k == "wide":
            bad = np.nonzero((a["layers"] != b["layers"]) | (a["status"] != b["status"]) |
                             (a["ip4_csum"] != b["ip4_csum"]) | (a["l4_csum"] != b["l4_csum"]))[0]
        else:
            bad = np.nonzero(a != b)[0]
        assert len(bad) == 0, "%s: %s differs at %d of %d, first %s: dev=%s ref=%s" % (
            what, k, len(bad), n, bad[:5], a[bad[:3]], b[bad[:3]])
    # and against the device's own 16-byte decode
    full = ctx.decode_host(device_parser(cfg), data, off, cap, layouts=False)
    r8, rw = got["records8"], full["records"]
    from gopacket_amd import _lib
    w = (r8["status"] & _lib.ST8_WIDE) != 0
    assert np.array_equal(got["wide"][w], rw[w]), what
    nw = ~w
    assert np.array_equal(r8["layers"][nw].astype(np.uint64), rw["layers"][nw]), what
    mask = ~np.uint32((0xFFF << 8))
    assert np.array_equal(r8["status"][nw] & mask, rw["status"][nw] & mask), what
    nl = (rw["status"] >> 8) & 0xFFF
    assert np.array_equal((r8["status"] >> 8) & 0xF, np.where(nl > 8, 15, nl).astype(np.uint32)), what
    assert np.array_equal(got["flows"], full["flows"]) and np.array_equal(got["err_args"], full["err_args"]), what
    return got, w


@pytest.mark.parametrize("cfg_name", sorted(CONFIGS))
def test_narrow_golden(gpu_ctx, cfg_name):
    data, off, cap = pktutil.pack(golden_packets())
    check_narrow(gpu_ctx, CONFIGS[cfg_name], data, off, cap, cfg_name)


@pytest.mark.parametrize("cfg_name", sorted(CONFIGS))
@pytest.mark.parametrize("align", [1, 16])
def test_narrow_fuzz(gpu_ctx, cfg_name, align):
    packets = pktutil.fuzz_packets(zlib.crc32(cfg_name.encode()) % 1000 + 7 * align, 40000)
    data, off, cap = pktutil.pack(packets, align=align, pad=align // 2)
    _, w = check_narrow(gpu_ctx, CONFIGS[cfg_name], data, off, cap, cfg_name)
    if cfg_name in ("statsassembly", "eth_ip4_tcp_payload"):
        assert 0 < w.sum() < len(w)  # the fuzzer's bad checksums widen some records, most stay narrow


@pytest.mark.parametrize("synth_cfg,cfg_name", [(2, "eth_ip4_udp_payload"), (3, "eth_ip4_tcp_payload"),
                                                (4, "statsassembly")])
def test_narrow_synthetic(gpu_ctx, synth_cfg, cfg_name):
    from gopacket_amd import synth
    data, off, cap = synth.host_batch(synth_cfg, 424242, 100000)
    check_narrow(gpu_ctx, CONFIGS[cfg_name], data, off, cap, "synth%d" % synth_cfg)


def _ip4(proto, payload, csum=None):
    h = struct.pack(">BBHHHBBH4s4s", 0x45, 0, 20 + len(payload), 7, 0, 64, proto, 0, b"\x0a\x00\x00\x01",
                    b"\x0a\x00\x00\x02")
    if csum is None:
        s = sum(struct.unpack(">10H", h))
        s = (s & 0xFFFF) + (s >> 16)
        s = (s & 0xFFFF) + (s >> 16)
        csum = ~s & 0xFFFF
    return h[:10] + struct.pack(">H", csum) + h[12:] + payload


def _csum(b):
    if len(b) % 2:
        b += b"\x00"
    s = sum(struct.unpack(">%dH" % (len(b) // 2), b))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return ~s & 0xFFFF


def _udp_ok(payload):
    """A UDP header + payload whose checksum is right under _ip4's addresses."""
    u = struct.pack(">HHHH", 40000, 40001, 8 + len(payload), 0) + payload
    ph = b"\x0a\x00\x00\x01\x0a\x00\x00\x02" + struct.pack(">BBH", 0, 17, len(u))
    c = _csum(ph + u) or 0xFFFF
    return u[:6] + struct.pack(">H", c) + u[8:]


def test_narrow_edge_records(gpu_ctx):
    """The cases the side array exists for: a UDP checksum of 0 (Valid, Correct
    != Actual), wrong IPv4 / UDP / TCP checksums, lists of 8, 9, 16 and 40
    entries; next to correct packets that stay narrow."""
    mac = b"\x02" * 12
    udp0 = struct.pack(">HHHH", 40000, 40001, 12, 0) + b"abcd"
    udpx = struct.pack(">HHHH", 40000, 40001, 12, 0x1234) + b"abcd"
    tcpx = struct.pack(">HHIIBBHHH", 1000, 80, 1, 2, 0x50, 0x18, 100, 0x4321, 0) + b"xyz"
    pkts = [mac + b"\x08\x00" + _ip4(17, udp0), mac + b"\x08\x00" + _ip4(17, udpx),
            mac + b"\x08\x00" + _ip4(6, tcpx), mac + b"\x08\x00" + _ip4(17, udp0, csum=0xBEEF)]
    for ntags in (4, 5, 6, 13, 37):  # Ethernet + tags + IPv4 + UDP + Payload: 8, 9, 10, 17, 41 entries
        tags = b"".join(struct.pack(">HH", 1, 0x8100) for _ in range(ntags - 1)) + struct.pack(">HH", 1, 0x0800)
        pkts.append(mac + b"\x81\x00" + tags + _ip4(17, _udp_ok(b"abcd")))
    pkts += [mac + b"\x08\x00" + _ip4(17, _udp_ok(bytes([i]) * (i % 37))) for i in range(200)]  # right: narrow
    data, off, cap = pktutil.pack(pkts)
    got, w = check_narrow(gpu_ctx, CONFIGS["statsassembly"], data, off, cap, "edges")
    assert list(w[:4]) == [True, True, True, True]
    nl = (got["records8"]["status"][4:9] >> 8) & 0xF
    assert list(nl) == [8, 15, 15, 15, 15] and list(w[4:9]) == [False, True, True, True, True]
    assert not w[9:].any()


def test_narrow_empty(gpu_ctx):
    got = narrow_device(gpu_ctx, CONFIGS["statsassembly"], np.zeros(16, np.uint8), np.zeros(0, np.uint64),
                        np.zeros(0, np.uint32))
    assert len(got["records8"]) == 0

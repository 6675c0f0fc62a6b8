"""Layer fields on the device (gpk_extract_fields) vs the oracle, bit for bit.

The device decodes with layouts, extracts the 128-byte gpk_fields records from
them, and both are compared with the oracle's layouts and its field
extraction (oracle_extract_fields, pinned in tests/test_fields_cpu.py against
the reference's field expectations) on the same bytes.
"""
import zlib

import numpy as np
import pytest
import torch

import pktutil
from configs import CONFIGS, assert_same, device_parser, oracle_parser
from gopacket_amd import _lib
from oracle import oracle as O

pytestmark = pytest.mark.gpu
FUSED_WAVES = 5  # gpk_kernels.hip GPK_SBF_WAVES


def device_fields(ctx, cfg, data, off, cap, layouts=True):
    r, f = ctx.decode_host_fields(device_parser(cfg), data, off, cap, layouts=layouts)
    return r, f.view(np.uint8).reshape(-1, 128)


def check(ctx, cfg_name, packets, align=1):
    """Both paths against the oracle: the decode with layouts + gpk_extract_fields,
    and the fused decode + fields launch (gpk_decode_batch_fields, no layouts),
    whose records, error arguments and flows must also equal the oracle's."""
    cfg = CONFIGS[cfg_name]
    data, off, cap = pktutil.pack(packets, align=align)
    ref = oracle_parser(cfg).decode(data, off, cap, nthreads=8, layouts=True)
    want = O.extract_fields(data, off, ref["layouts"])
    for layouts in (True, False):
        r, f = device_fields(ctx, cfg, data, off, cap, layouts=layouts)
        what = "%s (%s)" % (cfg_name, "layouts + extract" if layouts else "fused")
        if layouts:
            assert np.array_equal(r["layouts"].view(np.uint8), ref["layouts"].view(np.uint8)), what
        assert_same(r, ref, what)
        bad = np.nonzero((f != want).any(axis=1))[0]
        assert len(bad) == 0, "%s: %d packets differ, first %d: %s vs %s" % (
            what, len(bad), bad[0], f[bad[0]].tobytes().hex(), want[bad[0]].tobytes().hex())
    return f.view(_lib.FIELDS_DTYPE).reshape(-1)


@pytest.mark.parametrize("cfg_name", sorted(CONFIGS))
def test_fields_fuzz(gpu_ctx, cfg_name):
    packets = pktutil.fuzz_packets(zlib.crc32(cfg_name.encode()) % 1000 + 3, 20000)
    f = check(gpu_ctx, cfg_name, packets, align=1 + zlib.crc32(cfg_name.encode()) % 7)
    if cfg_name != "first_unregistered":  # that parser decodes no layer at all
        assert (f["present"] != 0).mean() > 0.05


@pytest.mark.parametrize("synth_cfg,cfg_name", [(2, "eth_ip4_udp_payload"), (3, "eth_ip4_tcp_payload"),
                                                (4, "statsassembly")])
def test_fields_synthetic(gpu_ctx, synth_cfg, cfg_name):
    from gopacket_amd import synth
    data, off, cap = synth.host_batch(synth_cfg, 987654321, 50000)
    packets = [bytes(data[int(o):int(o) + int(c)]) for o, c in zip(off, cap)]
    f = check(gpu_ctx, cfg_name, packets)
    if synth_cfg == 4:  # IMIX: IPv4 and IPv6, TCP and UDP, tagged and untagged all present
        p = f["present"]
        for slot in (1, 2, 3, 5, 6):
            assert (p & (1 << slot)).any(), slot


def test_fields_golden(gpu_ctx):
    g = pktutil.golden()
    packets = [bytes.fromhex(v["hex"]) for k, v in sorted(g.items()) if "hex" in v]
    for name in ("test_ethernet.pcap", "test_dns.pcap"):
        packets += pktutil.read_pcap(pktutil.GOLDEN + "/" + name)[1]
    for cfg_name in sorted(CONFIGS):
        check(gpu_ctx, cfg_name, packets)


@pytest.mark.parametrize("layout", ["sparse_mix", "gapped", "wave_shuffled", "reversed"])
def test_fields_fused_layouts(gpu_ctx, layout):
    """The fused kernel on unordered and sparse batches (its phase B after the
    parse, whose head/tail chunks then come from memory), the kernel named."""
    from test_gpu_parity import golden_packets, phase_b_layout
    packets = pktutil.fuzz_packets(77, 8000) + golden_packets()
    data, off, cap = phase_b_layout(packets, layout)
    for cfg_name in ("statsassembly", "eth_ip4_tcp_payload", "eth_ip4_udp_payload"):
        cfg = CONFIGS[cfg_name]
        dp = device_parser(cfg)
        assert gpu_ctx.kernel_name(dp, data, off, cap, layouts=_lib.NAME_FIELDS) == \
            "gpk::decode_sb_kernel<true,%d,6,true>" % FUSED_WAVES
        ref = oracle_parser(cfg).decode(data, off, cap, nthreads=8, layouts=True)
        r, f = device_fields(gpu_ctx, cfg, data, off, cap, layouts=False)
        assert_same(r, ref, layout + "/" + cfg_name)
        want = O.extract_fields(data, off, ref["layouts"])
        assert np.array_equal(f, want), layout + "/" + cfg_name


def test_fields_fused_output_subsets(gpu_ctx):
    """Every GPK_OUT_* subset through the fused launch (without the L4 checksum
    the kernel skips the stream before the parse)."""
    from gopacket_amd import synth
    data, off, cap = synth.host_batch(4, 4321, 30000)
    for outputs in range(8):
        cfg = dict(CONFIGS["statsassembly"], outputs=outputs)
        ref = oracle_parser(cfg).decode(data, off, cap, nthreads=8, layouts=True)
        r, f = device_fields(gpu_ctx, cfg, data, off, cap, layouts=False)
        if not outputs & 4:
            r["flows"][:] = 0
        assert_same(r, ref, "outputs=%d" % outputs)
        assert np.array_equal(f, O.extract_fields(data, off, ref["layouts"])), outputs


def test_fields_empty_batch(gpu_ctx):
    t = torch.zeros(16, dtype=torch.uint8, device="cuda")
    e = torch.zeros(0, dtype=torch.int64, device="cuda")
    gpu_ctx.extract_fields(t, e, e, t, t)  # n = 0: nothing launched, no error


def test_decode_batch_fields_api(gpu_ctx):
    """gopacket.DecodingLayerParser.DecodeBatch(fields=True): the device fields
    equal the layer structs Hydrate fills for the same packet."""
    from gopacket_amd import gopacket as gp, layers
    eth, ip4, ip6, tcp, udp = layers.Ethernet(), layers.IPv4(), layers.IPv6(), layers.TCP(), layers.UDP()
    p = gp.DecodingLayerParser(layers.LayerTypeEthernet, eth, layers.Dot1Q(), ip4, ip6, tcp, udp, gp.Payload(),
                               ctx=gpu_ctx)
    from gopacket_amd import synth
    data, off, cap = synth.host_batch(4, 5, 2000)
    res = p.DecodeBatch(gp.PacketBatch(data, off, cap), fields=True, layouts=True)
    assert res.fields is not None and len(res.fields) == len(off)
    decoded = []
    n = 0
    for i in range(len(off)):
        res.Hydrate(i, decoded)
        f = res.fields[i]
        if layers.LayerTypeTCP in decoded:
            assert (int(f["tcp_src_port"]), int(f["tcp_seq"]), int(f["tcp_window"])) == (int(tcp.SrcPort), tcp.Seq,
                                                                                          tcp.Window)
            n += 1
        if layers.LayerTypeIPv4 in decoded:
            assert (int(f["ip4_ttl"]), bytes(f["ip4_dst"])) == (ip4.TTL, bytes(ip4.DstIP))
    assert n > 100


def test_fields_header_ends_at_buffer_end(gpu_ctx):
    """A pure ACK whose TCP header ends past the 6-chunk LDS window and exactly
    at the end of the batch buffer (data_bytes = its last byte + 1): the 16-bit
    fields at the header's end (Checksum, Urgent) come from memory and read
    their own 2 bytes only (gpk_fields.hip Hdr::be16)."""
    import struct
    cfg = CONFIGS["statsassembly"]
    src, dst = bytes(range(16)), bytes(range(16, 32))
    hbh = bytes([6, 0, 1, 4, 0, 0, 0, 0])
    tcp = struct.pack(">HHIIBBHHH", 443, 51000, 7, 9, 0x50, 0x10, 512, 0x1234, 0xBEEF)
    ip6 = struct.pack(">IHBB16s16s", 0x60000000, len(hbh) + len(tcp), 0, 64, src, dst)
    ack = b"\x02" * 12 + b"\x86\xdd" + ip6 + hbh + tcp  # 82 bytes: Ethernet + IPv6 + HopByHop + TCP
    lead = pktutil.fuzz_packets(31, 300)
    data, off, cap = pktutil.pack(lead)
    last = (len(data) + 15) // 16 * 16 + 15  # packet byte 0 at window byte 15: window = 81 bytes
    buf = np.zeros(last + len(ack), np.uint8)
    buf[:len(data)] = data
    buf[last:] = np.frombuffer(ack, np.uint8)
    off = np.append(off, np.uint64(last))
    cap = np.append(cap, np.uint32(len(ack)))
    n = len(off)
    d_data = torch.from_numpy(buf).cuda()
    d_off = torch.from_numpy(off.view(np.int64)).cuda()
    d_cap = torch.from_numpy(cap.view(np.int32)).cuda()
    rec = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    err = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
    fl = torch.zeros(3 * n, dtype=torch.int64, device="cuda")
    lay = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
    fields = torch.zeros(n * 128, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    gpu_ctx.decode_device(device_parser(cfg), d_data, d_off, d_cap, rec, err, fl, lay, stream=s)
    gpu_ctx.extract_fields(d_data, d_off, d_cap, lay, fields, stream=s)
    torch.cuda.synchronize()
    ref = oracle_parser(cfg).decode(buf, off, cap, layouts=True)
    assert np.array_equal(lay.cpu().numpy().view(_lib.LAYOUT_DTYPE).view(np.uint8), ref["layouts"].view(np.uint8))
    want = O.extract_fields(buf, off, ref["layouts"])
    got = fields.cpu().numpy().reshape(-1, 128)
    assert np.array_equal(got, want)
    f = got[-1:].view(_lib.FIELDS_DTYPE).reshape(-1)[0]
    assert (int(f["tcp_checksum"]), int(f["tcp_urgent"]), int(f["tcp_window"])) == (0x1234, 0xBEEF, 512)


def test_decode_batch_fused_options(gpu_ctx):
    """DecodeBatch(fields=True) without layouts (one launch): the IPv4 and TCP
    option lists rebuilt from the device's option maps equal the ones Hydrate
    decodes on the host from a layouts run of the same packets."""
    from gopacket_amd import gopacket as gp, layers
    p = gp.DecodingLayerParser(layers.LayerTypeEthernet, layers.Ethernet(), layers.Dot1Q(), layers.IPv4(),
                               layers.IPv6(), layers.TCP(), layers.UDP(), gp.Payload(), ctx=gpu_ctx)
    pkts = pktutil.fuzz_packets(99, 6000)
    data, off, cap = pktutil.pack(pkts)
    batch = gp.PacketBatch(data, off, cap)
    fused = p.DecodeBatch(batch, fields=True)
    assert fused.layouts is None
    full = p.DecodeBatch(batch, layouts=True)
    n4 = nt = 0
    for i in range(len(off)):
        pkt = batch.packet(i)
        lay = full.layouts[i]
        s4, st = int(lay["start"][2]), int(lay["start"][5])
        if s4 != _lib.LAYOUT_ABSENT and int(fused.fields[i]["ip4_start"]) != 0xFF:
            v = layers.IPv4()  # fresh: the reference leaves Padding stale across packets
            v._hydrate(pkt[s4:int(lay["end"][2])])
            opts, pad = fused.IPv4Options(i)
            assert opts == v.Options and (pad or b"") == (v.Padding or b""), i
            n4 += len(opts) > 0
        if st != _lib.LAYOUT_ABSENT and int(fused.fields[i]["tcp_start"]) != 0xFF:
            v = layers.TCP()  # fresh: Multipath is stale across packets in the reference
            v._hydrate(pkt[st:int(lay["end"][5])])
            opts, pad, mp = fused.TCPOptions(i)
            assert opts == v.Options and pad == v.Padding and mp == v.Multipath, i
            nt += len(opts) > 0
    assert n4 > 20 and nt > 20


def test_fields_hopbyhop_maps(gpu_ctx):
    """The HopByHop option map (gpk_fields bytes 1-3, ip6.go:509-526) of
    Pad1 / PadN / Router Alert / Jumbo Payload mixes in headers of 8 to 32
    bytes, behind 0-2 tags: both device paths against the oracle, and the
    map set wherever the header fits it."""
    import hydrate_cases as H
    for cfg_name in ("statsassembly", "raw_ip6"):
        if cfg_name not in CONFIGS:
            continue
        pkts = H.hbh_packets(17, 3000)
        if cfg_name == "raw_ip6":
            pkts = [H.strip_ethernet(p) for p in pkts]
        f = check(gpu_ctx, cfg_name, pkts)
        m = f["hbh_opt_map"].astype(np.uint32)
        assert ((m[:, 0] | m[:, 1] << 8 | m[:, 2] << 16) != 0).mean() > 0.5, cfg_name

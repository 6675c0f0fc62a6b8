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
from configs import CONFIGS, device_parser, oracle_parser
from gopacket_amd import _lib
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def device_fields(ctx, cfg, data, off, cap):
    r, f = ctx.decode_host_fields(device_parser(cfg), data, off, cap)
    return r, f.view(np.uint8).reshape(-1, 128)


def check(ctx, cfg_name, packets, align=1):
    cfg = CONFIGS[cfg_name]
    data, off, cap = pktutil.pack(packets, align=align)
    r, f = device_fields(ctx, cfg, data, off, cap)
    ref = oracle_parser(cfg).decode(data, off, cap, nthreads=8, layouts=True)
    assert np.array_equal(r["layouts"].view(np.uint8), ref["layouts"].view(np.uint8)), cfg_name
    want = O.extract_fields(data, off, ref["layouts"])
    bad = np.nonzero((f != want).any(axis=1))[0]
    assert len(bad) == 0, "%s: %d packets differ, first %d: %s vs %s" % (
        cfg_name, len(bad), bad[0], f[bad[0]].tobytes().hex(), want[bad[0]].tobytes().hex())
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
    res = p.DecodeBatch(gp.PacketBatch(data, off, cap), fields=True)
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

"""Hydrate from the one-launch result on the device:
DecodeBatch(fields=True) without layouts (gpk_decode_batch_fields) against
DecodeBatch(layouts=True), struct by struct over fuzzed, golden, HopByHop and
synthetic packets, and no header read on the host for the C4 batch."""
import numpy as np
import pytest

import hydrate_cases as H
import pktutil
from gopacket_amd import _lib
from gopacket_amd import gopacket as G

pytestmark = pytest.mark.gpu


def _pair(gpu_ctx, pkts, decoders=H.DECODERS, first=17):
    batch = G.PacketBatch.from_packets(pkts)
    pa, pb = H.parser(decoders, first), H.parser(decoders, first)
    pa._ctx = pb._ctx = gpu_ctx
    ra = pa.DecodeBatch(batch, layouts=True)
    rb = pb.DecodeBatch(batch, fields=True)
    assert rb.layouts is None and rb.fields is not None
    return ra, rb, pa, pb


def test_hydrate_fused_equals_layouts_fuzz_golden(gpu_ctx):
    g = pktutil.golden()
    pkts = [bytes.fromhex(v["hex"]) for k, v in sorted(g.items()) if "hex" in v]
    pkts += pktutil.fuzz_packets(123, 6000) + H.hbh_packets(5, 1000)
    ra, rb, pa, pb = _pair(gpu_ctx, pkts)
    n = H.compare(ra, rb, pa, pb, range(len(pkts)))
    assert n == len(pkts)
    assert rb.host_decodes < 0.12 * n


def test_hydrate_fused_c4_no_host_reads(gpu_ctx):
    """50 000 packets of C4's IMIX mix (tags, QinQ, IPv4/IPv6, HopByHop):
    every struct from the device's record, zero host header reads."""
    from gopacket_amd import synth
    data, off, cap = synth.host_batch(4, 0, 50000)
    pkts = [bytes(data[int(o):int(o) + int(c)]) for o, c in zip(off, cap)]
    ra, rb, pa, pb = _pair(gpu_ctx, pkts)
    assert H.compare(ra, rb, pa, pb, range(len(pkts))) == 50000
    assert rb.host_decodes == 0
    hbh = sum(1 for i in range(len(pkts)) if int(rb.fields[i]["present"]) & 8
              and int(rb.fields[i]["ip6_next_header"]) == 0)
    assert hbh > 0  # the mix's HopByHop packets went through the map


def test_hydrate_fused_raw_ipv6(gpu_ctx):
    """ip6_test.go's vectors and HopByHop mixes from LayerTypeIPv6."""
    from gopacket_amd import layers as L
    pkts = [pktutil.golden_bytes("ip6_hopbyhop0"), pktutil.golden_bytes("ip6_destination0"),
            pktutil.golden_bytes("ip6_jumbogram_header") + b"\xfe" * 65536]
    pkts += [H.strip_ethernet(p) for p in H.hbh_packets(6, 500)]
    decs = (L.IPv6, L.IPv6ExtensionSkipper, L.TCP, L.UDP, G.Payload)
    ra, rb, pa, pb = _pair(gpu_ctx, pkts, decoders=decs, first=21)
    assert H.compare(ra, rb, pa, pb, range(len(pkts))) == len(pkts)

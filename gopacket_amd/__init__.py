"""gopacket_amd: gopacket's DecodingLayerParser fast path (decode + Internet
checksum + Flow.FastHash) as hand-written HIP kernels for MI355X (gfx950).

    from gopacket_amd import gopacket, layers
    eth, ip4, tcp, pl = layers.Ethernet(), layers.IPv4(), layers.TCP(), gopacket.Payload()
    parser = gopacket.NewDecodingLayerParser(layers.LayerTypeEthernet, eth, ip4, tcp, pl)
    decoded = []
    err = parser.DecodeLayers(packet_bytes, decoded)          # one packet, on the GPU
    res = parser.DecodeBatch(gopacket.PacketBatch.from_packets(pkts))   # a batch

The C ABI (include/gpk.h, libgpk.so) is the drop-in boundary; engine.py is
its thin object wrapper (device-resident batches via torch tensors).
"""
from . import _lib  # noqa: F401

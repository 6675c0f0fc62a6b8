#!/usr/bin/env python3
"""The reference's examples/statsassembly loop (main.go:128-209) over a capture
file, with the decode on the GPU.

The reference reads one packet at a time from a pcap handle, decodes it with
a DecodingLayerParser of Ethernet, Dot1Q, IPv4, IPv6, IPv6ExtensionSkipper,
TCP and Payload, takes the network flow of the last IPv4/IPv6 layer before
TCP, and hands the packet to tcpassembly. tcpassembly drops "useless" packets
(no SYN, FIN or RST and no payload, tcpassembly/assembly.go:537-543) and keys
the rest by key{netFlow, tcp.TransportFlow()} (:546).

Here a pcap or pcapng file is read in batches (pcapgo ReadBatch: the packets
the next ReadPacketData calls would return), each batch is decoded in one
launch (DecodingLayerParser.DecodeBatch), and the per-packet loop is the
reference's, over the layer structs as DecodeLayers leaves them (Hydrate).
The streams' statistics stand in for statsStream's (main.go:52-99): packets,
payload bytes, first and last capture time, and whether a SYN or a FIN/RST
was seen. tcpassembly's reassembly itself is out of scope, so
there are no out-of-order or skip counts.

--device-groups also forms the connection keys on the device
(gpk_group_batch, GPK_GROUP_CONNECTION) and checks that they split the
assembled packets exactly as the loop's keys do.

  python examples/statsassembly.py tests/golden/test_ethernet.pcap -v
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class StatsStream:
    """main.go:52-57, without the reassembly's ordering state."""

    def __init__(self, net, transport, seen):
        self.net, self.transport = net, transport
        self.bytes = self.packets = 0
        self.start = self.end = seen
        self.sawStart = self.sawEnd = False

    def assemble(self, tcp, seen):
        self.packets += 1
        self.bytes += len(tcp.LayerPayload())
        self.end = max(self.end, seen)
        self.sawStart = self.sawStart or tcp.SYN
        self.sawEnd = self.sawEnd or tcp.FIN or tcp.RST


def open_reader(f):
    from gopacket_amd import pcapgo
    magic = f.read(4)
    f.seek(0)
    return pcapgo.NewNgReader(f) if magic == b"\x0a\x0d\x0d\x0a" else pcapgo.NewReader(f)


def run(path, count=-1, batch=1 << 16, verbose=False, device_groups=False, log=print):
    """Returns (streams in order of first appearance, packets read, bytes of
    the packets decoded without error)."""
    from gopacket_amd import gopacket, layers, pcapgo
    eth, dot1q, ip4, ip6 = layers.Ethernet(), layers.Dot1Q(), layers.IPv4(), layers.IPv6()
    ip6extensions, tcp, payload = layers.IPv6ExtensionSkipper(), layers.TCP(), gopacket.Payload()
    parser = gopacket.NewDecodingLayerParser(layers.LayerTypeEthernet, eth, dot1q, ip4, ip6, ip6extensions, tcp,
                                             payload)
    decoded = []
    streams = {}  # key{netFlow, TransportFlow} -> StatsStream; dict order = the order streams were created
    read = byte_count = 0
    start = time.time()
    with open(path, "rb") as f:
        r = open_reader(f)
        while count != 0:
            try:
                b = r.ReadBatch(batch if count < 0 else min(batch, count))
            except pcapgo.EOFErrorGo:
                break
            except pcapgo.PcapgoError as e:  # the reference logs it and reads on; a file reader is done here
                log("error getting packet: %s" % e)
                break
            first = read
            read += len(b)
            if count > 0:
                count -= len(b)
            pb = gopacket.PacketBatch(b.data, b.offsets, b.caplens)
            res = parser.DecodeBatch(pb, layouts=True)
            assembled = []
            for i in range(len(pb)):
                err = res.Hydrate(i, decoded)
                if err is not None:
                    log("error decoding packet: %s" % err.Error())
                    continue
                if verbose:
                    log("decoded the following layers: [%s]" % " ".join(t.String() for t in decoded))
                byte_count += int(pb.caplens[i])
                seen = int(b.ci[i]["ts_sec"]) + int(b.ci[i]["ts_nsec"]) * 1e-9
                found_net, net_flow = False, None
                for typ in decoded:
                    if typ == layers.LayerTypeIPv4:
                        net_flow, found_net = ip4.NetworkFlow(), True
                    elif typ == layers.LayerTypeIPv6:
                        net_flow, found_net = ip6.NetworkFlow(), True
                    elif typ == layers.LayerTypeTCP:
                        if not found_net:
                            log("could not find IPv4 or IPv6 layer, inoring")
                        elif tcp.SYN or tcp.FIN or tcp.RST or len(tcp.LayerPayload()):  # assembly.go:537-543
                            key = (net_flow, tcp.TransportFlow())
                            s = streams.get(key)
                            if s is None:
                                log("new stream %s:%s started" % (key[0], key[1]))
                                s = streams[key] = StatsStream(key[0], key[1], seen)
                            s.assemble(tcp, seen)
                            assembled.append((i, key))
                        break
                else:
                    log("could not find TCP layer")
            if device_groups:
                check_device_groups(parser, pb, assembled)
    for s in streams.values():
        secs = s.end - s.start
        log("Reassembly of stream %s:%s complete - start:%.6f end:%.6f bytes:%d packets:%d bps:%s pps:%s "
            "sawStart:%s sawEnd:%s" % (s.net, s.transport, s.start, s.end, s.bytes, s.packets,
                                       "%.1f" % (s.bytes / secs) if secs > 0 else "+Inf",
                                       "%.1f" % (s.packets / secs) if secs > 0 else "+Inf",
                                       str(s.sawStart).lower(), str(s.sawEnd).lower()))
    log("processed %d bytes in %.3fs" % (byte_count, time.time() - start))
    return list(streams.values()), read, byte_count


def check_device_groups(parser, pb, assembled):
    """The same batch decoded and grouped on the device (gpk_group_batch,
    CONNECTION): every key of the loop must be exactly one device group and
    no two keys one group. The device also keys packets whose decode failed
    after TCP; the loop skips those (DecodeLayers returned an error), so only
    the loop's packets are compared."""
    import numpy as np
    import torch
    from gopacket_amd import flows
    n = len(pb)
    d = torch.from_numpy(np.concatenate([pb.data, np.zeros(16, np.uint8)])).cuda()
    o = torch.from_numpy(pb.offsets.astype(np.int64)).cuda()
    c = torch.from_numpy(pb.caplens.astype(np.int32)).cuda()
    rec = torch.empty(16 * n, dtype=torch.uint8, device="cuda")
    err = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
    fl = torch.empty(3 * n, dtype=torch.int64, device="cuda")
    lay = torch.empty(64 * n, dtype=torch.uint8, device="cuda")
    parser.ctx().decode_device(parser._config(), d, o, c, rec, err, fl, lay)
    g = flows.Grouper(max(n, 1))
    group_of = g.group(d, o, c, rec, layouts=lay, flows=fl, kind=flows.CONNECTION)["group_of"].cpu().numpy()
    g.close()
    key_of_group = {}
    group_of_key = {}
    for i, key in assembled:
        gid = int(group_of[i])
        if gid < 0 or key_of_group.setdefault(gid, key) != key or group_of_key.setdefault(key, gid) != gid:
            raise AssertionError("packet %d: device group %d, loop key %s:%s" % (i, gid, key[0], key[1]))


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("file", help="a pcap or pcapng capture")
    ap.add_argument("-c", type=int, default=-1, help="quit after this many packets (negative: all)")
    ap.add_argument("-v", action="store_true", help="log every packet's decoded layers")
    ap.add_argument("--batch", type=int, default=1 << 16, help="packets per DecodeBatch launch")
    ap.add_argument("--device-groups", action="store_true",
                    help="also group on the device (gpk_group_batch) and check it against the loop")
    a = ap.parse_args()
    run(a.file, a.c, a.batch, a.v, a.device_groups)


if __name__ == "__main__":
    main()

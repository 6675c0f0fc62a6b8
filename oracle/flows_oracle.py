"""Pure-Python restatement of the flow-keyed consumers of the decode path
(SURVEY.md §8(f)3): how tcpassembly and ip4defrag key the packets a
DecodingLayerParser hands them, and the FastHash sharding idiom of doc.go.

TEST INFRASTRUCTURE ONLY: imported by tests/ and bench.py as the checker of
gopacket_amd/csrc/gpk_flows.hip. The product package never imports it.

Input: the decode oracle's per-packet results (oracle/oracle.py: records with
the decoded list, layouts = the byte range each layer struct was last decoded
from, flows) and the packet bytes. Each layer struct's fields are read from
its range the way the reference's DecodeFromBytes sets them.

  tcpassembly/assembly.go:292      type key [2]gopacket.Flow
  tcpassembly/assembly.go:525-545  AssembleWithTimestamp: "ignoring useless
                                   packet" (no SYN/FIN/RST, empty payload), then
                                   key{netFlow, t.TransportFlow()} and the pool's
                                   map lookup (StreamPool.getConnection :498-517)
  ip4defrag/defrag.go:85-105       DefragIPv4WithTimestamp: dontDefrag (:160-170),
                                   securityChecks (:173-196, uint16 arithmetic),
                                   then ipFlows[ipv4{ip.NetworkFlow(), ip.Id}]
  ip4defrag/defrag.go:328-341      type ipv4 / newIPv4
  doc.go:219-225                   int(net.NetworkFlow().FastHash()) & 0x7
  flows.go:142-146, layers/ip4.go:63-65, ip6.go:49-51, tcp.go:614-616
                                   Flow values (type, src, dst) compared whole

Harness rules: netFlow = the last network layer in decoded
before TCP; a layer is keyed when it is in decoded; an IPv4 struct left
mid-decode by a failed IPv4 decode is not keyed for defrag.

group(): dict key -> packet indices in batch order, keys in order of first
appearance (a Python dict keeps insertion order), and a per-packet code.
"""
NONE, USELESS, FRAG_TOO_SMALL, FRAG_OFFSET, FRAG_OVERRUN, UNKNOWN = -1, -2, -3, -4, -5, -6
CONNECTION, DEFRAG, NET_BUCKET = 1, 2, 3

CODE_IP4, CODE_IP6, CODE_TCP = 3, 4, 9
SLOT_IP4, SLOT_IP6, SLOT_TCP = 2, 3, 5
ST_NET_FLOW = 1 << 26
ABSENT = 0xFFFFFFFF
IP4_ERRS = range(20, 28)


def _codes(layers_word, n):
    return [(int(layers_word) >> (4 * k)) & 15 for k in range(min(n, 16))]


def packet_key(kind, pkt, rec, lay, net_hash, buckets):
    status = int(rec["status"])
    nl = (status >> 8) & 0xFFF
    if kind == NET_BUCKET:
        if not status & ST_NET_FLOW:
            return NONE
        return ("bucket", int(net_hash) & (buckets - 1))
    start, end = lay["start"], lay["end"]
    if kind == CONNECTION:
        t0 = int(start[SLOT_TCP])
        if t0 == ABSENT:
            return NONE
        codes = _codes(rec["layers"], nl)
        if CODE_TCP not in codes:
            return UNKNOWN
        net = None
        for c in codes[:codes.index(CODE_TCP)]:
            if c in (CODE_IP4, CODE_IP6):
                net = c
        if net is None:
            return NONE
        tcp = pkt[t0:int(end[SLOT_TCP])]
        flags, doff = tcp[13], tcp[12] >> 4
        fin, syn, rst = flags & 1, flags & 2, flags & 4
        if not syn and not fin and not rst and len(tcp) - doff * 4 == 0:
            return USELESS
        if net == CODE_IP4:
            ip = pkt[int(start[SLOT_IP4]):]
            net_flow = (1, bytes(ip[12:16]), bytes(ip[16:20]))
        else:
            ip = pkt[int(start[SLOT_IP6]):]
            net_flow = (2, bytes(ip[8:24]), bytes(ip[24:40]))
        return ("conn", net_flow, (4, bytes(tcp[0:2]), bytes(tcp[2:4])))
    # DEFRAG
    s = int(start[SLOT_IP4])
    if s == ABSENT or (status & 0x7F) in IP4_ERRS:
        return NONE
    data = pkt[s:int(end[SLOT_IP4])]
    ff = data[6] << 8 | data[7]
    flags, fo = ff >> 13, ff & 0x1FFF
    if flags & 2:  # IPv4DontFragment
        return NONE
    if not flags & 1 and fo == 0:
        return NONE
    length = data[2] << 8 | data[3]
    if length == 0:
        length = len(data) & 0xFFFF
    ihl = data[0] & 15
    frag_size = (length - ihl * 4) & 0xFFFF
    if flags & 1 and frag_size < 8:
        return FRAG_TOO_SMALL
    if fo > 8183:
        return FRAG_OFFSET
    if ((fo * 8 + length) & 0xFFFF) > 65535:
        return FRAG_OVERRUN
    return ("frag", (1, bytes(data[12:16]), bytes(data[16:20])), data[4] << 8 | data[5])


def group(kind, packets, records, layouts, flows=None, buckets=8):
    """-> (groups: dict key -> [packet index], codes: per packet its group id, or a code < 0)."""
    n = len(packets)
    groups, codes = {}, [None] * n
    for i, pkt in enumerate(packets):
        k = packet_key(kind, pkt, records[i], layouts[i] if layouts is not None else None,
                       flows[n + i] if flows is not None else 0, buckets)
        if isinstance(k, int):
            codes[i] = k
        else:
            groups.setdefault(k, []).append(i)  # the map lookup; insertion order = first appearance
    for g, idx in enumerate(groups.values()):
        for i in idx:
            codes[i] = g
    return groups, codes

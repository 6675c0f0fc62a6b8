"""Parser configurations exercised by the parity tests (first LayerType,
decoders in Put order, options, table overrides)."""
ETH, D1Q, IP4, IP6, EXT, TCP, UDP, PAY, FRAG = ("ETHERNET", "DOT1Q", "IPV4", "IPV6", "IPV6_EXT", "TCP", "UDP",
                                                "PAYLOAD", "FRAGMENT")
DEC = dict(ETHERNET=1, DOT1Q=2, IPV4=3, IPV6=4, IPV6_EXT=5, TCP=6, UDP=7, PAYLOAD=8, FRAGMENT=9)

CONFIGS = {
    # layers/decode_test.go:192 / BASELINE C1, C3
    "eth_ip4_tcp_payload": dict(first=17, decoders=[ETH, IP4, TCP, PAY]),
    # BASELINE C2
    "eth_ip4_udp_payload": dict(first=17, decoders=[ETH, IP4, UDP, PAY]),
    # BASELINE C4 (examples/statsassembly/main.go:134-142 + UDP)
    "statsassembly": dict(first=17, decoders=[ETH, D1Q, IP4, IP6, EXT, TCP, UDP, PAY]),
    "statsassembly_ignore_unsupported": dict(first=17, decoders=[ETH, D1Q, IP4, IP6, EXT, TCP, UDP, PAY],
                                             ignore_unsupported=True),
    "raw_ip4": dict(first=20, decoders=[IP4, TCP, UDP, PAY]),
    "raw_ip6": dict(first=21, decoders=[IP6, EXT, TCP, UDP, PAY]),
    "first_unregistered": dict(first=22, decoders=[ETH, IP4]),
    "fragment_no_payload": dict(first=17, decoders=[ETH, D1Q, IP4, FRAG, TCP, UDP]),
    "overrides": dict(first=17, decoders=[ETH, D1Q, IP4, IP6, TCP, UDP, PAY],
                      ethertype={0x1234: 20}, tcp_port={80: 1234, 443: 2}, udp_port={53: 2},
                      ipprotocol={200: 44}),
    # 100 extra TCP ports: the compact LDS hash tables with collisions/probing
    "many_ports": dict(first=17, decoders=[ETH, IP4, IP6, TCP, UDP, PAY],
                       tcp_port={p: (2 if p % 3 else 1000 + p % 7) for p in range(1, 101)},
                       udp_port={p * 97 % 65536: 2 for p in range(1, 40)}),
    # 200 distinct LayerTypes: does not fit the compact tables, global tables used
    "tables_overflow": dict(first=17, decoders=[ETH, IP4, TCP, UDP, PAY],
                            tcp_port={p: 3000 + p for p in range(1, 201)}),
}


def oracle_parser(cfg):
    from oracle import oracle as O
    return O.OracleParser(cfg["first"], cfg["decoders"], ignore_unsupported=cfg.get("ignore_unsupported", False),
                          outputs=cfg.get("outputs", 7), ethertype=cfg.get("ethertype"),
                          ipprotocol=cfg.get("ipprotocol"), tcp_port=cfg.get("tcp_port"),
                          udp_port=cfg.get("udp_port"))


def device_parser(cfg):
    from gopacket_amd import engine
    p = engine.ParserConfig(cfg["first"], [DEC[d] for d in cfg["decoders"]],
                            ignore_unsupported=cfg.get("ignore_unsupported", False), outputs=cfg.get("outputs", 7))
    for k, v in (cfg.get("ethertype") or {}).items():
        p.set_ethertype(k, v)
    for k, v in (cfg.get("ipprotocol") or {}).items():
        p.set_ipprotocol(k, v)
    for k, v in (cfg.get("tcp_port") or {}).items():
        p.set_tcp_port(k, v)
    for k, v in (cfg.get("udp_port") or {}).items():
        p.set_udp_port(k, v)
    return p


def assert_same(dev, ref, what=""):
    """Bit-exact comparison of device and oracle results."""
    import numpy as np
    rd, rr = dev["records"], ref["records"]
    n = len(rr)
    bad = np.nonzero((rd["layers"] != rr["layers"]) | (rd["status"] != rr["status"]) |
                     (rd["ip4_csum"] != rr["ip4_csum"]) | (rd["l4_csum"] != rr["l4_csum"]))[0]
    assert len(bad) == 0, "%s: %d/%d records differ, first %s: dev=%s ref=%s" % (
        what, len(bad), n, bad[:5], rd[bad[:3]], rr[bad[:3]])
    err = (rr["status"] & 0x7F) != 0
    ea_d = dev["err_args"].reshape(n, 2)[err]
    ea_r = ref["err_args"].reshape(n, 2)[err]
    assert np.array_equal(ea_d, ea_r), "%s: err_args differ" % what
    assert np.array_equal(dev["flows"], ref["flows"]), "%s: flows differ" % what
    if dev.get("layouts") is not None and ref.get("layouts") is not None:
        assert np.array_equal(dev["layouts"]["start"], ref["layouts"]["start"]), "%s: layout start" % what
        assert np.array_equal(dev["layouts"]["end"], ref["layouts"]["end"]), "%s: layout end" % what

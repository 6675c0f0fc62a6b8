"""The flow-keyed grouping oracle (oracle/flows_oracle.py) pinned on
ip4defrag's own test frames and the field values of its struct-based tests,
and on tcpassembly's keying rules. CPU only: the oracle and the library's
exports; the device path is tests/test_flows_gpu.py."""
import numpy as np

import flowcases
import pktutil
from configs import oracle_parser
from oracle import flows_oracle as FO


def oracle_results(packets, cfg=flowcases.DEFRAG_PARSER):
    data, off, cap = pktutil.pack(packets)
    res = oracle_parser(cfg).decode(data, off, cap, layouts=True)
    return res


def test_defrag_frames_group_by_datagram():
    frames, same = flowcases.defrag_frames()
    # the injection order of TestDefragPing1and2 (defrag_test.go:110-131)
    order = ["testPing1Frag1", "testPing1Frag3", "testPing2Frag3", "testPing2Frag4", "testPing1Frag2",
             "testPing2Frag1", "testPing1Frag4", "testPing2Frag2"]
    pk = [frames[k] for k in order]
    res = oracle_results(pk)
    groups, codes = FO.group(FO.DEFRAG, pk, res["records"], res["layouts"])
    assert len(groups) == 2
    got = [sorted(order[i] for i in idx) for idx in groups.values()]
    assert got == [sorted(s) for s in same]
    # the key is ipv4{NetworkFlow, Id}: Id from the frames (TestDefragIDField, :264-276)
    k0 = list(groups)[0]
    assert k0[2] == int.from_bytes(frames["testPing1Frag1"][18:20], "big")
    assert codes == [0, 0, 1, 1, 0, 1, 0, 1]


def test_defrag_security_checks_and_dont_defrag():
    cases = flowcases.defrag_struct_cases()
    res = oracle_results([f for _, f in cases])
    _, codes = FO.group(FO.DEFRAG, [f for _, f in cases], res["records"], res["layouts"])
    want = {
        "TestNotFrag (DF)": FO.NONE,                        # returns in, nil (defrag_test.go:22-36)
        "TestDefragTooSmall Length 27 MF": FO.FRAG_TOO_SMALL,  # err (:153-165)
        "TestDefragTooSmall Length 28 MF": 0,               # ok (:167-170)
        "TestDefragSmallFinalFragment": FO.NONE,            # final, offset 0: not a fragment (:177-194)
        "TestDefragFragmentOffset 0": 0,
        "TestDefragFragmentOffset 8184": FO.FRAG_OFFSET,    # err (:210-220)
        "TestDefragMaxSize Length 65535": 0,                # ok (:235-249)
        "TestDefragMaxSize Length 28 off 1": 0,             # ok: uint16 sum never overruns (:251-261)
        "last fragment, offset 8183": 1,
        "TSO Length 0 with MF": 2,
        "Length 0, IHL 5, short": FO.FRAG_TOO_SMALL,  # Length = uint16(len(data)) = 22: fragment of 2
    }
    labels = [l for l, _ in cases]
    for l, c in zip(labels, codes):
        assert c == want[l], (l, c)


def test_connection_keys_are_directional_and_filter_useless():
    pk = flowcases.connection_cases()
    res = oracle_results(pk)
    groups, codes = FO.group(FO.CONNECTION, pk, res["records"], res["layouts"])
    assert codes == [0, 1, FO.USELESS, FO.USELESS, 0, 2, 2, 3, 0]
    keys = list(groups)
    assert keys[0][1][0] == 1 and keys[2][1][0] == 2 and keys[0][2][0] == 4
    assert keys[0][1][1] == keys[1][1][2]  # reversed direction: src <-> dst


def test_net_bucket_is_fasthash_low_bits():
    from gopacket_amd import synth
    data, off, cap = synth.host_batch(6, 0, 2000)
    pk = [bytes(data[o:o + c]) for o, c in zip(off, cap)]
    res = oracle_parser(flowcases.DEFRAG_PARSER).decode(data, off, cap, layouts=True)
    groups, codes = FO.group(FO.NET_BUCKET, pk, res["records"], res["layouts"], res["flows"], buckets=8)
    n = len(pk)
    for i in range(0, n, 97):
        if codes[i] >= 0:
            assert list(groups)[codes[i]][1] == int(res["flows"][n + i]) & 7
    # symmetric: both directions of a flow land in one bucket (doc.go:226-227)
    assert len(groups) == 8


def test_c6_traffic_has_repeating_flows_in_both_directions():
    from gopacket_amd import synth
    data, off, cap = synth.host_batch(6, 0, 20000)
    pk = [bytes(data[o:o + c]) for o, c in zip(off, cap)]
    res = oracle_parser(flowcases.DEFRAG_PARSER).decode(data, off, cap, layouts=True)
    groups, codes = FO.group(FO.CONNECTION, pk, res["records"], res["layouts"])
    sizes = sorted((len(v) for v in groups.values()), reverse=True)
    keyed = sum(1 for c in codes if c >= 0)
    assert sizes[0] > 20 and len(groups) < 0.97 * keyed
    assert codes.count(FO.USELESS) > 500
    fgroups, fcodes = FO.group(FO.DEFRAG, pk, res["records"], res["layouts"])
    assert len(fgroups) > 100 and max(len(v) for v in fgroups.values()) >= 2
    assert fcodes.count(FO.NONE) > 0.8 * len(pk)


def test_c_restatement_equals_python_oracle():
    """oracle/flows_oracle.c (the CPU baseline) keys exactly like the Python oracle."""
    from gopacket_amd import synth
    from oracle import oracle as O
    data, off, cap = synth.host_batch(6, 500, 30000)
    pk = [bytes(data[o:o + c]) for o, c in zip(off, cap)] + pktutil.fuzz_packets(8, 5000)
    frames, _ = flowcases.defrag_frames()
    pk += list(frames.values()) + [f for _, f in flowcases.defrag_struct_cases()] + flowcases.connection_cases()
    d, o, c = pktutil.pack(pk)
    res = oracle_parser(flowcases.DEFRAG_PARSER).decode(d, o, c, layouts=True)
    for kind, buckets in ((FO.CONNECTION, 8), (FO.DEFRAG, 8), (FO.NET_BUCKET, 8), (FO.NET_BUCKET, 256)):
        groups, codes = FO.group(kind, pk, res["records"], res["layouts"], res["flows"], buckets)
        g, out = O.group_batch(kind, d, o, res["records"], res["layouts"], res["flows"], buckets)
        assert g == len(groups) and out.tolist() == codes, kind

"""gpk_bpf_run / gpk_bpf_select (classic BPF on the device) against the
oracle (libpcap's bpf_filter restated): the reference's TestBPFInstruction
cases through BPF.Matches, hand-written programs over every opcode class and
random programs on fuzzed, golden and synthetic packets with wire lengths
different from the capture lengths, and the compacted selection."""
import numpy as np
import pytest

import bpfcases
import pktutil
from gopacket_amd import bpf, synth
from gopacket_amd.pcapgo import CaptureInfo
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def dev_batch(packets, wire=None):
    import torch
    data, off, cap = pktutil.pack(packets)
    d = torch.from_numpy(data).cuda()
    o = torch.from_numpy(off.astype(np.int64)).cuda()
    c = torch.from_numpy(cap.astype(np.int32)).cuda()
    w = torch.from_numpy(np.asarray(wire, np.int64).astype(np.int32)).cuda() if wire is not None else None
    return (data, off, cap), (d, o, c, w)


def test_reference_cases_through_matches(gpu_ctx):
    g = bpfcases.golden()
    pk = pktutil.read_pcap(pktutil.GOLDEN + "/test_ethernet.pcap")[1]
    for case in g["instruction_cases"]:
        if case["error"]:
            with pytest.raises(bpf.BPFError):
                bpf.NewBPFInstructionFilter(case["insns"] if not case["oversized"] else [(0, 0, 0, 0)] * 4097)
            continue
        f = bpf.NewBPFInstructionFilter([bpf.BPFInstruction(*x) for x in case["insns"]])
        data = pk[case["packet"]]
        assert f.Matches(CaptureInfo((0, 0), len(data), len(data)), data) == case["result"], case["filter"]
        assert f.String() == "BPF Instruction Filter"
        f.close()


def run_both(prog, packets, wire):
    (data, off, cap), (d, o, c, w) = dev_batch(packets, wire)
    f = bpf.NewBPFInstructionFilter(prog)
    got = f.Run(d, o, c, w).cpu().numpy().astype(np.uint32)
    ref = O.bpf_batch(prog, data, off, cap, wire)
    f.close()
    return got, ref


def test_programs_and_random_programs(gpu_ctx):
    rng = np.random.default_rng(23)
    pk = pktutil.fuzz_packets(41, 6000) + pktutil.read_pcap(pktutil.GOLDEN + "/test_ethernet.pcap")[1]
    pk += pktutil.read_pcap(pktutil.GOLDEN + "/test_dns.pcap")[1]
    hd, ho, hc = synth.host_batch(4, 3, 4000)
    pk += [bytes(hd[a:a + b]) for a, b in zip(ho, hc)]
    wire = [len(p) + (0 if k % 3 else int(rng.integers(0, 2000))) for k, p in enumerate(pk)]
    progs = [c["insns"] for c in bpfcases.golden()["instruction_cases"] if not c["error"]]
    progs += list(bpfcases.PROGRAMS.values())
    progs += [bpfcases.random_program(rng) for _ in range(150)]
    progs += [bpfcases.random_program(rng, n=400) for _ in range(5)]
    for prog in progs:
        got, ref = run_both(prog, pk, wire)
        bad = np.nonzero(got != ref)[0]
        assert len(bad) == 0, (prog, bad[:5], got[bad[:5]], ref[bad[:5]])


def test_select_compacts_matches_in_order(gpu_ctx):
    import torch
    prog = bpfcases.golden()["instruction_cases"][2]["insns"]  # tcp ack
    hd, ho, hc = synth.host_batch(4, 11, 300000)
    d = torch.from_numpy(hd).cuda()
    o = torch.from_numpy(ho.astype(np.int64)).cuda()
    c = torch.from_numpy(hc.astype(np.int32)).cuda()
    f = bpf.NewBPFInstructionFilter(prog)
    oo, oc, oi, cnt = f.Select(d, o, c)
    torch.cuda.synchronize()
    ref = O.bpf_batch(prog, hd, ho, hc)
    idx = np.nonzero(ref)[0]
    k = int(cnt.item())
    assert k == len(idx) and 0 < k < len(ho)
    assert np.array_equal(oi[:k].cpu().numpy(), idx)
    assert np.array_equal(oo[:k].cpu().numpy(), ho[idx].astype(np.int64))
    assert np.array_equal(oc[:k].cpu().numpy(), hc[idx].astype(np.int32))
    # empty batch
    oo, oc, oi, cnt = f.Select(d, o[:0], c[:0])
    torch.cuda.synchronize()
    assert int(cnt.item()) == 0
    f.close()


def test_non_terminating_program_stops(gpu_ctx):
    prog = [(0x05, 0, 0, 0xffffffff), (0x6, 0, 0, 1)]  # JA -1: jumps to itself for ever
    got, ref = run_both(prog, pktutil.fuzz_packets(3, 70), None)
    assert np.all(got == 0) and np.all(ref == 0)

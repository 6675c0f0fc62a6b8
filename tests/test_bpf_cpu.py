"""The classic-BPF oracle (oracle/bpf_oracle.c, libpcap's bpf_filter restated)
pinned on the reference's TestBPFInstruction programs and results, checked
against a second independent restatement on random programs; the
NewBPFInstructionFilter errors of the C ABI (argument checks run before any
device call)."""
import ctypes

import numpy as np
import pytest

import bpfcases
import pktutil
from gopacket_amd import _lib, bpf
from oracle import oracle as O


def ethernet_packets():
    return pktutil.read_pcap(pktutil.GOLDEN + "/test_ethernet.pcap")[1]


def test_reference_instruction_cases():
    g = bpfcases.golden()
    pk = ethernet_packets()
    seen = 0
    for case in g["instruction_cases"]:
        data = pk[case["packet"]]  # the test reads the next packet for every case
        if case["error"]:
            continue
        got = O.bpf_filter(case["insns"], data) != 0
        assert got == case["result"], case["filter"]
        seen += 1
    assert seen == 3


def test_create_errors_match_the_reference():
    L = _lib.lib()
    h = ctypes.c_void_p()
    err = ctypes.create_string_buffer(128)
    assert L.gpk_bpf_create(ctypes.byref(h), None, 0, err, 128) == _lib.GPK_EINVAL
    assert err.value == b"bpfInstructions must not be empty"
    big = np.zeros(4097, _lib.BPF_INSN_DTYPE)
    assert L.gpk_bpf_create(ctypes.byref(h), big.ctypes.data, 4097, err, 128) == _lib.GPK_EINVAL
    assert err.value == b"bpfInstructions must not be larger than 4096"
    with pytest.raises(bpf.BPFError, match="^bpfInstructions must not be empty$"):
        bpf.NewBPFInstructionFilter([])
    with pytest.raises(bpf.BPFError, match="^bpfInstructions must not be larger than 4096$"):
        bpf.NewBPFInstructionFilter([(0, 0, 0, 0)] * 4097)


def test_hand_written_programs():
    pk = ethernet_packets() + pktutil.fuzz_packets(5, 300)
    for name, prog in bpfcases.PROGRAMS.items():
        for p in pk:
            for wire in (len(p), len(p) + 100):
                assert O.bpf_filter(prog, p, wire) == bpfcases.py_bpf(prog, p, wire), (name, p.hex()[:40])
    p = ethernet_packets()[0]
    assert O.bpf_filter(bpfcases.PROGRAMS["backward_loop"], p) == 3
    assert O.bpf_filter(bpfcases.PROGRAMS["fall_off"], p) == 0
    assert O.bpf_filter(bpfcases.PROGRAMS["bad_opcode"], p) == 0
    assert O.bpf_filter(bpfcases.PROGRAMS["div_by_zero"], p) == 0
    assert O.bpf_filter(bpfcases.PROGRAMS["len_gt_500_ret_a"], p, 600) == 600


def test_random_programs_two_restatements_agree():
    rng = np.random.default_rng(17)
    pk = pktutil.fuzz_packets(6, 200) + ethernet_packets()
    for _ in range(400):
        prog = bpfcases.random_program(rng)
        for p in pk[::7]:
            wire = len(p) + int(rng.integers(0, 3)) * 50
            assert O.bpf_filter(prog, p, wire) == bpfcases.py_bpf(prog, p, wire), prog

"""Classic BPF programs for the filter tests: the reference's own
(tests/golden/bpf_programs.json, harvested from pcap_test.go), hand-written
tcpdump -dd style programs over every opcode class, and a random program
generator (forward jumps only unless asked; in-range and out-of-range loads,
scratch memory, division by zero, shifts >= 32)."""
import json
import os

import numpy as np

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bpf_programs.json")


def golden():
    return json.load(open(GOLD))


# tcpdump -dd style programs (hand-assembled)
PROGRAMS = {
    # ip and tcp and dst port 80 (IPv4 only, fragment check, MSH)
    "ip_tcp_dport80": [(0x28, 0, 0, 12), (0x15, 0, 8, 0x800), (0x30, 0, 0, 23), (0x15, 0, 6, 6),
                       (0x28, 0, 0, 20), (0x45, 4, 0, 0x1fff), (0xb1, 0, 0, 14), (0x48, 0, 0, 16),
                       (0x15, 0, 1, 80), (0x6, 0, 0, 0x40000), (0x6, 0, 0, 0)],
    # vlan-aware: skip one 802.1Q tag, then ip6
    "vlan_ip6": [(0x28, 0, 0, 12), (0x15, 0, 3, 0x8100), (0x28, 0, 0, 16), (0x15, 0, 1, 0x86dd),
                 (0x6, 0, 0, 262144), (0x6, 0, 0, 0)],
    # len > 500 via LEN and X compare, TAX/TXA, return A
    "len_gt_500_ret_a": [(0x80, 0, 0, 0), (0x07, 0, 0, 0), (0x87, 0, 0, 0), (0x01, 0, 0, 500),
                         (0x2d, 0, 1, 0), (0x16, 0, 0, 0), (0x6, 0, 0, 0)],
    # scratch memory and ALU: A = (p[14] & 0xf) * 4 + p[23]; mem; compare
    "alu_mem": [(0x30, 0, 0, 14), (0x54, 0, 0, 0xf), (0x64, 0, 0, 2), (0x02, 0, 0, 3), (0x30, 0, 0, 23),
                (0x07, 0, 0, 0), (0x60, 0, 0, 3), (0x0c, 0, 0, 0), (0x94, 0, 0, 7), (0x74, 0, 0, 1),
                (0x84, 0, 0, 0), (0xa4, 0, 0, 0xffffffff), (0x16, 0, 0, 0)],
    # division by X = 0 -> no match; LD W IND at the end of the packet
    "div_by_zero": [(0x01, 0, 0, 0), (0x00, 0, 0, 10), (0x3c, 0, 0, 0), (0x6, 0, 0, 1)],
    "ind_tail": [(0x80, 0, 0, 0), (0x14, 0, 0, 4), (0x07, 0, 0, 0), (0x40, 0, 0, 0), (0x16, 0, 0, 0)],
    # JA over instructions, shifts by X >= 32, JSET X
    "ja_shift": [(0x05, 0, 0, 2), (0x6, 0, 0, 7), (0x6, 0, 0, 8), (0x01, 0, 0, 40), (0x00, 0, 0, 0xff),
                 (0x6c, 0, 0, 0), (0x15, 0, 1, 0), (0x6, 0, 0, 9), (0x6, 0, 0, 10)],
    # a backward jump (as ip6 protochain emits): loop three times over a counter in M[0]
    "backward_loop": [(0x00, 0, 0, 0), (0x02, 0, 0, 0), (0x60, 0, 0, 0), (0x04, 0, 0, 1), (0x02, 0, 0, 0),
                      (0x15, 1, 0, 3), (0x05, 0, 0, 0xfffffffa), (0x16, 0, 0, 0)],
    # falls off the end / unknown opcode / mem index out of range
    "fall_off": [(0x00, 0, 0, 1)],
    "bad_opcode": [(0xff, 0, 0, 0), (0x6, 0, 0, 1)],
    "mem_oob": [(0x02, 0, 0, 16), (0x6, 0, 0, 1)],
}

OPS_K = [0x04, 0x14, 0x24, 0x34, 0x94, 0x54, 0x44, 0xa4, 0x64, 0x74]
OPS_X = [0x0c, 0x1c, 0x2c, 0x3c, 0x9c, 0x5c, 0x4c, 0xac, 0x6c, 0x7c]
LOADS = [0x20, 0x28, 0x30, 0x40, 0x48, 0x50, 0xb1]
JUMPS = [0x25, 0x35, 0x15, 0x45, 0x2d, 0x3d, 0x1d, 0x4d]


def random_program(rng, n=None):
    n = n or int(rng.integers(2, 40))
    prog = []
    for pc in range(n - 1):
        r = rng.random()
        room = n - pc - 2  # jump targets stay inside the program
        if r < 0.3:
            op = int(rng.choice(LOADS))
            k = int(rng.choice([rng.integers(0, 80), rng.integers(0, 1600), 0xfffffff0, 1 << 31]))
            prog.append((op, 0, 0, k))
        elif r < 0.5:
            op = int(rng.choice(OPS_K + OPS_X))
            k = int(rng.choice([0, 1, 3, 31, 32, 40, rng.integers(0, 1 << 32)]))
            prog.append((op, 0, 0, k))
        elif r < 0.7 and room > 0:
            op = int(rng.choice(JUMPS))
            prog.append((op, int(rng.integers(0, min(room, 255) + 1)), int(rng.integers(0, min(room, 255) + 1)),
                         int(rng.choice([0, 0x800, 6, 17, rng.integers(0, 1 << 32)]))))
        elif r < 0.75 and room > 0:
            prog.append((0x05, 0, 0, int(rng.integers(0, room + 1))))
        elif r < 0.85:
            prog.append((int(rng.choice([0x00, 0x01, 0x80, 0x81, 0x07, 0x87, 0x84])), 0, 0,
                         int(rng.integers(0, 1 << 32))))
        elif r < 0.93:
            prog.append((int(rng.choice([0x02, 0x03, 0x60, 0x61])), 0, 0, int(rng.integers(0, 17))))
        else:
            prog.append((int(rng.choice([0x06, 0x16])), 0, 0, int(rng.integers(0, 3))))
    prog.append((int(rng.choice([0x06, 0x16])), 0, 0, int(rng.integers(0, 1 << 32))))
    return prog


def py_bpf(prog, p, wirelen):
    """A second, independent restatement of libpcap's bpf_filter (for the oracle's own test)."""
    M32 = 0xFFFFFFFF
    A = X = 0
    mem = [0] * 16
    pc = 0
    buflen = len(p)
    for _ in range(1 << 20):
        if pc >= len(prog):
            return 0
        c, jt, jf, k = prog[pc]
        if c == 0x06:
            return k
        if c == 0x16:
            return A
        if c in (0x20, 0x28, 0x30, 0x40, 0x48, 0x50):
            size = {0x20: 4, 0x28: 2, 0x30: 1, 0x40: 4, 0x48: 2, 0x50: 1}[c]
            off = k if c < 0x40 else (X + k) & M32
            if c >= 0x40 and (k + X) > M32:  # the u32 sum wraps: libpcap's checks fail it
                return 0
            if off + size > buflen:
                return 0
            A = int.from_bytes(p[off:off + size], "big")
        elif c == 0xb1:
            if k >= buflen:
                return 0
            X = (p[k] & 0xf) << 2
        elif c == 0x80:
            A = wirelen
        elif c == 0x81:
            X = wirelen
        elif c == 0x00:
            A = k
        elif c == 0x01:
            X = k
        elif c in (0x60, 0x61, 0x02, 0x03):
            if k >= 16:
                return 0
            if c == 0x60:
                A = mem[k]
            elif c == 0x61:
                X = mem[k]
            elif c == 0x02:
                mem[k] = A
            else:
                mem[k] = X
        elif c == 0x05:
            pc = (pc + k) & M32
        elif c in JUMPS:
            v = k if c & 0x08 == 0 else X
            cond = {0x20: A > v, 0x30: A >= v, 0x10: A == v, 0x40: (A & v) != 0}[c & 0xf0]
            pc += jt if cond else jf
        elif c in OPS_K or c in OPS_X:
            v = k if c in OPS_K else X
            op = c & 0xf0
            if op in (0x30, 0x90) and v == 0:
                return 0
            if op in (0x60, 0x70):
                if c in OPS_X and v >= 32:
                    A = 0
                else:
                    s = v & 31
                    A = (A << s) & M32 if op == 0x60 else A >> s
            else:
                A = {0x00: A + v, 0x10: A - v, 0x20: A * v, 0x30: A // max(v, 1), 0x90: A % max(v, 1),
                     0x50: A & v, 0x40: A | v, 0xa0: A ^ v}[op] & M32
        elif c == 0x84:
            A = (-A) & M32
        elif c == 0x07:
            X = A
        elif c == 0x87:
            A = X
        else:
            return 0
        pc += 1
    return 0

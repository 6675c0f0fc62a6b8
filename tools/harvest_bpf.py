#!/usr/bin/env python3
"""Harvest the classic-BPF programs of pcap/pcap_test.go's TestBPFInstruction
(:154-262) as data into tests/golden/bpf_programs.json: each case's
instructions, whether NewBPFInstructionFilter must fail, the expected
BPF.Matches result, and the test_ethernet.pcap packet the test reads for it
(case k reads packet k-1). Also the expression-filter cases of TestBPF
(:119-152; libpcap would compile them, absent here) for the record. Reads the
reference source as text only."""
import json
import os
import re

SRC = "/root/reference/pcap/pcap_test.go"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "bpf_programs.json")


def main():
    src = open(SRC).read()
    body = src[src.index("func TestBPFInstruction"):src.index("func ExampleBPF")]
    cases = []
    for m in re.finditer(r'\{"([^"]*)",\s*(\[\]BPFInstruction\{(.*?)\}|oversizedBpfInstructionBuffer\[:\]),\s*(true|false),\s*(true|false)\}',
                         body, re.S):
        insns = [[int(a, 16), int(b), int(c), int(d, 16)] for a, b, c, d in
                 re.findall(r"\{(0x[0-9a-fA-F]+), (\d+), (\d+), (0x[0-9a-fA-F]+)\}", m.group(3) or "")]
        oversized = m.group(2).startswith("oversized")
        cases.append(dict(filter=m.group(1), insns=insns, oversized=oversized, error=m.group(4) == "true",
                          result=m.group(5) == "true", packet=len(cases)))
    assert len(cases) == 5, cases
    tb = src[src.index("func TestBPF("):src.index("func TestBPFInstruction")]
    exprs = [dict(expr=a, error=b == "true", result=c == "true", packet=i)
             for i, (a, b, c) in enumerate(re.findall(r'\{"([^"]*)", (true|false), (true|false)\}', tb))]
    json.dump({"source": "pcap/pcap_test.go:154-262 (TestBPFInstruction), :119-152 (TestBPF)",
               "max_bpf_instructions": 4096, "pcap": "tests/golden/test_ethernet.pcap",
               "instruction_cases": cases, "expression_cases_unpinned": exprs}, open(OUT, "w"), indent=1)
    print("wrote", OUT, [(c["filter"], len(c["insns"]), c["error"], c["result"]) for c in cases])


if __name__ == "__main__":
    main()

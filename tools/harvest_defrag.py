#!/usr/bin/env python3
"""Harvest ip4defrag's test frames (ip4defrag/defrag_test.go:304-1499,
testPing{1,2}Frag{1..4}) as data into tests/golden/defrag_frames.json, with
what the reference's tests assert about them (TestDefragPing1and2 :106-151:
the four fragments of each ping reassemble together, the two pings apart).
Reads the reference source as text only; nothing of it is executed."""
import json
import os
import re

SRC = "/root/reference/ip4defrag/defrag_test.go"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "defrag_frames.json")


def main():
    src = open(SRC).read()
    frames = {}
    for m in re.finditer(r"var (testPing\dFrag\d) = \[\]byte\{(.*?)\n\}", src, re.S):
        body = re.sub(r"//[^\n]*", "", m.group(2))
        vals = [int(x, 16) for x in re.findall(r"0x([0-9a-fA-F]{2})", body)]
        frames[m.group(1)] = bytes(vals).hex()
    assert len(frames) == 8, sorted(frames)
    json.dump({"source": "ip4defrag/defrag_test.go:304-1499", "frames": frames,
               "same_datagram": [["testPing1Frag1", "testPing1Frag2", "testPing1Frag3", "testPing1Frag4"],
                                 ["testPing2Frag1", "testPing2Frag2", "testPing2Frag3", "testPing2Frag4"]]},
              open(OUT, "w"), indent=1)
    print("wrote", OUT, {k: len(v) // 2 for k, v in frames.items()})


if __name__ == "__main__":
    main()

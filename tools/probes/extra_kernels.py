"""One launch each of the row (f)3/(f)4 kernels on 16 M packets, for rocprofv3
PMC passes (HBM bytes per packet): BPF (tcp ack program) over C4, grouping
(connection key) over C6 decoded with layouts."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from gopacket_amd import bpf, engine, flows, synth  # noqa: E402

n = 16 << 20
ctx = engine.Context(0)
d, o, c = synth.device_batch(4, 0, n)
g = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests", "golden",
                                "bpf_programs.json")))
prog = g["instruction_cases"][2]["insns"]
f = bpf.NewBPFInstructionFilter(prog)
for _ in range(2):
    f.Run(d, o, c)
torch.cuda.synchronize()
del d, o, c
d, o, c = synth.device_batch(6, 0, n)
parser = engine.ParserConfig(17, [1, 2, 3, 4, 5, 6, 7, 8], outputs=7)
rec = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
err = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
fl = torch.zeros(3 * n, dtype=torch.int64, device="cuda")
lay = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
ctx.decode_device(parser, d, o, c, rec, err, fl, lay)
gr = flows.Grouper(n)
for _ in range(2):
    gr.group(d, o, c, rec, lay, fl, kind=flows.CONNECTION)
torch.cuda.synchronize()
print("ok", n)

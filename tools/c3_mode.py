"""C3's two speeds by allocation, for PMC passes: K
fresh allocations of the 100 GB C3 batch in one process (torch's allocator,
the cache emptied between them), each generated, warmed with 2 launches and
timed over 4 single launches (HIP events around each: per-dispatch PMC
collection adds microseconds to a 16-18 ms kernel). Prints one line per
allocation; under rocprofv3 --pmc the decode dispatches come in the same
order, 6 per allocation (tools/c3_mode_pmc.sh pairs them)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
from gopacket_amd import engine, synth  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 4
ctx = engine.Context(0)
cfg = bench.CONFIGS["c3"]
parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in cfg["decoders"]], outputs=cfg["outputs"])
n = 64 * 2**20
stream = torch.cuda.current_stream()
rec = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
err = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
fl = torch.empty(3 * n, dtype=torch.int64, device="cuda")
for k in range(K):
    data, off, cap = synth.device_batch(3, 0, n, stream=stream)
    ts = []
    for j in range(6):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        ctx.decode_device(parser, data, off, cap, rec, err, fl, stream=stream)
        e1.record(stream)
        torch.cuda.synchronize()
        if j >= 2:
            ts.append(e0.elapsed_time(e1))
    print("alloc %d at %#x: %.3f ms (%s)" % (k, data.data_ptr(), float(np.median(ts)),
                                         " ".join("%.3f" % t for t in ts)), flush=True)
    del data, off, cap
    torch.cuda.empty_cache()

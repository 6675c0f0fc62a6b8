"""C3 timing against the batch's placement inside one allocation (diagnostic):
the same 100 GB batch generated at shifts of 0 .. 1 MiB from the start of a
fixed allocation, plus the allocation's device address."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from gopacket_amd import _lib, engine, synth  # noqa: E402

ctx = engine.Context(0)
cfg = bench.CONFIGS["c3"]
parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in cfg["decoders"]], outputs=cfg["outputs"])
n = 64 * 2**20
stream = torch.cuda.current_stream()
total = synth.total_bytes(3, 0, n) + 256
buf = torch.empty(total + (4 << 20), dtype=torch.uint8, device="cuda")
off = torch.empty(n, dtype=torch.int64, device="cuda")
cap = torch.empty(n, dtype=torch.int32, device="cuda")
rec = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
err = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
fl = torch.empty(3 * n, dtype=torch.int64, device="cuda")
print("allocation at 0x%x" % buf.data_ptr(), flush=True)
for shift in (0, 4096, 65536, 1 << 19, 1 << 20, 3 << 20, 0):
    data = buf[shift:shift + total]
    assert _lib.synth_lib().gpk_synth_device(3, 0, n, data.data_ptr(), off.data_ptr(), cap.data_ptr(),
                                             stream.cuda_stream) == 0

    def step():
        ctx.decode_device(parser, data, off, cap, rec, err, fl, stream=stream)
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(20):
        step()
    e1.record(stream)
    torch.cuda.synchronize()
    print("shift %8d (addr %% 2 MiB = %7d): %.3f ms" % (shift, data.data_ptr() % (2 << 20), e0.elapsed_time(e1) / 20),
          flush=True)

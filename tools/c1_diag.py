"""C1: bench.run_config's timing vs a direct gpk_decode_batch loop on the same tensors (diagnostic)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from gopacket_amd import _lib, engine  # noqa: E402

ctx = engine.Context(0)
cfg = bench.CONFIGS["c1"]
kinds = [engine.DECODER_KINDS[d] for d in cfg["decoders"]]
parser = engine.ParserConfig(17, kinds, outputs=cfg["outputs"])
n = cfg["packets"]
data, off, cap = bench.pcap_tiled(cfg["pcap"], n)
rec = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
err = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
stream = torch.cuda.current_stream()
L = _lib.lib()
b = _lib.Batch(data.data_ptr(), off.data_ptr(), cap.data_ptr(), n, data.numel())
r = _lib.Results(rec.data_ptr(), err.data_ptr(), None, None)


def t_engine(steps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        ctx.decode_device(parser, data, off, cap, rec, err, None, stream=stream)
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def t_direct(steps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        assert L.gpk_decode_batch(ctx.h, parser.h, ctypes.byref(b), ctypes.byref(r), ctypes.c_void_p(stream.cuda_stream)) == 0
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


for f in (t_engine, t_direct):
    f(3)
for rnd in range(3):
    print("engine %.4f ms  direct %.4f ms  engine(5) %.4f  direct(5) %.4f" % (t_engine(20), t_direct(20), t_engine(5),
                                                                         t_direct(5)), flush=True)

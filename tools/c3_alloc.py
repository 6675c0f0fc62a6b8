"""C3 timing against the allocation of its 100 GB batch (diagnostic): torch's
allocator three times in one process, then hipExtMallocWithFlags with
hipDeviceMallocContiguous, each filled by the same generator and timed like
bench.py (20 launches after a warmup)."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from gopacket_amd import _lib, engine, synth  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
ctx = engine.Context(0)
cfg = bench.CONFIGS["c3"]
parser = engine.ParserConfig(17, [engine.DECODER_KINDS[d] for d in cfg["decoders"]], outputs=cfg["outputs"])
n = 64 * 2**20
stream = torch.cuda.current_stream()


class Raw:
    def __init__(self, p, nbytes):
        self.p, self.nbytes = p, nbytes

    def data_ptr(self):
        return self.p

    def numel(self):
        return self.nbytes


def timeit(data, off, cap, rec, err, fl):
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
    return e0.elapsed_time(e1) / 20


rec = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
err = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
fl = torch.empty(3 * n, dtype=torch.int64, device="cuda")
for k in range(3):
    data, off, cap = synth.device_batch(3, 0, n, stream=stream)
    print("torch alloc %d: %.3f ms" % (k, timeit(data, off, cap, rec, err, fl)), flush=True)
    del data, off, cap
    torch.cuda.empty_cache()
total = synth.total_bytes(3, 0, n) + 256
for flag, name in ((0x4, "contiguous"), (0x0, "hipExtMalloc default")):
    p = ctypes.c_void_p()
    rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(total), ctypes.c_uint(flag))
    if rc != 0:
        print("%s: hipExtMallocWithFlags rc %d" % (name, rc), flush=True)
        continue
    off = torch.empty(n, dtype=torch.int64, device="cuda")
    cap = torch.empty(n, dtype=torch.int32, device="cuda")
    assert _lib.synth_lib().gpk_synth_device(3, 0, n, p.value, off.data_ptr(), cap.data_ptr(), stream.cuda_stream) == 0
    print("%s: %.3f ms" % (name, timeit(Raw(p.value, total), off, cap, rec, err, fl)), flush=True)
    torch.cuda.synchronize()
    hip.hipFree(p)

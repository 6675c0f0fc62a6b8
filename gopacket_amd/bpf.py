"""pcap-shaped classic BPF filters evaluated on the device (include/gpk_bpf.h,
SURVEY.md §8(f)4).

  BPFInstruction(Code, Jt, Jf, K)           pcap.BPFInstruction (pcap/pcap.go:146-151)
  MaxBpfInstructions                        pcap.go:36
  NewBPFInstructionFilter(insns) -> BPF     Handle.NewBPFInstructionFilter (pcap.go:565-576)
  BPF.Matches(ci, data)                     BPF.Matches (pcap.go:599-601)
  BPF.String()                              "BPF Instruction Filter" (pcap.go:568)
  BPF.Run(batch tensors) / BPF.Select(...)  the batch forms (gpk_bpf_run / gpk_bpf_select)

Every evaluation runs the HIP kernel; there is no CPU path.
"""
import ctypes
from collections import namedtuple

import numpy as np

from . import _lib

MaxBpfInstructions = _lib.BPF_MAX_INSNS
BPFInstruction = namedtuple("BPFInstruction", "Code Jt Jf K")


class BPFError(Exception):
    pass


def _insn_array(insns):
    arr = np.zeros(len(insns), _lib.BPF_INSN_DTYPE)
    for i, x in enumerate(insns):
        arr[i] = (int(x[0]) & 0xFFFF, int(x[1]) & 0xFF, int(x[2]) & 0xFF, int(x[3]) & 0xFFFFFFFF)
    return arr


class BPF:
    def __init__(self, insns, orig="BPF Instruction Filter"):
        self.orig = orig
        self.insns = _insn_array(insns)
        self.h = ctypes.c_void_p()
        err = ctypes.create_string_buffer(256)
        rc = _lib.lib().gpk_bpf_create(ctypes.byref(self.h), self.insns.ctypes.data if len(insns) else None,
                                       len(insns), err, 256)
        if rc != _lib.GPK_OK:
            self.h = None
            if rc == _lib.GPK_EINVAL and err.value:  # the reference's error text
                raise BPFError(err.value.decode())
            _lib.check(rc)

    def String(self):
        return self.orig

    def Run(self, data, offsets, caplens, wirelens=None, ret=None, stream=None):
        """ret[i] = the filter's return value for packet i (torch device tensors)."""
        import torch
        n = offsets.numel()
        if ret is None:
            ret = torch.empty(n, dtype=torch.int32, device=offsets.device)
        b = _lib.Batch(data.data_ptr(), offsets.data_ptr(), caplens.data_ptr(), n, data.numel())
        sp = None if stream is None else (stream if isinstance(stream, int) else stream.cuda_stream)
        _lib.check(_lib.lib().gpk_bpf_run(self.h, ctypes.byref(b), wirelens.data_ptr() if wirelens is not None
                                          else None, ret.data_ptr(), sp))
        return ret

    def Select(self, data, offsets, caplens, wirelens=None, stream=None):
        """The matching packets: (offsets, caplens, index, count) device tensors, batch order."""
        import torch
        n = offsets.numel()
        dev = offsets.device
        oo = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        oc = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        oi = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        cnt = torch.zeros(1, dtype=torch.int32, device=dev)
        b = _lib.Batch(data.data_ptr(), offsets.data_ptr(), caplens.data_ptr(), n, data.numel())
        sp = None if stream is None else (stream if isinstance(stream, int) else stream.cuda_stream)
        _lib.check(_lib.lib().gpk_bpf_select(self.h, ctypes.byref(b), wirelens.data_ptr() if wirelens is not None
                                             else None, oo.data_ptr(), oc.data_ptr(), oi.data_ptr(), cnt.data_ptr(),
                                             sp))
        return oo, oc, oi, cnt

    def Matches(self, ci, data):
        """One packet (gopacket.CaptureInfo-like with .Length, bytes): run on the device."""
        import torch
        data = bytes(data)
        d = torch.zeros(max(len(data), 1) + 16, dtype=torch.uint8, device="cuda")
        if data:
            d[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
        off = torch.zeros(1, dtype=torch.int64, device="cuda")
        cap = torch.full((1,), len(data), dtype=torch.int32, device="cuda")
        wire = torch.full((1,), int(ci.Length), dtype=torch.int32, device="cuda")
        return int(self.Run(d, off, cap, wire)[0].item()) != 0

    def close(self):
        if self.h:
            _lib.lib().gpk_bpf_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def NewBPFInstructionFilter(insns):
    return BPF(insns)

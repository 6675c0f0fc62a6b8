"""Synthetic benchmark batches: C2 64 B UDP, C3 1500 B TCP,
C4 IMIX with VLAN tags and IPv6. Deterministic per packet index, generated
identically on the host (for oracle sampling) and on the device (C3 at 64 M
packets is ~100 GB: generated in HBM, never copied).
"""
import numpy as np

from . import _lib

C2_UDP64, C3_TCP1500, C4_IMIX = 2, 3, 4
NAMES = {C2_UDP64: "C2-udp64", C3_TCP1500: "C3-tcp1500", C4_IMIX: "C4-imix-vlan-v4v6"}


def packet(cfg, i):
    S = _lib.synth_lib()
    buf = np.zeros(2048, np.uint8)
    n = S.gpk_synth_fill(cfg, i, buf.ctypes.data)
    return bytes(buf[:n])


def host_batch(cfg, first, n):
    """Packed host batch of packets [first, first+n): (data, offsets, caplens)."""
    S = _lib.synth_lib()
    total = S.gpk_synth_batch_host(cfg, first, n, None, None, None)
    data = np.zeros(total + 16, np.uint8)
    offsets = np.zeros(n, np.uint64)
    caplens = np.zeros(n, np.uint32)
    S.gpk_synth_batch_host(cfg, first, n, data.ctypes.data, offsets.ctypes.data, caplens.ctypes.data)
    return data, offsets, caplens


def total_bytes(cfg, first, n):
    return int(_lib.synth_lib().gpk_synth_bytes(cfg, first, n))


def device_batch(cfg, first, n, device="cuda", stream=None):
    """Device batch in HBM as torch tensors (data, offsets, caplens)."""
    import torch
    total = total_bytes(cfg, first, n)
    data = torch.empty(total + 256, dtype=torch.uint8, device=device)
    offsets = torch.empty(n, dtype=torch.int64, device=device)
    caplens = torch.empty(n, dtype=torch.int32, device=device)
    s = stream if stream is not None else torch.cuda.current_stream()
    rc = _lib.synth_lib().gpk_synth_device(cfg, first, n, data.data_ptr(), offsets.data_ptr(), caplens.data_ptr(),
                                           s.cuda_stream)
    if rc != 0:
        raise RuntimeError("gpk_synth_device failed: %d" % rc)
    return data, offsets, caplens

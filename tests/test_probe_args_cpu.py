"""The skeleton probes reject, before any launch, a write form that would
store past the buffer they are given (round 4's probe
fault stored flows into a 16-byte-per-packet buffer). No GPU needed: every
rejected call returns -1 before touching HIP."""
import pytest

from gopacket_amd import _lib

N = 1 << 20


@pytest.fixture(scope="module")
def S():
    return _lib.synth_lib()


@pytest.mark.parametrize("wbytes,flags,size", [
    (40, 2, 16 * N),          # flows into a records-only buffer
    (40, 2 | 256, 16 * N),    # the round-4 fault: wave-0 form, flows past a 16 B/packet buffer
    (16, 2 | 512, 16 * N),    # interleaved form needs 40 B per packet
    (168, 2, 40 * N),         # fields past a 40 B/packet buffer
    (24, 2, 40 * N),          # not a form
    (0, 2 | 256, 16 * N),     # the wave-0 form stores 16-byte records whatever wbytes says
    (8, 2 | 512, 40 * N),     # the interleaved form is the 40-byte one
    (32, 2, 16 * N),          # narrow records + flows past a 16 B/packet buffer
])
def test_skeleton_rejects_overrun(S, wbytes, flags, size):
    assert S.gpk_probe_skeleton_idx(16, 16, 16, N, 16, size, wbytes, flags, 16, None) == -1


def test_storer_rejects_overrun(S):
    assert S.gpk_probe_skeleton_storer(16, 16, 16, N, 16, 16 * N, 40, 16, None) == -1
    assert S.gpk_probe_skeleton_storer(16, 16, 16, N, 16, 168 * N, 168, 16, None) == -1

"""The root package's helpers around the hot path in the host mirror
(gopacket_amd/gopacket.py): ComputeChecksum / FoldChecksum (checksum.go:35-58),
the LayerType registry (layertype.go:22-111) and the LayerClass forms
(layerclass.go:9-107). Pinned by checksum_test.go:16-50's known answers and
by the device: the mirror's checksum of a packet equals the Correct value of
the engine's decode of it (tests/test_gopacket_api_gpu.py for the device side;
here against the CPU oracle, which the GPU parity tests pin to the device)."""
import numpy as np
import pytest

import pktutil
from gopacket_amd import gopacket as G
from oracle import oracle as O


@pytest.mark.parametrize("name,want", [("cksum_two_carries", 0xfffe), ("cksum_wikipedia", 0xb861)])
def test_checksum_known_answers(name, want):
    """checksum_test.go:16-50 (the IPv4 header with its checksum field zeroed)."""
    b = bytearray(pktutil.golden_bytes(name))
    b[10] = b[11] = 0
    assert G.FoldChecksum(G.ComputeChecksum(bytes(b))) == want


def test_checksum_against_oracle_and_wrap():
    rng = np.random.default_rng(5)
    for n in (0, 1, 2, 3, 57, 1500, 65537, 262145):
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for c0 in (0, 1, 0xFFFF, 0xFFFFFFFF - 3):
            assert G.ComputeChecksum(d, c0) == O.compute_checksum(d, c0)
            assert G.FoldChecksum(G.ComputeChecksum(d, c0)) == O.fold_checksum(O.compute_checksum(d, c0))
    # the sum is a uint32: 70000 words of 0xffff wrap past 2^32 (checksum.go keeps adding)
    assert G.ComputeChecksum(b"\xff\xff" * 70000) == (0xFFFF * 70000) % (1 << 32)
    assert G.FoldChecksum(0) == 0xFFFF and G.FoldChecksum(0xFFFF) == 0 and G.FoldChecksum(0x1FFFE) == 0


def test_layer_type_registry():
    t = G.RegisterLayerType(1777, G.LayerTypeMetadata("Gpk1777"))
    assert t.String() == "Gpk1777" and G.DecodersByLayerName["Gpk1777"] is None
    assert G.UnsupportedLayerType(t).Error() == "No decoder for layer type Gpk1777"
    with pytest.raises(G.GoPanic, match="Layer type already exists"):
        G.RegisterLayerType(1777, G.LayerTypeMetadata("again"))
    with pytest.raises(G.GoPanic, match="Layer type already exists"):
        G.RegisterLayerType(int(G.LayerTypePayload), G.LayerTypeMetadata("Payload2"))
    assert G.OverrideLayerType(1777, G.LayerTypeMetadata("Renamed")).String() == "Renamed"
    assert G.RegisterLayerType(-5, G.LayerTypeMetadata("Negative")).String() == "Negative"  # the map half
    assert G.LayerType(123456).String() == "123456"
    assert G.LayerType(1777).Contains(1777) and G.LayerType(1777).LayerTypes() == [1777]


def test_layer_classes():
    s = G.NewLayerClass([G.LayerType(2), G.LayerType(7)])
    assert isinstance(s, G.LayerClassSlice) and len(s) == 8
    assert s.Contains(7) and not s.Contains(3) and not s.Contains(99) and s.LayerTypes() == [2, 7]
    m = G.NewLayerClass([G.LayerType(2), G.LayerType(2001)])
    assert isinstance(m, G.LayerClassMap) and m.Contains(2001) and not m.Contains(3)
    assert sorted(m.LayerTypes()) == [2, 2001]
    assert isinstance(G.NewLayerClass([G.LayerType(2000)]), G.LayerClassSlice)  # > maxLayerType only

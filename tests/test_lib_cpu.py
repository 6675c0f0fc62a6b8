"""libgpk.so on the CPU side only: it loads, exports every symbol include/*.h
declares, and its host-side pieces (parser configuration, error text, layer
names) match the oracle. No GPU call is made here."""
import ctypes
import os
import re

import pytest

from gopacket_amd import _lib, engine
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    names = set()
    for h in sorted(os.listdir(os.path.join(ROOT, "include"))):
        src = open(os.path.join(ROOT, "include", h)).read()
        names |= set(re.findall(r"^(?:int|int64_t|void|const char\*)\s+(gpk_\w+)\(", src, re.M))
    return sorted(names)


def test_exports_every_declared_symbol():
    L = _lib.lib()
    names = header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(_lib.EXPORTS)
    assert L.gpk_abi_version() == 2


def test_parser_config_container_semantics():
    # DecodingLayerMap.Put: every type of CanDecode(), later Put overrides (parser.go:150-158)
    p = engine.ParserConfig(17, [1, 5, 8])
    assert p.decoder_for(17) == 1
    assert [p.decoder_for(t) for t in (46, 47, 48, 49)] == [5, 5, 5, 5]
    assert p.decoder_for(2) == 8 and p.decoder_for(20) == 0 and p.decoder_for(-1) == 0
    assert p.decoder_for(5000) == 0
    with pytest.raises(_lib.GpkError):
        p.add_decoder(42)
    with pytest.raises(_lib.GpkError):
        p.set_outputs(8)
    with pytest.raises(_lib.GpkError):
        p.set_ipprotocol(256, 20)


ERR_ARGS = [(0, 0), (1, 0), (20, 5), (136, 0), (65535, 4294967295), (2, 3), (44, 7)]


@pytest.mark.parametrize("code", [1, 2, 3, 4] + list(range(10, 12)) + list(range(20, 28)) + list(range(30, 40)) +
                         list(range(40, 56)) + [60, 61])
def test_error_text_matches_oracle(code):
    op = O.OracleParser(17, ["ETHERNET"])
    for a0, a1 in ERR_ARGS:
        assert engine.format_error(code, a0, a1) == op.error_string(code, a0, a1), (code, a0, a1)


def test_layer_type_names():
    # LayerType.String(), layertype.go:101-111
    assert engine.layer_type_name(17) == "Ethernet"
    assert engine.layer_type_name(107) == "DNS"
    assert engine.layer_type_name(1010) == "GTPv2"
    assert engine.layer_type_name(999) == "999"
    assert engine.format_error(1, 22) == "No decoder for layer type LLC"
    assert engine.format_error(33, 17) == "IPv6 length 0, but next header is UDP, not HopByHop"
    assert engine.format_error(33, 253) == "IPv6 length 0, but next header is UnknownIPProtocol, not HopByHop"


def test_code_table():
    L = _lib.lib()
    assert [L.gpk_code_layer_type(c) for c in range(13)] == list(engine.CODE_TO_LAYER_TYPE)
    assert L.gpk_code_layer_type(13) == -1


def test_gopacket_api_objects():
    from gopacket_amd import gopacket, layers
    assert str(layers.LayerTypeEthernet) == "Ethernet" and int(layers.LayerTypeTCP) == 44
    f = gopacket.NewFlow(gopacket.EndpointIPv4, bytes([1, 2, 3, 4]), bytes([5, 6, 7, 8]))
    assert f.FastHash() == f.Reverse().FastHash()
    assert f.FastHash() == O.flow_fast_hash(1, bytes([1, 2, 3, 4]), bytes([5, 6, 7, 8]))
    e = gopacket.Endpoint(gopacket.EndpointTCPPort, bytes([0, 80]))
    assert e.String() == "80"
    assert gopacket.UnsupportedLayerType(107).Error() == "No decoder for layer type DNS"


def _rss_mib():
    for line in open("/proc/self/status"):
        if line.startswith("VmRSS:"):
            return int(line.split()[1]) / 1024
    return 0.0


def test_host_view_is_a_view_and_does_not_grow_the_process():
    """The replay and pump callbacks see library memory through _lib.host_view.
    Its arrays alias the memory (same address, writes visible), carry the
    record dtypes, and making them for 20 000 distinct lengths costs no memory
    (np.ctypeslib.as_array caches a ctypes array type per length: about 90 MB
    here, without bound in a long capture)."""
    import numpy as np
    buf = np.arange(1 << 20, dtype=np.uint8)
    p = buf.ctypes.data
    v = _lib.host_view(p, 4096, np.uint32)
    assert v.ctypes.data == p and np.array_equal(v, buf[:16384].view(np.uint32))
    v[0] = 0xDEADBEEF
    assert buf[:4].view(np.uint32)[0] == 0xDEADBEEF
    r = _lib.host_view(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint8)), 100, _lib.RECORD_DTYPE)
    assert r.dtype == _lib.RECORD_DTYPE and r.ctypes.data == p and r.tobytes() == buf[:1600].tobytes()
    assert _lib.host_view(p, 10, _lib.CAPINFO_DTYPE).tobytes() == buf[:240].tobytes()
    r0 = _rss_mib()
    for n in range(1000, 21000):
        _lib.host_view(p, n, _lib.RECORD_DTYPE)
        _lib.host_view(p, 3 * n, np.uint64)
    assert _rss_mib() - r0 < 16

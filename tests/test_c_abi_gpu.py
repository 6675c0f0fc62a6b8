"""The C-language caller decodes the golden packets (reference vectors, the
reference's capture files, fuzzed packets) through gpk_decode_batch_host and
compares records, error arguments, flow hashes and Go error texts with the
committed oracle expectations (tools/make_c_abi_golden.py)."""
import os
import subprocess

import pytest

from test_c_abi_cpu import ROOT, build_c_abi_test

pytestmark = pytest.mark.gpu


def test_c_abi_decode_mode():
    exe = os.path.join(ROOT, "tests", "c_abi", "gpk_abi_test")
    if not os.path.exists(exe):  # built by __graft_entry__.build(); the box has gcc too
        exe = build_c_abi_test()
    out = subprocess.run([exe, "decode", os.path.join(ROOT, "tests", "golden", "c_abi")], capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "all checks passed (decode)" in out.stdout
    assert "statsassembly: 639 packets" in out.stdout
    assert "fields records checked" in out.stdout


def test_c_abi_replay_with_fields(tmp_path):
    """The C caller drives gpk_replay_file with gpk_replay_opts.fields_cb over a
    synthetic C4 capture and the reference's own capture files: results in
    packet order, every batch's fields before its records, the packet count
    equal to the capture reader's, and for every packet decoded without error
    the fields' present bits equal to the decoders its decoded list names."""
    from gopacket_amd import _lib
    exe = os.path.join(ROOT, "tests", "c_abi", "gpk_abi_test")
    if not os.path.exists(exe):
        exe = build_c_abi_test()
    synth = str(tmp_path / "c4.pcapng")
    assert _lib.synth_lib().gpk_synth_write_pcapng(synth.encode(), 4, 5, 20000, 4) > 0
    g = os.path.join(ROOT, "tests", "golden")
    files = [synth] + [os.path.join(g, "pcapgo", "le", "test%03d.pcapng" % k) for k in (1, 5, 10)] + \
        [os.path.join(g, "pcapgo", "epb.pcapng"), os.path.join(g, "test_ethernet.pcap")]
    out = subprocess.run([exe, "replay"] + files, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "all checks passed (replay)" in out.stdout
    import re
    m = re.search(r"replay c4\.pcapng: (\d+) packets, (\d+) checked", out.stdout)
    assert m and int(m.group(1)) == 20000 and int(m.group(2)) > 15000, out.stdout

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

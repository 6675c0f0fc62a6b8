"""The Python side's view of every C-ABI struct (the ctypes Structures and
numpy dtypes in gopacket_amd/_lib.py) against the C compiler's: a C file
generated from the Python field names prints sizeof and offsetof for each
struct of include/*.h, so a renamed, reordered or resized member (a new
trailing callback in an options struct, a widened field) fails here before it
reaches a GPU. A name missing on the C side fails the compile."""
import ctypes
import json
import os
import shutil
import subprocess

import pytest

from gopacket_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STRUCTS = {  # C type -> Python mirror
    "gpk_batch": _lib.Batch,
    "gpk_results": _lib.Results,
    "gpk_results8": _lib.Results8,
    "gpk_replay_range": _lib.ReplayRange,
    "gpk_groups": _lib.Groups,
    "gpk_tp_opts": _lib.TpOpts,
    "gpk_tp_pump_opts": _lib.PumpOpts,
    "gpk_tp_pump_stats": _lib.PumpStats,
    "gpk_capindex": _lib.CapIndex,
    "gpk_ng_interface": _lib.NgInterface,
    "gpk_replay_opts": _lib.ReplayOpts,
    "gpk_replay_stats": _lib.ReplayStats,
    "gpk_record": _lib.RECORD_DTYPE,
    "gpk_record8": _lib.RECORD8_DTYPE,
    "gpk_layout": _lib.LAYOUT_DTYPE,
    "gpk_fields": _lib.FIELDS_DTYPE,
    "gpk_bpf_insn": _lib.BPF_INSN_DTYPE,
    "gpk_tp_info": _lib.TPINFO_DTYPE,
    "gpk_capture_info": _lib.CAPINFO_DTYPE,
}


def _python_layout(mirror):
    if isinstance(mirror, type) and issubclass(mirror, ctypes.Structure):
        return ctypes.sizeof(mirror), {name: getattr(mirror, name).offset for name, *_ in mirror._fields_}
    return mirror.itemsize, {name: mirror.fields[name][1] for name in mirror.names}


@pytest.fixture(scope="module")
def c_layouts(tmp_path_factory):
    if not shutil.which("gcc"):
        pytest.skip("needs gcc")
    lines = ['#include <stddef.h>', '#include <stdio.h>', '#include "gpk.h"', '#include "gpk_capture.h"',
             '#include "gpk_afpacket.h"', '#include "gpk_flows.h"', '#include "gpk_bpf.h"',
             "int main(void) {", '  printf("{");']
    first = True
    for cname, mirror in STRUCTS.items():
        _, fields = _python_layout(mirror)
        lines.append('  printf("%s\\"%s\\": [%%zu, {", sizeof(%s));' % ("" if first else ",", cname, cname))
        for k, name in enumerate(fields):
            lines.append('  printf("%s\\"%s\\": %%zu", offsetof(%s, %s));' % ("" if k == 0 else ",", name, cname, name))
        lines.append('  printf("}]");')
        first = False
    lines += ['  printf("}\\n");', "  return 0;", "}"]
    d = tmp_path_factory.mktemp("abi")
    src, exe = d / "layout.c", d / "layout"
    src.write_text("\n".join(lines) + "\n")
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), "-o", str(exe),
                        str(src)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60, check=True).stdout
    return json.loads(out)


@pytest.mark.parametrize("cname", sorted(STRUCTS))
def test_python_mirror_matches_c_layout(c_layouts, cname):
    size, offsets = _python_layout(STRUCTS[cname])
    c_size, c_offsets = c_layouts[cname]
    assert offsets == c_offsets, cname
    assert size == c_size, (cname, size, c_size)

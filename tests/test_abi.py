"""The C ABI library loads and exports every symbol include/lincheck.h
declares; device entry points fail loudly (no CPU fallback) without a GPU."""
import ctypes as C
import os
import re

import pytest

from lincheck import _native as N

HEADER = os.path.join(os.path.dirname(__file__), "..", "include", "lincheck.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(lc_[a-z0-9_]+)\s*\(", src)) - {"lc_DESC"})


def test_header_symbols_exported():
    L = C.CDLL(N.LIB_PATH)
    names = declared()
    assert len(names) >= 20
    for name in names:
        assert hasattr(L, name), name
    assert set(names) == set(N.SIGNATURES), set(names) ^ set(N.SIGNATURES)


def test_abi_version():
    assert N.lib().lc_abi_version() == N.LC_ABI_VERSION


STRUCTS = {"lc_history": N.LcHistory, "lc_batch": N.LcBatch, "lc_result": N.LcResult, "lc_opts": N.LcOpts,
           "lc_stats": N.LcStats, "lc_pack_opts": N.LcPackOpts, "lc_synth_opts": N.LcSynthOpts}


def test_struct_layouts_match_header(tmp_path):
    """Every field offset and struct size the ctypes (and JNA) bindings use
    equals the C compiler's for include/lincheck.h (x86-64 LP64)."""
    import subprocess
    lines = ["#include <stdio.h>", "#include <stddef.h>", f'#include "{os.path.abspath(HEADER)}"',
             "int main(void) {"]
    for cname, py in STRUCTS.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines += ["return 0; }"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-o", str(exe), str(src)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {tuple(l.split()[:2]): int(l.split()[2]) for l in out if l}
    for cname, py in STRUCTS.items():
        assert got[(cname, "size")] == C.sizeof(py), cname
        for fname, _ in py._fields_:
            assert got[(cname, fname)] == getattr(py, fname).offset, (cname, fname)


@pytest.mark.skipif(N.lib().lc_device_count() > 0, reason="a GPU is visible")
def test_device_calls_fail_loudly_without_gpu():
    from lincheck.checker import Device
    with pytest.raises(N.LincheckError, match="device"):
        Device(0)


def test_bad_options_rejected():
    o = N.LcOpts()
    o.algorithm = 7
    h = C.c_void_p()
    assert N.lib().lc_create(C.byref(o), C.byref(h)) == -1
    assert b"algorithm" in N.lib().lc_last_error()


@pytest.mark.parametrize("algo", [1, 2])
def test_wgl_and_competition_accepted(algo):
    """LC_ALGO_WGL / _COMPETITION pass option validation (F-3); without a GPU
    the call then fails on the device, not on the option."""
    o = N.LcOpts()
    o.algorithm = algo
    h = C.c_void_p()
    rc = N.lib().lc_create(C.byref(o), C.byref(h))
    if rc == 0:
        N.lib().lc_destroy(h)
    else:
        assert b"algorithm" not in N.lib().lc_last_error()


def test_spec_ck_range_checked():
    """spec_ck packs (ck1 + 1) | (ck2 + 1) << 16 into an int32; a
    ck2 past 32766 wraps the word negative.  lc_create refuses such a word
    and the Python binding refuses the pair before packing it."""
    from lincheck.checker import Device
    o = N.LcOpts()
    o.spec_ck = -((1 << 31) - 1)  # what (0, 40000) would have wrapped to
    h = C.c_void_p()
    assert N.lib().lc_create(C.byref(o), C.byref(h)) == -1
    assert b"spec_ck" in N.lib().lc_last_error()
    for bad in [(0, 40000), (-1, 5), (70000, 5)]:
        with pytest.raises(ValueError, match="spec_ck"):
            Device(0, spec_ck=bad)

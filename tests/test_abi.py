"""The C-ABI library loads, exports every entry point include/ppgpu.h declares, carries gfx950
code, and refuses to decode without an MI355X (there is no CPU fallback)."""
import os
import re

import parallelparsing_amd as pp
from parallelparsing_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    with open(os.path.join(ROOT, "include", "ppgpu.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"\b(ppg_\w+)\s*\(", src)))


def test_header_symbols_exported_and_bound():
    names = declared()
    assert len(names) > 20
    for n in names:
        assert hasattr(_lib.lib, n), n          # dlsym succeeds
    assert sorted(_lib.EXPORTED) == names       # the Python binding covers the header exactly


def test_library_carries_gfx950_code_object():
    """The clang offload bundle inside .hip_fatbin names its gfx950 code object."""
    with open(_lib.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"__CLANG_OFFLOAD_BUNDLE__" in blob
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_version_string():
    assert b"gfx950" in _lib.lib.ppg_version()


def test_no_cpu_fallback_without_device():
    if pp.device_count() > 0:
        return   # on a GPU box this is covered by the gpu tests
    try:
        pp.Device(0)
    except pp.PpgError as e:
        assert e.code == _lib.PPG_NO_DEVICE
    else:
        raise AssertionError("opened a device context without a GPU")

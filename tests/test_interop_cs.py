"""The C# side of the boundary (interop/*.cs, the classes a maintainer adds next to the
reference's LibZ, Interop/PlatformInterop.cs:6-35).  No .NET SDK exists in this image, so the
sources cannot be compiled here; this checks them against include/ppgpu.h instead: PpGpu.cs
declares exactly the header's entry points, each with the header's parameter count, and the
enumerator only calls externs PpGpu.cs declares."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _read(*p):
    with open(os.path.join(ROOT, *p)) as f:
        return f.read()


def _c_decls():
    src = re.sub(r"/\*.*?\*/", "", _read("include", "ppgpu.h"), flags=re.S)
    out = {}
    for m in re.finditer(r"\b(ppg_\w+)\s*\(([^;{]*?)\)\s*;", src):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return out


def _cs_decls():
    src = _read("interop", "PpGpu.cs")
    out = {}
    for m in re.finditer(r"extern\s+[\w\*]+\s+(ppg_\w+)\s*\(([^;]*?)\)\s*;", src, flags=re.S):
        args = re.sub(r"/\*.*?\*/", "", m.group(2)).strip()
        out[m.group(1)] = 0 if not args else args.count(",") + 1
    return out


def test_pinvoke_class_matches_header():
    c, cs = _c_decls(), _cs_decls()
    assert len(c) > 40
    assert sorted(cs) == sorted(c)
    for name, n in c.items():
        assert cs[name] == n, (name, cs[name], n)


def test_enumerator_uses_declared_externs():
    cs = _cs_decls()
    used = set(re.findall(r"PpGpu\.(ppg_\w+)", _read("interop", "GpuBatchedFASTQ.cs")))
    assert {"ppg_cursor_open", "ppg_cursor_next", "ppg_cursor_close", "ppg_dist_decompress_all",
            "ppg_file_decompress_all", "ppg_comm_init"} <= used
    assert used <= set(cs)


def test_batch_struct_layout_matches_header():
    """ppg_batch's fields in order (the C# struct is LayoutKind.Sequential)."""
    h = _read("include", "ppgpu.h")
    body = h[h.index("typedef struct {", h.index("ppg_cursor;")):h.index("} ppg_batch;")]
    c_fields = re.findall(r"\*?(\w+);", body)
    cs = _read("interop", "PpGpu.cs")
    sb = cs[cs.index("struct PpgBatch"):]
    sb = sb[:sb.index("}")]
    cs_fields = re.findall(r"public [\w\*]+ (\w+);", sb)
    norm = lambda x: x.replace("_", "").lower()   # noqa: E731
    assert [norm(f) for f in c_fields] == [norm(f) for f in cs_fields]

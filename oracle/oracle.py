"""TEST INFRASTRUCTURE ONLY — Python handle on oracle/_build/liboracle.so (oracle/oracle.c).

The oracle is the parity checker for the GPU path; only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import it.  See oracle/oracle.c's header for what it restates
(file:line) and for its pinning status ("parity unpinned" against reference-owned vectors: the
reference ships none; pinned to the gzip trailer, Python's zlib and oracle/oracle_py.py).
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "_build", "liboracle.so")


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _load():
    if not os.path.exists(SO):
        build()
    L = C.CDLL(SO)
    vp, i64, i32 = C.c_void_p, C.c_int64, C.c_int32
    L.orc_build_index.restype = C.c_int
    L.orc_build_index.argtypes = [vp, i64, C.c_uint32, C.POINTER(vp)]
    L.orc_index_free.argtypes = [vp]
    L.orc_index_count.restype = C.c_int
    L.orc_index_count.argtypes = [vp]
    L.orc_index_chunk_max_bytes.restype = i32
    L.orc_index_chunk_max_bytes.argtypes = [vp]
    L.orc_index_point.restype = vp
    L.orc_index_point.argtypes = [vp, C.c_int]
    L.orc_point_get.argtypes = [vp, C.POINTER(i64), C.POINTER(i64), C.POINTER(i32), C.POINTER(i32)]
    L.orc_point_window.restype = vp
    L.orc_point_window.argtypes = [vp]
    L.orc_point_offset.restype = vp
    L.orc_point_offset.argtypes = [vp]
    L.orc_extract.restype = i64
    L.orc_extract.argtypes = [vp, i64, vp, vp, vp, i64]
    L.orc_parse.restype = i64
    L.orc_parse.argtypes = [vp, i64, vp, i64, vp, i64, vp]
    L.orc_serialize.restype = C.c_int
    L.orc_serialize.argtypes = [vp, C.c_char_p]
    L.orc_deserialize.restype = C.c_int
    L.orc_deserialize.argtypes = [C.c_char_p, C.POINTER(vp)]
    L.orc_index_from_points.restype = C.c_int
    L.orc_index_from_points.argtypes = [C.c_int, vp, vp, vp, vp, vp, vp, C.POINTER(vp)]
    L.orc_decompress_all.restype = i64
    L.orc_decompress_all.argtypes = [vp, vp, i64, C.c_int, C.c_int, C.c_int, C.c_int, vp]
    return L


L = _load()


def _u8(b):
    return np.frombuffer(bytes(b), np.uint8) if not isinstance(b, np.ndarray) else np.ascontiguousarray(b, np.uint8)


class OracleIndex:
    def __init__(self, h):
        self.h = C.c_void_p(h)

    def __del__(self):
        if getattr(self, "h", None) is not None and self.h.value and L is not None:   # L is None at exit
            L.orc_index_free(self.h)
            self.h = None

    @property
    def count(self):
        return L.orc_index_count(self.h)

    @property
    def chunk_max_bytes(self):
        return L.orc_index_chunk_max_bytes(self.h)

    def point(self, i):
        """(output, input, bits, window bytes, offset bytes)."""
        p = L.orc_index_point(self.h, i)
        o, n, b, ol = C.c_int64(), C.c_int64(), C.c_int32(), C.c_int32()
        L.orc_point_get(p, C.byref(o), C.byref(n), C.byref(b), C.byref(ol))
        w = C.string_at(L.orc_point_window(p), 32768)
        off = C.string_at(L.orc_point_offset(p), ol.value) if ol.value else b""
        return o.value, n.value, b.value, w, off

    def points(self):
        return [self.point(i) for i in range(self.count)]

    def serialize(self, path):
        rc = L.orc_serialize(self.h, os.fsencode(path))
        if rc:
            raise RuntimeError(f"orc_serialize {rc}")


def build_index(gz, chunksize):
    """Core.BuildDeflateIndex restated (oracle.c).  Returns OracleIndex or raises with the code."""
    a = _u8(gz)
    h = C.c_void_p()
    rc = L.orc_build_index(C.c_void_p(a.ctypes.data), a.size, chunksize & 0xFFFFFFFF, C.byref(h))
    if rc:
        raise OracleError(rc)
    return OracleIndex(h.value)


def index_from_points(output, inp, bits, windows, offset_len, offsets):
    a = [np.ascontiguousarray(x, t) for x, t in ((output, np.int64), (inp, np.int64), (bits, np.int32),
                                                  (windows, np.uint8), (offset_len, np.int32))]
    offs = np.ascontiguousarray(offsets if len(offsets) else np.zeros(1), np.uint8)
    h = C.c_void_p()
    L.orc_index_from_points(len(a[0]), *[C.c_void_p(x.ctypes.data) for x in a], C.c_void_p(offs.ctypes.data),
                            C.byref(h))
    return OracleIndex(h.value)


def deserialize(path):
    h = C.c_void_p()
    rc = L.orc_deserialize(os.fsencode(path), C.byref(h))
    if rc:
        raise OracleError(rc)
    return OracleIndex(h.value)


class OracleError(RuntimeError):
    def __init__(self, code):
        self.code = code
        super().__init__(f"oracle error {code}")


def extract(gz, ix, k):
    """Core.ExtractDeflateIndex on chunk k (slice as LazyFileReader reads it).  Returns bytes."""
    a = _u8(gz)
    p0, p1 = L.orc_index_point(ix.h, k), L.orc_index_point(ix.h, k + 1)
    o0, i0, _, _, _ = ix.point(k)
    o1, i1, _, _, _ = ix.point(k + 1)
    lo, n = i0 - 1, i1 - i0 + 1
    buf = np.zeros(max(1, o1 - o0), np.uint8)
    got = L.orc_extract(C.c_void_p(a.ctypes.data + lo), n, C.c_void_p(p0), C.c_void_p(p1),
                        C.c_void_p(buf.ctypes.data), buf.size)
    if got < 0:
        raise OracleError(got)
    return buf[:got].tobytes()


def parse(offset, chunk):
    """Parsing.Parse restated: (n,4) uint32 newline positions per record over offset ++ chunk."""
    off = _u8(offset or b"\0")
    ch = _u8(chunk or b"\0")
    ol, cl = len(offset or b""), len(chunk or b"")
    n = L.orc_parse(C.c_void_p(off.ctypes.data), ol, C.c_void_p(ch.ctypes.data), cl, None, 0, None)
    rec = np.zeros((max(1, n), 4), np.uint32)
    L.orc_parse(C.c_void_p(off.ctypes.data), ol, C.c_void_p(ch.ctypes.data), cl, C.c_void_p(rec.ctypes.data), n, None)
    return rec[:n]


def decompress_all(gz, ix, threads=1, mode=0, first=0, last=None):
    """Threaded DecompressAll (CPU baseline).  Returns (total records, per-chunk counts)."""
    a = _u8(gz)
    if last is None:
        last = ix.count - 1
    counts = np.zeros(ix.count, np.int64)
    tot = L.orc_decompress_all(ix.h, C.c_void_p(a.ctypes.data), a.size, first, last, threads, mode,
                               C.c_void_p(counts.ctypes.data))
    if tot < 0:
        raise OracleError(tot)
    return tot, counts[first:last]

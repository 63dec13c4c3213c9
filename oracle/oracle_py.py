"""TEST INFRASTRUCTURE ONLY — a second, independent restatement of Core.BuildDeflateIndex
(Decompressor/Core.cs:14-131) written in Python against libz 1.2.11 through ctypes, with the
z_stream layout of Interop/PlatformInterop.cs:37-76 (LP64, 112 bytes).

It exists to pin oracle/oracle.c: two restatements written separately, in different languages,
must produce identical points on every fixture (tests/test_oracle.py).  Pure-Python byte loops
are replaced by bytes.count/rfind, so it handles fixture-sized inputs (a few MB) in seconds.
"""
import ctypes as C
import ctypes.util

WINSIZE = 32768
CHUNK = 16384
Z_OK, Z_STREAM_END, Z_NEED_DICT = 0, 1, 2
Z_STREAM_ERROR, Z_DATA_ERROR, Z_MEM_ERROR, Z_BUF_ERROR, Z_VERSION_ERROR = -2, -3, -4, -5, -6
Z_BLOCK = 5


class z_stream(C.Structure):   # Interop/PlatformInterop.cs:37-76
    _fields_ = [("next_in", C.c_void_p), ("avail_in", C.c_uint), ("total_in", C.c_ulong),
                ("next_out", C.c_void_p), ("avail_out", C.c_uint), ("total_out", C.c_ulong),
                ("msg", C.c_char_p), ("state", C.c_void_p), ("zalloc", C.c_void_p), ("zfree", C.c_void_p),
                ("opaque", C.c_void_p), ("data_type", C.c_int), ("adler", C.c_ulong), ("reserved", C.c_ulong)]


_z = C.CDLL(ctypes.util.find_library("z") or "libz.so.1")
_z.inflateInit2_.argtypes = [C.POINTER(z_stream), C.c_int, C.c_char_p, C.c_int]
_z.inflate.argtypes = [C.POINTER(z_stream), C.c_int]
_z.inflateReset.argtypes = [C.POINTER(z_stream)]
_z.inflateEnd.argtypes = [C.POINTER(z_stream)]
assert C.sizeof(z_stream) == 112


class IndexError_(RuntimeError):
    pass


def build_index(gz: bytes, chunksize: int):
    """Returns (chunk_max_bytes, [(output, input, bits, window, offset), ...]) or raises."""
    pts = []
    cmb = [0]

    def add_point(bits, inp, out, left, window, offset):      # Common/Index.cs:24-48
        if not pts:
            cmb[0] = C.c_int32(out).value
        else:
            sz = C.c_int32((C.c_int32(out).value - C.c_int32(pts[-1][0]).value) & 0xFFFFFFFF).value
            cmb[0] = max(cmb[0], sz)
        w = bytes(window)
        pts.append((out, inp, bits, w[WINSIZE - left:] + w[:WINSIZE - left], bytes(offset)))

    strm = z_stream()
    ret = _z.inflateInit2_(C.byref(strm), 47, b"1.2.11", C.sizeof(z_stream))
    if ret != Z_OK:
        raise IndexError_(ret)
    inp = C.create_string_buffer(CHUNK)
    window = C.create_string_buffer(WINSIZE)
    fpos, flen = 0, len(gz)
    records = 0
    partial = bytearray()
    threshold = (chunksize - 8) & 0xFFFFFFFF
    totin = totout = 0
    have_window = False
    strm.avail_out = 0
    try:
        while True:
            piece = gz[fpos:fpos + CHUNK]
            fpos += len(piece)
            C.memmove(inp, piece, len(piece))
            strm.avail_in = len(piece)
            if strm.avail_in == 0:
                raise IndexError_(Z_DATA_ERROR)
            strm.next_in = C.addressof(inp)
            while True:
                if strm.avail_out == 0:
                    strm.avail_out = WINSIZE
                    strm.next_out = C.addressof(window)
                    have_window = True
                before = strm.avail_out
                totin += strm.avail_in
                totout += strm.avail_out
                ret = _z.inflate(C.byref(strm), Z_BLOCK)
                totin -= strm.avail_in
                totout -= strm.avail_out
                if ret in (Z_NEED_DICT, Z_MEM_ERROR, Z_DATA_ERROR, Z_STREAM_ERROR, Z_BUF_ERROR, Z_VERSION_ERROR):
                    raise IndexError_(ret)
                if have_window:
                    new = window.raw[WINSIZE - before:WINSIZE - strm.avail_out]
                    c = new.count(b"@")
                    # the carried partial record plus the bytes before this call's first '@' must
                    # fit the 32 KiB offset buffer (runs after an '@' are shorter than one call)
                    run = len(partial) + (new.find(b"@") if c else len(new))
                    if run > WINSIZE:
                        raise IndexError_(-50)   # C# IndexOutOfRangeException (Q4, Core.cs:93)
                    if c:
                        records += c
                        partial = bytearray(new[new.rfind(b"@"):])
                    else:
                        partial += new
                    dt = strm.data_type
                    if (dt & 128) and not (dt & 64):
                        if totout == 0:
                            add_point(dt & 7, totin, 0, strm.avail_out, window.raw, b"")
                        elif records > threshold:
                            add_point(dt & 7, totin, totout, strm.avail_out, window.raw, partial)
                            records = 0
                if ret == Z_STREAM_END:
                    if strm.avail_in != 0 or fpos != flen:
                        ret = _z.inflateReset(C.byref(strm))
                        if ret != Z_OK:
                            raise IndexError_(ret)
                        if strm.avail_in != 0:
                            continue
                        break
                    add_point(strm.data_type & 7, totin, totout, strm.avail_out, window.raw, b"")
                    return cmb[0], pts
                if strm.avail_in == 0:
                    break
    finally:
        _z.inflateEnd(C.byref(strm))

"""parallelparsing_amd — MI355X-native chunked-gzip FASTQ DecompressAll.

Host-side mirror of the reference's API surface (names, argument meaning, error behaviour) over
the C ABI of libppgpu.so (include/ppgpu.h):

  Core.BuildDeflateIndex(path_or_bytes, chunksize)        Decompressor/Core.cs:14-131 (CreateIndex)
  Core.ExtractDeflateIndex(file_buffer, index, k, buf)     Decompressor/Core.cs:133-192 (Decompress)
  Parsing.Parse(chunk)                                     Decompressor/Parsing.cs:11-51
  IndexIO.Serialize(index, path) / IndexIO.Deserialize    Common/IndexIO.cs:7-53
  BatchedFASTQ(index_or_path, gzip_path, ssd)              Decompressor/BatchedFASTQ.cs:10-101 (DecompressAll)
  FastqRecord / Index / Point                              Common/FastqRecord.cs, Common/Index.cs

Errors raise PpgError (the ZException of Interop/Conventions.cs:33-41) carrying the ZResult code.
The decode runs only on the GPU; there is no CPU fallback.
"""
import ctypes as C
import os

import numpy as np

from ._lib import lib, check, PpgError, PPG_NO_DEVICE, PPG_STREAM_END, PpgBatch, synth  # noqa: F401
from . import _lib

WINSIZE = 32768
CHUNK = 16384


def _ptr(a):
    return C.c_void_p(a.ctypes.data) if a is not None else None


class Point:
    """Common/Index.cs:51-82 (read-only view)."""

    __slots__ = ("Output", "Input", "Bits", "Window", "offset")

    def __init__(self, output, inp, bits, window, offset):
        self.Output, self.Input, self.Bits, self.Window, self.offset = output, inp, bits, window, offset

    def __repr__(self):
        return f"Point(Output={self.Output}, Input={self.Input}, Bits={self.Bits}, |offset|={len(self.offset)})"


class Index:
    """Common/Index.cs: the checkpoint list, owned by libppgpu (ppg_index)."""

    def __init__(self, handle):
        self._h = C.c_void_p(handle)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and lib is not None:   # (lib is None at interpreter exit)
            lib.ppg_index_free(h)
            self._h = None

    @property
    def handle(self):
        return self._h

    @property
    def Count(self):
        return lib.ppg_index_count(self._h)

    def __len__(self):
        return self.Count

    @property
    def ChunkMaxBytes(self):
        return lib.ppg_index_chunk_max_bytes(self._h)

    def point_fields(self, i):
        o, n, b, ol = C.c_int64(), C.c_int64(), C.c_int32(), C.c_int32()
        check(lib.ppg_index_point(self._h, i, C.byref(o), C.byref(n), C.byref(b), C.byref(ol)), "Index[i]")
        return o.value, n.value, b.value, ol.value

    def __getitem__(self, i):
        if i < 0:
            i += self.Count
        o, n, b, ol = self.point_fields(i)
        w = C.string_at(lib.ppg_index_window(self._h, i), WINSIZE)
        off = C.string_at(lib.ppg_index_offset(self._h, i), ol) if ol else b""
        return Point(o, n, b, w, off)

    def validate(self, first=0, n=None):
        """ppg_index_validate: raises PpgError(PPG_UNSUPPORTED) if a chunk of [first, first+n) is
        too large for the decode kernels (output >= 2^31 bytes, or >= 2^32 - 2^12 compressed bits)."""
        if n is None:
            n = self.Count - 1 - first
        check(lib.ppg_index_validate(self._h, int(first), int(n)), "Index.validate")
        return self

    def arrays(self):
        """(output, input, bits) int64 numpy arrays over all points."""
        n = self.Count
        out = np.empty(n, np.int64)
        inp = np.empty(n, np.int64)
        bits = np.empty(n, np.int64)
        for i in range(n):
            out[i], inp[i], bits[i], _ = self.point_fields(i)
        return out, inp, bits

    def windows_array(self):
        """All Point windows as one uint8 array (Count * 32768; the index stores them contiguously)."""
        n = self.Count
        if n == 0:
            return np.zeros(0, np.uint8)
        return np.frombuffer(C.string_at(lib.ppg_index_window(self._h, 0), n * WINSIZE), np.uint8)

    def set_side_points(self, bits, outputs, windows):
        """Attach side points (inner deflate block starts: absolute bit, output offset, the 32 KiB
        before each) found by the host, as BuildDeflateIndexGpu(side_bytes=...) records them
        (ppg_index_set_side_points)."""
        b, o = np.ascontiguousarray(bits, np.int64), np.ascontiguousarray(outputs, np.int64)
        w = np.ascontiguousarray(windows, np.uint8)
        assert w.size == 32768 * b.size and o.size == b.size
        check(lib.ppg_index_set_side_points(self._h, b.size, _ptr(b), _ptr(o), _ptr(w)), "ppg_index_set_side_points")
        return self

    def side_points(self, first=0, n=None):
        """(bits, outputs, windows) of the side points BuildDeflateIndexGpu(side_bytes=...) recorded,
        those inside chunks [first, first+n) (a Shard's range) -- Shard.set_split's arguments."""
        m = lib.ppg_index_side_count(self._h)
        bits, outs = np.zeros(max(1, m), np.int64), np.zeros(max(1, m), np.int64)
        win = np.zeros(max(1, m) * 32768, np.uint8)
        check(lib.ppg_index_side_points(self._h, _ptr(bits), _ptr(outs), _ptr(win)), "side_points")
        if n is None:
            n = self.Count - 1 - first
        lo, hi = self.point_fields(first)[0], self.point_fields(first + n)[0]
        keep = np.nonzero((outs[:m] > lo) & (outs[:m] < hi))[0]
        return bits[keep], outs[keep], win.reshape(-1, 32768)[keep].ravel()

    @staticmethod
    def from_points(output, inp, bits, windows, offset_len, offsets, chunk_max_bytes=0):
        """Index from arrays (ppg_index_from_points): windows is count*32768 bytes."""
        output = np.ascontiguousarray(output, np.int64)
        inp = np.ascontiguousarray(inp, np.int64)
        bits = np.ascontiguousarray(bits, np.int32)
        windows = np.ascontiguousarray(windows, np.uint8)
        offset_len = np.ascontiguousarray(offset_len, np.int32)
        offsets = np.ascontiguousarray(offsets, np.uint8) if len(offsets) else np.zeros(1, np.uint8)
        h = C.c_void_p()
        check(lib.ppg_index_from_points(len(output), _ptr(output), _ptr(inp), _ptr(bits), _ptr(windows),
                                        _ptr(offset_len), _ptr(offsets), int(chunk_max_bytes), C.byref(h)),
              "Index.from_points")
        return Index(h.value)


class IndexIO:
    """Common/IndexIO.cs."""

    @staticmethod
    def Serialize(index, path):
        check(lib.ppg_index_serialize(index.handle, os.fsencode(path)), "IndexIO.Serialize")

    @staticmethod
    def Deserialize(path):
        h = C.c_void_p()
        check(lib.ppg_index_deserialize(os.fsencode(path), C.byref(h)), "IndexIO.Deserialize")
        return Index(h.value)


class Device:
    """One GPU context (ppg_ctx): a HIP stream on an MI355X."""

    _default = {}

    def __init__(self, device=0):
        h = C.c_void_p()
        check(lib.ppg_open(int(device), C.byref(h)), f"ppg_open({device})")
        self._h = h
        self.device = device

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and lib is not None:   # (lib is None at interpreter exit)
            lib.ppg_close(h)
            self._h = None

    @property
    def handle(self):
        return self._h

    @property
    def stream(self):
        return lib.ppg_ctx_stream(self._h)

    def wait_stream(self, stream):
        """Order this ctx's later work after everything queued on `stream` (a hipStream_t handle, or
        a torch.cuda.Stream) so far -- ppg_ctx_wait_stream, no host drain."""
        check(lib.ppg_ctx_wait_stream(self._h, C.c_void_p(_stream_handle(stream))), "ppg_ctx_wait_stream")

    def stream_wait(self, stream):
        """Order `stream`'s later work after everything queued on this ctx so far (ppg_stream_wait_ctx)."""
        check(lib.ppg_stream_wait_ctx(self._h, C.c_void_p(_stream_handle(stream))), "ppg_stream_wait_ctx")

    def release_file_buffers(self):
        """Free what decompress_file keeps in this ctx between calls (ppg_file_release): its device
        pieces and their shards' outputs, the pinned staging; the next call allocates them again."""
        check(lib.ppg_file_release(self._h), "ppg_file_release")

    def decompress_chunk_stats(self):
        """{calls, launches, max_batch, split_chunks, side_points} of ppg_decompress_chunk on this
        ctx: how the thread-safe per-chunk Decompress combined concurrent calls into launches, and
        how many chunks it split at inner block starts it found on the GPU."""
        v = [C.c_int64() for _ in range(5)]
        check(lib.ppg_decompress_chunk_stats(self._h, *[C.byref(x) for x in v[:3]]), "ppg_decompress_chunk_stats")
        check(lib.ppg_decompress_chunk_split_stats(self._h, *[C.byref(x) for x in v[3:]]),
              "ppg_decompress_chunk_split_stats")
        return dict(zip(("calls", "launches", "max_batch", "split_chunks", "side_points"), (x.value for x in v)))

    def after_torch(self):
        """wait_stream(torch's current stream on this device): call before a ppg call reads device
        memory torch's stream writes, or writes memory it may still read."""
        import torch
        self.wait_stream(torch.cuda.current_stream(torch.device("cuda", self.device)))

    @classmethod
    def default(cls, device=None):
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        if device not in cls._default:
            cls._default[device] = cls(device)
        return cls._default[device]


def _stream_handle(stream):
    if stream is None:
        return 0
    return int(getattr(stream, "cuda_stream", stream))


def device_count():
    n = C.c_int(0)
    lib.ppg_device_count(C.byref(n))
    return n.value


class FastqRecord:
    """Common/FastqRecord.cs: Identifier, Sequence, Other, Quality (bytes fields, lazy str)."""

    __slots__ = ("raw", "start", "n1", "n2", "n3", "n4")

    def __init__(self, raw, start, n1, n2, n3, n4):
        self.raw, self.start, self.n1, self.n2, self.n3, self.n4 = raw, start, n1, n2, n3, n4

    # field slices exactly as Parsing.cs:37-40
    @property
    def identifier(self):
        return bytes(self.raw[self.start + 1:self.n1])

    @property
    def sequence(self):
        return bytes(self.raw[self.n1 + 1:self.n2])

    @property
    def other(self):
        return bytes(self.raw[self.n2 + 2:self.n3])

    @property
    def quality(self):
        return bytes(self.raw[self.n3 + 1:self.n4])

    Identifier = property(lambda s: s.identifier.decode("ascii", "replace"))
    Sequence = property(lambda s: s.sequence.decode("ascii", "replace"))
    Other = property(lambda s: s.other.decode("ascii", "replace"))
    Quality = property(lambda s: s.quality.decode("ascii", "replace"))

    def __repr__(self):
        return f"FastqRecord({self.identifier!r})"


def records_from_descriptors(raw, desc):
    """FastqRecords of one chunk from its (n,4) uint32 descriptors over raw = offset ++ chunk."""
    recs = []
    start = 0
    for n1, n2, n3, n4 in np.asarray(desc).reshape(-1, 4).tolist():
        recs.append(FastqRecord(raw, start, n1, n2, n3, n4))
        start = n4 + 1
    return recs


class Parsing:
    """Decompressor/Parsing.cs — the GPU record scan runs inside Core/Shard; this helper rebuilds
    FastqRecord objects from its descriptors."""

    @staticmethod
    def Parse(offset, chunk, desc):
        raw = bytes(offset or b"") + bytes(chunk)
        return records_from_descriptors(raw, desc)


def _as_u8(buf):
    if isinstance(buf, np.ndarray):
        return np.ascontiguousarray(buf, np.uint8)
    return np.frombuffer(bytes(buf), np.uint8)


class Core:
    """Decompressor/Core.cs."""

    @staticmethod
    def BuildDeflateIndex(gz, chunksize):
        """CreateIndex over a path or in-memory .gz bytes (Core.cs:14-131)."""
        h = C.c_void_p()
        if isinstance(gz, (str, os.PathLike)):
            check(lib.ppg_index_build_file(os.fsencode(gz), int(chunksize) & 0xFFFFFFFF, C.byref(h)),
                  "Core.BuildDeflateIndex")
        else:
            a = _as_u8(gz)
            check(lib.ppg_index_build_mem(_ptr(a), a.size, int(chunksize) & 0xFFFFFFFF, C.byref(h)),
                  "Core.BuildDeflateIndex")
        return Index(h.value)

    @staticmethod
    def BuildDeflateIndexGpu(gz, chunksize, device=None, piece_bytes=0, out_capacity=0, side_bytes=0):
        """CreateIndex on the GPU (ppg_index_gpu.cpp): the same Points as BuildDeflateIndex for a
        single-member gzip, from a block-parallel decode.  gz: a path, bytes / uint8 array (host),
        or a uint8 torch tensor on the device.  Raises PpgError(PPG_UNSUPPORTED) for zlib-wrapped
        or multi-member input (BuildDeflateIndex handles those).  side_bytes > 0 (in-memory input)
        also records side points every >= side_bytes of output inside chunks (Index.side_points,
        for Shard.set_split)."""
        dev = device or Device.default()
        h = C.c_void_p()
        cs = int(chunksize) & 0xFFFFFFFF
        if isinstance(gz, (str, os.PathLike)):
            if side_bytes:
                raise ValueError("side_bytes needs the member in memory (host or device)")
            rc = lib.ppg_index_build_gpu_file(dev.handle, os.fsencode(gz), cs, int(piece_bytes), C.byref(h))
        elif hasattr(gz, "data_ptr"):
            import torch
            if not (gz.is_cuda and gz.dtype == torch.uint8 and gz.is_contiguous() and gz.dim() == 1):
                raise ValueError("BuildDeflateIndexGpu: a device tensor must be a contiguous 1-D uint8 CUDA tensor")
            if gz.data_ptr() % 4:
                raise ValueError("BuildDeflateIndexGpu: a device tensor must be 4-byte aligned")
            # the block finder and the inflate reader fetch whole 4-byte words and read ahead: bytes
            # past gz_len may be read (never used), so they must be mapped -- torch's caching
            # allocator rounds every block up to 512 B; ppgpu.h documents the requirement
            dev.wait_stream(torch.cuda.current_stream(gz.device))   # our stream reads what torch's wrote
            rc = lib.ppg_index_build_gpu_side(dev.handle, C.c_void_p(gz.data_ptr()), gz.numel(), 1, cs,
                                              int(piece_bytes), int(out_capacity), int(side_bytes), C.byref(h))
        else:
            a = _as_u8(gz)
            rc = lib.ppg_index_build_gpu_side(dev.handle, _ptr(a), a.size, 0, cs, int(piece_bytes),
                                              int(out_capacity), int(side_bytes), C.byref(h))
        check(rc, "Core.BuildDeflateIndexGpu")
        return Index(h.value)

    GPU_INDEX_STATS = ("finder_ms", "pass1_ms", "chain_ms", "pass2_ms", "census_ms", "total_ms", "pieces",
                       "real_pieces", "redo1", "resolve_ms", "batches", "blocks", "points", "output_bytes",
                       "upload_ms", "pass2_alloc_ms", "spec_redos", "serial_redos")

    @staticmethod
    def gpu_index_stats(device=None):
        """Timings and counts of the last BuildDeflateIndexGpu on a device (ppg_index_build_gpu_stats)."""
        dev = device or Device.default()
        v = (C.c_double * len(Core.GPU_INDEX_STATS))()
        check(lib.ppg_index_build_gpu_stats(dev.handle, v, len(v)), "ppg_index_build_gpu_stats")
        return dict(zip(Core.GPU_INDEX_STATS, list(v)))

    @staticmethod
    def ExtractDeflateIndex(file_buffer, index, k, buf=None, device=None, with_records=False):
        """Decompress checkpoint k (Core.cs:133-192) on the GPU.  file_buffer = file bytes
        [Index[k].Input-1, Index[k+1].Input-1].  Returns the produced byte count written into buf
        (allocated if None) — and the (n,4) record descriptors if with_records.  Thread safe, as
        README.md:38-50 requires: concurrent calls on one Device share launches
        (ppg_decompress_chunk; ctypes releases the GIL for the call)."""
        dev = device or Device.default()
        src = _as_u8(file_buffer)
        o0, _, _, _ = index.point_fields(k)
        o1, _, _, _ = index.point_fields(k + 1)
        need = max(0, o1 - o0)
        if buf is None:
            buf = np.empty(need, np.uint8)   # every produced byte is written
        produced = C.c_int64()
        nrec = C.c_int64()
        # descriptor rows for >= 64-B records (a FASTQ record is hundreds); a chunk of smaller ones
        # reports its record count with PPG_BUF_ERROR and is decoded again into an exact table
        # (r05: rows for 4-B records made every call zero 4x its output bytes in the allocator)
        recs = np.empty((_rec_rows(need), 4), np.uint32) if with_records else None
        rc = lib.ppg_decompress_chunk(dev.handle, index.handle, int(k), _ptr(src), src.size, _ptr(buf), buf.size,
                                      C.byref(produced), _ptr(recs), recs.shape[0] if with_records else 0,
                                      C.byref(nrec))
        if with_records and rc == _lib.PPG_BUF_ERROR and nrec.value > recs.shape[0]:
            recs = np.empty((nrec.value, 4), np.uint32)
            rc = lib.ppg_decompress_chunk(dev.handle, index.handle, int(k), _ptr(src), src.size, _ptr(buf), buf.size,
                                          C.byref(produced), _ptr(recs), recs.shape[0], C.byref(nrec))
        check(rc, "Core.ExtractDeflateIndex")
        if with_records:
            return produced.value, buf, recs[:nrec.value]
        return produced.value, buf

    @staticmethod
    def ExtractDeflateIndexAsync(file_buffer, index, k, buf=None, device=None):
        """ExtractDeflateIndex queued without blocking (ppg_decompress_chunk_submit): returns a
        ChunkFuture whose result() is (produced, buf, records).  Many queued chunks share launches
        of up to 256 chunks; every future's result() must be taken (it frees the ticket)."""
        dev = device or Device.default()
        src = _as_u8(file_buffer)
        o0, _, _, _ = index.point_fields(k)
        o1, _, _, _ = index.point_fields(k + 1)
        need = max(0, o1 - o0)
        if buf is None:
            buf = np.empty(need, np.uint8)
        recs = np.empty((_rec_rows(need), 4), np.uint32)   # (too few: result() decodes it again)
        t = C.c_void_p()
        check(lib.ppg_decompress_chunk_submit(dev.handle, index.handle, int(k), _ptr(src), src.size, _ptr(buf), buf.size,
                                              _ptr(recs), recs.shape[0], C.byref(t)), "ppg_decompress_chunk_submit")
        return ChunkFuture(dev, t, (src, buf, recs, index, k))


def _rec_rows(nbytes):
    """Descriptor rows to offer for a chunk of nbytes of text: enough for records of >= 64 bytes."""
    return int(nbytes) // 64 + 256


class ChunkFuture:
    """A queued ExtractDeflateIndexAsync: result() waits (ppg_decompress_chunk_wait) -- once."""

    def __init__(self, dev, ticket, keep):
        self._dev, self._t, self._keep, self._res = dev, ticket, keep, None

    def result(self):
        if self._res is None:
            produced, nrec = C.c_int64(), C.c_int64()
            t, self._t = self._t, None
            if t is None:
                raise RuntimeError("ChunkFuture waited twice")
            rc = lib.ppg_decompress_chunk_wait(self._dev.handle, t, C.byref(produced), C.byref(nrec))
            src, buf, recs, index, k = self._keep
            self._keep = None
            if rc == _lib.PPG_BUF_ERROR and nrec.value > recs.shape[0]:   # records under 64 B: once more, exactly
                self._res = Core.ExtractDeflateIndex(src, index, k, buf=buf, device=self._dev, with_records=True)
                return self._res
            check(rc, "Core.ExtractDeflateIndexAsync")
            self._res = (produced.value, buf, recs[:nrec.value])
        return self._res

    def __del__(self):
        if getattr(self, "_t", None) is not None:   # never waited: wait now (the buffers must outlive it)
            try:
                self.result()
            except Exception:   # noqa: BLE001 - a finaliser must not raise
                pass


class Shard:
    """DecompressAll over index chunks [first, first+n) resident on one GPU (ppg_shard)."""

    def __init__(self, index, comp, first=0, n=None, device=None, comp_on_device=False, comp_len=None,
                 out_capacity=0):
        self.index = index
        self.dev = device or Device.default()
        if n is None:
            n = index.Count - 1 - first
        self.first, self.n = first, n
        self._on_device = bool(comp_on_device)
        if comp_on_device:
            ptr, length = int(comp), int(comp_len)
            # the library reads comp on its own stream: order that after torch's producers of comp
            # (a caller on another stream calls self.dev.wait_stream(its stream) itself)
            self._torch_order()
        else:
            self._host = _as_u8(comp)
            ptr, length = self._host.ctypes.data, self._host.size
        h = C.c_void_p()
        check(lib.ppg_shard_create(self.dev.handle, index.handle, first, n, C.c_void_p(ptr), length,
                                   1 if comp_on_device else 0, int(out_capacity), C.byref(h)), "ppg_shard_create")
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and lib is not None:   # (lib is None at interpreter exit)
            lib.ppg_shard_free(h)
            self._h = None

    @property
    def handle(self):
        return self._h

    def _torch_order(self):
        import sys
        if "torch" in sys.modules and sys.modules["torch"].cuda.is_initialized():
            self.dev.after_torch()

    def run(self):
        if self._on_device:
            self._torch_order()   # the caller may have rewritten comp since the last run
        check(lib.ppg_shard_run(self._h), "DecompressAll")
        return self

    def copy_output(self, off, length, dst=None):
        """Bytes [off, off+length) of the shard's decompressed output (relative to its first
        chunk's Output) into a new uint8 numpy array, or into `dst`: a numpy array (host) or a
        uint8 CUDA tensor on this device (device-to-device, stream-ordered after torch's stream)."""
        if dst is None:
            dst = np.empty(int(length), np.uint8)
        if hasattr(dst, "data_ptr"):
            if not (dst.is_cuda and dst.numel() >= length):
                raise ValueError("copy_output: dst tensor must be a CUDA tensor of >= length bytes")
            self.dev.after_torch()
            check(lib.ppg_shard_copy_output(self._h, int(off), int(length), C.c_void_p(dst.data_ptr()), 1),
                  "copy_output")
        else:
            if dst.nbytes < length:
                raise ValueError("copy_output: dst too small")
            check(lib.ppg_shard_copy_output(self._h, int(off), int(length), _ptr(dst), 0), "copy_output")
        return dst

    @property
    def batches(self):
        return lib.ppg_shard_batches(self._h)

    def set_split(self, bits, outputs, windows):
        """Decode chunks as several waves each, split at side points (deflate block starts inside
        the chunks: absolute bit, absolute output, 32 KiB window each; ppg_shard_set_split).
        Empty arrays restore one wave per chunk.  Results are identical either way."""
        bits = np.ascontiguousarray(bits, np.int64)
        outputs = np.ascontiguousarray(outputs, np.int64)
        windows = np.ascontiguousarray(windows, np.uint8)
        n = int(bits.size)
        if outputs.size != n or windows.size != n * 32768:
            raise ValueError("set_split: bits, outputs and windows (n * 32768 bytes) must agree")
        self._split = (bits, outputs, windows)
        check(lib.ppg_shard_set_split(self._h, n, _ptr(bits) if n else None, _ptr(outputs) if n else None,
                                      _ptr(windows) if n else None), "set_split")
        return self

    def set_keys(self, keys):
        """From the next run on, every output batch writes its records' spot keys (paired reads,
        ppg_record_keys) into `keys`, an int64 CUDA tensor on this device indexed by shard record
        number (ppg_shard_set_keys): works for shards of any number of batches.  None turns it off."""
        if keys is None:
            check(lib.ppg_shard_set_keys(self._h, None, 0), "set_keys")
            self._keys = None
            return self
        import torch
        if not (keys.is_cuda and keys.dtype == torch.int64 and keys.is_contiguous()):
            raise ValueError("set_keys: keys must be a contiguous int64 CUDA tensor")
        self._keys = keys   # kept alive while the library may write it
        check(lib.ppg_shard_set_keys(self._h, C.c_void_p(keys.data_ptr()), keys.numel()), "set_keys")
        return self

    def results(self):
        n = self.n
        rec, prod, end = (np.zeros(n, np.int64) for _ in range(3))
        st, fl = np.zeros(n, np.int32), np.zeros(n, np.int32)
        check(lib.ppg_shard_results(self._h, _ptr(rec), _ptr(prod), _ptr(st), _ptr(fl), _ptr(end)), "results")
        return {"records": rec, "produced": prod, "status": st, "flags": fl, "end_bit": end}

    @property
    def total_records(self):
        return lib.ppg_shard_total_records(self._h)

    def chunk_bytes(self, k):
        o0, _, _, _ = self.index.point_fields(self.first + k)
        o1, _, _, _ = self.index.point_fields(self.first + k + 1)
        dst = np.zeros(max(1, o1 - o0), np.uint8)
        ln = C.c_int64()
        check(lib.ppg_shard_copy_chunk(self._h, k, _ptr(dst), dst.size, C.byref(ln)), "copy_chunk")
        return dst[:ln.value]

    def chunk_records(self, k):
        nrec = C.c_int64()
        check(lib.ppg_shard_copy_records(self._h, k, None, 0, C.byref(nrec)), "copy_records")
        dst = np.zeros((max(1, nrec.value), 4), np.uint32)
        check(lib.ppg_shard_copy_records(self._h, k, _ptr(dst), dst.shape[0], C.byref(nrec)), "copy_records")
        return dst[:nrec.value]

    def record_base(self):
        b = np.zeros(self.n, np.int64)
        check(lib.ppg_shard_record_base(self._h, _ptr(b)), "record_base")
        return b

    def counts_to_device(self, dev_ptr):
        self._torch_order()
        check(lib.ppg_shard_counts_to_device(self._h, C.c_void_p(int(dev_ptr))), "counts_to_device")

    def timing(self):
        a, b, c = C.c_float(), C.c_float(), C.c_float()
        check(lib.ppg_shard_timing(self._h, C.byref(a), C.byref(b), C.byref(c)), "timing")
        return {"inflate_ms": a.value, "parse_ms": b.value, "total_ms": c.value}


class Comm:
    """ppg_comm: the communicator of multi-GPU DecompressAll's count all-gather (include/ppgpu.h).

    Comm.rccl(device, nranks, rank, uid)  RCCL, from a PPG_COMM_ID_BYTES id made by
                                          Comm.unique_id() on rank 0 and handed to every rank
    Comm.host(nranks, rank, name)         shared memory between processes of one machine (the
                                          one-GPU rehearsal: RCCL refuses two ranks on one GPU)"""

    def __init__(self, handle, device=None):
        self._h = C.c_void_p(handle)
        self.dev = device

    @staticmethod
    def unique_id():
        buf = (C.c_uint8 * 128)()
        check(lib.ppg_comm_unique_id(buf), "ppg_comm_unique_id")
        return bytes(buf)

    @classmethod
    def rccl(cls, device, nranks, rank, uid):
        h = C.c_void_p()
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        check(lib.ppg_comm_init(device.handle, int(nranks), int(rank), buf, C.byref(h)), "ppg_comm_init")
        return cls(h.value, device)

    @classmethod
    def host(cls, nranks, rank, name):
        h = C.c_void_p()
        check(lib.ppg_comm_init_host(int(nranks), int(rank), name.encode(), C.byref(h)), "ppg_comm_init_host")
        return cls(h.value)

    @property
    def handle(self):
        return self._h

    def alltoallv(self, send, counts):
        """ppg_comm_alltoallv over host memory (the host transport): counts[src, dst] int64 values go
        from rank src to rank dst; `send` holds this rank's by destination.  Returns what this rank
        receives, by source."""
        c = np.ascontiguousarray(counts, np.int64)
        r, n = self.rank_size()
        assert c.shape == (n, n)
        snd = np.ascontiguousarray(send, np.int64)
        assert snd.size == c[r].sum()
        rcv = np.zeros(max(1, int(c[:, r].sum())), np.int64)
        check(lib.ppg_comm_alltoallv(self._h, _ptr(snd if snd.size else np.zeros(1, np.int64)), _ptr(rcv), _ptr(c), 0),
              "ppg_comm_alltoallv")
        return rcv[:int(c[:, r].sum())]

    def rank_size(self):
        r, n = C.c_int32(), C.c_int32()
        check(lib.ppg_comm_rank(self._h, C.byref(r), C.byref(n)), "ppg_comm_rank")
        return r.value, n.value

    def close(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.ppg_comm_free(h)
            self._h = None

    def __del__(self):
        self.close()


def build_info():
    """The library in use: ppg_version() and ppg_build_id() (a hash of the inflate kernels' object)."""
    return {"ppg_version": lib.ppg_version().decode(), "build_id": lib.ppg_build_id().decode()}


def rccl_version():
    v = C.c_int()
    return v.value if lib.ppg_rccl_version(C.byref(v)) == 0 else None


def partition(index, nranks, first=0, n=None):
    """ppg_partition: contiguous chunk ranges balanced by compressed bytes -> bounds[nranks + 1]."""
    if n is None:
        n = index.Count - 1 - first
    b = np.zeros(nranks + 1, np.int32)
    check(lib.ppg_partition(index.handle, int(first), int(n), int(nranks), _ptr(b)), "ppg_partition")
    return b


def gather_counts(shard, comm, bounds):
    """ppg_shard_gather_counts: (counts, bases, total) of every chunk of [bounds[0], bounds[-1])."""
    bounds = np.ascontiguousarray(bounds, np.int32)
    m = int(bounds[-1] - bounds[0])
    counts, bases = np.zeros(max(m, 1), np.int64), np.zeros(max(m, 1), np.int64)
    tot = C.c_int64()
    check(lib.ppg_shard_gather_counts(shard.handle, comm.handle, _ptr(bounds), _ptr(counts), _ptr(bases),
                                      C.byref(tot)), "ppg_shard_gather_counts")
    return counts[:m], bases[:m], tot.value


def dist_decompress_all(index, gzip_path, comm, device=None, out_capacity=0):
    """ppg_dist_decompress_all: this rank's share of the file decoded, counts gathered over comm.
    Returns (counts, bases, total) over every chunk of the index."""
    dev = device or Device.default()
    m = index.Count - 1
    counts, bases = np.zeros(max(m, 1), np.int64), np.zeros(max(m, 1), np.int64)
    tot = C.c_int64()
    check(lib.ppg_dist_decompress_all(dev.handle, comm.handle, index.handle, os.fsencode(gzip_path),
                                      int(out_capacity), _ptr(counts), _ptr(bases), C.byref(tot)),
          "ppg_dist_decompress_all")
    return counts[:m], bases[:m], tot.value


def decompress_file(index, gzip_path, first=0, n=None, piece_bytes=8 << 30, threads=8, device=None):
    """DecompressAll of chunks [first, first+n) straight from a .gz file (ppg_file_decompress_all):
    reader threads pread ~piece_bytes pieces into pinned buffers, H2D overlaps the decode of the
    previous piece (the LazyFileReader path, Decompressor/LazyFileReader.cs:10-98).
    Returns (per-chunk record counts, total records, wall seconds)."""
    dev = device or Device.default()
    if n is None:
        n = index.Count - 1 - first
    rec = np.zeros(max(n, 1), np.int64)
    tot = C.c_int64(0)
    sec = C.c_double(0)
    check(lib.ppg_file_decompress_all(dev.handle, index.handle, os.fsencode(gzip_path), int(first), int(n),
                                      int(piece_bytes), int(threads), _ptr(rec), C.byref(tot), C.byref(sec)),
          "decompress_file")
    return rec[:n], tot.value, sec.value


class Cursor:
    """Bounded-memory record streaming (ppg_cursor): chunks [first, first+n) of a .gz file in
    batches of whole chunks of at most batch_bytes of text, read and decoded on the GPU while the
    previous batch is consumed.  Iterating yields Batch objects; a batch's arrays are views of the
    library's pinned buffers and stay valid only until the next batch is requested (as a
    FastqRecord is invalid after the next MoveNext, BatchedFASTQ.cs:56)."""

    def __init__(self, index, gzip_path, first=0, n=None, batch_bytes=1 << 30, threads=8, device=None):
        self.index = index
        self.dev = device or Device.default()
        if n is None:
            n = index.Count - 1 - first
        h = C.c_void_p()
        check(lib.ppg_cursor_open(self.dev.handle, index.handle, os.fsencode(gzip_path), int(first), int(n),
                                  int(batch_bytes), int(threads), C.byref(h)), "ppg_cursor_open")
        self._h = h

    def __del__(self):
        self.close()

    def close(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.ppg_cursor_close(h)
            self._h = None

    @property
    def batches(self):
        return lib.ppg_cursor_batches(self._h)

    def next_batch(self):
        b = PpgBatch()
        rc = lib.ppg_cursor_next(self._h, C.byref(b))
        if rc == PPG_STREAM_END:
            return None
        check(rc, "ppg_cursor_next")
        return Batch(b)

    def __iter__(self):
        while True:
            b = self.next_batch()
            if b is None:
                return
            yield b


class Batch:
    """One ppg_batch: text (uint8), raw_off / rec_off (int64, nchunks + 1), desc (nrecords x 4)."""

    def __init__(self, b):
        self.first_chunk, self.nchunks = b.first_chunk, b.nchunks
        self.record_base, self.nrecords = b.record_base, b.nrecords
        self.raw_off = np.ctypeslib.as_array(b.raw_off, (b.nchunks + 1,))
        self.rec_off = np.ctypeslib.as_array(b.rec_off, (b.nchunks + 1,))
        nt = int(self.raw_off[-1])
        self.text = np.ctypeslib.as_array(C.cast(b.text, C.POINTER(C.c_uint8)), (max(nt, 1),))[:nt]
        nd = 4 * int(b.nrecords)
        self.desc = np.ctypeslib.as_array(b.desc, (max(nd, 1),))[:nd].reshape(-1, 4)

    def raw(self, k):
        """raw_k = offset_k ++ chunk_k of the batch's k-th chunk."""
        return self.text[self.raw_off[k]:self.raw_off[k + 1]]

    def records(self, k):
        """Descriptors (n, 4) of the batch's k-th chunk."""
        return self.desc[self.rec_off[k]:self.rec_off[k + 1]]


class BatchedFASTQ:
    """Decompressor/BatchedFASTQ.cs:10-101 — DecompressAll as an iterable of FastqRecord.

    The reference yields records in a nondeterministic interleaving; this yields the
    canonical order: chunk 0's records, then chunk 1's, ...  enable_ssd_optimization is accepted
    for signature parity (it selected 1 or 8 FileStreams, LazyFileReader.cs:27-33)."""

    def __init__(self, index, gzip_path, enable_ssd_optimization=False, device=None, rank=None, world=None,
                 comm=None):
        if isinstance(index, (str, os.PathLike)):
            index = IndexIO.Deserialize(index)
        self.index = index
        self.gzip_path = gzip_path
        self.enable_ssd_optimization = enable_ssd_optimization
        self.dev = device
        self._shard = None
        # one rank of a multi-GPU job (the reference's Task.Run fan-out, BatchedFASTQ.cs:62-77, on
        # GPUs): iteration yields this rank's share -- the contiguous chunk range ppg_partition
        # gives it -- so the ranks' records, concatenated in rank order, are the file's
        # comm (a Comm of this job): Count() decodes only this rank's share and gathers every rank's
        # counts (ppg_dist_decompress_all), as the C# GpuBatchedFASTQ(..., GpuJob) does
        self.comm = comm
        if comm is not None and world is None:
            rank, world = comm.rank_size()
        self.rank, self.world = rank, world
        if (rank is None) != (world is None) or (world is not None and not 0 <= rank < world):
            raise ValueError("rank and world go together, 0 <= rank < world")

    def chunk_range(self):
        """(first, n): the chunks this enumerator streams (all of them, or this rank's share)."""
        m = self.index.Count - 1
        if self.world is None:
            return 0, m
        b = partition(self.index, self.world, 0, m)
        return int(b[self.rank]), int(b[self.rank + 1] - b[self.rank])

    def _run(self):
        if self._shard is None:
            n = self.index.Count - 1
            _, i0, _, _ = self.index.point_fields(0)
            _, i1, _, _ = self.index.point_fields(n)
            with open(self.gzip_path, "rb") as f:
                f.seek(i0 - 1)
                comp = f.read(i1 - i0 + 1)
            self._shard = Shard(self.index, comp, 0, n, device=self.dev).run()
        return self._shard

    def Count(self):
        """Number of records (Enumerable.Count over the enumerator, Decompressor/Program.cs:48-52):
        streamed from the file, nothing materialised on the host."""
        if self._shard is not None:
            return self._shard.total_records
        if self.world is not None:
            # one rank of a job: its own share decoded, the counts gathered -- every rank returns the
            # whole file's total (never each rank decoding the whole file)
            if self.comm is None:
                raise ValueError("Count() of a rank's BatchedFASTQ needs the job's comm (BatchedFASTQ(..., comm=))")
            _, _, total = dist_decompress_all(self.index, self.gzip_path, self.comm, device=self.dev)
            return total
        _, total, _ = decompress_file(self.index, self.gzip_path, device=self.dev,
                                      threads=16 if self.enable_ssd_optimization else 8)
        return total

    # text per streamed batch (ppg_cursor): up to five batches in flight, each ~1.13x this + its
    # compressed bytes of pinned host memory (ppg_cursor_open caps the slots by available memory)
    batch_bytes = 1 << 30

    def __iter__(self):
        """Records streamed through ppg_cursor in bounded memory, canonical chunk order; each
        batch's bytes are copied out before the next one is requested."""
        first, n = self.chunk_range()
        cur = Cursor(self.index, self.gzip_path, first=first, n=n, batch_bytes=self.batch_bytes,
                     threads=16 if self.enable_ssd_optimization else 8, device=self.dev)
        try:
            for b in cur:
                for k in range(b.nchunks):
                    yield from records_from_descriptors(b.raw(k).tobytes(), b.records(k))
        finally:
            cur.close()

    def Dispose(self):
        self._shard = None

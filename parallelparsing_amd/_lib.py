"""ctypes binding of libppgpu.so (include/ppgpu.h) and libppgsynth.so.

The HIP library is required: there is no CPU fallback for the decode path.  Importing this
module without a built libppgpu.so raises ImportError; opening a context without an MI355X
(gfx950) raises PpgError(PPG_NO_DEVICE).
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PPG_LIB_PATH") or os.path.join(_HERE, "libppgpu.so")
SYNTH_PATH = os.path.join(_HERE, "libppgsynth.so")

PPG_OK = 0
PPG_STREAM_END = 1
PPG_DATA_ERROR = -3
PPG_BUF_ERROR = -5
PPG_INDEX_OUT_OF_RANGE = -50
PPG_IO_ERROR = -51
PPG_ARG_ERROR = -52
PPG_UNSUPPORTED = -53
PPG_DEVICE_ERROR = -100
PPG_NO_DEVICE = -101

# ZResult names (Interop/Conventions.cs:9-20) for messages
_NAMES = {0: "OK", 1: "STREAM_END", 2: "NEED_DICT", -1: "ERRNO", -2: "STREAM_ERROR", -3: "DATA_ERROR",
          -4: "MEM_ERROR", -5: "BUF_ERROR", -6: "VERSION_ERROR", -50: "INDEX_OUT_OF_RANGE", -51: "IO_ERROR",
          -52: "ARG_ERROR", -53: "UNSUPPORTED", -100: "DEVICE_ERROR", -101: "NO_DEVICE"}


class PpgError(RuntimeError):
    """A non-zero status from libppgpu — the ZException of Interop/Conventions.cs:33-41."""

    def __init__(self, code, what=""):
        self.code = code
        super().__init__(f"{what}: {_NAMES.get(code, code)} ({code})")


def check(code, what):
    if code != PPG_OK:
        raise PpgError(code, what)
    return code


def _load(path, what):
    if not os.path.exists(path):
        raise ImportError(f"{what} not built at {path}: run `make -C parallelparsing_amd/csrc` "
                          f"(or __graft_entry__.build()); there is no fallback implementation")
    return C.CDLL(path)


# One HIP runtime per process: torch (when present) bundles its own libamdhip64 with the same soname
# as /opt/rocm's.  Whichever loads first serves both, and torch fails to initialise the GPU on the
# other's.  Importing torch first makes libppgpu bind to torch's runtime, as in bench.py.
try:
    import torch  # noqa: F401
except ImportError:
    pass

lib = _load(LIB_PATH, "libppgpu.so")

vp = C.c_void_p
i32, i64, u32 = C.c_int32, C.c_int64, C.c_uint32
P = C.POINTER

_SIGS = {
    "ppg_index_build_file": (C.c_int, [C.c_char_p, u32, P(vp)]),
    "ppg_index_build_mem": (C.c_int, [vp, i64, u32, P(vp)]),
    "ppg_index_build_gpu": (C.c_int, [vp, vp, i64, C.c_int, u32, i64, i64, P(vp)]),
    "ppg_index_build_gpu_side": (C.c_int, [vp, vp, i64, C.c_int, u32, i64, i64, i64, P(vp)]),
    "ppg_index_side_count": (C.c_int, [vp]),
    "ppg_index_set_side_points": (C.c_int, [vp, i32, vp, vp, vp]),
    "ppg_index_side_points": (C.c_int, [vp, vp, vp, vp]),
    "ppg_index_build_gpu_file": (C.c_int, [vp, C.c_char_p, u32, i64, P(vp)]),
    "ppg_index_build_gpu_stats": (C.c_int, [vp, P(C.c_double), i32]),
    "ppg_index_serialize": (C.c_int, [vp, C.c_char_p]),
    "ppg_index_deserialize": (C.c_int, [C.c_char_p, P(vp)]),
    "ppg_index_from_points": (C.c_int, [i32, vp, vp, vp, vp, vp, vp, i32, P(vp)]),
    "ppg_index_count": (i32, [vp]),
    "ppg_index_chunk_max_bytes": (i32, [vp]),
    "ppg_index_point": (C.c_int, [vp, i32, P(i64), P(i64), P(i32), P(i32)]),
    "ppg_index_window": (vp, [vp, i32]),
    "ppg_index_offset": (vp, [vp, i32]),
    "ppg_index_free": (None, [vp]),
    "ppg_index_validate": (C.c_int, [vp, i32, i32]),
    "ppg_device_count": (C.c_int, [P(C.c_int)]),
    "ppg_open": (C.c_int, [C.c_int, P(vp)]),
    "ppg_close": (None, [vp]),
    "ppg_ctx_stream": (vp, [vp]),
    "ppg_ctx_wait_stream": (C.c_int, [vp, vp]),
    "ppg_stream_wait_ctx": (C.c_int, [vp, vp]),
    "ppg_decompress_chunk": (C.c_int, [vp, vp, i32, vp, i64, vp, i64, P(i64), vp, i64, P(i64)]),
    "ppg_decompress_chunk_stats": (C.c_int, [vp, P(i64), P(i64), P(i64)]),
    "ppg_decompress_chunk_submit": (C.c_int, [vp, vp, i32, vp, i64, vp, i64, vp, i64, P(vp)]),
    "ppg_decompress_chunk_wait": (C.c_int, [vp, vp, P(i64), P(i64)]),
    "ppg_decompress_chunk_split_stats": (C.c_int, [vp, P(i64), P(i64)]),
    "ppg_shard_create": (C.c_int, [vp, vp, i32, i32, vp, i64, C.c_int, i64, P(vp)]),
    "ppg_shard_free": (None, [vp]),
    "ppg_shard_run": (C.c_int, [vp]),
    "ppg_shard_results": (C.c_int, [vp, vp, vp, vp, vp, vp]),
    "ppg_shard_total_records": (i64, [vp]),
    "ppg_shard_batches": (i32, [vp]),
    "ppg_shard_set_split": (C.c_int, [vp, i32, vp, vp, vp]),
    "ppg_shard_copy_chunk": (C.c_int, [vp, i32, vp, i64, P(i64)]),
    "ppg_shard_copy_records": (C.c_int, [vp, i32, vp, i64, P(i64)]),
    "ppg_shard_record_base": (C.c_int, [vp, vp]),
    "ppg_shard_copy_output": (C.c_int, [vp, i64, i64, vp, C.c_int]),
    "ppg_shard_keys": (C.c_int, [vp, vp, i64]),
    "ppg_shard_set_keys": (C.c_int, [vp, vp, i64]),
    "ppg_shard_counts_to_device": (C.c_int, [vp, vp]),
    "ppg_shard_timing": (C.c_int, [vp, P(C.c_float), P(C.c_float), P(C.c_float)]),
    "ppg_file_decompress_all": (C.c_int, [vp, vp, C.c_char_p, i32, i32, i64, C.c_int, vp, P(i64), P(C.c_double)]),
    "ppg_file_release": (C.c_int, [vp]),
    "ppg_version": (C.c_char_p, []),
    "ppg_build_id": (C.c_char_p, []),
    "ppg_cursor_open": (C.c_int, [vp, vp, C.c_char_p, i32, i32, i64, C.c_int, P(vp)]),
    "ppg_cursor_next": (C.c_int, [vp, vp]),
    "ppg_cursor_batches": (i32, [vp]),
    "ppg_cursor_close": (None, [vp]),
    "ppg_comm_unique_id": (C.c_int, [vp]),
    "ppg_comm_init": (C.c_int, [vp, i32, i32, vp, P(vp)]),
    "ppg_comm_from_rccl": (C.c_int, [vp, vp, i32, i32, P(vp)]),
    "ppg_comm_init_host": (C.c_int, [i32, i32, C.c_char_p, P(vp)]),
    "ppg_comm_rank": (C.c_int, [vp, P(i32), P(i32)]),
    "ppg_comm_free": (None, [vp]),
    "ppg_rccl_version": (C.c_int, [P(C.c_int)]),
    "ppg_partition": (C.c_int, [vp, i32, i32, i32, vp]),
    "ppg_shard_gather_counts": (C.c_int, [vp, vp, vp, vp, vp, P(i64)]),
    "ppg_dist_decompress_all": (C.c_int, [vp, vp, vp, C.c_char_p, i64, vp, vp, P(i64)]),
    "ppg_shard_keys_ready": (C.c_int, [vp]),
    "ppg_comm_alltoallv": (C.c_int, [vp, vp, vp, vp, C.c_int]),
    "ppg_pairs_create": (C.c_int, [P(vp)]),
    "ppg_pairs_check": (C.c_int, [vp, vp, vp, vp, vp]),
    "ppg_pairs_records": (C.c_int, [vp, i32, i64, i64, vp]),
    "ppg_pairs_free": (None, [vp]),
    "ppg_pairs_emit_begin": (C.c_int, [vp, vp, vp, vp, i64, i64]),
    "ppg_pairs_emit_run": (C.c_int, [vp, vp, vp, i64, i64]),
    "ppg_pairs_emit_next": (C.c_int, [vp, P(i64), P(i64)]),
    "ppg_pairs_chunk": (C.c_int, [vp, i64, i32, P(vp), P(i64), P(vp), P(i64)]),
    "ppg_pairs_copy_chunk": (C.c_int, [vp, i64, i32, vp, i64, P(i64), vp, i64, P(i64)]),
    "ppg_pairs_emit_stats": (C.c_int, [vp, P(C.c_double), i32]),
}


class PpgBatch(C.Structure):
    """ppg_batch (include/ppgpu.h)."""
    _fields_ = [("first_chunk", C.c_int32), ("nchunks", C.c_int32), ("record_base", C.c_int64),
                ("nrecords", C.c_int64), ("text", C.c_void_p), ("raw_off", C.POINTER(C.c_int64)),
                ("desc", C.POINTER(C.c_uint32)), ("rec_off", C.POINTER(C.c_int64))]


class PpgPairResult(C.Structure):
    """ppg_pair_result (include/ppgpu.h)."""
    _fields_ = [("pairs", C.c_int64), ("records", C.c_int64 * 2), ("duplicates", C.c_int64 * 2),
                ("mismatches", C.c_int64), ("first_bad", C.c_int64), ("first_keys", C.c_int64 * 2)]


for _name, (_res, _args) in _SIGS.items():
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args

EXPORTED = sorted(_SIGS)

_synth = None


def synth():
    """libppgsynth.so: synthetic Generator-shape FASTQ and gzip (tests / bench input only)."""
    global _synth
    if _synth is None:
        s = _load(SYNTH_PATH, "libppgsynth.so")
        s.ppg_synth_fastq_size.restype = i64
        s.ppg_synth_fastq_size.argtypes = [i64, i64, C.c_int]
        s.ppg_synth_fastq.restype = i64
        s.ppg_synth_fastq.argtypes = [C.c_uint64, i64, i64, C.c_int, vp, i64, C.c_int]
        s.ppg_synth_fastq_size_mate.restype = i64
        s.ppg_synth_fastq_size_mate.argtypes = [i64, i64, C.c_int, C.c_int]
        s.ppg_synth_fastq_mate.restype = i64
        s.ppg_synth_fastq_mate.argtypes = [C.c_uint64, C.c_int, i64, i64, C.c_int, vp, i64, C.c_int]
        s.ppg_synth_illumina_size.restype = i64
        s.ppg_synth_illumina_size.argtypes = [C.c_uint64, i64, i64]
        s.ppg_synth_illumina.restype = i64
        s.ppg_synth_illumina.argtypes = [C.c_uint64, i64, i64, vp, i64, C.c_int]
        s.ppg_synth_gzip.restype = i64
        s.ppg_synth_gzip.argtypes = [vp, i64, C.c_int, i64, C.c_int, vp, i64]
        s.ppg_synth_segment.restype = i64
        s.ppg_synth_segment.argtypes = [vp, i64, C.c_int, i64, C.c_int, vp, i64, P(C.c_uint32)]
        s.ppg_synth_tiled_frame.restype = None
        s.ppg_synth_tiled_frame.argtypes = [C.c_uint32, i64, i64, vp, vp]
        s.ppg_synth_segment_blocks.restype = i64
        s.ppg_synth_segment_blocks.argtypes = [vp, i64, i64, vp, vp, i64]
        s.ppg_synth_tiled_points.restype = i64
        s.ppg_synth_tiled_points.argtypes = [vp, i64, i64, i64, vp, vp, i64, u32, vp, vp, vp, vp, vp, i64]
        s.ppg_synth_tiled_fill.restype = None
        s.ppg_synth_tiled_fill.argtypes = [vp, i64, vp, vp, vp, i64, i64, vp, vp]
        _synth = s
    return _synth

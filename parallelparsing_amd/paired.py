"""Paired-end, record-aligned pair chunks (BASELINE configs[4]).

The reference names the goal only (README.md:9); there is no code and no oracle beyond per-file
parity.  A read pair is two files R1/R2 whose record i belong together: Generator-shape headers
"SRR<id>.<spot>.<mate>" with equal spot numbers.  Each file is decoded by its own
DecompressAll (the per-file parity path); pair chunk j is pairs [j*K, (j+1)*K), pair i being the
i-th record of both files once the records the reference parses twice (a Point on a
record start) are dropped -- else every later pair would shift by one.

The pairing runs in libppgpu behind the C ABI (ppg_pairs_*, csrc/ppg_pairs.hip): spot keys on the
device, duplicates dropped through a map, keys compared; on N ranks every key moves to the rank
that owns its pair number over the library's communicator (RCCL ncclSend/ncclRecv over xGMI, or
the host transport for a one-GPU rehearsal).  This module is the Python surface over it, as
interop/GpuPairedFASTQ.cs is the C# one.
"""
import ctypes as C

import numpy as np

from . import Device, IndexIO, Shard, records_from_descriptors
from ._lib import lib, check, PpgPairResult

DUP = -2      # key of a record parsed twice (Q1), dropped before pairing
NOKEY = -1    # identifier without an "SRR<id>.<spot>." field


def attach_keys(shard, max_records):
    """Give a shard a device key buffer that every output batch of its later runs fills
    (ppg_shard_set_keys): pairing then works on shards of any number of batches, e.g. configs[4]'s
    2 x 25 GB on one GPU, whose outputs cannot both stay resident."""
    import torch
    keys = torch.empty(max(1, int(max_records)), dtype=torch.int64, device=torch.device("cuda", shard.dev.device))
    shard.dev.wait_stream(torch.cuda.current_stream(keys.device))   # the block may be recycled
    return shard.set_keys(keys)


def shard_keys(shard):
    """Spot numbers of all records of a shard, in record order, as a device tensor (int64; DUP /
    NOKEY markers kept) -- a diagnostic view; pairing itself is Pairs.check.  GPU kernel
    ppg_record_keys: run per batch during the shard's run when attach_keys() gave it a buffer, else
    (one-batch shards) extracted now."""
    import torch
    n = shard.total_records
    if getattr(shard, "_keys", None) is not None:
        if n > shard._keys.numel():
            raise ValueError("key buffer smaller than the shard's records")
        if not lib.ppg_shard_keys_ready(shard.handle):   # attached after the run, or the run failed
            raise ValueError("the shard's key buffer was not filled by its last run (attach keys before run())")
        # the keys were written on the ctx stream: torch's stream must not read them earlier
        shard.dev.stream_wait(torch.cuda.current_stream(shard._keys.device))
        return shard._keys[:n]
    dev = torch.device("cuda", shard.dev.device)
    keys = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    # the kernel writes on the ctx's stream: torch's caching allocator may have handed out a block
    # that kernels still queued on torch's stream read, so the ctx waits for torch's stream first
    shard.dev.wait_stream(torch.cuda.current_stream(dev))
    check(lib.ppg_shard_keys(shard.handle, C.c_void_p(keys.data_ptr()), n), "ppg_shard_keys")
    return keys[:n]


class Pairs:
    """ppg_pairs: the device pair check of an R1 and an R2 shard (ppg_pairs_check), on one rank or
    over a Comm; keeps its device scratch across checks."""

    def __init__(self):
        h = C.c_void_p()
        check(lib.ppg_pairs_create(C.byref(h)), "ppg_pairs_create")
        self._h = h

    def check(self, r1, r2, comm=None):
        """{pairs, records, duplicates, mismatches, first_bad, first_keys} -- every rank gets the
        same result (duplicates: this rank's)."""
        r = PpgPairResult()
        check(lib.ppg_pairs_check(self._h, r1.handle, r2.handle, comm.handle if comm is not None else None,
                                  C.byref(r)), "ppg_pairs_check")
        return {"pairs": r.pairs, "records": tuple(r.records), "duplicates": tuple(r.duplicates),
                "mismatches": r.mismatches, "first_bad": r.first_bad, "first_keys": tuple(r.first_keys)}

    def records(self, f, lo, hi):
        """Shard record numbers (file f: 0 = R1) of pair numbers [lo, hi); -1 where another rank
        holds the record."""
        out = np.zeros(max(1, hi - lo), np.int64)
        check(lib.ppg_pairs_records(self._h, int(f), int(lo), int(hi), C.c_void_p(out.ctypes.data)), "ppg_pairs_records")
        return out[:hi - lo]

    # ---- record-aligned pair chunks (ppg_pairs_emit_*) ----
    def emit(self, r1, r2, pair_chunk, comm=None, window_bytes=0):
        """Yield windows (j0, j1) of this rank's record-aligned pair chunks [j0, j1) of `pair_chunk`
        pairs, packed on the device (ppg_pairs_emit_begin / _next).  After check() on the same
        shards and comm; a window's halves are read with chunk() / copy_chunk() before the next one
        is made.  N ranks: every rank iterates (the first window is collective)."""
        check(lib.ppg_pairs_emit_begin(self._h, r1.handle, r2.handle, comm.handle if comm is not None else None,
                                       int(pair_chunk), int(window_bytes)), "ppg_pairs_emit_begin")
        j0, j1 = C.c_int64(), C.c_int64()
        while True:
            rc = lib.ppg_pairs_emit_next(self._h, C.byref(j0), C.byref(j1))
            if rc == 1:   # PPG_STREAM_END
                return
            check(rc, "ppg_pairs_emit_next")
            yield j0.value, j1.value

    def emit_run(self, r1, r2, pair_chunk, window_bytes=0):
        """The same windows with no check first, the emission driving the shards' own run
        (ppg_pairs_emit_run): each output batch of both shards decoded once and its records packed
        while resident.  Both shards need attach_keys; after the last window both have run (as
        Shard.run leaves them) and check() may follow."""
        for r in (r1, r2):
            if r._on_device:
                r._torch_order()   # the caller may have rewritten comp since the last run
        check(lib.ppg_pairs_emit_run(self._h, r1.handle, r2.handle, int(pair_chunk), int(window_bytes)),
              "ppg_pairs_emit_run")
        j0, j1 = C.c_int64(), C.c_int64()
        while True:
            rc = lib.ppg_pairs_emit_next(self._h, C.byref(j0), C.byref(j1))
            if rc == 1:   # PPG_STREAM_END
                return
            check(rc, "ppg_pairs_emit_next")
            yield j0.value, j1.value

    def chunk(self, j, f):
        """(device address of the bytes, length, device address of the descriptors, records) of
        file f's half of pair chunk j (current window)."""
        b, d, n, r = C.c_void_p(), C.c_void_p(), C.c_int64(), C.c_int64()
        check(lib.ppg_pairs_chunk(self._h, int(j), int(f), C.byref(b), C.byref(n), C.byref(d), C.byref(r)),
              "ppg_pairs_chunk")
        return b.value, n.value, d.value, r.value

    def copy_chunk(self, j, f):
        """(bytes, (n,4) uint32 descriptors) of file f's half of pair chunk j, in host memory."""
        _, n, _, r = self.chunk(j, f)
        buf = np.empty(max(1, n), np.uint8)
        desc = np.empty((max(1, r), 4), np.uint32)
        ln, nr = C.c_int64(), C.c_int64()
        check(lib.ppg_pairs_copy_chunk(self._h, int(j), int(f), C.c_void_p(buf.ctypes.data), buf.size, C.byref(ln),
                                       C.c_void_p(desc.ctypes.data), desc.shape[0], C.byref(nr)), "ppg_pairs_copy_chunk")
        return buf[:n], desc[:r]

    def emit_stats(self):
        v = (C.c_double * 8)()
        check(lib.ppg_pairs_emit_stats(self._h, v, 8), "ppg_pairs_emit_stats")
        return {"rerun_ms": v[0], "pack_ms": v[1], "exchange_ms": v[2], "emit_ms": v[3], "reruns": int(v[4]),
                "pair_chunks": int(v[5]), "mine": (int(v[6]), int(v[7]))}

    def close(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.ppg_pairs_free(h)
            self._h = None

    def __del__(self):
        self.close()


def require_pairs(res):
    """Raise ValueError unless a Pairs.check result is a read pair; returns the pair count."""
    if res["records"][0] != res["records"][1]:
        raise ValueError(f"R1 has {res['records'][0]} records, R2 {res['records'][1]}: not a read pair")
    if res["mismatches"]:
        raise ValueError(f"{res['mismatches']} mismatched pairs; first at pair {res['first_bad']}: spot "
                         f"{res['first_keys'][0]} vs {res['first_keys'][1]}")
    return res["pairs"]


def _read_range(path, index):
    n = index.Count - 1
    _, i0, _, _ = index.point_fields(0)
    _, i1, _, _ = index.point_fields(n)
    with open(path, "rb") as f:
        f.seek(i0 - 1)
        return f.read(i1 - i0 + 1)


class PairedFASTQ:
    """Two BatchedFASTQ streams zipped into record-aligned pair chunks of `pair_chunk` records
    (default 50,000, BASELINE configs[4]).  Both files are decoded on one GPU and their pairing
    is verified on the device (ppg_pairs_check) before any pair is handed out; the pair chunks
    themselves are packed on the device by the library (ppg_pairs_emit_*) window by window, and
    each half is one copy out (FastqRecords over its bytes and descriptors)."""

    def __init__(self, index1, gz1, index2, gz2, pair_chunk=50_000, device=None, out_capacity=0,
                 window_bytes=0):
        self.index = [IndexIO.Deserialize(i) if isinstance(i, str) else i for i in (index1, index2)]
        self.paths = [gz1, gz2]
        self.K = int(pair_chunk)
        self.dev = device or Device.default()
        self.shards = []
        for ix, p in zip(self.index, self.paths):
            sh = Shard(ix, _read_range(p, ix), 0, ix.Count - 1, device=self.dev, out_capacity=out_capacity)
            if sh.batches > 1:   # the spot keys per batch while resident (ppg_shard_set_keys)
                attach_keys(sh, int(ix.point_fields(ix.Count - 1)[0]) // 32 + 4096)
            self.shards.append(sh.run())
        self._pairs = Pairs()
        self.result = self._pairs.check(self.shards[0], self.shards[1])
        self.pairs = require_pairs(self.result)
        self.window_bytes = window_bytes
        self._it = None          # the emission pair_chunk() advances (random access)
        self._win = (0, 0)       # its current window [j0, j1)

    def Count(self):
        return self.pairs

    @property
    def chunks(self):
        return (self.pairs + self.K - 1) // self.K

    def pair_chunks(self):
        """Yield (j, R1 records, R2 records) for every pair chunk in order."""
        self._it, self._win = None, (0, 0)   # this emission replaces pair_chunk()'s
        for j0, j1 in self._pairs.emit(self.shards[0], self.shards[1], self.K, window_bytes=self.window_bytes):
            for j in range(j0, j1):
                yield (j,) + tuple(records_from_descriptors(*self._pairs.copy_chunk(j, f)) for f in (0, 1))

    def pair_chunk(self, j):
        """(R1 records, R2 records) of pair chunk j: pairs [j*K, min((j+1)*K, Count)).  Only chunk j
        is copied out: the emission's windows are advanced (not copied) until one holds j, and kept
        for the next call, so ascending calls walk the windows once (every earlier pair
        chunk was copied and parsed before, O(j) per call); a j behind the current window restarts
        the emission (multi-batch shards re-run their batches)."""
        if not 0 <= j < self.chunks:
            raise IndexError(j)
        j0, j1 = self._win
        if not (j0 <= j < j1):
            if self._it is None or j < j0:
                self._it = self._pairs.emit(self.shards[0], self.shards[1], self.K, window_bytes=self.window_bytes)
            for w in self._it:
                self._win = w
                if w[0] <= j < w[1]:
                    break
            else:
                self._it, self._win = None, (0, 0)
                raise IndexError(j)
        return tuple(records_from_descriptors(*self._pairs.copy_chunk(j, f)) for f in (0, 1))

    def __iter__(self):
        for _, a, b in self.pair_chunks():
            yield from zip(a, b)

"""Synthetic "tiled" .fastq.gz for the 50 GB configuration (bench input, not the hot path).

One gzip member = header + S_deflate * T + empty final block + trailer, where S is a segment of
whole Generator-shape records (synth.cpp) deflated pigz-style with no history before it and a
byte-aligned sync-flush end, so its compressed bytes can be repeated T times; the stream
decompresses to S^T.  The CreateIndex points of the whole file are derived from the segment's
deflate block list (ppg_synth_tiled_points), exactly as Core.BuildDeflateIndex (Core.cs:14-131)
would place them — tests/test_tiled.py checks this against the oracle's serial pass.
"""
import ctypes as C

import numpy as np

from ._lib import synth
from . import Index


def saved_bytes_estimate(records, read_len=150, mate=0, blank_lines=False):
    """Upper bound on what TiledFile.save writes for a member of `records`-record segments: the
    segment text, its deflate (well under half the text at level 6), the block list and the points
    (a few hundred bytes per chunk) -- for the free-space check of the directory it goes to."""
    n = synth().ppg_synth_fastq_size_mate(0, records, read_len, mate)
    if blank_lines:
        n += records
    return int(1.6 * n) + (64 << 20)


class TiledFile:
    def __init__(self, records, repeats, chunksize, read_len=150, seed=0, level=6, piece=4 << 20, threads=16,
                 mate=0, blank_lines=False):
        S = synth()
        self.records, self.repeats, self.chunksize = records, repeats, chunksize
        self.blank_lines = blank_lines
        n = S.ppg_synth_fastq_size_mate(0, records, read_len, mate)
        self.text = np.empty(n, np.uint8)
        assert S.ppg_synth_fastq_mate(seed, mate, 0, records, read_len, C.c_void_p(self.text.ctypes.data), n,
                                      threads) == n
        if blank_lines:
            # an empty line after every record: every chunk fails R-P3 and takes the
            # declined-chunk parse (ppg_parse_chain); each record still parses, its Identifier
            # starting with the '@' (the blank line is what Parsing.cs:19 skips)
            ends = np.nonzero(self.text == 10)[0][3::4] + 1
            self.text = np.insert(self.text, ends, np.uint8(10))
            n = self.text.size
        cap = n // 2 + (1 << 20)
        seg = np.empty(cap, np.uint8)
        crc = C.c_uint32()
        m = S.ppg_synth_segment(C.c_void_p(self.text.ctypes.data), n, level, piece, threads,
                                C.c_void_p(seg.ctypes.data), cap, C.byref(crc))
        assert m > 0
        self.seg = seg[:m].copy()
        self.seg_crc = crc.value
        self.header = np.zeros(10, np.uint8)
        self.tail = np.zeros(10, np.uint8)
        S.ppg_synth_tiled_frame(self.seg_crc, n, repeats, C.c_void_p(self.header.ctypes.data),
                                C.c_void_p(self.tail.ctypes.data))
        self.file_len = 10 + repeats * m + 10
        # deflate block ends of the segment
        bcap = m // 16 + 1024
        be, oe = np.empty(bcap, np.int64), np.empty(bcap, np.int64)
        nb = S.ppg_synth_segment_blocks(C.c_void_p(self.seg.ctypes.data), m, n, C.c_void_p(be.ctypes.data),
                                        C.c_void_p(oe.ctypes.data), bcap)
        assert 0 < nb <= bcap
        self.block_bit_end, self.block_out_end = be[:nb].copy(), oe[:nb].copy()
        # point metadata for the whole member (windows/offsets are filled per range: windows())
        pcap = (records * repeats) // max(1, chunksize - 8) + 64
        pcap = min(pcap, nb * repeats + 2)
        out, inp = np.empty(pcap, np.int64), np.empty(pcap, np.int64)
        bits, ol, at = np.empty(pcap, np.int32), np.empty(pcap, np.int32), np.empty(pcap, np.int64)
        npts = S.ppg_synth_tiled_points(C.c_void_p(self.text.ctypes.data), n, m, repeats,
                                        C.c_void_p(self.block_bit_end.ctypes.data),
                                        C.c_void_p(self.block_out_end.ctypes.data), nb, chunksize & 0xFFFFFFFF,
                                        C.c_void_p(out.ctypes.data), C.c_void_p(inp.ctypes.data),
                                        C.c_void_p(bits.ctypes.data), C.c_void_p(ol.ctypes.data),
                                        C.c_void_p(at.ctypes.data), pcap)
        assert npts > 0, npts
        self.p_output, self.p_input, self.p_bits = out[:npts].copy(), inp[:npts].copy(), bits[:npts].copy()
        self.p_offlen, self._p_at = ol[:npts].copy(), at[:npts].copy()
        self.npoints = int(npts)

    # ---- sharing one build between the ranks of a job (bench.py, N > 1) ----
    _ARRAYS = ("text", "seg", "header", "tail", "block_bit_end", "block_out_end", "p_output", "p_input", "p_bits",
               "p_offlen", "_p_at")
    _SCALARS = ("records", "repeats", "chunksize", "blank_lines", "seg_crc", "file_len", "npoints")

    def save(self, d):
        """Write the member's description (segment text, deflated segment, block list, points) to
        directory d, e.g. under /dev/shm, for TiledFile.load; "ready" is written last."""
        import json
        import os
        os.makedirs(d, exist_ok=True)
        for k in self._ARRAYS:
            np.save(os.path.join(d, k.lstrip("_") + ".npy"), getattr(self, k))
        with open(os.path.join(d, "meta.json"), "w") as f:
            json.dump({k: (bool(v) if isinstance(v, (bool, np.bool_)) else int(v))
                       for k in self._SCALARS for v in [getattr(self, k)]}, f)
        with open(os.path.join(d, "ready"), "w") as f:
            f.write("ok")

    @classmethod
    def load(cls, d):
        """The TiledFile saved in d, its arrays memory-mapped read-only (no rebuild, no copy: the
        ranks of one node share the pages)."""
        import json
        import os
        t = cls.__new__(cls)
        with open(os.path.join(d, "meta.json")) as f:
            for k, v in json.load(f).items():
                setattr(t, k, v)
        for k in cls._ARRAYS:
            setattr(t, k, np.load(os.path.join(d, k.lstrip("_") + ".npy"), mmap_mode="r"))
        return t

    def expected_records(self):
        """Records DecompressAll emits for the whole member: every record once, plus one duplicate
        per Point that falls exactly on a record start (its offset then holds the whole previous
        record, which the next chunk parses again: SURVEY Q1, Core.cs:86-94 + Parsing.cs:11-51)."""
        dup = 0
        tl = self.text.size
        for p in np.nonzero(self.p_offlen)[0]:
            a = int(self._p_at[p]) % tl
            n = int(self.p_offlen[p])
            seg = self.text[a:a + n] if a + n <= tl else np.concatenate([self.text[a:], self.text[:a + n - tl]])
            dup += int(np.count_nonzero(seg == 10) == (5 if self.blank_lines else 4))
        return self.records * self.repeats + dup

    def windows(self, lo=0, hi=None):
        """(windows uint8[(hi-lo)*32768], offsets uint8[...]) of points [lo, hi)."""
        if hi is None:
            hi = self.npoints
        win = np.empty((hi - lo) * 32768, np.uint8)
        offs = np.empty(max(1, int(self.p_offlen[lo:hi].sum())), np.uint8)
        synth().ppg_synth_tiled_fill(C.c_void_p(self.text.ctypes.data), self.text.size,
                                     C.c_void_p(self.p_output.ctypes.data), C.c_void_p(self.p_offlen.ctypes.data),
                                     C.c_void_p(self._p_at.ctypes.data), lo, hi, C.c_void_p(win.ctypes.data),
                                     C.c_void_p(offs.ctypes.data))
        return win, offs[: int(self.p_offlen[lo:hi].sum())]

    def side_points(self, lo=0, hi=None, per_chunk=2):
        """Side points for Shard.set_split over points [lo, hi): up to per_chunk - 1 deflate block
        starts inside each chunk, spread evenly by output.  (bits, outputs, windows) with absolute
        file bit positions and output offsets, windows = the 32 KiB of text before each."""
        if hi is None:
            hi = self.npoints
        po = self.p_output[lo:hi]
        if per_chunk < 2 or po.size < 2:
            return np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.uint8)
        tl, segbits = self.text.size, 8 * self.seg.size
        frac = np.arange(1, per_chunk, dtype=np.float64) / per_chunk
        tgt = (po[:-1, None] + (np.diff(po)[:, None] * frac[None, :])).astype(np.int64).ravel()
        # first block end at or after each target (block ends repeat every segment)
        r = tgt // tl
        b = np.searchsorted(self.block_out_end, tgt - r * tl, side="left")
        wrap = b >= self.block_out_end.size
        r, b = np.where(wrap, r + 1, r), np.where(wrap, 0, b)
        outs = r * tl + self.block_out_end[b]
        bits = 80 + r * segbits + self.block_bit_end[b]
        # strictly inside their chunk, one per block end
        c = np.repeat(np.arange(po.size - 1), per_chunk - 1)
        keep = (outs > po[c]) & (outs < po[c + 1])
        outs, bits = outs[keep], bits[keep]
        outs, first = np.unique(outs, return_index=True)
        bits = bits[first]
        win = np.empty(outs.size * 32768, np.uint8)
        z32, z64 = np.zeros(max(1, outs.size), np.int32), np.zeros(max(1, outs.size), np.int64)
        if outs.size:
            synth().ppg_synth_tiled_fill(C.c_void_p(self.text.ctypes.data), tl, C.c_void_p(outs.ctypes.data),
                                         C.c_void_p(z32.ctypes.data), C.c_void_p(z64.ctypes.data), 0, outs.size,
                                         C.c_void_p(win.ctypes.data), C.c_void_p(z64.ctypes.data))
        return bits.astype(np.int64), outs.astype(np.int64), win

    @property
    def text_len(self):
        return self.text.size

    def index(self, lo=0, hi=None):
        """Index (libppgpu) of points [lo, hi): chunks lo..hi-2 of the member."""
        if hi is None:
            hi = self.npoints
        win, offs = self.windows(lo, hi)
        return Index.from_points(self.p_output[lo:hi], self.p_input[lo:hi], self.p_bits[lo:hi], win,
                                 self.p_offlen[lo:hi], offs)

    def file_bytes(self, lo=0, hi=None):
        """Bytes [lo, hi) of the tiled file (host copy; for tests and the CPU baseline sample)."""
        if hi is None:
            hi = self.file_len
        out = np.empty(hi - lo, np.uint8)
        m = self.seg.size
        pos = lo
        while pos < hi:
            if pos < 10:
                take = min(hi, 10) - pos
                out[pos - lo:pos - lo + take] = self.header[pos:pos + take]
            elif pos < 10 + self.repeats * m:
                off = (pos - 10) % m
                take = min(hi - pos, m - off)
                out[pos - lo:pos - lo + take] = self.seg[off:off + take]
            else:
                off = pos - 10 - self.repeats * m
                take = hi - pos
                out[pos - lo:pos - lo + take] = self.tail[off:off + take]
            pos += take
        return out

    def fill_device(self, dst, lo, hi):
        """Write file bytes [lo, hi) into the uint8 torch tensor dst (on a GPU) by device copies
        of the segment: the 50 GB member never exists in host memory."""
        import torch
        dev = dst.device
        seg = torch.from_numpy(self.seg).to(dev)
        hdr = torch.from_numpy(self.header).to(dev)
        tail = torch.from_numpy(self.tail).to(dev)
        m = self.seg.size
        pos = lo
        while pos < hi:
            if pos < 10:
                take = min(hi, 10) - pos
                dst[pos - lo:pos - lo + take].copy_(hdr[pos:pos + take])
            elif pos < 10 + self.repeats * m:
                off = (pos - 10) % m
                take = min(hi - pos, m - off)
                dst[pos - lo:pos - lo + take].copy_(seg[off:off + take])
            else:
                off = pos - 10 - self.repeats * m
                take = hi - pos
                dst[pos - lo:pos - lo + take].copy_(tail[off:off + take])
            pos += take

"""BASELINE.json configs[0]: a 1 M-read synthetic .fastq.gz, chunk = 10,000, DecompressAll on the
host CPU -- the plumbing configuration, run here with the CPU restatement of the reference
(oracle/oracle.c: Core.BuildDeflateIndex + the threaded BatchedFASTQ DecompressAll over zlib 1.2.11)
and the library's host CreateIndex / IndexIO, no GPU.  (configs[0] had no 1 M-read run.)"""
import ctypes as C
import zlib

import numpy as np

import parallelparsing_amd as pp
from oracle import oracle as O


def test_configs0_one_million_reads_on_cpu(tmp_path):
    S = pp.synth()
    nrec = 1_000_000
    sz = S.ppg_synth_fastq_size(0, nrec, 150)
    txt = np.zeros(sz, np.uint8)
    S.ppg_synth_fastq(2024, 0, nrec, 150, C.c_void_p(txt.ctypes.data), sz, 8)
    gzb = np.zeros(sz // 2 + (1 << 20), np.uint8)
    L = S.ppg_synth_gzip(C.c_void_p(txt.ctypes.data), sz, 6, 4 << 20, 8, C.c_void_p(gzb.ctypes.data), gzb.size)
    gz = gzb[:L].tobytes()
    assert int.from_bytes(gz[-8:-4], "little") == zlib.crc32(txt.tobytes())
    # CreateIndex: the library's host restatement == the oracle's, and the .gzi round-trips
    ix = pp.Core.BuildDeflateIndex(gz, 10000)
    oi = O.build_index(gz, 10000)
    assert ix.Count == oi.count > 90
    for i in range(0, ix.Count, 7):
        o, n, b, w, off = oi.point(i)
        p = ix[i]
        assert (p.Output, p.Input, p.Bits, p.Window, p.offset) == (o, n, b, w, off), i
    pp.IndexIO.Serialize(ix, str(tmp_path / "x.gzi"))
    oi.serialize(str(tmp_path / "o.gzi"))
    assert (tmp_path / "x.gzi").read_bytes() == (tmp_path / "o.gzi").read_bytes()
    # DecompressAll on the host: every record counted once (no Q1 duplicates at zlib -6 here)
    tot, counts = O.decompress_all(gz, oi, threads=8)
    assert tot == nrec and counts.sum() == nrec
    assert (counts[:-1] >= 10000 - 7).all()   # R-I5: a chunk ends after > chunksize - 8 of its records

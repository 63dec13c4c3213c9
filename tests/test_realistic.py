"""Parity on realistic FASTQ at BASELINE's 1 M-read size (VERDICT r02 missing #3 / next #3).

The Generator shape the bench uses has no '@' outside headers, so SURVEY Q2 stays inert there.
Real Illumina data (Phred+33 qualities over '!'..'J') carries '@' (Q31) inside quality lines:
Core.BuildDeflateIndex counts each one as a record start (Core.cs:86-94), so Points land inside
records, the next chunk's Parse starts mid-quality (Parsing.cs:11-51) and emits the reference's
deterministic misparse.  These files (libppgsynth's Illumina-like records: variable read lengths,
N bases, qualities over '!'..'J') are decoded on the GPU and compared chunk by chunk -- bytes and
record tables -- with the oracle (oracle.c restating Core.cs / Parsing.cs over zlib 1.2.11); a
Z_HUFFMAN_ONLY member of the same text ends blocks at arbitrary bytes, so Points also fall on
record starts (the duplicated record) and anywhere inside lines.  The CPU part checks the host CreateIndex against the oracle on the same data."""
import ctypes as C
import hashlib
import zlib

import numpy as np
import pytest

import parallelparsing_amd as pp
from oracle import oracle as O


def illumina_text(nrec, seed=7):
    S = pp.synth()
    sz = S.ppg_synth_illumina_size(seed, 0, nrec)
    txt = np.zeros(sz, np.uint8)
    assert S.ppg_synth_illumina(seed, 0, nrec, C.c_void_p(txt.ctypes.data), sz, 8) == sz
    return txt


def gzip_level6(txt):
    S = pp.synth()
    gzb = np.zeros(txt.size // 2 + (1 << 20), np.uint8)
    L = S.ppg_synth_gzip(C.c_void_p(txt.ctypes.data), txt.size, 6, 4 << 20, 8, C.c_void_p(gzb.ctypes.data), gzb.size)
    assert L > 0
    return gzb[:L].tobytes()


def gzip_huffman_only(txt):
    c = zlib.compressobj(6, zlib.DEFLATED, 31, 8, zlib.Z_HUFFMAN_ONLY)
    return c.compress(txt.tobytes()) + c.flush()


def record_starts(txt):
    """Offsets of true record starts (the '@' of every 4th line)."""
    nl = np.flatnonzero(txt == 10)
    return np.concatenate([[0], nl[3:-1:4] + 1])


def q2_shifted_points(ix, txt):
    """Points whose offset (the partial record carried into the next chunk) does not start at a
    true record start: CreateIndex reset it at an '@' inside a quality line."""
    starts = set(record_starts(txt).tolist())
    out = 0
    for i in range(1, ix.Count - 1):
        o, _, _, ol = ix.point_fields(i)
        if ol and (o - ol) not in starts:
            out += 1
    return out


def _index_matches_oracle(gz, chunk):
    ix = pp.Core.BuildDeflateIndex(gz, chunk)
    oi = O.build_index(gz, chunk)
    assert ix.Count == oi.count
    for i in range(ix.Count):
        o, n, b, w, off = oi.point(i)
        p = ix[i]
        assert (p.Output, p.Input, p.Bits) == (o, n, b), i
        assert p.offset == off and p.Window == w, i
    return ix, oi


@pytest.mark.parametrize("comp", ["level6", "huffman_only"])
def test_realistic_index_equals_oracle_cpu(comp):
    """Host CreateIndex (ppg_index_build_mem) = the oracle's on Q2-heavy data (100k reads)."""
    txt = illumina_text(100_000, seed=3)
    gz = gzip_level6(txt) if comp == "level6" else gzip_huffman_only(txt)
    ix, _ = _index_matches_oracle(gz, 2000)
    assert q2_shifted_points(ix, txt) > (ix.Count - 2) // 10   # ~36% (level 6), ~19% (Huffman-only)


def _gpu_vs_oracle(gz, txt, chunk, device):
    ix, oi = _index_matches_oracle(gz, chunk)
    n = ix.Count - 1
    _, i0, _, _ = ix.point_fields(0)
    _, i1, _, _ = ix.point_fields(n)
    sh = pp.Shard(ix, np.frombuffer(gz[i0 - 1:i1], np.uint8), 0, n, device=device).run()
    r = sh.results()
    assert (r["status"] == 0).all()
    h = hashlib.sha256()
    exp_total = 0
    for k in range(n):
        exp = O.extract(gz, oi, k)
        got = sh.chunk_bytes(k).tobytes()
        assert got == exp, k
        h.update(got)
        er = O.parse(oi.point(k)[4], exp)
        assert np.array_equal(sh.chunk_records(k), er), k
        exp_total += len(er)
    assert h.hexdigest() == hashlib.sha256(txt.tobytes()).hexdigest()   # the whole text, in order
    assert sh.total_records == exp_total
    tot, _ = O.decompress_all(gz, oi, threads=8)
    assert tot == exp_total
    return ix, sh


@pytest.mark.gpu
def test_realistic_1m_reads_level6_equals_oracle(device):
    """configs[1]'s size (1 M reads, chunk = 10,000) with Illumina-like qualities: every chunk's
    bytes and record table equal the oracle's, and over a fifth of the Points (~36%) carry Q2-shifted offsets."""
    txt = illumina_text(1_000_000)
    gz = gzip_level6(txt)
    ix, sh = _gpu_vs_oracle(gz, txt, 10_000, device)
    q2 = q2_shifted_points(ix, txt)
    assert ix.Count > 200 and q2 > (ix.Count - 2) // 5, (ix.Count, q2)
    # the misparse is real: the reference's record count differs from the true one
    assert sh.total_records != 1_000_000


@pytest.mark.gpu
def test_realistic_1m_reads_huffman_only_equals_oracle(device):
    """The same 1 M reads as one Z_HUFFMAN_ONLY member: literal-only blocks end at arbitrary bytes,
    so Points fall on record starts (Q1 duplicates) or inside quality lines (Q2)."""
    txt = illumina_text(1_000_000)
    gz = gzip_huffman_only(txt)
    ix, sh = _gpu_vs_oracle(gz, txt, 10_000, device)
    assert q2_shifted_points(ix, txt) > (ix.Count - 2) // 10

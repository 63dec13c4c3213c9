"""ppg_parse_chain: chunks the newline census declines (an empty line somewhere: R-P3 fails) are
parsed from their newline positions, one wave per chunk, instead of byte by byte on one lane
(VERDICT r01 #9).  Both paths must give Parsing.Parse's records exactly (oracle/oracle.c restates
Parsing.cs:11-69), on texts whose empty lines land at every place the state machine's two skipped
bytes can fall (a record's start, the '+' position, the file's first byte, runs of them)."""
import zlib

import numpy as np
import pytest

import parallelparsing_amd as pp
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _text(seed):
    import ctypes as C
    S = pp.synth()
    nrec = 3000
    sz = S.ppg_synth_fastq_size(0, nrec, 100)
    txt = np.zeros(sz, np.uint8)
    S.ppg_synth_fastq(seed, 0, nrec, 100, C.c_void_p(txt.ctypes.data), sz, 4)
    lines = txt.tobytes().split(b"\n")
    rng = np.random.default_rng(seed)
    out = [b""] if seed % 2 else []                   # raw[0] == '\n' for odd seeds
    for i, ln in enumerate(lines):
        out.append(ln)
        r = rng.random()
        if r < 0.08:
            out += [b""] * int(rng.integers(1, 4))   # 1-3 empty lines anywhere
        elif r < 0.12 and i % 4 == 1:
            out.append(b"")                          # right after a sequence line: the skipped '+' byte
    return b"\n".join(out)


def _gz(text):
    c = zlib.compressobj(6, zlib.DEFLATED, 31)
    return c.compress(text) + c.flush()


@pytest.mark.parametrize("seed,chunk", [(1, 40), (2, 40), (3, 300), (4, 1000)])
def test_chain_parse_equals_oracle_and_bytewise(seed, chunk, device, monkeypatch):
    text = _text(seed)
    gz = _gz(text)
    ix = pp.Core.BuildDeflateIndex(gz, chunk)
    oi = O.build_index(gz, chunk)
    n = ix.Count - 1
    _, i0, _, _ = ix.point_fields(0)
    _, i1, _, _ = ix.point_fields(n)
    comp = np.frombuffer(gz[i0 - 1:i1], np.uint8)
    runs = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("PPG_PARSE_CHAIN", mode)
        sh = pp.Shard(ix, comp, 0, n, device=device).run()
        runs[mode] = sh
        r = sh.results()
        assert (r["status"] == 0).all()
        assert (r["flags"] & 8).sum() >= n // 2          # most chunks declined by the census
        tot = 0
        for k in range(n):
            exp = O.parse(oi.point(k)[4], O.extract(gz, oi, k))
            got = sh.chunk_records(k)
            assert np.array_equal(got, exp), (mode, k, len(got), len(exp))
            tot += len(exp)
        assert sh.total_records == tot
    assert (runs["0"].record_base() == runs["1"].record_base()).all()


def test_chain_parse_tiled_blank_member(device, monkeypatch):
    """bench.py --blank-lines at small scale: split and unsplit, chain and bytewise, agree with the
    member's expected record count."""
    from parallelparsing_amd.tiled import TiledFile
    tf = TiledFile(6000, 5, 700, threads=4, blank_lines=True)
    f = tf.file_bytes()
    ix = tf.index()
    n = tf.npoints - 1
    _, i0, _, _ = ix.point_fields(0)
    _, i1, _, _ = ix.point_fields(n)
    comp = f[i0 - 1:i1]
    base = None
    for mode in ("1", "0"):
        monkeypatch.setenv("PPG_PARSE_CHAIN", mode)
        for per in (1, 4):
            sh = pp.Shard(ix, comp, 0, n, device=device)
            if per > 1:
                sh.set_split(*tf.side_points(per_chunk=per))
            sh.run()
            assert sh.total_records == tf.expected_records()
            recs = [sh.chunk_records(k) for k in range(n)]
            if base is None:
                base = recs
            assert all(np.array_equal(a, b) for a, b in zip(recs, base))

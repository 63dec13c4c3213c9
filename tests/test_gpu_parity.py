"""GPU parity: the HIP path (through the C ABI) against the golden fixtures and the oracle.

Bit-exact decompressed bytes and identical per-chunk Parsing.Parse record tables are required
(integer/byte work: no tolerance)."""
import hashlib
import os
import zlib

import numpy as np
import pytest

import parallelparsing_amd as pp
from conftest import CASES, CORRUPT, GOLDEN, load_case
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def comp_range(gz, index, first, n):
    _, i0, _, _ = index.point_fields(first)
    _, i1, _, _ = index.point_fields(first + n)
    return np.frombuffer(gz[i0 - 1:i1], np.uint8)


@pytest.mark.parametrize("name", CASES)
def test_shard_matches_golden(name, device):
    meta, gz = load_case(name)
    ix = pp.Core.BuildDeflateIndex(gz, meta["chunksize"])
    assert ix.Count == meta["points"]
    n = ix.Count - 1
    sh = pp.Shard(ix, comp_range(gz, ix, 0, n), 0, n, device=device).run()
    r = sh.results()
    assert (r["status"] == 0).all()
    for k, c in enumerate(meta["chunks"]):
        b = sh.chunk_bytes(k)
        assert len(b) == c["out_len"], (name, k)
        assert sha(b) == c["sha256"], (name, k)
        rec = sh.chunk_records(k)
        assert len(rec) == c["records"], (name, k)
        assert sha(np.ascontiguousarray(rec, "<u4").tobytes()) == c["rec_sha256"], (name, k)
        # R-E5: the chunk ends right before its block's end-of-block code (flag bits 1|2|4)
        if k < n - 1:
            assert r["flags"][k] & 7 == 0, (name, k, r["flags"][k])
    assert sh.total_records == meta["total_records"]


@pytest.mark.parametrize("name", ["l6_c20", "memlevel1_c10", "stored_c50", "huffonly_c20"])
def test_extract_single_chunk(name, device):
    """README "Decompress": one checkpoint from the LazyFileReader slice (Core.cs:133-192)."""
    meta, gz = load_case(name)
    ix = pp.Core.BuildDeflateIndex(gz, meta["chunksize"])
    for k in range(ix.Count - 1):
        sl = comp_range(gz, ix, k, 1)
        got, buf, rec = pp.Core.ExtractDeflateIndex(sl, ix, k, device=device, with_records=True)
        assert got == meta["chunks"][k]["out_len"]
        assert sha(buf[:got]) == meta["chunks"][k]["sha256"]
        assert len(rec) == meta["chunks"][k]["records"]


@pytest.mark.parametrize("name", CORRUPT)
def test_corrupt_streams(name, device):
    """Corrupted compressed bytes: the same DATA_ERROR as zlib, or the same garbage bytes."""
    meta, gz = load_case(name)
    with open(os.path.join(GOLDEN, "corrupt_clean.gz"), "rb") as f:
        ix = pp.Core.BuildDeflateIndex(f.read(), meta["chunksize"])
    k = meta["chunk"]
    sh = pp.Shard(ix, comp_range(gz, ix, k, 1), k, 1, device=device)
    if meta["oracle_status"] != 0:
        with pytest.raises(pp.PpgError) as e:
            sh.run()
        assert e.value.code == meta["oracle_status"]
    else:
        sh.run()
        b = sh.chunk_bytes(0)
        assert len(b) == meta["out_len"] and sha(b) == meta["out_sha256"]


def test_batched_output_matches_single_batch(device):
    """out_capacity forces several batches through one reused output buffer."""
    meta, gz = load_case("memlevel1_c10")
    ix = pp.Core.BuildDeflateIndex(gz, meta["chunksize"])
    n = ix.Count - 1
    one = pp.Shard(ix, comp_range(gz, ix, 0, n), 0, n, device=device).run().results()
    sh = pp.Shard(ix, comp_range(gz, ix, 0, n), 0, n, device=device, out_capacity=8192)
    assert sh.batches > 4
    many = sh.run().results()
    for key in ("records", "produced", "status"):
        assert (one[key] == many[key]).all(), key
    assert sh.total_records == meta["total_records"]


def test_batched_fastq_fields_match_oracle(tmp_path, device):
    """BatchedFASTQ (DecompressAll) record fields == the oracle's Parsing.Parse, chunk order."""
    meta, gz = load_case("l6_c20")
    p = tmp_path / "x.fastq.gz"
    p.write_bytes(gz)
    ix = pp.Core.BuildDeflateIndex(str(p), meta["chunksize"])
    pp.IndexIO.Serialize(ix, str(tmp_path / "x.gzi"))
    bf = pp.BatchedFASTQ(str(tmp_path / "x.gzi"), str(p), False, device=device)
    assert bf.Count() == meta["total_records"]
    recs = list(bf)
    oi = O.build_index(gz, meta["chunksize"])
    exp = []
    for k in range(oi.count - 1):
        off = oi.point(k)[4]
        ch = O.extract(gz, oi, k)
        raw = off + ch
        exp += pp.records_from_descriptors(raw, O.parse(off, ch))
    assert len(recs) == len(exp)
    for a, b in zip(recs, exp):
        assert (a.identifier, a.sequence, a.other, a.quality) == (b.identifier, b.sequence, b.other, b.quality)


def test_larger_file_vs_oracle_and_trailer(device):
    """200k records (~75 MB text), chunk 10000: every chunk vs the oracle, and the CRC-32 of
    the GPU output against the gzip trailer (a size-independent whole-stream check)."""
    import ctypes as C
    S = pp.synth()
    nrec = 200_000
    sz = S.ppg_synth_fastq_size(0, nrec, 150)
    txt = np.zeros(sz, np.uint8)
    S.ppg_synth_fastq(99, 0, nrec, 150, C.c_void_p(txt.ctypes.data), sz, 8)
    gzb = np.zeros(sz, np.uint8)
    L = S.ppg_synth_gzip(C.c_void_p(txt.ctypes.data), sz, 6, 4 << 20, 8, C.c_void_p(gzb.ctypes.data), gzb.size)
    gz = gzb[:L].tobytes()
    ix = pp.Core.BuildDeflateIndex(gz, 10000)
    n = ix.Count - 1
    sh = pp.Shard(ix, comp_range(gz, ix, 0, n), 0, n, device=device).run()
    oi = O.build_index(gz, 10000)
    crc = 0
    tot = 0
    for k in range(n):
        b = sh.chunk_bytes(k)
        exp = O.extract(gz, oi, k)
        assert b.tobytes() == exp, k
        rec = sh.chunk_records(k)
        assert np.array_equal(rec, O.parse(oi.point(k)[4], exp)), k
        crc = zlib.crc32(b.tobytes(), crc)
        tot += len(rec)
    assert crc == int.from_bytes(gz[-8:-4], "little")
    assert tot == sh.total_records == nrec   # zlib -6 never places a Point at a record start here


@pytest.mark.parametrize("level,strategy,wbits,mem", [(1, zlib.Z_DEFAULT_STRATEGY, 15, 8),
                                                       (9, zlib.Z_DEFAULT_STRATEGY, 15, 9),
                                                       (4, zlib.Z_FILTERED, 15, 8),
                                                       (6, zlib.Z_RLE, 15, 8),
                                                       (6, zlib.Z_DEFAULT_STRATEGY, 9, 1),
                                                       (3, zlib.Z_FIXED, 12, 4)])
def test_encoder_variants_vs_oracle(level, strategy, wbits, mem, device):
    """One member from each of several zlib encoder settings (level, strategy, window bits --
    shorter windows mean shorter match distances --, memLevel: block sizes), 20k records, chunk
    1,000: DecompressAll (every chunk) and the lone-chunk Decompress path (its inner block starts
    found on the GPU, pieces written out from their symbols) against the oracle, bytes and records,
    plus the CRC-32 of the whole output against the gzip trailer."""
    import ctypes as C
    S = pp.synth()
    nrec = 20_000
    sz = S.ppg_synth_fastq_size(0, nrec, 150)
    txt = np.zeros(sz, np.uint8)
    S.ppg_synth_fastq(level * 7 + wbits, 0, nrec, 150, C.c_void_p(txt.ctypes.data), sz, 8)
    co = zlib.compressobj(level, zlib.DEFLATED, 16 + wbits, mem, strategy)
    gz = co.compress(txt.tobytes()) + co.flush()
    ix = pp.Core.BuildDeflateIndex(gz, 1000)
    oi = O.build_index(gz, 1000)
    n = ix.Count - 1
    assert n == oi.count - 1 and n >= 5
    sh = pp.Shard(ix, comp_range(gz, ix, 0, n), 0, n, device=device).run()
    crc = 0
    for k in range(n):
        exp = O.extract(gz, oi, k)
        rexp = O.parse(oi.point(k)[4], exp)
        b = sh.chunk_bytes(k)
        assert b.tobytes() == exp, k
        assert np.array_equal(sh.chunk_records(k), rexp), k
        crc = zlib.crc32(b.tobytes(), crc)
        if k % 4 == 1:
            got, buf, rec = pp.Core.ExtractDeflateIndex(comp_range(gz, ix, k, 1), ix, k, device=device,
                                                        with_records=True)
            assert buf[:got].tobytes() == exp and np.array_equal(rec, rexp), k
    assert crc == int.from_bytes(gz[-8:-4], "little")


@pytest.mark.parametrize("name,piece", [("l6_c20", 1), ("memlevel1_c10", 20000), ("stored_c50", 1),
                                        ("pigz_c100", 1 << 30), ("huffonly_c20", 50000)])
def test_file_ingest_matches_golden(name, piece, tmp_path, device):
    """Host ingest (ppg_file_decompress_all, the LazyFileReader path): pieces as small as one
    chunk stream through pinned buffers + a copy stream; per-chunk record counts == fixtures."""
    meta, gz = load_case(name)
    p = tmp_path / "f.gz"
    p.write_bytes(gz)
    ix = pp.Core.BuildDeflateIndex(gz, meta["chunksize"])
    rec, tot, sec = pp.decompress_file(ix, str(p), piece_bytes=piece, threads=3, device=device)
    assert [int(x) for x in rec] == [c["records"] for c in meta["chunks"]]
    assert tot == meta["total_records"] and sec > 0
    # a sub-range of the chunks
    if ix.Count > 4:
        rec2, tot2, _ = pp.decompress_file(ix, str(p), first=1, n=ix.Count - 3, piece_bytes=piece, device=device)
        assert [int(x) for x in rec2] == [c["records"] for c in meta["chunks"][1:ix.Count - 2]]
    # the kept buffers freed (ppg_file_release, twice: a no-op the second time), then allocated again
    device.release_file_buffers()
    device.release_file_buffers()
    rec3, tot3, _ = pp.decompress_file(ix, str(p), piece_bytes=piece, threads=2, device=device)
    assert [int(x) for x in rec3] == [c["records"] for c in meta["chunks"]] and tot3 == tot


def test_file_ingest_errors(tmp_path, device):
    meta, gz = load_case("l6_c20")
    ix = pp.Core.BuildDeflateIndex(gz, meta["chunksize"])
    with pytest.raises(pp.PpgError) as e:
        pp.decompress_file(ix, str(tmp_path / "missing.gz"), device=device)
    assert e.value.code == -51   # PPG_IO_ERROR
    # a truncated file: the read of the last piece comes up short
    p = tmp_path / "t.gz"
    p.write_bytes(gz[: len(gz) // 2])
    with pytest.raises(pp.PpgError) as e:
        pp.decompress_file(ix, str(p), piece_bytes=1, device=device)
    assert e.value.code == -51


def test_file_ingest_large_vs_oracle(tmp_path, device):
    """200k records through 4 MB pieces: counts == the oracle's threaded DecompressAll."""
    import ctypes as C
    S = pp.synth()
    nrec = 200_000
    sz = S.ppg_synth_fastq_size(0, nrec, 150)
    txt = np.zeros(sz, np.uint8)
    S.ppg_synth_fastq(7, 0, nrec, 150, C.c_void_p(txt.ctypes.data), sz, 8)
    gzb = np.zeros(sz, np.uint8)
    L = S.ppg_synth_gzip(C.c_void_p(txt.ctypes.data), sz, 6, 4 << 20, 8, C.c_void_p(gzb.ctypes.data), gzb.size)
    gz = gzb[:L].tobytes()
    p = tmp_path / "big.gz"
    p.write_bytes(gz)
    ix = pp.Core.BuildDeflateIndex(str(p), 10000)
    rec, tot, _ = pp.decompress_file(ix, str(p), piece_bytes=4 << 20, threads=4, device=device)
    oi = O.build_index(gz, 10000)
    exp_tot, _ = O.decompress_all(gz, oi, threads=8)
    assert tot == exp_tot == nrec
    assert pp.BatchedFASTQ(ix, str(p), True, device=device).Count() == nrec


@pytest.mark.parametrize("nl_bytes", ["1099511627776", "1"])
def test_census_capacity_extremes(nl_bytes, device, monkeypatch):
    """The newline census fused into the inflate flush stores at most nl_cap positions per chunk;
    chunks past it take the body-scan fallback (ppg_parse_emit).  Capacity 0 (every chunk with
    newlines overflows) and capacity >= every byte must both give the golden record tables."""
    monkeypatch.setenv("PPG_NL_BYTES", nl_bytes)
    for name in CASES:
        meta, gz = load_case(name)
        ix = pp.Core.BuildDeflateIndex(gz, meta["chunksize"])
        n = ix.Count - 1
        sh = pp.Shard(ix, comp_range(gz, ix, 0, n), 0, n, device=device).run()
        for k, c in enumerate(meta["chunks"]):
            rec = sh.chunk_records(k)
            assert len(rec) == c["records"], (name, k)
            assert sha(np.ascontiguousarray(rec, "<u4").tobytes()) == c["rec_sha256"], (name, k)
        assert sh.total_records == meta["total_records"]


def dense_side_points(gz, ix, chunksize=9):
    """Side points for ppg_shard_set_split from the oracle's CreateIndex at a tiny chunk size (a
    Point at almost every block end, with its window): those strictly inside ix's chunks."""
    dx = O.build_index(gz, chunksize)
    outs = np.array([ix.point_fields(k)[0] for k in range(ix.Count)], np.int64)
    bits, out, wins = [], [], []
    for o, n, b, w, _ in dx.points():
        c = int(np.searchsorted(outs, o, side="right")) - 1
        if 0 <= c < ix.Count - 1 and outs[c] < o < outs[c + 1]:
            bits.append(8 * n - b)
            out.append(o)
            wins.append(np.frombuffer(w, np.uint8))
    win = np.concatenate(wins) if wins else np.zeros(0, np.uint8)
    return np.array(bits, np.int64), np.array(out, np.int64), win


def assert_same_run(a, b, n):
    ra, rb = a.results(), b.results()
    for key in ra:
        assert (ra[key] == rb[key]).all(), key
    assert a.total_records == b.total_records
    assert (a.record_base() == b.record_base()).all()
    for k in range(n):
        assert sha(a.chunk_bytes(k)) == sha(b.chunk_bytes(k)), k
        assert (a.chunk_records(k) == b.chunk_records(k)).all(), k


@pytest.mark.parametrize("name", CASES)
def test_split_chunks_match_golden(name, device):
    """Chunks decoded as several waves (side points at inner block starts, ppg_shard_set_split)
    give exactly the golden bytes and record tables, and the same results as one wave per chunk."""
    meta, gz = load_case(name)
    ix = pp.Core.BuildDeflateIndex(gz, meta["chunksize"])
    n = ix.Count - 1
    bits, outs, win = dense_side_points(gz, ix)
    one = pp.Shard(ix, comp_range(gz, ix, 0, n), 0, n, device=device).run()
    sh = pp.Shard(ix, comp_range(gz, ix, 0, n), 0, n, device=device).set_split(bits, outs, win).run()
    for k, c in enumerate(meta["chunks"]):
        assert sha(sh.chunk_bytes(k)) == c["sha256"], (name, k)
        assert sha(np.ascontiguousarray(sh.chunk_records(k), "<u4").tobytes()) == c["rec_sha256"], (name, k)
    assert_same_run(one, sh, n)
    # and back to one wave per chunk
    sh.set_split([], [], np.zeros(0, np.uint8)).run()
    assert_same_run(one, sh, n)


@pytest.mark.parametrize("per", [2, 3, 8])
def test_split_tiled_member(per, device):
    """bench.py's --split path: TiledFile.side_points over a small tiled member."""
    from parallelparsing_amd.tiled import TiledFile
    tf = TiledFile(3000, 6, 1000, threads=4)
    f = tf.file_bytes()
    ix = tf.index()
    n = tf.npoints - 1
    one = pp.Shard(ix, comp_range(f, ix, 0, n), 0, n, device=device).run()
    bits, outs, win = tf.side_points(per_chunk=per)
    assert bits.size > n // 2
    sh = pp.Shard(ix, comp_range(f, ix, 0, n), 0, n, device=device).set_split(bits, outs, win).run()
    assert_same_run(one, sh, n)
    assert sh.total_records == tf.expected_records()
    text = tf.text.tobytes() * tf.repeats
    for k in range(n):
        assert sh.chunk_bytes(k).tobytes() == text[tf.p_output[k]:tf.p_output[k + 1]], k


@pytest.mark.parametrize("nl_bytes", ["1099511627776", "1"])
def test_split_census_capacity_extremes(nl_bytes, device, monkeypatch):
    monkeypatch.setenv("PPG_NL_BYTES", nl_bytes)
    for name in ["l6_c200", "crlf_c100", "fixed_c100"]:
        meta, gz = load_case(name)
        ix = pp.Core.BuildDeflateIndex(gz, meta["chunksize"])
        n = ix.Count - 1
        bits, outs, win = dense_side_points(gz, ix)
        sh = pp.Shard(ix, comp_range(gz, ix, 0, n), 0, n, device=device).set_split(bits, outs, win).run()
        for k, c in enumerate(meta["chunks"]):
            assert sha(np.ascontiguousarray(sh.chunk_records(k), "<u4").tobytes()) == c["rec_sha256"], (name, k)
        assert sh.total_records == meta["total_records"]


@pytest.mark.parametrize("name", CASES)
def test_split_whole_member_chunk(name, device):
    """One chunk spanning the member (CreateIndex at a chunk size no file reaches), split at every
    inner block end: the bytes are the member's text, the records the oracle's DecompressAll, and
    both equal the one-wave run -- covers every golden case (fixed, stored, CRLF, NUL, malformed)."""
    meta, gz = load_case(name)
    big = 1 << 30
    ix = pp.Core.BuildDeflateIndex(gz, big)
    n = ix.Count - 1
    bits, outs, win = dense_side_points(gz, ix)
    one = pp.Shard(ix, comp_range(gz, ix, 0, n), 0, n, device=device).run()
    sh = pp.Shard(ix, comp_range(gz, ix, 0, n), 0, n, device=device).set_split(bits, outs, win).run()
    assert_same_run(one, sh, n)
    text = zlib.decompress(gz, 47)
    assert b"".join(sh.chunk_bytes(k).tobytes() for k in range(n)) == text
    tot, _ = O.decompress_all(gz, O.build_index(gz, big), threads=4)
    assert sh.total_records == tot


def test_split_rejects_bad_side_points(device):
    meta, gz = load_case("memlevel1_c10")
    ix = pp.Core.BuildDeflateIndex(gz, meta["chunksize"])
    n = ix.Count - 1
    bits, outs, win = dense_side_points(gz, ix)
    assert bits.size >= 2
    sh = pp.Shard(ix, comp_range(gz, ix, 0, n), 0, n, device=device)
    with pytest.raises(RuntimeError):   # not sorted
        sh.set_split(bits[::-1].copy(), outs[::-1].copy(), win)
    with pytest.raises(RuntimeError):   # on a chunk Point, not strictly inside a chunk
        o0 = ix.point_fields(1)[0]
        sh.set_split(bits[:1], np.array([o0], np.int64), win[:32768])
    # a side point one byte late: the piece before it cannot end there
    sh.set_split(bits[:1], outs[:1] + 1, win[:32768])
    with pytest.raises(RuntimeError):
        sh.run()
    r = sh.results()
    assert (r["status"] != 0).sum() == 1


@pytest.mark.parametrize("name", ["memlevel1_c10", "l6_c200", "crlf_c100", "fixed_c100", "malformed_c40"])
def test_split_multi_batch_shards(name, device):
    """a shard whose output does not fit one batch can still be split; each batch
    launches its chunks' pieces and the results equal the unsplit, one-batch run."""
    meta, gz = load_case(name)
    ix = pp.Core.BuildDeflateIndex(gz, meta["chunksize"])
    n = ix.Count - 1
    bits, outs, win = dense_side_points(gz, ix)
    one = pp.Shard(ix, comp_range(gz, ix, 0, n), 0, n, device=device).run()
    cap = int(ix.point_fields(n)[0] - ix.point_fields(0)[0]) // 5 + 1
    sh = pp.Shard(ix, comp_range(gz, ix, 0, n), 0, n, device=device, out_capacity=cap)
    assert sh.batches >= min(n, 3)
    sh.set_split(bits, outs, win).run()
    ra, rb = one.results(), sh.results()
    for key in ra:
        assert (ra[key] == rb[key]).all(), key
    assert sh.total_records == meta["total_records"]
    assert (sh.record_base() == one.record_base()).all()

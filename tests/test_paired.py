"""Paired-end record-aligned pair chunks through the C ABI's pair check
(ppg_pairs_*, csrc/ppg_pairs.hip): two synthetic mate files against their generated text, on one
rank and on 2 / 3 ranks of the one GPU over the library's host transport (the key exchange's
collective is covered on the CPU in tests/test_dist.py)."""
import ctypes as C
import os
import socket
import uuid

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import parallelparsing_amd as pp
from parallelparsing_amd import paired


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _mate_file(mate, seed, nrec, tmp_path):
    S = pp.synth()
    sz = S.ppg_synth_fastq_size_mate(0, nrec, 150, mate)
    txt = np.zeros(sz, np.uint8)
    assert S.ppg_synth_fastq_mate(seed, mate, 0, nrec, 150, C.c_void_p(txt.ctypes.data), sz, 8) == sz
    gzb = np.zeros(sz, np.uint8)
    L = S.ppg_synth_gzip(C.c_void_p(txt.ctypes.data), sz, 6, 1 << 20, 8, C.c_void_p(gzb.ctypes.data), gzb.size)
    p = tmp_path / f"r{mate}.fastq.gz"
    p.write_bytes(gzb[:L].tobytes())
    return str(p), txt.tobytes()


def test_mate_files_share_spots():
    """Generator pair mode: R1/R2 record i have the same SRR id and spot, mates 1 and 2."""
    import tempfile, pathlib
    with tempfile.TemporaryDirectory() as d:
        _, t1 = _mate_file(1, 0, 50, pathlib.Path(d))
        _, t2 = _mate_file(2, 1, 50, pathlib.Path(d))
    h1 = [l for l in t1.split(b"\n") if l.startswith(b"@")]
    h2 = [l for l in t2.split(b"\n") if l.startswith(b"@")]
    assert len(h1) == len(h2) == 50
    for i, (a, b) in enumerate(zip(h1, h2)):
        ia, ib = a.split(b" ")[0].split(b"."), b.split(b" ")[0].split(b".")
        assert ia[0] == ib[0] and ia[1] == ib[1] == str(i + 1).encode() and (ia[2], ib[2]) == (b"1", b"2")


@pytest.mark.gpu
def test_paired_fastq_pairs(tmp_path):
    nrec = 30_000
    p1, t1 = _mate_file(1, 0, nrec, tmp_path)
    p2, t2 = _mate_file(2, 1, nrec, tmp_path)
    # different chunk sizes: the files' chunk boundaries never line up
    ix1 = pp.Core.BuildDeflateIndex(p1, 700)
    ix2 = pp.Core.BuildDeflateIndex(p2, 1100)
    pf = paired.PairedFASTQ(ix1, p1, ix2, p2, pair_chunk=4000)
    assert pf.Count() == nrec and pf.chunks == 8
    recs1 = t1.split(b"\n")
    # random access (only chunk j copied out; ascending calls walk the windows once,
    # a chunk behind the current window restarts the emission), then the iteration agrees
    pf.window_bytes = 3 << 20   # several windows
    for j in (0, 3, 7, 5, 5, 1):
        a, b = pf.pair_chunk(j)
        assert len(a) == len(b) == min(4000, nrec - 4000 * j)
        for i in (0, len(a) // 2, len(a) - 1):
            g = 4000 * j + i
            assert a[i].identifier == recs1[4 * g][1:]
            assert a[i].identifier.split(b".")[:2] == b[i].identifier.split(b".")[:2]
    it = {j: ([r.identifier for r in a], [r.sequence for r in b]) for j, a, b in pf.pair_chunks() if j in (2, 6)}
    for j in (2, 6):
        a2, b2 = pf.pair_chunk(j)
        assert ([r.identifier for r in a2], [r.sequence for r in b2]) == it[j]


@pytest.mark.gpu
def test_paired_fastq_rejects_misaligned(tmp_path):
    p1, _ = _mate_file(1, 0, 5000, tmp_path)
    S = pp.synth()
    # R2 starting one spot later: every pair mismatches
    sz = S.ppg_synth_fastq_size_mate(1, 5000, 150, 2)
    txt = np.zeros(sz, np.uint8)
    S.ppg_synth_fastq_mate(1, 2, 1, 5000, 150, C.c_void_p(txt.ctypes.data), sz, 8)
    gzb = np.zeros(sz, np.uint8)
    L = S.ppg_synth_gzip(C.c_void_p(txt.ctypes.data), sz, 6, 1 << 20, 8, C.c_void_p(gzb.ctypes.data), gzb.size)
    p2 = tmp_path / "bad.gz"
    p2.write_bytes(gzb[:L].tobytes())
    ix1 = pp.Core.BuildDeflateIndex(p1, 1000)
    ix2 = pp.Core.BuildDeflateIndex(str(p2), 1000)
    with pytest.raises(ValueError):
        paired.PairedFASTQ(ix1, p1, ix2, str(p2))


@pytest.mark.gpu
def test_record_keys_drop_q1_duplicates(tmp_path):
    """Deflate blocks that end on record boundaries put Points on record starts:
    those chunk-first records are marked DUP and the deduplicated keys are exactly spots 1..n."""
    S = pp.synth()
    nrec = 4000
    sz = S.ppg_synth_fastq_size_mate(0, nrec, 150, 1)
    txt = np.zeros(sz, np.uint8)
    S.ppg_synth_fastq_mate(0, 1, 0, nrec, 150, C.c_void_p(txt.ctypes.data), sz, 8)
    import zlib
    lines = txt.tobytes().split(b"\n")
    co = zlib.compressobj(6, zlib.DEFLATED, 31)
    gz = b""
    for g in range(0, nrec, 10):   # a block ends after every 10 records
        gz += co.compress(b"\n".join(lines[4 * g:4 * (g + 10)]) + b"\n") + co.flush(zlib.Z_FULL_FLUSH)
    gz += co.flush()
    ix = pp.Core.BuildDeflateIndex(gz, 20)
    n = ix.Count - 1
    _, i0, _, _ = ix.point_fields(0)
    _, i1, _, _ = ix.point_fields(n)
    sh = pp.Shard(ix, np.frombuffer(gz[i0 - 1:i1], np.uint8), 0, n).run()
    keys = paired.shard_keys(sh)
    kept = keys[keys != paired.DUP]
    assert sh.total_records > nrec                       # the reference's duplicates are there
    assert int((keys == paired.DUP).sum()) == sh.total_records - nrec
    assert torch.equal(kept.cpu(), torch.arange(1, nrec + 1))
    # the library's pair check drops the same records: the file pairs with itself, nrec pairs
    res = paired.Pairs().check(sh, sh)
    assert res["pairs"] == nrec and res["mismatches"] == 0 and res["duplicates"] == (sh.total_records - nrec,) * 2
    # the same keys with every chunk split at its inner block start (bench --paired's auto split)
    from test_gpu_parity import dense_side_points
    bits, outs, win = dense_side_points(gz, ix)
    assert bits.size >= n // 2
    s2 = pp.Shard(ix, np.frombuffer(gz[i0 - 1:i1], np.uint8), 0, n).set_split(bits, outs, win).run()
    assert torch.equal(paired.shard_keys(s2), keys)


def _ref_keys(raw, desc, olen):
    """ppg_record_keys' byte loop (ppg_parse.hip), restated for the test: the digits between the
    Identifier's first two '.', at most 18 of them, within its first 96 bytes; -2 for a chunk's
    first record lying wholly inside offset_k (parsed twice)."""
    out = []
    for j, (n1, n2, n3, n4) in enumerate(desc.tolist()):
        start = 0 if j == 0 else desc[j - 1][3] + 1
        if j == 0 and n4 < olen:
            out.append(-2)
            continue
        end = min(n1, start + 96)
        i, key = start + 1, -1
        while i < end and raw[i] != ord("."):
            i += 1
        if i < end:
            i += 1
            v = nd = c = 0
            while i < end:
                c = raw[i]
                if not (48 <= c <= 57 and nd < 18):
                    break
                v, nd, i = v * 10 + c - 48, nd + 1, i + 1
            if nd > 0 and i < end and c == ord("."):
                key = v
        out.append(key)
    return out


HEADERS = [
    b"@SRR1.{n}.1 {n} length=8",                          # the ordinary shape
    b"@" + b"A" * 60 + b".{n}.2 tail",                    # first '.' past the 48-byte window
    b"@X" + b"B" * 100 + b".{n}.1",                       # past the 96-byte bound: -1
    b"@SRR.123456789012345678.1",                         # 18 digits
    b"@SRR.1234567890123456789.1",                        # 19 digits: -1
    b"@SRR.{n} no second dot",                            # -1
    b"@SRR..1",                                           # empty spot: -1
    b"@SRR.{n}",                                          # the line ends inside the digits: -1
    b"@" + b"C" * 31 + b".{n}.",                          # identifier of 48 bytes-ish, decided at the end
    b"@" + b"D" * 38 + b".12345678.",                     # exactly 48 bytes after the '@'
    b"@.{n}.x",                                           # the first byte is the '.'
    b"@noDots",
]


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [7, 23])
def test_record_keys_identifier_edge_cases(chunk, device):
    """ppg_record_keys' 48-byte register window and its byte-loop fallback against the
    byte loop restated in Python, on identifiers that reach every branch, with headers straddling
    Points (small chunks, Huffman-only: Points land on record starts too, giving Q1 duplicates)."""
    import zlib
    recs = []
    for i in range(600):
        h = HEADERS[i % len(HEADERS)].replace(b"{n}", str(1000 + i).encode())
        recs.append(h + b"\nACGTACGT\n+\n????????\n")
    text = b"".join(recs)
    c = zlib.compressobj(6, zlib.DEFLATED, 31, 8, zlib.Z_HUFFMAN_ONLY)
    gz = c.compress(text) + c.flush()
    ix = pp.Core.BuildDeflateIndex(gz, chunk)
    n = ix.Count - 1
    _, i0, _, _ = ix.point_fields(0)
    _, i1, _, _ = ix.point_fields(n)
    sh = pp.Shard(ix, np.frombuffer(gz[i0 - 1:i1], np.uint8), 0, n, device=device).run()
    got = paired.shard_keys(sh).cpu().numpy().tolist()
    exp = []
    for k in range(n):
        off = ix[k].offset
        raw = off + sh.chunk_bytes(k).tobytes()
        exp += _ref_keys(raw, sh.chunk_records(k), len(off))
    assert got == exp
    assert exp.count(-1) > 100 and 123456789012345678 in exp   # Q1 (-2): test_record_keys_drop_q1_duplicates
    assert {1000 + i for i in range(0, 600, len(HEADERS))} <= set(exp)   # ordinary keys decoded


def _text_gz(txt):
    S = pp.synth()
    a = np.frombuffer(txt, np.uint8)
    gzb = np.zeros(a.size, np.uint8)
    L = S.ppg_synth_gzip(C.c_void_p(a.ctypes.data), a.size, 6, 1 << 20, 8, C.c_void_p(gzb.ctypes.data), gzb.size)
    return gzb[:L].tobytes()


def _pair_files(tmp_path, nrec, case):
    """R1 / R2 mate files; case 'swap' exchanges R2's records 5000 and 5001, 'short' drops R2's last."""
    p1, _ = _mate_file(1, 0, nrec, tmp_path)
    _, t2 = _mate_file(2, 1, nrec, tmp_path)
    lines = t2.split(b"\n")[:-1]
    recs = [b"\n".join(lines[4 * i:4 * i + 4]) + b"\n" for i in range(nrec)]
    if case == "swap":
        recs[5000], recs[5001] = recs[5001], recs[5000]
    if case == "short":
        recs = recs[:-1]
    p2 = tmp_path / f"r2_{case}.fastq.gz"
    p2.write_bytes(_text_gz(b"".join(recs)))
    return p1, str(p2)


EXPECT = {"ok": (30_000, 0, -1), "swap": (30_000, 2, 5000), "short": (29_999, 1, 29_999)}


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["ok", "swap", "short"])
def test_pairs_check_one_rank(case, tmp_path, device):
    p1, p2 = _pair_files(tmp_path, 30_000, case)
    shards = []
    for p, chunk in ((p1, 700), (p2, 1100)):
        ix = pp.Core.BuildDeflateIndex(p, chunk)
        n = ix.Count - 1
        shards.append(pp.Shard(ix, paired._read_range(p, ix), 0, n, device=device).run())
    pr = paired.Pairs()
    res = pr.check(shards[0], shards[1])
    assert (res["pairs"], res["mismatches"], res["first_bad"]) == EXPECT[case], res
    if case == "swap":
        assert res["first_keys"] == (5001, 5002)
    if case == "ok":
        assert (pr.records(0, 0, 30_000) == np.arange(30_000)).all()   # no Q1 duplicates in these files


def _pair_rank(rank, world, name, p1, p2, q):
    try:
        import parallelparsing_amd as pp2
        from parallelparsing_amd import paired as P
        dev = pp2.Device(0)
        comm = pp2.Comm.host(world, rank, name)
        shards = []
        for p, chunk in ((p1, 700), (p2, 1100)):   # the files' rank ranges never line up
            ix = pp2.Core.BuildDeflateIndex(p, chunk)
            b = pp2.partition(ix, world)
            a, e = int(b[rank]), int(b[rank + 1])
            _, i0, _, _ = ix.point_fields(a)
            _, i1, _, _ = ix.point_fields(e)
            with open(p, "rb") as f:
                f.seek(i0 - 1)
                comp = np.frombuffer(f.read(i1 - i0 + 1), np.uint8)
            shards.append(pp2.Shard(ix, comp, a, e - a, device=dev).run())
        pr = P.Pairs()
        res = pr.check(shards[0], shards[1], comm)
        res2 = pr.check(shards[0], shards[1], comm)      # reused scratch, same answer
        comm.close()
        q.put((rank, res, res2 == res))
    except Exception as e:   # noqa: BLE001 - reported to the parent
        q.put((rank, repr(e), False))


@pytest.mark.gpu
@pytest.mark.parametrize("world,case", [(2, "ok"), (2, "swap"), (3, "short"), (3, "ok")])
def test_pairs_check_multi_rank_on_one_gpu(world, case, tmp_path, device):
    """ppg_pairs_check on `world` processes of the box's one GPU over the host transport: each rank
    decodes its own chunk ranges of R1 and R2, every key moves to its pair's owner
    (ppg_comm_alltoallv), and every rank gets the single-rank result."""
    import torch.multiprocessing as mp
    p1, p2 = _pair_files(tmp_path, 30_000, case)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = f"/ppg_test_{uuid.uuid4().hex[:12]}"
    procs = [ctx.Process(target=_pair_rank, args=(r, world, name, p1, p2, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=180) for _ in procs]
    for pr in procs:
        pr.join(60)
    for r in res:
        assert isinstance(r[1], dict), r
        assert (r[1]["pairs"], r[1]["mismatches"], r[1]["first_bad"]) == EXPECT[case], r
        assert r[2]

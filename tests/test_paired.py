"""Paired-end record-aligned pair chunks.  CPU: the distributed pair check over
gloo (world 2); GPU: pairing two synthetic mate files against their generated text."""
import ctypes as C
import os
import socket

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


def _worker(rank, world, port, case, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 1000
        keys = torch.arange(1, n + 1, dtype=torch.int64)
        # the two files split differently over the ranks (their chunk boundaries differ)
        c1, c2 = [0, 337, n], [0, 612, n]
        k1 = keys[c1[rank]:c1[rank + 1]].clone()
        k2 = keys[c2[rank]:c2[rank + 1]].clone()
        if case == "swap" and rank == 1:
            k2[5], k2[6] = k2[6].item(), k2[5].item()
        if case == "short" and rank == 1:
            k2 = k2[:-1]
        q.put((rank, paired.distributed_pair_check(k1, k2)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case,expect", [("ok", (1000, 0)), ("swap", (1000, 2)), ("short", (999, 1))])
def test_distributed_pair_check_gloo(case, expect):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, case, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    assert res[0] == res[1] == expect


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
    for j in (0, 3, 7):
        a, b = pf.pair_chunk(j)
        assert len(a) == len(b) == min(4000, nrec - 4000 * j)
        for i in (0, len(a) // 2, len(a) - 1):
            g = 4000 * j + i
            assert a[i].identifier == recs1[4 * g][1:]
            assert a[i].identifier.split(b".")[:2] == b[i].identifier.split(b".")[:2]


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
    kept, _ = paired.dedup(keys)
    assert sh.total_records > nrec                       # the reference's duplicates are there
    assert int((keys == paired.DUP).sum()) == sh.total_records - nrec
    assert torch.equal(kept.cpu(), torch.arange(1, nrec + 1))
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

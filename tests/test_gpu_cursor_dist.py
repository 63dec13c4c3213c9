"""The C ABI's streamed records (ppg_cursor) and multi-GPU DecompressAll (ppg_comm,
ppg_shard_gather_counts, ppg_dist_decompress_all) -- VERDICT r01 item 3.

BatchedFASTQ.cs:29-101 hands records out of a bounded cache; the cursor must give the golden
record tables through many small batches.  The multi-rank gather runs with two processes on the
one GPU of the box through the host shared-memory transport (RCCL refuses two ranks on one GPU),
and with RCCL itself at world size 1."""
import hashlib
import os
import uuid

import numpy as np
import pytest

import parallelparsing_amd as pp
from conftest import CASES, load_case
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


@pytest.mark.parametrize("name", CASES)
def test_cursor_batches_match_golden(name, tmp_path, device):
    meta, gz = load_case(name)
    p = tmp_path / "f.gz"
    p.write_bytes(gz)
    ix = pp.Core.BuildDeflateIndex(gz, meta["chunksize"])
    n = ix.Count - 1
    text_total = int(ix.point_fields(n)[0])
    cur = pp.Cursor(ix, str(p), batch_bytes=max(1, text_total // 6), threads=2, device=device)
    if n >= 6:
        assert cur.batches > 4
    k, base = 0, 0
    for b in cur:
        assert b.first_chunk == k and b.record_base == base
        for j in range(b.nchunks):
            c = meta["chunks"][k]
            off = ix[k].offset
            raw = b.raw(j)
            assert raw[:len(off)].tobytes() == off
            assert sha(raw[len(off):]) == c["sha256"], (name, k)
            assert sha(np.ascontiguousarray(b.records(j), "<u4").tobytes()) == c["rec_sha256"], (name, k)
            k += 1
        base += b.nrecords
    assert k == n and base == meta["total_records"]


@pytest.mark.parametrize("pack,slots", [("0", "2"), ("1", "5"), ("2", "3")])
def test_cursor_transfer_modes_match_golden(pack, slots, tmp_path, device, monkeypatch):
    """Every way a batch can reach the host (PPG_CURSOR_PACK: per-chunk copies, device pack + one
    copy, pack kernel storing into pinned memory) and slot counts give the golden bytes/records."""
    monkeypatch.setenv("PPG_CURSOR_PACK", pack)
    monkeypatch.setenv("PPG_CURSOR_SLOTS", slots)
    meta, gz = load_case("l6_c20")
    p = tmp_path / "f.gz"
    p.write_bytes(gz)
    ix = pp.Core.BuildDeflateIndex(gz, meta["chunksize"])
    n = ix.Count - 1
    cur = pp.Cursor(ix, str(p), batch_bytes=max(1, int(ix.point_fields(n)[0]) // 7), threads=2, device=device)
    assert cur.batches > int(slots)
    k = 0
    for b in cur:
        for j in range(b.nchunks):
            c = meta["chunks"][k]
            raw = b.raw(j)
            assert sha(raw[len(ix[k].offset):]) == c["sha256"], (pack, k)
            assert sha(np.ascontiguousarray(b.records(j), "<u4").tobytes()) == c["rec_sha256"], (pack, k)
            k += 1
    assert k == n


def test_cursor_large_file_records_equal_oracle(tmp_path, device):
    """200k records through ~8 MB batches (>40 of them), every record's fields vs the oracle."""
    import ctypes as C
    S = pp.synth()
    nrec = 200_000
    sz = S.ppg_synth_fastq_size(0, nrec, 150)
    txt = np.zeros(sz, np.uint8)
    S.ppg_synth_fastq(5, 0, nrec, 150, C.c_void_p(txt.ctypes.data), sz, 8)
    gzb = np.zeros(sz, np.uint8)
    L = S.ppg_synth_gzip(C.c_void_p(txt.ctypes.data), sz, 6, 4 << 20, 8, C.c_void_p(gzb.ctypes.data), gzb.size)
    gz = gzb[:L].tobytes()
    p = tmp_path / "big.gz"
    p.write_bytes(gz)
    ix = pp.Core.BuildDeflateIndex(gz, 2000)
    oi = O.build_index(gz, 2000)
    cur = pp.Cursor(ix, str(p), batch_bytes=8 << 20, device=device)
    assert cur.batches > 8
    got = 0
    for b in cur:
        for j in range(b.nchunks):
            k = b.first_chunk + j
            exp = O.extract(gz, oi, k)
            assert b.raw(j)[len(ix[k].offset):].tobytes() == exp, k
            assert np.array_equal(b.records(j), O.parse(oi.point(k)[4], exp)), k
            got += len(b.records(j))
    assert got == nrec
    # BatchedFASTQ iterates through the cursor: whole records, canonical order
    bf = pp.BatchedFASTQ(ix, str(p), device=device)
    bf.batch_bytes = 4 << 20
    recs = list(bf)
    assert len(recs) == nrec
    assert recs[0].identifier == txt[1:txt.tobytes().index(b"\n")].tobytes()


@pytest.mark.parametrize("world", [2, 3])
def test_rank_enumeration_concatenates_to_the_file(world, tmp_path, device):
    """Multi-GPU enumeration (VERDICT r02 missing #5): each rank's BatchedFASTQ yields the records
    of its ppg_partition share; in rank order they are exactly the single-GPU enumeration's."""
    meta, gz = load_case("l6_c200")
    p = tmp_path / "f.gz"
    p.write_bytes(gz)
    ix = pp.Core.BuildDeflateIndex(gz, meta["chunksize"])
    whole = pp.BatchedFASTQ(ix, str(p), device=device)
    whole.batch_bytes = 1 << 16
    exp = [(r.identifier, r.sequence, r.other, r.quality) for r in whole]
    got, ranges = [], []
    for r in range(world):
        bf = pp.BatchedFASTQ(ix, str(p), device=device, rank=r, world=world)
        bf.batch_bytes = 1 << 16
        ranges.append(bf.chunk_range())
        got += [(x.identifier, x.sequence, x.other, x.quality) for x in bf]
    assert all(n > 0 for _, n in ranges) and ranges[0][0] == 0
    assert all(ranges[i][0] + ranges[i][1] == ranges[i + 1][0] for i in range(world - 1))
    assert got == exp and len(got) == meta["total_records"]


def test_rccl_comm_world1(device):
    meta, gz = load_case("l6_c200")
    ix = pp.Core.BuildDeflateIndex(gz, meta["chunksize"])
    n = ix.Count - 1
    _, i0, _, _ = ix.point_fields(0)
    _, i1, _, _ = ix.point_fields(n)
    sh = pp.Shard(ix, np.frombuffer(gz[i0 - 1:i1], np.uint8), 0, n, device=device).run()
    comm = pp.Comm.rccl(device, 1, 0, pp.Comm.unique_id())
    assert comm.rank_size() == (0, 1)
    bounds = pp.partition(ix, 1)
    counts, bases, tot = pp.gather_counts(sh, comm, bounds)
    assert tot == meta["total_records"]
    assert counts.tolist() == [c["records"] for c in meta["chunks"]]
    assert (bases == np.concatenate([[0], np.cumsum(counts)[:-1]])).all()
    assert pp.rccl_version() >= 22600
    comm.close()


def _rank(rank, world, name, path, chunksize, q):
    try:
        import parallelparsing_amd as pp2
        dev = pp2.Device(0)
        ix = pp2.Core.BuildDeflateIndex(path, chunksize)
        comm = pp2.Comm.host(world, rank, name)
        bounds = pp2.partition(ix, world)
        a, b = int(bounds[rank]), int(bounds[rank + 1])
        _, i0, _, _ = ix.point_fields(a)
        _, i1, _, _ = ix.point_fields(b)
        with open(path, "rb") as f:
            f.seek(i0 - 1)
            comp = np.frombuffer(f.read(i1 - i0 + 1), np.uint8)
        sh = pp2.Shard(ix, comp, a, b - a, device=dev).run()
        c1, b1, t1 = pp2.gather_counts(sh, comm, bounds)
        c2, b2, t2 = pp2.dist_decompress_all(ix, path, comm, device=dev)
        # a rank's BatchedFASTQ.Count(): its own share decoded, every rank's counts gathered
        t3 = pp2.BatchedFASTQ(ix, path, device=dev, comm=comm).Count()
        comm.close()
        q.put((rank, c1.tolist(), b1.tolist(), t1, c2.tolist(), b2.tolist(), t2 if t3 == t2 else -1, bounds.tolist()))
    except Exception as e:   # noqa: BLE001 - reported to the parent
        q.put((rank, repr(e)))


@pytest.mark.parametrize("world", [2, 3])
def test_abi_gather_multi_rank_on_one_gpu(world, tmp_path, device):
    """ppg_shard_gather_counts and ppg_dist_decompress_all with `world` processes on the box's one
    GPU (host transport): every rank gets the same canonical counts / bases / total as one rank."""
    import torch.multiprocessing as mp
    meta, gz = load_case("l6_c200")
    p = tmp_path / "f.gz"
    p.write_bytes(gz)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = f"/ppg_test_{uuid.uuid4().hex[:12]}"
    procs = [ctx.Process(target=_rank, args=(r, world, name, str(p), meta["chunksize"], q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=180) for _ in procs]
    for pr in procs:
        pr.join(60)
    exp = [c["records"] for c in meta["chunks"]]
    exp_b = np.concatenate([[0], np.cumsum(exp)[:-1]]).tolist()
    for r in res:
        assert len(r) == 8, r
        _, c1, b1, t1, c2, b2, t2, bounds = r
        assert c1 == exp and c2 == exp and b1 == exp_b and b2 == exp_b
        assert t1 == t2 == meta["total_records"]
        assert bounds[0] == 0 and bounds[-1] == len(exp) and len(bounds) == world + 1


def _rank_bad(rank, world, name, path, chunksize, q):
    try:
        import parallelparsing_amd as pp2
        dev = pp2.Device(0)
        ix = pp2.Core.BuildDeflateIndex(path, chunksize)
        comm = pp2.Comm.host(world, rank, name)
        codes = []
        # rank 1 names a file that does not exist: every rank must get its IO_ERROR, none may hang
        try:
            pp2.dist_decompress_all(ix, path if rank == 0 else path + ".missing", comm, device=dev)
            codes.append(0)
        except pp2.PpgError as e:
            codes.append(e.code)
        # then a shard whose run failed (rank 0: a corrupt compressed range) joins the count gather
        bounds = pp2.partition(ix, world)
        a, b = int(bounds[rank]), int(bounds[rank + 1])
        _, i0, _, _ = ix.point_fields(a)
        _, i1, _, _ = ix.point_fields(b)
        with open(path, "rb") as f:
            f.seek(i0 - 1)
            comp = np.frombuffer(f.read(i1 - i0 + 1), np.uint8).copy()
        if rank == 0:
            comp[len(comp) // 3:] ^= 0x5A
        sh = pp2.Shard(ix, comp, a, b - a, device=dev)
        try:
            sh.run()
        except pp2.PpgError:
            pass
        try:
            pp2.gather_counts(sh, comm, bounds)
            codes.append(0)
        except pp2.PpgError as e:
            codes.append(e.code)
        # and the comm still works for a good round afterwards
        sh2 = pp2.Shard(ix, np.frombuffer(open(path, "rb").read()[i0 - 1:i1], np.uint8), a, b - a, device=dev).run()
        _, _, tot = pp2.gather_counts(sh2, comm, bounds)
        comm.close()
        q.put((rank, codes, tot))
    except Exception as e:   # noqa: BLE001 - reported to the parent
        q.put((rank, repr(e), None))


def test_failing_rank_never_leaves_the_others_waiting(tmp_path, device):
    """a rank whose input is unreadable, or whose DecompressAll failed, still
    joins the count gather; every rank returns the first failing rank's status."""
    import torch.multiprocessing as mp
    from parallelparsing_amd._lib import PPG_IO_ERROR
    meta, gz = load_case("l6_c200")
    p = tmp_path / "f.gz"
    p.write_bytes(gz)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = f"/ppg_test_{uuid.uuid4().hex[:12]}"
    procs = [ctx.Process(target=_rank_bad, args=(r, 2, name, str(p), meta["chunksize"], q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for pr in procs:
        pr.join(60)
    assert all(r[2] == meta["total_records"] for r in res), res
    c0, c1 = res[0][1], res[1][1]
    assert c0 == c1, res
    assert c0[0] == PPG_IO_ERROR
    assert c0[1] < 0     # rank 0's own decode error, returned by both ranks

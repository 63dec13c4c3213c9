"""Multi-rank path on CPU: chunk partition + the padded all-gather of per-chunk record counts,
run with torch.distributed gloo at world_size 2 (the GPU run uses nccl = RCCL)."""
import os
import socket

import numpy as np
import pytest

import parallelparsing_amd as pp
from conftest import load_case
from parallelparsing_amd.dist import partition_chunks


def test_partition_balanced_contiguous():
    inputs = np.cumsum(np.r_[10, np.random.default_rng(0).integers(900, 1100, 999)])
    for world in (1, 2, 3, 8):
        ranges = partition_chunks(inputs, world)
        assert ranges[0][0] == 0 and ranges[-1][1] == len(inputs) - 1
        assert all(ranges[i][1] == ranges[i + 1][0] for i in range(world - 1))
        cost = [inputs[b] - inputs[a] for a, b in ranges]
        assert max(cost) - min(cost) <= 2 * 1100


def test_partition_more_ranks_than_chunks():
    ranges = partition_chunks([10, 100, 200], 4)
    assert sum(b - a for a, b in ranges) == 2 and ranges[-1][1] == 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, counts_all, ranges, q):
    import torch
    import torch.distributed as dist
    from parallelparsing_amd.dist import gather_counts
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a, b = ranges[rank]
    counts, bases = gather_counts(torch.tensor(counts_all[a:b], dtype=torch.int64), ranges)
    q.put((rank, counts.tolist(), bases.tolist()))
    dist.destroy_process_group()


def test_gather_counts_gloo_world2():
    import torch.multiprocessing as mp
    meta, _ = load_case("memlevel1_c10")
    counts_all = [c["records"] for c in meta["chunks"]]
    ranges = partition_chunks(meta["inputs"], 2)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, counts_all, ranges, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(60)
    exp_bases = np.concatenate([[0], np.cumsum(counts_all)[:-1]]).tolist()
    for _, counts, bases in res:
        assert counts == counts_all and bases == exp_bases


def test_abi_partition_matches_python_partition():
    """ppg_partition (the C ABI's) and dist.partition_chunks agree on every golden index."""
    import parallelparsing_amd as pp
    from conftest import CASES
    for name in CASES:
        meta, gz = load_case(name)
        ix = pp.Core.BuildDeflateIndex(gz, meta["chunksize"])
        _, inp, _ = ix.arrays()
        for world in (1, 2, 3, 8):
            b = pp.partition(ix, world).tolist()
            assert [(b[r], b[r + 1]) for r in range(world)] == partition_chunks(inp, world), (name, world)


def _host_comm_rank(rank, world, name, q):
    import parallelparsing_amd as pp
    c = pp.Comm.host(world, rank, name)
    q.put(c.rank_size())
    c.close()


def test_host_comm_rendezvous_world3():
    """ppg_comm_init_host: three processes meet in one shared-memory segment (no GPU needed)."""
    import uuid
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = f"/ppg_cpu_{uuid.uuid4().hex[:12]}"
    procs = [ctx.Process(target=_host_comm_rank, args=(r, 3, name, q)) for r in range(3)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
    assert got == [(0, 3), (1, 3), (2, 3)]


def _failing_rank(rank, world, name, path, chunksize, bad, q):
    """ppg_dist_decompress_all through the C ABI with no device context (this container has no
    GPU): every rank fails before decoding, one also with no index; all must still meet in the
    gather and return the same status instead of leaving the others waiting."""
    import ctypes as C
    import os as _os
    import parallelparsing_amd as pp
    from parallelparsing_amd._lib import lib
    try:
        ix = pp.Core.BuildDeflateIndex(path, chunksize)
        comm = pp.Comm.host(world, rank, name)
        m = ix.Count - 1
        counts, bases = (C.c_int64 * m)(), (C.c_int64 * m)()
        tot = C.c_int64(-1)
        rc = lib.ppg_dist_decompress_all(None, comm.handle, None if (bad and rank == 1) else ix.handle,
                                         _os.fsencode(path), 0, counts, bases, C.byref(tot))
        # the comm is still usable afterwards: a second call meets again and fails again
        rc2 = lib.ppg_dist_decompress_all(None, comm.handle, ix.handle, _os.fsencode(path), 0, counts, bases,
                                          C.byref(tot))
        comm.close()
        q.put((rank, rc, rc2))
    except Exception as e:   # noqa: BLE001 - reported to the parent
        q.put((rank, repr(e), None))


@pytest.mark.parametrize("bad", [False, True])
def test_failing_ranks_all_return_the_same_status(bad, tmp_path):
    """a rank that fails never returns before the collective."""
    import uuid
    import torch.multiprocessing as mp
    from parallelparsing_amd._lib import PPG_ARG_ERROR
    meta, gz = load_case("l6_c200")
    p = tmp_path / "f.gz"
    p.write_bytes(gz)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = f"/ppg_cpu_{uuid.uuid4().hex[:12]}"
    procs = [ctx.Process(target=_failing_rank, args=(r, 2, name, str(p), meta["chunksize"], bad, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    got = sorted(q.get(timeout=120) for _ in procs)
    for pr in procs:
        pr.join(60)
    assert got == [(0, PPG_ARG_ERROR, PPG_ARG_ERROR), (1, PPG_ARG_ERROR, PPG_ARG_ERROR)], got


def _stale_name_rank(name, q):
    import parallelparsing_amd as pp
    try:
        pp.Comm.host(2, 0, name)
        q.put("opened")
    except pp.PpgError as e:
        q.put(e.code)


def test_host_comm_refuses_a_stale_segment():
    """rank 0 never reuses an existing segment of the same name (stale arrive /
    generation counters would release the first barrier early)."""
    import uuid
    import torch.multiprocessing as mp
    from parallelparsing_amd._lib import PPG_IO_ERROR
    name = f"/ppg_cpu_{uuid.uuid4().hex[:12]}"
    path = "/dev/shm" + name
    with open(path, "wb") as f:   # what a crashed job leaves behind
        f.write(b"\1" * 4096)
    try:
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        pr = ctx.Process(target=_stale_name_rank, args=(name, q))
        pr.start()
        assert q.get(timeout=60) == PPG_IO_ERROR
        pr.join(30)
    finally:
        os.remove(path)


@pytest.mark.parametrize("world", [1, 2, 5])
def test_rank_enumerators_cover_the_file_in_order(world):
    """BatchedFASTQ(rank=, world=): each rank streams its ppg_partition share; the shares are
    contiguous, in rank order and cover every chunk (the multi-GPU enumeration surface)."""
    meta, gz = load_case("l6_c200")
    ix = pp.Core.BuildDeflateIndex(gz, meta["chunksize"])
    m = ix.Count - 1
    nxt = 0
    for r in range(world):
        first, n = pp.BatchedFASTQ(ix, "unused.gz", rank=r, world=world).chunk_range()
        assert first == nxt and n >= 0
        nxt = first + n
    assert nxt == m
    with pytest.raises(ValueError):
        pp.BatchedFASTQ(ix, "unused.gz", rank=world, world=world)


def _a2a_rank(rank, world, name, counts, q):
    import numpy as _np
    import parallelparsing_amd as pp
    try:
        c = pp.Comm.host(world, rank, name)
        # rank r sends to rank d the values r * 10**7 + d * 10**6 + i, i < counts[r, d]
        send = _np.concatenate([rank * 10**7 + d * 10**6 + _np.arange(counts[rank, d], dtype=_np.int64)
                                for d in range(world)])
        got = c.alltoallv(send, counts)
        c.close()
        q.put((rank, got.tolist()))
    except Exception as e:   # noqa: BLE001 - reported to the parent
        q.put((rank, repr(e)))


@pytest.mark.parametrize("world", [2, 3])
def test_host_alltoallv_in_rounds(world):
    """ppg_comm_alltoallv over the host transport (the paired-read key exchange's collective,
    ppg_pairs_check, rehearsed on a one-GPU box): uneven counts, zero counts and counts larger than
    one round of the shared slots (8 MiB per rank) arrive complete and in source order.  No GPU.
    The RCCL form of the same exchange (grouped ncclSend / ncclRecv over xGMI) has not run with more
    than one GPU: only its error paths are covered, with fake entry points
    (tests/native/host_check.cpp, run under ASan / TSan by tests/test_sanitizers.py)."""
    import uuid
    import torch.multiprocessing as mp
    rng = np.random.default_rng(world)
    counts = rng.integers(0, 3000, (world, world)).astype(np.int64)
    counts[0, world - 1] = 1_300_000   # several rounds
    counts[world - 1, 0] = 0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = f"/ppg_cpu_{uuid.uuid4().hex[:12]}"
    procs = [ctx.Process(target=_a2a_rank, args=(r, world, name, counts, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(60)
    for r in range(world):
        exp = np.concatenate([s * 10**7 + r * 10**6 + np.arange(counts[s, r], dtype=np.int64) for s in range(world)])
        assert res[r] == exp.tolist(), (r, str(res[r])[:200])


def _pairs_no_device(rank, world, name, q):
    import parallelparsing_amd as pp
    from parallelparsing_amd._lib import lib, PpgPairResult
    import ctypes as C
    try:
        c = pp.Comm.host(world, rank, name)
        h = C.c_void_p()
        assert lib.ppg_pairs_create(C.byref(h)) == 0
        res = PpgPairResult()
        # no shards on any rank (no GPU here): every rank joins the status gather and fails alike
        rc = lib.ppg_pairs_check(h, None, None, c.handle, C.byref(res))
        lib.ppg_pairs_free(h)
        c.close()
        q.put((rank, rc))
    except Exception as e:   # noqa: BLE001 - reported to the parent
        q.put((rank, repr(e)))


def test_pairs_check_failing_ranks_meet():
    """ppg_pairs_check on two ranks with nothing to check: both join the status gather and return
    the same PPG_ARG_ERROR instead of one waiting in the key exchange."""
    import uuid
    import torch.multiprocessing as mp
    from parallelparsing_amd._lib import PPG_ARG_ERROR
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = f"/ppg_cpu_{uuid.uuid4().hex[:12]}"
    procs = [ctx.Process(target=_pairs_no_device, args=(r, 2, name, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
    assert res == {0: PPG_ARG_ERROR, 1: PPG_ARG_ERROR}

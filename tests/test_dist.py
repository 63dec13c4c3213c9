"""Multi-rank path on CPU: chunk partition + the padded all-gather of per-chunk record counts,
run with torch.distributed gloo at world_size 2 (the GPU run uses nccl = RCCL)."""
import os
import socket

import numpy as np
import pytest

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

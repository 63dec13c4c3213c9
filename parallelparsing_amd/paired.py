"""Paired-end, record-aligned pair chunks (BASELINE configs[4]).

The reference names the goal only (README.md:9); there is no code and no oracle beyond per-file
parity.  A read pair is two files R1/R2 whose record i belong together: Generator-shape headers
"SRR<id>.<spot>.<mate>" with equal spot numbers.  Each file is decoded by its own
DecompressAll (the per-file parity path); pair chunk j is records [j*K, (j+1)*K) of both files,
by global record number.  Records the reference parses twice (a Point on a record
start) are dropped first, or every later pair would shift by one.

Multi-GPU: ranks hold contiguous record ranges of each file that do not line up between the
files (chunk boundaries differ), so checking pairs is a real exchange step: one all_to_all of
8-byte spot keys moves every key to the rank that owns its pair number (RCCL over xGMI).
"""
import ctypes as C

import numpy as np

from . import Device, IndexIO, Shard, records_from_descriptors
from ._lib import lib, check

DUP = -2      # key of a record parsed twice (Q1), dropped before pairing
NOKEY = -1    # identifier without an "SRR<id>.<spot>." field


def attach_keys(shard, max_records):
    """Give a shard a device key buffer that every output batch of its later runs fills
    (ppg_shard_set_keys): pairing then works on shards of any number of batches, e.g. configs[4]'s
    2 x 25 GB on one GPU, whose outputs cannot both stay resident."""
    import torch
    keys = torch.empty(max(1, int(max_records)), dtype=torch.int64, device=torch.device("cuda", shard.dev.device))
    shard.dev.wait_stream(torch.cuda.current_stream(keys.device))   # the block may be recycled
    return shard.set_keys(keys)


def shard_keys(shard):
    """Spot numbers of all records of a shard, in record order, as a device tensor (int64; DUP /
    NOKEY markers kept).  GPU kernel ppg_record_keys: run per batch during the shard's run when
    attach_keys() gave it a buffer, else (one-batch shards) extracted now."""
    import torch
    n = shard.total_records
    if getattr(shard, "_keys", None) is not None:
        if n > shard._keys.numel():
            raise ValueError("key buffer smaller than the shard's records")
        # the keys were written on the ctx stream: torch's stream must not read them earlier
        shard.dev.stream_wait(torch.cuda.current_stream(shard._keys.device))
        return shard._keys[:n]
    dev = torch.device("cuda", shard.dev.device)
    keys = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    # the kernel writes on the ctx's stream: torch's caching allocator may have handed out a block
    # that kernels still queued on torch's stream read (e.g. a boolean mask freed by the caller
    # while its gather is in flight), so the ctx waits for torch's stream first (stream-ordered,
    # ppg_ctx_wait_stream; r01 drained torch's stream from the host here)
    shard.dev.wait_stream(torch.cuda.current_stream(dev))
    check(lib.ppg_shard_keys(shard.handle, C.c_void_p(keys.data_ptr()), n), "ppg_shard_keys")
    return keys[:n]


def dedup(keys):
    """(kept keys, their record numbers in the shard) — Q1 duplicates removed."""
    import torch
    keep = keys != DUP
    idx = torch.nonzero(keep).flatten()
    return keys[keep], idx


def check_pairs(k1, k2):
    """Pair invariant on two aligned key arrays: same length, every key present, equal spots.
    Returns the number of pairs; raises ValueError on the first violation."""
    import torch
    if k1.numel() != k2.numel():
        raise ValueError(f"R1 has {k1.numel()} records, R2 {k2.numel()}: not a read pair")
    bad = (k1 != k2) | (k1 < 0)
    nbad = int(bad.sum())
    if nbad:
        i = int(torch.nonzero(bad)[0])
        raise ValueError(f"{nbad} mismatched pairs; first at pair {i}: spot {int(k1[i])} vs {int(k2[i])}")
    return k1.numel()


def _read_range(path, index):
    n = index.Count - 1
    _, i0, _, _ = index.point_fields(0)
    _, i1, _, _ = index.point_fields(n)
    with open(path, "rb") as f:
        f.seek(i0 - 1)
        return f.read(i1 - i0 + 1)


class PairedFASTQ:
    """Two BatchedFASTQ streams zipped into record-aligned pair chunks of `pair_chunk` records
    (default 50,000, BASELINE configs[4]).  Both files are decoded on one GPU and their pairing
    is verified on the device before any pair is handed out."""

    def __init__(self, index1, gz1, index2, gz2, pair_chunk=50_000, device=None):
        self.index = [IndexIO.Deserialize(i) if isinstance(i, str) else i for i in (index1, index2)]
        self.paths = [gz1, gz2]
        self.K = int(pair_chunk)
        self.dev = device or Device.default()
        self.shards = [Shard(ix, _read_range(p, ix), 0, ix.Count - 1, device=self.dev).run()
                       for ix, p in zip(self.index, self.paths)]
        keys = [shard_keys(s) for s in self.shards]
        (k1, self._rec1), (k2, self._rec2) = dedup(keys[0]), dedup(keys[1])
        self.pairs = check_pairs(k1, k2)
        self._bases = [np.asarray(s.record_base(), np.int64) for s in self.shards]
        self._rec = [self._rec1.cpu().numpy(), self._rec2.cpu().numpy()]

    def Count(self):
        return self.pairs

    @property
    def chunks(self):
        return (self.pairs + self.K - 1) // self.K

    def _records(self, f, lo, hi):
        """FastqRecords of file f for pair numbers [lo, hi)."""
        sh, ix, bases, rec = self.shards[f], self.index[f], self._bases[f], self._rec[f]
        out, cache = [], {}
        for r in rec[lo:hi]:                       # shard record number of pair r
            k = int(np.searchsorted(bases, r, side="right") - 1)
            if k not in cache:
                raw = bytes(ix[k].offset) + sh.chunk_bytes(k).tobytes()
                cache = {k: records_from_descriptors(raw, sh.chunk_records(k))}
            out.append(cache[k][int(r - bases[k])])
        return out

    def pair_chunk(self, j):
        """(R1 records, R2 records) of pair chunk j: pairs [j*K, min((j+1)*K, Count))."""
        lo, hi = j * self.K, min((j + 1) * self.K, self.pairs)
        if not 0 <= lo < hi:
            raise IndexError(j)
        return self._records(0, lo, hi), self._records(1, lo, hi)

    def __iter__(self):
        for j in range(self.chunks):
            a, b = self.pair_chunk(j)
            yield from zip(a, b)


def distributed_pair_check(k1_local, k2_local, group=None):
    """Multi-rank pair check.  Rank r holds the (deduplicated) keys of a contiguous range of R1
    records and of R2 records, in rank order.  Every key is sent to the rank owning its pair
    number (pairs split evenly), with one all_gather of counts and one all_to_all_single per
    file; then each rank compares its pairs.  Returns (pairs, mismatches) over all ranks."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = k1_local.device
    n = torch.tensor([k1_local.numel(), k2_local.numel()], dtype=torch.int64, device=dev)
    allc = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(allc, n, group=group)
    cnt = torch.stack(allc).cpu().numpy()          # [world, 2]
    tot1, tot2 = int(cnt[:, 0].sum()), int(cnt[:, 1].sum())
    pairs = min(tot1, tot2)
    own = [pairs * r // world for r in range(world + 1)]   # rank r owns pairs [own[r], own[r+1])

    def to_owners(keys, f):
        start = int(cnt[:rank, f].sum())
        end = start + keys.numel()
        send = [max(0, min(end, own[r + 1]) - max(start, own[r])) for r in range(world)]
        recv = []
        for src in range(world):
            s0 = int(cnt[:src, f].sum())
            s1 = s0 + int(cnt[src, f])
            recv.append(max(0, min(s1, own[rank + 1]) - max(s0, own[rank])))
        lo = max(0, own[0] - start)
        body = keys[lo:lo + sum(send)].contiguous()
        out = torch.empty(sum(recv), dtype=keys.dtype, device=dev)
        dist.all_to_all_single(out, body, recv, send, group=group)
        return out

    a, b = to_owners(k1_local, 0), to_owners(k2_local, 1)
    bad = ((a != b) | (a < 0)).sum() if a.numel() == b.numel() else torch.tensor(max(a.numel(), b.numel()))
    res = torch.tensor([int(bad) + (abs(tot1 - tot2) if rank == 0 else 0)], dtype=torch.int64, device=dev)
    dist.all_reduce(res, group=group)
    return pairs, int(res.item())

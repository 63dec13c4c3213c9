"""Multi-GPU DecompressAll: static chunk sharding + one all-gather of per-chunk record counts.

SURVEY §8(e): chunks are independent given their Points (Common/Index.cs:42-46 carries each
window), so rank r owns one contiguous chunk range balanced by compressed bytes and decodes it
with no data-path collective.  The only exchange is an all-gather(v) of per-chunk record counts
(int64), followed by an exclusive scan that yields every chunk's global record id.  RCCL has no
all-gatherv, so counts are padded to the largest shard (torch.distributed all_gather_into_tensor,
backend "nccl" = RCCL over xGMI on MI355X; "gloo" in the CPU tests).  One process per GPU.
"""
import numpy as np


def partition_chunks(inputs, world):
    """Contiguous chunk ranges [a_r, b_r) balanced by compressed bytes.

    inputs: Point.Input for every point (len = chunks + 1).  Chunk k reads
    inputs[k+1] - inputs[k] + 1 bytes (LazyFileReader.cs:64)."""
    inputs = np.asarray(inputs, dtype=np.int64)
    nchunks = len(inputs) - 1
    cost = inputs[1:] - inputs[:-1] + 1
    cum = np.concatenate([[0], np.cumsum(cost)])
    total = cum[-1]
    bounds = [0]
    for r in range(1, world):
        target = total * r / world
        k = int(np.searchsorted(cum, target, side="left"))
        k = min(max(k, bounds[-1]), nchunks)
        bounds.append(k)
    bounds.append(nchunks)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


def gather_counts(local_counts, ranges, group=None, device=None):
    """All-gather per-chunk record counts of every rank's range; returns (counts, bases) over all
    chunks in canonical order (bases = exclusive scan = global id of each chunk's first record).

    local_counts: 1-D int64 torch tensor of this rank's chunk counts (on `device`)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    width = max(b - a for a, b in ranges)
    width = max(width, 1)
    buf = torch.zeros(width, dtype=torch.int64, device=device)
    buf[: local_counts.numel()] = local_counts
    out = torch.empty(world * width, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(out, buf, group=group)
    out = out.view(world, width).cpu().numpy()
    counts = np.concatenate([out[r, : b - a] for r, (a, b) in enumerate(ranges)])
    bases = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64)
    return counts, bases

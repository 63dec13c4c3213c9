"""Stream-ordered handoff between torch's stream and the library's (ppg_ctx_wait_stream /
ppg_stream_wait_ctx): no host synchronisation anywhere below."""
import numpy as np
import pytest

import parallelparsing_amd as pp
from conftest import load_case

pytestmark = pytest.mark.gpu


def _case():
    meta, gz = load_case("l6_c200")
    ix = pp.Core.BuildDeflateIndex(gz, meta["chunksize"])
    n = ix.Count - 1
    _, i0, _, _ = ix.point_fields(0)
    _, i1, _, _ = ix.point_fields(n)
    return meta, ix, n, np.frombuffer(gz[i0 - 1:i1], np.uint8).copy()


def test_shard_reads_comp_written_by_a_long_torch_kernel(device):
    """torch's stream spins ~50 ms, then writes the compressed bytes; the shard, created and run
    right away, must decode what torch wrote, not the zeros that were there before."""
    import torch
    meta, ix, n, comp_h = _case()
    dev = torch.device("cuda", device.device)
    ref = pp.Shard(ix, comp_h, 0, n, device=device).run()
    comp = torch.zeros(comp_h.size + 256, dtype=torch.uint8, device=dev)
    src = torch.from_numpy(comp_h).pin_memory()
    torch.cuda.synchronize()
    for _ in range(3):
        comp.zero_()
        torch.cuda._sleep(100_000_000)                    # ~50 ms of GPU time on torch's stream
        comp[: comp_h.size].copy_(src, non_blocking=True)
        sh = pp.Shard(ix, comp.data_ptr(), 0, n, device=device, comp_on_device=True, comp_len=comp_h.size).run()
        r = sh.results()
        assert (r["status"] == 0).all()
        assert sh.total_records == meta["total_records"]
        for k in range(n):
            assert np.array_equal(sh.chunk_bytes(k), ref.chunk_bytes(k)), k


def test_copy_output_to_device_then_torch_reads_it(device):
    """ppg_shard_copy_output into a torch tensor, then torch's stream consumes it after
    ppg_stream_wait_ctx: equal to the host copy of the same bytes."""
    import torch
    meta, ix, n, comp_h = _case()
    sh = pp.Shard(ix, comp_h, 0, n, device=device).run()
    total = int(ix.point_fields(n)[0] - ix.point_fields(0)[0])
    host = sh.copy_output(0, total)
    assert host.tobytes() == b"".join(sh.chunk_bytes(k).tobytes() for k in range(n))
    dev = torch.device("cuda", device.device)
    d = torch.empty(total, dtype=torch.uint8, device=dev)
    torch.cuda._sleep(50_000_000)                          # torch's stream is busy when the copy is queued
    sh.copy_output(0, total, d)
    device.stream_wait(torch.cuda.current_stream(dev))
    assert np.array_equal(d.cpu().numpy(), host)
    part = sh.copy_output(17, 1000)
    assert part.tobytes() == host[17:1017].tobytes()
    with pytest.raises(pp.PpgError):
        sh.copy_output(total - 10, 11)


def test_keys_written_into_a_recycled_block(device):
    """shard_keys allocates from torch's caching allocator: a block freed while torch's stream
    still reads it must not be overwritten early (the r01 race), with the wait on the device."""
    import torch
    from parallelparsing_amd import paired
    from parallelparsing_amd.tiled import TiledFile
    tf = TiledFile(20000, 2, 1000, threads=4, mate=1)
    f = tf.file_bytes()
    ix = tf.index()
    n = tf.npoints - 1
    _, i0, _, _ = ix.point_fields(0)
    _, i1, _, _ = ix.point_fields(n)
    sh = pp.Shard(ix, np.frombuffer(f[i0 - 1:i1], np.uint8), 0, n, device=device).run()
    ref = paired.shard_keys(sh).cpu()
    dev = torch.device("cuda", device.device)
    for _ in range(4):
        x = torch.arange(sh.total_records, dtype=torch.int64, device=dev)
        torch.cuda._sleep(50_000_000)
        y = x * 3                                          # queued behind the sleep, reads x
        del x                                              # x's block is free for the next allocation
        k = paired.shard_keys(sh)                          # likely gets x's block
        assert torch.equal(k.cpu(), ref)
        assert torch.equal(y.cpu(), torch.arange(sh.total_records, dtype=torch.int64) * 3)

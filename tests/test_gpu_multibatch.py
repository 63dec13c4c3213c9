"""Shards decoded in several output batches (VERDICT r02 missing #2 / weak #9): record descriptors
stay resident for every batch (ppg_shard_copy_records) and the spot keys of paired reads are
extracted per batch while its output is resident (ppg_shard_set_keys), so configs[4]'s 2 x 25 GB
pair decodes on one MI355X without both ~103 GB outputs resident."""
import ctypes as C

import numpy as np
import pytest
import torch

import parallelparsing_amd as pp
from parallelparsing_amd import paired
from parallelparsing_amd.tiled import TiledFile

pytestmark = pytest.mark.gpu


def _member(nrec, chunk, seed=0, mate=1):
    S = pp.synth()
    sz = S.ppg_synth_fastq_size_mate(0, nrec, 150, mate)
    txt = np.zeros(sz, np.uint8)
    S.ppg_synth_fastq_mate(seed, mate, 0, nrec, 150, C.c_void_p(txt.ctypes.data), sz, 8)
    gzb = np.zeros(sz, np.uint8)
    L = S.ppg_synth_gzip(C.c_void_p(txt.ctypes.data), sz, 6, 1 << 20, 8, C.c_void_p(gzb.ctypes.data), gzb.size)
    gz = gzb[:L].tobytes()
    return gz, pp.Core.BuildDeflateIndex(gz, chunk)


def _shard(gz, ix, device, out_capacity):
    n = ix.Count - 1
    _, i0, _, _ = ix.point_fields(0)
    _, i1, _, _ = ix.point_fields(n)
    return pp.Shard(ix, np.frombuffer(gz[i0 - 1:i1], np.uint8), 0, n, device=device, out_capacity=out_capacity)


def test_multi_batch_records_and_keys_equal_one_batch(device):
    gz, ix = _member(120_000, 2000)
    one = _shard(gz, ix, device, 0).run()
    many = _shard(gz, ix, device, 3 << 20)                  # ~3 MB of output per batch
    paired.attach_keys(many, 200_000)
    many.run()
    assert one.batches == 1 and many.batches > 8
    assert many.total_records == one.total_records == 120_000
    for k in range(ix.Count - 1):
        assert np.array_equal(many.chunk_records(k), one.chunk_records(k)), k
    k1 = paired.shard_keys(one)
    k2 = paired.shard_keys(many)
    assert torch.equal(k1, k2)
    assert (k2 >= 1).all()
    # a second run writes the same keys again (the buffer is reused per run)
    many.run()
    assert torch.equal(paired.shard_keys(many), k1)


def test_keys_buffer_too_small_fails_loudly(device):
    gz, ix = _member(20_000, 2000)
    sh = _shard(gz, ix, device, 1 << 20)
    paired.attach_keys(sh, 1000)
    with pytest.raises(pp.PpgError) as e:
        sh.run()
    assert e.value.code == pp._lib.PPG_BUF_ERROR


def test_configs4_full_size_pair_on_one_gpu(device):
    """BASELINE configs[4]: a read pair of two ~25 GB single-member .fastq.gz files (chunk =
    50,000), decoded on one MI355X in output batches of 40 GiB per file; every record's spot
    number is extracted on the device per batch, Q1 duplicates dropped, and R1[i].spot ==
    R2[i].spot checked for every pair."""
    reps = 102
    tfs = [TiledFile(2_621_440, reps, 50_000, seed=m - 1, mate=m, threads=16) for m in (1, 2)]
    assert all(tf.file_len > 24e9 for tf in tfs)
    dev = torch.device("cuda", device.device)
    shards, comps = [], []
    for tf in tfs:
        lo, hi = int(tf.p_input[0]) - 1, int(tf.p_input[-1])   # file bytes [Input_0 - 1, Input_n - 1]
        comp = torch.empty(hi - lo + 256, dtype=torch.uint8, device=dev)
        comp[hi - lo:].zero_()
        tf.fill_device(comp, lo, hi)
        torch.cuda.synchronize()
        sh = pp.Shard(tf.index(0, tf.npoints), comp.data_ptr(), first=0, n=tf.npoints - 1, device=device,
                      comp_on_device=True, comp_len=hi - lo, out_capacity=40 << 30)
        text = int(tf.p_output[-1])
        paired.attach_keys(sh, text // 200 + 4096)
        sh.run()
        assert sh.batches >= 3
        r = sh.results()
        assert (r["status"] == 0).all()
        assert (r["produced"] == np.diff(tf.p_output)).all()
        assert sh.total_records == tf.expected_records()
        shards.append(sh)
        comps.append(comp)
    # the pair check in the library (ppg_pairs_check: keys of every batch, Q1 duplicates dropped)
    res = paired.Pairs().check(shards[0], shards[1])
    assert res["pairs"] == 2_621_440 * reps and res["mismatches"] == 0, res
    assert res["records"] == (2_621_440 * reps,) * 2
    assert [sh.total_records - d for sh, d in zip(shards, res["duplicates"])] == [2_621_440 * reps] * 2
    # the same pairing restated with torch on the keys (test-side reference)
    k = [paired.shard_keys(sh) for sh in shards]
    k = [x[x != paired.DUP] for x in k]
    assert torch.equal(k[0], k[1]) and bool((k[0] >= 0).all())
    # record-aligned pair chunks at configs[4]'s K = 50,000 (the deliverable): every
    # window packed on the device -- the shards' 40 GiB batches run again as the windows advance and
    # pair chunks straddling a batch boundary carried -- every pair chunk once, K pairs each (the
    # last fewer), the halves' bytes adding up to each member's text; the first pair chunk of every
    # window (a carried one after each batch change) and the last compared byte for byte with the text
    K = 50_000
    pairs = 2_621_440 * reps
    pr = paired.Pairs()
    pr.check(shards[0], shards[1])

    def check_windows(it):
        nbytes, nxt, windows = [0, 0], 0, 0
        for j0, j1 in it:
            assert j0 == nxt
            for j in range(j0, j1):
                for f in (0, 1):
                    _, n, _, r = pr.chunk(j, f)
                    assert r == min(K, pairs - j * K), (j, f, r)
                    nbytes[f] += n
                if j == j0 or j == -(-pairs // K) - 1:
                    for f, tf in enumerate(tfs):
                        b, d = pr.copy_chunk(j, f)
                        eb = _records_text(tf, j * K, min((j + 1) * K, pairs))
                        assert b.tobytes() == eb, (j, f)
                        nl = np.nonzero(np.frombuffer(eb, np.uint8) == 10)[0].astype(np.uint32).reshape(-1, 4)
                        assert np.array_equal(d, nl), (j, f)
            nxt = j1
            windows += 1
        assert nxt == -(-pairs // K) and windows > 10
        assert nbytes == [int(tf.p_output[-1]) for tf in tfs]

    check_windows(pr.emit(shards[0], shards[1], K, window_bytes=8 << 30))
    assert pr.emit_stats()["reruns"] >= shards[0].batches + shards[1].batches
    # fused (ppg_pairs_emit_run, r05): the windows drive the shards' own run -- each 40 GiB batch
    # decoded once, no re-run -- and the check after it agrees
    check_windows(pr.emit_run(shards[0], shards[1], K, window_bytes=8 << 30))
    assert pr.emit_stats()["reruns"] == 0
    res2 = pr.check(shards[0], shards[1])
    assert res2["pairs"] == pairs and res2["mismatches"] == 0 and res2["duplicates"] == res["duplicates"], res2
    assert [sh.total_records for sh in shards] == [tf.expected_records() for tf in tfs]


_STARTS = {}


def _records_text(tf, lo, hi):
    """Bytes of records [lo, hi) of a tiled member: its segment's records, repeated."""
    if id(tf) not in _STARTS:
        nl = np.nonzero(tf.text == 10)[0]
        _STARTS[id(tf)] = np.concatenate([[0], nl[3::4] + 1]).astype(np.int64)
    st, n, out, i = _STARTS[id(tf)], tf.records, [], lo
    while i < hi:
        r = i % n
        take = min(hi - i, n - r)
        out.append(tf.text[int(st[r]):int(st[r + take])].tobytes())
        i += take
    return b"".join(out)

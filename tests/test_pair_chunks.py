"""Record-aligned pair chunks (BASELINE configs[4]; the reference's goal,
README.md:9) emitted by the library (ppg_pairs_emit_*, csrc/ppg_pairs.hip): pair chunk j = pairs
[j*K, (j+1)*K) of R1 and R2, each half packed on the device as its records' bytes back to back plus
one descriptor per record.  Every half is compared with the per-file oracle (oracle.c's Extract +
Parse over zlib, the records the reference parses twice -- SURVEY Q1 -- dropped): on one rank with
one-batch shards, with multi-batch shards (batches run again as the windows advance, pair chunks
straddling batches carried), and on 2 / 3 ranks of the one GPU over the host transport (records
moved to their pair chunk's owner by ppg_comm_alltoallv).  The full configs[4] pair is in
tests/test_gpu_multibatch.py."""
import ctypes as C
import hashlib
import uuid
import zlib

import numpy as np
import pytest

import parallelparsing_amd as pp
from oracle import oracle as O
from parallelparsing_amd import paired
from parallelparsing_amd import _lib

pytestmark = pytest.mark.gpu


def mate_gz(mate, nrec, seed, flush_every=0):
    """A mate file of the Generator shape; flush_every > 0 ends a deflate block after every that
    many records (full flush), so Points fall on record starts and Q1 duplicates appear."""
    S = pp.synth()
    sz = S.ppg_synth_fastq_size_mate(0, nrec, 150, mate)
    txt = np.zeros(sz, np.uint8)
    S.ppg_synth_fastq_mate(seed, mate, 0, nrec, 150, C.c_void_p(txt.ctypes.data), sz, 8)
    if not flush_every:
        gzb = np.zeros(sz, np.uint8)
        L = S.ppg_synth_gzip(C.c_void_p(txt.ctypes.data), sz, 6, 1 << 20, 8, C.c_void_p(gzb.ctypes.data), gzb.size)
        return gzb[:L].tobytes()
    lines = txt.tobytes().split(b"\n")
    co = zlib.compressobj(6, zlib.DEFLATED, 31)
    out = []
    for g in range(0, nrec, flush_every):
        out.append(co.compress(b"\n".join(lines[4 * g:4 * min(nrec, g + flush_every)]) + b"\n"))
        out.append(co.flush(zlib.Z_FULL_FLUSH))
    out.append(co.flush())
    return b"".join(out)


def oracle_records(gz, chunk):
    """The file's records as the reference parses them chunk by chunk (oracle: Core.cs:133-192 +
    Parsing.cs:11-69 over zlib), each record's bytes raw[start, n4] -- minus the Q1 duplicates
    (a chunk's first record lying wholly inside its Point's offset)."""
    oi = O.build_index(gz, chunk)
    recs, dups = [], 0
    for k in range(oi.count - 1):
        off = oi.point(k)[4]
        raw = off + O.extract(gz, oi, k)
        start = 0
        for j, (n1, n2, n3, n4) in enumerate(O.parse(off, raw[len(off):]).tolist()):
            if j == 0 and n4 < len(off):
                dups += 1
            else:
                recs.append(raw[start:n4 + 1])
            start = n4 + 1
    return recs, dups


def expected_half(recs, lo, hi):
    b = b"".join(recs[lo:hi])
    nl = np.nonzero(np.frombuffer(b, np.uint8) == 10)[0].astype(np.uint32)
    return b, nl.reshape(-1, 4) if nl.size else np.zeros((0, 4), np.uint32)


def shard_of(gz, ix, device, out_capacity=0, first=0, n=None):
    n = ix.Count - 1 - first if n is None else n
    _, i0, _, _ = ix.point_fields(first)
    _, i1, _, _ = ix.point_fields(first + n)
    sh = pp.Shard(ix, np.frombuffer(gz[i0 - 1:i1], np.uint8), first, n, device=device, out_capacity=out_capacity)
    if sh.batches > 1:
        paired.attach_keys(sh, 400_000)
    return sh.run()


@pytest.fixture(scope="module")
def pair_files():
    nrec = 30_000
    gz = [mate_gz(1, nrec, 0, flush_every=37), mate_gz(2, nrec, 1)]
    chunks = (700, 1100)   # the files' chunk boundaries never line up
    recs = []
    for g, c in zip(gz, chunks):
        r, d = oracle_records(g, c)
        recs.append((r, d))
    assert len(recs[0][0]) == len(recs[1][0]) == nrec
    assert recs[0][1] > 10 and recs[1][1] == 0   # R1 carries Q1 duplicates, R2 none
    return gz, chunks, recs, nrec


def check_window(pr, j0, j1, K, recs, nrec, seen):
    for j in range(j0, j1):
        lo, hi = j * K, min((j + 1) * K, nrec)
        for f in (0, 1):
            b, d = pr.copy_chunk(j, f)
            eb, ed = expected_half(recs[f][0], lo, hi)
            assert b.tobytes() == eb, (j, f)
            assert np.array_equal(d, ed), (j, f)
            # and the record reader over the half gives the oracle's records
            if j == j0:
                r = pp.records_from_descriptors(b.tobytes(), d)
                assert r[0].identifier == recs[f][0][lo][1:recs[f][0][lo].index(b"\n")]
        assert j not in seen
        seen.add(j)


@pytest.mark.parametrize("K,cap,window", [(4000, 0, 0), (4096, 0, 1 << 20), (2500, 3 << 20, 0), (7777, 2 << 20, 3 << 20)])
def test_pair_chunks_one_rank(pair_files, device, K, cap, window):
    """One rank: one-batch shards (one window, or windows of 1 MiB per half), and multi-batch
    shards (cap = 2-3 MB of output per batch: every window runs batches again, pair chunks straddle
    batches) -- every half equals the oracle's records, every pair chunk exactly once."""
    gz, chunks, recs, nrec = pair_files
    ix = [pp.Core.BuildDeflateIndex(g, c) for g, c in zip(gz, chunks)]
    sh = [shard_of(g, i, device, cap) for g, i in zip(gz, ix)]
    if cap:
        assert sh[0].batches >= 3 and sh[1].batches >= 3
    pr = paired.Pairs()
    res = pr.check(sh[0], sh[1])
    assert res["pairs"] == nrec and res["mismatches"] == 0 and res["duplicates"][0] == recs[0][1]
    seen = set()
    windows = 0
    for j0, j1 in pr.emit(sh[0], sh[1], K, window_bytes=window):
        check_window(pr, j0, j1, K, recs, nrec, seen)
        windows += 1
    assert seen == set(range(-(-nrec // K)))
    st = pr.emit_stats()
    if window or cap:
        assert windows > 1, st
    if cap:
        assert st["reruns"] >= sh[0].batches + sh[1].batches, st
    # a second emission over the same check gives the same halves (buffers reused)
    seen2 = set()
    for j0, j1 in pr.emit(sh[0], sh[1], K, window_bytes=window):
        check_window(pr, j0, j1, K, recs, nrec, seen2)
    assert seen2 == seen


@pytest.mark.parametrize("K,cap,window,short", [(4000, 0, 0, 0), (2500, 3 << 20, 0, 0), (7777, 2 << 20, 3 << 20, 0),
                                                (3000, 2 << 20, 0, 1234)])
def test_pair_chunks_fused_run(pair_files, device, K, cap, window, short):
    """ppg_pairs_emit_run: no check first -- the windows drive the shards' own (first) run, each
    output batch decoded once and packed while resident (no batch re-run), the Q1 numbering built
    batch by batch from the keys.  Every half equals the oracle's records; afterwards both shards
    stand as Shard.run leaves them (same record counts) and the check agrees.  short > 0: R2 has
    that many records fewer, so the pair count is only known once R2 has run."""
    gz, chunks, recs, nrec = pair_files
    if short:
        g2 = mate_gz(2, nrec - short, 1)
        r2, d2 = oracle_records(g2, chunks[1])
        gz = [gz[0], g2]
        recs = [recs[0], (r2, d2)]
    npairs = nrec - short
    ix = [pp.Core.BuildDeflateIndex(g, c) for g, c in zip(gz, chunks)]
    sh = []
    for g, i in zip(gz, ix):
        _, i0, _, _ = i.point_fields(0)
        _, i1, _, _ = i.point_fields(i.Count - 1)
        s_ = pp.Shard(i, np.frombuffer(g[i0 - 1:i1], np.uint8), 0, i.Count - 1, device=device, out_capacity=cap)
        paired.attach_keys(s_, 400_000)
        sh.append(s_)
    if cap:
        assert sh[0].batches >= 3 and sh[1].batches >= 3
    pr = paired.Pairs()
    seen = set()
    windows = 0
    for j0, j1 in pr.emit_run(sh[0], sh[1], K, window_bytes=window):
        check_window(pr, j0, j1, K, recs, npairs, seen)
        windows += 1
    assert seen == set(range(-(-npairs // K)))
    st = pr.emit_stats()
    assert st["reruns"] == 0 and st["pair_chunks"] == len(seen), st
    if cap:
        assert windows > 1, st
    res = pr.check(sh[0], sh[1])
    assert res["pairs"] == npairs and res["mismatches"] == short and res["duplicates"][0] == recs[0][1]
    assert res["records"] == (nrec, nrec - short)
    # the shards' own results: as a plain run leaves them
    for s_, g, i in zip(sh, gz, ix):
        ref = shard_of(g, i, device, cap)
        assert s_.total_records == ref.total_records
        assert np.array_equal(s_.results()["records"], ref.results()["records"])


def test_paired_fastq_surface(pair_files, device, tmp_path):
    """PairedFASTQ (Python mirror of the C# GpuPairedFASTQ) over .gz files: pair chunks from the
    library's emission, the pairs' identifiers those of the oracle's records."""
    gz, chunks, recs, nrec = pair_files
    paths = []
    for m, g in enumerate(gz):
        p = tmp_path / f"m{m}.fastq.gz"
        p.write_bytes(g)
        paths.append(str(p))
    ix = [pp.Core.BuildDeflateIndex(p, c) for p, c in zip(paths, chunks)]
    pf = paired.PairedFASTQ(ix[0], paths[0], ix[1], paths[1], pair_chunk=5000, device=device, out_capacity=4 << 20)
    assert pf.Count() == nrec and pf.chunks == 6
    n = 0
    for j, a, b in pf.pair_chunks():
        assert len(a) == len(b) == min(5000, nrec - 5000 * j)
        for i in (0, len(a) - 1):
            g = 5000 * j + i
            assert a[i].identifier == recs[0][0][g][1:recs[0][0][g].index(b"\n")]
            assert a[i].identifier.split(b".")[:2] == b[i].identifier.split(b".")[:2]
        n += len(a)
    assert n == nrec


def test_emit_refuses_bad_use(pair_files, device):
    gz, chunks, recs, nrec = pair_files
    ix = [pp.Core.BuildDeflateIndex(g, c) for g, c in zip(gz, chunks)]
    sh = [shard_of(g, i, device) for g, i in zip(gz, ix)]
    pr = paired.Pairs()
    with pytest.raises(pp.PpgError):   # no check yet
        next(pr.emit(sh[0], sh[1], 1000))
    pr.check(sh[0], sh[1])
    with pytest.raises(pp.PpgError):   # K < 1
        next(pr.emit(sh[0], sh[1], 0))
    it = pr.emit(sh[0], sh[1], 1000)
    j0, j1 = next(it)
    with pytest.raises(pp.PpgError):   # outside the current window
        pr.chunk(j1 + 5, 0)


def test_emit_run_edges(pair_files, device):
    """ppg_pairs_emit_run: shards without keys are refused; one pair chunk larger than all the
    pairs; a 1-byte window budget (one pair chunk per window); an emission stopped early leaves the
    shards unrun (the check refuses them) and a new emit_run starts over from their first batch."""
    gz, chunks, recs, nrec = pair_files
    ix = [pp.Core.BuildDeflateIndex(g, c) for g, c in zip(gz, chunks)]

    def fresh(keys=True):
        out = []
        for g, i in zip(gz, ix):
            _, i0, _, _ = i.point_fields(0)
            _, i1, _, _ = i.point_fields(i.Count - 1)
            s_ = pp.Shard(i, np.frombuffer(g[i0 - 1:i1], np.uint8), 0, i.Count - 1, device=device, out_capacity=2 << 20)
            if keys:
                paired.attach_keys(s_, 400_000)
            out.append(s_)
        return out
    pr = paired.Pairs()
    bare = fresh(keys=False)
    with pytest.raises(pp.PpgError):
        next(pr.emit_run(bare[0], bare[1], 1000))
    sh = fresh()
    seen = set()
    wins = list(pr.emit_run(sh[0], sh[1], 10 * nrec))
    assert wins == [(0, 1)]
    check_window(pr, 0, 1, 10 * nrec, recs, nrec, seen)
    seen = set()
    n = 0
    for j0, j1 in pr.emit_run(sh[0], sh[1], 5000, window_bytes=1):
        assert j1 == j0 + 1
        check_window(pr, j0, j1, 5000, recs, nrec, seen)
        n += 1
    assert n == -(-nrec // 5000)
    it = pr.emit_run(sh[0], sh[1], 3000)
    next(it)
    it.close()
    with pytest.raises(pp.PpgError):   # stopped early: the shards have not run
        pr.check(sh[0], sh[1])
    seen = set()
    for j0, j1 in pr.emit_run(sh[0], sh[1], 3000):
        check_window(pr, j0, j1, 3000, recs, nrec, seen)
    assert seen == set(range(-(-nrec // 3000)))
    assert pr.check(sh[0], sh[1])["mismatches"] == 0


def _emit_rank(rank, world, name, gz, chunks, K, q):
    try:
        import parallelparsing_amd as pp2
        from parallelparsing_amd import paired as P
        dev = pp2.Device(0)
        comm = pp2.Comm.host(world, rank, name)
        shards = []
        for g, c in zip(gz, chunks):
            ix = pp2.Core.BuildDeflateIndex(g, c)
            b = pp2.partition(ix, world)
            a, e = int(b[rank]), int(b[rank + 1])
            shards.append(shard_of(g, ix, dev, 0, a, e - a))
        pr = P.Pairs()
        res = pr.check(shards[0], shards[1], comm)
        out = {}
        for j0, j1 in pr.emit(shards[0], shards[1], K, comm):
            for j in range(j0, j1):
                halves = [pr.copy_chunk(j, f) for f in (0, 1)]
                out[j] = [(hashlib.sha256(b.tobytes()).hexdigest(), hashlib.sha256(d.tobytes()).hexdigest(), len(d))
                          for b, d in halves]
        st = pr.emit_stats()
        comm.close()
        q.put((rank, res["pairs"], out, st["mine"]))
    except Exception as e:   # noqa: BLE001 - reported to the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc(), None, None))


@pytest.mark.parametrize("world,K", [(2, 4000), (3, 2999), (3, 50_000)])
def test_pair_chunks_multi_rank_on_one_gpu(pair_files, world, K):
    """N processes of the box's one GPU over the host transport: each rank decodes its own chunk
    ranges of R1 and R2 (which do not line up), checks the pairs, and emits the pair chunks that
    start in its R1 range, the records it does not hold moved to it by ppg_comm_alltoallv.  The
    ranks' pair chunks partition [0, chunks) and every half equals the oracle's."""
    import torch.multiprocessing as mp
    gz, chunks, recs, nrec = pair_files
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = f"/ppg_test_{uuid.uuid4().hex[:12]}"
    procs = [ctx.Process(target=_emit_rank, args=(r, world, name, gz, chunks, K, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(60)
    allj = {}
    for rank, pairs, out, mine in got:
        assert out is not None, pairs
        assert pairs == nrec
        assert set(out) == set(range(mine[0], mine[1])), (rank, mine, sorted(out)[:5])
        for j in out:
            assert j not in allj
            allj[j] = out[j]
    npc = -(-nrec // K)
    assert set(allj) == set(range(npc))
    for j, halves in allj.items():
        lo, hi = j * K, min((j + 1) * K, nrec)
        for f in (0, 1):
            eb, ed = expected_half(recs[f][0], lo, hi)
            assert halves[f] == (hashlib.sha256(eb).hexdigest(), hashlib.sha256(ed.tobytes()).hexdigest(), hi - lo), (j, f)


def _maxrss_mb():
    import resource
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024


@pytest.mark.parametrize("form,perturb,guard", [("begin", "short", "emit_next_local"),
                                                ("run", "short", "emit_next_fused"),
                                                ("begin", "bases", "make_segs"),
                                                ("run", "bases", "make_segs")])
def test_no_progress_guards_end_the_emission(pair_files, device, capfd, monkeypatch, form, perturb, guard):
    """VERDICT r05 next #4 (the r05k memory-cap kill: a segment search that found no progress grew
    its list without end).  PPG_PAIRS_PERTURB (a test hook) makes the last output batch one pair chunk
    short of its records ("short": no batch can ever complete the last pair chunks) or leaves the
    segment search without record bases ("bases"); both emission forms must end with PPG_DATA_ERROR,
    promptly and in bounded host memory, at the guard named on stderr -- emit_next_local's "no batch
    completes the pair chunk" (ppg_pairs.hip, after carry_rest), emit_next_fused's "every batch has
    run", make_segs' "no record base"."""
    import time
    gz, chunks, recs, nrec = pair_files
    ix = [pp.Core.BuildDeflateIndex(g, c) for g, c in zip(gz, chunks)]
    cap = 3 << 20   # multi-batch shards: windows cross batches
    if form == "begin":
        sh = [shard_of(g, i, device, cap) for g, i in zip(gz, ix)]
        pr = paired.Pairs()
        assert pr.check(sh[0], sh[1])["mismatches"] == 0
    else:
        sh = []
        for g, i in zip(gz, ix):
            _, i0, _, _ = i.point_fields(0)
            _, i1, _, _ = i.point_fields(i.Count - 1)
            s_ = pp.Shard(i, np.frombuffer(g[i0 - 1:i1], np.uint8), 0, i.Count - 1, device=device, out_capacity=cap)
            paired.attach_keys(s_, 400_000)
            sh.append(s_)
        pr = paired.Pairs()
    assert sh[0].batches >= 3
    monkeypatch.setenv("PPG_PAIRS_PERTURB", perturb)
    rss0, t = _maxrss_mb(), time.time()
    windows = 0
    with pytest.raises(pp.PpgError) as ei:
        # one pair chunk per window (window_bytes=1): a finished file's last window would otherwise
        # reach its last record through the pair count, past the shortened range
        it = pr.emit(sh[0], sh[1], 2500, window_bytes=1) if form == "begin" else \
            pr.emit_run(sh[0], sh[1], 2500, window_bytes=1)
        for _ in it:
            windows += 1
            assert windows < 20
    assert ei.value.code == _lib.PPG_DATA_ERROR
    assert time.time() - t < 60 and _maxrss_mb() - rss0 < 512
    err = capfd.readouterr().err
    assert f"[ppg_pairs] PPG_DATA_ERROR at {guard}" in err, err[-2000:]
    if perturb == "short":
        assert windows >= 1   # the earlier pair chunks were emitted; the last ones cannot be
    # the hook off: the same shards emit every pair chunk again
    monkeypatch.delenv("PPG_PAIRS_PERTURB")
    if form == "run":
        for _ in pr.emit_run(sh[0], sh[1], 2500):
            pass
        assert pr.check(sh[0], sh[1])["pairs"] == nrec
    seen = set()
    for j0, j1 in pr.emit(sh[0], sh[1], 2500):
        check_window(pr, j0, j1, 2500, recs, nrec, seen)
    assert seen == set(range(-(-nrec // 2500)))


@pytest.mark.parametrize("form", ["begin", "run", "carry"])
def test_half_of_4gib_or_more_is_refused(pair_files, device, monkeypatch, form):
    """a pair chunk half's descriptors are u32 positions relative to the half,
    so a half of 4 GiB or more must be refused (PPG_UNSUPPORTED), never wrapped.  PPG_PAIR_HALF_MAX
    (a test hook) lowers the 4 GiB limit to 1 MB so the 30,000-record files reach it: one pair chunk
    of every pair (~11.5 MB per half) is refused in both emission forms, and with multi-batch shards
    the carried first part of a half is refused too; pair chunks under the limit still emit."""
    gz, chunks, recs, nrec = pair_files
    ix = [pp.Core.BuildDeflateIndex(g, c) for g, c in zip(gz, chunks)]
    cap = (3 << 20) if form == "carry" else 0
    monkeypatch.setenv("PPG_PAIR_HALF_MAX", str(1 << 20))
    if form == "run":
        sh = []
        for g, i in zip(gz, ix):
            _, i0, _, _ = i.point_fields(0)
            _, i1, _, _ = i.point_fields(i.Count - 1)
            s_ = pp.Shard(i, np.frombuffer(g[i0 - 1:i1], np.uint8), 0, i.Count - 1, device=device)
            paired.attach_keys(s_, 400_000)
            sh.append(s_)
        pr = paired.Pairs()
        it = pr.emit_run(sh[0], sh[1], 10 * nrec)
    else:
        sh = [shard_of(g, i, device, cap) for g, i in zip(gz, ix)]
        pr = paired.Pairs()
        pr.check(sh[0], sh[1])
        it = pr.emit(sh[0], sh[1], 10 * nrec)
    with pytest.raises(pp.PpgError) as ei:
        next(it)
    assert ei.value.code == _lib.PPG_UNSUPPORTED
    # ~2,700 records (~1 MB) per half fit the lowered limit
    if form != "run":
        seen = set()
        for j0, j1 in pr.emit(sh[0], sh[1], 2000):
            check_window(pr, j0, j1, 2000, recs, nrec, seen)
        assert seen == set(range(-(-nrec // 2000)))

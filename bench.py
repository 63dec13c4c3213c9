"""bench.py — DecompressAll (BatchedFASTQ.Count()) on MI355X: FASTQ records/s + decompressed MB/s.

Workload (BASELINE.json configs[2], the config the metric is quoted on): a ~50 GB synthetic
single-member .fastq.gz of 150 bp Generator-shape reads (~530 M records, ~205 GB decompressed),
chunk = 10,000 records.  The member is "tiled" (parallelparsing_amd/tiled.py): one ~1 GB-text
segment deflated once (zlib level 6, pigz-style pieces) and repeated inside one member, so it can
be built on the box in seconds; its CreateIndex points are derived exactly (tests/test_tiled.py).
The compressed bytes and the index (windows + offsets) are resident in HBM before timing; the
timed step is one DecompressAll pass over every chunk of this rank's shard: HIP inflate +
FASTQ record scan + descriptor emission, plus the all-gather of per-chunk record counts when
N > 1.  Decompressed output streams through a reused device buffer (out_capacity), as a
consumer enumerating records would.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload 50gb|1m]
  N > 1: one process per GPU, backend nccl = RCCL.  Under torch.distributed.run (WORLD_SIZE set)
  this process is one rank; started directly with --gpus N > 1 it launches the N ranks itself
  (torch.distributed.run as a child, before anything touches the GPU) and exits with its code.
  N > 1 defaults to strong scaling: one ~50 GB member split over the N GPUs (configs[3]).
"""
import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SEG_RECORDS = 10_485_760     # default 50 GB workload: a ~4 GB-text segment ...
REPEATS = 51                 # ... repeated 51 times in one member (~50 GB of gzip)
PAIRED_SEG_RECORDS = 2_621_440
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
REFERENCE_REC_S = 1.217e6  # Plots/csv_original/parallel_10k_false.csv:8 (Arm64, published; not this metric)


def log(*a):
    sys.stderr.write(" ".join(map(str, a)) + "\n")   # one write: ranks' lines do not interleave mid-line
    sys.stderr.flush()


def free_bytes(path):
    """Bytes an unprivileged writer can still put under `path` (statvfs f_bavail), or -1."""
    try:
        st = os.statvfs(path)
        return st.f_bavail * st.f_frsize
    except OSError:
        return -1


def share_dir(preferred, need):
    """Where local rank 0 publishes the input member for the other ranks: `preferred` (--shm-dir,
    /dev/shm by default) when it has room for `need` bytes plus 10% and 1 GiB, else the first of
    $TMPDIR, /tmp, /var/tmp that has (disk-backed: the ranks memory-map it from the page cache).
    VERDICT r04: /dev/shm on the 8-GPU node may be smaller than the ~5 GB the 50 GB member's
    description takes, and configs[3]'s first run would fail in setup.  Returns (dir, note)."""
    want = int(need * 1.1) + (1 << 30)
    cands = [preferred] + [d for d in (os.environ.get("TMPDIR"), "/tmp", "/var/tmp") if d and d != preferred]
    for d in cands:
        if os.path.isdir(d) and os.access(d, os.W_OK) and free_bytes(d) >= want:
            return d, (None if d == preferred else
                       f"{preferred} has {free_bytes(preferred) / 2**30:.1f} GiB free, {want / 2**30:.1f} GiB needed: "
                       f"fell back to {d}")
    raise OSError(f"no directory among {cands} has {want / 2**30:.1f} GiB free for the shared input "
                  f"({', '.join(f'{d}: {free_bytes(d) / 2**30:.1f} GiB' for d in cands)})")


def shared_tiled(args, key, build, need):
    """The synthetic member, built once per node: at N = 1 in this process; at N > 1 local rank 0
    builds it and saves it under /dev/shm (TiledFile.save), the other ranks memory-map that copy
    (TiledFile.load) instead of each rebuilding the ~4 GB text segment and deflating it (22 s and
    ~5 GB of host RAM per rank).  `need`: the bytes the save takes (checked
    against the directory's free space first: share_dir).  Returns (TiledFile, seconds, how)."""
    from parallelparsing_amd.tiled import TiledFile
    t = time.time()
    if args.world == 1:
        return build(), time.time() - t, "built"
    # a name no earlier (crashed) run can have left behind: a nonce from rank 0, broadcast (ADVICE
    # r03: a stale 'ready' of a deterministic name let ranks map files being rewritten); rank 0
    # also picks the directory (free space), so every rank looks in the same place
    import hashlib
    import uuid
    import torch.distributed as dist
    pick = [None, None, None]
    if dist.get_rank() == 0:
        try:
            pick = [uuid.uuid4().hex, *share_dir(args.shm_dir, need)]
        except OSError as e:
            pick = [None, None, str(e)]
    dist.broadcast_object_list(pick, 0)
    nonce, base, note = pick
    if nonce is None:
        raise OSError(note)
    if note:
        log(f"[bench] {note}")
    args.share_note = note
    d = os.path.join(base, "ppg_bench_" + hashlib.sha1(repr((nonce, key)).encode()).hexdigest()[:12])
    args.shm_paths.append(d)
    failed = os.path.join(d, "failed")
    if args.local_rank == 0:
        try:
            if setup_fault("input", args.rank):
                raise RuntimeError("injected input failure (PPG_BENCH_FAIL)")
            tf = build()
            tf.save(d)
        except Exception as e:
            # the other local ranks wait for "ready": tell them instead (they would wait 30 min)
            try:
                os.makedirs(d, exist_ok=True)
                with open(failed, "w") as f:
                    f.write(f"{type(e).__name__}: {e}")
            except OSError:
                pass
            raise
        return tf, time.time() - t, f"built (shared via {d})"
    ready = os.path.join(d, "ready")
    while not os.path.exists(ready):
        if os.path.exists(failed):
            with open(failed) as f:
                raise RuntimeError(f"local rank 0 failed to build the input: {f.read()}")
        if time.time() - t > 1800:
            raise TimeoutError(f"local rank 0 did not publish {d}")
        time.sleep(0.2)
    return TiledFile.load(d), time.time() - t, f"memory-mapped from {d}"


def gather_vec(vals, dist_on, xdev):
    """[vals of rank 0, vals of rank 1, ...] (floats) -- one all_gather (flat output: gloo wants it)."""
    import torch
    v = torch.tensor([float(x) for x in vals], dtype=torch.float64, device=xdev)
    if not dist_on:
        return [v.tolist()]
    import torch.distributed as dist
    world = dist.get_world_size()
    out = torch.zeros(world * v.numel(), dtype=torch.float64, device=xdev)
    dist.all_gather_into_tensor(out, v)
    return out.view(world, v.numel()).cpu().tolist()


def gather_pairs(x, y, dist_on, xdev):
    """[(x, y) of rank 0, (x, y) of rank 1, ...]."""
    return gather_vec([x, y], dist_on, xdev)


class SetupFailed(RuntimeError):
    """A rank's setup failed; every rank raises this with the failing ranks' messages (agree_setup)."""


MSG_BYTES = 480


def agree_setup(stage, err, dist_on, xdev):
    """Setup status agreed across ranks before the next collective:
    each rank's error (or None) from `stage` -- the input member, its shard (compressed range resident,
    Shard, set_split), the communicator -- is all-gathered as a status + a fixed-size message, and if
    any rank failed EVERY rank raises SetupFailed naming the failing ranks and the first one's message.
    Without it a rank that failed setup left its peers inside the next collective: gloo's TCP teardown
    ended the full-size world-8 rehearsal with "Connection closed by peer" on the surviving ranks
    (gpurun_out/r05zzh/w8.log), and under RCCL they would wait until torchrun's agent killed them.
    The reference's fan-out has no such step (BatchedFASTQ.cs:62-77: one process, Task.Run per chunk)."""
    if not dist_on:
        if err is not None:
            raise err
        return
    import torch
    import torch.distributed as dist
    msg = b"" if err is None else f"{type(err).__name__}: {err}".encode(errors="replace")[:MSG_BYTES - 1]
    v = torch.zeros(MSG_BYTES, dtype=torch.uint8)
    v[0] = 0 if err is None else 1
    if msg:
        v[1:1 + len(msg)] = torch.frombuffer(bytearray(msg), dtype=torch.uint8)
    world = dist.get_world_size()
    out = torch.zeros(world * MSG_BYTES, dtype=torch.uint8, device=xdev)
    dist.all_gather_into_tensor(out, v.to(xdev))
    rows = out.view(world, MSG_BYTES).cpu().numpy()
    bad = [r for r in range(world) if rows[r, 0]]
    if not bad:
        return
    first = bytes(rows[bad[0], 1:]).rstrip(b"\0").decode(errors="replace")
    raise SetupFailed(f"setup failed at '{stage}' on rank(s) {bad} of {world}; rank {bad[0]}: {first}")


def setup_fault(stage, rank):
    """Test hook (tests only, never set by the driver): PPG_BENCH_FAIL="<stage>@<rank>" makes that
    rank's setup fail at that stage -- input, shard, set_split (a real library error: side points
    outside their chunks) or comm."""
    v = os.environ.get("PPG_BENCH_FAIL", "")
    return bool(v) and v == f"{stage}@{rank}"


def drop_shared(args):
    """After every rank has loaded it (a barrier): local rank 0 removes the /dev/shm copy (the
    ranks' mappings stay valid)."""
    import shutil
    if args.local_rank == 0:
        for d in args.shm_paths:
            shutil.rmtree(d, ignore_errors=True)


def build_input(args):
    from parallelparsing_amd.tiled import TiledFile
    if args.workload == "50gb":
        # weak scaling: the member holds `repeats` segments per rank (~50 GB of gzip per GPU)
        # weak (default): ~50 GB of gzip per GPU; strong: one ~50 GB member split over the GPUs
        # (BASELINE configs[3] literally)
        reps = args.repeats * (args.world if args.scaling == "weak" else 1)
        key = ("50gb", args.seg_records, reps, args.chunk, args.blank_lines)
        build = lambda: TiledFile(args.seg_records, reps, args.chunk, threads=args.host_threads,   # noqa: E731
                                  blank_lines=args.blank_lines)
    else:  # 1m: configs[1], one non-repeated 1 M-read member
        key = ("1m", args.chunk)
        build = lambda: TiledFile(1_000_000, 1, args.chunk, threads=args.host_threads)   # noqa: E731
    from parallelparsing_amd.tiled import saved_bytes_estimate
    recs = args.seg_records if args.workload == "50gb" else 1_000_000
    tf, sec, how = shared_tiled(args, key, build, saved_bytes_estimate(recs, blank_lines=args.blank_lines))
    args.input_seconds, args.input_how = sec, how
    log(f"[bench] input: {tf.records * tf.repeats:,} records, {tf.text_len * tf.repeats / 1e9:.1f} GB text, "
        f"{tf.file_len / 1e9:.2f} GB gz, {tf.npoints - 1} chunks, {how} in {sec:.1f}s")
    return tf


def host_cpu_info():
    """What the CPU baseline ran on: nproc, the scheduler affinity, the cgroup quota, the model."""
    info = {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            info["cgroup_cpu_quota"] = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        info["cgroup_cpu_quota"] = None
    try:
        with open("/proc/cpuinfo") as f:
            info["model"] = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), None)
    except OSError:
        info["model"] = None
    return info


def usable_cpus():
    """Host cores this process can actually run on: the scheduler affinity, capped by the cgroup
    CPU quota (the GPU box shows 256 CPUs but grants a 16-CPU quota: 256 threads there measured
    slower than 16, r02).  BASELINE.md §2's T = all host cores; nproc is reported beside it and
    timed as a variant."""
    info = host_cpu_info()
    n = info["affinity"] or 1
    if info["cgroup_cpu_quota"]:
        n = min(n, max(1, int(round(info["cgroup_cpu_quota"]))))
    return n


def _timed(fn, warm, runs):
    """BASELINE.md §2 protocol: `warm` untimed runs, then the median of `runs` timed ones."""
    for _ in range(warm):
        fn()
    ts, res = [], None
    for _ in range(runs):
        t = time.perf_counter()
        res = fn()
        ts.append(time.perf_counter() - t)
    return res, statistics.median(ts), ts


def cpu_baseline(tf, ix_out, ix_in, nchunks, threads):
    """The oracle's threaded DecompressAll (C restatement of BatchedFASTQ over zlib 1.2.11) on a
    bounded prefix of the same file, timed on this host (rank 0, N = 1 only): T = every host core
    (usable_cpus()), 2 warm-ups + the median of 5, plus one thread, nproc threads and the
    C#-shaped consumer that materialises every record as FastqRecord does (median of 3 each)."""
    from oracle import oracle as O
    sample = min(nchunks, int(os.environ.get("PPG_CPU_SAMPLE_CHUNKS", "4096")))
    hi = int(ix_in[sample])
    gz = tf.file_bytes(0, hi)
    win, offs = tf.windows(0, sample + 1)
    oi = O.index_from_points(tf.p_output[: sample + 1], tf.p_input[: sample + 1], tf.p_bits[: sample + 1],
                             win, tf.p_offlen[: sample + 1], offs)
    (recs, _), dt, ts = _timed(lambda: O.decompress_all(gz, oi, threads=threads, first=0, last=sample), 2, 5)
    out_bytes = int(ix_out[sample] - ix_out[0])
    # SURVEY 8d variants: one thread, and the C#-shaped consumer that materialises every record
    # into its own buffer as FastqRecord does (Parsing.cs:41-47, mode 1), on smaller prefixes
    variants = {}
    nproc = min(512, os.cpu_count() or 1)   # capped for the box's process/thread limit
    runs = [("1 thread", 1, 0, min(sample, 128)),
            (f"{threads} threads, records materialised", threads, 1, min(sample, 2048))]
    if nproc != threads:
        runs.append((f"{nproc} threads (= nproc, over the {threads}-CPU quota)", nproc, 0, sample))
    for name, th, mode, n in runs:
        (r1, _), d1, _ = _timed(lambda: O.decompress_all(gz, oi, threads=th, mode=mode, first=0, last=n), 1, 3)
        variants[name] = {"records_per_s": r1 / d1, "cores": th, "chunks": n, "seconds_median": d1}
    return {"value": recs / dt, "unit": "records/s", "cores": threads, "kind": "port",
            "sample": f"first {sample} of {nchunks} chunks ({recs:,} records, {out_bytes / 1e9:.2f} GB out) "
                      f"of the same file, {threads} threads (every usable host core: affinity and cgroup quota), median "
                      f"of 5 after 2 warm-ups: "
                      f"{dt:.2f} s",
            "runs_s": [round(t, 3) for t in ts], "host": host_cpu_info(),
            "decompressed_MBps": out_bytes / dt / 1e6, "variants": variants}


def pmc_traffic(workload, build, path=None):
    """HBM bytes per inflate launch from the committed rocprofv3 PMC passes of this same command
    (profiles/traffic.json, written by tools/profile_round.sh + tools/traffic_summary.py), or None.
    The file names the workload and the library build it measured (ppg_version + ppg_build_id, a
    hash of the inflate object): counters of another build or workload are never quoted."""
    path = path or os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    if t.get("workload") != workload or t.get("build") != build:
        return None
    return t.get("hbm_bytes_per_launch")


def issue_roofline(build, path=None):
    """The inflate kernel's issue-side bounds from the committed rocprofv3 stall passes of this same
    build (profiles/inflate_stalls.json, tools/pmc_stalls.sh + tools/stall_summary.py; pinned to
    ppg_version + ppg_build_id as traffic.json is), or None: SALU instructions per CU-cycle (the CU's
    one scalar unit issues at most one per cycle), the VALU pipe's busy share (a wave64 VALU op
    occupies a SIMD-32 for two cycles, MI355X_MICROARCH.md), and the wave-cycle split."""
    path = path or os.path.join(ROOT, "profiles", "inflate_stalls.json")
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    if t.get("build") != build:
        return None
    c = t["counters"]
    cyc = c["GRBM_GUI_ACTIVE"] / 8          # GRBM_GUI_ACTIVE sums the 8 XCDs
    cus, simds = 256, 1024
    return {"salu_per_cu_cycle": c["SQ_INSTS_SALU"] / (cus * cyc), "salu_peak_per_cu_cycle": 1.0,
            "valu_busy": 2 * c["SQ_INSTS_VALU"] / (simds * cyc),
            "wave_cycles": t.get("wave_cycle_split"), "source": os.path.relpath(path, ROOT),
            "workload": t.get("workload")}


def pcie_d2h_GBps(dev, gib=4, h2d=False):
    """Device -> pinned host copy rate of this box (the bound of any leg that lands decompressed
    text in host memory), or with h2d pinned host -> device (the bound of the ingest leg, whose
    compressed bytes cross that way): one 4 GiB hipMemcpy, best of three."""
    import torch
    n = gib << 30
    d = torch.empty(n, dtype=torch.uint8, device=dev)
    h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    best = 0.0
    for _ in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        if h2d:
            d.copy_(h, non_blocking=True)
        else:
            h.copy_(d, non_blocking=True)
        torch.cuda.synchronize()
        best = max(best, n / (time.perf_counter() - t) / 1e9)
    del d, h
    return best


def enumerate_run(tf, ix, path, dev, threads, batch_gib, pcie):
    """BatchedFASTQ's enumerator through the C ABI (ppg_cursor, BatchedFASTQ.cs:54-98): every
    record's raw bytes (offset_k ++ chunk_k) and descriptor landed in pinned host memory, batch by
    batch, from the .gz file in page cache.  PCIe-bound: ~385 B of text per
    record cross device -> host."""
    import parallelparsing_amd as pp
    t0 = time.perf_counter()
    cur = pp.Cursor(ix, path, batch_bytes=int(batch_gib * (1 << 30)), threads=threads, device=dev)
    t_open = time.perf_counter() - t0
    nrec = text = nb = 0
    t1 = time.perf_counter()
    for b in cur:
        nrec += b.nrecords
        text += int(b.raw_off[-1])
        nb += 1
    sec = time.perf_counter() - t1
    cur.close()
    assert nrec == tf.expected_records(), (nrec, tf.expected_records())
    host_bytes = text + 16 * nrec
    bound = pcie * 1e9 / (host_bytes / nrec)
    return {"records_per_s": nrec / sec, "records_per_s_incl_open": nrec / (sec + t_open), "seconds": sec,
            "open_s": t_open, "batches": nb, "batch_GiB": batch_gib, "host_GBps": host_bytes / sec / 1e9,
            "pcie_d2h_GBps": pcie, "pcie_bound_records_per_s": bound, "frac_of_pcie_bound": nrec / sec / bound,
            "note": "ppg_cursor: pread -> pinned -> H2D -> decode -> device pack -> one D2H of raw text + "
                    "descriptors per batch, 4 batches in flight in stage order (own stream + worker thread each), "
                    "buffers sized once at open; records counted, not materialised as objects; not the bench "
                    "value"}


def ingest_run(tf, ix, dev, threads, piece_gib=8.0, enum_gib=0.0):
    """Host-ingest path (ppg_file_decompress_all): the same member written to $TMPDIR as a real
    file, streamed from page cache through pinned buffers, PCIe and the kernels.  With enum_gib > 0
    the enumerator leg (enumerate_run) reads the same file afterwards."""
    import parallelparsing_amd as pp
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"ppg_ingest_{os.getpid()}.fastq.gz")
    try:
        t = time.perf_counter()
        with open(path, "wb") as f:
            for lo in range(0, tf.file_len, 1 << 30):
                f.write(tf.file_bytes(lo, min(tf.file_len, lo + (1 << 30))))
        wt = time.perf_counter() - t
        pb = int(piece_gib * (1 << 30))
        pp.decompress_file(ix, path, device=dev, threads=threads, piece_bytes=pb)   # warm: buffers, page cache
        _, tot, sec = pp.decompress_file(ix, path, device=dev, threads=threads, piece_bytes=pb)
        assert tot == tf.expected_records(), (tot, tf.expected_records())
        import torch
        h2d = pcie_d2h_GBps(torch.device("cuda", dev.device), h2d=True)
        out = {"records_per_s": tot / sec, "compressed_GBps": tf.file_len / sec / 1e9,
               "pcie_h2d_GBps": h2d, "frac_of_pcie_bound": tf.file_len / sec / 1e9 / h2d,
               "decompressed_GBps": tf.text_len * tf.repeats / sec / 1e9, "seconds": sec,
               "file_GB": tf.file_len / 1e9, "write_s": wt,
               "note": f"file in page cache -> pread ({threads} threads) -> pinned -> H2D -> decode, {piece_gib:g} GiB "
                       "pieces (three device slots, per-slot streams: a piece's decode overlaps the previous one's "
                       "tail); PCIe-inclusive, not the bench value"}
        enum = None
        if enum_gib > 0:
            try:
                import torch
                pcie = pcie_d2h_GBps(torch.device("cuda", dev.device))
                enum = enumerate_run(tf, ix, path, dev, threads, enum_gib, pcie)
            except (OSError, AssertionError, RuntimeError) as e:
                enum = {"error": f"{type(e).__name__}: {e}"}
        return out, enum
    finally:
        if os.path.exists(path):
            os.remove(path)


def ingest_pieces(args, tf, a, b, slots):
    """(piece_bytes, waves per chunk) for a rank's end-to-end leg over chunks [a, b): about four
    pieces per rank (<= --ingest-piece-gib), so the read of piece k+1 overlaps the decode of piece k
    even for an N = 8 rank's ~6 GB; chunks split at side points (<= 16 waves) into enough waves for
    ~1.5 generations per piece, as the resident split does for a small rank."""
    rng = int(tf.p_input[b] - tf.p_input[a]) + 1
    pb = int(min(args.ingest_piece_gib * (1 << 30), max(1 << 30, rng / 4)))
    per_piece = max(1, (b - a) * pb // max(1, rng))
    return pb, int(min(16, max(1, -(-3 * slots // (2 * per_piece)))))


def dist_ingest_run(tf, args, ctx, a, b, rank, world, dist_on, xdev):
    """The N > 1 end-to-end leg (and a --share rehearsal's): local rank 0 writes the member to a
    file once (the directory with room for it: share_dir), every rank streams its own chunk range
    [a, b) from it -- pread into pinned buffers, H2D, decode, piece by piece (ppg_file_decompress_all,
    the role of LazyFileReader.cs:41-97 feeding BatchedFASTQ.cs:62-77's tasks) -- one untimed run, a
    barrier, the timed run; the per-rank seconds and record totals are gathered and the records
    checked exactly.  Every decision and failure is agreed across ranks, so no rank is left in a
    collective.  Never the bench value."""
    import torch
    import parallelparsing_amd as pp
    pick = [None, None]
    if rank == 0:
        try:
            base, note = share_dir(os.environ.get("TMPDIR") or "/tmp", tf.file_len)
            pick = [os.path.join(base, f"ppg_e2e_{os.getpid()}_{int(time.time())}.fastq.gz"), note]
        except OSError as e:
            pick = [None, str(e)]
    if dist_on:
        import torch.distributed as dist
        dist.broadcast_object_list(pick, 0)
    path, note = pick
    if path is None:
        return {"error": f"no room for the {tf.file_len / 1e9:.1f} GB file: {note}"}
    err, wt = None, 0.0
    if args.local_rank == 0:
        try:
            t = time.perf_counter()
            with open(path, "wb") as f:
                for lo in range(0, tf.file_len, 1 << 30):
                    f.write(tf.file_bytes(lo, min(tf.file_len, lo + (1 << 30))))
            wt = time.perf_counter() - t
        except OSError as e:
            err = e
    try:
        try:
            agree_setup("e2e file", err, dist_on, xdev)
        except (SetupFailed, OSError) as e:
            return {"error": str(e)}
        pb, waves = ingest_pieces(args, tf, a, b, wave_slots(torch.device("cuda", ctx.device)))
        status, sec, recs = 0.0, 0.0, 0
        try:
            ix = tf.index(a, b + 1)
            if waves > 1:
                ix.set_side_points(*tf.side_points(a, b + 1, waves))
            pp.decompress_file(ix, path, 0, b - a, piece_bytes=pb, threads=args.host_threads, device=ctx)  # warm
            if dist_on:
                dist.barrier()
            _, recs, sec = pp.decompress_file(ix, path, 0, b - a, piece_bytes=pb, threads=args.host_threads,
                                              device=ctx)
        except Exception as e:   # noqa: BLE001 - every rank still joins the gather below
            status = 1.0
            log(f"[bench] rank {rank}: end-to-end leg failed: {type(e).__name__}: {e}")
        finally:
            ctx.release_file_buffers()
        rows = gather_vec([status, sec, recs, b - a, int(tf.p_input[b] - tf.p_input[a]) + 1], dist_on, xdev)
        if any(r[0] for r in rows):
            return {"error": f"ppg_file_decompress_all failed on rank(s) {[i for i, r in enumerate(rows) if r[0]]}"}
        total = int(sum(r[2] for r in rows))
        smax = max(r[1] for r in rows)
        exact = args.share > 1 or total == tf.expected_records()
        assert exact, ("end-to-end records", total, tf.expected_records())
        gz = sum(r[4] for r in rows)
        return {"records_per_s": total / smax, "compressed_GBps": gz / smax / 1e9,
                "decompressed_GBps": (tf.text_len * tf.repeats if args.share == 1 else
                                      int(tf.p_output[b] - tf.p_output[a])) / smax / 1e9,
                "seconds_max_over_ranks": smax, "records": total,
                "per_rank": [{"rank": i, "seconds": round(r[1], 4), "records": int(r[2]), "chunks": int(r[3]),
                              "gz_GB": round(r[4] / 1e9, 3), "compressed_GBps": round(r[4] / max(r[1], 1e-9) / 1e9, 2)}
                             for i, r in enumerate(rows)],
                "piece_GiB": round(pb / (1 << 30), 3), "waves_per_chunk": f"<= {waves} (side points)",
                "file_GB": tf.file_len / 1e9, "write_s": wt, **({"dir_note": note} if note else {}),
                "note": "every rank: its chunk range of the file (page cache) -> pread -> pinned -> H2D -> decode, "
                        "piece by piece (ppg_file_decompress_all, three device slots); one untimed run, a barrier, "
                        "then the timed run; records exact over all ranks; PCIe-inclusive, not the bench value"
                        + ("; --share rehearsal: rank 0's range alone" if args.share > 1 else "")}
    finally:
        if dist_on:
            dist.barrier()
        if args.local_rank == 0 and os.path.exists(path):
            os.remove(path)


def decompress_chunk_run(tf, dev, counts, threads_list=(1, 8, 64), per_thread=16, max_chunks=1024, side=16):
    """README "Decompress" (ppg_decompress_chunk, thread safe): T host threads calling it on one ctx,
    each for its own chunk at a time, as the reference's one task per chunk does
    (BatchedFASTQ.cs:62-77).  Slices from host memory, bytes + descriptors back into host buffers;
    the per-chunk record counts are checked against the timed DecompressAll run's.  Three ways: the
    plain index (launches of <= 256 chunks find each chunk's inner block starts on the GPU and decode
    it as up to 16 waves), the same with that search off (PPG_CHUNK_NO_FIND: one wave per chunk), and
    with the index's own side points attached (up to `side` waves per chunk)."""
    import threading
    import parallelparsing_amd as pp
    nmax = min(max_chunks, len(counts), per_thread * max(threads_list))
    slices = [np.frombuffer(tf.file_bytes(int(tf.p_input[k]) - 1, int(tf.p_input[k + 1])), np.uint8)
              for k in range(nmax)]
    plain = tf.index(0, nmax + 1)
    split = tf.index(0, nmax + 1).set_side_points(*tf.side_points(0, nmax + 1, side))

    def leg(ix, T, runs=1):
        """T threads (one untimed run first and the median of `runs` when runs > 1: HBM freed just
        before the legs -- the ingest's pieces, the shard -- is cleared by the driver for seconds
        after, and the clearing shares the copy engines with the launches' H2D/D2H; r05: one T = 64
        run read 23 M records/s there, 36-42 M in other runs)."""
        if runs > 1:
            leg(ix, T)
            return sorted((leg(ix, T) for _ in range(runs)), key=lambda r: r["records_per_s"])[runs // 2]
        n = min(nmax, per_thread * T)
        before = dev.decompress_chunk_stats()
        nxt = [0]
        lock = threading.Lock()
        got = np.zeros(n, np.int64)
        errs = []

        def work():
            try:
                while True:
                    with lock:
                        k = nxt[0]
                        nxt[0] += 1
                    if k >= n:
                        return
                    _, _, rec = pp.Core.ExtractDeflateIndex(slices[k], ix, k, device=dev, with_records=True)
                    got[k] = len(rec)
            except Exception as e:   # noqa: BLE001 - re-raised below
                errs.append(e)
        th = [threading.Thread(target=work) for _ in range(T)]
        t = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        sec = time.perf_counter() - t
        if errs:
            raise errs[0]
        assert (got == counts[:n]).all(), "ppg_decompress_chunk record counts differ from DecompressAll's"
        after = dev.decompress_chunk_stats()
        calls, launches = after["calls"] - before["calls"], after["launches"] - before["launches"]
        return {"chunks": n, "records_per_s": float(got.sum()) / sec, "chunks_per_s": n / sec,
                "ms_per_call": sec * 1e3 * T / n, "seconds": sec, "launches": launches,
                "chunks_per_launch": calls / max(1, launches),
                "split_chunks": after["split_chunks"] - before["split_chunks"],
                "found_side_points": after["side_points"] - before["side_points"]}

    def no_find(T):
        os.environ["PPG_CHUNK_NO_FIND"] = "1"
        try:
            return leg(plain, T)
        finally:
            os.environ.pop("PPG_CHUNK_NO_FIND", None)

    def async_once(ix, depth):
        n = min(nmax, depth)
        before = dev.decompress_chunk_stats()
        t = time.perf_counter()
        futs = [pp.Core.ExtractDeflateIndexAsync(slices[k], ix, k, device=dev) for k in range(n)]
        got = np.array([len(f.result()[2]) for f in futs], np.int64)
        sec = time.perf_counter() - t
        assert (got == counts[:n]).all(), "ppg_decompress_chunk_submit record counts differ from DecompressAll's"
        after = dev.decompress_chunk_stats()
        return {"chunks": n, "records_per_s": float(got.sum()) / sec, "chunks_per_s": n / sec, "seconds": sec,
                "launches": after["launches"] - before["launches"]}

    def async_leg(ix, depth):
        """One caller thread queues `depth` chunks (ppg_decompress_chunk_submit) and then takes the
        results in order (ppg_decompress_chunk_wait): one untimed run, then the median of 3 (a launch
        slot first used grows its block-search scratch by GBs, hipFree + hipMalloc; r05: a slot first
        used inside the timed depth-1024 run took 3.85 s there)."""
        async_once(ix, depth)
        runs = sorted((async_once(ix, depth) for _ in range(3)), key=lambda r: r["records_per_s"])
        return runs[1]

    # warm: the launcher thread, and the launch slots' buffers grown to full launches (256 chunks each)
    async_once(plain, nmax)
    leg(plain, 8)
    out = {f"T{T}": leg(plain, T, runs=3) for T in threads_list}
    out["async"] = {f"depth{d}": async_leg(plain, d) for d in (256, 1024)}
    out["no_find"] = {f"T{T}": no_find(T) for T in threads_list}
    out["side_points"] = {f"T{T}": leg(split, T) for T in threads_list}
    out["note"] = ("ppg_decompress_chunk from T host threads on one ctx (concurrent calls combined into shared "
                   "launches, four launch slots); async: one thread queues `depth` chunks (ppg_decompress_chunk_submit) "
                   "then waits for each; plain index and async: median of 3 after an untimed run; plain index: each chunk's inner block starts found on the GPU "
                   "(<= 16 waves per chunk); no_find: one wave per chunk; side_points: the index's own, "
                   f"<= {side} waves per chunk (ppg_index_set_side_points); host slices in, bytes + descriptors out; "
                   "not the bench value")
    return out


def create_index_run(tf, args, dev):
    """GPU CreateIndex (ppg_index_build_gpu) over the whole member resident in HBM, checked Point by
    Point against the member's exactly derived index, beside the host zlib CreateIndex (the
    reference's algorithm, IndexBuilder) timed on one segment of the same data."""
    import torch
    import parallelparsing_amd as pp
    from parallelparsing_amd.tiled import TiledFile
    gz = torch.empty(tf.file_len + 256, dtype=torch.uint8, device=dev)
    gz[tf.file_len:].zero_()
    tf.fill_device(gz, 0, tf.file_len)
    torch.cuda.synchronize()
    g = gz[: tf.file_len]
    runs, phases = [], []
    ix = None
    for _ in range(2):                                             # first run: allocation warm-up
        ix = None
        t = time.perf_counter()
        ix = pp.Core.BuildDeflateIndexGpu(g, args.chunk, out_capacity=int(args.ix_capacity_gib * (1 << 30)),
                                          piece_bytes=int(args.ix_piece_kib * 1024))
        runs.append(time.perf_counter() - t)
        st = pp.Core.gpu_index_stats()
        phases.append({k: round(st[k], 1) for k in ("finder_ms", "pass1_ms", "chain_ms", "resolve_ms", "pass2_ms",
                                                    "pass2_alloc_ms", "census_ms")})
        log(f"[bench] GPU CreateIndex: {runs[-1]:.2f} s, {ix.Count} points, phases {phases[-1]}")
    del gz, g
    torch.cuda.empty_cache()
    out, inp, bits = ix.arrays()
    ok = (ix.Count == tf.npoints and (out == tf.p_output).all() and (inp == tf.p_input).all()
          and (bits == tf.p_bits).all())
    if ok:
        win, offs = tf.windows(0, tf.npoints)
        ok = bool(np.array_equal(ix.windows_array(), win))
        o = 0
        for i in range(tf.npoints):
            n = int(tf.p_offlen[i])
            ok = ok and ix[i].offset == offs[o:o + n].tobytes() if n else ok and ix.point_fields(i)[3] == 0
            o += n
    assert ok, "GPU CreateIndex differs from the member's index"
    log("[bench] GPU CreateIndex verified against the member's index")
    sec = runs[-1]
    text = tf.text_len * tf.repeats
    # host CreateIndex (serial zlib Z_BLOCK pass) on a one-segment member of the same data
    one = TiledFile(args.seg_records, 1, args.chunk, threads=args.host_threads)
    one_gz = one.file_bytes(0, one.file_len)
    t = time.perf_counter()
    cix = pp.Core.BuildDeflateIndex(one_gz, args.chunk)
    csec = time.perf_counter() - t
    assert cix.Count == one.npoints
    cpu_gbs = one.text_len / csec / 1e9
    return {"seconds": sec, "first_run_s": runs[0], "phases_ms_per_run": phases, "points": ix.Count,
            "gz_GBps": tf.file_len / sec / 1e9,
            "decompressed_GBps": text / sec / 1e9,
            "phases_ms": {k: round(st[k], 2) for k in ("finder_ms", "pass1_ms", "chain_ms", "resolve_ms", "pass2_ms", "pass2_alloc_ms",
                                                       "census_ms")},
            "pieces": int(st["pieces"]), "real_pieces": int(st["real_pieces"]), "redo1": int(st["redo1"]),
            "spec_redos": int(st["spec_redos"]), "serial_redos": int(st["serial_redos"]),
            "pass2_batches": int(st["batches"]),
            "pass2_capacity": f"{args.ix_capacity_gib:g} GiB" if args.ix_capacity_gib else "default (96 GiB or free HBM - 4 GiB)",
            "blocks": int(st["blocks"]), "verified": "every Point (Output, Input, Bits, Window, offset) of the member",
            "cpu_reference": {"seconds": csec, "decompressed_GBps": cpu_gbs, "cores": 1,
                              "sample": f"host zlib CreateIndex (Core.cs:14-131 restated) of a 1-segment member "
                                        f"({one.file_len / 1e9:.2f} GB gz, {one.npoints} points)",
                              "projected_seconds_full_member": text / 1e9 / cpu_gbs}}


def paired_run(args, dev, world=1, rank=0, xdev=None, backend="nccl"):
    """BASELINE configs[4]-shaped paired-end run: two tiled members (R1 / R2 of a read pair: equal
    spot numbers, different SRR ids and bases), chunk = 50,000, both decoded and resident, every
    record's spot key extracted on the GPU, Q1 duplicates dropped and the pair invariant checked
    (paired.PairedFASTQ's path).  On N ranks each rank decodes its contiguous chunk range of BOTH
    files (dist.partition_chunks per file); the files' record ranges do not line up across ranks,
    so the pair check is a real exchange: ppg_pairs_check (C ABI) all-gathers the counts and moves
    every spot key to the rank owning its pair number (ppg_comm_alltoallv: RCCL ncclSend/ncclRecv
    over xGMI; the host transport in the one-GPU rehearsal).  Size per
    file: --paired-repeats segments (default 102: configs[4]'s ~25 GB of gzip per file at any N).
    The spot keys are extracted per output batch while it is resident (ppg_shard_set_keys), so a
    rank's range may decode in several batches of --paired-out-gib: on one GPU the two ~103 GB
    outputs never need to be resident together."""
    import torch
    import parallelparsing_amd as pp
    from parallelparsing_amd import paired
    from parallelparsing_amd.dist import partition_chunks
    from parallelparsing_amd.tiled import TiledFile
    reps = args.paired_repeats or 102
    t = time.time()
    from parallelparsing_amd.tiled import saved_bytes_estimate
    tfs = [shared_tiled(args, ("paired", args.seg_records, reps, m),
                        lambda m=m: TiledFile(args.seg_records, reps, 50_000, seed=m - 1, mate=m,
                                              threads=args.host_threads),
                        saved_bytes_estimate(args.seg_records, mate=m))[0]
           for m in (1, 2)]
    args.input_seconds = time.time() - t
    log(f"[bench] paired input: 2 x {tfs[0].records * tfs[0].repeats:,} records, "
        f"{tfs[0].file_len / 1e9:.2f} + {tfs[1].file_len / 1e9:.2f} GB gz, ready in {args.input_seconds:.1f}s")
    # one ctx (= one HIP stream) per file, so the two DecompressAll passes run concurrently: at
    # chunk = 50,000 one file has only ~2.7k chunks, a third of the GPU's 8k wave slots
    ctxs = [pp.Device(dev.index), pp.Device(dev.index)]
    ranges = [partition_chunks(tf.p_input, world)[rank] for tf in tfs]
    args.split, _ = auto_split(args, wave_slots(dev), sum(b - a for a, b in ranges))
    shards, bufs = [], []
    t_setup = time.time()
    for tf, ctx, (a, b) in zip(tfs, ctxs, ranges):
        lo, hi = int(tf.p_input[a]) - 1, int(tf.p_input[b])
        comp = torch.empty(hi - lo + 256, dtype=torch.uint8, device=dev)
        comp[hi - lo:].zero_()
        tf.fill_device(comp, lo, hi)
        bufs.append(comp)
        text = int(tf.p_output[b] - tf.p_output[a])
        out_cap = min(text + (1 << 20), int(args.paired_out_gib * (1 << 30)))
        sh = pp.Shard(tf.index(a, b + 1), comp.data_ptr(), first=0, n=b - a, device=ctx,
                      comp_on_device=True, comp_len=hi - lo, out_capacity=out_cap)
        # keys per output batch, into a buffer sized for >= 200-B records (the run fails loudly,
        # PPG_BUF_ERROR, if a file has more)
        paired.attach_keys(sh, text // 200 + 4096)
        if args.split > 1:
            sh.set_split(*tf.side_points(a, b + 1, args.split))
        shards.append(sh)
    torch.cuda.synchronize()
    setup_s = time.time() - t_setup
    log(f"[bench] rank {rank}: R1 chunks [{ranges[0][0]},{ranges[0][1]}), R2 chunks [{ranges[1][0]},{ranges[1][1]}), "
        f"{shards[0].batches} + {shards[1].batches} output batches, setup {setup_s:.1f}s")

    import threading
    pairs = paired.Pairs()
    comm, via = (None, "ppg_pairs_check on one GPU")
    if world > 1:
        comm, via = make_comm(ctxs[0], world, rank, backend, xdev)
        if comm is None:
            raise RuntimeError(f"paired run needs the library's communicator: {via}")
        via = "ppg_pairs_check: keys to pair owners by ppg_comm_alltoallv (" + via.split(" over ")[-1] + ")"

    K = args.pair_chunk
    emit_ms = []

    def step(emit=True):
        if emit and world == 1:
            # one rank: the emission drives the shards' own run (ppg_pairs_emit_run): each output
            # batch of both files decoded once and its pair chunk halves packed while it is
            # resident, then the check over the keys the batches wrote
            t = time.perf_counter()
            for _ in pairs.emit_run(shards[0], shards[1], K, window_bytes=int(args.pair_window_gib * (1 << 30))):
                pass
            emit_ms.append((time.perf_counter() - t) * 1e3)
            return paired.require_pairs(pairs.check(shards[0], shards[1]))
        errs = []

        def run(sh):
            try:
                sh.run()
            except pp.PpgError as e:   # raised below, after the threads (and, N > 1, the other ranks) meet
                errs.append(e)
        th = [threading.Thread(target=run, args=(sh,)) for sh in shards]   # ctypes drops the GIL
        for x in th:
            x.start()
        for x in th:
            x.join()
        # every rank joins the check: a rank whose decode failed reports it there, and every rank
        # raises the first failing rank's status (ppg_pairs_check's status gather)
        res = pairs.check(shards[0], shards[1], comm)
        if errs:
            raise errs[0]
        n = paired.require_pairs(res)
        if emit:
            # the deliverable: every record-aligned pair chunk of this rank packed on the device
            # (ppg_pairs_emit_*: one rank re-runs multi-batch shards window by window; N ranks move
            # the mates' records to each pair chunk's owner), each window consumed before the next
            t = time.perf_counter()
            for _ in pairs.emit(shards[0], shards[1], K, comm, window_bytes=int(args.pair_window_gib * (1 << 30))):
                pass
            emit_ms.append((time.perf_counter() - t) * 1e3)
        return n

    import torch.distributed as dist
    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        npairs = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=xdev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    assert npairs == tfs[0].records * tfs[0].repeats, (npairs, tfs[0].records * tfs[0].repeats)
    text = sum(int(tf.p_output[-1] - tf.p_output[0]) for tf in tfs)
    est = pairs.emit_stats()
    emission = {"pair_chunk": K, "pair_chunks": est["pair_chunks"], "this_rank": list(est["mine"]) if world > 1 else None,
                "ms_per_step": statistics.median(emit_ms[-args.steps:]) if emit_ms else None,
                "last_step_ms": {k: round(est[k], 2) for k in ("rerun_ms", "pack_ms", "exchange_ms", "emit_ms")},
                "batches_rerun_per_step": est["reruns"],
                "verified": verify_pair_chunks(pairs, tfs, K, shards, comm, world, rank),
                "note": "every pair chunk of this rank packed on the device per step (records back to back + "
                        "descriptors per half, ppg_pairs_emit_*), inside the timed step; one rank: the emission "
                        "drives the shards' own run (ppg_pairs_emit_run: each output batch decoded once, its "
                        "halves packed while resident; ms_per_step = decode + packing, rerun_ms = the batches' "
                        "runs), the pair check after it; N ranks: decode, check, then the records moved to "
                        "their pair chunk's owner"}
    # the previous round's line (decode + check, no emission) for comparison, timed after the main loop
    t1 = time.perf_counter()
    for _ in range(args.steps):
        step(emit=False)
    torch.cuda.synchronize()
    check_only = (time.perf_counter() - t1) / args.steps
    return {
        "metric": f"paired-end record pairs/sec (R1+R2 DecompressAll + pair check + record-aligned pair chunks), "
                  f"{world} MI355X",
        "value": npairs * args.steps / elapsed,
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if world > 1 else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (Generator-shape 150 bp read pairs, tiled single gzip members, zlib level 6)",
        "config": {"workload": f"configs[4]-shaped: 2 x {tfs[0].file_len / 1e9:.1f} GB .fastq.gz over {world} GPU(s), "
                               f"chunk=50000, pair chunks of 50,000 records",
                   "pairs": npairs, "gz_bytes": [tf.file_len for tf in tfs], "decompressed_bytes": text,
                   "output_batches_per_file": [sh.batches for sh in shards],
                   "keys": "per output batch while resident (ppg_shard_set_keys)",
                   "pair_check": via,
                   "pair_chunks": f"{K:,} pairs each, packed on the device (ppg_pairs_emit_*)",
                   "waves_per_chunk": f"<= {args.split} (side points)" if args.split > 1 else 1},
        "decompressed_MBps": text * args.steps / elapsed / 1e6,
        "setup_s": {"input": round(args.input_seconds, 2), "shards": round(setup_s, 2)},
        "emission": emission,
        "without_emission": {"pairs_per_s": npairs / check_only if world == 1 else None,
                             "ms_per_step": check_only * 1e3,
                             "note": "decode + pair check only (the r04 line), rank 0's own clock"},
    }


def verify_pair_chunks(pairs, tfs, K, shards, comm, world, rank, samples=3):
    """Spot-check emitted pair chunks against the tiled members' text (after the timed loop): a few
    pair chunks of this rank -- the first, one straddling an output batch boundary when there is
    one, the last -- copied to the host, each half's bytes and descriptors equal to records
    [j*K, (j+1)*K) of its member (pair i = record i mod the segment's records of both files)."""
    want = set()
    it = pairs.emit_run(shards[0], shards[1], K) if world == 1 else pairs.emit(shards[0], shards[1], K, comm)
    for j0, j1 in it:
        span = list(range(j0, j1))
        pick = {span[0], span[-1], span[len(span) // 2]} if span else set()
        for j in sorted(pick)[:samples]:
            for f, tf in enumerate(tfs):
                b, d = pairs.copy_chunk(j, f)
                eb = tiled_records(tf, j * K, min((j + 1) * K, tf.records * tf.repeats))
                assert b.tobytes() == eb, ("pair chunk bytes differ", j, f)
                nl = np.nonzero(np.frombuffer(eb, np.uint8) == 10)[0].astype(np.uint32).reshape(-1, 4)
                assert np.array_equal(d, nl), ("pair chunk descriptors differ", j, f)
                want.add(j)
    return f"{len(want)} pair chunks of rank {rank} byte-compared with the members' text" if want else "none on this rank"


_REC_STARTS = {}


def tiled_records(tf, lo, hi):
    """Bytes of records [lo, hi) of a tiled member (its segment's records repeated)."""
    key = id(tf.text)
    if key not in _REC_STARTS:
        nl = np.nonzero(np.asarray(tf.text) == 10)[0]
        _REC_STARTS[key] = np.concatenate([[0], nl[3::4] + 1]).astype(np.int64)
    st = _REC_STARTS[key]
    n = tf.records
    out = []
    i = lo
    while i < hi:
        r = i % n
        take = min(hi - i, n - r)
        out.append(np.asarray(tf.text[int(st[r]):int(st[r + take])]).tobytes())
        i += take
    return b"".join(out)


def wave_slots(dev):
    """Resident wave slots of the GPU: CUs x 32 (8 waves per SIMD, the inflate kernel's occupancy)."""
    import torch
    return torch.cuda.get_device_properties(dev).multi_processor_count * 32


def auto_split(args, slots, chunks):
    """(S, K): split the last K of a rank's chunks into up to S waves each (ppg_shard_set_split).
    --split S > 0: every chunk.  --split 0 (auto): a rank holding less than one generation of
    resident waves (CUs x 32; --split-gens) splits every chunk, into enough waves for ~6
    generations and at least --tail-split (at most 64: in practice every inner block start, ~15 per
    10k-record chunk); a larger rank splits its last --tail-gens generations into --tail-split = 8,
    so the launch's tail drains in an eighth of a chunk's time.  --tail-gens auto: half a generation
    once the rank holds 2.5 generations or more (its waves' start times have spread out by the last
    generation), else one whole generation: with 1.6 generations (N = 4) the chunks left whole then
    all start at once, beside the pieces, instead of a last 0.1 generation of whole chunks starting
    when the first generation ends (r04: the N = 4 share 188.9 -> 175.6 ms).  Measured on one MI355X
    for the N = 1 step and the N = 2/4/8 strong-scaling shares."""
    if args.split > 0:
        return args.split, chunks
    if chunks < getattr(args, "split_gens", 1) * slots:
        return int(min(64, max(args.tail_split, -(-6 * slots // max(1, chunks))))), chunks
    gens = args.tail_gens
    if gens in (None, "auto"):
        gens = 0.5 if chunks >= 2.5 * slots else 1.0
    return args.tail_split, min(chunks, int(float(gens) * slots))


def tail2_split(args, slots, ksplit):
    """(S2, K2): of the K split chunks, the last K2 into up to S2 waves each (--tail2 S2:G2, default
    64 for the last quarter generation: the launch drains on pieces of single deflate blocks; "off"
    = none).  Measured (DESIGN.md §5, r04 on the r03 v5 kernel): the N = 8 share 91.3 (16) / 88.5
    (32) -> 86.9 ms (64), N = 1 688.8 -> 684.9, N = 2 / 4 346.3 / 188.9 -> 341.2 / 171.3 ms."""
    if not args.tail2 or args.tail2 == "off":
        return args.split, 0
    s2, g2 = args.tail2.split(":")
    if int(s2) <= args.split:
        return args.split, 0
    return int(s2), min(ksplit, int(float(g2) * slots))


def split_points(tf, args, c0, c1, slots):
    """Side points splitting chunks [c0, c1) into up to args.split waves each, and the last K2 of
    them into up to S2 (tail2_split)."""
    s2, k2 = tail2_split(args, slots, c1 - c0)
    if not k2:
        return tf.side_points(c0, c1 + 1, args.split)
    parts = [tf.side_points(c0, c1 - k2 + 1, args.split), tf.side_points(c1 - k2, c1 + 1, s2)]
    return tuple(np.concatenate([p[i] for p in parts]) for i in range(3))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_cmd(n, argv, port):
    """The torch.distributed.run command that starts n ranks of this script on one node."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def launch_ranks(n, argv):
    """`python bench.py --gpus N` without a launcher: start the N ranks (one process per GPU) as a
    child torch.distributed.run and return its exit code.  Nothing in this process has touched the
    GPU, and it starts a child rather than exec-ing (rank 0's JSON line passes straight through)."""
    cmd = launch_cmd(n, argv, _free_port())
    log(f"[bench] launching {n} ranks: {' '.join(cmd[1:])}")
    return subprocess.run(cmd).returncode


def make_comm(ctx, world, rank, backend, xdev):
    """The count all-gather's communicator inside libppgpu (ppg_comm): RCCL from a unique id that
    rank 0 makes and torch.distributed broadcasts (backend nccl), or the host shared-memory
    transport for the one-GPU rehearsal (gloo).  If the library cannot make one, the bench keeps
    going with torch.distributed's all_gather of the same counts and says so in the line."""
    import uuid
    import torch
    import torch.distributed as dist
    import parallelparsing_amd as pp
    if backend == "nccl":
        uid = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            try:
                uid = torch.frombuffer(bytearray(pp.Comm.unique_id()), dtype=torch.uint8)
            except pp.PpgError as e:
                log(f"[bench] ppg_comm_unique_id failed ({e})")
        u = uid.to(xdev)
        dist.broadcast(u, 0)
        uid = bytes(u.cpu().numpy().tobytes())
        ok = torch.tensor([0], dtype=torch.int64, device=xdev)
        comm = None
        if any(uid):
            try:
                comm = pp.Comm.rccl(ctx, world, rank, uid)
            except pp.PpgError as e:
                log(f"[bench] rank {rank}: ppg_comm_init failed ({e})")
                ok += 1
        else:
            ok += 1
        dist.all_reduce(ok)   # all ranks or none use the library's communicator
        if int(ok.item()):
            return None, "torch.distributed all_gather (libppgpu's RCCL communicator failed to initialise)"
        return comm, "libppgpu ppg_shard_gather_counts over RCCL (ncclAllGather)"
    names = [f"/ppg_bench_{uuid.uuid4().hex[:12]}" if rank == 0 else None]
    dist.broadcast_object_list(names, 0)
    return pp.Comm.host(world, rank, names[0]), "libppgpu ppg_shard_gather_counts over host shared memory (rehearsal)"


def rccl_info(world, backend):
    """The communicator the run actually used (reported in the line)."""
    import torch
    import torch.distributed as dist
    import parallelparsing_amd as pp
    on = dist.is_available() and dist.is_initialized()
    info = {"world_size": dist.get_world_size() if on else 1, "backend": backend if on else None,
            "libppgpu_rccl_version": pp.rccl_version()}
    try:
        info["rccl_version"] = ".".join(map(str, torch.cuda.nccl.version()))
    except Exception:   # noqa: BLE001 - informational only
        info["rccl_version"] = None
    return info


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="50gb", choices=["50gb", "1m"])
    ap.add_argument("--chunk", type=int, default=10000)
    # the 50 GB member repeats one segment of distinct text: 10.5 M records (~4 GB of text, ~1 GB of
    # gzip) x 51 = ~50 GB gz, ~535 M records (r01: a 1 GB segment x 203)
    ap.add_argument("--seg-records", type=int, default=None, help=f"records per segment (default {SEG_RECORDS:,})")
    ap.add_argument("--repeats", type=int, default=REPEATS)          # per GPU (weak) or in all (strong)
    ap.add_argument("--scaling", default=None, choices=["weak", "strong"],
                    help="strong (default for N > 1, BASELINE configs[3]): one ~50 GB member split over the N "
                         "GPUs; weak: ~50 GB of gzip per GPU")
    ap.add_argument("--out-capacity-gib", type=float, default=192.0)   # one batch: 50 GB gz + 192 GiB out fit 288 GB
    ap.add_argument("--host-threads", type=int, default=16)
    ap.add_argument("--shm-dir", default="/dev/shm",
                    help="N > 1: where local rank 0 publishes the built input member for the other ranks")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--ingest-piece-gib", type=float, default=8,
                    help="ingest leg: compressed GiB per pipelined piece (ppg_file_decompress_all piece_bytes)")
    ap.add_argument("--ix-piece-kib", type=float, default=0,
                    help="--create-index: compressed bytes per pass-1 piece in KiB (0 = the library's default)")
    ap.add_argument("--ix-capacity-gib", type=float, default=0,
                    help="--create-index: pass-2 output buffer in GiB (0 = the library's default)")
    ap.add_argument("--create-index", action="store_true",
                    help="also time the GPU CreateIndex over the whole member (reported under 'create_index')")
    ap.add_argument("--paired", action="store_true",
                    help="configs[4]-shaped paired-end run on one GPU (prints its own line instead)")
    ap.add_argument("--paired-repeats", type=int, default=0)   # 0: 102 (configs[4]: ~25 GB gz per file)
    ap.add_argument("--pair-chunk", type=int, default=50_000,
                    help="--paired: pairs per record-aligned pair chunk (BASELINE configs[4]: 50,000)")
    ap.add_argument("--pair-window-gib", type=float, default=8.0,
                    help="--paired: device bytes per emission window and file (ppg_pairs_emit_begin)")
    ap.add_argument("--paired-out-gib", type=float, default=56.0,
                    help="--paired: output buffer per file in GiB (a rank's range decodes in batches of this; the "
                         "spot keys are extracted per batch)")
    ap.add_argument("--tail2", default="64:0.25",
                    help="S2:G2 -- of the split chunks, the last G2 generations into up to S2 waves each "
                         "(default 64:0.25, in practice every inner block start; off = none)")
    ap.add_argument("--split-gens", type=float, default=1,
                    help="--split 0: a rank with fewer chunks than this many generations of wave slots splits every "
                         "chunk; a larger one splits its last --tail-gens generations into --tail-split waves")
    ap.add_argument("--tail-split", type=int, default=8,
                    help="--split 0 on a large rank: waves per chunk for its last generation of chunks (1 = off)")
    ap.add_argument("--tail-gens", default="auto",
                    help="--split 0 on a large rank: how many generations of its last chunks to split (auto: 0.5 "
                         "from 2.5 generations of chunks up, else 1)")
    ap.add_argument("--split", type=int, default=0,
                    help="decode each chunk as up to S waves, split at inner deflate block starts "
                         "(ppg_shard_set_split; side points from the member's block list); 1 = one wave per chunk; "
                         "0 (default) = auto (auto_split): the last half-generation of a rank's chunks into 8 waves "
                         "each; every chunk, into >= 8, on a rank with less than one generation (N = 8 strong)")
    ap.add_argument("--share", type=int, default=1,
                    help="rehearsal on one GPU: decode only rank 0's chunk range of an N-way strong split (the "
                         "per-rank step of configs[3] at N GPUs, without the other ranks); records checked per range")
    ap.add_argument("--blank-lines", action="store_true",
                    help="side measurement: an empty line after every record, so every chunk takes the declined-chunk "
                         "parse (ppg_parse_chain; PPG_PARSE_CHAIN=0: the byte-serial lane) -- not the metric's workload")
    ap.add_argument("--no-ingest", action="store_true",
                    help="skip the end-to-end leg (N = 1): DecompressAll straight from the .gz file on disk (host "
                         "ingest, PCIe-inclusive; reported under 'ingest', never as value)")
    ap.add_argument("--ingest", action="store_true", help=argparse.SUPPRESS)   # on by default since r02
    ap.add_argument("--no-enumerate", action="store_true",
                    help="skip the enumerator leg (N = 1, after the ingest leg): every record's bytes and descriptor "
                         "landed in host memory through ppg_cursor (reported under 'enumerate', never as value)")
    ap.add_argument("--no-chunk-api", action="store_true",
                    help="skip the per-chunk Decompress leg (N = 1): ppg_decompress_chunk from 1/8/64 host threads "
                         "(reported under 'decompress_chunk', never as value)")
    ap.add_argument("--enum-batch-gib", type=float, default=8.0, help="enumerator leg: text per cursor batch (GiB)")
    args = ap.parse_args()
    if args.seg_records is None:   # the paired files keep 1 GB segments: two members must fit one GPU
        args.seg_records = PAIRED_SEG_RECORDS if args.paired else SEG_RECORDS

    # 8 hardware queues per process (the box exports HIP's default, 4): with 4, the runtime maps some
    # of the library's streams onto one queue, where they run in order -- the host ingest's copy
    # stream behind a piece's decode kernels (r06: the 50 GB ingest 1.24 -> 1.08 s, profiles/r06h_*;
    # the library also puts that copy stream at the greatest priority).  Set before anything
    # initialises HIP; the ranks a launch starts inherit it.
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("PPG_BENCH_HW_QUEUES", "8")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    args.world = world
    if args.scaling is None:
        args.scaling = "strong" if world > 1 else "weak"
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    args.local_rank, args.rank, args.shm_paths = local, rank, []
    # PPG_BENCH_FORCE_DIST=1 (tests): the N > 1 glue -- process group, the library's RCCL
    # communicator from a broadcast unique id, the count all-gather -- even at world size 1
    dist_on = world > 1 or os.environ.get("PPG_BENCH_FORCE_DIST") == "1"
    if world != args.gpus:
        log(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    if os.environ.get("PPG_BENCH_DRYRUN"):   # launcher test (tests/test_bench_launch.py): no GPU
        with open(os.path.join(os.environ["PPG_BENCH_DRYRUN"], f"rank{rank}.json"), "w") as f:
            json.dump({"rank": rank, "local_rank": local, "world": world, "scaling": args.scaling,
                       "master": f"{os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}"}, f)
        return
    import torch
    # rehearsal knobs (never set by the driver): PPG_BENCH_ONE_DEVICE=1 puts every rank on cuda:0 and
    # PPG_DIST_BACKEND=gloo exchanges through host memory, so the N > 1 path runs on a 1-GPU box
    if os.environ.get("PPG_BENCH_ONE_DEVICE") == "1":
        local = 0
    backend = os.environ.get("PPG_DIST_BACKEND", "nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if dist_on:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)   # RCCL over xGMI
        else:
            dist.init_process_group(backend)
    xdev = dev if backend == "nccl" else torch.device("cpu")   # where collectives' tensors live

    import parallelparsing_amd as pp
    from parallelparsing_amd.dist import partition_chunks, gather_counts

    if args.paired:
        line = paired_run(args, dev, world, rank, xdev, backend)
        line["communicator"] = rccl_info(world, backend)
        if rank == 0:
            print(json.dumps(line), flush=True)
        if dist_on:
            dist.barrier()
            drop_shared(args)
            dist.destroy_process_group()
        return

    try:
        return run_bench(args, dev, world, rank, local, dist_on, backend, xdev)
    except SetupFailed as e:
        # every rank got here with the same message (agree_setup): exit non-zero, no rank stranded
        log(f"[bench] rank {rank}: {e}")
        drop_shared(args)   # every rank is past the agreement: the shared input (or its failure file) can go
        if dist_on:
            # every rank has said so before any exits (torchrun stops the others at the first exit)
            dist.barrier()
            dist.destroy_process_group()
        sys.exit(3)


def run_bench(args, dev, world, rank, local, dist_on, backend, xdev):
    import torch
    import parallelparsing_amd as pp
    from parallelparsing_amd.dist import partition_chunks, gather_counts
    if dist_on:
        import torch.distributed as dist

    # setup, in stages whose status every rank agrees on before the next collective (agree_setup)
    err = tf = None
    try:
        if setup_fault("input", rank) and local != 0:
            raise RuntimeError("injected input failure (PPG_BENCH_FAIL)")
        tf = build_input(args)
    except SetupFailed:
        raise
    except Exception as e:   # noqa: BLE001 - agreed with the other ranks, then raised on all of them
        err = e
    agree_setup("input", err, dist_on, xdev)
    ix_out, ix_in = tf.p_output, tf.p_input
    nchunks = tf.npoints - 1
    ranges = partition_chunks(ix_in, world)
    a, b = ranges[rank]
    if args.share > 1:   # rehearsal: one GPU times rank 0's share of an N-way strong split, alone
        assert world == 1, "--share emulates one rank of a larger job on a single process"
        a, b = partition_chunks(ix_in, args.share)[0]
        ranges = [(a, b)]
    lo, hi = int(ix_in[a]) - 1, int(ix_in[b])   # file bytes [Input_a - 1, Input_b - 1]
    comp_len = hi - lo
    t_setup = time.time()
    err = comp = shard = ctx = None
    n_side = 0
    try:
        if setup_fault("shard", rank):
            raise RuntimeError("injected shard failure (PPG_BENCH_FAIL)")
        comp = torch.empty(comp_len + 256, dtype=torch.uint8, device=dev)
        comp[comp_len:].zero_()
        tf.fill_device(comp, lo, hi)
        torch.cuda.synchronize()
        index = tf.index(a, b + 1)   # this rank's points only: its chunks are index chunks 0..b-a-1
        ctx = pp.Device(local)
        out_cap = int(args.out_capacity_gib * (1 << 30))
        shard = pp.Shard(index, comp.data_ptr(), first=0, n=b - a, device=ctx, comp_on_device=True,
                         comp_len=comp_len, out_capacity=out_cap)
        args.split, ksplit = auto_split(args, wave_slots(dev), b - a)
        if args.split > 1:
            sb, so, sw = split_points(tf, args, b - ksplit, b, wave_slots(dev))
            if setup_fault("set_split", rank):
                # a real library error: side points past their chunks' outputs (PPG_ARG_ERROR)
                so = so + int(ix_out[b] - ix_out[a]) + (1 << 20)
            shard.set_split(sb, so, sw)
            n_side = int(sb.size)
            log(f"[bench] rank {rank}: last {ksplit} chunks split, {b - a + sb.size} waves ({sb.size} side points)")
        args.split_chunks = ksplit if args.split > 1 else 0
        args.tail2_s, args.tail2_k = tail2_split(args, wave_slots(dev), ksplit) if args.split > 1 else (1, 0)
    except Exception as e:   # noqa: BLE001 - agreed with the other ranks, then raised on all of them
        err = e
    agree_setup("shard", err, dist_on, xdev)
    setup_s = time.time() - t_setup
    log(f"[bench] rank {rank}: chunks [{a},{b}) {comp_len / 1e9:.2f} GB gz resident, "
        f"{shard.batches} output batch(es), setup {setup_s:.1f}s")
    counts_dev = torch.zeros(max(1, b - a), dtype=torch.int64, device=dev)
    err = None
    comm, gather_via = None, None
    try:
        if setup_fault("comm", rank):
            raise RuntimeError("injected communicator failure (PPG_BENCH_FAIL)")
        if dist_on:
            comm, gather_via = make_comm(ctx, world, rank, backend, xdev)
    except Exception as e:   # noqa: BLE001 - agreed with the other ranks, then raised on all of them
        err = e
    agree_setup("comm", err, dist_on, xdev)
    bounds = np.array([r[0] for r in ranges] + [ranges[-1][1]], np.int32)
    # per-rank setup seconds (input ready, shard ready) of every rank, in the line
    setup_ranks = gather_pairs(args.input_seconds, setup_s, dist_on, xdev)
    if dist_on:
        drop_shared(args)   # every rank has mapped the shared input by now

    def step():
        err = None
        try:
            shard.run()
        except pp.PpgError as e:
            err = e
        if dist_on:
            if comm is not None:
                # the C ABI's count all-gather (ppg_shard_gather_counts): a rank whose run failed
                # still joins, and every rank raises the first failing rank's status
                c, bs, _ = pp.gather_counts(shard, comm, bounds)
                return c, bs
            f = torch.tensor([1 if err else 0], dtype=torch.int64, device=xdev)
            dist.all_reduce(f)   # the torch fallback: agree on failure before the gather
            if int(f.item()):
                raise err or RuntimeError("DecompressAll failed on another rank")
            shard.counts_to_device(counts_dev.data_ptr())
            return gather_counts(counts_dev[: b - a].to(xdev), ranges, device=xdev)
        if err:
            raise err
        return None

    for _ in range(args.warmup):
        step()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    infl_ms = parse_ms = 0.0
    for _ in range(args.steps):
        g = step()
        tm = shard.timing()
        infl_ms += tm["inflate_ms"]
        parse_ms += tm["parse_ms"]
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    own_elapsed = elapsed
    if dist_on:
        e = torch.tensor([elapsed], dtype=torch.float64, device=xdev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())

    # correctness of the run (size-independent checks; bit parity is tests/test_gpu_parity.py)
    r = shard.results()
    # per-rank evidence: every rank's own step time, inflate launch time,
    # output batches, chunks, waves and records, so an N > 1 curve can be diagnosed from its line
    per_rank = [{"rank": i, "ms_per_step": round(v[0], 3), "inflate_ms_per_step": round(v[1], 3),
                 "parse_ms_per_step": round(v[2], 3), "batches": int(v[3]), "chunks": int(v[4]),
                 "waves": int(v[5]), "records": int(v[6]), "gz_GB": round(v[7] / 1e9, 3)}
                for i, v in enumerate(gather_vec([own_elapsed / args.steps * 1e3, infl_ms / args.steps,
                                                  parse_ms / args.steps, shard.batches, b - a, b - a + n_side,
                                                  int(r["records"].sum()), comp_len], dist_on, xdev))]
    assert (r["status"] == 0).all(), "chunk errors"
    assert (r["produced"] == (ix_out[a + 1:b + 1] - ix_out[a:b])).all(), "produced != to.Output - from.Output"
    local_records = int(r["records"].sum())
    if dist_on:
        counts, bases = g
        total_records = int(counts.sum())
    else:
        total_records = local_records
    expect = tf.expected_records()   # includes the reference's Q1 duplicates
    if args.share > 1:
        expect = None   # a share: produced lengths and statuses are checked above, counts per range below
        line_share = {"share_of": args.share, "chunks": [a, b], "records": total_records}
    if expect is not None and not (os.environ.get("PPG_PROBE_NO_CENSUS") or os.environ.get("PPG_PROBE")):
        # (an A/B timing probe: no records, or wrong bytes by design)
        assert total_records == expect, (total_records, expect)

    text_bytes = int(ix_out[-1] - ix_out[0])
    comp_total = int(ix_in[-1] - ix_in[0])
    rec_s = total_records * args.steps / elapsed
    # roofline of the dominant kernel (inflate): algorithmic bytes per launch / its mean duration
    alg_local = int((ix_in[a + 1:b + 1] - ix_in[a:b] + 1).sum() + (ix_out[a + 1:b + 1] - ix_out[a:b]).sum())
    launches = shard.batches * args.steps
    mean_launch_s = infl_ms / 1e3 / launches
    achieved = alg_local / shard.batches / mean_launch_s / 1e9
    workload = ("configs[1]: 1 M-read .fastq.gz, chunk=10000" if args.workload != "50gb"
                else "configs[2]: ~50 GB .fastq.gz per GPU, chunk=10000" if args.scaling == "weak" or world == 1
                else f"configs[3]: ~50 GB .fastq.gz sharded across {world} GPUs, chunk=10000")
    build = pp.build_info()
    line = {
        "metric": "FASTQ records/sec + decompressed MB/s, 50 GB .fastq.gz, 1/2/4/8 MI355X",
        "value": rec_s,
        "unit": "records/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "u8",
        "data": f"synthetic (Generator-shape 150 bp FASTQ, tiled single gzip member: one {tf.text_len / 1e9:.1f} GB "
                f"text segment x {tf.repeats}, zlib level 6)"
                + (", an empty line after every record (side measurement)" if args.blank_lines else ""),
        "config": {"workload": workload,
                   "records": total_records, "gz_bytes": tf.file_len, "decompressed_bytes": text_bytes,
                   "chunks": nchunks, "parallelism": f"chunk-sharded x{world}",
                   "waves_per_chunk": (f"<= {args.split} for the last {args.split_chunks} chunks per rank"
                                       + (f", <= {args.tail2_s} for the last {args.tail2_k}" if args.tail2_k else "")
                                       + " (side points)") if args.split > 1 else 1},
        "decompressed_MBps": text_bytes * args.steps / elapsed / 1e6,
        "kernel_ms_per_step": {"inflate": infl_ms / args.steps, "parse": parse_ms / args.steps},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic(workload, build),
                     "kernel": "ppg_inflate_kernel", "alg_bytes_per_launch": alg_local / shard.batches,
                     "issue": issue_roofline(build),
                     "mean_launch_ms": mean_launch_s * 1e3,
                     # memory-side bytes (2 x FETCH_SIZE + WRITE_SIZE, calibrated, Infinity-Cache hits
                     # included) over the same launch time: how much of the HBM peak the traffic is
                     **({"traffic_GBps": traffic / mean_launch_s / 1e9,
                         "traffic_frac": traffic / mean_launch_s / 1e9 / HBM_PEAK_GBS}
                        if (traffic := pmc_traffic(workload, build)) else {}),
                     # SURVEY §8d's secondary terms (not in alg_bytes), per launch of this rank
                     "secondary_bytes_per_launch": {
                         "windows": 32768 * (b - a + n_side) // shard.batches,
                         "offsets": int(tf.p_offlen[a:b].sum()) // shard.batches,
                         "census_positions": 2 * 4 * 4 * local_records // shard.batches,   # 4 B per newline, written + read
                         "descriptors": 16 * local_records // shard.batches,
                         "parse_reread": 0}},   # the newline census is fused into the inflate flush
        "reference_published_rec_s": REFERENCE_REC_S,
        **({"rehearsal_share": line_share} if args.share > 1 else {}),
        "communicator": dict(rccl_info(world, backend), count_gather=gather_via),
        "build": build,
        # seconds per rank before timing: the input member ready (built once per node, shared via
        # /dev/shm for N > 1), then the rank's shard resident in HBM (compressed range, windows)
        "setup_s": {"input_how": args.input_how, **({"share_dir_note": args.share_note} if getattr(args, "share_note", None) else {}),
                    "per_rank": [{"input": round(x, 2), "shard": round(y, 2)}
                                                               for x, y in setup_ranks]},
        "per_rank": {"ranks": per_rank,
                     "ms_per_step_min_max": [min(p["ms_per_step"] for p in per_rank),
                                             max(p["ms_per_step"] for p in per_rank)],
                     "inflate_ms_min_max": [min(p["inflate_ms_per_step"] for p in per_rank),
                                            max(p["inflate_ms_per_step"] for p in per_rank)],
                     "note": "each rank's own clock over the timed steps (value uses the max over ranks, "
                             "barrier-bracketed); inflate/parse: HIP-event launch times of its shard"},
    }
    if (dist_on or args.share > 1) and args.workload == "50gb" and not args.no_ingest and not args.blank_lines:
        # end to end at N > 1 ("scaling limits are host file read and
        # PCIe H2D"): every rank streams its own [P[a].Input - 1, P[b].Input - 1] range of the member
        # from a file in page cache (LazyFileReader.cs:41-97's role) through ppg_file_decompress_all;
        # max-over-ranks seconds beside the resident number.  The resident shard is freed first.
        shard = comp = None
        torch.cuda.empty_cache()
        line["ingest"] = dist_ingest_run(tf, args, ctx, a, b, rank, world, dist_on, xdev)
    args.ingest = world == 1 and args.workload == "50gb" and not args.no_ingest and not args.blank_lines and args.share == 1
    chunk_legs = world == 1 and args.workload == "50gb" and not args.no_chunk_api and args.share == 1
    if rank == 0 and world == 1 and (args.ingest or args.create_index or chunk_legs):
        # the measured shard (~270 GB of HBM at configs[2]) is done with: the legs below get the device
        shard = comp = None
        torch.cuda.empty_cache()
        # (r05: allocations over the freed HBM are slow for seconds after -- one of 284 GB right
        # after took 7.9 s, the first multi-GB grow of a launch slot's scratch 3.3-5.6 s; the
        # per-chunk legs warm every slot first)
    if rank == 0 and world == 1 and args.create_index:
        line["create_index"] = create_index_run(tf, args, dev)
    if rank == 0 and world == 1 and args.ingest:
        # on the bench's own ctx (r05: a second ctx measured 345 against 398 M records/s, one box,
        # profiles/r05zv_ingest_ctx.txt); its buffers -- three 8 GiB pieces and their shards'
        # outputs -- are freed after it (ppg_file_release), before the per-chunk legs
        try:
            line["ingest"], enum = ingest_run(tf, tf.index(0, tf.npoints), ctx, args.host_threads,
                                              args.ingest_piece_gib, 0 if args.no_enumerate else args.enum_batch_gib)
            if enum is not None:
                line["enumerate"] = enum
        except (OSError, AssertionError, RuntimeError) as e:   # e.g. no room for the file in $TMPDIR
            line["ingest"] = {"error": f"{type(e).__name__}: {e}"}
        finally:
            ctx.release_file_buffers()
    if rank == 0 and chunk_legs:
        free_b, total_b = torch.cuda.mem_get_info(ctx.device)
        print(f"[bench] chunk legs: {free_b / 1e9:.1f} of {total_b / 1e9:.1f} GB of HBM free", file=sys.stderr, flush=True)
        try:
            line["decompress_chunk"] = decompress_chunk_run(tf, ctx, r["records"])
        except (AssertionError, RuntimeError, pp.PpgError) as e:
            line["decompress_chunk"] = {"error": f"{type(e).__name__}: {e}"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(tf, ix_out, ix_in, nchunks, usable_cpus())
    if rank == 0:
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.close()
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

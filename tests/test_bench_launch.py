"""bench.py's own rank launcher (the driver may start `python bench.py --gpus N` directly): with
no WORLD_SIZE in the environment it must start N ranks through torch.distributed.run, each with
its RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, before anything touches a GPU.  PPG_BENCH_DRYRUN
makes every rank report its environment and exit, so this runs on the CPU."""
import glob
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    with tempfile.TemporaryDirectory() as d:
        env.update(PPG_BENCH_DRYRUN=d, **(extra_env or {}))
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                           text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        out = []
        for p in sorted(glob.glob(os.path.join(d, "rank*.json"))):
            with open(p) as f:
                out.append(json.load(f))
        return out


def test_launcher_starts_n_ranks():
    lines = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert sorted(x["rank"] for x in lines) == [0, 1]
    assert sorted(x["local_rank"] for x in lines) == [0, 1]
    assert all(x["world"] == 2 for x in lines)
    assert all(x["scaling"] == "strong" for x in lines)          # configs[3] by default for N > 1
    assert all(x["master"].startswith("127.0.0.1:") for x in lines)


def test_single_gpu_stays_in_process():
    lines = _run(["--gpus", "1"])
    assert lines == [{"rank": 0, "local_rank": 0, "world": 1, "scaling": "weak", "master": "None:None"}]


def test_weak_flag_kept_for_n_ranks():
    lines = _run(["--gpus", "2", "--scaling", "weak"])
    assert [x["scaling"] for x in lines] == ["weak", "weak"]


def test_launch_cmd_shape():
    sys.path.insert(0, ROOT)
    import bench
    cmd = bench.launch_cmd(8, ["--gpus", "8", "--steps", "3"], 29511)
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=8" in cmd and "127.0.0.1" in cmd and "--master-port=29511" in cmd
    assert cmd[-3:] == ["--gpus", "8", "--steps", "3"][-3:]


def _pairs_rank(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    q.put((rank, bench.gather_pairs(float(rank), 10.0 + rank, True, "cpu")))
    dist.destroy_process_group()


def test_gather_pairs_gloo_world2():
    """bench.py's per-rank setup-seconds gather over gloo (the one-GPU rehearsal's backend)."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_pairs_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    assert got[0] == got[1] == [[0.0, 10.0], [1.0, 11.0]]


def test_share_dir_falls_back_when_shm_is_small(monkeypatch, tmp_path):
    """The shared input's directory (/dev/shm on the 8-GPU node may be smaller than the
    ~6 GB the 50 GB member's description takes): --shm-dir when it has room, else $TMPDIR (then
    /tmp, /var/tmp), with the reason in the line; no room anywhere is an OSError before any save."""
    sys.path.insert(0, ROOT)
    import bench
    from parallelparsing_amd.tiled import saved_bytes_estimate
    need = saved_bytes_estimate(10_485_760)   # the default 50 GB member's segment
    assert 4 << 30 < need < 8 << 30
    shm, tmpd = str(tmp_path / "shm"), str(tmp_path / "tmp")
    os.makedirs(shm)
    os.makedirs(tmpd)
    free = {shm: 2 << 30, tmpd: 100 << 30}
    monkeypatch.setattr(bench, "free_bytes", lambda p: free.get(p, 0))
    monkeypatch.setenv("TMPDIR", tmpd)
    d, note = bench.share_dir(shm, need)
    assert d == tmpd and note and "fell back" in note
    free[shm] = 64 << 30
    assert bench.share_dir(shm, need) == (shm, None)
    free[shm] = free[tmpd] = 1 << 30
    try:
        bench.share_dir(shm, need)
        raise AssertionError("no room anywhere must raise")
    except OSError as e:
        assert "GiB free" in str(e)


def _agree_rank(rank, world, port, bad, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, ROOT)
    import bench
    out = []
    for stage in ("input", "shard", "comm"):
        err = RuntimeError(f"rank {rank} broke at {stage}") if (rank, stage) in bad else None
        try:
            bench.agree_setup(stage, err, True, "cpu")
            out.append((stage, "ok"))
        except bench.SetupFailed as e:
            out.append((stage, str(e)))
            break
    # a collective after the agreement still meets (nobody is stranded)
    dist.barrier()
    q.put((rank, out))
    dist.destroy_process_group()


def _agree(world, bad):
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_agree_rank, args=(r, world, port, bad, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    return got


def test_setup_failure_on_one_rank_is_every_ranks_failure():
    """a setup stage that fails on rank 1 (gloo, world 2) makes BOTH ranks raise
    SetupFailed at that stage with rank 1's message -- no rank goes on into the next collective."""
    got = _agree(2, {(1, "shard")})
    for r in (0, 1):
        assert got[r][0] == ("input", "ok")
        stage, msg = got[r][1]
        assert stage == "shard" and "on rank(s) [1] of 2" in msg and "rank 1 broke at shard" in msg
        assert len(got[r]) == 2


def test_setup_failure_names_every_failing_rank():
    got = _agree(4, {(2, "comm"), (3, "comm")})
    for r in range(4):
        assert [s for s, _ in got[r]] == ["input", "shard", "comm"]
        msg = got[r][2][1]
        assert "on rank(s) [2, 3] of 4" in msg and "rank 2 broke at comm" in msg


def test_setup_agreement_single_process_raises_its_own_error():
    sys.path.insert(0, ROOT)
    import bench
    bench.agree_setup("shard", None, False, "cpu")
    try:
        bench.agree_setup("shard", ValueError("x"), False, "cpu")
        raise AssertionError("must raise")
    except ValueError:
        pass
    os.environ["PPG_BENCH_FAIL"] = "set_split@3"
    try:
        assert bench.setup_fault("set_split", 3) and not bench.setup_fault("set_split", 2)
        assert not bench.setup_fault("shard", 3)
    finally:
        del os.environ["PPG_BENCH_FAIL"]


def test_ingest_pieces_keep_four_pieces_per_rank():
    """The N > 1 end-to-end leg's piece size and split (bench.ingest_pieces) on configs[3]'s shape."""
    sys.path.insert(0, ROOT)
    import bench
    import numpy as np

    class TF:   # ~50 GB over 52,467 chunks, as the default member
        p_input = np.linspace(11, 50e9, 52468).astype(np.int64)

    class A:
        ingest_piece_gib = 8.0
    slots = 256 * 32
    for world in (2, 4, 8):
        a, b = 0, 52467 // world
        pb, waves = bench.ingest_pieces(A, TF, a, b, slots)
        rng = TF.p_input[b] - TF.p_input[a] + 1
        assert 3.9 <= rng / pb <= 4.1 or pb == 8 << 30
        assert 1 <= waves <= 16
    assert bench.ingest_pieces(A, TF, 0, 52467 // 8, slots)[1] > bench.ingest_pieces(A, TF, 0, 52467 // 2, slots)[1]

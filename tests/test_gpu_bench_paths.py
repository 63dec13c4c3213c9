"""bench.py's multi-rank paths, rehearsed on the one GPU of the box (every rank on cuda:0,
PPG_BENCH_ONE_DEVICE=1) with gloo for torch.distributed and the library's host transport for the
count all-gather: the driver's `python bench.py --gpus N` (the bench launches its own ranks) and
the paired configs[4] path on two ranks, which must find exactly the single-rank pair count."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, ranks=1, timeout=240):
    env = dict(os.environ, PPG_BENCH_ONE_DEVICE="1", PPG_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py")] + args
    if ranks > 1 and "--gpus" not in args:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
               "--master-addr", "127.0.0.1", "--master-port", str(29400 + os.getpid() % 500)] + cmd[1:]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return lines[0]


SMALL = ["--seg-records", "40000", "--repeats", "6", "--steps", "1", "--warmup", "1", "--no-cpu-baseline",
         "--no-ingest"]


def test_bench_launches_its_own_ranks_and_gathers_in_the_abi():
    one = _bench(SMALL)
    two = _bench(SMALL + ["--gpus", "2"])
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["scaling"] == "strong" and two["config"]["workload"].startswith("configs[3]")
    assert two["config"]["records"] == one["config"]["records"]          # the bench asserts the exact count too
    assert two["communicator"]["world_size"] == 2
    assert "ppg_shard_gather_counts" in two["communicator"]["count_gather"]


def test_bench_paired_two_ranks_same_pairs():
    args = ["--paired", "--seg-records", "100000", "--paired-repeats", "3", "--steps", "1", "--warmup", "1"]
    one = _bench(args)
    two = _bench(args, ranks=2)
    assert one["config"]["pairs"] == two["config"]["pairs"] == 300000
    assert two["n_gpus"] == 2 and two["config"]["pair_check"].startswith("ppg_pairs_check: keys to pair owners")


def test_bench_rccl_glue_world1():
    """The bench's N > 1 glue under nccl = RCCL, at world size 1 (one GPU on this box): the process
    group, rank 0's ppg_comm_unique_id broadcast, ppg_comm_init, and ppg_shard_gather_counts over
    RCCL every step."""
    env = dict(os.environ, PPG_BENCH_FORCE_DIST="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "PPG_BENCH_ONE_DEVICE", "PPG_DIST_BACKEND"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(29000 + os.getpid() % 400),
           os.path.join(ROOT, "bench.py")] + SMALL
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    c = line["communicator"]
    assert c["backend"] == "nccl" and c["world_size"] == 1
    assert c["count_gather"] == "libppgpu ppg_shard_gather_counts over RCCL (ncclAllGather)"
    one = _bench(SMALL)
    assert line["config"]["records"] == one["config"]["records"]
    assert len(line["setup_s"]["per_rank"]) == 1


def test_bench_shares_the_input_between_ranks():
    """N > 1: local rank 0 builds the member once and the other ranks memory-map it from /dev/shm
    (VERDICT r02 next #2); the shared copy is gone after the run."""
    import glob
    before = set(glob.glob("/dev/shm/ppg_bench_*"))
    two = _bench(SMALL + ["--gpus", "2"])
    st = two["setup_s"]
    assert st["input_how"].startswith("built (shared via /dev/shm/")
    assert len(st["per_rank"]) == 2
    assert set(glob.glob("/dev/shm/ppg_bench_*")) == before


def test_bench_world8_rehearsal():
    """configs[3]'s world size on the one-GPU box: `bench.py --gpus 8` starts
    eight ranks (all on cuda:0, gloo + the library's host transport for the count gather) and runs
    the whole N = 8 path -- ppg_partition's ranges, the per-rank auto split, gather_pairs, the count
    gather, max-over-ranks timing -- to the single-rank record count (the bench asserts it)."""
    one = _bench(SMALL + ["--repeats", "16"])
    eight = _bench(SMALL + ["--repeats", "16", "--gpus", "8"], timeout=420)
    assert eight["n_gpus"] == 8 and eight["scaling"] == "strong"
    assert eight["config"]["workload"].startswith("configs[3]")
    assert eight["config"]["records"] == one["config"]["records"]
    assert eight["communicator"]["world_size"] == 8
    assert "ppg_shard_gather_counts" in eight["communicator"]["count_gather"]
    assert len(eight["setup_s"]["per_rank"]) == 8

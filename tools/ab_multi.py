"""A/B of several libppgpu.so builds in ONE process over ONE resident copy of the bench member.

    python tools/ab_multi.py [--rounds R] [--steps K] tag=path/libppgpu.so[,VAR=val] ...

Each build is dlopen'ed on its own (ctypes, RTLD_LOCAL: the builds' identical symbols do not
clash), gets its own ctx, index and shard over the same device buffer of compressed bytes, and the
builds take turns: R rounds x (every build: 1 warm-up + K timed DecompressAll runs), so drift on
the box hits every build alike, and the ~25 s of building the 50 GB member is paid once instead of
once per build (tools/ab_interleave.sh).  Reports, per build, the inflate ms per launch of every
round (the library's own HIP-event timing, ppg_shard_timing) and the record total (must equal
the member's).  VAR=val is set in the environment while that build opens its ctx (PPG_RING_BITS).
"""
import argparse
import ctypes as C
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def bind(path):
    L = C.CDLL(path)
    vp, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
    sig = {
        "ppg_open": (C.c_int, [C.c_int, C.POINTER(vp)]),
        "ppg_close": (None, [vp]),
        "ppg_index_from_points": (C.c_int, [i32, vp, vp, vp, vp, vp, vp, i32, C.POINTER(vp)]),
        "ppg_index_free": (None, [vp]),
        "ppg_shard_create": (C.c_int, [vp, vp, i32, i32, vp, i64, C.c_int, i64, C.POINTER(vp)]),
        "ppg_shard_set_split": (C.c_int, [vp, i32, vp, vp, vp]),
        "ppg_shard_run": (C.c_int, [vp]),
        "ppg_shard_total_records": (i64, [vp]),
        "ppg_shard_timing": (C.c_int, [vp, C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_float)]),
        "ppg_shard_free": (None, [vp]),
        "ppg_build_id": (C.c_char_p, []),
    }
    for n, (r, a) in sig.items():
        f = getattr(L, n)
        f.restype, f.argtypes = r, a
    return L


def ptr(a):
    return C.c_void_p(a.ctypes.data)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--repeats", type=int, default=51)
    ap.add_argument("--seg-records", type=int, default=10_485_760)
    ap.add_argument("builds", nargs="+")
    args = ap.parse_args()
    import torch
    import bench
    from parallelparsing_amd.tiled import TiledFile
    t = time.time()
    tf = TiledFile(args.seg_records, args.repeats, 10000, threads=16)
    n = tf.npoints - 1
    print(f"[ab] member: {n} chunks, {tf.file_len / 1e9:.2f} GB gz, built in {time.time() - t:.1f}s", file=sys.stderr,
          flush=True)
    dev = torch.device("cuda", 0)
    lo, hi = int(tf.p_input[0]) - 1, int(tf.p_input[-1])
    comp = torch.empty(hi - lo + 256, dtype=torch.uint8, device=dev)
    comp[hi - lo:].zero_()
    tf.fill_device(comp, lo, hi)
    torch.cuda.synchronize()
    win, offs = tf.windows(0, tf.npoints)
    arrs = [np.ascontiguousarray(x, tp) for x, tp in ((tf.p_output, np.int64), (tf.p_input, np.int64),
                                                       (tf.p_bits, np.int32), (win, np.uint8),
                                                       (tf.p_offlen, np.int32))]
    offs = np.ascontiguousarray(offs if len(offs) else np.zeros(1), np.uint8)
    # the bench's own split of the chunks (auto split, r04 rule)
    sa = argparse.Namespace(split=0, tail_split=8, tail_gens="auto", split_gens=1, tail2="64:0.25")
    slots = bench.wave_slots(dev)
    sa.split, ksplit = bench.auto_split(sa, slots, n)
    sb, so, sw = bench.split_points(tf, sa, n - ksplit, n, slots) if sa.split > 1 else (None, None, None)
    expect = tf.expected_records()
    builds = []
    for spec in args.builds:
        tag, rest = spec.split("=", 1)
        path, *envs = rest.split(",")
        old = {}
        for e in envs:
            k, v = e.split("=", 1)
            old[k] = os.environ.get(k)
            os.environ[k] = v
        L = bind(os.path.abspath(path))
        ctx, ix, sh = C.c_void_p(), C.c_void_p(), C.c_void_p()
        assert L.ppg_open(0, C.byref(ctx)) == 0
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        assert L.ppg_index_from_points(tf.npoints, *[ptr(a) for a in arrs], ptr(offs), 0, C.byref(ix)) == 0
        builds.append({"tag": tag, "L": L, "ctx": ctx, "ix": ix, "id": L.ppg_build_id().decode(),
                       "env": envs, "ms": []})
    for r in range(args.rounds):
        for b in builds:
            # a shard per turn: one build's one-batch output buffer (~206 GB) is most of the HBM
            L, sh = b["L"], C.c_void_p()
            assert L.ppg_shard_create(b["ctx"], b["ix"], 0, n, C.c_void_p(comp.data_ptr()), hi - lo, 1, 192 << 30,
                                      C.byref(sh)) == 0
            if sb is not None:
                assert L.ppg_shard_set_split(sh, int(sb.size), ptr(sb), ptr(so), ptr(sw)) == 0
            assert L.ppg_shard_run(sh) == 0
            vals = []
            for _ in range(args.steps):
                assert L.ppg_shard_run(sh) == 0
                fi, fp, ft = C.c_float(), C.c_float(), C.c_float()
                L.ppg_shard_timing(sh, C.byref(fi), C.byref(fp), C.byref(ft))
                vals.append(fi.value)
            assert L.ppg_shard_total_records(sh) == expect, (b["tag"], L.ppg_shard_total_records(sh), expect)
            L.ppg_shard_free(sh)
            b["ms"].append(statistics.median(vals))
            print(f"[ab] round {r} {b['tag']}: inflate {b['ms'][-1]:.2f} ms", file=sys.stderr, flush=True)
    out = {"member": {"chunks": n, "gz_bytes": tf.file_len, "records": expect},
           "split": f"<= {sa.split} waves for the last {ksplit} chunks, tail2 64:0.25",
           "builds": {b["tag"]: {"build_id": b["id"], "env": b["env"], "inflate_ms_per_round": [round(x, 2) for x in b["ms"]],
                                 "median": round(statistics.median(b["ms"]), 2)} for b in builds}}
    print(json.dumps(out))
    for b in builds:
        b["L"].ppg_index_free(b["ix"])
        b["L"].ppg_close(b["ctx"])


if __name__ == "__main__":
    main()

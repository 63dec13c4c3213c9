"""Why the strong-scaled N = 8 share sits ~1.7% above N = 1's eighth: a model of the inflate launch
as greedy list scheduling of its sub-jobs (chunks or pieces, in ljobs order: longest first, the
order ppg_shard_set_split launches them) on the GPU's 8,192 wave slots, each job taking time in
proportion to its output bytes.  The pieces are the bench's own (TiledFile.side_points of the 50 GB
member: block ends nearest even fractions of each chunk), so no piece is smaller than one deflate
block (~124 KB of text here) -- the granularity that bounds the drain.  CPU only (builds the
member's metadata, ~100 s on 8 cores):  python tools/share_sim.py [--out profiles/r05_share_sim.json]"""
import argparse
import heapq
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench   # noqa: E402
from parallelparsing_amd.tiled import TiledFile   # noqa: E402

SLOTS = 8192   # 256 CUs x 32 resident inflate waves (bench.wave_slots)


def pieces(tf, lo, hi, per_chunk):
    """Output bytes of the pieces of chunks [lo, hi) split as TiledFile.side_points(lo, hi + 1, per_chunk)."""
    po, boe, tl = tf.p_output, tf.block_out_end, tf.text.size
    out = []
    for c in range(lo, hi):
        a, b = int(po[c]), int(po[c + 1])
        if per_chunk < 2:
            out.append(b - a)
            continue
        tg = (a + (b - a) * np.arange(1, per_chunk) / per_chunk).astype(np.int64)
        r = tg // tl
        k = np.searchsorted(boe, tg - r * tl, side="left")
        wrap = k >= boe.size
        r, k = np.where(wrap, r + 1, r), np.where(wrap, 0, k)
        o = r * tl + boe[k]
        o = np.unique(o[(o > a) & (o < b)])
        out.extend(np.diff(np.concatenate([[a], o, [b]])).tolist())
    return out


def plan(tf, c0, c1, S, K, S2, K2):
    """Chunks [c0, c1): the last K split into up to S pieces, of those the last K2 into up to S2."""
    return np.array(pieces(tf, c0, c1 - K, 1) + pieces(tf, c1 - K, c1 - K2, S) + pieces(tf, c1 - K2, c1, S2),
                    np.float64)


def makespan(jobs):
    """(greedy longest-first makespan, ideal = total / SLOTS)."""
    h = [0.0] * SLOTS
    for x in np.sort(jobs)[::-1]:
        t = heapq.heappop(h)
        heapq.heappush(h, t + x)
    return max(h), jobs.sum() / SLOTS


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--threads", type=int, default=8)
    args = ap.parse_args()
    t = time.time()
    tf = TiledFile(bench.SEG_RECORDS, bench.REPEATS, 10000, threads=args.threads)
    nch = tf.npoints - 1
    res = {"chunks": nch, "slots": SLOTS, "build_s": round(time.time() - t, 1), "cases": {}}
    # N = 1 as bench.py runs it: the last half generation into 8, the last quarter into 64
    m1, i1 = makespan(plan(tf, 0, nch, 8, SLOTS // 2, 64, SLOTS // 4))
    res["cases"]["n1"] = {"makespan_over_ideal": round(m1 / i1, 4)}
    share = nch // 8
    variants = {"S8 + tail2 64:0.25 (shipped)": (8, share, 64, 2048), "S8": (8, share, 8, 0),
                "S6": (6, share, 6, 0), "S16": (16, share, 16, 0), "S64 (every block)": (64, share, 64, 0),
                "S8 + tail2 64:0.5": (8, share, 64, 4096), "S8 + tail2 64:0.125": (8, share, 64, 1024)}
    for name, (S, K, S2, K2) in variants.items():
        J = plan(tf, 0, share, S, K, S2, K2)
        m, i = makespan(J)
        res["cases"][f"share8 {name}"] = {
            "jobs": int(J.size), "makespan_over_ideal": round(m / i, 4),
            "over_n1_eighth": round(m / (m1 / 8), 4),
            "piece_kb": {"p1": round(np.percentile(J, 1) / 1e3, 1), "median": round(np.median(J) / 1e3, 1),
                         "max": round(J.max() / 1e3, 1)}}
    print(json.dumps(res, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()

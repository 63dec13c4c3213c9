"""Summarise tools/profile_round.sh outputs (gpurun_out/) into profiles/.

  python tools/traffic_summary.py <tag>
writes profiles/<tag>_bench_kernel_stats.csv (rocprofv3 --stats, copied), profiles/<tag>_bench.json
(the bench line of the profiled run) and profiles/traffic.json (HBM bytes per inflate launch, read
by bench.py for roofline.traffic).  Counter conventions (MI355X_MICROARCH.md, HBM section, and
tools/fetch_calib.hip, profiles/r02_fetch_calib.json): on gfx950 FETCH_SIZE tallies 64 B per
128-B memory-side request for every read shape the inflate kernel uses -- a coalesced 4-B-per-lane
read of B bytes reports B/2 (as the guide's 16-B-per-lane case), and a 4-B read landing in its own
128-B line reports 64 B -- so FETCH_SIZE is doubled for every kernel.  WRITE_SIZE is taken as
reported.  rocprofv3 reports both in KiB.  Infinity-Cache hits are counted too: the figure is
memory-side traffic out of the L2s, an upper bound on HBM bytes."""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")


def counters(c):
    tot, launches = defaultdict(float), defaultdict(set)
    for path in glob.glob(os.path.join(G, f"prof_{c}", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] != c:
                continue
            k = r["Kernel_Name"]
            tot[k] += float(r["Counter_Value"]) * 1024.0   # rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB
            launches[k].add(r["Dispatch_Id"])
    return tot, {k: len(v) for k, v in launches.items()}


def short(k):
    return k.split("(")[0].replace("void ", "")


def main(tag):
    stats = glob.glob(os.path.join(G, "prof_stats", "**", "*kernel_stats.csv"), recursive=True)
    shutil.copy(stats[0], os.path.join(ROOT, "profiles", f"{tag}_bench_kernel_stats.csv"))
    line = open(os.path.join(G, "prof_stats.json")).read().strip().splitlines()[-1]
    open(os.path.join(ROOT, "profiles", f"{tag}_bench.json"), "w").write(line + "\n")
    b = json.loads(open(os.path.join(G, "prof_FETCH_SIZE.json")).read().strip().splitlines()[-1])
    fetch, nf = counters("FETCH_SIZE")
    write, _ = counters("WRITE_SIZE")
    inf = [k for k in fetch if "ppg_inflate_kernel" in k][0]
    n = nf[inf]
    out = {
        "workload": b["config"]["workload"],
        # the library the counters were taken on (bench.py refuses the file for any other build)
        "build": b.get("build"),
        "command": "tools/profile_round.sh: rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE, separate pass) -- "
                   "python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ingest",
        "kernel": short(inf),
        "launches": n,
        "fetch_size_reported_bytes": fetch[inf] / n,
        "fetch_bytes": 2 * fetch[inf] / n,
        "write_bytes": write.get(inf, 0.0) / n,
        "hbm_bytes_per_launch": (2 * fetch[inf] + write.get(inf, 0.0)) / n,
        "alg_bytes_per_launch": b["roofline"]["alg_bytes_per_launch"],
        "note": "fetch_bytes = 2 x FETCH_SIZE: calibrated on gfx950 for the inflate kernel's own read shapes "
                "(tools/fetch_calib.hip, profiles/r02_fetch_calib.json: coalesced 4-B-per-lane and scattered 4-B "
                "reads both tally 64 B per 128-B request).  Memory-side traffic out of the L2s, Infinity-Cache hits "
                "included (an upper bound on HBM bytes).  WRITE_SIZE covers the decompressed bytes and the census's "
                "stored newline positions.",
        "other_kernels": {short(k): {"fetch_bytes_x2": 2 * v, "write_bytes": write.get(k, 0.0)}
                          for k, v in fetch.items() if k != inf and "ppg_" in k},
    }
    json.dump(out, open(os.path.join(ROOT, "profiles", "traffic.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])

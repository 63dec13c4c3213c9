"""Stall breakdown of ppg_inflate_kernel from tools/pmc_stalls.sh's passes
(gpurun_out/stall_<g>/) plus, when present, the PPG_STAMPS diagnostic build's per-phase cycles
(gpurun_out/ab_stamps.log) and the timing probes (gpurun_out/ab_<probe>.json).

  python tools/stall_summary.py <tag>      -> profiles/<tag>_inflate_stalls.json

Counter conventions (MI355X_MICROARCH.md, rocprofv3 PMC slots): SQ_WAIT_ANY (wave parked on
s_waitcnt / barrier), SQ_WAIT_INST_ANY (issue stall) and SQ_ACTIVE_INST_ANY (issuing) partition
SQ_WAVE_CYCLES; SQ_* cycle counters are quad-cycles; GRBM_GUI_ACTIVE sums the 8 XCDs."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")


def passes():
    """Counter totals over the inflate launches; a counter collected in several passes is taken from
    the first pass that has it (not summed over passes).  Also returns the kernel instantiation(s)
    the summed rows name (the label comes from the rows, not a literal)."""
    out, names = {}, set()
    for path in sorted(glob.glob(os.path.join(G, "stall_*", "**", "*counter_collection.csv"), recursive=True)):
        tot = defaultdict(float)
        for r in csv.DictReader(open(path)):
            if "ppg_inflate_kernel" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                names.add(kernel_label(r["Kernel_Name"]))
        for k, v in tot.items():
            out.setdefault(k, v)
    return out, sorted(names)


def kernel_label(name):
    """'void ppg_inflate_kernel<11, 8, false, true, false>(unsigned int const*, ...)' ->
    'ppg_inflate_kernel<11, 8, false, true, false>' (the form traffic.json's "kernel" uses)."""
    m = re.search(r"ppg_inflate_kernel<[^>]*>", name)
    return m.group(0) if m else name


def main(tag):
    c, names = passes()
    if len(names) != 1:
        raise SystemExit(f"the stall passes summed over {len(names)} inflate instantiations: {names}")
    wc = c["SQ_WAVE_CYCLES"]
    out = {
        "kernel": names[0],
        "workload": "bench.py --repeats 40 --steps 1 (40 x 4.04 GB text, chunk = 10,000), one launch",
        "command": "tools/pmc_stalls.sh: one rocprofv3 --pmc pass per counter group (A-E)",
        "counters": c,
        "wave_cycle_split": {"waiting (SQ_WAIT_ANY: s_waitcnt)": c["SQ_WAIT_ANY"] / wc,
                             "issue-stalled (SQ_WAIT_INST_ANY)": c["SQ_WAIT_INST_ANY"] / wc,
                             "issuing (SQ_ACTIVE_INST_ANY)": c["SQ_ACTIVE_INST_ANY"] / wc},
        "instructions": {k: c[k] for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH",
                                           "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SMEM") if k in c},
        "lds": {"bank_conflict_cycles_over_lds_active": c.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, c.get("SQ_LDS_IDX_ACTIVE", 1))},
        "occupancy_waves_per_simd": wc * 4 / (1024 * c["GRBM_GUI_ACTIVE"] / 8) * 1 if "GRBM_GUI_ACTIVE" in c else None,
    }
    stamps = os.path.join(G, "ab_stamps.log")
    if os.path.exists(stamps):
        ln = [x for x in open(stamps) if x.startswith("PPG_STAMPS")]
        if ln:
            m = dict(re.findall(r"(decode|walk|read|far|dep\+write|tail|total) ([\d.]+)", ln[-1]))
            out["round_phases_cycles_per_round_per_wave"] = {k: float(v) for k, v in m.items()}
            out["round_phases_note"] = ("PPG_STAMPS diagnostic build (s_memtime at each phase boundary of every "
                                        "token round, 50 GB step): wall cycles a wave spends per round in each "
                                        "phase, other waves interleaved; the stamps themselves add ~14%")
    probes = {}
    for t in ("base", "nostore", "nofar", "stamps"):
        p = os.path.join(G, f"ab_{t}.json")
        if os.path.exists(p):
            probes[t] = json.load(open(p))["kernel_ms_per_step"]["inflate"]
    if probes:
        out["probes_inflate_ms_50gb_step"] = probes
        out["probes_note"] = ("same box, tools/ab_bench.sh: nostore = no output stores (far bytes read garbage), "
                              "nofar = far bytes read from the ring: timing probes only, wrong output")
    # the build the passes measured (the bench's JSON line in a pass's log): bench.py quotes these
    # counters (roofline.issue) only for the same ppg_version + ppg_build_id
    for g in "ABCDE":
        p = os.path.join(G, f"stall_{g}.log")
        if os.path.exists(p):
            ln = [x for x in open(p) if x.startswith("{")]
            if ln:
                out["build"] = json.loads(ln[-1]).get("build")
                break
    path = os.path.join(ROOT, "profiles", f"{tag}_inflate_stalls.json")
    json.dump(out, open(path, "w"), indent=1)
    if out.get("build"):
        json.dump(out, open(os.path.join(ROOT, "profiles", "inflate_stalls.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])

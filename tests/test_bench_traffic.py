"""roofline.traffic is quoted from profiles/traffic.json only for the build it measured
(VERDICT r02 weak #6): the file names the workload and the library build (ppg_version +
ppg_build_id, a hash of the inflate object); any other build gets null."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import parallelparsing_amd as pp  # noqa: E402

W = "configs[2]: ~50 GB .fastq.gz per GPU, chunk=10000"


def _write(tmp_path, **kw):
    t = {"workload": W, "hbm_bytes_per_launch": 1.5e12, "build": pp.build_info()}
    t.update(kw)
    p = tmp_path / "traffic.json"
    p.write_text(json.dumps(t))
    return str(p)


def test_build_id_names_the_inflate_object():
    b = pp.build_info()
    assert b["build_id"].startswith("inflate-") and len(b["build_id"]) == len("inflate-") + 16
    assert "gfx950" in b["ppg_version"]


def test_matching_build_is_quoted(tmp_path):
    assert bench.pmc_traffic(W, pp.build_info(), _write(tmp_path)) == 1.5e12


def test_stale_build_is_refused(tmp_path):
    stale = dict(pp.build_info(), build_id="inflate-0123456789abcdef")
    assert bench.pmc_traffic(W, pp.build_info(), _write(tmp_path, build=stale)) is None
    # a file from before builds were recorded
    assert bench.pmc_traffic(W, pp.build_info(), _write(tmp_path, build=None)) is None


def test_other_workload_is_refused(tmp_path):
    assert bench.pmc_traffic("configs[1]: 1 M-read .fastq.gz, chunk=10000", pp.build_info(), _write(tmp_path)) is None


def test_issue_roofline_only_for_the_same_build(tmp_path):
    """roofline.issue: SALU per CU-cycle and VALU busy from the committed stall
    passes, quoted only for the build they measured."""
    b = {"ppg_version": "v", "build_id": "inflate-aaaa"}
    c = {"GRBM_GUI_ACTIVE": 8 * 1.0e9, "SQ_INSTS_SALU": 0.5 * 256 * 1.0e9, "SQ_INSTS_VALU": 0.25 * 1024 * 1.0e9}
    p = tmp_path / "stalls.json"
    p.write_text(json.dumps({"build": b, "counters": c, "workload": "w", "wave_cycle_split": {}}))
    r = bench.issue_roofline(b, str(p))
    assert abs(r["salu_per_cu_cycle"] - 0.5) < 1e-9 and abs(r["valu_busy"] - 0.5) < 1e-9
    assert bench.issue_roofline({"ppg_version": "v", "build_id": "inflate-bbbb"}, str(p)) is None
    assert bench.issue_roofline(b, str(tmp_path / "missing.json")) is None


def test_committed_stall_and_traffic_files_name_the_same_kernel():
    """roofline.issue's source (profiles/inflate_stalls.json) and roofline.traffic's
    (profiles/traffic.json) must describe the same inflate instantiation and build; the stall file's
    label comes from the rocprof rows it sums (tools/stall_summary.py), never a literal."""
    with open(os.path.join(ROOT, "profiles", "inflate_stalls.json")) as f:
        st = json.load(f)
    with open(os.path.join(ROOT, "profiles", "traffic.json")) as f:
        tr = json.load(f)
    assert st["kernel"] == tr["kernel"], (st["kernel"], tr["kernel"])
    assert st["build"] == tr["build"]


def test_stall_label_comes_from_the_rows():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import stall_summary
    n = "void ppg_inflate_kernel<11, 8, false, true, false>(unsigned int const*, unsigned long, PpgInflateJob const*)"
    assert stall_summary.kernel_label(n) == "ppg_inflate_kernel<11, 8, false, true, false>"

"""Host C++ under AddressSanitizer + UBSan and ThreadSanitizer: builds
tests/native (the host translation units of libppgpu with the sanitizer, the regular kernel
objects) and runs host_check -- CreateIndex, IndexIO, validate, partition, from_points, and the
shared-memory communicator's two-phase gather with failing ranks, from several threads."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")


def test_host_code_is_sanitizer_clean():
    r = subprocess.run(["make", "-s", "-C", NATIVE, "run"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    for name, bad in (("asan", "ERROR: AddressSanitizer"), ("tsan", "WARNING: ThreadSanitizer")):
        log = open(os.path.join(NATIVE, "_build", f"{name}.log")).read()
        assert "host_check: ok (0 failures)" in log, log[-3000:]
        assert f"{name} exit 0" in log and bad not in log and "runtime error" not in log, log[-3000:]

"""Coverage-guided fuzzing of every parser that sees outside bytes
(native/fuzz/, `make fuzz`): builds the libFuzzer targets with ROCm's clang
(ASan + UBSan) and runs each one briefly. A crash, a sanitizer report or a
broken invariant (e.g. GetPreferredAllocation returning an ID it never
advertised -- found this way, pinned by
tests/test_preferred.py::test_rechosen_replicas_are_checked_too) fails the test
with the target's log.
"""

import os
import subprocess

import pytest

from k8s_gpu_sharing_plugin_amd import REPO_ROOT

CLANG = "/opt/rocm/lib/llvm/bin/clang++"
TARGETS = ["plugin", "h2", "h2_diff", "h2_client", "proto", "config", "grantfile", "procscan", "relay"]


@pytest.mark.slow
@pytest.mark.skipif(not os.path.exists(CLANG), reason="needs ROCm's clang (libFuzzer)")
def test_fuzz_targets_run_clean():
    fuzz_dir = os.path.join(REPO_ROOT, "build", "fuzz")
    for f in os.listdir(fuzz_dir) if os.path.isdir(fuzz_dir) else []:
        if f.endswith(".failed"):
            os.unlink(os.path.join(fuzz_dir, f))
    r = subprocess.run(["make", "-s", "fuzz", "FUZZ_SECONDS=4", f"JOBS={min(8, os.cpu_count() or 1)}"],
                       cwd=REPO_ROOT, capture_output=True, text=True, timeout=900)
    logs = ""
    for t in TARGETS:
        p = os.path.join(fuzz_dir, f"fuzz_{t}.log")
        if os.path.exists(os.path.join(fuzz_dir, f"fuzz_{t}.failed")) and os.path.exists(p):
            logs += f"--- fuzz_{t}.log\n" + open(p).read()[-4000:]
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:] + logs
    done = [ln.split()[0] for ln in r.stdout.splitlines() if "DONE" in ln]
    assert sorted(done) == sorted(TARGETS), r.stdout

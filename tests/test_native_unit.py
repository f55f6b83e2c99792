"""Runs the C++ unit-test binary (codec, config, prioritizer, topology, gRPC loopback)."""

import subprocess

from k8s_gpu_sharing_plugin_amd import UNIT_TESTS


def test_concurrency_stress():
    """Allocate/ListAndWatch/health flips/restarts all at once (TSan/ASan-clean via `make tsan asan`)."""
    from k8s_gpu_sharing_plugin_amd import binary
    res = subprocess.run([binary("adp_stress"), binary("libamdsmi_mock.so"), "1.5"], stdout=subprocess.PIPE,
                         stderr=subprocess.STDOUT, text=True, timeout=120)
    assert res.returncode == 0, res.stdout[-3000:]
    assert "stress: pods=" in res.stdout


def test_native_unit_tests_pass():
    res = subprocess.run([UNIT_TESTS], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=120)
    assert res.returncode == 0, res.stdout
    assert ", 0 failed" in res.stdout

"""`amdgpu-device-plugin --doctor`: what a deployment needs on this node, one
line per check ("ok" / "warn" / "FAIL") with what to change; exit 1 on a
failure. Real hardware: tests/test_gpu.py::test_doctor_on_real_gpu."""

import os

import pytest
import subprocess

from k8s_gpu_sharing_plugin_amd import DAEMON, MOCK_LIB
from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import kubelet


def _doctor(tmp_path, *args, fx=None, lib=MOCK_LIB):
    env = dict(os.environ, AMD_SMI_LIB=lib,
               AMDSMI_MOCK_FIXTURE=fixtures.write(fx or fixtures.node(2), str(tmp_path / "fx")))
    r = subprocess.run([DAEMON, "--doctor", *args], capture_output=True, text=True, timeout=60, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    return r.returncode, lines


def _find(lines, text):
    return next((ln for ln in lines if text in ln), None)


def test_healthy_node_with_a_kubelet(tmp_path):
    d = tmp_path / "dp"
    d.mkdir()
    k = kubelet.StubKubelet(str(d / "kubelet.sock")).start()
    try:
        rc, lines = _doctor(tmp_path, "--device-plugin-path", str(d), "--resource-config", "gpu:sharedgpu:4")
    finally:
        k.stop()
    assert rc == 0, lines
    assert _find(lines, "enumeration: 2 GPU(s)").startswith("ok")
    assert _find(lines, "resources: amd.com/sharedgpu x8").startswith("ok")
    assert _find(lines, "kubelet socket").startswith("ok")
    assert _find(lines, "plugin directory").startswith("ok")
    assert _find(lines, "health events").startswith("ok")
    assert _find(lines, "CPU budget").startswith("ok")
    assert lines[-1].startswith("doctor: ") and "0 failure(s)" in lines[-1]
    # the mock's render nodes do not exist on this machine: a warning that says so
    dev = _find(lines, "device nodes")
    assert dev.startswith("warn") and "not present" in dev


def test_missing_kubelet_is_a_warning_and_an_unwritable_plugin_dir_a_failure(tmp_path):
    rc, lines = _doctor(tmp_path, "--device-plugin-path", "/proc/1")
    assert rc == 1, lines
    assert _find(lines, "kubelet socket").startswith("warn")
    assert _find(lines, "plugin directory /proc/1 not writable").startswith("FAIL")
    assert "1 failure(s)" in lines[-1]


def test_no_amdsmi_is_a_failure_with_a_hint(tmp_path):
    rc, lines = _doctor(tmp_path, "--device-plugin-path", str(tmp_path), lib="/nonexistent/libamd_smi.so")
    assert rc == 1 and lines[0].startswith("FAIL") and "libamd_smi.so" in lines[0], lines


def test_devices_filter_that_matches_nothing_fails(tmp_path):
    rc, lines = _doctor(tmp_path, "--device-plugin-path", str(tmp_path), "--devices", "0000:99:00.0")
    assert rc == 1 and _find(lines, "enumeration").startswith("FAIL"), lines


def test_enforced_grants_check_the_shim_and_the_host_proc(tmp_path):
    from k8s_gpu_sharing_plugin_amd import BUILD_DIR
    rc, lines = _doctor(tmp_path, "--device-plugin-path", str(tmp_path), "--resource-config", "gpu:gpu-mem-gb:-1",
                        "--enforce-memory-units", "--memcap-lib", os.path.join(BUILD_DIR, "libadp_memcap.so"),
                        "--metrics-addr", "127.0.0.1:0")
    assert _find(lines, "HBM-cap shim").startswith("ok"), lines
    assert _find(lines, "driver-side HBM check") is not None, lines
    assert _find(lines, "resources: amd.com/gpu-mem-gb x588").startswith("ok")


def test_device_cgroup_denial_is_named(tmp_path):
    """Under a device cgroup that denies /dev/kfd and /dev/dri/* (the EPERM
    libadp_devcgroup_sim.so injects) the device-node check warns, names the
    cause and the fix, and the node can still serve (exit 0)."""
    from k8s_gpu_sharing_plugin_amd import BUILD_DIR
    sim = os.path.join(BUILD_DIR, "libadp_devcgroup_sim.so")
    env = dict(os.environ, LD_PRELOAD=" ".join(x for x in (os.environ.get("LD_PRELOAD", ""), sim) if x),
               AMD_SMI_LIB=MOCK_LIB, AMDSMI_MOCK_FIXTURE=fixtures.write(fixtures.node(2), str(tmp_path / "fx")))
    r = subprocess.run([DAEMON, "--doctor", "--device-plugin-path", str(tmp_path)], capture_output=True, text=True,
                       timeout=60, env=env)
    lines = r.stdout.splitlines()
    dev = _find(lines, "device nodes")
    assert r.returncode == 0 and dev.startswith("warn"), r.stdout
    assert "Operation not permitted" in dev and "device cgroup" in dev and "privileged" in dev


def test_python_cli_doctor(tmp_path):
    import sys
    env = dict(os.environ, AMD_SMI_LIB=MOCK_LIB,
               AMDSMI_MOCK_FIXTURE=fixtures.write(fixtures.node(1), str(tmp_path / "fx")))
    r = subprocess.run([sys.executable, "-m", "k8s_gpu_sharing_plugin_amd", "doctor", "--device-plugin-path",
                        str(tmp_path)], capture_output=True, text=True, timeout=60, env=env)
    assert r.returncode == 0 and "enumeration: 1 GPU(s)" in r.stdout, r.stdout + r.stderr


def test_other_plugins_and_a_running_instance_are_reported(tmp_path):
    """Live sockets in the kubelet's directory: a running instance of this
    plugin (warn: starting another takes its sockets over), another GPU plugin
    (warn: the kubelet keeps whichever registered last), a non-GPU plugin (ok);
    a stale socket file nobody listens on is not reported."""
    import socket as so
    from k8s_gpu_sharing_plugin_amd.utils import harness
    d = tmp_path / "dp"
    d.mkdir()
    k = kubelet.StubKubelet(str(d / "kubelet.sock")).start()
    running = harness.Daemon(str(d), fixtures.node(2), args=["--resource-config", "gpu:sharedgpu:4"]).start()
    socks = []
    try:
        k.wait_registration()
        for name, listen in (("amd.com_gpu", True), ("rdma-hca.sock", True), ("stale-gpu.sock", False)):
            s = so.socket(so.AF_UNIX, so.SOCK_STREAM)
            s.bind(str(d / name))
            if listen:
                s.listen(1)
                socks.append(s)
            else:
                s.close()  # the file stays, nothing listens
        rc, lines = _doctor(tmp_path, "--device-plugin-path", str(d), "--resource-config", "gpu:sharedgpu:4")
    finally:
        for s in socks:
            s.close()
        running.stop()
        k.stop()
    mine = _find(lines, "another instance of this plugin serves")
    assert mine and mine.startswith("warn") and "amd-gpu.sock" in mine, lines
    other = _find(lines, "other device plugins serve here")
    assert other.startswith("warn") and "amd.com_gpu" in other and "rdma-hca.sock" in other, lines
    assert "stale-gpu.sock" not in other
    assert rc == 0, lines  # warnings, not failures


@pytest.mark.parametrize("unit_args,level,says", [
    (["--auto-replica-unit", "mib", "--memory-unit-cu-slots", "proportional"], "warn", "proportional"),
    (["--auto-replica-unit", "mib", "--memory-unit-cu-slots", "whole"], "warn", "sit idle"),
    ([], "ok", "units are CU slots")])
def test_doctor_reports_memory_unit_cu_slots(tmp_path, unit_args, level, says):
    """Memory units with CU shares: MiB units get proportional slots (packed
    neighbours can share one) or whole slots (disjoint, but partly held slots
    idle) -- both warnings; CU-slot units (the default with --replica-cu-mask)
    are disjoint with nothing idle; no line without --replica-cu-mask."""
    d = tmp_path / "dp"
    d.mkdir()
    args = ["--device-plugin-path", str(d), "--resource-config", "gpu:gpu-mem-gb:-1"]
    _, lines = _doctor(tmp_path, *args, "--replica-cu-mask", *unit_args)
    line = _find(lines, "CU shares:")
    assert line and line.split()[0] == level and "amd.com/gpu-mem-gb" in line and says in line, lines
    _, lines = _doctor(tmp_path, *args)
    assert _find(lines, "CU shares:") is None


def test_doctor_reports_the_container_device_order(tmp_path):
    """KFD-node order is how a container numbers its GPUs; the doctor says it
    and whether it differs from amdsmi's enumeration order on this node."""
    fx = fixtures.node(3)
    _, lines = _doctor(tmp_path, "--device-plugin-path", str(tmp_path), fx=fx)
    line = _find(lines, "device order:")
    assert line.startswith("ok") and "amdsmi indices 0,1,2)" in line and "differs" not in line, line
    fx["gpus"][0]["kfd_node"] = 40
    _, lines = _doctor(tmp_path, "--device-plugin-path", str(tmp_path), fx=fx)
    line = _find(lines, "device order:")
    assert "amdsmi indices 1,2,0" in line and "differs from amdsmi's order" in line, line
    fx["gpus"][1]["kfd_node"] = None
    _, lines = _doctor(tmp_path, "--device-plugin-path", str(tmp_path), fx=fx)
    assert _find(lines, "device order:").startswith("warn")


def test_verdicts_in_the_state_file_and_a_waiting_request_are_named(tmp_path):
    """The operator's next question after "why is this GPU out": --doctor names
    each GPU the state file keeps out of service, with the reason and the way
    back, and a return-to-service request nobody took."""
    fx = fixtures.node(2)
    d = tmp_path / "dp"
    d.mkdir()
    state = tmp_path / "health.state"
    state.write_text(f"adp-health v1\n{fx['gpus'][1]['uuid']}\t-\t0\t4\tGPU_PRE_RESET: mode1 reset"
                     "\tgap=the event relay restarted\n")
    drain = tmp_path / "drain"
    (tmp_path / "drain.return").write_text("0\n")
    rc, lines = _doctor(tmp_path, "--device-plugin-path", str(d), "--health-state-file", str(state),
                        "--drain-file", str(drain), fx=fx)
    bdf1 = fx["gpus"][1]["bdf"]
    line = _find(lines, f"GPU {bdf1} is out of service by the state file")
    assert line and line.startswith("warn") and "GPU_PRE_RESET: mode1 reset" in line, lines
    assert f"--return-to-service {bdf1}" in line
    assert "after an event gap -- the event relay restarted -- the polled check returns it" in line
    assert _find(lines, f"GPU {fx['gpus'][0]['bdf']} is out of service") is None
    assert _find(lines, "a return-to-service request is waiting"), lines


def _state_fx(tmp_path, **files):
    """A 2-GPU node whose mock reads runtime knobs from a state directory."""
    state = tmp_path / "state"
    state.mkdir(exist_ok=True)
    for name, body in files.items():
        (state / name).write_text(body)
    return dict(fixtures.node(2), state_dir=str(state))


def test_enumeration_failure_is_a_failure_with_a_hint(tmp_path):
    rc, lines = _doctor(tmp_path, "--device-plugin-path", str(tmp_path), fx=_state_fx(tmp_path, enumerate_fail=""))
    line = _find(lines, "enumeration")
    assert rc == 1 and line.startswith("FAIL") and "amdgpu driver loaded" in line, lines


@pytest.mark.parametrize("args,fx_extra,says", [
    (["--health-events=false"], {}, "health events: off by configuration -- resets are seen by polling only"),
    ([], {"events_supported": False}, "health events: "),
])
def test_health_events_off_is_a_warning_that_says_why(tmp_path, args, fx_extra, says):
    rc, lines = _doctor(tmp_path, "--device-plugin-path", str(tmp_path), *args, fx=dict(fixtures.node(2), **fx_extra))
    line = _find(lines, says)
    assert rc == 0 and line and line.startswith("warn"), lines


def test_ecc_unreadable_on_some_gpus_is_a_warning(tmp_path):
    rc, lines = _doctor(tmp_path, "--device-plugin-path", str(tmp_path), fx=_state_fx(tmp_path, **{"gpu1.ecc": "x"}))
    line = _find(lines, "uncorrectable ECC readable on 1 of 2 GPU(s)")
    assert rc == 0 and line and line.startswith("warn") and "not detected on the others" in line, lines


def test_drain_file_entries_are_checked_against_the_node(tmp_path):
    """--drain-file: the doctor names the GPUs the file takes out of service
    here and the entries that match no GPU of this node (a typo drains
    nothing); a partition's PCI function counts as its GPU."""
    fx = fixtures.node(2, modes="CPX")
    drain = tmp_path / "drain"
    drain.write_text(f"{fx['gpus'][1]['bdf'][:-1]}5  # a partition of GPU 1\n0000:0c:00.9,GPU-nope  # typos\n")
    rc, lines = _doctor(tmp_path, "--device-plugin-path", str(tmp_path), "--partition-strategy", "single",
                        "--drain-file", str(drain), fx=fx)
    got = _find(lines, "drained by the operator")
    assert got and got.startswith("warn") and fx["gpus"][1]["bdf"] in got and fx["gpus"][0]["bdf"] not in got, lines
    bad = _find(lines, "names no GPU of this node")
    assert bad and bad.startswith("warn") and "0000:0c:00.9, GPU-nope" in bad, lines
    assert rc == 0, lines

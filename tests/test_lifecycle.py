"""Daemon lifecycle: restart triggers, signals, init-failure policy, retries.

Parity: reference main.go:205-326 -- failOnInitError (block forever when false),
restart on kubelet.sock re-creation (inotify) and SIGHUP, stop + exit on
SIGINT/SIGTERM/SIGQUIT, restart loop when a plugin fails to start (here with
backoff, fixing B17), and main.go:140-157 flag validation.
"""

import os
import signal
import subprocess
import time

import pytest

from k8s_gpu_sharing_plugin_amd import DAEMON, MOCK_LIB
from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet


def sock(scratch):
    return os.path.join(scratch, "kubelet.sock")


def test_sigterm_stops_and_removes_socket(scratch):
    k = kubelet.StubKubelet(sock(scratch)).start()
    d = harness.Daemon(scratch).start()
    k.wait_registration()
    assert os.path.exists(os.path.join(scratch, "amd-gpu.sock"))
    assert d.stop() == 0
    assert not os.path.exists(os.path.join(scratch, "amd-gpu.sock"))
    assert "shutting down" in d.log()
    k.stop()


@pytest.mark.parametrize("sig", [signal.SIGINT, signal.SIGQUIT])
def test_other_terminating_signals(scratch, sig):
    k = kubelet.StubKubelet(sock(scratch)).start()
    d = harness.Daemon(scratch).start()
    k.wait_registration()
    d.signal(sig)
    assert d.proc.wait(10) == 0
    k.stop()


def test_sighup_restarts_and_reregisters(scratch):
    k = kubelet.StubKubelet(sock(scratch)).start()
    d = harness.Daemon(scratch).start()
    k.wait_registration()
    d.signal(signal.SIGHUP)
    reg = k.wait_registration()
    assert reg.resource_name == "amd.com/gpu"
    assert "received SIGHUP, restarting" in d.log()
    assert d.stop() == 0
    k.stop()


def test_kubelet_restart_is_detected(scratch):
    k = kubelet.StubKubelet(sock(scratch)).start()
    d = harness.Daemon(scratch).start()
    k.wait_registration()
    # the daemon has the Register() response (stopping the stub earlier fails
    # the call, and the retry is a full restart) and its monitor runs
    d.wait_log("health monitor watching")
    k.stop()
    if os.path.exists(sock(scratch)):
        os.unlink(sock(scratch))
    k2 = kubelet.StubKubelet(sock(scratch)).start()  # re-creates kubelet.sock -> inotify
    reg = k2.wait_registration(15)
    assert reg.endpoint == "amd-gpu.sock"
    d.wait_log("kubelet.sock created, restarting")
    c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
    assert len(c.watch()[0].get(timeout=5).devices) == 2
    c.close()
    # the same plugins re-registered: no re-enumeration, the health monitor kept
    log = d.log()
    assert "re-registering plugins (devices and health monitor unchanged)" in log
    assert log.count("health monitor watching") == 1 and log.count("retrieving plugins") == 1
    assert d.stop() == 0
    k2.stop()


def test_deleted_plugin_socket_is_recreated(scratch):
    k = kubelet.StubKubelet(sock(scratch)).start()
    d = harness.Daemon(scratch).start()
    k.wait_registration()
    os.unlink(os.path.join(scratch, "amd-gpu.sock"))
    reg = k.wait_registration(15)  # restarted and registered again
    assert reg.endpoint == "amd-gpu.sock"
    assert os.path.exists(os.path.join(scratch, "amd-gpu.sock"))
    assert "was removed, restarting" in d.log()
    # our own restarts (SIGHUP) must not loop on the deletions they cause
    d.signal(signal.SIGHUP)
    k.wait_registration(15)
    time.sleep(0.5)
    assert d.log().count("was removed, restarting") == 1
    assert d.stop() == 0
    k.stop()


def test_waits_for_kubelet_with_backoff(scratch):
    d = harness.Daemon(scratch, env={}).start()
    d.wait_log("retrying in 1000 ms", timeout=15)
    k = kubelet.StubKubelet(sock(scratch)).start()
    reg = k.wait_registration(20)
    assert reg.resource_name == "amd.com/gpu"
    assert d.stop() == 0
    k.stop()


def test_grpc_crash_budget_is_fatal(scratch):
    """A plugin's gRPC server that keeps crashing (test hook: its first loop
    fails each time it starts) is restarted, and after more than 5 crashes in
    an hour the daemon exits 1 -- the reference's crash budget
    (server.go:191-203), left to the DaemonSet's restart."""
    if not _hooks_compiled():
        pytest.skip("this build has no test hooks (-DADP_TEST_HOOKS=OFF)")
    k = kubelet.StubKubelet(sock(scratch)).start()
    d = harness.Daemon(scratch, env={"ADP_DEBUG_GRPC_LOOP_CRASH": "1"}).start()
    try:
        assert d.proc.wait(20) == 1
        log = d.log()
        assert log.count("crashed: INTERNAL: ADP_DEBUG_GRPC_LOOP_CRASH") == 7, log[-3000:]
        assert "has repeatedly crashed recently; giving up" in log
        assert "exhausted its crash budget; exiting" in log
    finally:
        d.stop()
        k.stop()


def _hooks_compiled():
    from k8s_gpu_sharing_plugin_amd import DAEMON
    return b"ADP_DEBUG_GRPC_LOOP_CRASH" in open(DAEMON, "rb").read()


def test_rejected_registration_retries(scratch):
    k = kubelet.StubKubelet(sock(scratch), reject_with="nope").start()
    d = harness.Daemon(scratch).start()
    d.wait_log("plugin start failed", timeout=15)
    assert "nope" in d.log()
    assert d.proc.poll() is None
    assert d.stop() == 0
    k.stop()


def test_fail_on_init_error_true_exits(scratch):
    fx = fixtures.node(1)
    fx["init_status"] = 8
    d = harness.Daemon(scratch, fx).start()
    assert d.proc.wait(10) == 1
    assert "failed to initialize amdsmi" in d.log()


def test_fail_on_init_error_false_blocks(scratch):
    d = harness.Daemon(scratch, args=["--fail-on-init-error=false"],
                       env={"AMD_SMI_LIB": "/nonexistent/libamd_smi.so"}).start()
    d.wait_log("blocking until terminated")
    time.sleep(0.3)
    assert d.proc.poll() is None
    d.signal(signal.SIGHUP)  # not a terminating signal
    time.sleep(0.2)
    assert d.proc.poll() is None
    assert d.stop() == 0


def test_fail_on_init_error_from_env(scratch):
    d = harness.Daemon(scratch, env={"AMD_SMI_LIB": "/nonexistent.so", "FAIL_ON_INIT_ERROR": "false"}).start()
    d.wait_log("blocking until terminated")
    assert d.stop() == 0


def test_no_devices_waits_indefinitely(scratch):
    k = kubelet.StubKubelet(sock(scratch)).start()
    d = harness.Daemon(scratch, {"gpus": []}).start()
    d.wait_log("no devices found; waiting indefinitely")
    assert k.registrations.empty()
    assert d.stop() == 0
    k.stop()


def test_strategy_error_is_fatal(scratch):
    k = kubelet.StubKubelet(sock(scratch)).start()
    d = harness.Daemon(scratch, fixtures.node(2, ["SPX", "CPX"], memory="NPS2"),
                       args=["--partition-strategy", "single"]).start()
    assert d.proc.wait(10) == 1
    assert "same compute partition mode" in d.log()
    k.stop()


def test_mixed_strategy_runs_one_socket_per_resource(scratch):
    k = kubelet.StubKubelet(sock(scratch)).start()
    d = harness.Daemon(scratch, fixtures.CONFIGS["mixed8"](), args=["--partition-strategy", "mixed"]).start()
    regs = {k.wait_registration().resource_name for _ in range(2)}
    assert regs == {"amd.com/gpu", "amd.com/cpx-1xcd.36gb"}
    assert os.path.exists(os.path.join(scratch, "amd-cpx-1xcd.36gb.sock"))
    assert d.stop() == 0
    k.stop()


@pytest.mark.parametrize("args,msg", [
    (["--device-list-strategy", "bogus"], "invalid --device-list-strategy option: bogus"),
    (["--device-id-strategy", "bogus"], "invalid --device-id-strategy option: bogus"),
    (["--partition-strategy", "bogus"], "invalid --partition-strategy option: bogus"),
    (["--resource-config", "gpu:x"], "invalid --resource-config option"),
    (["--replica-policy", "bogus"], "invalid --replica-policy option"),
    (["--http2-server", "h3"], "invalid --http2-server option"),
    (["--loop-affinity", "numa"], "invalid --loop-affinity option"),
])
def test_invalid_flags(scratch, args, msg):
    d = harness.Daemon(scratch, args=args).start()
    assert d.proc.wait(10) == 1
    assert msg in d.log()


def test_unknown_flag_and_version_and_help():
    r = subprocess.run([DAEMON, "--bogus"], capture_output=True, text=True, timeout=10)
    assert r.returncode == 1 and "flag provided but not defined: --bogus" in r.stderr
    r = subprocess.run([DAEMON, "--version"], capture_output=True, text=True, timeout=10)
    assert r.returncode == 0 and "amdgpu-device-plugin version" in r.stdout
    r = subprocess.run([DAEMON, "--help"], capture_output=True, text=True, timeout=10)
    assert "--partition-strategy" in r.stdout and "FAIL_ON_INIT_ERROR" in r.stdout


def test_dry_run_reports_allocatable(scratch):
    import json
    fx = fixtures.write(fixtures.CONFIGS["mixed8"](), scratch + ".fixture")
    env = dict(os.environ, AMD_SMI_LIB=MOCK_LIB, AMDSMI_MOCK_FIXTURE=fx, ADP_LOG_LEVEL="error")
    r = subprocess.run([DAEMON, "--dry-run", "--partition-strategy", "mixed", "--resource-config",
                        "gpu:gpu:2", "--device-plugin-path", scratch], capture_output=True, text=True,
                       timeout=20, env=env)
    assert r.returncode == 0, r.stderr
    rep = json.loads(r.stdout)
    assert len(rep["gpus"]) == 8
    res = {x["resource"]: x["allocatable"] for x in rep["resources"]}
    assert res == {"amd.com/gpu": 8, "amd.com/cpx-1xcd.36gb": 32}
    assert not os.path.exists(os.path.join(scratch, "amd-gpu.sock"))
    lab = rep["labels"]
    assert lab["amd.com/gpu.count"] == "8" and lab["amd.com/gpu.product"] == "AMD-Instinct-MI355X"
    assert lab["amd.com/gpu.compute-partition"] == "mixed" and lab["amd.com/gpu.interconnect"] == "xgmi-full-mesh"


@pytest.mark.parametrize("rc,needle", [
    ("gpu:gpu:1,cpx-2xcd.72gb:half:1", "resource-config entry 'cpx-2xcd.72gb:half' matches no resource on this node"),
    ("gpu:shared:40000", "above the 4 MiB a kubelet's gRPC client accepts"),
])
def test_dry_run_flags_config_that_cannot_work(scratch, rc, needle):
    """A resource-config key that names no resource here (typo, another node's
    profile) is warned about; a device list too big for the kubelet's gRPC
    client (4 MiB receive limit) is an error in the log."""
    fx = fixtures.write(fixtures.CONFIGS["mixed8"](), scratch + ".fixture")
    env = dict(os.environ, AMD_SMI_LIB=MOCK_LIB, AMDSMI_MOCK_FIXTURE=fx, ADP_LOG_LEVEL="warn")
    r = subprocess.run([DAEMON, "--dry-run", "--partition-strategy", "mixed", "--resource-config", rc,
                        "--device-plugin-path", scratch], capture_output=True, text=True, timeout=60, env=env)
    assert r.returncode == 0, r.stderr
    assert needle in r.stdout + r.stderr
    ok = subprocess.run([DAEMON, "--dry-run", "--partition-strategy", "mixed", "--resource-config",
                         "gpu:gpu:4,cpx-1xcd.36gb:cpx:2", "--device-plugin-path", scratch],
                        capture_output=True, text=True, timeout=60, env=env)
    assert "matches no resource" not in ok.stdout + ok.stderr and "4 MiB" not in ok.stdout + ok.stderr


@pytest.mark.parametrize("cpu_max,threads,spin", [("50000 100000", 1, False), ("300000 100000", 3, True),
                                                   ("max 100000", None, True)])
def test_cpu_limit_sizes_loops_and_busy_poll(scratch, tmp_path, cpu_max, threads, spin):
    """A DaemonSet with resources.limits.cpu: the default loop count follows the
    cgroup CPU quota, and below 2 CPUs the loops block instead of spinning."""
    import json
    import signal
    (tmp_path / "cpu.max").write_text(cpu_max + "\n")
    k = kubelet.StubKubelet(sock(scratch)).start()
    d = harness.Daemon(scratch, env={"ADP_CGROUP_ROOT": str(tmp_path)}).start()
    try:
        k.wait_registration()
        d.signal(signal.SIGUSR1)
        text = d.wait_log("stats: {")
        stats = json.loads([ln for ln in text.splitlines() if "stats: {" in ln][-1].split("stats: ", 1)[1])
        want = threads if threads is not None else min(8, len(os.sched_getaffinity(0)))
        assert stats["server_threads"] == want
        assert ("busy-poll off" in text) is (not spin)
    finally:
        d.stop()
        k.stop()


def test_sigusr1_dumps_stats(scratch):
    k = kubelet.StubKubelet(sock(scratch)).start()
    d = harness.Daemon(scratch).start()
    reg = k.wait_registration()
    c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
    ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
    for _ in range(5):
        c.allocate([ids[0]])
    d.signal(signal.SIGUSR1)
    d.wait_log('"allocate_calls": 5')
    c.close()
    assert d.stop() == 0
    k.stop()


def test_repartition_is_detected_and_reenumerated(scratch):
    """An operator re-partitions GPU 0 (SPX/NPS1 -> CPX/NPS2) under the running
    daemon: polling sees the mode change, amdsmi is re-initialised, the node is
    re-enumerated and the new partition resource registers (the reference needs a
    manual restart after MIG reconfiguration)."""
    fixture_dir = scratch + ".fixture"
    state = os.path.join(fixture_dir, "state")
    os.makedirs(state, exist_ok=True)
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fixtures.node(2), args=["--partition-strategy", "mixed"], state_dir=state,
                       env={"DP_HEALTH_POLL_MS": "100"}).start()
    try:
        assert k.wait_registration().resource_name == "amd.com/gpu"
        fx = fixtures.node(2, ["CPX", "SPX"], memory="NPS2")
        fx["state_dir"] = state
        fixtures.write(fx, fixture_dir)
        with open(os.path.join(state, "gpu0.partition"), "w") as f:
            f.write("CPX NPS2\n")
        names = {k.wait_registration(10).resource_name for _ in range(2)}
        assert "amd.com/gpu" in names
        part = [n for n in names if n != "amd.com/gpu"]
        assert len(part) == 1 and part[0].startswith("amd.com/cpx-1xcd."), names
        log = d.wait_log("amdsmi re-initialised")
        assert "partition mode changed SPX/NPS1 -> CPX/NPS2" in log
        c = kubelet.PluginClient(os.path.join(scratch, "amd-" + part[0].split("/")[1] + ".sock"))
        assert len(c.watch()[0].get(timeout=5).devices) == 8
        c.close()
        time.sleep(0.5)  # several poll periods: no second re-enumeration
        assert d.log().count("amdsmi re-initialised") == 1
    finally:
        assert d.stop() == 0
        k.stop()


@pytest.mark.parametrize("what", ["enumeration", "amdsmi re-init"])
def test_failure_on_restart_is_retried_with_backoff(scratch, what):
    """amdsmi refuses to enumerate, or to initialise again, at a SIGHUP (a
    driver mid-reload): the daemon re-initialises amdsmi and tries again on a
    doubling timer, and serves the same devices once amdsmi works again (the
    reference exits and relies on the pod's restart)."""
    fixture_dir = scratch + ".fixture"
    state = os.path.join(fixture_dir, "state")
    os.makedirs(state, exist_ok=True)
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fixtures.node(2), state_dir=state).start()
    fx = fixtures.node(2)
    fx["state_dir"] = state
    try:
        first = k.wait_registration()
        fail = os.path.join(state, "enumerate_fail")
        if what == "enumeration":
            open(fail, "w").close()
        else:
            fixtures.write(dict(fx, init_status=34), fixture_dir)  # DRIVER_NOT_LOADED
        d.signal(signal.SIGHUP)
        d.wait_log(what + " failed; retrying in 1000 ms", timeout=10)
        d.wait_log(what + " failed; retrying in 2000 ms", timeout=10)  # the timer's retry, failing again
        if what == "enumeration":
            os.unlink(fail)
        else:
            fixtures.write(fx, fixture_dir)
        reg = k.wait_registration(10)
        assert reg.resource_name == first.resource_name and reg.endpoint == first.endpoint
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        assert len(c.watch()[0].get(timeout=5).devices) == 2
        c.close()
        log = d.log()
        assert log.count("device enumeration failed" if what == "enumeration"
                         else "amdsmi re-initialisation failed") == 2
        assert "amdsmi re-initialised" in log
    finally:
        assert d.stop() == 0
        k.stop()


def _cpu_seconds(pid):
    with open(f"/proc/{pid}/stat") as f:
        fields = f.read().rsplit(")", 1)[1].split()
    return (int(fields[11]) + int(fields[12])) / os.sysconf("SC_CLK_TCK")  # utime + stime


def test_idle_daemon_uses_no_cpu(scratch):
    """Busy-polling only follows activity: an idle daemon (after a burst of RPCs)
    sleeps in epoll_wait and burns no CPU."""
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fixtures.node(8), args=["--busy-poll-us", "1000"]).start()
    try:
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        law = c.watch()[0].get(timeout=5)
        for x in law.devices:
            c.allocate([x.ID])
        time.sleep(0.2)
        before = _cpu_seconds(d.proc.pid)
        time.sleep(2.0)
        used = _cpu_seconds(d.proc.pid) - before
        assert used < 0.1, f"idle daemon used {used:.2f} CPU-s in 2 s"
        c.close()
    finally:
        assert d.stop() == 0
        k.stop()


def test_xgmi_link_loss_rescores_topology(scratch):
    """xGMI links of GPU 2 go down: after two polls the node is re-enumerated and
    GetPreferredAllocation steers a 2-GPU pod away from the degraded GPU."""
    state = os.path.join(scratch + ".fixture", "state")
    os.makedirs(state, exist_ok=True)
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fixtures.node(4), state_dir=state, env={"DP_HEALTH_POLL_MS": "100"}).start()
    try:
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
        avail = ids[1:4]
        before = list(c.preferred(avail, size=2).container_responses[0].deviceIDs)
        assert ids[2] in before  # equal scores: the lowest-index pair
        c.close()
        with open(os.path.join(state, "gpu2.xgmi_down"), "w") as f:
            f.write("3\n")
        k.wait_registration(10)  # re-registered after re-enumeration
        log = d.wait_log("amdsmi re-initialised")
        assert "xGMI links down 0 -> 3" in log
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        c.watch()[0].get(timeout=5)
        after = list(c.preferred(avail, size=2).container_responses[0].deviceIDs)
        assert sorted(after) == sorted([ids[1], ids[3]])
        c.close()
        time.sleep(0.5)
        assert d.log().count("amdsmi re-initialised") == 1
    finally:
        assert d.stop() == 0
        k.stop()


def test_node_labels_file_for_nfd(scratch):
    """--node-labels-file: node-feature-discovery local-source file, rewritten on
    every re-enumeration and removed when the daemon exits."""
    path = os.path.join(scratch + ".fixture", "amd-gpu.features")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    k = kubelet.StubKubelet(sock(scratch)).start()
    d = harness.Daemon(scratch, fixtures.node(4, "CPX", memory="NPS2"),
                       args=["--node-labels-file", path, "--partition-strategy", "single"]).start()
    try:
        k.wait_registration()
        d.wait_log("wrote node labels")
        labels = dict(line.split("=", 1) for line in open(path).read().splitlines())
        assert labels == {
            "amd.com/gpu.present": "true", "amd.com/gpu.count": "4",
            "amd.com/gpu.product": "AMD-Instinct-MI355X", "amd.com/gpu.memory-mib": str(fixtures.MI355X_VRAM_MIB),
            "amd.com/gpu.compute-partition": "CPX", "amd.com/gpu.memory-partition": "NPS2",
            "amd.com/gpu.partitions": "32", "amd.com/gpu.partition-profile": "cpx-1xcd.36gb",
            "amd.com/gpu.interconnect": "xgmi-full-mesh", "amd.com/gpu.xgmi-links-down": "0"}
        assert all(len(v) <= 63 for v in labels.values())
    finally:
        assert d.stop() == 0
        k.stop()
    assert not os.path.exists(path)


def test_python_cli_report_on_mock(scratch):
    import sys
    fx = fixtures.write(fixtures.CONFIGS["mixed8"](), scratch + ".fixture")
    env = dict(os.environ, AMD_SMI_LIB=MOCK_LIB, AMDSMI_MOCK_FIXTURE=fx, ADP_LOG_LEVEL="error")
    r = subprocess.run([sys.executable, "-m", "k8s_gpu_sharing_plugin_amd", "report", "--partition-strategy", "mixed",
                        "--device-plugin-path", scratch], capture_output=True, text=True, timeout=60, env=env)
    assert r.returncode == 0, r.stderr
    assert "amd.com/cpx-1xcd.36gb" in r.stdout and "amd.com/gpu.count=8" in r.stdout
    h = subprocess.run([sys.executable, "-m", "k8s_gpu_sharing_plugin_amd", "--help"], capture_output=True, text=True)
    assert h.returncode == 0 and "validate" in h.stdout


@pytest.mark.parametrize("fixture_name,args", [
    ("spx8", ["--resource-config", "gpu:gpu-mem-gb:-1"]),
    ("cpx8", ["--partition-strategy", "single"]),
    ("mixed8", ["--partition-strategy", "mixed", "--resource-config", "gpu:sharedgpu:3"]),
])
def test_device_ids_survive_daemon_restarts(scratch, fixture_name, args):
    """The kubelet checkpoints allocated IDs across plugin restarts (SURVEY §5,
    checkpoint/resume): every advertised ID -- replicas and partitions included --
    must be identical after the daemon is restarted from scratch."""
    def advertised():
        k = kubelet.StubKubelet(sock(scratch)).start()
        d = harness.Daemon(scratch, fixtures.CONFIGS[fixture_name](), args=args).start()
        try:
            out = {}
            regs = 2 if fixture_name == "mixed8" else 1
            for _ in range(regs):
                reg = k.wait_registration()
                c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
                out[reg.resource_name] = sorted(x.ID for x in c.watch()[0].get(timeout=5).devices)
                c.close()
            return out
        finally:
            assert d.stop() == 0
            k.stop()
    first = advertised()
    second = advertised()
    assert first == second and all(first.values())
    assert all(len(i) <= 63 for ids in first.values() for i in ids)


def test_json_log_format(scratch):
    import json
    k = kubelet.StubKubelet(sock(scratch)).start()
    d = harness.Daemon(scratch, env={"ADP_LOG_FORMAT": "json"}).start()
    try:
        k.wait_registration()
        d.wait_log("registered device plugin")
    finally:
        assert d.stop() == 0
        k.stop()
    recs = [json.loads(line) for line in d.log().splitlines() if line.strip()]
    assert recs and all({"ts", "level", "component", "msg"} <= set(r) for r in recs)
    cfg = [r for r in recs if r["msg"].startswith("running with config:")]
    assert cfg and "\n" in cfg[0]["msg"]  # multi-line messages stay one record


def test_config_file_changes_are_applied_live(scratch):
    """Editing the config file (atomic replace, like a ConfigMap update) reloads
    it and re-registers with the new resources; a broken edit is ignored."""
    cfg_dir = scratch + ".fixture"
    os.makedirs(cfg_dir, exist_ok=True)
    path = os.path.join(cfg_dir, "config.yaml")

    def write(body):
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            f.write(body)
        os.rename(tmp, path)
    write("version: v1\nflags:\n  resourceConfig: gpu:sharedgpu:2\n")
    k = kubelet.StubKubelet(sock(scratch)).start()
    d = harness.Daemon(scratch, args=["--config-file", path]).start()
    try:
        reg = k.wait_registration()
        assert reg.resource_name == "amd.com/sharedgpu"
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        assert len(c.watch()[0].get(timeout=5).devices) == 4
        c.close()
        write("version: v1\nflags:\n  resourceConfig: gpu:sharedgpu:3\n")
        reg = k.wait_registration(10)
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        assert len(c.watch()[0].get(timeout=5).devices) == 6
        c.close()
        write("version: v2\n")  # invalid: logged, running config kept
        d.wait_log("config not reloaded")
        write("version: v1\nflags:\n  resourceConfig: gpu:timeshared:1\n")
        assert k.wait_registration(10).resource_name == "amd.com/timeshared"
        # SIGHUP re-reads too (environment / flags / file)
        write("version: v1\nflags:\n  resourceConfig: gpu:sharedgpu:5\n  deviceIDStrategy: index\n")
        reg = k.wait_registration(10)
        assert reg.resource_name == "amd.com/sharedgpu"
        d.signal(signal.SIGHUP)
        reg = k.wait_registration(10)
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        assert len(c.watch()[0].get(timeout=5).devices) == 10
        c.close()
        assert "reloaded config" in d.log()
    finally:
        assert d.stop() == 0
        k.stop()


def test_configmap_style_update_is_applied(scratch):
    """Kubernetes updates a mounted ConfigMap by swapping the `..data` symlink."""
    cm = scratch + ".cm"
    os.makedirs(cm, exist_ok=True)

    def publish(n, body):
        ts = os.path.join(cm, f"..ts{n}")
        os.makedirs(ts)
        with open(os.path.join(ts, "config.yaml"), "w") as f:
            f.write(body)
        tmp = os.path.join(cm, "..data_tmp")
        os.symlink(f"..ts{n}", tmp)
        os.rename(tmp, os.path.join(cm, "..data"))
    publish(1, "version: v1\nflags:\n  resourceConfig: gpu:sharedgpu:2\n")
    os.symlink("..data/config.yaml", os.path.join(cm, "config.yaml"))
    k = kubelet.StubKubelet(sock(scratch)).start()
    d = harness.Daemon(scratch, args=["--config-file", os.path.join(cm, "config.yaml")]).start()
    try:
        assert k.wait_registration().resource_name == "amd.com/sharedgpu"
        publish(2, "version: v1\nflags:\n  resourceConfig: gpu:cmgpu:2\n")
        assert k.wait_registration(10).resource_name == "amd.com/cmgpu"
    finally:
        assert d.stop() == 0
        k.stop()


def test_devices_filter_by_index_uuid_and_pci_address(scratch):
    import json
    fx = fixtures.node(4)
    path = fixtures.write(fx, scratch + ".fixture")
    env = dict(os.environ, AMD_SMI_LIB=MOCK_LIB, AMDSMI_MOCK_FIXTURE=path, ADP_LOG_LEVEL="error")
    uuid2 = fx["gpus"][2]["uuid"]
    bdf3 = fx["gpus"][3]["bdf"]            # "0000:6c:00.0"
    short1 = fx["gpus"][1]["bdf"][5:-2]    # "2c:00" (no domain, no function)
    r = subprocess.run([DAEMON, "--dry-run", "--devices", f"0,{uuid2.upper()},{bdf3},{short1}",
                        "--device-plugin-path", scratch], capture_output=True, text=True, timeout=20, env=env)
    assert r.returncode == 0, r.stderr
    got = sorted(g["uuid"] for g in json.loads(r.stdout)["gpus"])
    assert got == sorted(fx["gpus"][i]["uuid"] for i in range(4))
    r = subprocess.run([DAEMON, "--dry-run", "--devices", uuid2, "--device-plugin-path", scratch],
                       capture_output=True, text=True, timeout=20, env=env)
    assert [g["uuid"] for g in json.loads(r.stdout)["gpus"]] == [uuid2]


@pytest.mark.parametrize("args", [["--http2-server", "nghttp2", "--loop-affinity", "none"],
                                  ["--http2-server", "native", "--loop-affinity", "peer-l3"]])
def test_engine_and_affinity_options_serve(scratch, args):
    k = kubelet.StubKubelet(sock(scratch)).start()
    d = harness.Daemon(scratch, args=args, env={"ADP_LOG_LEVEL": "debug"}).start()
    reg = k.wait_registration()
    c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
    ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
    assert c.allocate(ids[:1]).container_responses[0].devices
    c.close()
    # peer-l3 follows the (visible) caller; none never moves a loop
    if os.path.exists("/sys/devices/system/cpu/cpu0/cache/index3/shared_cpu_list"):
        assert ("served from its L3" in d.log()) == ("peer-l3" in args)
    assert d.stop() == 0
    k.stop()


def _foreign_socket(path):
    """A listening Unix socket bound at `path` by this process (another plugin instance)."""
    import socket as so
    s = so.socket(so.AF_UNIX, so.SOCK_STREAM)
    s.bind(path)
    s.listen(1)
    return s


def test_replaced_socket_is_not_removed_on_stop(scratch):
    """A second instance (DaemonSet rollout with maxSurge) that atomically
    replaced our socket file keeps it when we stop: Stop() removes only the
    file it bound. (The reference removes its socket path unconditionally.)"""
    k = kubelet.StubKubelet(sock(scratch)).start()
    d = harness.Daemon(scratch).start()
    k.wait_registration()
    path = os.path.join(scratch, "amd-gpu.sock")
    other = _foreign_socket(path + ".new")
    os.rename(path + ".new", path)  # atomic takeover: no delete event for the old file
    ino = os.stat(path).st_ino
    assert d.stop() == 0
    assert os.path.exists(path) and os.stat(path).st_ino == ino
    other.close()
    k.stop()


def test_takeover_by_another_instance_stands_by(scratch):
    """Our socket unlinked and bound again by another process: no tug of war
    (re-binding would unlink theirs in turn); we log that we stand by, do not
    re-register, and leave their socket on exit."""
    k = kubelet.StubKubelet(sock(scratch)).start()
    d = harness.Daemon(scratch).start()
    k.wait_registration()
    path = os.path.join(scratch, "amd-gpu.sock")
    # Frozen while the other instance unlinks and binds, so the daemon reads
    # the delete event only once the new file is in place (deterministic).
    d.signal(signal.SIGSTOP)
    try:
        os.unlink(path)
        other = _foreign_socket(path)
    finally:
        d.signal(signal.SIGCONT)
    ino = os.stat(path).st_ino
    d.wait_log("now belongs to another process")
    time.sleep(1.5)  # longer than a restart's first backoff
    assert "was removed, restarting" not in d.log()
    assert os.stat(path).st_ino == ino
    assert d.stop() == 0
    assert os.path.exists(path) and os.stat(path).st_ino == ino
    other.close()
    k.stop()


def test_unlink_then_bind_takeover_stands_by(scratch):
    """The other instance's real sequence, unfrozen: unlink our socket, then
    bind its own microseconds later. The daemon looks again before taking the
    path back, sees the new file and stands by."""
    k = kubelet.StubKubelet(sock(scratch)).start()
    d = harness.Daemon(scratch).start()
    k.wait_registration()
    path = os.path.join(scratch, "amd-gpu.sock")
    os.unlink(path)
    other = _foreign_socket(path)
    ino = os.stat(path).st_ino
    d.wait_log("now belongs to another process")
    time.sleep(1.5)
    assert "was removed, restarting" not in d.log()
    assert os.stat(path).st_ino == ino
    assert d.stop() == 0
    assert os.stat(path).st_ino == ino
    other.close()
    k.stop()


def test_sigterm_during_the_socket_recheck_exits_at_once(scratch):
    """A deleted plugin socket is looked at again from a one-shot timer, not a
    sleep inside the event loop: signals and kubelet events are handled in the
    meantime. With the re-check window widened to 5 s, SIGTERM right after the
    delete still exits at once (the old usleep held the loop for the window)."""
    k = kubelet.StubKubelet(sock(scratch)).start()
    d = harness.Daemon(scratch, env={"ADP_DEBUG_SOCKET_RECHECK_MS": "5000"}).start()
    k.wait_registration()
    os.unlink(os.path.join(scratch, "amd-gpu.sock"))
    time.sleep(0.2)  # the delete event is read and the re-check armed
    t = time.monotonic()
    assert d.stop() == 0
    assert time.monotonic() - t < 2.0
    assert "was removed, restarting" not in d.log()  # the re-check never ran
    k.stop()


def test_socket_recheck_window_reregisters_after_it(scratch):
    """The deleted socket stays deleted through the window: the daemon
    re-registers once the timer fires."""
    k = kubelet.StubKubelet(sock(scratch)).start()
    d = harness.Daemon(scratch, env={"ADP_DEBUG_SOCKET_RECHECK_MS": "300"}).start()
    k.wait_registration()
    os.unlink(os.path.join(scratch, "amd-gpu.sock"))
    t = time.monotonic()
    d.wait_log("was removed, restarting", timeout=5)
    assert time.monotonic() - t >= 0.25
    k.wait_registration()
    assert os.path.exists(os.path.join(scratch, "amd-gpu.sock"))
    assert d.stop() == 0
    k.stop()


def test_a_standing_by_instance_pauses_its_health_monitor(scratch, tmp_path):
    """Once another instance serves every socket, this one's health monitor
    pauses: the serving instance owns the verdicts -- the state file both
    would write, and the operator's return-to-service requests, which the
    standing-by one must not take. When the kubelet restarts (the socket
    disappears), it serves again with a monitor reading the other instance's
    verdicts from the state file."""
    drain = tmp_path / "drain"
    state = tmp_path / "health.state"
    fx = fixtures.node(2)
    k = kubelet.StubKubelet(sock(scratch)).start()
    d = harness.Daemon(scratch, fx, args=["--drain-file", str(drain), "--health-state-file", str(state)],
                       env={"DP_HEALTH_POLL_MS": "100"}).start()
    try:
        k.wait_registration()
        d.wait_log("health poll #1")
        path = os.path.join(scratch, "amd-gpu.sock")
        d.signal(signal.SIGSTOP)
        try:
            os.unlink(path)
            other = _foreign_socket(path)
        finally:
            d.signal(signal.SIGCONT)
        d.wait_log("its health monitor pauses")
        req = str(drain) + ".return"
        with open(req, "w") as f:
            f.write(fx["gpus"][0]["bdf"] + "\n")
        time.sleep(0.6)  # six polls of a running monitor
        assert os.path.exists(req), "the standing-by instance took the request:\n" + d.log()[-3000:]
        # the other instance's verdicts, as it writes them
        state.write_text(f"adp-health v1\n{fx['gpus'][1]['uuid']}\t-\t0\t4\tGPU_PRE_RESET: seen by the other\n")
        os.unlink(req)
        other.close()
        os.unlink(path)  # the other instance is gone; the kubelet restarts
        k.stop()
        k = kubelet.StubKubelet(sock(scratch)).start()
        k.wait_registration(15)
        log = d.wait_log("stays unhealthy from an earlier generation")
        assert "GPU_PRE_RESET: seen by the other" in log
    finally:
        d.stop()
        k.stop()

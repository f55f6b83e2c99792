"""HBM caps for memory-unit sharing (--enforce-memory-units, libadp_memcap.so).

The reference hands out `gpu-mem-gb` units without telling or limiting the
workload (server.go:99-111). Here Allocate() of a memory-unit resource can
mount + preload a shim that refuses HIP allocations past the granted HBM and
reports the grant as the device's memory. CPU: the shim in front of a
libamdhip64 stand-in, called through the PLT like a framework does, and the
daemon's Allocate() responses on the amdsmi mock. The real-HIP / PyTorch run is
tests/test_gpu.py::test_memcap_caps_torch_allocations.
"""

import glob
import re
import json
import os
import subprocess
import time

import hypothesis
import pytest
from hypothesis import strategies as st

from k8s_gpu_sharing_plugin_amd import BUILD_DIR
from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet

SHIM = os.path.join(BUILD_DIR, "libadp_memcap.so")
# The shim after whatever this environment already preloads.
PRELOAD = " ".join(x for x in (os.environ.get("LD_PRELOAD", ""), SHIM) if x)
CHECK = os.path.join(BUILD_DIR, "adp_memcap_check")


# Every grant key of this file carries the test process's tag, so the cleanup
# below never removes a segment a concurrent test process (pytest -n) still uses.
TAG = f"w{os.getpid()}"


def _key(name):
    return f"{TAG}-{name}-{time.monotonic_ns()}"


@pytest.fixture(autouse=True)
def _no_leftover_segments():
    """The shim's container-wide counters live in /dev/shm/adp-memcap-key-*;
    drop the ones a test created (in a pod they go with the pod)."""
    yield
    for f in glob.glob(f"/dev/shm/adp-memcap-key-{TAG}-*"):
        os.unlink(f)


def _run(env_extra, *args):
    env = dict(os.environ, **env_extra)
    env.setdefault("ADP_MEMCAP_KEY", _key("test"))
    r = subprocess.run([CHECK, *args], capture_output=True, text=True, timeout=60, env=env)
    assert r.returncode == 0, r.stderr
    return {d["step"]: d for d in map(json.loads, r.stdout.splitlines())}, r.stderr


def test_without_the_shim_nothing_is_capped():
    out, _ = _run({})
    assert out["d0 malloc 50"]["rc"] == 0 and out["d0 info"]["total_mib"] == 294912


def test_caps_per_device_in_hip_order():
    out, err = _run({"LD_PRELOAD": PRELOAD, "AMD_GPU_MEMORY_LIMIT_MIB": "100,50"})
    oom = 2  # hipErrorOutOfMemory
    # device 0: 100 MiB
    assert out["d0 malloc 60"]["rc"] == 0
    assert out["d0 malloc 50"]["rc"] == oom and out["d0 refused ptr"]["null"]
    assert (out["d0 info"]["free_mib"], out["d0 info"]["total_mib"]) == (40, 100)
    assert out["d0 malloc 50 again"]["rc"] == 0  # after the free
    assert out["d0 info after"]["free_mib"] == 50
    assert out["d0 info pitch"]["free_mib"] == 49  # counted at the padded pitch, once
    assert out["d0 memcreate 60"]["rc"] == oom and out["d0 memcreate 40"]["rc"] == 0  # VMM handles
    assert out["d0 info vmm"]["free_mib"] == 50  # released
    # device 1: 50 MiB, stream-ordered allocations on a device-1 stream
    assert out["d1 malloc 60"]["rc"] == oom
    assert out["d1 mallocasync 40"]["rc"] == 0 and out["d1 mallocasync 20"]["rc"] == oom
    assert out["d1 mallocasync 20 again"]["rc"] == 0  # after hipFreeAsync
    assert (out["d1 info"]["free_mib"], out["d1 info"]["total_mib"]) == (30, 50)
    assert out["d1 totalmem value"]["mib"] == 50
    # device 2: past the list, not capped
    assert out["d2 malloc 100000"]["rc"] == 0 and out["d2 info"]["total_mib"] == 294912
    assert out["props"] == {"step": "props", "d0_mib": 100, "d2_mib": 294912}
    assert "device 0: refused 50.0 MiB (60.0 of 100.0 MiB in use" in err  # once per device


def test_accounting_is_exact_under_concurrent_allocations():
    """8 threads x 20k sync / stream-ordered allocations and frees against a
    40 MiB cap (one thread alone holds more than that): some are refused, and
    when all is freed the whole cap is free."""
    out, _ = _run({"LD_PRELOAD": PRELOAD, "AMD_GPU_MEMORY_LIMIT_MIB": "40"}, "stress")
    assert out["stress"]["granted"] > 1000 and out["stress"]["refused"] > 100
    assert (out["stress info"]["free_mib"], out["stress info"]["total_mib"]) == (40, 40)


def _env(key, cap="100"):
    return dict(os.environ, LD_PRELOAD=PRELOAD, AMD_GPU_MEMORY_LIMIT_MIB=cap, ADP_MEMCAP_KEY=key)


def _hold(env, mib):
    p = subprocess.Popen([CHECK, "hold", "0", str(mib)], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                         stderr=subprocess.DEVNULL, text=True, env=env)
    first = json.loads(p.stdout.readline())
    assert first == {"step": "hold", "rc": 0}
    p.stdout.readline()  # info
    return p


def _try(env, mib):
    r = subprocess.run([CHECK, "try", "0", str(mib)], capture_output=True, text=True, timeout=30, env=env)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(ln) for ln in r.stdout.splitlines()]
    return lines[0]["rc"], lines[1]["free_mib"]


def test_processes_of_a_container_share_one_grant():
    """The grant is the container's: a second process gets what the first left
    over, and a process that exits gives its bytes back."""
    env = _env(_key("share"))
    a = _hold(env, 60)
    try:
        assert _try(env, 50) == (2, 40)  # refused: 60 of 100 held by the other process
        assert _try(env, 40) == (0, 0)   # fits, and is given back when that process exits
        assert _try(env, 40) == (0, 0)
    finally:
        a.stdin.close()
        assert a.wait(10) == 0
    assert _try(env, 90) == (0, 10)  # the holder exited normally: its 60 MiB are back


def test_bytes_of_a_killed_process_are_reclaimed():
    import signal
    env = _env(_key("kill"))
    a = _hold(env, 60)
    a.send_signal(signal.SIGKILL)
    a.wait(10)
    assert _try(env, 90) == (0, 10)  # the dead holder's slot was reclaimed on the refusal path


def test_forked_child_draws_on_the_same_grant():
    env = _env(_key("fork"))
    r = subprocess.run([CHECK, "fork", "60"], capture_output=True, text=True, timeout=30, env=env)
    out = {d["step"]: d for d in map(json.loads, r.stdout.splitlines())}
    assert out["parent malloc"]["rc"] == 0
    assert out["child malloc full"]["rc"] == 2 and out["child malloc half"]["rc"] == 0
    assert out["parent info after child"]["free_mib"] == 40  # the child's 30 MiB came back at its exit


def test_other_grants_and_other_containers_are_separate():
    key = _key("sep")
    a = _hold(_env(key), 60)
    try:
        assert _try(_env(key + "-other"), 90) == (0, 10)  # another container
        assert _try(_env(key, cap="200"), 150) == (0, 50)  # another grant
    finally:
        a.stdin.close()
        a.wait(10)


def test_shim_exports_hip_versioned_entry_points_only():
    r = subprocess.run(["nm", "-D", "--defined-only", SHIM], capture_output=True, text=True, check=True)
    syms = {ln.split()[-1] for ln in r.stdout.splitlines() if " T " in ln}
    assert {"hipMalloc@@hip_4.2", "hipFree@@hip_4.2", "hipMemGetInfo@@hip_4.2", "hipMallocAsync@@hip_5.1",
            "hipMemCreate@@hip_5.1", "hipGetDevicePropertiesR0600@@hip_6.0", "hipGetDeviceProperties@@hip_4.2",
            "hipMalloc3D@@hip_4.2", "hipMallocArray@@hip_4.2", "hipMalloc3DArray@@hip_4.2",
            "hipArrayCreate@@hip_4.2", "hipArray3DCreate@@hip_4.2", "hipArrayDestroy@@hip_4.3",
            "hipMemAllocPitch@@hip_4.2", "hipMallocMipmappedArray@@hip_4.2"} <= syms
    # every interposed symbol carries the version node the real library gives it
    real = subprocess.run(["objdump", "-T", "/opt/rocm/lib/libamdhip64.so"], capture_output=True, text=True)
    if real.returncode == 0:
        nodes = {ln.split()[-1]: ln.split()[-2] for ln in real.stdout.splitlines() if " hip" in ln and "DF" in ln}
        for sym in syms:
            name, node = sym.split("@@")
            assert nodes.get(name, node) == node, (sym, nodes.get(name))
    assert all(s.startswith("hip") for s in syms), syms
    r = subprocess.run(["ldd", SHIM], capture_output=True, text=True, check=True)
    assert "libamdhip64" not in r.stdout and "libstdc++" not in r.stdout  # resolved at run time; no C++ runtime


def test_shim_loads_into_old_glibc_images():
    """PyTorch-ROCm wheels target glibc 2.28 (manylinux_2_28): the shim imports
    only libc symbols at versions every glibc since 2.4 has, nothing from the
    C++ runtime, and runs no initialiser when it is preloaded."""
    import re
    r = subprocess.run(["objdump", "-T", SHIM], capture_output=True, text=True, check=True)
    versions = set(re.findall(r"\((GLIBC_[0-9.]+)\)", r.stdout))
    newest = max(tuple(int(x) for x in v[6:].split(".")) for v in versions)
    assert newest <= (2, 4), sorted(versions)
    undefined = [ln.split()[-1] for ln in r.stdout.splitlines() if "*UND*" in ln]
    assert not [u for u in undefined if u.startswith("_Z") or "cxa_guard" in u or "gxx" in u], undefined
    nm = subprocess.run(["nm", SHIM], capture_output=True, text=True, check=True).stdout
    assert "_GLOBAL__sub_I" not in nm  # nothing runs at load: the state is constant-initialised


def _allocate(scratch, rc, extra=(), take=3, enforce=True):
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    args = ["--resource-config", rc, "--replica-policy", "pack", *extra]
    if enforce:
        args += ["--enforce-memory-units", "--memcap-lib", SHIM]
    d = harness.Daemon(scratch, args=args).start()
    try:
        reg = k.wait_registration()
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
        resp = c.allocate(ids[:take]).container_responses[0]
        c.close()
        return resp, d.log()
    finally:
        d.stop()
        k.stop()


def test_memory_unit_pods_get_the_shim(scratch):
    resp, log = _allocate(scratch, "gpu:gpu-mem-gb:-1")
    envs = dict(resp.envs)
    installed = os.path.join(scratch, "amdgpu-dp", "libadp_memcap.so")
    assert envs["LD_PRELOAD"] == "/usr/local/lib/amdgpu-dp/libadp_memcap.so"
    assert envs["AMD_GPU_MEMORY_LIMIT_MIB"] == "3000"
    # the device reports the grant as its memory under the shim: the fraction of it is 1
    assert envs["AMD_GPU_MEMORY_FRACTION"] == "1.0000"
    mounts = [(m.container_path, m.host_path, m.read_only) for m in resp.mounts]
    grant = os.path.join(scratch, "amdgpu-dp", "grants", "3000.mib")
    # the shim, and the grant itself, read-only, one file per device in HIP order
    assert mounts == [("/usr/local/lib/amdgpu-dp/libadp_memcap.so", installed, True),
                      ("/run/amdgpu-dp/grant/0", grant, True)]
    assert open(installed, "rb").read() == open(SHIM, "rb").read()
    assert open(grant).read() == "3000\n" and os.stat(grant).st_mode & 0o222 == 0
    # every grant size a device can be given was written before registration
    sizes = sorted(int(f[:-4]) for f in os.listdir(os.path.dirname(grant)))
    assert sizes == [1000 * k for k in range(1, 295)]
    assert "HBM-cap shim installed at" in log


def _grant_dir(tmp_path, *mib):
    d = tmp_path / "grant"
    d.mkdir()
    for i, m in enumerate(mib):
        (d / str(i)).write_text(f"{m}\n")
    return str(d)


@pytest.mark.parametrize("env_value", [None, "", "999999,999999", "abc", "0,0"])
def test_daemon_grant_cannot_be_raised_or_dropped_from_the_env(tmp_path, env_value):
    """The grant files the daemon mounts read-only are the caps: a pod that
    empties, drops or raises AMD_GPU_MEMORY_LIMIT_MIB still gets 100/50 MiB."""
    env = {"LD_PRELOAD": PRELOAD, "ADP_MEMCAP_GRANT_DIR": _grant_dir(tmp_path, 100, 50)}
    if env_value is not None:
        env["AMD_GPU_MEMORY_LIMIT_MIB"] = env_value
    base = dict(os.environ)
    base.pop("AMD_GPU_MEMORY_LIMIT_MIB", None)
    r = subprocess.run([CHECK], capture_output=True, text=True, timeout=60,
                       env=dict(base, ADP_MEMCAP_KEY=_key("grant"), **env))
    assert r.returncode == 0, r.stderr
    out = {d["step"]: d for d in map(json.loads, r.stdout.splitlines())}
    assert out["d0 malloc 50"]["rc"] == 2 and out["d0 info"]["total_mib"] == 100
    assert out["d1 malloc 60"]["rc"] == 2 and out["d1 totalmem value"]["mib"] == 50
    assert out["d2 info"]["total_mib"] == 294912  # not granted, not capped


def test_env_can_only_lower_the_daemon_grant(tmp_path):
    out, _ = _run({"LD_PRELOAD": PRELOAD, "ADP_MEMCAP_GRANT_DIR": _grant_dir(tmp_path, 100, 50),
                   "AMD_GPU_MEMORY_LIMIT_MIB": "80,500,20"})
    assert out["d0 info"]["total_mib"] == 80       # lowered
    assert out["d1 totalmem value"]["mib"] == 50   # 500 > grant: the grant stands
    assert out["d2 info"]["total_mib"] == 20       # past the grant: the env still caps


def test_stream_ordered_pools_never_hold_memory_past_the_cap():
    """hipMallocAsync -> hipFreeAsync keeps the block in the pool (reserved);
    the shim counts it until a refusal trims the pools and reads back what they
    still hold, so the device (mock: live allocations + pool reserve) never
    holds more than the grant."""
    out, _ = _run({"LD_PRELOAD": PRELOAD, "AMD_GPU_MEMORY_LIMIT_MIB": "100"}, "pool")
    assert out["phys after freeasync"]["physical_mib"] == 80   # the pool keeps the freed block
    assert out["info after freeasync"]["free_mib"] == 100      # reported as free: it can be trimmed
    assert out["malloc 50"]["rc"] == 0 and out["phys after malloc 50"]["physical_mib"] == 50  # trimmed first
    assert out["malloc 40"]["rc"] == 0 and out["phys after malloc 40"]["physical_mib"] == 100
    assert out["malloc 10"]["rc"] == 2 and out["phys after malloc 10"]["physical_mib"] == 100
    assert out["frompool 30"]["rc"] == 0 and out["malloc 100"]["rc"] == 0
    assert out["phys after malloc 100"]["physical_mib"] == 100
    assert max(v["physical_mib"] for v in out.values() if "physical_mib" in v) <= 100
    assert (out["info end"]["free_mib"], out["info end"]["total_mib"]) == (100, 100)


@pytest.mark.parametrize("delay_us", ["0", "50"])
def test_pool_trim_racing_stream_ordered_allocations_never_passes_the_cap(delay_us):
    """Advisor round 3: ReconcilePools read a pool's reserve without the lock,
    then subtracted a pool_live that another thread's hipMallocAsync had grown
    meanwhile -- giving back bytes the pool still held, so later allocations
    passed the grant (the pre-fix shim let the mock device reach 110-120 MiB
    under a 100 MiB cap in 2 of 5 runs of this check). Now the reserve is
    applied only when no stream-ordered allocation or free moved in between."""
    for _ in range(5):
        out, _ = _run({"LD_PRELOAD": PRELOAD, "AMD_GPU_MEMORY_LIMIT_MIB": "100",
                       "HIP_MOCK_POOL_ATTR_DELAY_US": delay_us}, "poolrace")
        r = out["poolrace"]
        assert r["max_physical_mib"] <= 100.0, r
        assert r["async_ok"] > 1000 and r["sync_ok"] > 500, r  # the trims still give memory back
        assert (out["poolrace info"]["free_mib"], out["poolrace info"]["total_mib"]) == (100, 100)


def test_without_the_shim_a_pool_holds_past_the_cap():
    """The same sequence uncapped: the pool's reserve plus the next hipMalloc
    is what the shim has to bound (80 + 50 here)."""
    out, _ = _run({}, "pool")
    assert out["phys after malloc 50"]["physical_mib"] == 130


def test_arrays_3d_mipmaps_and_overflowing_sizes_are_capped():
    out, err = _run({"LD_PRELOAD": PRELOAD, "AMD_GPU_MEMORY_LIMIT_MIB": "100"}, "arrays")
    oom = 2
    assert out["array 16"]["rc"] == 0 and out["3darray 128"]["rc"] == oom
    assert out["arraycreate 16"]["rc"] == 0 and out["array3dcreate 64"]["rc"] == 0
    assert out["info arrays"]["free_mib"] == 4
    assert out["malloc3d 1000x1000x5"]["rc"] == oom  # 4.9 MiB > 4 left
    assert out["info freed"]["free_mib"] == 36         # hipFreeArray / hipArrayDestroy give back
    assert out["malloc3d again"]["rc"] == 0
    assert out["info malloc3d"]["free_mib"] == 31      # at the 1024-byte pitch: 1024 x 1000 x 5
    assert out["mipmap 64"]["rc"] == oom               # 64 MiB base + levels > 31 left
    assert out["info before overflow"]["free_mib"] == 100
    # SIZE_MAX (an OOM probe, an overflowed size) is refused and leaves the count alone
    assert out["malloc size_max"]["rc"] == oom and out["pitch overflow"]["rc"] == oom
    assert out["async size_max"]["rc"] == oom
    assert out["info after overflow"]["free_mib"] == 99
    assert out["legacy props"]["rc"] == 0 and out["legacy props value"]["mib"] == 100  # HIP-5 binaries
    assert out["info end"]["free_mib"] == 100


def test_shim_reinstalled_when_its_directory_is_wiped(scratch):
    """A kubelet cleaning its plugin directory removes the shim; the daemon puts
    it back (the path in Allocate() responses stays valid)."""
    import shutil
    import time
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, args=["--resource-config", "gpu:gpu-mem-gb:-1", "--enforce-memory-units",
                                      "--memcap-lib", SHIM]).start()
    try:
        k.wait_registration()
        installed = os.path.join(scratch, "amdgpu-dp", "libadp_memcap.so")
        assert os.path.exists(installed)
        shutil.rmtree(os.path.join(scratch, "amdgpu-dp"))
        deadline = time.time() + 5
        while time.time() < deadline and not os.path.exists(installed):
            time.sleep(0.02)
        assert os.path.exists(installed) and open(installed, "rb").read() == open(SHIM, "rb").read()
        d.wait_log("was removed; reinstalling")
        grant = os.path.join(scratch, "amdgpu-dp", "grants", "1000.mib")
        deadline = time.time() + 5
        while time.time() < deadline and not os.path.exists(grant):
            time.sleep(0.02)
        assert open(grant).read() == "1000\n"  # the grants are back too
    finally:
        d.stop()
        k.stop()


@pytest.mark.parametrize("extra", [["--device-list-strategy", "volume-mounts"],
                                   ["--device-list-strategy", "cdi-annotations"],
                                   ["--device-list-strategy", "cdi-cri"],
                                   ["--device-id-strategy", "index"]])
def test_shim_with_every_device_list_and_id_strategy(tmp_path, extra):
    d = str(tmp_path / "dp")
    os.makedirs(d)
    args = [*extra, "--cdi-spec-dir", str(tmp_path / "cdi")]
    resp, _ = _allocate(d, "gpu:gpu-mem-gb:-1", args)
    envs = dict(resp.envs)
    assert envs["LD_PRELOAD"] == "/usr/local/lib/amdgpu-dp/libadp_memcap.so"
    assert envs["AMD_GPU_MEMORY_LIMIT_MIB"] == "3000"
    shim = [m for m in resp.mounts if m.container_path == envs["LD_PRELOAD"]]
    assert len(shim) == 1 and shim[0].read_only and shim[0].host_path.endswith("amdgpu-dp/libadp_memcap.so")
    grant = [m for m in resp.mounts if m.container_path.startswith("/run/amdgpu-dp/grant/")]
    assert [(m.container_path, m.read_only) for m in grant] == [("/run/amdgpu-dp/grant/0", True)]
    assert any(dev.container_path == "/dev/kfd" for dev in resp.devices)


def test_time_slice_pods_do_not_get_the_shim(scratch):
    resp, _ = _allocate(scratch, "gpu:shared:4")
    assert "LD_PRELOAD" not in dict(resp.envs) and not list(resp.mounts)


def test_time_slice_replicas_with_hbm_shares(scratch):
    """--replica-hbm-share: each of R time-slice replicas holds 1/R of the HBM,
    reported like a memory-unit grant; enforced with --enforce-memory-units."""
    from k8s_gpu_sharing_plugin_amd.models import fixtures
    quarter = fixtures.MI355X_VRAM_MIB // 4
    resp, _ = _allocate(scratch, "gpu:shared:4", ["--replica-hbm-share"], take=2, enforce=False)
    envs = dict(resp.envs)
    assert envs["AMD_GPU_MEMORY_LIMIT_MIB"] == str(2 * quarter)  # two replicas of GPU 0 (pack)
    assert envs["AMD_GPU_MEMORY_FRACTION"] == "0.5000" and "LD_PRELOAD" not in envs


def test_time_slice_hbm_shares_enforced(tmp_path):
    from k8s_gpu_sharing_plugin_amd.models import fixtures
    d = str(tmp_path / "dp")
    os.makedirs(d)
    resp, _ = _allocate(d, "gpu:shared:4", ["--replica-hbm-share"], take=1)
    envs = dict(resp.envs)
    assert envs["AMD_GPU_MEMORY_LIMIT_MIB"] == str(fixtures.MI355X_VRAM_MIB // 4)
    assert envs["LD_PRELOAD"] == "/usr/local/lib/amdgpu-dp/libadp_memcap.so" and len(resp.mounts) == 2
    assert resp.mounts[1].host_path.endswith(f"/grants/{fixtures.MI355X_VRAM_MIB // 4}.mib")


def test_missing_shim_is_a_startup_error(scratch):
    d = harness.Daemon(scratch, args=["--resource-config", "gpu:gpu-mem-gb:-1", "--enforce-memory-units",
                                      "--memcap-lib", "/nonexistent/libadp_memcap.so"]).start()
    assert d.proc.wait(20) == 1
    assert "libadp_memcap.so not found" in d.log()


def test_missing_accounting_file_falls_back_to_dev_shm():
    """ADP_MEMCAP_FILE names the daemon's per-grant file; when it is absent
    (say the kubelet wiped the plugin directory) the grant is still enforced,
    counted in the pod's /dev/shm."""
    env = dict(_env(_key("nofile")), ADP_MEMCAP_FILE="/nonexistent/memcap")
    a = _hold(env, 60)
    try:
        assert _try(env, 50) == (2, 40)  # the two processes still share the grant
    finally:
        a.stdin.close()
        a.wait(10)


def test_memory_unit_pods_get_an_accounting_file_with_metrics(scratch):
    resp, _ = _allocate(scratch, "gpu:gpu-mem-gb:-1", ["--metrics-addr", "127.0.0.1:0"])
    envs = dict(resp.envs)
    assert envs["ADP_MEMCAP_FILE"] == "/run/amdgpu-dp/memcap"
    mounts = {m.container_path: (m.host_path, m.read_only) for m in resp.mounts}
    host, ro = mounts["/run/amdgpu-dp/memcap"]
    assert not ro and host.startswith(os.path.join(scratch, "amdgpu-dp", "usage") + "/")
    deadline = time.time() + 5
    while not os.path.isfile(host) and time.time() < deadline:  # written just after Allocate() returns
        time.sleep(0.005)
    assert os.path.getsize(host) > 100_000  # the whole accounting area
    # opted out, or no metrics endpoint: nothing extra is mounted
    resp, _ = _allocate(scratch, "gpu:gpu-mem-gb:-1", ["--metrics-addr", "127.0.0.1:0",
                                                      "--container-hbm-metrics=false"])
    assert "ADP_MEMCAP_FILE" not in dict(resp.envs) and len(resp.mounts) == 2  # shim + grant


def test_hbm_command_lists_grant_files(scratch):
    """`amdgpu-device-plugin --list-grants` (kubectl exec into the plugin pod)
    and `python -m k8s_gpu_sharing_plugin_amd hbm`: what each enforced grant
    holds, from its accounting file."""
    import sys
    resp, _ = _allocate(scratch, "gpu:gpu-mem-gb:-1", ["--metrics-addr", "127.0.0.1:0"])
    envs = dict(resp.envs)
    host = {m.container_path: m.host_path for m in resp.mounts}["/run/amdgpu-dp/memcap"]
    assert os.path.isfile(host)  # written before the daemon exited
    env = dict(os.environ, LD_PRELOAD=PRELOAD, AMD_GPU_MEMORY_LIMIT_MIB=envs["AMD_GPU_MEMORY_LIMIT_MIB"],
               ADP_MEMCAP_FILE=host)
    env.pop("ADP_MEMCAP_KEY", None)
    a = _hold(env, 1200)
    try:
        r = subprocess.run([sys.executable, "-m", "k8s_gpu_sharing_plugin_amd", "hbm",
                            "--device-plugin-path", scratch], capture_output=True, text=True, timeout=60)
        listed = json.loads(subprocess.run([harness.DAEMON, "--list-grants", "--device-plugin-path", scratch],
                                           capture_output=True, text=True, timeout=60, check=True).stdout)
    finally:
        a.stdin.close()
        a.wait(10)
    assert r.returncode == 0, r.stderr
    rows = [ln.split() for ln in r.stdout.splitlines()[1:]]
    key = os.path.basename(host)[:-len(".memcap")]
    assert len(rows) == 1 and rows[0][:6] == [key, "0", "1200", "3000", "1200", "0"]
    assert rows[0][6].count("-replica-") == 3  # the grant's three memory units
    (g,) = listed["grants"]
    assert (g["key"], g["used"], g["granted"], g["peak"], g["refused"]) == (key, [1200 << 20], [3000 << 20],
                                                                             [1200 << 20], [0])


def test_restarted_container_reclaims_its_predecessors_bytes(scratch):
    """A restarted container keeps its Allocate() response, so the same grant
    file: the bytes of the killed processes are reclaimed when the first
    process of the new container attaches."""
    import signal
    resp, _ = _allocate(scratch, "gpu:gpu-mem-gb:-1", ["--metrics-addr", "127.0.0.1:0"])
    envs = dict(resp.envs)
    host = {m.container_path: m.host_path for m in resp.mounts}["/run/amdgpu-dp/memcap"]
    env = dict(os.environ, LD_PRELOAD=PRELOAD, AMD_GPU_MEMORY_LIMIT_MIB=envs["AMD_GPU_MEMORY_LIMIT_MIB"],
               ADP_MEMCAP_FILE=host)
    env.pop("ADP_MEMCAP_KEY", None)
    a = _hold(env, 2500)
    a.send_signal(signal.SIGKILL)  # the container is killed
    a.wait(10)
    assert _try(env, 2900) == (0, 100)  # all 3000 MiB are the new container's


def test_ld_so_preload_list_keeps_the_shim_under_a_pods_own_ld_preload(scratch):
    """--memcap-ld-so-preload: the response also mounts, read-only, an
    /etc/ld.so.preload naming the shim -- glibc's loader reads it for every
    process whatever LD_PRELOAD the pod spec sets (which overrides the
    plugin's variable)."""
    resp, log = _allocate(scratch, "gpu:gpu-mem-gb:-1", ["--memcap-ld-so-preload"])
    mounts = {m.container_path: (m.host_path, m.read_only) for m in resp.mounts}
    host, ro = mounts["/etc/ld.so.preload"]
    assert ro and host == os.path.join(scratch, "amdgpu-dp", "ld.so.preload")
    assert open(host).read() == "/usr/local/lib/amdgpu-dp/libadp_memcap.so\n"
    assert dict(resp.envs)["LD_PRELOAD"] == "/usr/local/lib/amdgpu-dp/libadp_memcap.so"
    resp, _ = _allocate(scratch, "gpu:gpu-mem-gb:-1")  # off by default
    assert "/etc/ld.so.preload" not in {m.container_path for m in resp.mounts}


def _model_caps(lim, physical=294912, devices=64):
    """The shim's reading of AMD_GPU_MEMORY_LIMIT_MIB (strtoull per comma field;
    only 0 < MiB < 2^43 caps), as MiB per device; None = uncapped."""
    caps, dev, p = {}, 0, 0
    while p is not None and p < len(lim) and dev < devices:
        q = p
        while q < len(lim) and lim[q] in " \t\n\v\f\r":
            q += 1
        neg = q < len(lim) and lim[q] == "-"
        if q < len(lim) and lim[q] in "+-":
            q += 1
        d = q
        while d < len(lim) and lim[d].isdigit() and lim[d].isascii():
            d += 1
        if d > q:
            v = int(lim[q:d])
            v = (2 ** 64 - 1) if v >= 2 ** 64 else v
            if neg and v:
                v = 2 ** 64 - v
            if 0 < v < 2 ** 43:
                caps[dev] = v
        c = lim.find(",", p)
        p = c + 1 if c >= 0 else None
        dev += 1
    return {k: min(v, physical) for k, v in caps.items()}


@hypothesis.settings(max_examples=120, deadline=None, suppress_health_check=list(hypothesis.HealthCheck))
@hypothesis.given(st.lists(st.one_of(st.integers(0, 400000).map(str), st.sampled_from(["", " 7", "+9", "-5", "-0",
                                       "1e3", "0x10", "18446744073709551617", "8796093022208", "12abc", " "])),
                           min_size=0, max_size=4).map(",".join))
def test_env_caps_parse_like_strtoull(lim):
    """Whatever the pod's AMD_GPU_MEMORY_LIMIT_MIB holds, the shim never
    crashes and caps exactly the fields strtoull reads as 0 < MiB < 2^43 (a
    negative, zero, overflowing or non-numeric field leaves its device
    uncapped)."""
    out, _ = _run({"LD_PRELOAD": PRELOAD, "AMD_GPU_MEMORY_LIMIT_MIB": lim})
    want = _model_caps(lim)
    assert out["d0 info"]["total_mib"] == want.get(0, 294912), (lim, want)
    assert out["d1 totalmem value"]["mib"] == want.get(1, 294912), (lim, want)


def _model_grant(contents):
    """The shim's reading of grant files 0, 1, ...: stops at the first that is
    not a number followed by nothing or a newline (what follows the newline is
    not read), with 0 < MiB <= 2^43 (strtoull: leading blanks and a sign are
    read too)."""
    caps = {}
    for i, body in enumerate(contents):
        m = re.fullmatch(r"[ \t\n\v\f\r]*([+-]?)(\d+)(\n.*)?", body[:31], re.S)
        if not m:
            break
        v = min(int(m.group(2)), 2 ** 64 - 1)
        if m.group(1) == "-" and v:
            v = 2 ** 64 - v
        if v == 0 or v > 2 ** 43:
            break
        caps[i] = min(v, 294912)
    return caps


@hypothesis.settings(max_examples=80, deadline=None, suppress_health_check=list(hypothesis.HealthCheck))
@hypothesis.given(st.lists(st.one_of(st.integers(1, 400000).map(lambda v: f"{v}\n"),
                                     st.sampled_from(["", "0\n", "12", "12\n\n", "12 ", " 5\n", "-3\n", "x\n",
                                                      "8796093022209\n", "99999999999999999999\n"])),
                           min_size=0, max_size=3))
def test_grant_files_parse_and_stop_at_the_first_bad_one(tmp_path_factory, contents):
    d = tmp_path_factory.mktemp("g")
    for i, body in enumerate(contents):
        (d / str(i)).write_text(body)
    out, _ = _run({"LD_PRELOAD": PRELOAD, "ADP_MEMCAP_GRANT_DIR": str(d)})
    want = _model_grant(contents)
    assert out["d0 info"]["total_mib"] == want.get(0, 294912), (contents, want)
    assert out["d1 totalmem value"]["mib"] == want.get(1, 294912), (contents, want)

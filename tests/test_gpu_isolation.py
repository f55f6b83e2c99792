"""Real-MI355X checks of the round-4 isolation work (run on the GPU box).

* Container device order: a process that can open only the allocated render
  nodes (libadp_devcgroup_sim.so, the errno a container's device cgroup gives)
  numbers its HIP devices exactly as Allocate()'s AMD_GPU_MEMORY_DEVICES lists
  them (KFD node order), and sees nothing without them.
* CU-slot memory units: two packed 4-unit pods own disjoint whole CU slots;
  the first keeps its solo kernel latency next to a CU hog, with all its CUs.
* Event relay: the daemon under a device-cgroup denial gets amdsmi event
  notification through the relay running on real libamd_smi.
* Driver-side HBM scan: KFD's GPU-process list finds a live HIP allocation
  with the same bytes as the full /proc walk, reading a fraction of the fds;
  run by the event relay for a daemon that may read no other process, it
  reports the same allocation on /metrics.
"""

import json
import os
import re
import subprocess
import sys
import time

import pytest

from k8s_gpu_sharing_plugin_amd import BUILD_DIR
from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet, native

pytestmark = pytest.mark.gpu

SIM = os.path.join(BUILD_DIR, "libadp_devcgroup_sim.so")
OUT = "gpurun_out/r4"


def _save(name, obj):
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, name), "w") as f:
        json.dump(obj, f, indent=1)


@pytest.fixture(scope="module")
def snap():
    s = native.snapshot()
    assert s["gpus"], "libamd_smi enumerated no GPUs"
    return s


@pytest.fixture(scope="module")
def probe_exe():
    from k8s_gpu_sharing_plugin_amd.utils import build
    build.build_probe()
    return build.PROBE_EXE


def _hip_list(probe_exe, allow):
    env = {k: v for k, v in os.environ.items() if k not in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES")}
    env["LD_PRELOAD"] = " ".join(x for x in (env.get("LD_PRELOAD", ""), SIM) if x)
    env["ADP_DEVCGROUP_ALLOW"] = ":".join(allow)
    r = subprocess.run([probe_exe, "--list"], env=env, capture_output=True, text=True, timeout=60)
    out = r.stdout.strip().splitlines()
    try:
        devs = json.loads(out[-1]) if out else None
    except json.JSONDecodeError:
        devs = None
    return r.returncode, devs, r.stderr[-1500:]


def test_container_hip_order_is_the_memory_device_order(scratch, snap, probe_exe):
    """Allocate() lists a grant's devices in KFD node order; inside a
    container (only the allocated render nodes openable) HIP device i is
    entry i. On this 1-GPU box the list has one entry; the driver's 8-GPU run
    records the node's three orders in the bench's topology block."""
    bdf_of = {g["uuid"]: g["bdf"] for g in snap["gpus"]}
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, real_smi=True, args=["--resource-config", "gpu:gpu-mem-gb:-1"]).start()
    try:
        reg = k.wait_registration(30)
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        ids = [x.ID for x in c.watch()[0].get(timeout=10).devices]
        by_gpu = {}
        for i in ids:
            by_gpu.setdefault(i.split("-replica-")[0], []).append(i)
        want = [u[:2] for u in by_gpu.values()]  # 2 units on every GPU the box shows
        resp = c.allocate([i for w in want for i in w]).container_responses[0]
        c.close()
    finally:
        assert d.stop() == 0
        k.stop()
    envs = dict(resp.envs)
    order = [bdf_of[u] for u in envs["AMD_GPU_MEMORY_DEVICES"].split(",")]
    nodes = [s.host_path for s in resp.devices]
    rc, devs, err = _hip_list(probe_exe, nodes)
    record = {"memory_devices": envs["AMD_GPU_MEMORY_DEVICES"], "bdf_order": order, "hip_list": devs,
              "kfd_nodes": {g["bdf"]: g.get("kfd_node") for g in snap["gpus"]},
              "hip_ids": {g["bdf"]: g["partitions"][0].get("hip_id") for g in snap["gpus"]}}
    denied_rc, denied, denied_err = _hip_list(probe_exe, ["/dev/kfd"])
    record.update({"denied_rc": denied_rc, "denied_list": denied, "denied_err": denied_err[-300:]})
    _save("hip_order.json", record)
    assert rc == 0 and devs, (rc, devs, err)
    assert [x["pci"] for x in devs] == order, record
    assert all(g.get("kfd_node") is not None for g in snap["gpus"]), record
    # without the render node (a container not given the GPU) HIP sees none:
    # the probe reports hipGetDeviceCount's "no ROCm-capable device"
    assert denied_rc != 0 and "no ROCm-capable device" in str(denied), record


def test_cu_slot_units_isolate_neighbours_with_every_cu(scratch, snap, probe_exe):
    """--replica-cu-mask with the default unit (one CU slot + its share of
    HBM): two packed 4-unit pods get 0:0-31 and 0:32-63 -- 32 CUs each, 4 on
    every XCD, nothing shared and nothing idle -- and the first keeps its solo
    kernel latency next to a CU-saturating neighbour."""
    if snap["gpus"][0]["partitioned"]:
        pytest.skip("box GPU is partitioned")
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, real_smi=True, args=["--devices", "0", "--resource-config", "gpu:gpu-mem-gb:-1",
                                                     "--replica-cu-mask"]).start()
    try:
        reg = k.wait_registration(30)
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        free = [x.ID for x in c.watch()[0].get(timeout=10).devices]
        assert len(free) == 32
        grants = []
        for _ in range(2):
            ids = list(c.preferred(free, size=4).container_responses[0].deviceIDs)
            for i in ids:
                free.remove(i)
            grants.append(dict(c.allocate(ids).container_responses[0].envs))
        c.close()
    finally:
        assert d.stop() == 0
        k.stop()
    masks = [g["HSA_CU_MASK"] for g in grants]
    unit = snap["gpus"][0]["vram_mib"] // 32
    assert masks == ["0:0-31", "0:32-63"], masks
    assert [g["AMD_GPU_MEMORY_LIMIT_MIB"] for g in grants] == [str(4 * unit)] * 2
    base = {k_: v for k_, v in os.environ.items() if k_ != "HSA_CU_MASK"}
    census = subprocess.run([probe_exe, "--device", "0", "--census", "--expect-cus-seen", "32"],
                            env={**base, "HSA_CU_MASK": masks[0]}, capture_output=True, text=True, timeout=60)
    assert census.returncode == 0, census.stdout + census.stderr[-2000:]
    per_xcc = json.loads(census.stdout.strip().splitlines()[-1])["per_xcc"]

    def latency():
        r = subprocess.run([probe_exe, "--device", "0", "--latency", "1000"], env={**base, "HSA_CU_MASK": masks[0]},
                           capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr[-2000:]
        return json.loads(r.stdout.strip().splitlines()[-1])
    solo = latency()
    agg = subprocess.Popen([probe_exe, "--device", "0", "--aggressor", "5"], env={**base, "HSA_CU_MASK": masks[1]},
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        time.sleep(1.0)
        shared = latency()
    finally:
        out, err = agg.communicate(timeout=60)
    assert agg.returncode == 0, err[-2000:]
    launches = json.loads(out.strip().splitlines()[-1])["aggressor_launches"]
    _save("cu_slot_units.json", {"masks": masks, "unit_mib": unit, "census_per_xcc": per_xcc, "solo": solo,
                                 "with_neighbour": shared, "aggressor_launches": launches})
    assert per_xcc == [4] * 8
    assert launches > 100
    assert shared["p50_us"] < 1.5 * solo["p50_us"], (solo, shared)


def test_event_relay_on_real_amdsmi(scratch, snap, tmp_path):
    """The relay registers real amdsmi event notification; the daemon, denied
    /dev/kfd and the render nodes like an unprivileged pod, runs with events on
    through it."""
    sock = str(tmp_path / "events.sock")
    rdir = scratch + "-relay"
    os.makedirs(rdir, exist_ok=True)
    relay = harness.Daemon(rdir, real_smi=True, args=["--event-relay", "--health-event-socket", sock]).start()
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = None
    try:
        relay.wait_log("relaying amdsmi events on", 30)
        env = {"LD_PRELOAD": " ".join(x for x in (os.environ.get("LD_PRELOAD", ""), SIM) if x)}
        d = harness.Daemon(scratch, real_smi=True, args=["--devices", "0", "--health-event-socket", sock],
                           env=env).start()
        k.wait_registration(30)
        d.wait_log("health monitor watching", 30)
        log = d.wait_log("events on through the relay", 30)
        ping = subprocess.run([harness.DAEMON, "--relay-ping", "--health-event-socket", sock], capture_output=True,
                              text=True, timeout=30)
        _save("event_relay.json", {"relay_log": relay.log()[-3000:], "daemon_log": log[-4000:],
                                   "relay_ping": {"rc": ping.returncode, "out": ping.stdout}})
        assert ping.returncode == 0 and ping.stdout.startswith("hello v1 events=ok"), ping.stdout + ping.stderr
        assert "event notification registered on" in relay.log(), relay.log()[-2000:]
        assert "events on through the relay" in log, log[-3000:]
        assert "device access: Operation not permitted: /dev/kfd" in log  # the daemon itself is denied
        # The daemon's view of the processors (denied the device nodes) matches
        # the relay's on real amdsmi: its restarts keep the registration, and
        # the relay says nothing was missed.
        import signal
        for i in range(2):
            d.signal(signal.SIGHUP)
            d.wait_log("events on through the relay", 30, count=i + 2)
        rlog = relay.wait_log("nothing missed", 30, count=2)
        _save("event_relay_restarts.json", {"relay_log": rlog[-4000:]})
        assert rlog.count("registration kept") == 3 and "re-enumerating" not in rlog, rlog[-3000:]
    finally:
        if d:
            assert d.stop() == 0
        k.stop()
        assert relay.stop() == 0


_HOLDER = r'''
import ctypes, sys
lib = ctypes.CDLL("libamdhip64.so")
p = ctypes.c_void_p()
rc = lib.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 30))
lib.hipMemset(p, 1, ctypes.c_size_t(1 << 30)); lib.hipDeviceSynchronize()
print("holding", rc, flush=True)
sys.stdin.read()
'''


def _hold_1gib():
    """A child process holding 1 GiB of HBM until its stdin closes."""
    p = subprocess.Popen([sys.executable, "-c", _HOLDER], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    line = p.stdout.readline().split()
    if line[:2] != ["holding", "0"]:
        p.stdin.close()
        p.wait(timeout=30)
        raise AssertionError((line, p.stderr.read()[-2000:]))
    return p


def test_driver_scan_reads_the_gpu_processes_kfd_lists(tmp_path):
    """A HIP process holding 1 GiB: the scan through KFD's process list finds
    it with the same bytes as the full /proc walk, reading only GPU processes."""
    p = _hold_1gib()
    try:
        kfd_dir = "/sys/class/kfd/kfd/proc"
        listed = sorted(int(x) for x in os.listdir(kfd_dir) if x.isdigit()) if os.path.isdir(kfd_dir) else []
        fast = native.driver_scan("/proc", kfd_proc_dir=kfd_dir)
        full = native.driver_scan("/proc")
        mine = lambda s: sum(x["bytes"] for x in s["procs"] if x["pid"] == p.pid)  # noqa: E731
        _save("driver_scan_real.json", {"kfd_listed": listed, "child": p.pid,
                                        "kfd": {k_: fast[k_] for k_ in ("pid_source", "pids_scanned", "fd_entries",
                                                                        "scan_us", "total")},
                                        "full": {k_: full[k_] for k_ in ("pid_source", "pids_scanned", "fd_entries",
                                                                         "scan_us", "total")},
                                        "child_bytes": {"kfd": mine(fast), "full": mine(full)}})
        assert listed, "KFD lists no GPU process"
        if p.pid in listed:  # this /proc is the host PID namespace's: KFD's list is used
            assert fast["pid_source"] == "kfd" and fast["pids_scanned"] == len(listed)
            assert fast["fd_entries"] <= full["fd_entries"]
        else:  # a PID namespace of its own (KFD names host PIDs): the scan falls back to the walk
            assert fast["pid_source"] == "proc"
        assert mine(fast) >= 1 << 30 and mine(fast) == mine(full)
    finally:
        p.stdin.close()
        p.wait(timeout=30)


def test_driver_scan_through_the_relay(scratch, snap, tmp_path):
    """The chart's layout, every feature at once: the daemon is denied the GPU
    device nodes (an unprivileged pod's device cgroup, through the simulator)
    and given a --host-proc that does not exist; the relay (real libamd_smi,
    the host's /proc) holds the events and runs the driver-side scans.
    - a HIP process holding 1 GiB shows on /metrics (the relay's scan);
    - health events are on through the relay;
    - --replica-cu-mask still cuts CU-slot units (CU counts from KFD topology):
      a 4-unit pod gets HSA_CU_MASK 0:0-31 and 4 slots' HBM;
    - the node label names the product (the board's PCI product_name);
    - /healthz answers 200."""
    from test_metrics import _get, _parse
    sock = str(tmp_path / "events.sock")
    rdir = scratch + "-relay"
    os.makedirs(rdir, exist_ok=True)
    relay = harness.Daemon(rdir, real_smi=True, args=["--event-relay", "--health-event-socket", sock]).start()
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = None
    holder = None
    try:
        relay.wait_log("relaying amdsmi events on", 30)
        holder = _hold_1gib()
        env = {"LD_PRELOAD": " ".join(x for x in (os.environ.get("LD_PRELOAD", ""), SIM) if x)}
        d = harness.Daemon(scratch, real_smi=True, env=env, args=[
            "--devices", "0", "--health-event-socket", sock, "--metrics-addr", "127.0.0.1:0",
            "--resource-config", "gpu:gpu-mem-gb:-1", "--enforce-memory-units", "--memcap-lib",
            os.path.join(BUILD_DIR, "libadp_memcap.so"), "--host-proc",
            str(tmp_path / "nosuch"), "--driver-hbm-poll-ms", "200", "--replica-cu-mask",
            "--node-labels-file", str(tmp_path / "labels")]).start()
        port = int(re.search(r"on port (\d+)", d.wait_log("serving /metrics", 30)).group(1))
        reg = k.wait_registration(30)
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        free = [x.ID for x in c.watch()[0].get(timeout=10).devices]
        pod = list(c.preferred(free, size=4).container_responses[0].deviceIDs)
        envs = dict(c.allocate(pod).container_responses[0].envs)
        c.close()
        layout = {"units": len(free), "hsa_cu_mask": envs.get("HSA_CU_MASK"),
                  "limit_mib": envs.get("AMD_GPU_MEMORY_LIMIT_MIB"),
                  "labels": open(str(tmp_path / "labels")).read().splitlines(),
                  "healthz": _get(port, "/healthz")[0],
                  "events": "events on through the relay" in d.wait_log("events on through the relay", 30)}
        bdf = snap["gpus"][0]["bdf"]
        def get(samples, name, **labels):  # None until the first scan has run
            want = set(labels.items())
            hits = [v for (n, ls), v in samples.items() if n == name and want <= set(ls)]
            return hits[0] if len(hits) == 1 else None
        deadline = time.time() + 30
        while True:
            text = _get(port, "/metrics")[1]
            m = _parse(text)
            held = get(m, "amdgpu_dp_gpu_hbm_driver_bytes", bdf=bdf)
            if (held or 0) >= 1 << 30 or time.time() > deadline:
                break
            time.sleep(0.2)
        record = {"gpu_driver_bytes": held, "scan_failures": get(m, "amdgpu_dp_driver_hbm_scan_failures_total"),
                  "scan_processes": {str(dict(ls)): v for (n, ls), v in m.items()
                                     if n == "amdgpu_dp_driver_hbm_scan_processes"},
                  "scan_seconds": get(m, "amdgpu_dp_driver_hbm_scan_seconds"),
                  "driver_metric_lines": [ln for ln in text.splitlines() if "driver" in ln and not ln.startswith("#")],
                  "daemon_log": [ln for ln in d.log().splitlines() if "driver-hbm" in ln or "inventory" in ln][:8],
                  "relay_log": [ln for ln in relay.log().splitlines() if "scan" in ln][:4], "layout": layout}
        _save("driver_scan_relay.json", record)
        assert (held or 0) >= 1 << 30, record
        assert record["scan_failures"] == 0, record
        assert "first HBM scan for a daemon" in relay.log()
        if not snap["gpus"][0]["partitioned"]:
            unit = snap["gpus"][0]["vram_mib"] // 32
            assert layout["units"] == 32 and layout["hsa_cu_mask"] == "0:0-31", layout
            assert layout["limit_mib"] == str(4 * unit), layout
        assert layout["healthz"] == 200 and layout["events"], layout
        product = [ln for ln in layout["labels"] if ln.startswith("amd.com/gpu.product=")]
        assert product and product[0] != "amd.com/gpu.product=", layout["labels"]
    finally:
        if holder:
            holder.stdin.close()
            holder.wait(timeout=30)
        if d:
            assert d.stop() == 0
        k.stop()
        assert relay.stop() == 0


def _userns_mounts_ok():
    try:
        return subprocess.run(["unshare", "-rm", "sh", "-c", "mount --rbind /dev /mnt && true"], capture_output=True,
                              timeout=20).returncode == 0
    except (OSError, subprocess.TimeoutExpired):
        return False


def test_images_on_the_real_gpu(scratch, snap, tmp_path):
    """The assembled DaemonSet image (tests/test_image_rootfs.py) on the
    MI355X: its own libamd_smi enumerates the GPU and its daemon allocates it
    to a kubelet; the validation image's HIP runtime runs the probe's
    checksummed HBM copy. With user+mount namespaces the images run chrooted
    with the host's /dev, /sys and /proc bound in (as the chart mounts them);
    without them (this pool's boxes) the image's own loader runs them with
    only the image's library directories, and LD_DEBUG=files shows every
    shared object came from the image."""
    from k8s_gpu_sharing_plugin_amd.utils import image
    binds = ("/dev", "/sys", "/proc")
    chroot = _userns_mounts_ok()

    def cmd(rootfs, argv):
        return image.chroot_cmd(rootfs, argv, binds) if chroot else image.loader_cmd(rootfs, argv)
    env = {k: v for k, v in os.environ.items() if k not in ("LD_PRELOAD", "LD_LIBRARY_PATH", "AMD_SMI_LIB")}
    dbg = dict(env, LD_DEBUG="files")
    rt = str(tmp_path / "runtime")
    image.build_rootfs(rt)
    rep = subprocess.run(cmd(rt, ["/usr/bin/amdgpu-device-plugin", "--smi-report"]), capture_output=True,
                         text=True, timeout=120, env=dbg)
    report = json.loads(rep.stdout[rep.stdout.index("{"):]) if rep.returncode == 0 and "{" in rep.stdout else {}
    daemon_libs = image.loaded_files(rep.stderr)
    pdir = os.path.join(rt, "var/lib/kubelet/device-plugins") if chroot else scratch
    os.makedirs(pdir, exist_ok=True)
    k = kubelet.StubKubelet(os.path.join(pdir, "kubelet.sock")).start()
    dm = image.image_daemon(rt, ["--devices", "0"], binds=binds, loader=not chroot,
                            plugin_dir="/var/lib/kubelet/device-plugins" if chroot else scratch)
    try:
        reg = k.wait_registration(60)
        c = kubelet.PluginClient(os.path.join(pdir, reg.endpoint))
        ids = [x.ID for x in c.watch()[0].get(timeout=20).devices]
        specs = [s.container_path for s in c.allocate(ids[:1]).container_responses[0].devices]
        maps = open(f"/proc/{dm.proc.pid}/maps").read() if dm.proc.poll() is None else ""
        c.close()
    finally:
        code = dm.stop()
        k.stop()
    smi_mapped = sorted({ln.split()[-1] for ln in maps.splitlines() if "libamd_smi" in ln})
    val = str(tmp_path / "validation")
    image.build_rootfs(val, stage="validation")
    probe = subprocess.run(cmd(val, ["/usr/bin/amdgpu-dp-probe", "--device", "0", "--bytes", str(64 << 20),
                                     "--iters", "2"]), capture_output=True, text=True, timeout=180, env=dbg)
    result = json.loads(probe.stdout.strip().splitlines()[-1]) if probe.stdout.strip() else {}
    probe_libs = image.loaded_files(probe.stderr)
    # Libraries the environment preloads into every process (outside any
    # image) show up in a bare `--list` of the image's loader as well.
    base = subprocess.run(image.loader_cmd(rt, ["/usr/bin/amdgpu-device-plugin"])[:-1] + ["--list"] +
                          image.loader_cmd(rt, ["/usr/bin/amdgpu-device-plugin"])[-1:],
                          capture_output=True, text=True, timeout=60, env=dbg)
    preloaded = {f for f in image.loaded_files(base.stderr) if not f.startswith(rt)}
    outside = [f for f in daemon_libs + probe_libs if not f.startswith((rt, val)) and f not in preloaded]
    _save("images_on_gpu.json", {"mode": "chroot" if chroot else "image loader", "smi_report_rc": rep.returncode,
                                 "enumeration": report.get("enumeration"), "daemon_libs": daemon_libs,
                                 "daemon_libamd_smi_mapped": smi_mapped, "advertised": ids, "device_specs": specs,
                                 "daemon_exit": code, "probe": result, "probe_libs": probe_libs,
                                 "loaded_from_outside_the_images": outside,
                                 "probe_stderr_tail": [ln for ln in probe.stderr.splitlines()
                                                       if "file=" not in ln][-20:]})
    assert rep.returncode == 0 and report.get("enumeration") == "ok", rep.stderr[-2000:]
    assert ids == [snap["gpus"][0]["uuid"]] and "/dev/kfd" in specs
    assert specs[-1] == snap["gpus"][0]["partitions"][0]["render"]
    assert code == 0
    assert smi_mapped and all(p.startswith(rt) for p in smi_mapped), smi_mapped
    assert probe.returncode == 0 and result.get("checksum_ok"), result
    assert not outside, outside  # every shared object came from the images


def test_kfd_topology_cus_match_asic_info(snap, tmp_path):
    """The CU-count fallback on real hardware: KFD topology gives every GPU the
    CU count asic_info does, and a daemon denied the render nodes (the chart's
    drop-ALL container, through the device-cgroup simulator) still cuts 32
    CU-slot units per SPX GPU."""
    topo = "/sys/class/kfd/kfd/topology/nodes"
    rows = []
    for g in snap["gpus"]:
        for p in g["partitions"]:
            node = p.get("kfd_node")
            rows.append({"bdf": g["bdf"], "partition": p.get("partition_id"), "kfd_node": node,
                         "asic_info_cus": p.get("cus"),
                         "topology_cus": native.kfd_topology_cus(topo, node) if node is not None else None})
    # what else the node exposes without the render node (a market-name source, if any)
    extra = {}
    for g in snap["gpus"]:
        for path in (f"/sys/bus/pci/devices/{g['bdf']}/product_name",
                     f"{topo}/{g['partitions'][0].get('kfd_node')}/name"):
            try:
                with open(path) as f:
                    extra[path] = f.read().strip()
            except OSError as e:
                extra[path] = f"unreadable: {e.strerror}"
    env = {"LD_PRELOAD": " ".join(x for x in (os.environ.get("LD_PRELOAD", ""), SIM) if x)}
    r = subprocess.run([harness.DAEMON, "--device-plugin-path", str(tmp_path), "--dry-run", "--replica-cu-mask",
                        "--resource-config", "gpu:gpu-mem-gb:-1"], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, **env))
    dry = json.loads(r.stdout) if r.returncode == 0 else {"rc": r.returncode}
    log = [ln for ln in r.stderr.splitlines() if "KFD topology" in ln or "CU" in ln]
    _save("kfd_topology.json", {"rows": rows, "sysfs": extra, "denied_dry_run": dry, "denied_log": log})
    assert all(x["topology_cus"] == x["asic_info_cus"] and x["topology_cus"] for x in rows), rows
    assert r.returncode == 0, r.stderr[-2000:]
    spx = [g for g in dry["gpus"] if g["partitions"] == 1]
    assert all(g["cus"] == 256 for g in spx), dry["gpus"]
    if spx and len(spx) == len(dry["gpus"]):
        assert dry["resources"][0]["allocatable"] == 32 * len(spx), dry["resources"]
    assert any("from KFD topology" in ln for ln in log), log
    # the board's FRU name labels the node even without the render node
    fru = [v for k, v in extra.items() if k.endswith("product_name") and not v.startswith("unreadable")]
    if fru and fru[0]:
        assert dry["labels"]["amd.com/gpu.product"] == "-".join(fru[0].split()), dry["labels"]


def test_every_write_lands_on_a_mounted_volume_on_real_amdsmi(scratch, snap, tmp_path):
    """The chart's layout on real libamd_smi with every filesystem write logged
    (libadp_devcgroup_sim.so, ADP_FS_WRITE_LOG): the plugin (denied the device
    nodes) and the relay (allowed /dev) write only to the volumes the chart
    mounts writable -- what readOnlyRootFilesystem needs, including whatever
    libamd_smi itself writes."""
    from test_chart_layout import _writes
    plugin_dir = scratch
    state_dir, nfd_dir, sock_dir = str(tmp_path / "state"), str(tmp_path / "nfd"), scratch + ".events"
    for d in (state_dir, nfd_dir, sock_dir):
        os.makedirs(d)
    sock = os.path.join(sock_dir, "events.sock")
    dlog, rlog = str(tmp_path / "daemon.writes"), str(tmp_path / "relay.writes")
    pre = " ".join(x for x in (os.environ.get("LD_PRELOAD", ""), SIM) if x)
    relay = harness.Daemon(scratch + "-relay", real_smi=True, args=["--event-relay", "--health-event-socket", sock],
                           env={"LD_PRELOAD": pre, "ADP_DEVCGROUP_ALLOW": "/dev", "ADP_FS_WRITE_LOG": rlog}).start()
    k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = None
    try:
        relay.wait_log("relaying amdsmi events on", 30)
        d = harness.Daemon(scratch, real_smi=True, env={"LD_PRELOAD": pre, "ADP_FS_WRITE_LOG": dlog,
                                                        "DP_HEALTH_POLL_MS": "200"}, args=[
            "--devices", "0", "--resource-config", "gpu:gpu-mem-gb:-1", "--replica-cu-mask",
            "--enforce-memory-units", "--memcap-lib", os.path.join(BUILD_DIR, "libadp_memcap.so"),
            "--metrics-addr", "127.0.0.1:0", "--health-event-socket", sock, "--driver-hbm-poll-ms", "200",
            "--health-state-file", os.path.join(state_dir, "health.state"),
            "--drain-file", os.path.join(state_dir, "drain"),
            "--node-labels-file", os.path.join(nfd_dir, "amd-gpu")]).start()
        reg = k.wait_registration(30)
        c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
        ids = [x.ID for x in c.watch()[0].get(timeout=10).devices]
        c.allocate(ids[:4])
        c.close()
        d.wait_log("events on through the relay", 30)
        d.wait_log("health poll #1", 30)
        time.sleep(1.0)  # a few health polls and relay scans
    finally:
        if d:
            assert d.stop() == 0
        k.stop()
        assert relay.stop() == 0
    allowed = [plugin_dir, state_dir, nfd_dir, sock_dir, "/dev/"]
    summary = {}
    for who, log in (("daemon", dlog), ("relay", rlog)):
        w = _writes(log)
        summary[who] = {"writes": len(w), "calls": sorted({c for c, _ in w}),
                        "outside_mounts": sorted({p for _, p in w if not any(p.startswith(a) for a in allowed)}),
                        "dev": sorted({p for _, p in w if p.startswith("/dev/")})}
    _save("fs_writes.json", summary)
    assert summary["daemon"]["writes"] and summary["relay"]["writes"], summary
    assert not summary["daemon"]["outside_mounts"] and not summary["relay"]["outside_mounts"], summary


_RENDER_HOLDER = r'''
import ctypes, glob, os, sys
drm = ctypes.CDLL("libdrm_amdgpu.so.1")
class Req(ctypes.Structure):
    _fields_ = [("alloc_size", ctypes.c_uint64), ("phys_alignment", ctypes.c_uint64),
                ("preferred_heap", ctypes.c_uint32), ("flags", ctypes.c_uint64)]
dev, node = ctypes.c_void_p(), None
for path in sorted(glob.glob("/dev/dri/renderD*")):
    try:
        fd = os.open(path, os.O_RDWR)
    except OSError:
        continue
    major, minor = ctypes.c_uint32(), ctypes.c_uint32()
    if drm.amdgpu_device_initialize(fd, ctypes.byref(major), ctypes.byref(minor), ctypes.byref(dev)) == 0:
        node = path
        break
    os.close(fd)
size = int(sys.argv[1]) << 20
bo, ptr = ctypes.c_void_p(), ctypes.c_void_p()
# AMDGPU_GEM_DOMAIN_VRAM, AMDGPU_GEM_CREATE_CPU_ACCESS_REQUIRED
rc = drm.amdgpu_bo_alloc(dev, ctypes.byref(Req(size, 4096, 4, 1)), ctypes.byref(bo)) if node else -1
rc_map = drm.amdgpu_bo_cpu_map(bo, ctypes.byref(ptr)) if rc == 0 else -1
if rc_map == 0:
    ctypes.memset(ptr, 1, size)
print("holding", rc, rc_map, node, flush=True)
sys.stdin.read()
'''


def test_render_only_vram_holder_is_seen_by_a_full_walk(snap):
    """Advisor round 4, on the MI355X: a process that allocates VRAM through
    libdrm_amdgpu on a render node -- no /dev/kfd open, so in no KFD process
    list -- holds HBM the driver counts in its DRM fdinfo. The full walk finds
    it and counts it render-only; the plugin's periodic full walk
    (ADP_DRIVER_FULL_WALK_MS) exists for exactly this holder."""
    mib = 256
    p = subprocess.Popen([sys.executable, "-c", _RENDER_HOLDER, str(mib)], stdin=subprocess.PIPE,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        line = p.stdout.readline().split()
        assert line[:3] == ["holding", "0", "0"], (line, p.stderr.read()[-2000:] if p.poll() is not None else "")
        links = [os.readlink(f"/proc/{p.pid}/fd/{f}") for f in os.listdir(f"/proc/{p.pid}/fd")]
        assert "/dev/kfd" not in links and any(t.startswith("/dev/dri/renderD") for t in links), links
        full = native.driver_scan("/proc")
        rows = [r for r in full["procs"] if r["pid"] == p.pid]
        kfd = native.driver_scan("/proc", kfd_proc_dir="/sys/class/kfd/kfd/proc")
        _save("render_only_holder.json", {
            "holder": {"pid": p.pid, "render_node": line[3], "bo_mib": mib, "fds": sorted(set(links))},
            "full_walk": {"rows": rows, "render_only": full["render_only"], "pids_scanned": full["pids_scanned"]},
            "kfd_list_scan": {"pid_source": kfd["pid_source"], "pids_scanned": kfd["pids_scanned"],
                              "holder_rows": [r for r in kfd["procs"] if r["pid"] == p.pid]}})
        assert rows and sum(r["bytes"] for r in rows) >= mib << 20, rows
        assert full["render_only"] >= 1
    finally:
        p.stdin.close()
        p.wait(timeout=30)

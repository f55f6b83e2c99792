"""End-to-end: the real daemon binary + grpcio stub kubelet + amdsmi mock (BASELINE config 1).

kubelet receives Register(amd.com/gpu), opens ListAndWatch, sees 2 Healthy
devices, Allocate(1) returns DeviceSpecs [/dev/kfd, /dev/dri/renderD128].
"""

import collections
import os
import re
import subprocess
import urllib.request

import grpc
import pytest

from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet


@pytest.fixture
def running(scratch):
    started = []

    def start(fixture=None, args=(), env=None, **kw):
        k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
        d = harness.Daemon(scratch, fixture or fixtures.node(2), args=args, env=env, **kw).start()
        started.append((d, k))
        return d, k
    yield start
    for d, k in started:
        d.stop()
        k.stop()


def test_minimum_slice(running, scratch):
    d, k = running()
    reg = k.wait_registration()
    assert reg.version == "v1beta1"
    assert reg.endpoint == "amd-gpu.sock"
    assert reg.resource_name == "amd.com/gpu"
    assert reg.options.get_preferred_allocation_available
    c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
    opts = c.options()
    assert not opts.pre_start_required and opts.get_preferred_allocation_available
    q, call = c.watch()
    law = q.get(timeout=5)
    assert len(law.devices) == 2
    assert all(x.health == "Healthy" for x in law.devices)
    assert [n.ID for n in law.devices[0].topology.nodes] == [0]
    r = c.allocate([law.devices[0].ID])
    cr = r.container_responses[0]
    assert [(s.container_path, s.host_path, s.permissions) for s in cr.devices] == [
        ("/dev/kfd", "/dev/kfd", "rw"), ("/dev/dri/renderD128", "/dev/dri/renderD128", "rw")]
    assert dict(cr.envs) == {"AMD_VISIBLE_DEVICES": law.devices[0].ID}
    assert c.prestart([law.devices[0].ID]) is not None
    call.cancel()
    c.close()


def test_allocate_unknown_device_is_invalid_argument(running, scratch):
    d, k = running()
    reg = k.wait_registration()
    c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
    with pytest.raises(grpc.RpcError) as e:
        c.allocate(["no-such-device"])
    assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
    assert "unknown device: no-such-device" in e.value.details()
    c.close()


def test_multi_container_allocate_and_index_strategy(running, scratch):
    d, k = running(fixtures.node(4), args=["--device-id-strategy", "index", "--device-list-strategy",
                                           "volume-mounts"])
    reg = k.wait_registration()
    c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
    law = c.watch()[0].get(timeout=5)
    ids = [x.ID for x in law.devices]
    r = c.allocate([ids[2], ids[0]], [ids[3]])
    a, b = r.container_responses
    assert dict(a.envs) == {"AMD_VISIBLE_DEVICES": "/var/run/amd-container-devices"}
    assert [m.container_path for m in a.mounts] == ["/var/run/amd-container-devices/0",
                                                    "/var/run/amd-container-devices/2"]
    assert all(m.host_path == "/dev/null" for m in a.mounts)
    assert [s.container_path for s in a.devices] == ["/dev/kfd", "/dev/dri/renderD128", "/dev/dri/renderD144"]
    assert [s.container_path for s in b.devices] == ["/dev/kfd", "/dev/dri/renderD152"]
    c.close()


def test_driver_root_prefixes_host_paths(running, scratch):
    d, k = running(args=["--driver-root", "/run/amd/driver"])
    reg = k.wait_registration()
    c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
    law = c.watch()[0].get(timeout=5)
    r = c.allocate([law.devices[1].ID])
    assert [(s.container_path, s.host_path) for s in r.container_responses[0].devices] == [
        ("/dev/kfd", "/run/amd/driver/dev/kfd"), ("/dev/dri/renderD136", "/run/amd/driver/dev/dri/renderD136")]
    c.close()


def test_no_device_library_calls_on_the_rpc_path(running, scratch):
    """B5: the reference re-enumerates NVML twice per GetPreferredAllocation; we never touch amdsmi."""
    counter = os.path.join(scratch + ".fixture", "calls")
    os.makedirs(scratch + ".fixture", exist_ok=True)
    d, k = running(fixtures.node(8), env={"AMDSMI_MOCK_CALL_COUNT_FILE": counter,
                                         "DP_DISABLE_HEALTHCHECKS": "all"})
    reg = k.wait_registration()
    c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
    ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
    before = open(counter).read()
    for size in (1, 2, 4, 8):
        got = list(c.preferred(ids, [], size).container_responses[0].deviceIDs)
        c.allocate(got)
    assert open(counter).read() == before
    c.close()


def test_cdi_spec_and_cdi_names(running, scratch):
    import json
    cdi = os.path.join(scratch, "cdi")
    d, k = running(fixtures.node(2), args=["--device-list-strategy", "cdi-cri", "--cdi-spec-dir", cdi])
    reg = k.wait_registration()
    spec = json.load(open(os.path.join(cdi, "amd.com-gpu.json")))
    assert spec["kind"] == "amd.com/gpu" and spec["cdiVersion"] == "0.5.0"
    assert spec["containerEdits"]["deviceNodes"][0]["path"] == "/dev/kfd"
    names = [dev["name"] for dev in spec["devices"]]
    assert spec["devices"][1]["containerEdits"]["deviceNodes"][0]["path"] == "/dev/dri/renderD136"
    c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
    ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
    r = c.allocate([ids[1]]).container_responses[0]
    assert [x.name for x in r.cdi_devices] == [f"amd.com/gpu={names[1]}"]
    c.close()


def test_cdi_annotations(running, scratch):
    d, k = running(fixtures.node(2), args=["--device-list-strategy", "cdi-annotations", "--cdi-spec-dir",
                                           os.path.join(scratch, "cdi"), "--device-id-strategy", "index"])
    reg = k.wait_registration()
    c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
    ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
    r = c.allocate(ids).container_responses[0]
    assert dict(r.annotations) == {"cdi.k8s.io/amd-gpu-device-plugin_0": "amd.com/gpu=0,amd.com/gpu=1"}
    c.close()


def test_trace_logs_each_rpc(running, scratch):
    d, k = running(fixtures.node(1), args=["--trace"])
    reg = k.wait_registration()
    c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
    ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
    c.allocate(ids)
    log = d.wait_log("/v1beta1.DevicePlugin/Allocate OK")
    assert "handler=" in log
    c.close()


def test_native_stub_kubelet_sees_devices(scratch):
    """Same flow through the native stub kubelet (amdgpu-dp-kubelet serve)."""
    k = harness.NativeKubelet(os.path.join(scratch, "kubelet.sock")).start()
    d = harness.Daemon(scratch, fixtures.node(8)).start()
    try:
        reg = k.wait(lambda e: e.get("event") == "register")
        assert reg["resource"] == "amd.com/gpu" and reg["preferred"]
        dev = k.wait(lambda e: e.get("event") == "devices")
        assert dev["total"] == 8 and dev["healthy"] == 8
        assert dev["numa"] == {"0": 4, "1": 4}
    finally:
        assert d.stop() == 0
        k.stop()


def test_memory_units_report_granted_hbm(running, scratch):
    """gpu-mem-gb (replicas=-1): the container learns how much HBM it was granted
    per device, in enumeration order (AMD_GPU_MEMORY_DEVICES names the devices);
    plain and time-slice resources do not."""
    d, k = running(args=["--resource-config", "gpu:gpu-mem-gb:-1", "--replica-policy", "pack"])
    reg = k.wait_registration()
    assert reg.resource_name == "amd.com/gpu-mem-gb"
    c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
    ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
    assert len(ids) == 2 * 294
    gpu0 = [i for i in ids if i.startswith(ids[0].split("-replica-")[0])]
    gpu1 = [i for i in ids if i not in gpu0]
    envs = dict(c.allocate(gpu0[:36]).container_responses[0].envs)
    assert envs["AMD_GPU_MEMORY_LIMIT_MIB"] == "36000"
    assert envs["AMD_GPU_MEMORY_FRACTION"] == f"{36000 / 294896:.4f}"
    envs = dict(c.allocate(gpu1[:2] + gpu0[:3]).container_responses[0].envs)
    order = envs["AMD_GPU_MEMORY_DEVICES"].split(",")
    assert sorted(order) == sorted(envs["AMD_VISIBLE_DEVICES"].split(","))
    want = {gpu0[0].split("-replica-")[0]: "3000", gpu1[0].split("-replica-")[0]: "2000"}
    assert envs["AMD_GPU_MEMORY_LIMIT_MIB"].split(",") == [want[u] for u in order]
    # an ID listed twice is one unit: never twice the HBM
    envs = dict(c.allocate([gpu0[0], gpu0[0], gpu0[1]]).container_responses[0].envs)
    assert envs["AMD_GPU_MEMORY_LIMIT_MIB"] == "2000"
    c.close()


def test_memory_lists_follow_enumeration_order_not_uuid_order(running, scratch):
    """GPU 0's UUID sorts after GPU 1's: AMD_VISIBLE_DEVICES (uuid strategy) lists
    GPU 1 first, but the memory lists -- like HSA_CU_MASK and HIP's device
    ordinals inside the container -- follow enumeration order."""
    fx = fixtures.node(2)
    fx["gpus"][0]["uuid"] = "ffffffff-0000-1000-80c0-000000000000"
    fx["gpus"][1]["uuid"] = "00000000-0000-1000-80c0-000000000001"
    d, k = running(fx, args=["--resource-config", "gpu:gpu-mem-gb:-1", "--replica-policy", "pack",
                             "--replica-cu-mask", "--auto-replica-unit", "mib"])
    reg = k.wait_registration()
    c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
    ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
    g0 = sorted(i for i in ids if i.startswith("ffffffff"))
    g1 = sorted(i for i in ids if i.startswith("00000000"))
    envs = dict(c.allocate(g0[:5] + g1[:2]).container_responses[0].envs)
    assert envs["AMD_VISIBLE_DEVICES"].split(",")[0].startswith("00000000")  # UUID order
    assert envs["AMD_GPU_MEMORY_DEVICES"].split(",")[0].startswith("ffffffff")  # enumeration order
    assert envs["AMD_GPU_MEMORY_LIMIT_MIB"] == "5000,2000"
    assert envs["HSA_CU_MASK"].startswith("0:")  # agent 0 = GPU 0, same order
    c.close()


def test_time_slice_replicas_carry_no_memory_envs(running, scratch):
    d, k = running(args=["--resource-config", "gpu:sharedgpu:4"])
    reg = k.wait_registration()
    c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
    ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
    envs = dict(c.allocate(ids[:2]).container_responses[0].envs)
    assert "AMD_GPU_MEMORY_LIMIT_MIB" not in envs
    assert "HSA_CU_MASK" not in envs  # CU shares are opt-in (--replica-cu-mask)
    c.close()


def test_replica_cu_mask_splits_compute_units(running, scratch):
    """--replica-cu-mask: replica r of 4 runs on its own quarter of every XCD's CUs
    (HSA_CU_MASK bit i -> XCD i % 8, profiles/r1/session18/); adjacent shares merge,
    agents are numbered in enumeration order inside the container."""
    d, k = running(args=["--resource-config", "gpu:sharedgpu:4", "--replica-cu-mask"])
    reg = k.wait_registration()
    c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
    ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
    g0, g1 = ids[:4], ids[4:]  # advertised in enumeration order, replicas 0..3
    assert all(i.endswith(f"-replica-{r}") for r, i in enumerate(g0))

    def mask(req):
        return dict(c.allocate(req).container_responses[0].envs).get("HSA_CU_MASK")
    assert mask([g0[0]]) == "0:0-63"
    assert mask([g0[3]]) == "0:192-255"
    assert mask([g0[2], g0[1]]) == "0:64-191"
    assert mask([g0[3], g0[1]]) == "0:64-127,192-255"
    assert mask([g1[2], g0[0]]) == "0:0-63;1:128-191"
    assert mask([g1[1]]) == "0:64-127"
    c.close()


def test_replica_cu_mask_on_cpx_partitions(running, scratch):
    fx = fixtures.node(1, "CPX", memory="NPS2")
    d, k = running(fx, args=["--partition-strategy", "single", "--resource-config", "gpu:gpu:4",
                             "--replica-cu-mask"])
    reg = k.wait_registration()
    c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
    ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
    assert len(ids) == 32
    envs = dict(c.allocate([ids[5]]).container_responses[0].envs)
    assert envs["HSA_CU_MASK"] == "0:8-15"  # one XCD, 32 CUs: replica 1 of 4
    c.close()


def test_replica_cu_mask_needs_a_possible_split(running, scratch):
    # 64 replicas > 32 CUs per XCD: no split, the daemon says so, no mask is set.
    d, k = running(args=["--resource-config", "gpu:sharedgpu:64", "--replica-cu-mask"])
    reg = k.wait_registration()
    c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
    ids = [x.ID for x in c.watch()[0].get(timeout=5).devices]
    assert "HSA_CU_MASK" not in dict(c.allocate(ids[:1]).container_responses[0].envs)
    assert "cannot be split into 64 CU shares" in d.log()
    c.close()


def test_memory_units_get_proportional_cu_shares(running, scratch):
    """gpu-mem-gb with --replica-cu-mask: a pod's CUs follow the HBM it holds. The
    k-th unit ID in name order owns CU slot floor(k*32/294) (one CU per XCD per
    slot), so pods admitted the kubelet's way (GetPreferredAllocation with pack,
    then Allocate) get contiguous slots -- a proportional CU share, not an
    isolating slice: neighbours may share one boundary slot."""
    d, k = running(args=["--resource-config", "gpu:gpu-mem-gb:-1", "--replica-policy", "pack",
                         "--replica-cu-mask", "--auto-replica-unit", "mib"])
    reg = k.wait_registration()
    c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
    free = [x.ID for x in c.watch()[0].get(timeout=5).devices]

    def admit(size):
        ids = list(c.preferred(free, size=size).container_responses[0].deviceIDs)
        for i in ids:
            free.remove(i)
        return dict(c.allocate(ids).container_responses[0].envs)
    envs = admit(36)
    assert envs["HSA_CU_MASK"] == "0:0-31" and envs["AMD_GPU_MEMORY_LIMIT_MIB"] == "36000"
    assert admit(36)["HSA_CU_MASK"] == "0:24-63"  # shares slot 3 with the first pod
    assert admit(222)["HSA_CU_MASK"] == "0:56-255"  # the rest of GPU 0
    c.close()


@pytest.mark.parametrize("sizes", [[36, 36, 36, 36, 36, 36, 36, 36, 6], [1] * 40, [5, 13, 1, 40, 9, 2, 100, 3],
                                   [10] * 29])
def test_memory_unit_cu_shares_overlap_at_most_one_boundary_slot(running, scratch, sizes):
    """The documented bound of the proportional CU share: pods admitted the
    kubelet's way (pack) each get one contiguous run of slots, and two pods
    never share more than one slot -- only at a boundary. A slot is shared only
    when both pods hold units of it."""
    d, k = running(fixture=fixtures.node(1), args=["--resource-config", "gpu:gpu-mem-gb:-1",
                                                   "--replica-policy", "pack", "--replica-cu-mask", "--auto-replica-unit", "mib"])
    reg = k.wait_registration()
    c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
    free = [x.ID for x in c.watch()[0].get(timeout=5).devices]
    slots = []
    for size in sizes:
        ids = list(c.preferred(free, size=size).container_responses[0].deviceIDs)
        for i in ids:
            free.remove(i)
        mask = dict(c.allocate(ids).container_responses[0].envs)["HSA_CU_MASK"]
        agent, ranges = mask.split(":")
        assert agent == "0" and "," not in ranges, mask  # one contiguous range
        lo, hi = map(int, ranges.split("-"))
        assert lo % 8 == 0 and (hi + 1) % 8 == 0, mask  # whole slots (one CU on each of 8 XCDs)
        slots.append(set(range(lo // 8, (hi + 1) // 8)))
    c.close()
    for i in range(len(slots)):
        for j in range(i + 1, len(slots)):
            shared = slots[i] & slots[j]
            assert len(shared) <= 1, (sizes[i], sizes[j], sorted(slots[i]), sorted(slots[j]))
            if shared:  # a boundary of both runs
                (s_,) = shared
                assert s_ in (min(slots[i]), max(slots[i])) and s_ in (min(slots[j]), max(slots[j]))


def _slot_model(ids, units=294, per=32):
    """The k-th unit ID in name order owns slot k*per//units (plugin.cc
    MemoryUnitCuRanges): slot of each ID and the number of units per slot."""
    num = {i: int(re.search(r"(\d+)$", i).group(1)) for i in ids}
    by_name = sorted(ids, key=lambda i: str(num[i]))
    slot = {i: k * per // units for k, i in enumerate(by_name)}
    size = collections.Counter(slot.values())
    return slot, size


@pytest.mark.parametrize("sizes", [[36, 36, 222], [36] * 8 + [6], [1] * 40, [5, 13, 1, 40, 9, 2, 100, 3],
                                   [10] * 29, [19] * 15])
def test_whole_cu_slots_never_share_a_cu(running, scratch, sizes):
    """--memory-unit-cu-slots whole: a container gets only the CU slots all of
    whose units it holds, so two containers that each fill a slot never share a
    CU; one that fills none keeps its partial slots and is counted in
    amdgpu_dp_partial_cu_slot_allocations_total. Checked against a model of the
    slot map for every pod, admitted the kubelet's way (pack)."""
    d, k = running(fixture=fixtures.node(1), args=["--resource-config", "gpu:gpu-mem-gb:-1", "--replica-policy",
                                                   "pack", "--replica-cu-mask", "--auto-replica-unit", "mib", "--memory-unit-cu-slots", "whole",
                                                   "--metrics-addr", "127.0.0.1:0"])
    port = int(re.search(r"serving /metrics and /healthz on port (\d+)",
                         d.wait_log("serving /metrics and /healthz on port")).group(1))
    reg = k.wait_registration()
    c = kubelet.PluginClient(os.path.join(scratch, reg.endpoint))
    free = [x.ID for x in c.watch()[0].get(timeout=5).devices]
    slot_of, slot_size = _slot_model(free)
    owned, partial = [], 0
    for size in sizes:
        ids = list(c.preferred(free, size=size).container_responses[0].deviceIDs)
        for i in ids:
            free.remove(i)
        held = collections.Counter(slot_of[i] for i in ids)
        whole = {s for s, n in held.items() if n == slot_size[s]}
        want = whole or set(held)
        partial += not whole
        mask = dict(c.allocate(ids).container_responses[0].envs)["HSA_CU_MASK"]
        agent, ranges = mask.split(":")
        got = set()
        for r in ranges.split(","):
            lo, hi = map(int, r.split("-"))
            assert lo % 8 == 0 and (hi + 1) % 8 == 0, mask
            got |= set(range(lo // 8, (hi + 1) // 8))
        assert agent == "0" and got == want, (size, mask, sorted(want))
        if size >= 19:  # any 19 consecutive units fill a slot (at most 10 units each)
            assert whole, (size, sorted(held.items()))
        if whole:
            owned.append(got)
    c.close()
    for i in range(len(owned)):
        for j in range(i + 1, len(owned)):
            assert not owned[i] & owned[j], (sorted(owned[i]), sorted(owned[j]))
    with urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5) as r:
        text = r.read().decode()
    assert f'amdgpu_dp_partial_cu_slot_allocations_total{{resource="amd.com/gpu-mem-gb"}} {partial}' in text, partial


def test_memory_unit_cu_slots_rejects_unknown_modes(scratch):
    r = subprocess.run([harness.DAEMON, "--device-plugin-path", scratch, "--memory-unit-cu-slots",
                        "exclusive", "--dry-run"], capture_output=True, text=True, timeout=30,
                       env=harness.Daemon(scratch, fixtures.node(1)).env)
    assert r.returncode != 0 and "invalid --memory-unit-cu-slots option: exclusive" in r.stdout + r.stderr

"""Per-resource replica policy and CU-slot memory units.

* ``--replica-policy auto`` (the default): memory-unit resources (replicas -1)
  pack a request onto as few GPUs as possible, time-slice replicas keep the
  reference's spread (/root/reference/cmd/nvidia-device-plugin/replica.go:149-190).
  A resource-config entry's 4th field (``gpu:sharedgpu:4:pack``) overrides it
  for that resource; ``--replica-policy spread|pack`` overrides it globally.
* ``--auto-replica-unit cu-slot`` (the default with ``--replica-cu-mask``): a
  memory unit is one CU slot -- one CU on every XCD -- plus VRAM / (CUs per XCD)
  of HBM, so every grant owns whole slots: no slot is shared between pods and
  none is left idle. The reference derives units from memory alone
  (/root/reference/cmd/nvidia-device-plugin/server.go:99-111).
"""

import collections
import os

import pytest

from k8s_gpu_sharing_plugin_amd.models import fixtures
from k8s_gpu_sharing_plugin_amd.utils import harness, kubelet

MIB = 294896


def _gpu_of(i):
    return i.split("-replica-")[0]


@pytest.fixture
def daemon(scratch):
    started = []

    def start(fx, args):
        k = kubelet.StubKubelet(os.path.join(scratch, "kubelet.sock")).start()
        d = harness.Daemon(scratch, fx, args=args).start()
        started.append((d, k))
        return d, k
    yield start
    for d, k in started:
        d.stop()
        k.stop()


def _client(scratch, k, resource):
    regs = {}
    while resource not in regs:
        r = k.wait_registration()
        regs[r.resource_name] = r
    c = kubelet.PluginClient(os.path.join(scratch, regs[resource].endpoint))
    return c, [x.ID for x in c.watch()[0].get(timeout=5).devices]


def _gpus(c, ids, size):
    got = list(c.preferred(ids, size=size).container_responses[0].deviceIDs)
    assert len(got) == size
    return collections.Counter(_gpu_of(i) for i in got)


def test_auto_policy_packs_memory_units_and_spreads_time_slices(daemon, scratch):
    """One daemon, mixed strategy: gpu-mem-gb (memory units) and a time-slice
    partition resource. Under the default auto policy the former packs, the
    latter spreads -- no global switch serves both."""
    fx = fixtures.node(3, ["SPX", "SPX", "CPX"], memory="NPS1")
    d, k = daemon(fx, ["--partition-strategy", "mixed", "--resource-config",
                       "gpu:gpu-mem-gb:-1,cpx-1xcd.36gb:cpxshared:4"])
    mem, mem_ids = _client(scratch, k, "amd.com/gpu-mem-gb")
    assert len(_gpus(mem, mem_ids, 20)) == 1  # 20 units from one GPU
    ts, ts_ids = _client(scratch, k, "amd.com/cpxshared")
    assert len(ts_ids) == 8 * 4
    assert len(_gpus(ts, ts_ids, 3)) == 3  # three replicas on three different partitions
    log = d.log()
    assert "'amd.com/gpu-mem-gb': preferred allocation packs replicas (auto: memory units)" in log
    assert "'amd.com/cpxshared': preferred allocation spreads replicas (auto: time-slice replicas)" in log
    mem.close()
    ts.close()


def test_entry_policy_overrides_auto(daemon, scratch):
    d, k = daemon(fixtures.node(2), ["--resource-config", "gpu:sharedgpu:4:pack"])
    c, ids = _client(scratch, k, "amd.com/sharedgpu")
    assert len(_gpus(c, ids, 3)) == 1  # packed despite being time-slice replicas
    c.close()


def test_global_policy_overrides_auto(daemon, scratch):
    d, k = daemon(fixtures.node(2), ["--resource-config", "gpu:gpu-mem-gb:-1", "--replica-policy", "spread"])
    c, ids = _client(scratch, k, "amd.com/gpu-mem-gb")
    assert len(_gpus(c, ids, 2)) == 2  # the reference's spread, as asked
    c.close()


def test_entry_policy_beats_global_policy(daemon, scratch):
    d, k = daemon(fixtures.node(2), ["--resource-config", "gpu:gpu-mem-gb:-1:pack", "--replica-policy", "spread"])
    c, ids = _client(scratch, k, "amd.com/gpu-mem-gb")
    assert len(_gpus(c, ids, 2)) == 1
    c.close()


def test_bad_entry_policy_is_rejected(scratch):
    import subprocess
    r = subprocess.run([harness.DAEMON, "--device-plugin-path", scratch, "--resource-config", "gpu:shared:4:tight",
                        "--dry-run"], capture_output=True, text=True, timeout=30,
                       env=harness.Daemon(scratch, fixtures.node(1)).env)
    assert r.returncode != 0 and "replica policy must be spread, pack or auto" in r.stdout + r.stderr


def _slots(mask):
    agent, ranges = mask.split(":")
    out = set()
    for r in ranges.split(","):
        lo, hi = map(int, r.split("-"))
        assert lo % 8 == 0 and (hi + 1) % 8 == 0, mask
        out |= set(range(lo // 8, (hi + 1) // 8))
    return agent, out


@pytest.mark.parametrize("sizes", [[1, 2, 4, 8, 8, 4, 2, 1, 2], [8, 8, 8, 8], [1] * 32, [4] * 8, [2, 8, 1, 4, 1, 8, 8]])
def test_cu_slot_units_fill_whole_slots(daemon, scratch, sizes):
    """--replica-cu-mask with the default unit: one unit = one CU slot plus
    294,896 / 32 MiB of HBM. Packing a GPU with 1-, 2-, 4- and 8-unit pods the
    kubelet's way leaves 0 shared slots and 0 idle slots, and every pod's CUs
    are exactly its units' slots."""
    d, k = daemon(fixtures.node(1), ["--resource-config", "gpu:gpu-mem-gb:-1", "--replica-cu-mask"])
    c, free = _client(scratch, k, "amd.com/gpu-mem-gb")
    assert len(free) == 32
    unit = MIB // 32
    owned = []
    for size in sizes:
        ids = list(c.preferred(free, size=size).container_responses[0].deviceIDs)
        for i in ids:
            free.remove(i)
        envs = dict(c.allocate(ids).container_responses[0].envs)
        agent, slots = _slots(envs["HSA_CU_MASK"])
        assert agent == "0" and len(slots) == size, (size, envs["HSA_CU_MASK"])
        assert envs["AMD_GPU_MEMORY_LIMIT_MIB"] == str(size * unit)
        owned.append(slots)
    for i in range(len(owned)):
        for j in range(i + 1, len(owned)):
            assert not owned[i] & owned[j]
    used = set().union(*owned)
    if sum(sizes) == 32:
        assert used == set(range(32))  # no idle slot
    assert "amdgpu_dp_partial" not in d.log()
    c.close()


def test_cu_slot_units_on_cpx_partitions(daemon, scratch):
    """A CPX partition (1 XCD, 32 CUs) has 32 slots of one CU each: 32 units of
    its 36,862 MiB / 32."""
    fx = fixtures.node(1, "CPX", memory="NPS2")
    d, k = daemon(fx, ["--partition-strategy", "single", "--resource-config", "gpu:gpu-mem-gb:-1",
                       "--replica-cu-mask"])
    c, ids = _client(scratch, k, "amd.com/gpu-mem-gb")
    assert len(ids) == 8 * 32
    got = list(c.preferred(ids, size=4).container_responses[0].deviceIDs)
    envs = dict(c.allocate(got).container_responses[0].envs)
    assert envs["HSA_CU_MASK"] == "0:0-3"
    assert envs["AMD_GPU_MEMORY_LIMIT_MIB"] == str(4 * ((MIB // 8) // 32))
    c.close()


def test_mib_units_stay_available(daemon, scratch):
    d, k = daemon(fixtures.node(1), ["--resource-config", "gpu:gpu-mem-gb:-1", "--replica-cu-mask",
                                     "--auto-replica-unit", "mib"])
    c, ids = _client(scratch, k, "amd.com/gpu-mem-gb")
    assert len(ids) == 294
    c.close()


def test_cu_slot_units_without_cu_masks(daemon, scratch):
    """--auto-replica-unit cu-slot alone: slot-sized units, no HSA_CU_MASK."""
    d, k = daemon(fixtures.node(1), ["--resource-config", "gpu:gpu-mem-gb:-1", "--auto-replica-unit", "cu-slot"])
    c, ids = _client(scratch, k, "amd.com/gpu-mem-gb")
    assert len(ids) == 32
    envs = dict(c.allocate(ids[:3]).container_responses[0].envs)
    assert "HSA_CU_MASK" not in envs and envs["AMD_GPU_MEMORY_LIMIT_MIB"] == str(3 * (MIB // 32))
    c.close()


def test_two_resources_with_cu_masks_warn(daemon, scratch):
    """Mixed strategy with two time-slice resources under --replica-cu-mask:
    each numbers HSA_CU_MASK agents from the container's first GPU, so a
    container requesting both would get one plugin's value; the daemon says so."""
    fx = fixtures.node(2, ["SPX", "CPX"], memory="NPS1")
    d, k = daemon(fx, ["--partition-strategy", "mixed", "--resource-config",
                       "gpu:sharedgpu:4,cpx-1xcd.36gb:cpxshared:2", "--replica-cu-mask"])
    k.wait_registration()
    log = d.wait_log("each set HSA_CU_MASK")
    assert "amd.com/sharedgpu" in log and "amd.com/cpxshared" in log


def test_unknown_unit_mode_is_rejected(scratch):
    import subprocess
    r = subprocess.run([harness.DAEMON, "--device-plugin-path", scratch, "--auto-replica-unit", "gb", "--dry-run"],
                       capture_output=True, text=True, timeout=30, env=harness.Daemon(scratch, fixtures.node(1)).env)
    assert r.returncode != 0 and "invalid --auto-replica-unit option: gb" in r.stdout + r.stderr
